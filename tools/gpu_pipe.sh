# superframe pipeline experiment (tools/pipe_exp.py) on the product build and
# on build/var/<variant>.so, at 262,144 and 65,536 channels
#   tools/gpu_pipe.sh <variant> [<variant> ...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pipe && export TMPDIR=/tmp &&
for C in 262144 65536; do
  timeout -k 10 200 python tools/pipe_exp.py $C 6 > gpurun_out/pipe/cur_$C.json 2> gpurun_out/pipe/cur_$C.err || exit 1
  for v in "$@"; do
    MELPE_AMD_LIB=build/var/$v.so timeout -k 10 200 python tools/pipe_exp.py $C 6 > gpurun_out/pipe/${v}_$C.json 2> gpurun_out/pipe/${v}_$C.err || exit 1
  done
done
