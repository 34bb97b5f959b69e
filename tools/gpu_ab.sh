# A/B iteration: encode/decode GPU parity on the current build, then the
# encode-only bench for build/var/<variant>.so vs the current build at
# 262,144 and 32,768 channels, then the stage profile of the current build
#   tools/gpu_ab.sh <variant> [<variant> ...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_encode.py tests/test_decode.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
for C in 262144 32768; do
  timeout -k 10 200 python $B --channels $C > gpurun_out/ab/cur_$C.json 2> gpurun_out/ab/cur_$C.err || exit 1
  for v in "$@"; do
    MELPE_AMD_LIB=build/var/$v.so timeout -k 10 200 python $B --channels $C > gpurun_out/ab/${v}_$C.json 2> gpurun_out/ab/${v}_$C.err || exit 1
  done
done &&
{ [ ! -f pairphone_amd/libmelpe_amd_prof.so ] || timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/ab/stage.txt 2> gpurun_out/ab/stage.err; }
