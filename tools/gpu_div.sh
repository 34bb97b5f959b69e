# divergence fixes: GPU parity of encode / decode / 2400 / streams / lane
# order on the current build, then the encode + decode bench of the current
# build and of build/var/<variant>.so at 262,144 and 32,768 channels
#   tools/gpu_div.sh <variant> [<variant> ...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dv && export TMPDIR=/tmp &&
timeout -k 10 500 python -u -m pytest tests/test_encode.py tests/test_decode.py tests/test_r2400.py tests/test_stream.py tests/test_lane_order.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/dv/tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
for C in 262144 32768; do
  timeout -k 10 200 python $B --channels $C > gpurun_out/dv/cur_$C.json 2> gpurun_out/dv/cur_$C.err || exit 1
  for v in "$@"; do
    MELPE_AMD_LIB=build/var/$v.so timeout -k 10 200 python $B --channels $C > gpurun_out/dv/${v}_$C.json 2> gpurun_out/dv/${v}_$C.err || exit 1
  done
done
