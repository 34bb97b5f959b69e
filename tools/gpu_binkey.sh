# class-key variants of the pitch-class lane order (MELPE_BIN_KEY=<mode>):
# encode/decode GPU parity under each, then the encode + decode bench per mode
#   tools/gpu_binkey.sh <mode> [<mode> ...]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/binkey && export TMPDIR=/tmp &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
for m in "$@"; do
  MELPE_BIN_KEY=$m timeout -k 10 300 python -u -m pytest tests/test_encode.py tests/test_decode.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/binkey/tests_$m.log 2>&1 || exit 1
  for C in 262144 32768; do
    MELPE_BIN_KEY=$m timeout -k 10 200 python $B --channels $C > gpurun_out/binkey/k${m}_$C.json 2> gpurun_out/binkey/k${m}_$C.err || exit 1
  done
done
