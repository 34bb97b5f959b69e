# encoder lane-order class keys (MELPE_ENC_KEY=<mode>, engine.hip bin_class):
# encode GPU parity under each, then the encode bench at 262,144 channels
#   tools/gpu_enckey.sh <mode> [<mode> ...]   (0 = the default key)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/enckey && export TMPDIR=/tmp &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode" &&
for m in "$@"; do
  MELPE_ENC_KEY=$m timeout -k 10 300 python -u -m pytest tests/test_encode.py tests/test_lane_order.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/enckey/tests_$m.log 2>&1 || exit 1
  MELPE_ENC_KEY=$m timeout -k 10 200 python $B --channels 262144 > gpurun_out/enckey/k${m}.json 2> gpurun_out/enckey/k${m}.err || exit 1
done
