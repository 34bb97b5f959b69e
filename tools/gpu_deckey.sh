# decoder lane-order key from the superframe being decoded (k_dec_key) vs the
# last superframe's (MELPE_DEC_KEY=prev): GPU parity, then the bench at
# 262,144 and 32,768 channels under each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/deckey && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_lane_order.py tests/test_decode.py tests/test_scale.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/deckey/tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
for C in 262144 32768; do
  MELPE_DEC_KEY=prev timeout -k 10 200 python $B --channels $C > gpurun_out/deckey/prev_$C.json 2> gpurun_out/deckey/prev_$C.err || exit 1
  timeout -k 10 200 python $B --channels $C > gpurun_out/deckey/cur_$C.json 2> gpurun_out/deckey/cur_$C.err || exit 1
done
