# split lane analysis (k_enc_ana -> k_enc_harm -> k_enc_tail): the encode
# GPU tests (goldens, edge signals vs the live reference, ragged masks, lane
# order, config 4 at scale), then the 262,144-channel step split vs
# MELPE_HARM=0, twice interleaved, and a kernel trace of the split step
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest -s tests/test_encode.py tests/test_lane_order.py tests/test_state.py tests/test_scale.py tests/test_vad.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
for r in 1 2; do
  timeout -k 10 300 python $B > gpurun_out/$1/b_split_$r.json 2> gpurun_out/$1/b_split_$r.err || exit 1
  MELPE_HARM=0 timeout -k 10 300 python $B > gpurun_out/$1/b_whole_$r.json 2> gpurun_out/$1/b_whole_$r.err || exit 1
done &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/prof_kt -o kt -- python3 $B --steps 4 > gpurun_out/$1/kt.log 2>&1
