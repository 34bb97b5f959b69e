# round 3, first measurement set of the multi-wave analysis build: the
# 32,768-channel step (N=8 shard) with the engine's choice (4 waves / 64
# channels) and lane-per-channel for comparison, the default 262,144-channel
# line without the CPU baseline (and with MW forced for comparison), a kernel
# trace of the 32,768-channel step, then the GPU tests not yet run this round
# (-s: the two-process test's ranks print progress)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/d && export TMPDIR=/tmp &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
timeout -k 10 300 python $B --channels 32768 > gpurun_out/d/b_32768.json 2> gpurun_out/d/b_32768.err &&
MELPE_ANA_NW=1 timeout -k 10 300 python $B --channels 32768 > gpurun_out/d/b_32768_nw1.json 2> gpurun_out/d/b_32768_nw1.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/d/kt32 -o kt -- python3 $B --channels 32768 > gpurun_out/d/kt32.log 2>&1 &&
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/d/bench.json 2> gpurun_out/d/bench.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python $B --no-decode > gpurun_out/d/b_262144_nw4.json 2> gpurun_out/d/b_262144_nw4.err &&
timeout -k 10 600 python -u -m pytest -s tests/test_shard.py tests/test_stream.py tests/test_state.py tests/test_vad.py tests/test_xcorr.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/d/tests_rest.log 2>&1
