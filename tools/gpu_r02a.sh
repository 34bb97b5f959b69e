# round 2, first call: GPU parity tests (incl. the new device-op, drop-in,
# state and melpe_n tests), the default bench line (weak + strong + tx legs),
# a 1-GPU run at the N=8 shard size (32,768 channels) and its kernel trace.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 python bench.py --channels 32768 --total-channels 0 --tx-channels 0 --no-cpu-baseline > gpurun_out/bench_32k.json 2> gpurun_out/bench_32k.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt32k -o kt -- python3 bench.py --channels 32768 --total-channels 0 --tx-channels 0 --no-cpu-baseline --no-side-legs > gpurun_out/prof_kt32k.log 2>&1
