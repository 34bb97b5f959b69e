cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline" &&
timeout -k 10 300 python $B > gpurun_out/s0.json 2> gpurun_out/s0.err &&
HSA_SCRATCH_SINGLE_LIMIT=16000000000 timeout -k 10 300 python $B > gpurun_out/s1.json 2> gpurun_out/s1.err
