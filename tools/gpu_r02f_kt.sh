# kernel trace of exactly the default bench command; its own JSON line is
# kept next to the trace so the HIP-event averages can be checked against it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/fk && export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/fk/prof_kt -o kt -- python3 bench.py > gpurun_out/fk/bench_under_kt.json 2> gpurun_out/fk/prof_kt.log
