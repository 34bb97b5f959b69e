# fresh-container re-check of the last committed engine: the whole GPU suite,
# then the default bench line under a kernel trace (one run gives both)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/g && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/g/full_tests.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/g/prof_kt -o kt -- python3 bench.py > gpurun_out/g/bench_under_kt.json 2> gpurun_out/g/prof_kt.log
