cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 900 python bench.py --cpu-sample-channels 96 > gpurun_out/bench.json 2> gpurun_out/bench.err
