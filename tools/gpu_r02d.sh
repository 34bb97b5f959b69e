# 2400 bps mode on the GPU + the full GPU suite + a bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u -m pytest tests/test_r2400.py -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/r24_tests.log 2>&1 &&
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 500 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
