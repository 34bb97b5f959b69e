# the GPU suite, then the bench line with the driver's command
#   bash tools/gpu_r05_full.sh <tag>
cd $GRAFT_REPO_ROOT && T=$1 && mkdir -p gpurun_out/$T && export TMPDIR=/tmp &&
timeout -k 10 700 python -u -m pytest -s tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/full_tests.log 2>&1 &&
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
