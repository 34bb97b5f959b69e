# the GPU suite, then tools/gpu_r05_ab.sh's bench A/B
#   bash tools/gpu_r05_tests_ab.sh <tag> <channels> <variant>...
cd $GRAFT_REPO_ROOT && T=$1 && mkdir -p gpurun_out/$T && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/full_tests.log 2>&1 &&
bash tools/gpu_r05_ab.sh "$@"
