# GPU suite (new: modem staging, device-side mapping gate) + the lane vs
# four-wave crossover + bench A/B line
cd $GRAFT_REPO_ROOT && T=$1 && mkdir -p gpurun_out/$T && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/full_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/mw_crossover.py > gpurun_out/$T/crossover.jsonl 2> gpurun_out/$T/crossover.err &&
bash tools/gpu_r05_ab.sh $T 262144 cur
