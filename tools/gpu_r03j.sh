# decoder (realIDFT fast path, doubled LDS cosine rows) and MW (batched dc
# removal from global PCM) check: their GPU tests, the default line without
# side legs, the 32,768-channel step and the MW phase profile
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests/test_decode.py tests/test_ana_mw.py tests/test_lane_order.py tests/test_r2400.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
timeout -k 10 600 python bench.py --no-cpu-baseline --no-side-legs --tx-channels 0 --total-channels 0 > gpurun_out/$1/bench.json 2> gpurun_out/$1/bench.err &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --channels 32768 > gpurun_out/$1/b_32768.json 2> gpurun_out/$1/b_32768.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/$1/mwprof_32768.txt 2>&1
