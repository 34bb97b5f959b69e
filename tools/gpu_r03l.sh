# MW: find_harm's FFT beside sc_ana, band 4 of the last frame on wave 1
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests/test_ana_mw.py tests/test_encode.py tests/test_state.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --channels 32768 > gpurun_out/$1/b_32768.json 2> gpurun_out/$1/b_32768.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/$1/mwprof_32768.txt 2>&1
