# MW step after the batched lsf scan and record copy-in: the MW GPU tests,
# the 32,768-channel encode step (engine's choice) and the phase profile
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_ana_mw.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
timeout -k 10 300 python $B --channels 32768 > gpurun_out/$1/b_32768.json 2> gpurun_out/$1/b_32768.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/$1/mwprof_32768.txt 2>&1
