# MW at 8 waves per workgroup vs 4: the MW / decoder GPU tests, the
# 32,768-channel step at both, the phase profile at 8, the default line
# without side legs
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests/test_ana_mw.py tests/test_decode.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --channels 32768" &&
MELPE_ANA_NW=8 timeout -k 10 300 python $B > gpurun_out/$1/b_32768_8.json 2> gpurun_out/$1/b_32768_8.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python $B > gpurun_out/$1/b_32768_4.json 2> gpurun_out/$1/b_32768_4.err &&
MELPE_ANA_NW=8 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/$1/mwprof_32768_8.txt 2>&1 &&
timeout -k 10 600 python bench.py --no-cpu-baseline --no-side-legs --tx-channels 0 --total-channels 0 > gpurun_out/$1/bench.json 2> gpurun_out/$1/bench.err
