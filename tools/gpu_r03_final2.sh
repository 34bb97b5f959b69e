# round-3 final set, part 2: the MW GPU tests, the 32,768-channel step and
# phase profile, then kernel trace + PMC passes at 32,768 and 262,144
# channels (profiles/r03_<tag>32k_*, r03_<tag>_*, pmc_latest.json)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest -s tests/test_ana_mw.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --channels 32768 > gpurun_out/$1/b_32768.json 2> gpurun_out/$1/b_32768.err &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/$1/mwprof_32768.txt 2>&1 &&
bash tools/gpu_r03_pmc.sh ${1}32k 32768 &&
bash tools/gpu_r03_pmc.sh $1 262144
