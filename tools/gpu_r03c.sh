# MW schedule / decoder dispersion pass: GPU tests of both, the MW phase
# profile at 32,768 channels, the encode step at 32,768 / 65,536 and the
# default 262,144-channel line with its decode leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/c && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_ana_mw.py tests/test_decode.py -x -v -m gpu -k "not 32768" --timeout 300 --timeout-method thread > gpurun_out/c/tests.log 2>&1 &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/c/mwprof_32768_4.txt 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
timeout -k 10 300 python $B --channels 32768 > gpurun_out/c/b_32768.json 2> gpurun_out/c/b_32768.err &&
timeout -k 10 300 python $B --channels 65536 > gpurun_out/c/b_65536.json 2> gpurun_out/c/b_65536.err &&
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 > gpurun_out/c/b_262144.json 2> gpurun_out/c/b_262144.err
