# MW kernel compiled for 2 resident waves per SIMD (256 VGPRs; every
# workgroup of a 32,768-channel launch resident at once): its GPU tests, the
# encode step at 32,768 and 65,536 channels with MW and lane-per-channel, and
# the MW phase profile at 32,768
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/e && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_ana_mw.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/e/tests.log 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
for C in 32768 65536; do
  for NW in 4 1; do
    MELPE_ANA_NW=$NW timeout -k 10 300 python $B --channels $C > gpurun_out/e/b_${C}_${NW}.json 2> gpurun_out/e/b_${C}_${NW}.err || exit 1
  done
done &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/e/mwprof_32768.txt 2>&1
