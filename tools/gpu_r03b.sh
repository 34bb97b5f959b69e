# multi-wave analysis after the selective copy-in: GPU tests of the kernel,
# the phase profile (stage-timer build) at 32,768 / 65,536 channels, and
# the encode step per wave count
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/b && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_ana_mw.py -x -v -m gpu -k "golden or agree" --timeout 300 --timeout-method thread > gpurun_out/b/tests.log 2>&1 &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/b/mwprof_32768_4.txt 2>&1 &&
MELPE_ANA_NW=2 timeout -k 10 300 python tools/mw_prof.py 32768 4 > gpurun_out/b/mwprof_32768_2.txt 2>&1 &&
MELPE_ANA_NW=4 timeout -k 10 300 python tools/mw_prof.py 65536 4 > gpurun_out/b/mwprof_65536_4.txt 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
for C in 32768 65536; do
  for NW in 1 4; do
    MELPE_ANA_NW=$NW timeout -k 10 300 python $B --channels $C > gpurun_out/b/b_${C}_${NW}.json 2> gpurun_out/b/b_${C}_${NW}.err || exit 1
  done
done
