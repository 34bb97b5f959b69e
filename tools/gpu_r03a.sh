# round 3, first look at the multi-wave analysis kernel (k_enc_ana_mw):
# its GPU tests, then the encode step at 32,768 / 65,536 / 262,144 channels
# with 1, 2 and 4 analysis waves per 64 channels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/a && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_ana_mw.py tests/test_device_helpers.py tests/test_shard.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/a/tests.log 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0" &&
for C in 32768 65536 131072 262144; do
  for NW in 1 2 4; do
    MELPE_ANA_NW=$NW timeout -k 10 300 python $B --channels $C > gpurun_out/a/b_${C}_${NW}.json 2> gpurun_out/a/b_${C}_${NW}.err || exit 1
  done
done
