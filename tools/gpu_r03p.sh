# voicing bands 1..4 in k_enc_band: the GPU tests, then the 262,144-channel
# encode step with the bands split (default) and kept in k_enc_ana, twice
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144" &&
for r in 1 2; do
  timeout -k 10 300 python $B > gpurun_out/$1/b_band_$r.json 2> gpurun_out/$1/b_band_$r.err || exit 1
  MELPE_BANDS=0 timeout -k 10 300 python $B > gpurun_out/$1/b_nob_$r.json 2> gpurun_out/$1/b_nob_$r.err || exit 1
done
