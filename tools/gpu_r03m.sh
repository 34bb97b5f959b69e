# lsf slices gathering their codebook rows (MELPE_LQ_GATHER build,
# build/var/lqg.so) against the scalar-cache waterfall: the MW tests on the
# variant, then the 32,768-channel step of both, twice, interleaved
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/lqg.so timeout -k 10 600 python -u -m pytest -s tests/test_ana_mw.py -x -v -m gpu -k "golden or wave_counts or 32768" --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 32768" &&
for r in 1 2; do
  timeout -k 10 300 python $B > gpurun_out/$1/b_cur_$r.json 2> gpurun_out/$1/b_cur_$r.err || exit 1
  MELPE_AMD_LIB=build/var/lqg.so timeout -k 10 300 python $B > gpurun_out/$1/b_lqg_$r.json 2> gpurun_out/$1/b_lqg_$r.err || exit 1
done
