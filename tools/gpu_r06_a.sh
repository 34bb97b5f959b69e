# round 6, first GPU call: A/B of the find_pitch / frac_cor block unrolling
# (build/var/fp1.so) against the round-5 product (build/var/base.so) at
# 262,144 and 32,768 channels, the encode / four-wave tests on fp1, and the
# new config-3 round-trip bench leg.
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06a && mkdir -p $O && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06a_ab 262144 base fp1 base fp1 &&
bash tools/gpu_r05_ab.sh r06a_ab32 32768 base fp1 &&
MELPE_AMD_LIB=build/var/fp1.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_encode.py tests/test_ana_mw.py -m gpu > $O/tests.txt 2>&1 &&
MELPE_AMD_LIB=build/var/fp1.so timeout -k 10 300 python3 -u bench.py --steps 6 --warmup 2 --no-host-leg --no-duplex \
  --no-side-legs --tx-channels 0 --total-channels 0 --no-decode --channels 65536 --cpu-jobs 16 --cpu-sample-channels 16 \
  > $O/rt.json 2> $O/rt.err
