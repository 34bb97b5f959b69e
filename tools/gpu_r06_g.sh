# round 6: NPP per-bin temporaries in registers (LDS image 9,980 -> 8,948 B),
# with (npp1p) and without (npp1r) a per-wave LDS copy of the math tables,
# one channel per workgroup; tests on npp1p
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06g && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/npp1p.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_npp.py tests/test_encode.py -m gpu > $O/tests.txt 2>&1 &&
bash tools/gpu_r05_ab.sh r06g_262k 262144 cur npp1p npp1r cur npp1p
