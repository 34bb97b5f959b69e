# round 6: NPP with the math tables in LDS (8 channels per workgroup:
# npp8), and at three waves per SIMD (fewer spills: *w3), against the
# product at 262,144 channels; the NPP / encode tests on npp8
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06d && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/npp8.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_npp.py tests/test_encode.py -m gpu > $O/tests.txt 2>&1 &&
bash tools/gpu_r05_ab.sh r06d_262k 262144 cur npp8 npp8w3 npp1w3 cur npp8
