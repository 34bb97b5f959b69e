# round 6: decode-only A/B of the two decoder mappings (MELPE_DEC_NW) of the
# two-wave decoder build (build/var/dec2.so) at 32,768 / 65,536 / 262,144
# channels, then the config-3 round trip test on it
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06b && mkdir -p $O && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06b_32k 32768 base dec2:MELPE_DEC_NW=1 dec2:MELPE_DEC_NW=2 &&
bash tools/gpu_r05_ab.sh r06b_65k 65536 base dec2:MELPE_DEC_NW=1 dec2:MELPE_DEC_NW=2 &&
bash tools/gpu_r05_ab.sh r06b_262k 262144 base dec2 &&
MELPE_AMD_LIB=build/var/dec2.so timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_scale.py -m gpu -k config3 > $O/tests_c3.txt 2>&1
