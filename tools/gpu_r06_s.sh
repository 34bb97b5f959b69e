# round 6: progress-driven priority in the lane analysis and decoder
# (progprio.h; build/var/prio4.so): the encode/decode goldens and config 4
# through that build, then the quick bench A/B against the product build
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06s && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/prio4.so timeout -k 10 900 python -u -m pytest tests/test_encode.py tests/test_decode.py tests/test_scale.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
bash tools/gpu_r05_ab.sh r06s_ab 262144 cur prio4 prio4:MELPE_ANA_PRIO=0,MELPE_DEC_PRIO=0 prio4:MELPE_DEC_PRIO=0 cur prio4 prio4:MELPE_ANA_PRIO=0,MELPE_DEC_PRIO=0
