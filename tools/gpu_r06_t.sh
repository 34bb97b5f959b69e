# round 6: progress-driven priority in the four-wave analysis (progprio.h;
# build/var/prio5.so): its tests through that build, then the quick bench A/B
# at the N=8 shard size
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06t && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/prio5.so timeout -k 10 900 python -u -m pytest tests/test_ana_mw.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
bash tools/gpu_r05_ab.sh r06t_ab 32768 cur prio5 prio5:MELPE_MW_PRIO=0 cur prio5 prio5:MELPE_MW_PRIO=0
