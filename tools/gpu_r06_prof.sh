# round 6: stage profiles of the profiling build (build/var/prof.so): the
# lane analysis, NPP (finer scopes) and the lane decoder at 262,144 channels,
# the two-wave decoder at 32,768
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06p && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/prof.so timeout -k 10 300 python3 -u tools/stage_prof.py 262144 6 > $O/stage_262k.txt 2>&1 &&
MELPE_AMD_LIB=build/var/prof.so timeout -k 10 300 python3 -u tools/stage_prof.py 32768 6 > $O/stage_32k.txt 2>&1
