# round 6: stage profile per quarter of the lane order at 262,144 channels
# (build/var/profq.so: -DMELPE_PROF -DMELPE_PROF_QUART)
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06o && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/profq.so timeout -k 10 300 python3 -u tools/stage_prof_q.py 262144 4 > $O/stage_q_262k.txt 2>&1
