# round 6: stage profile per quarter of the lane order, default priority and
# MELPE_ANA_PRIO=1 (quarter q at priority q), same box
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06q && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/profq.so timeout -k 10 300 python3 -u tools/stage_prof_q.py 262144 4 > $O/stage_q_p0.txt 2>&1 &&
MELPE_ANA_PRIO=1 MELPE_AMD_LIB=build/var/profq.so timeout -k 10 300 python3 -u tools/stage_prof_q.py 262144 4 > $O/stage_q_p1.txt 2>&1
