# round 6: how the lane analysis launch's waves finish (k_ana.hip
# MELPE_WAVE_TIMES build) at 262,144 and 65,536 channels
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06i && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/wt.so timeout -k 10 300 python3 -u tools/wave_times.py 262144 8 > $O/wt_262k.jsonl 2> $O/wt_262k.err &&
MELPE_AMD_LIB=build/var/wt.so timeout -k 10 300 python3 -u tools/wave_times.py 65536 8 > $O/wt_65k.jsonl 2> $O/wt_65k.err
