# round 6: per-wave end times and placement (HW_ID, XCC_ID) of the lane
# analysis launch at 262,144 channels (MELPE_WAVE_TIMES build)
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06m && mkdir -p $O && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/wt.so timeout -k 10 300 python3 -u tools/wave_times.py 262144 8 $O/wt_262k.npz > $O/wt_262k.jsonl 2> $O/wt_262k.err
