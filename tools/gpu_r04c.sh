# round-4 set C: the scratch probe, NPP A/B (bin 128 as a third vector
# pass), the stage-timer profile, then the knockout variants named on the
# command line (summarised on the box into $O/ko_traffic.json; the PMC
# databases are dropped to keep gpurun_out small)
#   bash tools/gpu_r04c.sh <tag> <variants...>
cd $GRAFT_REPO_ROOT && T=$1 && shift && O=gpurun_out/$T && mkdir -p $O && export TMPDIR=/tmp &&
echo "probe" >> $O/progress.log &&
timeout -k 10 200 python -u tools/scratch_probe.py 65536 > $O/probe_65536.txt 2>&1 &&
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode" &&
echo "npp" >> $O/progress.log &&
MELPE_AMD_LIB=build/var/npp_lane128.so timeout -k 10 300 python -u $B > $O/npp_lane128.json 2> $O/npp_lane128.err &&
timeout -k 10 300 python -u $B > $O/npp_cur.json 2> $O/npp_cur.err &&
echo "stage" >> $O/progress.log &&
timeout -k 10 300 python -u tools/stage_prof.py 262144 3 > $O/stage_prof.txt 2> $O/stage_prof.err &&
echo "ko" >> $O/progress.log &&
bash tools/gpu_r04_ko.sh $T "$@" &&
python3 tools/ko_summary.py $O $O/ko_traffic.json "$@" > $O/ko_summary.txt 2>&1 &&
python3 tools/prof_summary.py $O ko_$T 262144 > /dev/null 2>&1;
rc=$?; rm -rf $O/pmc_f_* $O/pmc_w_*; exit $rc
