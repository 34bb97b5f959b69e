# round-4 set A on the current build: the GPU suite, the driver's bench
# command (--steps 20 --warmup 5) and its kernel trace, and the NPP A/B
# (bin 128 as a third vector pass: build/var/npp_lane128.so), the encode
# step split over engines on concurrent streams (tools/split_exp.py) and the
# stage-timer profile (tools/stage_prof.py, libmelpe_amd_prof.so)
#   bash tools/gpu_r04a.sh <tag>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt_bench.err || exit $?
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode"
if [ -f build/var/npp_lane128.so ]; then
  MELPE_AMD_LIB=build/var/npp_lane128.so timeout -k 10 300 python $B > $O/npp_lane128.json 2> $O/npp_lane128.err || exit $?
fi
timeout -k 10 300 python $B > $O/npp_cur.json 2> $O/npp_cur.err || exit $?
timeout -k 10 300 python tools/split_exp.py 262144 1 2 4 > $O/split.txt 2> $O/split.err || exit $?
if [ -f pairphone_amd/libmelpe_amd_prof.so ]; then
  timeout -k 10 300 python tools/stage_prof.py 262144 3 > $O/stage_prof.txt 2> $O/stage_prof.err || exit $?
fi
python3 tools/prof_summary.py $O r04_$1 > $O/summary.log 2>&1
mkdir -p $O/profiles && cp profiles/r04_$1_* $O/profiles/ 2>/dev/null
exit $rc
