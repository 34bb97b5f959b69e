# round-4 set B on the current build: the GPU suite, the driver's bench
# command (--steps 20 --warmup 5), its kernel trace, the split-stream probe
#   bash tools/gpu_r04b.sh <tag>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
O=gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_kt -o kt -- python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt_bench.json 2> $O/kt_bench.err || exit $?
timeout -k 10 300 python -u tools/split_exp.py 262144 1 2 4 > $O/split.txt 2> $O/split.err || exit $?
python3 tools/prof_summary.py $O r04_$1 > $O/summary.log 2>&1
mkdir -p $O/profiles && cp profiles/r04_$1_* $O/profiles/ 2>/dev/null
exit $rc
