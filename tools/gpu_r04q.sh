# quick check of the current build: GPU tests (all, or those of the files
# named in $2), then the encode step at 262,144 channels and the
# 32,768-channel shard
#   bash tools/gpu_r04q.sh <tag> ["tests/test_encode.py tests/test_decode.py"]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
O=gpurun_out/$1
T=${2:-tests}
timeout -k 10 600 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > $O/full_tests.log 2>&1
rc=$?; echo "tests rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
B="bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0"
timeout -k 10 300 python -u $B > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 python -u $B --channels 32768 --no-decode > $O/bench_32k.json 2> $O/bench_32k.err || exit $?
exit $rc
