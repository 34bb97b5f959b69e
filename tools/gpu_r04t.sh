# the 32,768-channel step three times (run-to-run spread), the quick check,
# then the config-5 TX leg
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04t && export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode --channels 32768"
for i in 1 2 3; do timeout -k 10 200 python -u $B > gpurun_out/r04t/p$i.json 2> gpurun_out/r04t/p$i.err || exit $?; done
bash tools/gpu_r04q.sh r04t || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-side-legs --total-channels 0 --no-decode > gpurun_out/r04t/tx.json 2> gpurun_out/r04t/tx.err
