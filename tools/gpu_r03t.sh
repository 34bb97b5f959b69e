# lsf_vq wave kernel with register indices: the encode GPU tests on it, the
# 262,144-channel step with it and without, then its kernel trace
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
MELPE_LSFW=1 timeout -k 10 600 python -u -m pytest tests/test_encode.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144" &&
MELPE_LSFW=1 timeout -k 10 300 python $B > gpurun_out/$1/b_lsfw.json 2> gpurun_out/$1/b_lsfw.err &&
timeout -k 10 300 python $B > gpurun_out/$1/b_lane.json 2> gpurun_out/$1/b_lane.err &&
MELPE_LSFW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/kt -o kt --output-format csv -- python3 $B > gpurun_out/$1/b_kt.json 2> gpurun_out/$1/b_kt.err
