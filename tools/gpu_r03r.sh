# lsf_vq with a wave per channel (k_lsf.hip): the GPU tests, then the
# 262,144-channel encode step with it (default) and with lsf_vq kept in
# k_enc_ana (MELPE_LSFW=0), twice, then a kernel trace
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144" &&
for r in 1 2; do
  timeout -k 10 300 python $B > gpurun_out/$1/b_lsfw_$r.json 2> gpurun_out/$1/b_lsfw_$r.err || exit 1
  MELPE_LSFW=0 timeout -k 10 300 python $B > gpurun_out/$1/b_lane_$r.json 2> gpurun_out/$1/b_lane_$r.err || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/kt -o kt --output-format csv -- python3 $B > gpurun_out/$1/b_kt.json 2> gpurun_out/$1/b_kt.err
