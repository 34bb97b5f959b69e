# lsf_vq with a wave per channel (k_lsf.hip, MELPE_LSFW=1): the GPU tests on
# it, then the 262,144-channel encode step with it and with lsf_vq kept in
# k_enc_ana (default), twice, then a kernel trace of it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
MELPE_LSFW=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$1/tests.log 2>&1 &&
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144" &&
for r in 1 2; do
  MELPE_LSFW=1 timeout -k 10 300 python $B > gpurun_out/$1/b_lsfw_$r.json 2> gpurun_out/$1/b_lsfw_$r.err || exit 1
  timeout -k 10 300 python $B > gpurun_out/$1/b_lane_$r.json 2> gpurun_out/$1/b_lane_$r.err || exit 1
done &&
MELPE_LSFW=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/kt -o kt --output-format csv -- python3 $B > gpurun_out/$1/b_kt.json 2> gpurun_out/$1/b_kt.err
