set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --channels 65536 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b_small.json 2> gpurun_out/b_small.err &&
timeout -k 10 900 python bench.py > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err
