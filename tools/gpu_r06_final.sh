# round 6 set: the whole GPU suite, the bench line with the driver's command
# (--steps 20 --warmup 5, CPU baseline curve included), the 32,768-channel
# N=8 shard size with the same step count, and a kernel trace of the default
# command summarised into profiles/r06_<tag>_*; the PMC passes
# (tools/gpu_r06_pmc.sh at 262,144 and 32,768 channels) are a separate call
#   bash tools/gpu_r06_final.sh <tag>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1/profiles && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest -s tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/$1/full_tests.log 2>&1 &&
timeout -k 10 900 python bench.py --steps 20 --warmup 5 > gpurun_out/$1/bench.json 2> gpurun_out/$1/bench.err &&
timeout -k 10 600 python bench.py --channels 32768 --total-channels 32768 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-host-leg --no-duplex --no-side-legs --tx-channels 0 --rt-channels 0 > gpurun_out/$1/bench_32k.json 2> gpurun_out/$1/bench_32k.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/prof_kt -o kt -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$1/kt_bench.json 2> gpurun_out/$1/kt_bench.err &&
python3 tools/prof_summary.py gpurun_out/$1 r06_$1 > gpurun_out/$1/summary.log 2>&1 &&
cp profiles/r06_$1_* gpurun_out/$1/profiles/
