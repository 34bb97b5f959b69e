# round-2 measurement set after the call-site merges: the whole GPU suite first
# round 2 measurement set: kernel trace of the default bench and the PMC
# passes (one counter group per run), summarised into profiles/r02_k_* and
# profiles/pmc_latest.json (which the bench line reads for `traffic`), then
# the default bench line (weak-scaling encode + strong leg + side legs + CPU
# baseline) and a committed 1-GPU run at the N=8 shard size (32,768
# channels).  The box's profiles/ is copied back under gpurun_out/k/.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/k && export TMPDIR=/tmp &&
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/k/full_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/k/prof_kt -o kt -- python3 bench.py --no-cpu-baseline --steps 4 > gpurun_out/k/prof_kt.log 2>&1 &&
B="bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/k/pmc_fetch -o f -- python3 $B > gpurun_out/k/pmc_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/k/pmc_write -o w -- python3 $B > gpurun_out/k/pmc_write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE -d gpurun_out/k/pmc_a -o a -- python3 $B > gpurun_out/k/pmc_a.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/k/pmc_b -o b -- python3 $B > gpurun_out/k/pmc_b.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/k/pmc_c -o c -- python3 $B > gpurun_out/k/pmc_c.log 2>&1 &&
python3 tools/prof_summary.py gpurun_out/k r02_k 262144 > gpurun_out/k/summary.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/k/bench.json 2> gpurun_out/k/bench.err &&
timeout -k 10 300 python bench.py --channels 32768 --total-channels 0 --tx-channels 0 --no-cpu-baseline > gpurun_out/k/bench_32k.json 2> gpurun_out/k/bench_32k.err &&
mkdir -p gpurun_out/k/profiles && cp profiles/r02_k_* profiles/pmc_latest.json gpurun_out/k/profiles/
