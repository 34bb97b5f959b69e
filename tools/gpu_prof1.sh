# rocprofv3 passes over one k_encode launch at 65,536 channels (round 1).
# Each step has its own time limit; steps chained with && (stop on failure).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
B="bench.py --channels 65536 --steps 1 --warmup 0 --no-decode --no-cpu-baseline" &&
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt -- python3 bench.py --channels 65536 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE -d gpurun_out/pmc_a -o a -- python3 $B > gpurun_out/pmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_b -o b -- python3 $B > gpurun_out/pmc_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c -o c -- python3 $B > gpurun_out/pmc_c.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_d -o d -- python3 $B > gpurun_out/pmc_d.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_e -o e -- python3 $B > gpurun_out/pmc_e.log 2>&1
