# GPU parity tests (modem, full-duration scale), the default bench line, its
# kernel trace, and the PMC passes (one counter group per pass) at 262,144
# channels for this build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o kt -- python3 bench.py --no-cpu-baseline --total-channels 0 --tx-channels 0 > gpurun_out/prof_kt.log 2>&1 &&
B="bench.py --steps 2 --warmup 0 --no-cpu-baseline --total-channels 0 --tx-channels 0" &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o f -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o w -- python3 $B > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE -d gpurun_out/pmc_a -o a -- python3 $B > gpurun_out/pmc_a.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_b -o b -- python3 $B > gpurun_out/pmc_b.log 2>&1
