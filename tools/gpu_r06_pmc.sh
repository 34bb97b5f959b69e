# kernel trace + PMC passes of the encode/decode step at one channel count
# (one counter group per pass, each its own run and time limit), summarised
# into profiles/r05_<tag>_* and merged into profiles/pmc_latest.json (one
# set per channel count), copied back under gpurun_out/<tag>/profiles
#   bash tools/gpu_pmc.sh <tag> <channels>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1/profiles && export TMPDIR=/tmp &&
C=$2 &&
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-leg --no-duplex --no-side-legs --total-channels 0 --tx-channels 0 --rt-channels 0 --channels $C" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/prof_kt -o kt -- python3 bench.py --no-cpu-baseline --no-host-leg --no-duplex --no-side-legs --total-channels 0 --tx-channels 0 --rt-channels 0 --channels $C --steps 4 > gpurun_out/$1/prof_kt.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$1/pmc_fetch -o f -- python3 $B > gpurun_out/$1/pmc_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$1/pmc_write -o w -- python3 $B > gpurun_out/$1/pmc_write.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE -d gpurun_out/$1/pmc_a -o a -- python3 $B > gpurun_out/$1/pmc_a.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d gpurun_out/$1/pmc_b -o b -- python3 $B > gpurun_out/$1/pmc_b.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/$1/pmc_c -o c -- python3 $B > gpurun_out/$1/pmc_c.log 2>&1 &&
python3 tools/prof_summary.py gpurun_out/$1 r06_$1 $C > gpurun_out/$1/summary.log 2>&1 &&
cp profiles/r06_$1_* profiles/pmc_latest.json gpurun_out/$1/profiles/ &&
rm -rf gpurun_out/$1/pmc_fetch gpurun_out/$1/pmc_write gpurun_out/$1/pmc_a gpurun_out/$1/pmc_b gpurun_out/$1/pmc_c
