# arbitrary rocprofv3 --pmc passes over the encode step at one channel count
# (each pass its own run and time limit), dumped per kernel by
# tools/pmc_dump.py into gpurun_out/<tag>/pmc_dump.txt
#   bash tools/gpu_pmc_passes.sh <tag> <channels> "<counters of pass 1>" "<counters of pass 2>" ...
cd $GRAFT_REPO_ROOT && T=$1 && C=$2 && shift 2 && O=gpurun_out/$T && mkdir -p $O && export TMPDIR=/tmp &&
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-leg --no-duplex --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels $C" &&
i=0 &&
for p in "$@"; do
  i=$((i+1))
  echo "pass $i: $p" >> $O/progress.log
  timeout -s KILL 300 rocprofv3 --pmc $p -d $O/pmc_p$i -o p -- python3 $B > $O/pmc_p$i.log 2>&1 || exit $?
done &&
python3 tools/pmc_dump.py $O/pmc_p* > $O/pmc_dump.txt 2>&1
