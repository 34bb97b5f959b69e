# one PMC pass per library variant (cur = product build, else build/var/<v>.so)
# on the 262,144-channel encode step: where the analysis' memory-pipeline
# work goes, by stage knockout
#   bash tools/gpu_ko_pmc.sh <tag> "<counters>" cur ko_bpvc ...
cd $GRAFT_REPO_ROOT && T=$1 && P=$2 && shift 2 && O=gpurun_out/$T && mkdir -p $O && export TMPDIR=/tmp &&
B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-leg --no-duplex --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144" &&
for v in "$@"; do
  echo "$v" >> $O/progress.log
  if [ $v = cur ]; then L=pairphone_amd/libmelpe_amd.so; else L=build/var/$v.so; fi
  MELPE_AMD_LIB=$L timeout -s KILL 240 rocprofv3 --pmc $P -d $O/pmc_$v -o p -- python3 $B > $O/$v.json 2> $O/$v.err || exit $?
  python3 tools/pmc_dump.py $O/pmc_$v > $O/dump_$v.txt 2>&1
done
