# knockout pricing of the lane analysis at 262,144 channels: for the product
# build ("cur") and each build/var/ko_<stage>.so two PMC passes (FETCH_SIZE +
# SQ counters, whose bench line also gives the kernel times; WRITE_SIZE),
# each run under its own time limit
#   bash tools/gpu_r04_ko.sh <tag> cur bpvc pauto ...
cd $GRAFT_REPO_ROOT && T=$1 && shift && O=gpurun_out/$T && mkdir -p $O && export TMPDIR=/tmp &&
B="bench.py --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode --channels 262144 --steps 3 --warmup 1" &&
for v in "$@"; do
  echo "ko $v" >> $O/progress.log
  if [ $v = cur ]; then L=pairphone_amd/libmelpe_amd.so; else L=build/var/ko_$v.so; fi
  MELPE_AMD_LIB=$L timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $O/pmc_f_$v -o f -- python3 -u $B > $O/$v.json 2> $O/pmc_f_$v.log || exit $?
  MELPE_AMD_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w_$v -o w -- python3 -u $B > $O/pmc_w_$v.log 2>&1 || exit $?
done
