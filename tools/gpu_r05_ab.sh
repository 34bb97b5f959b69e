# A/B of library builds and environment settings on the 262,144-channel
# encode + decode step (no PMC): one bench line per variant, each under its
# own time limit.  A variant is LIB[:ENV=VAL[,ENV=VAL]] with LIB = cur (the
# product build) or the name of build/var/<name>.so.
#   bash tools/gpu_r05_ab.sh <tag> <channels> cur cur:MELPE_BIN=0 ko_analysis ...
cd $GRAFT_REPO_ROOT && T=$1 && C=$2 && shift 2 && O=gpurun_out/$T && mkdir -p $O && export TMPDIR=/tmp &&
B="bench.py --no-cpu-baseline --no-host-leg --no-duplex --no-side-legs --total-channels 0 --tx-channels 0 --rt-channels 0 --channels $C --steps 6 --warmup 2" &&
i=0 &&
for v in "$@"; do
  i=$((i+1))
  lib=${v%%:*}
  envs=""
  if [ "$lib" != "$v" ]; then envs=$(echo ${v#*:} | tr ',' ' '); fi
  if [ $lib = cur ]; then L=pairphone_amd/libmelpe_amd.so; else L=build/var/$lib.so; fi
  echo "$i $v" >> $O/progress.log
  env MELPE_AMD_LIB=$L $envs timeout -k 10 300 python3 -u $B > $O/v$i.json 2> $O/v$i.err || exit $?
  echo "$i $v $(python3 -c "import json,sys; d=json.load(open('$O/v$i.json')); r=d['roofline']; print('step %.2f ana %.2f npp %.2f dec %.2f' % (d['ms_per_step'], r['kernel_ms'], r['kernels'][1]['kernel_ms'], (d['decode'] or {}).get('kernel_ms', -1)))")" >> $O/summary.txt
done
