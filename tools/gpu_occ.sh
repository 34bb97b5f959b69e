# occupancy experiment on k_enc_ana: VGPR budget variants (build/var/w*.so)
# and LDS-capped residency (MELPE_ANA_LDS) at 262,144 and 32,768 channels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/occ && export TMPDIR=/tmp &&
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-side-legs --total-channels 0 --tx-channels 0" &&
for C in 262144 32768; do
  timeout -k 10 200 python $B --channels $C > gpurun_out/occ/base_$C.json 2> gpurun_out/occ/base_$C.err &&
  for v in w2 w1; do
    MELPE_AMD_LIB=build/var/$v.so timeout -k 10 200 python $B --channels $C > gpurun_out/occ/${v}_$C.json 2> gpurun_out/occ/${v}_$C.err || exit 1
  done &&
  for L in 40960 20480; do
    MELPE_ANA_LDS=$L timeout -k 10 200 python $B --channels $C > gpurun_out/occ/lds${L}_$C.json 2> gpurun_out/occ/lds${L}_$C.err || exit 1
  done || exit 1
done
