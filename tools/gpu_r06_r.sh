# round 6: the analysis waves' issue priority (MELPE_ANA_PRIO modes, k_ana.hip
# ana_wave_prio / ana_ckpt): per-wave end times of the serialised launch for
# each mode (build/var/wtp.so), then the bench step A/B (build/var/prio2.so)
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06r && mkdir -p $O && export TMPDIR=/tmp &&
for m in 0 1 3 5 6; do
  MELPE_ANA_PRIO=$m MELPE_AMD_LIB=build/var/wtp.so timeout -k 10 300 python3 -u tools/wave_times.py 262144 8 $O/wt_p$m.npz > $O/wt_p$m.jsonl 2> $O/wt_p$m.err || exit $?
  python3 tools/wave_place.py $O/wt_p$m.npz > $O/wt_p$m.txt || exit $?
done &&
bash tools/gpu_r05_ab.sh r06r_ab 262144 cur prio2:MELPE_ANA_PRIO=0 prio2:MELPE_ANA_PRIO=6 prio2:MELPE_ANA_PRIO=5 prio2:MELPE_ANA_PRIO=3 prio2:MELPE_ANA_PRIO=4 cur prio2:MELPE_ANA_PRIO=6 prio2:MELPE_ANA_PRIO=5 prio2:MELPE_ANA_PRIO=3
