# knockout timing: the encode bench (262,144 channels) on the current build
# and on each build/var/ko_<stage>.so (a build with that stage skipped), so
# each stage is priced by the kernel-time difference in product code
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ko && export TMPDIR=/tmp &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode --channels 262144" &&
timeout -k 10 200 python $B > gpurun_out/ko/cur.json 2> gpurun_out/ko/cur.err &&
for v in "$@"; do
  MELPE_AMD_LIB=build/var/ko_$v.so timeout -k 10 200 python $B > gpurun_out/ko/$v.json 2> gpurun_out/ko/$v.err || exit 1
done
