# a variant library's 32,768-channel step against the product's, twice each
#   bash tools/gpu_r04v.sh <tag> <variant.so>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp
B="bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode --channels 32768"
for i in 1 2; do
timeout -k 10 200 env MELPE_AMD_LIB=$2 python -u $B > gpurun_out/$1/var$i.json 2> gpurun_out/$1/var$i.err || exit $?
timeout -k 10 200 python -u $B > gpurun_out/$1/cur$i.json 2> gpurun_out/$1/cur$i.err || exit $?
done
