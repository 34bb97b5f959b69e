# stage profiles of two stage-timer builds over the same input (A/B of where
# the analysis time goes): the current libmelpe_amd_prof.so and build/var/$1.so
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/st && export TMPDIR=/tmp &&
timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/st/cur.txt 2> gpurun_out/st/cur.err &&
MELPE_AMD_LIB=build/var/$1.so timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/st/$1.txt 2> gpurun_out/st/$1.err
