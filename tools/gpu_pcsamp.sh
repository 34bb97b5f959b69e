# PC sampling (host trap) over a short encode run of a -g build (build/var/dbg.so)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/dbg.so timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 -d gpurun_out/pcs -o pcs --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode --no-side-legs --total-channels 0 --tx-channels 0 --channels 262144 > gpurun_out/pcs.log 2>&1
