# PC sampling (host trap) over a short encode run of a -g build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
MELPE_AMD_LIB=build/var/dbg.so timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d gpurun_out/pcs -o pcs -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-decode --channels 65536 > gpurun_out/pcs.log 2>&1
