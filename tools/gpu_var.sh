cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out &&
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 &&
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline" &&
timeout -k 10 300 python $B > gpurun_out/v1.json 2> gpurun_out/v1.err &&
MELPE_AMD_LIB=build/var/enc2.so timeout -k 10 300 python $B > gpurun_out/v2.json 2> gpurun_out/v2.err &&
MELPE_AMD_LIB=build/var/enc4.so timeout -k 10 300 python $B > gpurun_out/v4.json 2> gpurun_out/v4.err &&
timeout -k 10 300 python tools/stage_prof.py 65536 3 > gpurun_out/stage_prof.txt 2>&1
