# A/B of the current build against build/var/<variant>.so: encode/decode GPU
# parity on the current build, encode bench at 262,144 channels for both,
# then stage profiles of the current prof build and build/var/<variant>_prof.so
#   tools/gpu_ab2.sh <variant>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_encode.py tests/test_decode.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ab/tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --no-decode" &&
timeout -k 10 200 python $B --channels 262144 > gpurun_out/ab/cur.json 2> gpurun_out/ab/cur.err &&
MELPE_AMD_LIB=build/var/$1.so timeout -k 10 200 python $B --channels 262144 > gpurun_out/ab/$1.json 2> gpurun_out/ab/$1.err &&
timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/ab/stage_cur.txt 2> gpurun_out/ab/stage_cur.err &&
{ [ ! -f build/var/$1_prof.so ] || MELPE_AMD_LIB=build/var/$1_prof.so timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/ab/stage_$1.txt 2> gpurun_out/ab/stage_$1.err; }
