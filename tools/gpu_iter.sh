# iteration check: encode/decode GPU parity, an encode-only bench at 262,144
# and 32,768 channels, and the stage profile (timer build) at 262,144
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_encode.py tests/test_decode.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/iter_tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
timeout -k 10 200 python $B > gpurun_out/iter_262k.json 2> gpurun_out/iter_262k.err &&
timeout -k 10 200 python $B --channels 32768 > gpurun_out/iter_32k.json 2> gpurun_out/iter_32k.err &&
timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/iter_stage.txt 2> gpurun_out/iter_stage.err
