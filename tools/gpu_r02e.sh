# 2400 mode + codec parity after the lane_copy aliasing fix, then a bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 400 python -u -m pytest tests/test_r2400.py tests/test_encode.py tests/test_decode.py tests/test_npp.py tests/test_state.py -x -v -m gpu --timeout 250 --timeout-method thread > gpurun_out/e_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 > gpurun_out/e_bench.json 2> gpurun_out/e_bench.err
