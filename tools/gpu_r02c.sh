# config-5 scale parity + modem tests, then the default bench line
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 600 python -u -m pytest tests/test_scale.py::test_config5_tx_front_end_ragged_at_scale tests/test_modem.py -x -v -m gpu --timeout 500 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
