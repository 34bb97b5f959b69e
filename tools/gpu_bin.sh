# pitch-class lane order (engine.hip MELPE_BIN): GPU parity of encode, decode,
# ragged masks and state migration with the order on, then the encode +
# decode bench with it off (MELPE_BIN=0) and on at 262,144 and 32,768 channels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/bin && export TMPDIR=/tmp &&
timeout -k 10 500 python -u -m pytest tests/test_encode.py tests/test_decode.py tests/test_vad.py tests/test_state.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/bin/tests.log 2>&1 &&
B="bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0" &&
for C in 262144 32768; do
  MELPE_BIN=0 timeout -k 10 200 python $B --channels $C > gpurun_out/bin/off_$C.json 2> gpurun_out/bin/off_$C.err || exit 1
  timeout -k 10 200 python $B --channels $C > gpurun_out/bin/on_$C.json 2> gpurun_out/bin/on_$C.err || exit 1
done
