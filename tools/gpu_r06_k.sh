# round 6: the pipelined encode with its NPP on the engine's cin stream:
# headline step pipelined vs serialised, the host-fed leg, config 3
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06k && mkdir -p $O && export TMPDIR=/tmp &&
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-duplex --no-side-legs --tx-channels 0 \
  --total-channels 0 > $O/bench.json 2> $O/bench.err &&
MELPE_AMD_LIB=pairphone_amd/libmelpe_amd.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_encode.py -m gpu -k "pipe or host" > $O/tests.txt 2>&1
