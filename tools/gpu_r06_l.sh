# round 6: the pipelined step with pipelined warm-up at 32,768 channels
# (the side stream made before the timed region) and 262,144
cd $GRAFT_REPO_ROOT && O=gpurun_out/r06l && mkdir -p $O && export TMPDIR=/tmp &&
timeout -k 10 600 python bench.py --channels 32768 --total-channels 32768 --steps 20 --warmup 5 --no-cpu-baseline \
  --no-host-leg --no-duplex --no-side-legs --tx-channels 0 --rt-channels 0 > $O/bench_32k.json 2> $O/bench_32k.err &&
timeout -k 10 600 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-duplex --no-side-legs --tx-channels 0 \
  --total-channels 0 > $O/bench.json 2> $O/bench.err
