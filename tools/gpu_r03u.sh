# smoke() on the committed build, then the 32,768-channel strong shard step
# (the multi-wave analysis with per-lane lsf row gathers)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$1/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-side-legs --total-channels 0 --tx-channels 0 --channels 32768 > gpurun_out/$1/bench_32k.json 2> gpurun_out/$1/bench_32k.err
