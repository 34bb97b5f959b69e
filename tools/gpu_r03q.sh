# kernel trace of the encode step with the bands split
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
MELPE_BANDS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$1/kt -o kt --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-side-legs --no-decode --total-channels 0 --tx-channels 0 --channels 262144 > gpurun_out/$1/b.json 2> gpurun_out/$1/b.err
