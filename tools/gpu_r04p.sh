# scratch behaviour probe at two engine sizes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/p && export TMPDIR=/tmp &&
timeout -k 10 200 python -u tools/scratch_probe.py 65536 > gpurun_out/p/probe_65536.txt 2>&1 &&
timeout -k 10 200 python -u tools/scratch_probe.py 262144 > gpurun_out/p/probe_262144.txt 2>&1
