# stage profile of the current build (split lane analysis), default input and
# every-channel-same input (divergence price)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$1 && export TMPDIR=/tmp &&
timeout -k 10 300 python tools/stage_prof.py 262144 3 > gpurun_out/$1/st.txt 2> gpurun_out/$1/st.err &&
timeout -k 10 300 python tools/stage_prof.py 262144 3 1 > gpurun_out/$1/st_same.txt 2> gpurun_out/$1/st_same.err
