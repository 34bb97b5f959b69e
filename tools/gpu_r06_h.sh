# round 6: k_enc_ana compiled with other AMDGPU scheduling strategies
# (max-ilp, latency over occupancy, max-memory-clause) against the product
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06h_262k 262144 cur schilp schbias schclause cur
