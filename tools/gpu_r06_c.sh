# round 6: FLAT guard off in k_enc_ana (noguard) against the product at
# 262,144 channels; two-wave decoder variants (batched run reads: dec2b;
# one 64-channel group per workgroup: *g1) at 32,768 and 65,536
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06c_262k 262144 base noguard base noguard &&
bash tools/gpu_r05_ab.sh r06c_32k 32768 dec2 dec2b dec2g1 dec2bg1 &&
bash tools/gpu_r05_ab.sh r06c_65k 65536 dec2 dec2b dec2g1 dec2bg1 &&
mkdir -p gpurun_out/r06c && timeout -k 10 120 build/exp/record_layout > gpurun_out/r06c/record_layout.jsonl 2> gpurun_out/r06c/record_layout.err
