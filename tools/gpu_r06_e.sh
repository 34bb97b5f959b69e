# round 6: NPP workgroup size (channels per workgroup: npp2/4/8) and the LDS
# math tables (npp8nt: 8 per workgroup without them; npp1t: one per
# workgroup with them) against the product, 262,144 channels
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06e_262k 262144 cur npp8nt npp1t npp2 npp4 cur
