# round 6: 8-channel NPP workgroups with a wave-uniform channel index, with
# (npp8u) and without (npp8ntu) the LDS math tables, against the product
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash tools/gpu_r05_ab.sh r06f_262k 262144 cur npp8u npp8ntu cur npp8u
