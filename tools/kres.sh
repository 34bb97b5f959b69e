#!/bin/bash
# per-kernel resources (VGPRs, spills, scratch, LDS) of a built TU object
#   tools/kres.sh build/obj/libmelpe_amd/k_ana_mw.o
set -e
t=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$t/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$t/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/dev.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $t/dev.elf |
  grep -E "^\s+\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill|sgpr_spill|group_segment_fixed" |
  paste - - - - - - | sed 's/\s\+/ /g' | grep -v derive
rm -rf $t
