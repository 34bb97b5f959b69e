#!/bin/bash
# device-only compile of one kernel TU + per-kernel resource metadata
#   tools/kmeta.sh <tu> [extra hipcc flags...]     e.g. tools/kmeta.sh k_ana -DMELPE_INLINE_ALL
set -e
cd "$(dirname "$0")/.."
tu=$1; shift
mkdir -p /tmp/co
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 --cuda-device-only -c -Wno-unused-result -Wno-unused-value \
  -DMELPE_TABLES_BIN='"x"' -Ipairphone_amd/csrc "$@" pairphone_amd/csrc/$tu.hip -o /tmp/co/$tu$KTAG.co
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/co/$tu$KTAG.co \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/co/$tu$KTAG.elf 2>/dev/null || cp /tmp/co/$tu$KTAG.co /tmp/co/$tu$KTAG.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes /tmp/co/$tu$KTAG.elf | grep -E "^\s+\.name:|private_segment_fixed_size|\.vgpr_count|vgpr_spill|sgpr_spill" | paste - - - - - | sed 's/\s\+/ /g' | grep -v "derive"
