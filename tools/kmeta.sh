#!/bin/bash
# device-only compile of engine.hip + per-kernel resource metadata
set -e
cd "$(dirname "$0")/.."
mkdir -p /tmp/co
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 --cuda-device-only -c -Wno-unused-result -Wno-unused-value \
  -DMELPE_TABLES_BIN='"x"' -Ipairphone_amd/csrc "$@" pairphone_amd/csrc/engine.hip -o /tmp/co/k.co
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/co/k.co \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/co/k.elf
/opt/rocm/lib/llvm/bin/llvm-readelf --notes /tmp/co/k.elf | grep -E "^\s+\.name:|private_segment_fixed_size|\.vgpr_count|agpr_count|vgpr_spill|sgpr_spill" | paste - - - - - - | sed 's/\s\+/ /g' | grep -v "synth\|init_tables\|k_reset\|share\|melpe_i"
