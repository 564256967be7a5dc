#!/bin/bash
# Register / scratch / LDS use of the kernels in one object file of the build:
#   bash scripts/co_meta.sh gym-td_amd/build/td_step_half.o
set -e
T=$(mktemp -d); trap "rm -rf $T" EXIT
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1" $T/x.o
$B/clang-offload-bundler --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co --unbundle
$B/llvm-readelf --notes $T/k.co | grep -E "^\s+\.name:|sgpr_count|vgpr_count|private_segment_fixed|group_segment_fixed|spill_count" | paste - - - - - - - | sed 's/  */ /g'
