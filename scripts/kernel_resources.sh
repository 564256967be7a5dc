#!/bin/bash
# Per-kernel registers / scratch / occupancy / LDS of td_step.hip (a device-only compile
# with the kernel-resource-usage remarks):
#   bash scripts/kernel_resources.sh [extra hipcc flags]
cd "$(dirname "$0")/../gym-td_amd/csrc"
obj=$(mktemp /tmp/tdres_XXXXXX.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -w --cuda-device-only "$@" \
  -c td_step.hip -o "$obj" -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|SGPRs:|VGPRs:|ScratchSize|Occupancy|LDS Size" | paste - - - - - - |
  sed -E 's/td_step.hip:[0-9]*:[0-9]*: remark: //g; s/ \[-Rpass-analysis=kernel-resource-usage\]//g; s/Function Name: _ZN2td[0-9]+//; s/EEEvNS_8StepArgsE//; s/ScratchSize \[bytes\/lane\]/scratch/; s/Occupancy \[waves\/SIMD\]/occ/; s/LDS Size \[bytes\/block\]/lds/; s/TotalSGPRs/sgpr/; s/VGPRs/vgpr/' |
  awk '{$1=$1};1'
rm -f "$obj"
