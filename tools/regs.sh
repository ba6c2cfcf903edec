#!/bin/bash
# Register / occupancy report of the device kernels (compile only, no GPU needed).
cd "$(dirname "$0")/.." && cd /tmp && /opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  --offload-arch=gfx950 -c --cuda-device-only -Rpass-analysis=kernel-resource-usage "$@" \
  /root/repo/rsmcrt_amd/csrc/smcrt.hip -o /tmp/smcrt_dev.o 2>&1 |
  grep -E "Function Name|VGPRs:|SGPRs Spill|VGPRs Spill|Occupancy|LDS Size|ScratchSize" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//'
