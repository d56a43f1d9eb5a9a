#!/bin/bash
# Kernel resource usage (VGPRs, SGPRs, scratch, occupancy) of the product kernels, from the compiler
# (runs here, no GPU): bash profiles/kres.sh [extra hipcc flags]
cd "$(dirname "$0")/../3dgs-raytrace_amd" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize -mllvm -amdgpu-mfma-vgpr-form=1 \
  --offload-device-only -c -o /tmp/kres.o csrc/${KRES_FILE:-gsrt_render.hip} -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -E "Function Name|VGPRs:|ScratchSize|Occupancy|LDS Size|TotalSGPRs:" | sed 's/.*remark: //; s/ \[-Rpass.*//' |
  paste - - - - - - | sed 's/\t/  /g; s/Function Name: //'
