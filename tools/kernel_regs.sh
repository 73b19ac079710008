#!/bin/bash
# Per-kernel register use / spills / occupancy of pathtrace.hip (device-only compile, a few seconds).
# usage: tools/kernel_regs.sh [extra hipcc flags]
cd "$(dirname "$0")/.." || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize \
  --cuda-device-only -c -o /dev/null -Iinclude -Irust_gpu_raytracing_amd/csrc "$@" \
  -Rpass-analysis=kernel-resource-usage rust_gpu_raytracing_amd/csrc/pathtrace.hip 2>&1 |
  grep -E "Function Name|VGPRs:|SGPRs Spill|VGPRs Spill|Occupancy" |
  sed -E 's/.*remark: //' | paste - - - - - | grep pathtrace_kernel |
  sed -E "s/Function Name: _Z19rt_pathtrace_kernelIL(i[0-9])ELj([0-9]+)ELb([01])ELb([01])EEv10KernelArgs/mode \1 threads \2 tris \3 wide \4/"
