#!/bin/bash
# Resource usage (VGPRs, SGPRs, spills, occupancy, LDS) of the trace kernels from the compiler's remarks.
# usage: tools/kres.sh [extra hipcc flags]   (prints one line per trace kernel instantiation)
cd "$(dirname "$0")/../cuda-raytracer_amd"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-fast-math \
  -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I../include -Ihost -Icsrc \
  --cuda-device-only -Rpass-analysis=kernel-resource-usage "$@" -c csrc/rt_render.hip -o /tmp/kres_dev.o 2>&1 | \
python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1) if "trace" in m.group(1) else None
        if cur: print(); print(re.sub(r"EEEvNS_8DevScene.*", "", cur.replace("_ZN12_GLOBAL__N_1", "")), end="")
        continue
    m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\S+)", line)
    if cur and m: print(" %s=%s" % (m.group(1).split()[0], m.group(2)), end="")
print()'
