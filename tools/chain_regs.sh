#!/bin/bash
# Register use of the rtc_render_chain instantiations for a set of -D flags: tools/chain_regs.sh [flags...]
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 --cuda-device-only "$@" \
  -c "$(dirname "$0")/../raytracingc_amd/csrc/rtc_render.hip" -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 |
  python3 -c '
import re, sys
cur = None
for l in sys.stdin:
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1) if "rtc_render_chain" in m.group(1) else None
        if cur:
            t = re.search(r"ILb([01])ELb([01])E", cur); print("\nchain<%s,%s>" % t.groups(), end="")
        continue
    m = re.search(r"remark:\s+(VGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", l)
    if cur and m:
        print(" %s=%s" % (m.group(1).split()[0] + ("_spill" if "Spill" in m.group(1) else ""), m.group(2)), end="")
print()'
