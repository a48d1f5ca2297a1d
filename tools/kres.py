#!/usr/bin/env python3
"""Per-kernel VGPR / scratch / occupancy of verify_kernels.hip for gfx950
(clang -Rpass-analysis=kernel-resource-usage), one line per kernel."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "bdls_amd/csrc/verify_kernels.hip"
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src,
                      "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = re.sub(r"\(anonymous namespace\)::|bh::", "", cur).split("(")[0]
        rows[cur] = {}
        continue
    m = re.search(r"(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" ")[0]] = int(m.group(2))
for k, v in rows.items():
    print(f"{k:70s} vgpr={v.get('VGPRs')} scratch={v.get('ScratchSize')} occ={v.get('Occupancy')}")
