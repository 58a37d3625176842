#!/usr/bin/env python
"""Per-kernel resource table from hipcc -Rpass-analysis=kernel-resource-usage.
Usage: tools/kres.py csrc/file.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I../include", "-c", src,
                      "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if flt in k:
        dem = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
        print(f"{dem[:90]:90s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} occ={v.get('Occupancy [waves/SIMD]')} "
              f"lds={v.get('LDS Size [bytes/block]')} spill={v.get('VGPRs Spill')}/{v.get('SGPRs Spill')}")
