#!/usr/bin/env python
"""Per-kernel VGPR / AGPR / scratch / occupancy of a HIP source compiled for gfx950.

    python tools/res_usage.py vrvq_amd/csrc/conv.hip
"""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "vrvq_amd/csrc/conv.hip"
cmd = ["hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-slp-vectorize",
       "--offload-arch=gfx950", "-c", src, "-o", "/tmp/res_usage.o", "-Iinclude",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"n": m.group(1)}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[-Rpass", line)
    if m and cur is not None:
        key = m.group(1).strip()
        cur[key] = m.group(2)
        if key.startswith("LDS Size"):
            name = subprocess.run(["c++filt", cur["n"]], capture_output=True, text=True).stdout.strip()
            print(f"{name[:100]:100s} vgpr={cur.get('VGPRs')} agpr={cur.get('AGPRs')} "
                  f"scratch={cur.get('ScratchSize [bytes/lane]')} occ={cur.get('Occupancy [waves/SIMD]')}")
