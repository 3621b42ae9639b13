#!/usr/bin/env python3
"""Compile a .hip file for gfx950 and print per-kernel VGPRs / scratch / occupancy / LDS.
Usage: tools/kres.py dprf_amd/csrc/dprf_kernels.hip"""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/tmp/kres.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: (?:\S+ )?\s*([A-Za-z /\[\]]+?): (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    dem = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip().split("(")[0]
    print("%-40s VGPR %-4s AGPR %-3s scratch %-5s occ %-2s LDS %s" % (dem[:40], v.get("VGPRs"), v.get("AGPRs"),
          v.get("ScratchSize [bytes/lane]"), v.get("Occupancy [waves/SIMD]"), v.get("LDS Size [bytes/block]")))
