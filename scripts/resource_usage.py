#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / scratch / occupancy of hb_kern_nl8.hip for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel."""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.join(ROOT, "heartbeat_amd", "csrc", os.environ.get("HB_RU_SRC", "hb_kern_nl8.hip"))
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src,
                      "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("TotalSGPRs", "VGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]"):
        m = re.search(key + r": (\d+)", ln)
        if m and cur is not None:
            cur[key.split()[0].split("\\")[0]] = int(m.group(1))
for r in rows:
    print("%-60s vgpr=%-4s sgpr=%-4s scratch=%-4s occ=%-2s lds=%s" % (
        r["name"][:60], r.get("VGPRs"), r.get("TotalSGPRs"), r.get("ScratchSize"), r.get("Occupancy"), r.get("LDS")))
