#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / scratch / occupancy / LDS of one HIP source, one line per kernel.
usage: tools/resources.py statecatcher_amd/csrc/lucy_scan.hip [name-filter]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "statecatcher_amd", "csrc"),
       "-c", src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: +(.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '?'):>3} agpr "
              f"{r.get('ScratchSize [bytes/lane]', '?'):>4} scratch "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>2} occ  {r['name']}")
