#!/usr/bin/env python3
"""Kernel resource usage of one HIP source (VGPRs, AGPRs, scratch, occupancy)
from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
    python3 scripts/kres.py audio-network_amd/csrc/goertzel.hip [name-regex]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
       "-mcode-object-version=5", "-Iinclude", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for ln in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", ln)
    if not m:
        continue
    s = m.group(1)
    if s.startswith("Function Name:"):
        cur = {"name": s.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in s:
        k, v = s.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    nm = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    nm = nm.replace("fskd::", "").split("(")[0]
    if pat and not pat.search(nm):
        continue
    print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('AGPRs', '0'):>3} agpr "
          f"{r.get('ScratchSize [bytes/lane]', '?'):>4} scr occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {nm}")
