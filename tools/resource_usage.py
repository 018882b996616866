#!/usr/bin/env python3
"""VGPR / SGPR / scratch / occupancy of every k_trace instantiation (hipcc resource remarks).

usage: python tools/resource_usage.py [extra hipcc -D flags]
Template arguments are printed as METHOD DISK SPIN0 FAR HUGE INL [ACC]."""
import os, re, subprocess, sys

src = os.path.join(os.path.dirname(__file__), "..", "raytracing-engine-in-c_amd", "csrc")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
       "-c", "geodesic.hip", "-o", "/tmp/_ru.co", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, cwd=src, capture_output=True, text=True).stderr
rows, cur = {}, None
for l in out.splitlines():
    m = re.search(r"Function Name: (\S+)", l)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s*(.*?):\s*(\S+)\s*\[", l)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    m = re.search(r"k_traceILi(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)EL[bi](\d)E(?:Lb(\d)E)?", k)
    if not m:
        continue
    print("k_trace<%s>" % ",".join(g for g in m.groups() if g is not None), "VGPR", v.get("VGPRs"), "SGPR", v.get("TotalSGPRs"),
          "scratch", v.get("ScratchSize [bytes/lane]"), "waves", v.get("Occupancy [waves/SIMD]"))
