#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy table of mcc_kernels.hip (hipcc -Rpass-analysis=
kernel-resource-usage, device-only compile).  Usage: python tools/kres.py [filter]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-Wno-unused-function",
       "--cuda-device-only", "-c", f"{ROOT}/multi_camera_calibration_amd/csrc/mcc_kernels.hip", "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "Occupancy \\[waves/SIMD\\]", "LDS Size \\[bytes/block\\]",
                "ScratchSize \\[bytes/lane\\]"):
        m = re.search(r"\s" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split(" [")[0].replace("\\", "")] = int(m.group(1))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:70]:70s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>4} "
              f"vspill {r.get('VGPRs Spill', '?'):>4} sspill {r.get('SGPRs Spill', '?'):>4} scratch {r.get('ScratchSize', '?')}")
