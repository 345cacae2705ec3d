#!/usr/bin/env python3
"""Per-kernel resource usage (VGPR/AGPR/SGPR/scratch/LDS/occupancy) of a HIP source for gfx950.

  python tools/kres.py pytorch_cifar_amd/csrc/conv_mfma.hip [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
       "--cuda-device-only", "--no-gpu-bundle-output", "-c", "-Ipytorch_cifar_amd/csrc", src,
       "-o", "/tmp/kres.co", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: (.*)", line)
    if not m:
        continue
    t = m.group(1).replace(" [-Rpass-analysis=kernel-resource-usage]", "")
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt in r["name"]:
        n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        n = re.sub(r"\(.*", "", n)
        print(f"{n:70s} V{r.get('VGPRs','?'):>4} A{r.get('AGPRs','?'):>4} S{r.get('SGPRs','?'):>4} "
              f"scr{r.get('ScratchSize [bytes/lane]','?'):>4} lds{r.get('LDS Size [bytes/block]','?'):>7} "
              f"occ{r.get('Occupancy [waves/SIMD]','?'):>3}")
