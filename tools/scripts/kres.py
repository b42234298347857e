#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage), one line per
kernel: VGPRs, SGPRs, spills, occupancy, LDS. Usage: kres.py <file.hip> [extra hipcc flags...]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-Iinclude", "-Ideepreadmapper_amd/csrc",
       "--offload-arch=gfx950", "-ffp-contract=off", "-munsafe-fp-atomics", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for f, r in rows.items():
    name = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
    name = re.sub(r"\(drm::SearchArgs\)|drm::\(anonymous namespace\)::", "", name)
    print(f"{name[:70]:70s} V{r.get('VGPRs','?'):>4} S{r.get('TotalSGPRs','?'):>4} "
          f"Vsp{r.get('VGPRs Spill','?'):>3} Ssp{r.get('SGPRs Spill','?'):>4} occ{r.get('Occupancy [waves/SIMD]','?'):>2} "
          f"lds{r.get('LDS Size [bytes/block]','?')}")
