#!/usr/bin/env python3
"""Per-kernel VGPR / LDS / occupancy from hipcc -Rpass-analysis=kernel-resource-usage.
    python tools/resources.py <file.hip> [extra hipcc args]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-o", "/dev/null", src,
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    n = r["name"]
    m = re.search(r"k_axis_fastILi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELi(\d+)ELi(\d+)ELi(\d+)E", n)
    if m:
        n = "fast N=%s P=%s R0=%s row=%s T=%s mode=%s flags=%s" % m.groups()
    print(f"{n[:70]:70s} vgpr={r.get('vgpr')} lds={r.get('lds')} occ={r.get('occ')} scratch={r.get('scratch')}")
