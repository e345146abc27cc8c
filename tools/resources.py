#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / scratch / occupancy table from `make resource-usage` output on stdin."""
import re
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        name = m.group(1)
        k = re.search(r"rt4_(\w+?)_kernelI(?:Lj(\d+))?(?:ELb(\d))?", name)
        cur = {"name": (k.group(1) + ":" + (k.group(2) or "") + (":lut" if k.group(3) == "1" else "")) if k else name}
        rows.append(cur)
        continue
    for key, pat in (("sgpr", r"TotalSGPRs: (\d+)"), ("vgpr", r"VGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
for r in rows:
    if r["name"].startswith("trace"):
        print(f"{r['name']:>24s} vgpr {r.get('vgpr')} sgpr {r.get('sgpr')} scratch {r.get('scratch')} occ {r.get('occ')} lds {r.get('lds')}")
