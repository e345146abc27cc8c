#!/usr/bin/env python3
"""Table of bench.py JSON lines (tools/scenes_bench.sh output)."""
import json
import sys

for line in open(sys.argv[1]):
    if line.startswith("=="):
        last = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    c = d["config"]
    r = d["roofline"]
    print(f"{c['scene']:>18s} {c['width']}x{c['height_per_gpu']} spp{c['spp']:<3d} b{c['bounces']:<3d} "
          f"{c.get('frame_format', 'f32'):>5s} {d['value'] / 1e9:7.2f} G int/s  kernel {d['kernel_ms']:8.3f} ms  "
          f"VALU frac {r['frac'] * 100:5.2f}%  ops/unit {r['ops_per_unit']:.0f}")
