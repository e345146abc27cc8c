#!/usr/bin/env python3
"""Per-phase wave executions and lane occupancy from the -DRT4_LANESTATS diagnostic build.
Usage: RT4_LIB=<lanestats .so> python tools/lanestats.py [scene] [spp] [bounces]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

rt4 = importlib.import_module("4d_ray_tracing_amd")
scene = sys.argv[1] if len(sys.argv) > 1 else "sphere"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
bounces = int(sys.argv[3]) if len(sys.argv) > 3 else 8
t = rt4.Tracer(0, rt4.FLAG_SAMPLER_LUT | int(os.environ.get("RT4_EXTRA_FLAGS", "0"), 0), rt4.Scene.named(scene))
u = rt4.make_uniforms(1920, 1080, samples=spp, reflections=bounces, seed=12345)
frame = torch.zeros((1080, 1920, 4), device="cuda")
cnt = torch.zeros(64, dtype=torch.int64, device="cuda")
t.render_device(u, rt4.region(1920, 1080), frame.data_ptr(), 1920, cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
c = cnt.cpu().tolist()
names = ["loop iteration (active lanes)", "find (active)", "-", "miss", "hit", "reflect", "diffuse", "end of sample",
         "refill", "-"]
print(f"{scene} spp={spp} bounces={bounces} intersections={c[0]}")
for p, n in enumerate(names):
    e, l = c[16 + 2 * p], c[17 + 2 * p]
    if n == "-" or e == 0:
        continue
    print(f"  {n:>30s}: {e:12d} wave execs ({e / max(c[16], 1):5.3f} per iteration), {l / e:5.1f} lanes avg")
if c[40]:
    print(f"  {'exact sphere test (pending)':>30s}: {c[40]:12d} wave execs ({c[40] / max(c[16], 1):5.3f} per iteration), "
          f"{c[41] / c[40]:5.1f} lanes avg")
