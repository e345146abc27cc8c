#!/usr/bin/env python3
"""Per-phase wave executions and lane occupancy from the -DRT4_LANESTATS diagnostic build.

Usage: RT4_LIB=<lanestats .so> python tools/lanestats.py [scene] [spp] [bounces] [W] [H] [frames] [mode]
  mode: "pipelined" (frames in one rt4_render_frames_device call) or "fbf" (one launch per frame).
The counters accumulate over every launch of the run (counter[16..] per phase, counter[40..41] exact
sphere trips, counter[60..71] tiger tests)."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

rt4 = importlib.import_module("4d_ray_tracing_amd")
a = sys.argv[1:]
scene = a[0] if len(a) > 0 else "sphere"
spp = int(a[1]) if len(a) > 1 else 16
bounces = int(a[2]) if len(a) > 2 else 8
W = int(a[3]) if len(a) > 3 else 1920
H = int(a[4]) if len(a) > 4 else 1080
frames = int(a[5]) if len(a) > 5 else 1
mode = a[6] if len(a) > 6 else "fbf"
t = rt4.Tracer(0, rt4.FLAG_SAMPLER_LUT | int(os.environ.get("RT4_EXTRA_FLAGS", "0"), 0), rt4.Scene.named(scene))
u = rt4.make_uniforms(W, H, samples=spp, reflections=bounces, seed=12345)
frame = torch.zeros((H, W, 4), device="cuda")
cnt = torch.zeros(80, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
if mode == "pipelined" and frames > 1:
    t.reserve_frames(W, H)
ev0.record()
if mode == "pipelined":
    t.render_frames_device([u] * frames, rt4.region(W, H), frame.data_ptr(), 0, W, cnt.data_ptr(), s)
else:
    for _ in range(frames):
        t.render_device(u, rt4.region(W, H), frame.data_ptr(), W, cnt.data_ptr(), s)
ev1.record()
torch.cuda.synchronize()
c = cnt.cpu().tolist()
names = ["loop iteration (active lanes)", "find (active)", "-", "miss", "hit", "reflect", "diffuse", "end of sample",
         "refill", "parked / held"]
print(f"{scene} {W}x{H} spp={spp} bounces={bounces} frames={frames} {mode} frames/launch="
      f"{t.frames_per_launch(W, H) if mode == 'pipelined' else 1}: intersections={c[0]}, "
      f"{ev0.elapsed_time(ev1) / frames:.3f} ms/frame (lanestats build)")
for p, n in enumerate(names):
    e, l = c[16 + 2 * p], c[17 + 2 * p]
    if n == "-" or e == 0:
        continue
    print(f"  {n:>30s}: {e:12d} wave execs ({e / max(c[16], 1):5.3f} per iteration), {l / e:5.1f} lanes avg")
if c[40]:
    print(f"  {'exact sphere test (pending)':>30s}: {c[40]:12d} wave execs ({c[40] / max(c[16], 1):5.3f} per iteration), "
          f"{c[41] / c[40]:5.1f} lanes avg")
if c[58]:
    print(f"  {'hypercube cell test (pending)':>30s}: {c[58]:12d} wave execs ({c[58] / max(c[16], 1):5.3f} per iteration), "
          f"{c[59] / c[58]:5.1f} lanes avg")
if c[60]:
    print(f"  {'tiger test':>30s}: {c[60]:12d} wave execs ({c[60] / max(c[16], 1):5.3f} per iteration), "
          f"{c[61] / c[60]:5.1f} lanes avg")
if any(c[64:68]):
    print("  tiger tests by lanes needing them (share of tests, lanes avg):")
    for k, lab in enumerate(["1-16", "17-32", "33-48", "49-64"]):
        if c[64 + k]:
            print(f"    {lab:>6s}: {c[64 + k] / c[60]:6.3f}  {c[68 + k] / c[64 + k]:5.1f}")
if any(c[42:49]):
    tot = sum(c[42:49])
    print("  finds with pending spheres, by lanes pending (wave events share, lanes avg):")
    for k, lab in enumerate(["1", "2", "3-4", "5-8", "9-16", "17-32", "33-64"]):
        if c[42 + k]:
            print(f"    {lab:>6s}: {c[42 + k] / tot:6.3f}  {c[50 + k] / c[42 + k]:5.1f}")
print(f"  iterations per intersection: {c[16] / max(c[0], 1):.4f}")
