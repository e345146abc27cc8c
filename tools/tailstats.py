#!/usr/bin/env python3
"""Frame-end tail of the persistent trace kernel, from the -DRT4_TAILSTATS diagnostic build (never the
shipped one): per-wave start, queue-empty and exit times (s_memrealtime, 100 MHz).
Usage: RT4_LIB=<tailstats .so> python tools/tailstats.py [scene] [width] [height] [spp] [bounces] [frames]
(frames > 1: one rt4_render_frames_device call of that many frames)"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

rt4 = importlib.import_module("4d_ray_tracing_amd")
scene = sys.argv[1] if len(sys.argv) > 1 else "sphere"
w, h = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 16
bounces = int(sys.argv[5]) if len(sys.argv) > 5 else 8
nfr = int(sys.argv[6]) if len(sys.argv) > 6 else 1
t = rt4.Tracer(0, rt4.FLAG_SAMPLER_LUT, rt4.Scene.named(scene))
u = rt4.make_uniforms(w, h, samples=spp, reflections=bounces, seed=12345)
frame = torch.zeros((h, w, 4), device="cuda")
cnt = torch.zeros(64 + 3 * 65536, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for rep in range(3):
    cnt.zero_()
    torch.cuda.synchronize()
    if nfr > 1:
        t.reserve_frames(w, h)
        t.render_frames_device([u] * nfr, rt4.region(w, h), frame.data_ptr(), 0, w, cnt.data_ptr(), s)
    else:
        t.render_device(u, rt4.region(w, h), frame.data_ptr(), w, cnt.data_ptr(), s)
    torch.cuda.synchronize()
v = cnt[64:].view(-1, 3).cpu()
v = v[v[:, 2] > 0].double() * 10e-3  # 100 MHz ticks -> us
t0 = v[:, 0].min()
start, exh, end = v[:, 0] - t0, v[:, 1] - t0, v[:, 2] - t0
span = end.max().item()
busy = (end - start).sum().item()
first_exh = exh[exh > -t0 + 1].min().item()
print(f"{scene} {w}x{h} spp {spp} bounces {bounces} frames {nfr}: {len(v)} waves, kernel span {span:.1f} us, "
      f"{int(cnt[0].item())} intersections")
print(f"  wave start spread {start.max().item():.1f} us; queue empty at {first_exh:.1f} us "
      f"({first_exh / span * 100:.1f} % of the span)")
print(f"  wave exits: first {end.min().item():.1f} us, median {end.median().item():.1f} us, last {span:.1f} us")
print(f"  wave-slot occupancy over the span {busy / (len(v) * span) * 100:.1f} %; after the queue emptied "
      f"{((end - first_exh).clamp(min=0).sum().item()) / (len(v) * (span - first_exh)) * 100:.1f} %")
for q in (0.5, 0.9, 0.99):
    print(f"  {q * 100:.0f} % of waves exited by {end.quantile(q).item():.1f} us")
