#!/usr/bin/env python3
"""The reference's 4D view as a frame loop: three sections per frame (three_window_group.cpp:42-46, YXZ at the
main window's cells, YWZ and YXW at the additional window's), a moving camera (one launch per frame, main.cpp:93),
properties.txt's samples and bounces. Times K back-to-back rt4_render_sections_device calls with overlapped
launches (the default) and with RT4_FLAG_SERIAL_FRAMES, and checks that both give the same images and count.
Usage (GPU): python tools/sections_bench.py [--scene tiger] [--frames 40] [--scale 1]
--scale multiplies the windows' cell counts (1 = properties.txt: 121x75 and 60x37 cells)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scene", default="tiger")
    p.add_argument("--frames", type=int, default=40)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--scale", type=int, default=1)
    args = p.parse_args()
    import importlib

    import torch

    rt4 = importlib.import_module("4d_ray_tracing_amd.rt4")
    props = rt4.Properties(text=open(os.path.join(ROOT, "properties.txt")).read())
    cells = [rt4.window_cells(props, "main"), rt4.window_cells(props, "additional"), rt4.window_cells(props, "additional")]
    cells = [(w * args.scale, h * args.scale) for (w, h) in cells]
    secs = [rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW]
    bases = [rt4.uniforms_from_properties(props, w, h, s) for (w, h), s in zip(cells, secs)]
    result = {"scene": args.scene, "cells": cells, "samples": bases[0].samples,
              "bounces": bases[0].reflections_amount, "frames": args.frames}
    images = {}
    for label, flags in (("overlapped", rt4.FLAG_SAMPLER_LUT), ("serial", rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES)):
        t = rt4.Tracer(device=0, flags=flags, scene=rt4.Scene.named(args.scene))
        try:
            cam = rt4.Camera(props)
            frames = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for (w, h) in cells]
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            s = torch.cuda.current_stream()

            plan = []  # the camera path first (it does not depend on the frames), so the timed loop only submits
            for n in range(args.warmup + args.frames):
                jobs = []
                fn = cam.s.frame_number
                for q in range(3):
                    cam.s.frame_number = fn
                    u = cam.frame_uniforms(bases[q], secs[q], 1234 + n)
                    jobs.append((u, rt4.region(*cells[q]), frames[q].data_ptr(), cells[q][0]))
                plan.append(jobs)
                cam.move(rt4.KEY_FORWARD, 0.01)

            def frame(n):
                t.render_sections_device(plan[n], 0, cnt.data_ptr(), s.cuda_stream)

            for n in range(args.warmup):
                frame(n)
            torch.cuda.synchronize()
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for n in range(args.frames):
                frame(args.warmup + n)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.frames
            result[label] = {"ms_per_frame": ms, "intersections_per_frame": int(cnt.item()) / args.frames,
                             "G_int_per_s": int(cnt.item()) / args.frames / ms / 1e6}
            images[label] = [fr.cpu().numpy() for fr in frames]
        finally:
            t.close()
    result["same_images"] = all((a.view("u4") == b.view("u4")).all() for a, b in zip(images["overlapped"], images["serial"]))
    result["same_count"] = result["overlapped"]["intersections_per_frame"] == result["serial"]["intersections_per_frame"]
    print(json.dumps(result))
    if not (result["same_images"] and result["same_count"]):
        sys.exit(1)


if __name__ == "__main__":
    main()
