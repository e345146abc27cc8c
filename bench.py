#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: ray-bounce intersections/s at 1080p x 16 spp x 8 bounces.

Workload (BASELINE.json configs[1]): the sphere+plane+sun scene
(scenes/Шар, плоскость и светилник.frag), 1920x1080 pixels per GPU, 16 samples, 8 reflections,
seed 12345, default camera, old_frame = 0, part = 1. One "step" = one frame = one launch of the trace
kernel over the rank's pixels. The unit is one find_intersection() call (shader.frag:475), counted
on the device by the kernel itself.

Multi-GPU (torchrun): weak scaling — each rank renders 1920x1080 pixels of a 1920x(1080*N) frame,
dealt in 8-row bands round-robin (4d_ray_tracing_amd/shard.py). The frame is assembled on rank 0 by
ONE RCCL gather after the K frames, inside the timed region (accumulate locally,
gather once); --gather every gathers after every frame instead.

Prints ONE JSON line on rank 0 with `roofline` (fp32 VALU: oracle-counted fp32 ops per unit x units
per launch / average kernel time, vs the 157.3 TFLOP/s gfx950 vector peak) and `cpu_baseline`
(the scalar C++ oracle on this host's cores, on a bounded row sample of the same frame).
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md "Peak FP32 (vector)"
METRIC = "ray-bounce intersections/s per GPU at 1080p·16spp·8bounce; %VALU roofline"


def parse_args():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scene", default="sphere")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080, help="rows per GPU")
    p.add_argument("--spp", type=int, default=16)
    p.add_argument("--bounces", type=int, default=8)
    p.add_argument("--seed", type=int, default=12345)
    p.add_argument("--no-lut", action="store_true", help="disable the w_by_volume table (inline Newton loop)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--format", choices=["f32", "f16", "rgba8"], default="f32", help="frame format (rt4_frame_format)")
    p.add_argument("--gather", choices=["final", "every"], default="final",
                   help="N > 1: one RCCL gather after the timed frames (default) or one per frame")
    return p.parse_args()


def cpu_threads():
    for k in ("OMP_NUM_THREADS", "RT4_CPU_THREADS"):
        if os.environ.get(k, "").isdigit():
            return max(1, int(os.environ[k]))
    return max(1, min(16, os.cpu_count() or 1))


def cpu_baseline(rt4, scene, u, width, height, target_s):
    """Oracle (scalar C++ restatement) on rows y = y0 + k*step of the same frame, all host threads."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: only the cpu_baseline leg loads it

    threads = cpu_threads()
    # probe: two rows on one thread each -> per-row cost; then size the sample for ~target_s
    probe = rt4.region(width, 2, y0=height // 3, band_rows=1, band_step=height // 3)
    t0 = time.perf_counter()
    oracle_lib.render(scene.desc, u, probe, threads=2)
    per_row = max((time.perf_counter() - t0) / 1.0, 1e-6)  # 2 rows on 2 threads ~ one row's time
    rows_wanted = max(threads, int(target_s * threads / per_row))
    step = max(1, height // rows_wanted)
    y0 = 3 % step
    reg = rt4.region(width, len(range(y0, height, step)), y0=y0, band_rows=1, band_step=step)
    n, dt, reps = 0, 0.0, 0
    while dt < target_s and reps < 100:  # a whole frame can take less than the target: repeat it
        t0 = time.perf_counter()
        _, k, _, _ = oracle_lib.render(scene.desc, u, reg, threads=threads)
        dt += time.perf_counter() - t0
        n += k
        reps += 1
    what = "the whole frame" if step == 1 else f"every {step}th row ({reg.h} of {height} rows)"
    return {"value": n / dt, "unit": "ray-bounce intersections/s", "cores": threads, "kind": "port",
            "sample": f"{what} x {width} px, {u.samples} spp, {u.reflections_amount} bounces, rendered {reps}x: "
                      f"{n} intersections in {dt:.1f} s; oracle/rt4_oracle.cpp (-O3, scalar) on {threads} host threads"}


def ops_per_unit(rt4, scene, u, width, height):
    """Algorithmic fp32 ops per find_intersection (+ its shading), counted by the oracle on every 64th row."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    reg = rt4.region(width, len(range(7, height, 64)), y0=7, band_rows=1, band_step=64)
    _, n, ops, _ = oracle_lib.render(scene.desc, u, reg, threads=cpu_threads(), count_ops=True)
    return ops / max(n, 1), n


def pmc_traffic(config):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of the same workload
    (profiles/pmc_<scene>.json, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config['scene']}.json")
    if not os.path.exists(path):
        return None, None
    d = json.load(open(path))
    keys = ("width", "height_per_gpu", "spp", "bounces", "seed", "sampler_lut")
    pc = dict(d.get("config", {}))
    pc.setdefault("frame_format", "f32")  # profiles before frame formats existed were float4
    if any(pc.get(k) != config[k] for k in keys + ("frame_format",)):
        return None, None
    return d["derived"].get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")

    plan = shard.make_plan(args.width, args.height, world, band=8)
    scene = rt4.Scene.named(args.scene)
    flags = 0 if args.no_lut else rt4.FLAG_SAMPLER_LUT
    tracer = rt4.Tracer(device=local_rank, flags=flags, scene=scene)
    u = rt4.make_uniforms(plan.width, plan.height, samples=args.spp, reflections=args.bounces, seed=args.seed)
    reg = rt4.region(**plan.region_args(rank))

    fmt = {"f32": rt4.FRAME_RGBA32F, "f16": rt4.FRAME_RGBA16F, "rgba8": rt4.FRAME_RGBA8}[args.format]
    tdt = {"f32": torch.float32, "f16": torch.float16, "rgba8": torch.uint8}[args.format]
    frame = torch.zeros((plan.rows_per_rank, plan.width, 4), dtype=tdt, device=dev)
    counter = torch.zeros(1, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    def render():
        tracer.render_device_ex(u, reg, frame.data_ptr(), fmt, plan.width, counter.data_ptr(), sptr)

    def step():
        render()
        if world > 1:
            shard.gather_frame(frame, plan, rank)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    counter.zero_()
    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        k_start[i].record(stream)
        render()
        k_end[i].record(stream)
        if world > 1 and args.gather == "every":
            shard.gather_frame(frame, plan, rank)
    g0 = torch.cuda.Event(enable_timing=True)
    g1 = torch.cuda.Event(enable_timing=True)
    g0.record(stream)
    if world > 1 and args.gather == "final":
        shard.gather_frame(frame, plan, rank)  # the frame assembled on rank 0
    g1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in zip(k_start, k_end)) / args.steps

    gather_ms = g0.elapsed_time(g1)
    n_local = int(counter.item())
    stats = torch.tensor([elapsed, float(n_local), kernel_ms], dtype=torch.float64, device=dev)
    if world > 1:
        t_max = stats[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        n_sum = stats[1:2].clone()
        dist.all_reduce(n_sum, op=dist.ReduceOp.SUM)
        k_max = stats[2:3].clone()
        dist.all_reduce(k_max, op=dist.ReduceOp.MAX)
        elapsed, n_total, kernel_ms = float(t_max.item()), float(n_sum.item()), float(k_max.item())
    else:
        n_total = float(n_local)

    if rank == 0:
        value = n_total / elapsed
        units_per_launch = n_local / args.steps
        opu, _ = ops_per_unit(rt4, scene, u, plan.width, plan.height)
        achieved = opu * units_per_launch / (kernel_ms * 1e-3) / 1e12
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "ray-bounce intersections/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (fixed-seed procedural scene, no dataset)",
            "config": {
                "workload": f"{args.scene} scene, {plan.width}x{plan.rows_per_rank} px per GPU "
                            f"(frame {plan.width}x{plan.height}), {args.spp} spp, {args.bounces} bounces, seed {args.seed}",
                "scene": args.scene, "width": plan.width, "height_per_gpu": plan.rows_per_rank,
                "spp": args.spp, "bounces": args.bounces, "seed": args.seed,
                "sampler_lut": not args.no_lut,
                "parallelism": f"pixel-bands x{world}" + (f" + RCCL gather ({args.gather})" if world > 1 else ""),
                "frame_format": args.format,
            },
            "gather_ms": gather_ms if world > 1 else 0.0,
            "intersections_per_step": n_total / args.steps,
            "nominal_bound_per_step": plan.width * plan.height * args.spp * (args.bounces + 1),
            "kernel_ms": kernel_ms,
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": PEAK_FP32_VALU_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_VALU_TFLOPS,
                "traffic": None,
                "ops_per_unit": opu,
                "note": "fp32 ops (fma=2) per find_intersection+shading counted by the oracle; see DESIGN.md §5",
            },
        }
        traffic, src = pmc_traffic(line["config"])
        line["roofline"]["traffic"] = traffic
        if src:
            line["roofline"]["traffic_source"] = src + " (rocprofv3 FETCH_SIZE*2 + WRITE_SIZE, per launch)"
            line["roofline"]["algorithmic_bytes_per_launch"] = plan.width * plan.rows_per_rank * 32
        if not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(rt4, scene, u, plan.width, plan.rows_per_rank, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    tracer.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
