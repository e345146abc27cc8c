#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: ray-bounce intersections/s at 1080p x 16 spp x 8 bounces.

Workload (BASELINE.json configs[1], SURVEY.md §8(d) config 2, the default): the sphere+plane+sun
scene (scenes/Шар, плоскость и светилник.frag), 1920x1080 pixels per GPU, 16 samples, 8 reflections,
seed 12345, default camera, old_frame = 0, part = 1. One "step" = one frame of the rank's pixels; the K
timed frames go to the library in one rt4_render_frames_device call (frames pipelined through one pixel
queue, up to 64 per launch, then blended in order: the same final image as K launches), or one launch
per frame with --frame-by-frame or a gather after every frame. The unit is one find_intersection() call (shader.frag:475), counted
on the device by the kernel itself. `value` is the whole job's units / time (all ranks);
`value_per_gpu` divides by the GPU count.

--config picks another BASELINE config (the other fields default to it):
  2  sphere, 1920x1080 per GPU, 16 spp, 8 bounces, fp32 frame              (weak scaling)
  3  hypercube, same shape                                                 (weak scaling)
  4  tiger_two_mirrors, one 3840x2160 frame, 64 spp, 12 bounces            (strong: the frame is split)
  5  all_primitives, one 3840x2160 frame, 16 spp per progressive frame (part = 1/n, seed_n), 8 bounces,
     fp16 accumulator; --steps 256 (+ warmup) reaches 4096 spp            (strong)

Multi-GPU. `python bench.py --gpus N` starts N ranks itself (torch.distributed.run on 127.0.0.1, one
process per GPU, before anything touches a GPU) unless it already runs under a launcher
(WORLD_SIZE set). Pixel bands of 8 rows are dealt round-robin over the ranks
(4d_ray_tracing_amd/shard.py; any frame height, ragged last band); RCCL gathers the padded shards to
rank 0, which un-permutes them on the device.
  weak   (configs 2, 3): every rank renders width x height pixels of a width x (height*N) frame; ONE
         gather after the K frames, inside the timed region; --gather every: per frame.
  strong (configs 4, 5, or --strong): the width x height frame is split over the N ranks; config 4
         gathers every frame (each frame is a finished image), config 5 once after the progressive
         frames. Rank 0 first renders the whole frame alone (the T1 leg, same steps) and the line
         reports efficiency = T1 / (N * T_N), both including what the N-rank run does per step.

The JSON line carries `roofline` (fp32 VALU: oracle-counted fp32 ops per unit x units per launch /
average kernel time from HIP events on the launch stream, vs the 157.3 TFLOP/s gfx950 vector peak;
`frac_executed` drops the Newton-loop ops the sampler table replaces), `setup_ms` (context + sampler
table, scene upload + verification) and `cpu_baseline` (the scalar C++ oracle on this job's host
CPUs, on a bounded row sample of the same frame). `dtype` is the arithmetic type (fp32 in every
frame format: the blend is fp32, rt4.h rt4_frame_format); `accumulator` is the frame's storage type.
"""
import argparse
import glob
import importlib
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP32_VALU_TFLOPS = 157.3  # MI355X_MICROARCH.md "Peak FP32 (vector)"
# the same peak in VALU lane-operations: 256 CUs x 4 SIMDs x 32 lanes per cycle (a wave64 VALU instruction
# issues over 2 cycles, MI355X_MICROARCH.md) x 2.4 GHz; 157.3 TFLOP/s counts an fma as 2 FLOP
PEAK_VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E ~8 TB/s
METRIC = "ray-bounce intersections/s per GPU at 1080p·16spp·8bounce; %VALU roofline"  # BASELINE.json, verbatim
# `value` is the whole job's rate (the bench contract); at N = 1 it is the metric's per-GPU rate, and for N > 1
# the line also carries value_per_gpu = value / N

CONFIGS = {  # BASELINE.json configs[1..4]
    2: dict(scene="sphere", width=1920, height=1080, spp=16, bounces=8, format="f32", mode="weak", progressive=False),
    3: dict(scene="hypercube", width=1920, height=1080, spp=16, bounces=8, format="f32", mode="weak", progressive=False),
    4: dict(scene="tiger_two_mirrors", width=3840, height=2160, spp=64, bounces=12, format="f32", mode="strong",
            progressive=False),
    5: dict(scene="all_primitives", width=3840, height=2160, spp=16, bounces=8, format="f16", mode="strong",
            progressive=True),
}


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", type=int, choices=sorted(CONFIGS), default=2)
    p.add_argument("--scene")
    p.add_argument("--width", type=int)
    p.add_argument("--height", type=int, help="weak: rows per GPU; strong: rows of the frame")
    p.add_argument("--spp", type=int)
    p.add_argument("--bounces", type=int)
    p.add_argument("--seed", type=int, default=12345)
    p.add_argument("--format", choices=["f32", "f16", "rgba8"], help="frame format (rt4_frame_format)")
    g = p.add_mutually_exclusive_group()
    g.add_argument("--strong", dest="mode", action="store_const", const="strong", help="split one fixed frame")
    g.add_argument("--weak", dest="mode", action="store_const", const="weak", help="fixed pixels per GPU")
    p.add_argument("--progressive", action="store_true", default=None, help="part = 1/n, seed_n per step")
    p.add_argument("--gather", choices=["final", "every"], help="N > 1: RCCL gather once after the frames or per frame")
    p.add_argument("--no-t1", action="store_true", help="strong, N > 1: skip rank 0's whole-frame leg")
    p.add_argument("--no-lut", action="store_true", help="disable the w_by_volume table (inline Newton loop)")
    p.add_argument("--primary-reuse", action="store_true",
                   help="RT4_FLAG_PRIMARY_REUSE for the main leg: value becomes reference-equivalent (labelled)")
    p.add_argument("--no-reuse-leg", action="store_true", help="skip the extra primary-reuse leg (N = 1)")
    p.add_argument("--no-fbf-leg", action="store_true", help="skip the extra frame-by-frame leg (N = 1)")
    p.add_argument("--no-sections-leg", action="store_true", help="skip the extra 4D-view frame-loop leg (N = 1)")
    p.add_argument("--no-steady-leg", action="store_true", help="skip the extra sustained-clock leg (N = 1)")
    p.add_argument("--hw-queues", type=int, default=8,
                   help="GPU_MAX_HW_QUEUES for this process (0: keep the environment's)")
    p.add_argument("--frame-by-frame", action="store_true",
                   help="one launch per frame (rt4_render_device_ex) instead of the pipelined frames of "
                        "rt4_render_frames_device (always so with a gather after every frame)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-ops", action="store_true", help="skip the oracle op count (profiling passes)")
    a = p.parse_args(argv)
    c = CONFIGS[a.config]
    for k in ("scene", "width", "height", "spp", "bounces", "format", "mode", "progressive"):
        if getattr(a, k, None) is None:
            setattr(a, k, c[k])
    if a.gather is None:
        a.gather = "final" if (a.mode == "weak" or a.progressive) else "every"
    return a


# ------------------------------------------------------------------------------------------ host CPUs
def host_cpus():
    """CPUs this job may use: the affinity set, capped by the cgroup CPU quota and by the harness's
    per-GPU share (OMP_NUM_THREADS, 16 on the GPU box, where nproc shows the whole machine)."""
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    if quota:
        usable = min(usable, max(1, math.floor(quota)))
    share = os.environ.get("RT4_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    threads = min(usable, int(share)) if share and share.isdigit() and int(share) > 0 else usable
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"threads": max(1, threads), "nproc": nproc, "usable": usable, "cgroup_quota": quota,
            "share_env": share, "model": model}


def new_constants_scene(rt4, scene):
    """A copy of the scene whose radii and sun angular size are scaled by 1.0078125 (exact in fp32), so
    that rt4_context_set_scene has new divisors and a new sky threshold to verify (setup_ms)."""
    d = type(scene.desc).from_buffer_copy(scene.to_bytes())
    k = 1.0078125
    for i in range(d.n_spheres):
        d.spheres[i].r *= k
    for i in range(d.n_cylinders):
        d.cylinders[i].r *= k
    for i in range(d.n_unions):
        d.unions[i].cylinder1.r *= k
        d.unions[i].cylinder2.r *= k
    for i in range(d.n_tigers):
        t = d.tigers[i]
        for c in (t.inner_cyl1, t.outer_cyl1, t.inner_cyl2, t.outer_cyl2):
            c.r *= k
    d.sun.angular_size *= k
    return rt4.Scene(d)


def row_region(rt4, width, height, rows_wanted, y0_hint=3):
    step = max(1, height // max(1, rows_wanted))
    y0 = y0_hint % step
    return rt4.region(width, len(range(y0, height, step)), y0=y0, band_rows=1, band_step=step), step


def cpu_baseline(rt4, scene, u, width, height, target_s, cpus):
    """Oracle (scalar C++ restatement) on rows y = y0 + k*step of the same frame, on this job's CPUs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib  # test infrastructure: only the cpu_baseline / op-count legs load it

    threads = cpus["threads"]
    # probe: two rows on two threads ~ one row's time; then size the sample for ~target_s
    probe = rt4.region(width, 2, y0=height // 3, band_rows=1, band_step=max(1, height // 3))
    t0 = time.perf_counter()
    oracle_lib.render(scene.desc, u, probe, threads=2)
    per_row = max(time.perf_counter() - t0, 1e-6)
    reg, step = row_region(rt4, width, height, int(target_s * threads / per_row))
    n, dt, reps = 0, 0.0, 0
    while dt < target_s and reps < 100:  # a whole frame can take less than the target: repeat it
        t0 = time.perf_counter()
        _, k, _, _ = oracle_lib.render(scene.desc, u, reg, threads=threads)
        dt += time.perf_counter() - t0
        n += k
        reps += 1
    what = "the whole frame" if step == 1 else f"every {step}th row ({reg.h} of {height} rows)"
    return {"value": n / dt, "unit": "ray-bounce intersections/s", "cores": threads, "kind": "port",
            "nproc": cpus["nproc"], "cpu_model": cpus["model"], "cpus_usable": cpus["usable"],
            "sample": f"{what} x {width} px, {u.samples} spp, {u.reflections_amount} bounces, rendered {reps}x: "
                      f"{n} intersections in {dt:.1f} s; oracle/rt4_oracle.cpp (-O3, scalar) on {threads} threads "
                      f"(this GPU's CPU share; nproc {cpus['nproc']}, {cpus['model']})"}


def ops_per_unit(rt4, scene, u, width, height, threads):
    """Algorithmic fp32 ops per find_intersection (+ its shading), counted by the oracle on ~16 rows
    of the same frame: (all ops, ops without the Newton loop the sampler table replaces, units)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    reg, _ = row_region(rt4, width, height, 16, y0_hint=7)
    n, ops, sampler_ops = oracle_lib.count_ops(scene.desc, u, reg, threads=threads)
    n = max(n, 1)
    return ops / n, (ops - sampler_ops) / n, n


def gather_ceiling():
    """Random 4-B gathers per second from a 32 MiB table with every CU issuing (the sampler table's size and
    access pattern; tools/mall_probe.hip on an MI355X, profiles/r03_mall/probe.json), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "r03_mall", "probe.json")))
        return next(r["G_gathers_per_s"] for r in d["results"] if r["table_mib"] == 32) * 1e9
    except (OSError, ValueError, KeyError, StopIteration):
        return None


def pmc_profile(config, frames_per_dispatch):
    """The committed rocprofv3 PMC summary (profiles/**/pmc_*.json, tools/pmc_summary.py) of the same
    workload, kernel version and launch shape (frames per pipelined dispatch) as this run, or None."""
    keys = ("scene", "width", "height_per_gpu", "spp", "bounces", "seed", "sampler_lut", "frame_format",
            "kernel_version", "progressive")
    # the newest round's profile first (profiles/r06_v52 before profiles/r05_v52); only the per-config summaries
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "pmc_config*.json"), recursive=True), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        pc = d.get("config", {})
        if all(pc.get(k) == config.get(k) for k in keys) and d.get("frames_per_dispatch", 1) == frames_per_dispatch:
            return d, os.path.relpath(path, ROOT)
    return None, None


# ------------------------------------------------------------------------------------------ launcher
def spawn_ranks(args):
    """`--gpus N` outside a launcher: N fresh processes via torch.distributed.run (this process has
    not touched a GPU), then exit with their status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)



def sections_loop_leg(rt4, torch, gpu, flags, scene, stream, tracer, frames=40, warmup=10):
    """Extra leg (N = 1): the reference's 4D view as its frame loop runs it (three_window_group.cpp:42-46, main.cpp:93):
    three sections per frame at properties.txt's window cells (YXZ at the main window's, YWZ and YXW at the
    additional one's), its samples and bounces, the bench's scene, a moving camera, one rt4_render_sections_device
    call per frame. Timed with the launches overlapped (the default; on the bench's own context, as an application
    with one context runs it) and with RT4_FLAG_SERIAL_FRAMES (a second context); the images and counts of the two
    must agree bit for bit. Reported beside the headline, never as value."""
    props = rt4.Properties(text=open(os.path.join(ROOT, "properties.txt")).read())
    cells = [rt4.window_cells(props, "main"), rt4.window_cells(props, "additional"), rt4.window_cells(props, "additional")]
    secs = [rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW]
    bases = [rt4.uniforms_from_properties(props, w, h, q) for (w, h), q in zip(cells, secs)]
    sptr = stream.cuda_stream
    out, images = {}, {}
    for label, fl in (("overlapped", flags), ("serial", flags | rt4.FLAG_SERIAL_FRAMES)):
        t = tracer if label == "overlapped" else rt4.Tracer(device=gpu, flags=fl, scene=scene)
        try:
            cam = rt4.Camera(props)
            imgs = [torch.zeros((h, w, 4), dtype=torch.float32, device=f"cuda:{gpu}") for (w, h) in cells]
            cnt = torch.zeros(1, dtype=torch.int64, device=f"cuda:{gpu}")

            plan = []  # the camera path first (it does not depend on the frames), so the timed loop only submits
            for n in range(warmup + frames):
                fn = cam.s.frame_number
                jobs = []
                for q in range(3):
                    cam.s.frame_number = fn
                    jobs.append((cam.frame_uniforms(bases[q], secs[q], 4242 + n), rt4.region(*cells[q]),
                                 imgs[q].data_ptr(), cells[q][0]))
                plan.append(jobs)
                cam.move(rt4.KEY_FORWARD, 0.01)

            def frame(n):
                t.render_sections_device(plan[n], rt4.FRAME_RGBA32F, cnt.data_ptr(), sptr)

            for n in range(warmup):
                frame(n)
            torch.cuda.synchronize()
            cnt.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            for n in range(frames):
                frame(warmup + n)
            e1.record(stream)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            n_int = int(cnt.item())
            out[label] = {"ms_per_frame": el / frames * 1e3, "kernel_ms_per_frame": e0.elapsed_time(e1) / frames,
                          "value": n_int / el, "intersections_per_frame": n_int / frames}
            images[label] = [x.cpu().numpy() for x in imgs]
        finally:
            if t is not tracer:
                t.close()
    same = all((a.view("u4") == b.view("u4")).all() for a, b in zip(images["overlapped"], images["serial"]))
    same = same and out["overlapped"]["intersections_per_frame"] == out["serial"]["intersections_per_frame"]
    if not same:
        raise SystemExit("sections leg: overlapped and serial launches differ")
    return {"label": "the 4D view's frame loop: three sections per frame at properties.txt's cells "
                     f"({cells[0][0]}x{cells[0][1]}, 2x {cells[1][0]}x{cells[1][1]}), {bases[0].samples} spp, "
                     f"{bases[0].reflections_amount} bounces, a moving camera, one rt4_render_sections_device call "
                     "per frame; overlapped launches (default) against RT4_FLAG_SERIAL_FRAMES, same images and count",
            "frames": frames, "unit": "ray-bounce intersections/s", **out,
            "speedup": out["serial"]["ms_per_frame"] / out["overlapped"]["ms_per_frame"]}

def main():
    args = parse_args()
    # Hardware queues of this process (read by the HIP runtime when it starts, before any GPU call here; the ranks
    # spawned below inherit it). Overlapped launches of small frames run on up to 8 side streams;
    # with HIP's default of 4 queues they share queues (the sections leg: 0.25 ms per frame with 4, 0.17 with 8; the
    # headline, one stream, is unchanged: profiles/r04_ab.txt).
    if args.hw_queues > 0:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the multi-rank path on a one-GPU box (tests/test_gpu_bench.py): every rank renders on
    # GPU 0 and the gather / reductions run over gloo on host copies. Never used for a reported number.
    rehearse = os.environ.get("RT4_BENCH_REHEARSE") == "1"
    import torch
    import torch.distributed as dist

    gpu = 0 if rehearse else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    comm_dev = torch.device("cpu") if rehearse else dev
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    rt4 = importlib.import_module("4d_ray_tracing_amd")
    shard = importlib.import_module("4d_ray_tracing_amd.shard")

    strong = args.mode == "strong"
    plan = (shard.make_plan(args.width, height=args.height, world=world) if strong
            else shard.weak_plan(args.width, rows_per_rank=args.height, world=world))
    scene = rt4.Scene.named(args.scene)
    flags = (0 if args.no_lut else rt4.FLAG_SAMPLER_LUT) | (rt4.FLAG_PRIMARY_REUSE if args.primary_reuse else 0)

    # setup: context (+ sampler table build) and scene upload (+ divisor / threshold verification)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tracer = rt4.Tracer(device=gpu, flags=flags)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tracer.set_scene(scene)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    tracer.set_scene(scene)  # the same scene again: served from the verification cache
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    other = new_constants_scene(rt4, scene)  # a further new scene: radii and sun size not yet verified
    tracer.set_scene(other)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    tracer.set_scene(scene)
    torch.cuda.synchronize()
    setup = {"context_ms": (t1 - t0) * 1e3, "set_scene_ms": (t2 - t1) * 1e3, "set_scene_repeat_ms": (t3 - t2) * 1e3,
             "set_scene_new_constants_ms": (t4 - t3) * 1e3}

    base = rt4.make_uniforms(plan.width, plan.height, samples=args.spp, reflections=args.bounces, seed=args.seed)
    frame_no = [0]

    def uniforms():
        if not args.progressive:
            return base
        frame_no[0] += 1
        return rt4.progressive_uniforms(base, frame_no[0])

    fmt = {"f32": rt4.FRAME_RGBA32F, "f16": rt4.FRAME_RGBA16F, "rgba8": rt4.FRAME_RGBA8}[args.format]
    tdt = {"f32": torch.float32, "f16": torch.float16, "rgba8": torch.uint8}[args.format]
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    counter = torch.zeros(1, dtype=torch.int64, device=dev)

    # Frames pipelined in one call (rt4_render_frames_device): the same frames, the same final image, the
    # per-frame drain of the persistent launch paid once per call. Not with a gather after every frame,
    # which needs every frame's image in the frame buffer.
    pipelined = not args.frame_by_frame and not (world > 1 and args.gather == "every")

    # ---- T1 leg (strong, N > 1): rank 0 renders the whole frame alone, same warmup/steps and launches
    t1_ms = None
    if strong and world > 1 and not args.no_t1:
        dist.barrier()
        if rank == 0:
            full = torch.zeros((plan.height, plan.width, 4), dtype=tdt, device=dev)
            reg_full = rt4.region(plan.width, plan.height)
            def full_frames(n):
                if pipelined:
                    if n:
                        tracer.render_frames_device([uniforms() for _ in range(n)], reg_full, full.data_ptr(), fmt,
                                                    plan.width, 0, sptr)
                    return
                for _ in range(n):
                    tracer.render_device_ex(uniforms(), reg_full, full.data_ptr(), fmt, plan.width, 0, sptr)

            if pipelined:
                tracer.reserve_frames(reg_full.w, reg_full.h)
            full_frames(args.warmup)
            torch.cuda.synchronize()
            ta = time.perf_counter()
            full_frames(args.steps)
            torch.cuda.synchronize()
            t1_ms = (time.perf_counter() - ta) / args.steps * 1e3
            del full
            frame_no[0] = 0
        dist.barrier()

    reg = rt4.region(**plan.region_args(rank))
    frame = torch.zeros((plan.rows_max, plan.width, 4), dtype=tdt, device=dev)  # padded shard (gather)
    gathers = []

    def render():
        tracer.render_device_ex(uniforms(), reg, frame.data_ptr(), fmt, plan.width, counter.data_ptr(), sptr)

    def render_frames(n, cnt_ptr):
        tracer.render_frames_device([uniforms() for _ in range(n)], reg, frame.data_ptr(), fmt, plan.width, cnt_ptr, sptr)

    def gather_once():
        # a rank whose part of the gather fails posts the error and exits; its peers exit when their own gather
        # fails (gloo) or when sync() finds the report (RCCL): status 1 naming the rank, no hang (shard.py)
        try:
            if rehearse:
                shard.gather_frame(frame.cpu(), plan, rank)
            else:
                shard.gather_frame(frame, plan, rank)  # the frame assembled (un-permuted) on rank 0
        except Exception as e:  # noqa: BLE001 - any failure of the collective ends every rank
            shard.exit_failed(rank, f"{type(e).__name__}: {e}")

    def sync():
        # torch.cuda.synchronize, but with N > 1 a wait that also watches for a failed peer's report
        if world > 1:
            f = shard.wait_or_failure(stream)
            if f is not None:
                shard.exit_failed(rank, "a peer's gather failed")
        torch.cuda.synchronize()

    def gather():
        g0 = torch.cuda.Event(enable_timing=True)
        g1 = torch.cuda.Event(enable_timing=True)
        g0.record(stream)
        gather_once()
        g1.record(stream)
        gathers.append((g0, g1))

    if pipelined:
        tracer.reserve_frames(reg.w, reg.h)  # the scratch of the pipelined frames, outside the timed region
        if args.warmup:
            render_frames(args.warmup, counter.data_ptr())
    else:
        for _ in range(args.warmup):
            render()
            if world > 1 and args.gather == "every":
                gather_once()
    if world > 1 and (args.gather == "final" or not args.warmup):
        # one gather outside the timed region: the collective's one-time set-up (RCCL's point-to-point
        # connections behind dist.gather, the receive buffers' first allocation) is not part of a frame
        gather_once()
    sync()
    counter.zero_()
    k_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    k_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if pipelined:
        k_start[0].record(stream)
        render_frames(args.steps, counter.data_ptr())
        k_end[0].record(stream)
    else:
        for i in range(args.steps):
            k_start[i].record(stream)
            render()
            k_end[i].record(stream)
            if world > 1 and args.gather == "every":
                gather()
    if world > 1 and args.gather == "final":
        gather()
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if pipelined:  # per frame: the pipelined launch(es) and the fold, divided by the frames
        kernel_ms = k_start[0].elapsed_time(k_end[0]) / args.steps
    else:
        # first start to last end, gathers taken out: a single-frame launch's trace runs on a side stream and
        # overlaps the previous frame's drain (rt4.h RT4_FLAG_SERIAL_FRAMES), so per-frame event pairs on the
        # caller's stream would miss the part of a trace that starts before its own start event
        inner = gathers if (world > 1 and args.gather == "every") else []  # the gathers between the frames
        kernel_ms = (k_start[0].elapsed_time(k_end[-1]) - sum(a.elapsed_time(b) for a, b in inner)) / args.steps
    gather_ms = sum(a.elapsed_time(b) for a, b in gathers) / len(gathers) if gathers else 0.0

    n_local = int(counter.item())
    evaluated = tracer.evaluated() if args.primary_reuse else None

    # Extra leg (N = 1, pipelined headline): the same frames, one launch per frame (rt4_render_device_ex),
    # as the reference draws one frame per loop iteration (main.cpp:93, windows.cpp:45): the per-launch
    # drain is paid every frame. Reported beside the headline, never as value.
    fbf_leg = None
    if world == 1 and pipelined and not args.no_fbf_leg:
        frame_no[0] = 0
        frame.zero_()
        for _ in range(args.warmup):
            render()
        torch.cuda.synchronize()
        cnt_f = torch.zeros(1, dtype=torch.int64, device=dev)
        f_start = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        f_end = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        torch.cuda.synchronize()
        tf0 = time.perf_counter()
        for i in range(args.steps):
            f_start[i].record(stream)
            tracer.render_device_ex(uniforms(), reg, frame.data_ptr(), fmt, plan.width, cnt_f.data_ptr(), sptr)
            f_end[i].record(stream)
        torch.cuda.synchronize()
        el_f = time.perf_counter() - tf0
        n_f = int(cnt_f.item())
        fbf_leg = {
            "label": "one launch per frame (rt4_render_device_ex), as the reference draws one frame per loop "
                     "iteration; same frames, same image and count as the pipelined headline",
            "value": n_f / el_f, "unit": "ray-bounce intersections/s",
            "ms_per_step": el_f / args.steps * 1e3,
            # first start to last end on the caller's stream (the traces overlap): a device span per frame, which
            # includes host submission gaps between launches, not a kernel-only time
            "kernel_ms": f_start[0].elapsed_time(f_end[-1]) / args.steps,
            "kernel_ms_kind": "device span per frame: first start event to last end event on the caller's stream",
            "intersections_per_step": n_f / args.steps,
        }

    # Extra leg (N = 1): the same frames with RT4_FLAG_PRIMARY_REUSE, reported beside the headline
    # (a reference-equivalent rate, with the evaluated count next to it).
    reuse_leg = None
    if world == 1 and not args.primary_reuse and not args.no_reuse_leg:
        t_r = rt4.Tracer(device=gpu, flags=flags | rt4.FLAG_PRIMARY_REUSE, scene=scene)
        frame_no[0] = 0
        frame.zero_()
        def reuse_frames(n, cnt_ptr):
            if pipelined:
                if n:
                    t_r.render_frames_device([uniforms() for _ in range(n)], reg, frame.data_ptr(), fmt, plan.width,
                                             cnt_ptr, sptr)
                return
            for _ in range(n):
                t_r.render_device_ex(uniforms(), reg, frame.data_ptr(), fmt, plan.width, cnt_ptr, sptr)

        if pipelined:
            t_r.reserve_frames(reg.w, reg.h)
        reuse_frames(args.warmup, 0)
        torch.cuda.synchronize()
        t_r.evaluated()  # reset
        cnt_r = torch.zeros(1, dtype=torch.int64, device=dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        tr0 = time.perf_counter()
        ev0.record(stream)
        reuse_frames(args.steps, cnt_r.data_ptr())
        ev1.record(stream)
        torch.cuda.synchronize()
        el_r = time.perf_counter() - tr0
        n_r = int(cnt_r.item())
        reuse_leg = {
            "label": "reference-equivalent: RT4_FLAG_PRIMARY_REUSE evaluates each pixel's primary ray once and "
                     "starts its other samples from the cached candidate; same image, same reference count",
            "value": n_r / el_r, "unit": "ray-bounce intersections/s (reference-equivalent)",
            "ms_per_step": el_r / args.steps * 1e3, "kernel_ms": ev0.elapsed_time(ev1) / args.steps,
            "intersections_per_step": n_r / args.steps, "evaluated_per_step": t_r.evaluated() / args.steps,
        }
        t_r.close()
    # Extra leg (N = 1, pipelined): the headline's frames at the clock the chip holds under sustained load. The timed
    # frames above follow only `warmup` frames (the driver's 5: ~2 ms of work after idle), and the chip's clock is still
    # ramping through them: 2.0-2.2 GHz on config 2, against 2.35 after ~60 ms of load (tools/clock_probe.sh,
    # profiles/r06/clock). Here the same frames run two full launches to load the chip, then two more are timed.
    # Reported beside the headline, never as value.
    # Only where the timed frames are short (< 150 ms in all: configs 2 and 3); longer timed regions (configs 4, 5) run
    # past the ramp already. Two launches' worth of frames (at least the timed frames, so no launch drains more often
    # than the headline's), fewer when 150 ms of load takes fewer.
    steady_leg = None
    if world == 1 and pipelined and not args.no_steady_leg and kernel_ms * args.steps < 150.0:
        fpl_s = tracer.frames_per_launch(reg.w, reg.h)
        n_st = max(args.steps, min(2 * fpl_s, int(150.0 / max(kernel_ms, 1e-3))))
        frame_no[0] = 0
        frame.zero_()
        render_frames(n_st, 0)
        cnt_s = torch.zeros(1, dtype=torch.int64, device=dev)
        es0 = torch.cuda.Event(enable_timing=True)
        es1 = torch.cuda.Event(enable_timing=True)
        es0.record(stream)
        render_frames(n_st, cnt_s.data_ptr())
        es1.record(stream)
        torch.cuda.synchronize()
        n_s = int(cnt_s.item())
        ms_s = es0.elapsed_time(es1) / n_st
        steady_leg = {
            "label": "sustained clock: the same frames, timed after as many frames of load (the headline's timed "
                     "frames run while the clock ramps from idle; DESIGN.md section 9); never the value",
            "frames": n_st, "frames_before": n_st, "frames_per_launch": min(n_st, fpl_s),
            "value": n_s / (ms_s * 1e-3) / n_st, "unit": "ray-bounce intersections/s",
            "kernel_ms": ms_s, "intersections_per_step": n_s / n_st,
        }
    sections_leg = None
    if world == 1 and not args.no_sections_leg:
        sections_leg = sections_loop_leg(rt4, torch, gpu, flags, scene, stream, tracer)
    if world > 1:
        st = torch.tensor([elapsed, kernel_ms, gather_ms], dtype=torch.float64, device=comm_dev)
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        n_sum = torch.tensor([n_local], dtype=torch.int64, device=comm_dev)
        dist.all_reduce(n_sum, op=dist.ReduceOp.SUM)
        elapsed, kernel_ms, gather_ms = (float(x) for x in st.tolist())
        n_total = int(n_sum.item())
    else:
        n_total = n_local

    fpl = min(args.steps, tracer.frames_per_launch(reg.w, reg.h)) if pipelined else 1
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = n_total / elapsed
        units_per_launch = n_total / world / args.steps  # per rank (kernel_ms is the max over ranks)
        cpus = host_cpus()
        version = rt4.lib.rt4_build_info().decode().split()[2]
        config = {
            "workload": (f"config {args.config}: {args.scene} scene, frame {plan.width}x{plan.height}"
                         + (f" ({plan.width}x{plan.rows_max} px per GPU)" if world > 1 else "")
                         + f", {args.spp} spp{' per progressive frame' if args.progressive else ''}, "
                           f"{args.bounces} bounces, seed {args.seed}, {args.format} frame"),
            "config": args.config, "scene": args.scene, "width": plan.width,
            "height": plan.height, "height_per_gpu": plan.rows_max, "spp": args.spp, "bounces": args.bounces,
            "seed": args.seed, "sampler_lut": not args.no_lut, "frame_format": args.format,
            "progressive": bool(args.progressive), "kernel_version": version,
            "launch": (f"{args.steps} frames per rt4_render_frames_device call, {fpl} per pipelined launch"
                       if pipelined else "one launch per frame (rt4_render_device_ex)"),
            "parallelism": f"pixel-bands x{world}" + (f" + {'gloo rehearsal' if rehearse else 'RCCL'} gather "
                                                      f"({args.gather})" if world > 1 else ""),
        }
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "ray-bounce intersections/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.mode,
            "vs_baseline": None,
            "dtype": "fp32",
            "accumulator": args.format,
            "data": "synthetic (fixed-seed procedural scene, no dataset)",
            "config": config,
            "value_total": value,
            "value_per_gpu": value / world,
            "value_note": "value = the whole job's intersections / the max-over-ranks time (bench contract; "
                          "the driver derives scaling from it); the metric's per-GPU rate is value_per_gpu",
            "gather_ms": gather_ms,
            "intersections_per_step": n_total / args.steps,
            "nominal_bound_per_step": plan.width * plan.height * args.spp * (args.bounces + 1),
            "kernel_ms": kernel_ms,
            "kernel_ms_kind": ("HIP events around the pipelined launch(es) and the fold on the launch stream, per frame"
                               if pipelined else "device span per frame: first start event to last end event on the "
                               "caller's stream (the overlapped traces run on side streams)"),
            "frames_per_launch": fpl,
            "setup_ms": setup,
            "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
        }
        if args.primary_reuse:
            line["primary_reuse"] = True
            line["label"] = "reference-equivalent (RT4_FLAG_PRIMARY_REUSE): the primary ray is evaluated once per pixel"
            line["evaluated_per_step"] = evaluated / args.steps if world == 1 else None
        if reuse_leg:
            line["primary_reuse_leg"] = reuse_leg
        if fbf_leg:
            line["frame_by_frame_leg"] = fbf_leg
        if sections_leg:
            line["sections_loop_leg"] = sections_leg
        if steady_leg:
            line["steady_clock_leg"] = steady_leg
        if strong:
            line["t1_ms"] = t1_ms if world > 1 else ms_per_step
            line["efficiency"] = (line["t1_ms"] / (world * ms_per_step)) if line["t1_ms"] else None
        if not args.no_ops:
            opu, opu_exec, _ = ops_per_unit(rt4, scene, base, plan.width, plan.height, cpus["threads"])
            achieved = opu * units_per_launch / (kernel_ms * 1e-3) / 1e12
            achieved_exec = (opu if args.no_lut else opu_exec) * units_per_launch / (kernel_ms * 1e-3) / 1e12
            prof, src = pmc_profile(config, fpl)
            der = prof.get("derived", {}) if prof else {}
            cnt = prof.get("counters", {}) if prof else {}
            line["roofline"] = {
                "bound": "valu",
                "achieved": achieved,
                "peak": PEAK_FP32_VALU_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_VALU_TFLOPS,
                # memory-side bytes per frame: request-counted where the profile has the pmc_req pass (exact for
                # the table's 64-B requests), else FETCH_SIZE x 2 + WRITE_SIZE (an upper bound)
                "traffic": der.get("traffic_bytes_per_launch", der.get("hbm_bytes_per_launch")),
                "achieved_kind": "reference-equivalent: the reference's fp32 ops per unit (oracle op count, fma = 2) "
                                 "x units / kernel time; counts work the kernel skips exactly (tiger CSE, "
                                 "bounding-ball skips, the sampler table), so it is not a hardware utilisation",
                "ops_per_unit": opu,
                "frac_reference": achieved / PEAK_FP32_VALU_TFLOPS,
                # the reference's count without the Newton loop the sampler table replaces (round 1-5's "executed")
                "ops_per_unit_reference_lut": opu if args.no_lut else opu_exec,
                "frac_reference_lut": achieved_exec / PEAK_FP32_VALU_TFLOPS,
                "frac_executed": None,  # from the PMC profile's FLOP counters, below
                "units_per_launch": units_per_launch,
                "algorithmic_bytes_per_launch": reg.w * reg.h * 2 * rt4.frame_format_bytes(fmt),  # old_frame in, new out
                "note": "fp32 ops (fma=2) per find_intersection+shading counted by the oracle on a row sample of "
                        "the frame (frac = frac_reference); reference_lut = without the w_by_volume Newton ops the "
                        "sampler table replaces; frac_executed = the fp32 FLOPs the kernel executed (hardware FLOP "
                        "counter x lane utilisation, DESIGN.md §5) / kernel time / peak; "
                        "per launch = per frame (a pipelined launch holds frames_per_launch frames: its units, "
                        "bytes and time are divided by them); frac_counters = the VALU lane-operations the "
                        "hardware counted (SQ_THREAD_CYCLES_VALU, same config, kernel version and launch shape) / "
                        "(kernel time x 256 CU x 4 SIMD x 32 lanes x 2.4 GHz); see DESIGN.md §5",
            }
            if prof and cnt.get("SQ_THREAD_CYCLES_VALU"):
                lane_ops = cnt["SQ_THREAD_CYCLES_VALU"]  # per frame (pmc_summary divides a dispatch by its frames)
                line["roofline"]["frac_counters"] = lane_ops / (kernel_ms * 1e-3) / PEAK_VALU_LANE_OPS
                if steady_leg:
                    # the same frames' lane-ops over the sustained-clock leg's time: the VALU fraction once the clock
                    # has ramped (the work per frame does not depend on the clock)
                    steady_leg["frac_counters"] = lane_ops / (steady_leg["kernel_ms"] * 1e-3) / PEAK_VALU_LANE_OPS
                line["roofline"]["valu_lane_ops_per_frame"] = lane_ops
                line["roofline"]["valu_lane_utilisation"] = der.get("valu_lane_utilisation")
                line["roofline"]["valu_issue_frac"] = der.get("valu_issue_frac")
                if cnt.get("SQ_INSTS_VALU_FLOPS_FP32") and cnt.get("SQ_INSTS_VALU"):
                    # SQ_INSTS_VALU_FLOPS_FP32 counts a wave instruction's FLOPs once whatever its EXEC mask (fma = 2,
                    # add / mul / transcendental = 1); SQ_THREAD_CYCLES_VALU counts active lanes, a transcendental
                    # twice (tools/flops_calib.hip, profiles/r06/flops_calib.txt). Executed FLOPs = 64 x FLOPS_FP32 x
                    # the lane utilisation, the fp32 instructions taken at the kernel's mean utilisation.
                    util_c = lane_ops / (64.0 * (cnt["SQ_INSTS_VALU"] + cnt.get("SQ_INSTS_VALU_TRANS_F32", 0.0)))
                    flops = 64.0 * cnt["SQ_INSTS_VALU_FLOPS_FP32"] * util_c
                    line["roofline"]["frac_executed"] = flops / (kernel_ms * 1e-3) / (PEAK_FP32_VALU_TFLOPS * 1e12)
                    line["roofline"]["flops_executed_per_frame"] = flops
                    line["roofline"]["fp32_flops_per_valu_inst"] = cnt["SQ_INSTS_VALU_FLOPS_FP32"] / cnt["SQ_INSTS_VALU"]
                    line["roofline"]["frac_executed_kind"] = (
                        "fp32 FLOPs executed (SQ_INSTS_VALU_FLOPS_FP32 x 64 x lane utilisation, fma = 2) / kernel time / "
                        "157.3 TFLOP/s; = frac_counters x FLOPs per VALU instruction / 2")
                line["roofline"]["counters_source"] = src + (
                    f" (rocprofv3 PMC, {prof.get('frames_per_dispatch', 1)} frames per dispatch, per frame; trace "
                    f"{prof.get('avg_ns', 0) * 1e-6:.4f} ms per frame)")
            if prof and der.get("hbm_bytes_per_launch"):
                exact = "traffic_bytes_per_launch" in der
                line["roofline"]["traffic_source"] = src + (
                    " (rocprofv3 TCC_EA0_RDREQ by request size + WRITE_SIZE, per frame)" if exact
                    else " (rocprofv3 FETCH_SIZE*2 + WRITE_SIZE, per frame)")
                if prof.get("avg_ns"):
                    # the north star's "achieved HBM GB/s": the profiled traffic over the profiled trace time per
                    # frame (memory-side bytes: the sampler gathers are served by the Infinity Cache)
                    gbps = line["roofline"]["traffic"] / prof["avg_ns"]
                    line["roofline"]["traffic_gbps"] = gbps
                    line["roofline"]["traffic_frac_of_hbm_peak"] = gbps / HBM_PEAK_GBPS
            if prof and der.get("fabric_read_requests") and prof.get("avg_ns"):
                # the sampler gathers against the measured random-gather ceiling of a 32 MiB table
                # (tools/mall_probe.hip, profiles/r03_mall/probe.json: every CU issuing 4-B random loads)
                rate = der["fabric_read_requests"] / (prof["avg_ns"] * 1e-9)
                line["roofline"]["fabric_read_requests_per_s"] = rate
                ceiling = gather_ceiling()
                if ceiling:
                    line["roofline"]["gather_rate_frac"] = rate / ceiling
                    line["roofline"]["gather_ceiling_per_s"] = ceiling
            if prof and der.get("ea_read_latency_cycles"):
                line["roofline"]["ea_read_latency_cycles"] = der["ea_read_latency_cycles"]
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(rt4, scene, base, plan.width, plan.rows_max, args.cpu_seconds, cpus)
        print(json.dumps(line), flush=True)
    tracer.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
