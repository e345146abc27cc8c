"""Frames pipelined in one launch (rt4_render_frames_device) against the same frames rendered one launch
at a time (rt4_render_device_ex), bit for bit, and against the CPU oracle: progressive accumulation in
every frame format, repeated identical frames (the benchmark loop), chunking past RT4_MAX_FRAMES, the
primary-reuse, generic and inline-sampler kernels, and a band region. All calls go through the C ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = {0: np.float32, 1: np.float16, 2: np.uint8}


def frames_both_ways(rt4, scene, us, reg, fmt, flags, init=None):
    """(pipelined frame, its count), (sequential frame, its count) on the GPU."""
    import torch

    tdt = {0: torch.float32, 1: torch.float16, 2: torch.uint8}[fmt]
    out = []
    for pipelined in (True, False):
        t = rt4.Tracer(device=0, flags=flags, scene=scene)
        try:
            fr = torch.zeros((reg.h, reg.w, 4), dtype=tdt, device="cuda")
            if init is not None:
                fr.copy_(torch.from_numpy(init))
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            if pipelined:
                if len(us) % 2:  # odd frame counts also check that a reserved scratch is used as is
                    t.reserve_frames(reg.w, reg.h)
                t.render_frames_device(us, reg, fr.data_ptr(), fmt, reg.w, cnt.data_ptr(), s)
            else:
                for u in us:
                    t.render_device_ex(u, reg, fr.data_ptr(), fmt, reg.w, cnt.data_ptr(), s)
            torch.cuda.synchronize()
            out.append((fr.cpu().numpy(), int(cnt.item())))
        finally:
            t.close()
    return out


def same_bits(a, b):
    if a.dtype == np.uint8:
        return np.array_equal(a, b)
    v = np.uint16 if a.dtype == np.float16 else np.uint32
    return np.array_equal(a.view(v), b.view(v))


@pytest.mark.parametrize("fmt", [0, 1, 2])
@pytest.mark.parametrize("name", ["sphere", "hypercube", "all_primitives"])
def test_progressive_pipelined_equals_sequential(rt4, name, fmt):
    scene = rt4.Scene.named(name)
    base = rt4.make_uniforms(96, 56, samples=3, reflections=5, seed=4242)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 9)]
    reg = rt4.region(96, 56)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, fmt, rt4.FLAG_SAMPLER_LUT)
    assert np_ == nq
    assert same_bits(p, q)


def test_progressive_pipelined_equals_oracle(rt4, oracle):
    """Six progressive frames of the sphere scene in fp16, pipelined, against the oracle's six frames."""
    scene = rt4.Scene.named("sphere")
    base = rt4.make_uniforms(64, 40, samples=2, reflections=4, seed=99)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 7)]
    reg = rt4.region(64, 40)
    (p, n_gpu), _ = frames_both_ways(rt4, scene, us, reg, 1, rt4.FLAG_SAMPLER_LUT)
    c = np.zeros((40, 64, 4), np.float16)
    n_cpu = 0
    for u in us:
        _, k = oracle.render_fmt(scene.desc, u, reg, 1, frame=c)
        n_cpu += k
    assert n_gpu == n_cpu
    assert same_bits(p, c)


@pytest.mark.parametrize("flags", ["lut", "reuse", "generic", "inline"])
def test_repeated_frames_and_kernels(rt4, flags):
    """The benchmark loop (the same uniforms every frame, part 1) over a frame with old contents."""
    f = {"lut": rt4.FLAG_SAMPLER_LUT, "reuse": rt4.FLAG_SAMPLER_LUT | rt4.FLAG_PRIMARY_REUSE,
         "generic": rt4.FLAG_SAMPLER_LUT | rt4.FLAG_GENERIC_KERNEL, "inline": 0}[flags]
    scene = rt4.Scene.named("room")
    u = rt4.make_uniforms(80, 48, samples=2, reflections=3, seed=7)
    reg = rt4.region(80, 48)
    init = np.random.default_rng(1).random((48, 80, 4), dtype=np.float32)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, [u] * 5, reg, 0, f, init=init)
    assert np_ == nq
    assert same_bits(p, q)


def test_chunked_past_max_frames(rt4):
    """70 progressive frames: one pipelined launch of RT4_MAX_FRAMES (64) and one of 6."""
    scene = rt4.Scene.named("cylinder4d")
    base = rt4.make_uniforms(40, 24, samples=1, reflections=3, seed=5)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 71)]
    reg = rt4.region(40, 24)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 1, rt4.FLAG_SAMPLER_LUT)
    assert np_ == nq
    assert same_bits(p, q)


def test_band_region_pipelined(rt4):
    """A rank's band layout (rt4_region band_rows / band_step) with odd sizes, pipelined."""
    scene = rt4.Scene.named("tiger")
    base = rt4.make_uniforms(61, 72, samples=2, reflections=4, seed=31)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 5)]
    reg = rt4.region(61, 19, y0=3, band_rows=8, band_step=24)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 0, rt4.FLAG_SAMPLER_LUT)
    assert np_ == nq
    assert same_bits(p, q)


def test_frames_reject_changed_uniforms(rt4):
    """Only seed and part may change across the frames of one call (RT4_ERR_ARG otherwise)."""
    import torch

    scene = rt4.Scene.named("sphere")
    u0 = rt4.make_uniforms(32, 16, samples=1, reflections=1, seed=1)
    u1 = rt4.make_uniforms(32, 16, samples=2, reflections=1, seed=1)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        fr = torch.zeros((16, 32, 4), dtype=torch.float32, device="cuda")
        with pytest.raises(rt4.RT4Error):
            t.render_frames_device([u0, u1], rt4.region(32, 16), fr.data_ptr(), 0, 32)
    finally:
        t.close()


def test_mirror_room_runs_frame_by_frame(rt4):
    """The mirror-room tiger kernel (BASELINE config 4's scene) is not pipelined (measured slower);
    rt4_render_frames_device still equals the sequential frames there."""
    scene = rt4.Scene.named("tiger_two_mirrors")
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        assert t.frames_per_launch(64, 40) == 1
        t.set_scene(rt4.Scene.named("sphere"))
        assert t.frames_per_launch(1920, 1080) == 64 and t.frames_per_launch(3840, 2160) == 32
        assert t.frames_per_launch(8192, 16) == 1  # wider than the pipelined pixel word holds
    finally:
        t.close()
    base = rt4.make_uniforms(48, 32, samples=2, reflections=6, seed=3)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 4)]
    reg = rt4.region(48, 32)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 0, rt4.FLAG_SAMPLER_LUT)
    assert np_ == nq
    assert same_bits(p, q)


@pytest.mark.parametrize("fmt", ["f16", "rgba8"])
def test_cpp_host_pipelined_equals_frame_by_frame(rt4, tmp_path, fmt):
    """lib/rt4_render with one section and a resting camera hands its frames to rt4_render_frames_device;
    its PPM equals the frame-by-frame loop's byte for byte (same intersection count printed)."""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(rt4.LIB_PATH), "rt4_render")
    props = os.path.join(os.path.dirname(rt4.LIB_PATH), "..", "..", "properties.txt")
    outs = []
    for extra in ([], ["--frame-by-frame"]):
        pre = str(tmp_path / ("fbf" if extra else "pipe"))
        cmd = [exe, "-p", props, "-s", "hypercube", "-n", "5", "-W", "72", "-H", "40", "-f", fmt,
               "--seed", "77", "-o", pre] + extra
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        count = [ln for ln in r.stdout.splitlines() if "intersections" in ln][0].split("intersections ")[1].split(",")[0]
        outs.append((open(pre + "_yxz.ppm", "rb").read(), count))
    assert outs[0] == outs[1]
