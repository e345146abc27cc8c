"""Frames pipelined in one launch (rt4_render_frames_device) against the same frames rendered one launch
at a time (rt4_render_device_ex), bit for bit, and against the CPU oracle: progressive accumulation in
every frame format, repeated identical frames (the benchmark loop), chunking past RT4_MAX_FRAMES, the
primary-reuse, generic and inline-sampler kernels, and a band region. All calls go through the C ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DT = {0: np.float32, 1: np.float16, 2: np.uint8}


def frames_both_ways(rt4, scene, us, reg, fmt, flags, init=None, stride=None, rows=None, reserve=None):
    """(pipelined frame, its count), (sequential frame, its count) on the GPU. The frame buffer has
    `rows` rows of `stride` pixels (default: the region's h and w); the region's pixels start at
    column reg.x0 of that buffer, as rt4_render_device_ex addresses them (pixel (i, j) of the region
    at i * stride + j of d_frame, which the caller offsets by x0)."""
    import torch

    tdt = {0: torch.float32, 1: torch.float16, 2: torch.uint8}[fmt]
    stride = reg.w if stride is None else stride
    rows = reg.h if rows is None else rows
    reserve = (len(us) % 2 == 1) if reserve is None else reserve
    out = []
    for pipelined in (True, False):
        t = rt4.Tracer(device=0, flags=flags, scene=scene)
        try:
            fr = torch.zeros((rows, stride, 4), dtype=tdt, device="cuda")
            if init is not None:
                fr.copy_(torch.from_numpy(init))
            base = fr.data_ptr() + reg.x0 * 4 * fr.element_size()
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            if pipelined:
                if reserve:  # odd frame counts also check that a reserved scratch is used as is
                    t.reserve_frames(reg.w, reg.h)
                t.render_frames_device(us, reg, base, fmt, stride, cnt.data_ptr(), s)
            else:
                for u in us:
                    t.render_device_ex(u, reg, base, fmt, stride, cnt.data_ptr(), s)
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


def test_mirror_room_pipelined_equals_sequential(rt4):
    """The mirror-room tiger kernel (BASELINE config 4's scene) pipelines like every other kernel since
    r03-v34 (the phase-aligned refill removed its slowdown); rt4_render_frames_device equals
    the sequential frames there, in one launch and split over launches, and with a resting camera's
    identical frames (the bench's call)."""
    scene = rt4.Scene.named("tiger_two_mirrors")
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        assert t.frames_per_launch(64, 40) == 64 and t.frames_per_launch(3840, 2160) == 32
        assert t.frames_per_launch(8192, 16) == 1  # wider than the pipelined pixel word holds
        t.set_scene(rt4.Scene.named("sphere"))
        assert t.frames_per_launch(1920, 1080) == 64
    finally:
        t.close()
    base = rt4.make_uniforms(48, 32, samples=3, reflections=12, seed=3)
    reg = rt4.region(48, 32)
    for us in ([rt4.progressive_uniforms(base, n) for n in range(1, 5)], [base] * 3,
               [rt4.progressive_uniforms(base, n) for n in range(1, 71)]):  # 70 frames: two launches
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


def test_padded_stride_and_x_offset(rt4):
    """Pipelined frames into a sub-rectangle of a wider frame buffer (row_stride_px > w, x0 > 0): the
    fold pass's own addressing (i * row_stride_px + j) against the sequential launches; the pixels
    outside the region keep their old contents."""
    scene = rt4.Scene.named("hypercube")
    base = rt4.make_uniforms(100, 44, samples=2, reflections=4, seed=606)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 6)]
    reg = rt4.region(37, 44, x0=13)
    for fmt in (0, 1, 2):
        dt = DT[fmt]
        rng = np.random.default_rng(fmt)
        init = (rng.integers(0, 255, (44, 100, 4)).astype(np.uint8) if fmt == 2
                else rng.random((44, 100, 4)).astype(dt))
        (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, fmt, rt4.FLAG_SAMPLER_LUT, init=init, stride=100,
                                            rows=44)
        assert np_ == nq
        assert same_bits(p, q), fmt
        # columns outside [13, 50) are untouched, and the region's columns changed
        assert same_bits(np.ascontiguousarray(p[:, :13]), np.ascontiguousarray(init[:, :13]))
        assert same_bits(np.ascontiguousarray(p[:, 50:]), np.ascontiguousarray(init[:, 50:]))
        assert not same_bits(np.ascontiguousarray(p[:, 13:50]), np.ascontiguousarray(init[:, 13:50]))


@pytest.mark.parametrize("name", ["sphere", "hypercube"])
def test_bench_shape_progressive_1080p(rt4, name):
    """The bench's launch shape (BASELINE configs 2 / 3: 1920x1080, 16 spp, 8 bounces, 20 frames in one
    rt4_render_frames_device call) with a different seed and part every frame, so that every frame's
    slice of the multi-GB scratch and every 13-bit pixel field of the packed pixel word reaches the
    image: against 20 frame-by-frame launches, bit for bit."""
    scene = rt4.Scene.named(name)
    base = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=12345)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 21)]
    reg = rt4.region(1920, 1080)
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 0, rt4.FLAG_SAMPLER_LUT, reserve=True)
    assert np_ == nq
    assert same_bits(p, q)


def test_config5_chunk_pipelined_equals_sequential(rt4):
    """BASELINE config 5's launch shape: all_primitives at 3840x2160, 16 spp, 8 bounces, fp16 frame, 32
    progressive frames (one full pipelined chunk at 4K: a 4.2 GB scratch) against 32 rt4_render_device_ex
    launches, bit for bit, count included."""
    scene = rt4.Scene.named("all_primitives")
    base = rt4.make_uniforms(3840, 2160, samples=16, reflections=8, seed=12345)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 33)]
    reg = rt4.region(3840, 2160)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        assert t.frames_per_launch(3840, 2160) == 32
    finally:
        t.close()
    (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 1, rt4.FLAG_SAMPLER_LUT, reserve=True)
    assert np_ == nq
    assert same_bits(p, q)


def test_config4_pipelined_equals_sequential(rt4):
    """BASELINE config 4's launch shape since r03-v35: the mirror room at 3840x2160, 64 spp, 12 bounces,
    frames pipelined under the wave clock with four tiles per queue claim (§4.26), against
    frame-by-frame launches, bit for bit, count included: three identical frames (the bench's call) and
    three progressive ones."""
    scene = rt4.Scene.named("tiger_two_mirrors")
    base = rt4.make_uniforms(3840, 2160, samples=64, reflections=12, seed=12345)
    reg = rt4.region(3840, 2160)
    for identical, us in ((True, [base] * 3), (False, [rt4.progressive_uniforms(base, n) for n in range(1, 4)])):
        (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 0, rt4.FLAG_SAMPLER_LUT, reserve=True)
        assert np_ == nq
        if identical:
            assert np_ == 3 * 6898035764  # the config-4 frame's count (profiles/r05_v52/pmc_config4.json bench.intersections_per_step)
        assert same_bits(p, q)


@pytest.mark.parametrize("name", ["tiger", "room", "sphere"])
def test_lockstep_and_deferral_kernels_1080p(rt4, name):
    """The scheduling rules of round 3 at a full 1080p frame (16 spp, 8 bounces, 6 progressive frames):
    deferred tiger tests and four-tile claims (tiger), the wave clock (room), deferred exact sphere tests
    (sphere); pipelined against frame by frame, bit for bit, and with primary reuse."""
    scene = rt4.Scene.named(name)
    base = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=777)
    us = [rt4.progressive_uniforms(base, n) for n in range(1, 7)]
    reg = rt4.region(1920, 1080)
    for flags in (rt4.FLAG_SAMPLER_LUT, rt4.FLAG_SAMPLER_LUT | rt4.FLAG_PRIMARY_REUSE):
        (p, np_), (q, nq) = frames_both_ways(rt4, scene, us, reg, 0, flags)
        assert np_ == nq
        assert same_bits(p, q)
