"""GPU side of SURVEY.md 8(f) rows 1-2 against the CPU oracle, bit for bit: frame formats (fp16
accumulator, RGBA8 as the reference's RenderTexture), progressive accumulation, and the three
sections of ThreeWindowGroup batched into one launch. All calls go through the C ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMATS = {"f16": 1, "rgba8": 2, "f32": 0}


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype == np.uint8:
        return a == b
    ua = a.view(np.uint16 if a.dtype == np.float16 else np.uint32)
    ub = b.view(np.uint16 if b.dtype == np.float16 else np.uint32)
    return (ua == ub) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("name", ["sphere", "room", "tiger_two_mirrors", "all_primitives"])
@pytest.mark.parametrize("fmt", ["f16", "rgba8", "f32"])
def test_progressive_formats_bitwise(rt4, oracle, name, fmt):
    """Four progressive frames (part = 1/n, seed_n) into each frame format: GPU == oracle after every frame."""
    f = FORMATS[fmt]
    scene = rt4.Scene.named(name)
    base = rt4.make_uniforms(72, 44, samples=3, reflections=4, seed=2024)
    reg = rt4.region(72, 44)
    dt = oracle.FRAME_DTYPES[f]
    g = np.zeros((44, 72, 4), dt)
    c = np.zeros((44, 72, 4), dt)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        for n in range(1, 5):
            u = rt4.progressive_uniforms(base, n)
            ng = t.render_host_ex(u, reg, g, f)
            _, nc = oracle.render_fmt(scene.desc, u, reg, f, frame=c)
            assert ng == nc
            eq = bits_equal(g, c)
            assert eq.all(), f"frame {n}: {(~eq).sum()} values differ"
    finally:
        t.close()


def test_fp16_accumulator_vs_fp32(rt4):
    """BASELINE config 5 in miniature: 16 progressive frames of the all-primitive scene, fp16 accumulator
    against fp32. Tolerance: 4e-3 absolute (half's spacing just below 1 is 2^-11 = 4.9e-4; the
    per-frame rounding compounds over the frames)."""
    import torch

    scene = rt4.Scene.named("all_primitives")
    base = rt4.make_uniforms(256, 160, samples=4, reflections=8, seed=12345)
    reg = rt4.region(256, 160)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        f32 = torch.zeros((160, 256, 4), dtype=torch.float32, device="cuda")
        f16 = torch.zeros((160, 256, 4), dtype=torch.float16, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for n in range(1, 17):
            u = rt4.progressive_uniforms(base, n)
            t.render_device_ex(u, reg, f32.data_ptr(), rt4.FRAME_RGBA32F, 256, 0, s)
            t.render_device_ex(u, reg, f16.data_ptr(), rt4.FRAME_RGBA16F, 256, 0, s)
        torch.cuda.synchronize()
        d = (f16.float() - f32).abs()[..., :3]
        assert float(d.max()) <= 4e-3, float(d.max())
        assert float(f16[..., 3].float().min()) == 1.0
    finally:
        t.close()


def section_uniforms(rt4, section, w, h, seed=77):
    return rt4.make_uniforms(w, h, samples=3, reflections=4, seed=seed, section=section, fi=20.0, te=10.0, psi=30.0)


@pytest.mark.parametrize("fmt", ["f32", "f16"])
@pytest.mark.parametrize("name", ["tiger", "hypercube"])
def test_three_sections_one_launch(rt4, oracle, name, fmt):
    """ThreeWindowGroup::drawShaderImage (three_window_group.cpp:42-46): YXZ at the main window's
    resolution, YWZ and YXW at the additional one's, rendered in one launch; each image equals the
    oracle's render of that section alone, and the launch's count is the sum."""
    import torch

    f = FORMATS[fmt]
    scene = rt4.Scene.named(name)
    sizes = [(121, 75), (60, 37), (60, 37)]  # properties.txt:5-10 cells: 850/7 x (850/phi)/7, 600/10 x ...
    jobs, frames, us = [], [], []
    tdt = torch.float32 if f == 0 else torch.float16
    for sec, (w, h) in zip((rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW), sizes):
        u = section_uniforms(rt4, sec, w, h)
        fr = torch.zeros((h, w, 4), dtype=tdt, device="cuda")
        frames.append(fr)
        us.append(u)
        jobs.append((u, rt4.region(w, h), fr.data_ptr(), w))
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        t.render_sections_device(jobs, f, cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        total = 0
        for (w, h), u, fr in zip(sizes, us, frames):
            c, nc = oracle.render_fmt(scene.desc, u, rt4.region(w, h), f)
            total += nc
            eq = bits_equal(fr.cpu().numpy(), c)
            assert eq.all(), f"{(~eq).sum()} values differ"
        assert int(cnt.item()) == total
    finally:
        t.close()


def test_sections_reject_mismatched_shared_uniforms(rt4):
    import torch

    t = rt4.Tracer(device=0, scene=rt4.Scene.builtin("sphere"))
    try:
        fr = torch.zeros((20, 30, 4), dtype=torch.float32, device="cuda")
        u0 = section_uniforms(rt4, rt4.SECTION_YXZ, 30, 20)
        u1 = section_uniforms(rt4, rt4.SECTION_YWZ, 30, 20, seed=78)  # a different seed: not one frame
        with pytest.raises(rt4.RT4Error):
            t.render_sections_device([(u0, rt4.region(30, 20), fr.data_ptr(), 30),
                                      (u1, rt4.region(30, 20), fr.data_ptr(), 30)])
    finally:
        t.close()


@pytest.mark.parametrize("keys,fmt", [("", "f32"), ("WE", "rgba8")])
def test_cpp_host_program_matches_python_driver(rt4, tmp_path, keys, fmt):
    """lib/rt4_render (the C++ host over the C ABI: main.cpp's frame loop offscreen, three sections,
    progressive frames, optional WASD/EQ motion between frames) writes the same PPMs as the same loop
    driven from Python through the same ABI."""
    import os
    import subprocess

    import torch

    props_text = open(os.path.join(os.path.dirname(rt4.LIB_PATH), "..", "..", "properties.txt")).read()
    props_text = (props_text.replace("window.main.width = 850", "window.main.width = 140")
                  .replace("window.main.cell_size = 7", "window.main.cell_size = 2")
                  .replace("window.additional.width = 600", "window.additional.width = 100")
                  .replace("window.additional.cell_size = 10", "window.additional.cell_size = 4")
                  .replace("ray_tracing.samples = 100", "ray_tracing.samples = 2")
                  .replace("ray_tracing.reflections_amount = 4", "ray_tracing.reflections_amount = 3"))
    pfile = tmp_path / "properties.txt"
    pfile.write_text(props_text)
    exe = os.path.join(os.path.dirname(rt4.LIB_PATH), "rt4_render")
    cmd = [exe, "-p", str(pfile), "-s", "tiger", "-n", "3", "-3", "-f", fmt, "--seed", "4242", "-o", str(tmp_path / "cpp")]
    if keys:
        cmd += ["--keys", keys, "--move-seconds", "0.05"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr

    f = FORMATS[fmt]
    props = rt4.Properties(text=props_text)
    cam = rt4.Camera(props)
    cells = [rt4.window_cells(props, "main"), rt4.window_cells(props, "additional"), rt4.window_cells(props, "additional")]
    secs = [rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW]
    bases = [rt4.uniforms_from_properties(props, w, h, s) for (w, h), s in zip(cells, secs)]
    tdt = {0: torch.float32, 1: torch.float16, 2: torch.uint8}[f]
    frames = [torch.zeros((h, w, 4), dtype=tdt, device="cuda") for (w, h) in cells]
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=rt4.Scene.builtin("tiger"))
    keymask = sum({"W": rt4.KEY_FORWARD, "E": rt4.KEY_W_POS}[c] for c in keys)
    try:
        for n in range(1, 4):
            seed = 4242 ^ ((n * 0x9E3779B9) & 0xFFFFFFFF)
            fn = cam.s.frame_number
            jobs = []
            for q in range(3):
                cam.s.frame_number = fn
                u = cam.frame_uniforms(bases[q], secs[q], seed)
                jobs.append((u, rt4.region(*cells[q]), frames[q].data_ptr(), cells[q][0]))
            t.render_sections_device(jobs, f)
            if keymask:
                cam.move(keymask, 0.05)
        torch.cuda.synchronize()
    finally:
        t.close()
    for q, name in enumerate(("yxz", "ywz", "yxw")):
        ref = tmp_path / f"py_{name}.ppm"
        rt4.write_ppm(str(ref), frames[q].cpu().numpy(), f)
        assert (tmp_path / f"cpp_{name}.ppm").read_bytes() == ref.read_bytes(), name


def test_sections_argument_checks_and_empty_job(rt4, oracle):
    import torch

    scene = rt4.Scene.builtin("sphere")
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        fr = torch.zeros((20, 30, 4), dtype=torch.float32, device="cuda")
        u = section_uniforms(rt4, rt4.SECTION_YXZ, 30, 20)
        job = (u, rt4.region(30, 20), fr.data_ptr(), 30)
        with pytest.raises(rt4.RT4Error):
            t.render_sections_device([job] * 4)  # more than RT4_MAX_SECTIONS
        with pytest.raises(rt4.RT4Error):
            t.render_sections_device([job], fmt=9)  # unknown frame format
        with pytest.raises(rt4.RT4Error):
            t.render_sections_device([(u, rt4.region(30, 16384), fr.data_ptr(), 30)])  # h > 16383
        # an empty section next to a real one: the real one renders as if alone
        u2 = section_uniforms(rt4, rt4.SECTION_YWZ, 30, 20)
        t.render_sections_device([(u2, rt4.region(0, 0), 0, 0), job])
        torch.cuda.synchronize()
        c, _ = oracle.render_fmt(scene.desc, u, rt4.region(30, 20), 0)
        assert bits_equal(fr.cpu().numpy(), c).all()
    finally:
        t.close()


def test_launches_on_two_streams_and_a_large_frame(rt4, oracle):
    """One context used from two streams (the tile-order buffer is shared: launches run in submission
    order) and a frame above the preallocated 2^18 tiles (the buffer grows); images stay exact."""
    import torch

    scene = rt4.Scene.builtin("sphere")
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        u = rt4.make_uniforms(160, 100, samples=2, reflections=3, seed=9)
        reg = rt4.region(160, 100)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        frames = [torch.zeros((100, 160, 4), device="cuda") for _ in range(4)]
        for st in (s1, s2):  # the zero-fills (current stream) before the side streams' kernels
            st.wait_stream(torch.cuda.current_stream())
        for q, fr in enumerate(frames):
            st = s1 if q % 2 == 0 else s2
            t.render_device(u, reg, fr.data_ptr(), 160, 0, st.cuda_stream)
        torch.cuda.synchronize()
        c, _, _, _ = oracle.render(scene.desc, u, reg)
        for fr in frames:
            assert (fr.cpu().numpy().view(np.uint32) == c.view(np.uint32)).all()
        # 4160 x 4104 pixels = 520 x 513 tiles > 2^18: grows the order buffer
        W, H = 4160, 4104
        ub = rt4.make_uniforms(W, H, samples=1, reflections=1, seed=9)
        big = torch.zeros((H, W, 4), device="cuda")
        t.render_device(ub, rt4.region(W, H), big.data_ptr(), W, 0, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        rows = rt4.region(W, 3, y0=H // 2)
        cb, _, _, _ = oracle.render(scene.desc, ub, rows)
        assert (big[H // 2:H // 2 + 3].cpu().numpy().view(np.uint32) == cb.view(np.uint32)).all()
    finally:
        t.close()


def test_tile_order_reuse_follows_scene_and_camera(rt4, oracle):
    """The tile order is reused while the primary rays repeat: a new scene with the same camera, a
    moved camera, and back again all stay exact (any order is a permutation of the same tiles; this
    checks that a stale order never drops or repeats a tile)."""
    import torch

    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=rt4.Scene.builtin("sphere"))
    try:
        W, H = 96, 72
        reg = rt4.region(W, H)
        s = torch.cuda.current_stream().cuda_stream
        u0 = rt4.make_uniforms(W, H, samples=2, reflections=3, seed=5)
        u1 = rt4.make_uniforms(W, H, samples=2, reflections=3, seed=5)
        u1.focus[1] += 0.25  # moved camera
        u1.vec_to_mtr[0] += 0.1
        for name, u in (("sphere", u0), ("cylinder4d", u0), ("cylinder4d", u1), ("sphere", u1), ("sphere", u0)):
            scene = rt4.Scene.builtin(name)
            t.set_scene(scene)
            fr = torch.zeros((H, W, 4), device="cuda")
            t.render_device(u, reg, fr.data_ptr(), W, 0, s)
            t.render_device(u, reg, fr.data_ptr(), W, 0, s)  # second frame: reused order, accumulates
            torch.cuda.synchronize()
            c, _, _, _ = oracle.render(scene.desc, u, reg)
            c, _, _, _ = oracle.render(scene.desc, u, reg, frame=c)
            assert (fr.cpu().numpy().view(np.uint32) == c.view(np.uint32)).all(), name
    finally:
        t.close()


def test_queue_words_across_many_launches(rt4, oracle):
    """Each launch zeroes the next launch's rotating queue word (64 words, no memset between frames):
    150 launches, wrapping the words twice, on alternating streams with empty regions in between,
    must each render the whole frame. Per-launch intersection counts and the last frame are checked
    against the oracle."""
    import torch

    scene = rt4.Scene.builtin("sphere")
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        W, H = 40, 24
        u = rt4.make_uniforms(W, H, samples=1, reflections=2, seed=31)
        reg = rt4.region(W, H)
        c, n_ref, _, _ = oracle.render(scene.desc, u, reg)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        fr = torch.zeros((H, W, 4), device="cuda")
        counts = torch.zeros(150, dtype=torch.int64, device="cuda")
        for st in streams:  # the zero-fills (current stream) before the side streams' kernels
            st.wait_stream(torch.cuda.current_stream())
        for q in range(150):
            st = streams[(q // 7) % 2]
            if q % 11 == 5:  # an empty region launches nothing and must not consume a queue word
                t.render_device(u, rt4.region(0, 0), fr.data_ptr(), W, 0, st.cuda_stream)
            t.render_device(u, reg, fr.data_ptr(), W, counts[q:].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        assert counts.cpu().tolist() == [n_ref] * 150
        assert (fr.cpu().numpy().view(np.uint32) == c.view(np.uint32)).all()
    finally:
        t.close()


@pytest.mark.parametrize("fmt", ["f32", "f16"])
def test_progressive_resume_bitwise(rt4, tmp_path, fmt):
    """Accumulator checkpoint / resume (rt4_accum_save / rt4_accum_load): 5 progressive frames, a checkpoint,
    a fresh context and 4 more frames from the loaded accumulator equal 9 frames in one run, bit for bit
    (the blend part = 1/n and seed_n continue from the checkpoint's frame count; main.cpp:86-91)."""
    import torch

    f = FORMATS[fmt]
    tdt = {0: torch.float32, 1: torch.float16}[f]
    W, H = 96, 64
    base = rt4.make_uniforms(W, H, samples=3, reflections=5, seed=31337)
    reg = rt4.region(W, H)
    scene = rt4.Scene.named("all_primitives")

    def run(frame, first, last):
        t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
        try:
            t.render_frames_device([rt4.progressive_uniforms(base, n) for n in range(first, last + 1)], reg,
                                   frame.data_ptr(), f, W, 0, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
        finally:
            t.close()

    whole = torch.zeros((H, W, 4), dtype=tdt, device="cuda")
    run(whole, 1, 9)
    part = torch.zeros((H, W, 4), dtype=tdt, device="cuda")
    run(part, 1, 5)
    path = str(tmp_path / "acc.rt4")
    rt4.accum_save(path, part.cpu().numpy(), frames_done=5, seed=31337, fmt=f)
    host, done, seed = rt4.accum_load(path)
    assert (done, seed) == (5, 31337)
    resumed = torch.from_numpy(host).cuda()
    run(resumed, done + 1, 9)
    eq = bits_equal(resumed.cpu().numpy(), whole.cpu().numpy())
    assert eq.all(), f"{(~eq).sum()} values differ"


def test_cpp_host_program_resume(rt4, tmp_path):
    """rt4_render --checkpoint / --resume: 3 frames, checkpoint, 3 more resumed frames write the same PPM
    (and the same checkpoint) as 6 frames in one run."""
    import os
    import subprocess

    exe = os.path.join(os.path.dirname(rt4.LIB_PATH), "rt4_render")
    props = os.path.join(os.path.dirname(rt4.LIB_PATH), "..", "..", "properties.txt")
    common = [exe, "-p", props, "-s", "sphere", "-W", "120", "-H", "80", "--seed", "99", "-f", "f32"]

    def go(*args):
        r = subprocess.run(common + list(args), capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr

    go("-n", "6", "-o", str(tmp_path / "whole"), "--checkpoint", str(tmp_path / "whole.rt4"))
    go("-n", "3", "-o", str(tmp_path / "a"), "--checkpoint", str(tmp_path / "a.rt4"))
    assert rt4.accum_info(str(tmp_path / "a.rt4"))["frames_done"] == 3
    go("-n", "3", "-o", str(tmp_path / "b"), "--resume", str(tmp_path / "a.rt4"), "--checkpoint", str(tmp_path / "b.rt4"))
    assert (tmp_path / "b_yxz.ppm").read_bytes() == (tmp_path / "whole_yxz.ppm").read_bytes()
    assert (tmp_path / "b.rt4").read_bytes() == (tmp_path / "whole.rt4").read_bytes()
    r = subprocess.run(common[:-4] + ["--seed", "100", "-n", "1", "-o", str(tmp_path / "c"), "--resume",
                                      str(tmp_path / "a.rt4")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "another --seed" in r.stderr
    # the run key: another scene, another sample count or another resolution is refused
    assert rt4.accum_key_of(str(tmp_path / "a.rt4")) != 0
    for change in (["-s", "room"], ["-p", str(_props_samples(tmp_path, 7))]):
        args = list(common)
        i = args.index(change[0])
        args[i + 1] = change[1]
        r = subprocess.run(args + ["-n", "1", "-o", str(tmp_path / "d"), "--resume", str(tmp_path / "a.rt4")],
                           capture_output=True, text=True, timeout=120)
        assert r.returncode != 0 and "another scene, properties or camera" in r.stderr, (change, r.stderr)
    # a failed checkpoint write (the .tmp name taken) keeps the checkpoint being resumed from intact
    before = (tmp_path / "a.rt4").read_bytes()
    os.mkdir(str(tmp_path / "a.rt4") + ".tmp")
    r = subprocess.run(common + ["-n", "1", "-o", str(tmp_path / "e"), "--resume", str(tmp_path / "a.rt4"),
                                 "--checkpoint", str(tmp_path / "a.rt4")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and (tmp_path / "a.rt4").read_bytes() == before


def _props_samples(tmp_path, samples):
    import os
    import re

    src = open(os.path.join(os.path.dirname(__file__), "..", "properties.txt")).read()
    path = tmp_path / f"props_{samples}.txt"
    path.write_text(re.sub(r"ray_tracing\.samples = \d+", f"ray_tracing.samples = {samples}", src))
    return path


def test_cpp_host_program_png(rt4, tmp_path):
    """rt4_render --png writes PNGs whose pixels are the PPM's (rt4_write_png; decoded with zlib here)."""
    import os
    import struct
    import subprocess
    import zlib

    exe = os.path.join(os.path.dirname(rt4.LIB_PATH), "rt4_render")
    props = os.path.join(os.path.dirname(rt4.LIB_PATH), "..", "..", "properties.txt")
    common = [exe, "-p", props, "-s", "room", "-W", "96", "-H", "60", "-n", "2", "-f", "f16"]
    for extra, pre in (([], "a"), (["--png"], "b")):
        r = subprocess.run(common + ["-o", str(tmp_path / pre)] + extra, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
    ppm = (tmp_path / "a_yxz.ppm").read_bytes()[len(b"P6\n96 60\n255\n"):]
    png = (tmp_path / "b_yxz.png").read_bytes()
    n, = struct.unpack(">I", png[33:37])
    assert png[37:41] == b"IDAT"
    raw = zlib.decompress(png[41:41 + n])
    assert b"".join(raw[i * 289 + 1:(i + 1) * 289] for i in range(60)) == ppm


@pytest.mark.parametrize("fmt", ["f32", "f16", "rgba8"])
@pytest.mark.parametrize("name", ["sphere", "all_primitives"])
def test_overlapped_frames_equal_serial(rt4, name, fmt):
    """Single-frame launches overlap the previous frame's drain by default (rt4.h RT4_FLAG_SERIAL_FRAMES: the
    trace on a side stream into a slot buffer, the blend and the count on the caller's stream).
    A moving camera (new uniforms every frame, main.cpp:93), progressive parts, a pipelined call in between, a
    frame on a second stream and a scene change: every frame and the count equal the serial launches bit for
    bit after every step."""
    import torch

    f = FORMATS[fmt]
    tdt = {0: torch.float32, 1: torch.float16, 2: torch.uint8}[f]
    W, H = 131, 77
    reg = rt4.region(W, H)
    frames = [rt4.make_uniforms(W, H, samples=3, reflections=4, seed=40 + n, fi=5.0 * n, te=2.0 * n) for n in range(6)]
    runs = []
    for flags in (rt4.FLAG_SAMPLER_LUT, rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES):
        t = rt4.Tracer(device=0, flags=flags, scene=rt4.Scene.named(name))
        out = []
        try:
            fr = torch.zeros((H, W, 4), dtype=tdt, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            s = torch.cuda.current_stream()
            for n, u in enumerate(frames[:3]):
                t.render_device_ex(rt4.progressive_uniforms(u, n + 1), reg, fr.data_ptr(), f, W, cnt.data_ptr(),
                                   s.cuda_stream)
            out.append((fr.clone(), cnt.clone()))
            t.reserve_frames(W, H)
            t.render_frames_device([rt4.progressive_uniforms(frames[3], n) for n in (4, 5, 6)], reg, fr.data_ptr(), f,
                                   W, cnt.data_ptr(), s.cuda_stream)
            t.render_device_ex(rt4.progressive_uniforms(frames[4], 7), reg, fr.data_ptr(), f, W, cnt.data_ptr(),
                               s.cuda_stream)
            out.append((fr.clone(), cnt.clone()))
            side = torch.cuda.Stream()
            side.wait_stream(s)
            t.render_device_ex(rt4.progressive_uniforms(frames[5], 8), reg, fr.data_ptr(), f, W, cnt.data_ptr(),
                               side.cuda_stream)
            s.wait_stream(side)
            out.append((fr.clone(), cnt.clone()))
            t.set_scene(rt4.Scene.named("hypercube"))
            for n in range(2):
                t.render_device_ex(rt4.progressive_uniforms(frames[n], 9 + n), reg, fr.data_ptr(), f, W, cnt.data_ptr(),
                                   s.cuda_stream)
            out.append((fr.clone(), cnt.clone()))
            torch.cuda.synchronize()
        finally:
            t.close()
        runs.append([(a.cpu().numpy(), int(c.item())) for a, c in out])
    for step, ((a, na), (b, nb)) in enumerate(zip(*runs)):
        assert na == nb, (step, na, nb)
        eq = bits_equal(a, b)
        assert eq.all(), f"step {step}: {(~eq).sum()} values differ"


@pytest.mark.parametrize("fmt", ["f32", "rgba8"])
@pytest.mark.parametrize("name", ["tiger", "sphere"])
def test_overlapped_sections_equal_serial(rt4, name, fmt):
    """Sections launches (three_window_group.cpp:42-46: YXZ at the main window's size, YWZ and YXW at the
    additional one's) overlap like single frames: each section's image in its own part of the
    slot buffer, one blend per section. A moving camera over progressive frames, with single-frame launches of a
    larger region in between (the slot buffer grows and is shared): every image and the count equal the serial
    launches bit for bit."""
    import torch

    f = FORMATS[fmt]
    tdt = {0: torch.float32, 2: torch.uint8}[f]
    sizes = [(121, 75), (60, 37), (60, 37)]
    secs = (rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW)
    runs = []
    for flags in (rt4.FLAG_SAMPLER_LUT, rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES):
        t = rt4.Tracer(device=0, flags=flags, scene=rt4.Scene.named(name))
        out = []
        try:
            frames = [torch.zeros((h, w, 4), dtype=tdt, device="cuda") for (w, h) in sizes]
            big = torch.zeros((90, 150, 4), dtype=tdt, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            s = torch.cuda.current_stream().cuda_stream
            for n in range(5):
                jobs = []
                for q, ((w, h), sec) in enumerate(zip(sizes, secs)):
                    u = rt4.make_uniforms(w, h, samples=3, reflections=4, seed=90, section=sec, fi=20.0 + 4 * n,
                                          te=10.0, psi=30.0)
                    jobs.append((rt4.progressive_uniforms(u, n + 1), rt4.region(w, h), frames[q].data_ptr(), w))
                t.render_sections_device(jobs, f, cnt.data_ptr(), s)
                if n == 2:
                    ub = rt4.make_uniforms(150, 90, samples=3, reflections=4, seed=91)
                    t.render_device_ex(ub, rt4.region(150, 90), big.data_ptr(), f, 150, cnt.data_ptr(), s)
                out.append([fr.clone() for fr in frames] + [big.clone(), cnt.clone()])
            torch.cuda.synchronize()
        finally:
            t.close()
        runs.append([[x.cpu().numpy() for x in step[:-1]] + [int(step[-1].item())] for step in out])
    for n, (a, b) in enumerate(zip(*runs)):
        assert a[-1] == b[-1], (n, a[-1], b[-1])
        for q in range(4):
            eq = bits_equal(a[q], b[q])
            assert eq.all(), f"frame {n} image {q}: {(~eq).sum()} values differ"


@pytest.mark.parametrize("name", ["sphere", "all_primitives"])
def test_overlap_rotations_cap_and_memory(rt4, name):
    """The overlap's two rotations (rt4.h RT4_FLAG_SERIAL_FRAMES / RT4_FLAG_OVERLAP_SHALLOW; DESIGN.md §4.28,
    ADVICE r04): small frames run 8 deep with 8 slot buffers, frames that fill the chip 3 deep with 3 buffers, and
    switching between them drains the launches in flight. Small, big and small frames again, with the default, the
    3-deep cap and serial launches: every frame and the count equal the serial ones bit for bit, and the slot memory
    is what rt4.h states: launch s uses buffer s % 8 when small, s % 3 when big (so launches 0-2 and 6-7 leave small
    buffers 6 and 7 and big buffers 0-2 by default), buffer s % 3 with the cap, none serial."""
    import torch

    small, big = (131, 77), (1024, 640)  # 170 tiles; 10240 tiles: more than the chip holds waves
    seq = [small] * 3 + [big] * 3 + [small] * 2
    us = [rt4.make_uniforms(w, h, samples=2, reflections=2, seed=300 + n, fi=3.0 * n) for n, (w, h) in enumerate(seq)]
    px = {s: s[0] * s[1] * 16 for s in (small, big)}
    expect_bytes = {rt4.FLAG_SAMPLER_LUT: 3 * px[big] + 2 * px[small],
                    rt4.FLAG_SAMPLER_LUT | rt4.FLAG_OVERLAP_SHALLOW: 3 * px[big],
                    rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES: 0}
    runs = {}
    for flags, want in expect_bytes.items():
        t = rt4.Tracer(device=0, flags=flags, scene=rt4.Scene.named(name))
        try:
            frs = {s: torch.zeros((s[1], s[0], 4), device="cuda") for s in (small, big)}
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            stream = torch.cuda.current_stream().cuda_stream
            out = []
            for (w, h), u in zip(seq, us):
                t.render_device(u, rt4.region(w, h), frs[(w, h)].data_ptr(), w, cnt.data_ptr(), stream)
                out.append(frs[(w, h)].clone())
            torch.cuda.synchronize()
            assert t.overlap_bytes() == want, (flags, t.overlap_bytes(), want)
        finally:
            t.close()
        runs[flags] = ([x.cpu().numpy() for x in out], int(cnt.item()))
    ref_frames, ref_count = runs[rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES]
    for flags, (frames, count) in runs.items():
        assert count == ref_count, (flags, count, ref_count)
        for n, (a, b) in enumerate(zip(frames, ref_frames)):
            eq = bits_equal(a, b)
            assert eq.all(), f"flags {flags:#x} frame {n}: {(~eq).sum()} values differ"


def test_reserve_overlap_allocates_ahead(rt4):
    """rt4_context_reserve_overlap sizes the slot buffers a frame of that size uses (3 for a frame that fills
    the chip), so its first launch grows nothing; a serial context reserves nothing."""
    import torch

    W, H = 1024, 640
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=rt4.Scene.named("sphere"))
    try:
        assert t.overlap_bytes() == 0
        t.reserve_overlap(W, H)
        assert t.overlap_bytes() == 3 * W * H * 16
        fr = torch.zeros((H, W, 4), device="cuda")
        t.render_device(rt4.make_uniforms(W, H, samples=1, reflections=1, seed=5), rt4.region(W, H), fr.data_ptr(), W)
        torch.cuda.synchronize()
        assert t.overlap_bytes() == 3 * W * H * 16
    finally:
        t.close()
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT | rt4.FLAG_SERIAL_FRAMES, scene=rt4.Scene.named("sphere"))
    try:
        t.reserve_overlap(W, H)
        assert t.overlap_bytes() == 0
    finally:
        t.close()
