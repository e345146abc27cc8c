"""The BASELINE.json configs at their stated shapes on the MI355X, against the CPU oracle.

  config 2 / 3: the whole 1920x1080 frame (16 spp, 8 bounces) bit for bit, every pixel, and the
                intersection count (the oracle runs on all host threads, ~0.3-0.5 s per frame).
  config 4:     tiger + two mirrors, 3840x2160, 64 spp, 12 bounces: see test_gpu_shard.py (the frame
                split over 8 ranks == the whole frame) and test_gpu_parity.py (rows vs the oracle).
  config 5:     all_primitives, 3840x2160, progressive to 4096 spp (256 frames x 16 spp, part = 1/n,
                seed_n = seed ^ n*0x9E3779B9), fp16 accumulator against fp32: full-frame invariants at
                every size, bit-exactness against the oracle on two rows after frames 1, 2 and 256
                (all 256 frames of those rows run on the oracle), and the fp16 - fp32 difference
                against its derived bound.
Reference: executable/shader.frag:513-528 (main), src/main.cpp:72,86-88 (progressive frames).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU


def bits_equal(a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    ua = a.view(np.uint16 if a.dtype == np.float16 else np.uint32)
    ub = b.view(np.uint16 if b.dtype == np.float16 else np.uint32)
    return (ua == ub) | (np.isnan(a) & np.isnan(b))


@pytest.mark.parametrize("name,config", [("sphere", 2), ("hypercube", 3)])
def test_full_frame_1080p_bitwise(rt4, oracle, name, config):
    """BASELINE config 2 / 3: every pixel of the 1920x1080 x 16 spp x 8 bounce frame, seed 12345, with
    and without primary-ray reuse (RT4_FLAG_PRIMARY_REUSE: same image, same reference count, fewer
    evaluated find calls)."""
    import torch

    scene = rt4.Scene.named(name)
    u = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=12345)
    reg = rt4.region(1920, 1080)
    c, nc, _, _ = oracle.render(scene.desc, u, reg, threads=THREADS)
    for flags in (rt4.FLAG_SAMPLER_LUT, rt4.FLAG_SAMPLER_LUT | rt4.FLAG_PRIMARY_REUSE):
        t = rt4.Tracer(device=0, flags=flags, scene=scene)
        try:
            fr = torch.zeros((1080, 1920, 4), dtype=torch.float32, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
            t.render_device(u, reg, fr.data_ptr(), 1920, cnt.data_ptr(), torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            g = fr.cpu().numpy()
            n_eval = t.evaluated()
        finally:
            t.close()
        assert int(cnt.item()) == nc
        eq = bits_equal(g, c)
        assert eq.all(), f"config {config} flags {flags}: {(~eq).sum()} of {eq.size} values differ"
        assert (g[..., 3] == 1.0).all() and (g[..., :3] >= 0).all() and (g[..., :3] < 1).all()
        if flags & rt4.FLAG_PRIMARY_REUSE:
            # 16 primary finds per pixel become one: nc - 15 * W * H evaluated
            assert n_eval == nc - 15 * 1920 * 1080, (n_eval, nc)


@pytest.mark.parametrize("name,config", [("sphere", 2), ("hypercube", 3)])
def test_bench_call_1080p_bitwise(rt4, oracle, name, config):
    """The exact call the bench times for BASELINE config 2 / 3 (bench.py: 20 identical frames, part 1,
    one rt4_render_frames_device call after rt4_context_reserve_frames, into a frame that holds the
    warmup's image): the final frame equals the oracle's full 1920x1080 frame bit for bit and the
    count is 20 x the oracle's. Reference: shader.frag:513-528, main.cpp:57-111."""
    import torch

    scene = rt4.Scene.named(name)
    u = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=12345)
    reg = rt4.region(1920, 1080)
    c, nc, _, _ = oracle.render(scene.desc, u, reg, threads=THREADS)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    try:
        s = torch.cuda.current_stream().cuda_stream
        fr = torch.rand((1080, 1920, 4), dtype=torch.float32, device="cuda")  # old contents (part 1 replaces)
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        t.reserve_frames(1920, 1080)
        t.render_frames_device([u] * 3, reg, fr.data_ptr(), rt4.FRAME_RGBA32F, 1920, 0, s)  # the warmup
        t.render_frames_device([u] * 20, reg, fr.data_ptr(), rt4.FRAME_RGBA32F, 1920, cnt.data_ptr(), s)
        torch.cuda.synchronize()
        assert t.frames_per_launch(1920, 1080) >= 20  # one pipelined launch holds all 20 frames
        g = fr.cpu().numpy()
    finally:
        t.close()
    assert int(cnt.item()) == 20 * nc
    eq = bits_equal(g, c)
    assert eq.all(), f"config {config}: {(~eq).sum()} of {eq.size} values differ"


def fp16_blend_bound(n):
    """Worst-case |fp16 - fp32| accumulator difference after n progressive frames of values in [0, 1).

    Frame k stores v_k = RN16(old*(1 - 1/k) + c_k/k) instead of the fp32 value, an error of at most
    half an fp16 ulp below 1, 2^-12. The error e_k = e_(k-1) (1 - 1/k) + d_k telescopes to
    e_n = (1/n) sum_k k d_k, so |e_n| <= 2^-12 (n + 1) / 2 (the fp32 path's own rounding, < 2^-24 per
    frame, is below this bound's slack)."""
    return 2.0 ** -12 * (n + 1) / 2.0


def test_config5_progressive_4k_fp16_vs_fp32(rt4, oracle):
    """BASELINE config 5 at its stated shape: all_primitives, 3840x2160, 256 progressive frames x 16
    spp = 4096 spp, fp16 and fp32 accumulators on the GPU."""
    import torch

    W, H, N = 3840, 2160, 256
    scene = rt4.Scene.named("all_primitives")
    base = rt4.make_uniforms(W, H, samples=16, reflections=8, seed=12345)
    rows = (1003, 1703)  # image rows checked against the oracle (upper-middle and lower half)
    reg_rows = rt4.region(W, 2, y0=rows[0], band_rows=1, band_step=rows[1] - rows[0])
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT, scene=scene)
    s = torch.cuda.current_stream().cuda_stream
    snaps = {}
    try:
        f32 = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
        f16 = torch.zeros((H, W, 4), dtype=torch.float16, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
        reg = rt4.region(W, H)
        for n in range(1, N + 1):
            u = rt4.progressive_uniforms(base, n)
            t.render_device_ex(u, reg, f32.data_ptr(), rt4.FRAME_RGBA32F, W, cnt.data_ptr(), s)
            t.render_device_ex(u, reg, f16.data_ptr(), rt4.FRAME_RGBA16F, W, 0, s)
            if n in (1, 2, N):
                snaps[n] = (f32[list(rows)].cpu().numpy(), f16[list(rows)].cpu().numpy())
            if n in (1, 16, 64, N):
                d = (f16.float() - f32).abs()[..., :3]
                dmax = float(d.max())
                print(f"frame {n}: max |fp16 - fp32| = {dmax:.3e} (bound {fp16_blend_bound(n):.3e}), "
                      f"mean {float(d.mean()):.3e}")
                assert dmax <= fp16_blend_bound(n), (n, dmax)
        torch.cuda.synchronize()
        # full-frame invariants after 4096 spp
        c32 = f32[..., :3]
        assert float(c32.min()) >= 0.0 and float(c32.max()) < 1.0
        assert bool((f32[..., 3] == 1.0).all()) and bool((f16[..., 3] == 1.0).all())
        c16 = f16[..., :3].float()
        assert float(c16.min()) >= 0.0 and float(c16.max()) <= 1.0  # RN to fp16 may reach 1.0
        assert not bool(torch.isnan(f32).any()) and not bool(torch.isnan(f16.float()).any())
        n_gpu = int(cnt.item())
    finally:
        t.close()
    # the oracle runs all 256 frames on the two rows (its pixels do not depend on other rows)
    o32 = np.zeros((2, W, 4), np.float32)
    o16 = np.zeros((2, W, 4), np.float16)
    n_rows = 0
    for n in range(1, N + 1):
        u = rt4.progressive_uniforms(base, n)
        _, k = oracle.render_fmt(scene.desc, u, reg_rows, rt4.FRAME_RGBA32F, frame=o32, threads=THREADS)
        oracle.render_fmt(scene.desc, u, reg_rows, rt4.FRAME_RGBA16F, frame=o16, threads=THREADS)
        n_rows += k
        if n in snaps:
            g32, g16 = snaps[n]
            assert bits_equal(g32, o32).all(), f"fp32 rows differ after frame {n}"
            assert bits_equal(g16, o16).all(), f"fp16 rows differ after frame {n}"
    assert W * H * 16 * N <= n_gpu <= W * H * 16 * 9 * N  # >= 1 and <= bounces + 1 per sample, every frame
