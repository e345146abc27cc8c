"""Frame formats, progressive accumulation and the section bases on the CPU:
host logic of librt4.so and the oracle's format paths. The GPU side is in test_gpu_frames.py."""
import ctypes

import numpy as np
import pytest


def test_frame_format_bytes(rt4):
    assert [rt4.frame_format_bytes(f) for f in (rt4.FRAME_RGBA32F, rt4.FRAME_RGBA16F, rt4.FRAME_RGBA8)] == [16, 8, 4]
    assert rt4.frame_format_bytes(7) == 0


def test_progressive_uniforms(rt4):
    """part = 1/frameNumber (main.cpp:87); seed_n = seed ^ n*0x9E3779B9 (deterministic stand-in for the
    per-frame time seed, main.cpp:86)."""
    u = rt4.make_uniforms(64, 40, samples=4, reflections=2, seed=12345)
    for n in (1, 2, 3, 7, 256, 4096):
        v = rt4.progressive_uniforms(u, n)
        assert v.part == np.float32(1.0) / np.float32(n)
        assert (v.seed & 0xFFFFFFFF) == (12345 ^ (n * 0x9E3779B9)) & 0xFFFFFFFF
        assert bytes(v)[8:] != b"" and v.samples == u.samples and list(v.focus) == list(u.focus)
    with pytest.raises(rt4.RT4Error):
        rt4.progressive_uniforms(u, 0)


def test_half_conversion_matches_ieee(oracle):
    """The oracle's float->half (round to nearest even, subnormals, overflow) against numpy."""
    rng = np.random.default_rng(11)
    bits = rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32)
    special = np.array([0.0, -0.0, 1.0, -1.0, 65504.0, 65519.99, 65520.0, 1e6, np.inf, -np.inf, 2.0**-24, 2.0**-25,
                        2.0**-25 * 1.0000001, 3 * 2.0**-26, 2.0**-14, 2.0**-14 * (1 - 2.0**-12), 0.1, 1 / 3],
                       np.float32)
    x = np.concatenate([bits.view(np.float32), special,
                        rng.uniform(0, 1, 5000).astype(np.float32), rng.uniform(-7e-5, 7e-5, 5000).astype(np.float32)])
    x = x[~np.isnan(x)]
    got = oracle.float_to_half_bits(x)
    with np.errstate(over="ignore"):
        want = x.astype(np.float16).view(np.uint16)
    assert (got == want).all(), np.argwhere(got != want)[:5]
    h = np.arange(1 << 16, dtype=np.uint32).astype(np.uint16)
    back = oracle.half_bits_to_float(h)
    ref = h.view(np.float16).astype(np.float32)
    same = (back.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(back) & np.isnan(ref))
    assert same.all()


def test_oracle_formats_agree_with_fp32(rt4, oracle):
    """One frame into each format: fp16 is the fp32 blend rounded to half; RGBA8 (GL RenderTexture,
    windows.cpp:31) is the fp32 blend of the quantised old frame, quantised again."""
    scene = rt4.Scene.builtin("sphere")
    u = rt4.make_uniforms(48, 30, samples=2, reflections=3, seed=21)
    reg = rt4.region(48, 30)
    f32, n32, _, _ = oracle.render(scene.desc, u, reg, threads=4)
    f16, n16 = oracle.render_fmt(scene.desc, u, reg, rt4.FRAME_RGBA16F, threads=4)
    f8, n8 = oracle.render_fmt(scene.desc, u, reg, rt4.FRAME_RGBA8, threads=4)
    assert n32 == n16 == n8
    assert (f16 == f32.astype(np.float16)).all()  # part = 1, old = 0: the blend is exact, one rounding
    q = (np.clip(f32[..., :3], 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    assert (f8[..., :3] == q).all() and (f8[..., 3] == 255).all()


def test_progressive_rgba8_compounds_quantisation(rt4, oracle):
    """Several progressive frames: the 8-bit frame drifts from the fp32 one by the compounding per-frame
    quantisation the reference's RGBA8 texture has, and stays within a few 1/255 steps."""
    scene = rt4.Scene.builtin("room")
    base = rt4.make_uniforms(32, 20, samples=2, reflections=3, seed=99)
    reg = rt4.region(32, 20)
    f32 = np.zeros((20, 32, 4), np.float32)
    f8 = np.zeros((20, 32, 4), np.uint8)
    f16 = np.zeros((20, 32, 4), np.float16)
    for n in range(1, 9):
        u = rt4.progressive_uniforms(base, n)
        oracle.render(scene.desc, u, reg, frame=f32, threads=4)
        oracle.render_fmt(scene.desc, u, reg, rt4.FRAME_RGBA8, frame=f8, threads=4)
        oracle.render_fmt(scene.desc, u, reg, rt4.FRAME_RGBA16F, frame=f16, threads=4)
    d8 = np.abs(f8[..., :3].astype(np.float32) / 255 - f32[..., :3])
    d16 = np.abs(f16[..., :3].astype(np.float32) - f32[..., :3])
    assert d8.max() <= 8 / 255
    assert d16.max() <= 4e-3
