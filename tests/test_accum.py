"""Accumulator checkpoint / resume (rt4_accum_save / rt4_accum_info / rt4_accum_load, include/rt4.h) on the CPU:
round trips in every frame format, padded strides, and the error paths. The reference keeps its progressive
average only in the window texture (main.cpp:86-91) and restarts it when the camera moves (controls.cpp:132,
181,190); the GPU test (test_gpu_frames.py::test_progressive_resume_bitwise) shows a resumed run continues the
blend bit for bit."""
import ctypes
import os

import numpy as np
import pytest


@pytest.mark.parametrize("dtype", ["float32", "float16", "uint8"])
def test_round_trip_every_format(rt4, tmp_path, dtype):
    rng = np.random.default_rng(7)
    if dtype == "uint8":
        frame = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    else:
        frame = rng.random((37, 53, 4)).astype(dtype)
        frame[0, 0, 0] = np.nan  # bits, not values: a NaN channel survives
    path = str(tmp_path / "acc.rt4")
    rt4.accum_save(path, frame, frames_done=41, seed=0xDEADBEEF)
    info = rt4.accum_info(path)
    assert info == {"w": 53, "h": 37, "format": {"float32": rt4.FRAME_RGBA32F, "float16": rt4.FRAME_RGBA16F,
                                                  "uint8": rt4.FRAME_RGBA8}[dtype],
                    "frames_done": 41, "seed": 0xDEADBEEF}
    back, n, seed = rt4.accum_load(path)
    assert back.dtype == frame.dtype and back.shape == frame.shape
    assert back.tobytes() == frame.tobytes()
    assert (n, seed) == (41, 0xDEADBEEF)
    assert os.path.getsize(path) == 40 + frame.nbytes  # header + rows without padding


def test_padded_stride_and_header_layout(rt4, tmp_path):
    lib = rt4.lib
    h, w, stride = 5, 7, 11
    buf = np.arange(h * stride * 4, dtype=np.float32).reshape(h, stride, 4)
    path = str(tmp_path / "s.rt4")
    err = ctypes.create_string_buffer(256)
    assert lib.rt4_accum_save(os.fsencode(path), ctypes.c_void_p(buf.ctypes.data), rt4.FRAME_RGBA32F, w, h, stride,
                              3, 9, err, len(err)) == 0
    raw = open(path, "rb").read()
    assert raw[:8] == b"RT4ACC1\0"
    version, fw, fh, fmt, done, seed, res = np.frombuffer(raw[8:40], dtype="<i4,<i4,<i4,<i4,<i8,<u4,<u4")[0]
    assert (version, fw, fh, fmt, done, seed, res) == (2, w, h, rt4.FRAME_RGBA32F, 3, 9, 0)  # key 0: not recorded
    pixels = np.frombuffer(raw[40:], dtype=np.float32).reshape(h, w, 4)
    assert np.array_equal(pixels, buf[:, :w])  # the padding columns are not stored
    out = np.full((h, stride, 4), -1.0, dtype=np.float32)
    n, sd = ctypes.c_int64(), ctypes.c_uint32()
    assert lib.rt4_accum_load(os.fsencode(path), ctypes.c_void_p(out.ctypes.data), rt4.FRAME_RGBA32F, w, h, stride,
                              ctypes.byref(n), ctypes.byref(sd), err, len(err)) == 0
    assert np.array_equal(out[:, :w], buf[:, :w]) and (out[:, w:] == -1.0).all()
    assert (n.value, sd.value) == (3, 9)


def test_errors(rt4, tmp_path):
    lib = rt4.lib
    err = ctypes.create_string_buffer(256)
    frame = np.zeros((4, 4, 4), dtype=np.float32)
    good = str(tmp_path / "g.rt4")
    rt4.accum_save(good, frame, 2, 1)
    # wrong size / format on load: RT4_ERR_ARG, buffer untouched
    out = np.ones((4, 5, 4), dtype=np.float32)
    rc = lib.rt4_accum_load(os.fsencode(good), ctypes.c_void_p(out.ctypes.data), rt4.FRAME_RGBA32F, 5, 4, 5, None,
                            None, err, len(err))
    assert rc == -1 and b"4x4" in err.value and (out == 1).all()
    rc = lib.rt4_accum_load(os.fsencode(good), ctypes.c_void_p(out.ctypes.data), rt4.FRAME_RGBA16F, 4, 4, 4, None,
                            None, err, len(err))
    assert rc == -1
    # not a checkpoint, a truncated one, an unknown version, a missing file
    bad = tmp_path / "b.rt4"
    bad.write_bytes(b"P6\n4 4\n255\n" + bytes(48))
    with pytest.raises(rt4.RT4Error, match="not an rt4 accumulator checkpoint"):
        rt4.accum_info(str(bad))
    raw = open(good, "rb").read()
    (tmp_path / "t.rt4").write_bytes(raw[:-16])
    with pytest.raises(rt4.RT4Error, match="truncated"):
        rt4.accum_load(str(tmp_path / "t.rt4"))
    (tmp_path / "v.rt4").write_bytes(raw[:8] + (3).to_bytes(4, "little") + raw[12:])
    with pytest.raises(rt4.RT4Error, match="version 3"):
        rt4.accum_info(str(tmp_path / "v.rt4"))
    with pytest.raises(rt4.RT4Error, match="cannot open"):
        rt4.accum_info(str(tmp_path / "missing.rt4"))
    # bad arguments on save
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 99, 4, 4, 4, 0, 0, err, len(err)) == -1
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 0, 4, 4, 3, 0, 0, err, len(err)) == -1
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 0, 4, 4, 4, -1, 0, err, len(err)) == -1


def test_version1_files_still_load(rt4, tmp_path):
    """A round-3 checkpoint (version 1, reserved word 0) loads; its key reads as 0 (not recorded)."""
    frame = np.arange(3 * 5 * 4, dtype=np.float32).reshape(3, 5, 4)
    path = str(tmp_path / "v1.rt4")
    rt4.accum_save(path, frame, 7, 11, key=0x1234)
    raw = bytearray(open(path, "rb").read())
    raw[8:12] = (1).to_bytes(4, "little")  # version 1, key field back to the reserved 0
    raw[36:40] = bytes(4)
    open(path, "wb").write(bytes(raw))
    back, n, sd = rt4.accum_load(path)
    assert back.tobytes() == frame.tobytes() and (n, sd) == (7, 11)
    assert rt4.accum_key_of(path) == 0


def test_run_key_records_what_decides_the_image(rt4, tmp_path):
    """rt4_accum_key: another scene, sample count, bounce count, resolution or camera pose changes the key; the
    seed and part (which change every frame) do not. rt4_accum_save_key records it (a resume with
    another -s or properties.txt must be refused, not blended in silently)."""
    u = rt4.make_uniforms(64, 40, samples=4, reflections=4, seed=1)
    sphere, cube = rt4.Scene.builtin("sphere"), rt4.Scene.builtin("hypercube")
    k = rt4.accum_key(sphere, u)
    assert k != 0 and k == rt4.accum_key(sphere, rt4.make_uniforms(64, 40, samples=4, reflections=4, seed=99))
    assert k == rt4.accum_key(sphere, rt4.progressive_uniforms(u, 5))  # part = 1/5, seed_5
    others = [rt4.accum_key(cube, u),
              rt4.accum_key(sphere, rt4.make_uniforms(64, 40, samples=5, reflections=4, seed=1)),
              rt4.accum_key(sphere, rt4.make_uniforms(64, 40, samples=4, reflections=3, seed=1)),
              rt4.accum_key(sphere, rt4.make_uniforms(64, 41, samples=4, reflections=4, seed=1))]
    moved = rt4.make_uniforms(64, 40, samples=4, reflections=4, seed=1)
    moved.focus[1] += 0.25
    others.append(rt4.accum_key(sphere, moved))
    assert all(o != k for o in others) and len(set(others)) == len(others)
    path = str(tmp_path / "k.rt4")
    rt4.accum_save(path, np.zeros((40, 64, 4), np.float32), 3, 1, key=k)
    assert rt4.accum_key_of(path) == k and rt4.accum_info(path)["frames_done"] == 3


def test_failed_save_keeps_the_previous_checkpoint(rt4, tmp_path):
    """The save writes <path>.tmp and renames it over path: when the write fails (here the .tmp name is taken
    by a directory), the previous checkpoint survives untouched and no partial file is left (ADVICE r03:
    --resume ck --checkpoint ck must never destroy the only good checkpoint)."""
    path = str(tmp_path / "ck.rt4")
    good = np.full((6, 9, 4), 0.5, np.float32)
    rt4.accum_save(path, good, 4, 77)
    before = open(path, "rb").read()
    os.mkdir(path + ".tmp")
    with pytest.raises(rt4.RT4Error, match="cannot open"):
        rt4.accum_save(path, np.zeros((6, 9, 4), np.float32), 5, 77)
    assert open(path, "rb").read() == before
    os.rmdir(path + ".tmp")
    rt4.accum_save(path, np.zeros((6, 9, 4), np.float32), 5, 77)  # and a good save replaces it
    assert rt4.accum_info(path)["frames_done"] == 5 and not os.path.exists(path + ".tmp")
