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
    assert (version, fw, fh, fmt, done, seed, res) == (1, w, h, rt4.FRAME_RGBA32F, 3, 9, 0)
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
    (tmp_path / "v.rt4").write_bytes(raw[:8] + (2).to_bytes(4, "little") + raw[12:])
    with pytest.raises(rt4.RT4Error, match="version 2"):
        rt4.accum_info(str(tmp_path / "v.rt4"))
    with pytest.raises(rt4.RT4Error, match="cannot open"):
        rt4.accum_info(str(tmp_path / "missing.rt4"))
    # bad arguments on save
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 99, 4, 4, 4, 0, 0, err, len(err)) == -1
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 0, 4, 4, 3, 0, 0, err, len(err)) == -1
    assert lib.rt4_accum_save(os.fsencode(good), ctypes.c_void_p(frame.ctypes.data), 0, 4, 4, 4, -1, 0, err, len(err)) == -1
