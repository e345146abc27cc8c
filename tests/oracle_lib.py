"""ctypes loader of the CPU oracle (oracle/build/librt4_oracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and only as
the checker / CPU baseline; the product (librt4.so) never loads it.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_int64, c_uint32, c_uint64, c_void_p

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "build", "librt4_oracle.so")
# native-math mode: glibc built-ins and unfused shader forms; a sensitivity probe, never the checker
NATIVE_PATH = os.path.join(ROOT, "oracle", "build", "librt4_oracle_native.so")


def load(path=ORACLE_PATH):
    if not os.path.exists(path):
        raise FileNotFoundError(f"oracle not built: {path} (make -C oracle)")
    lib = ctypes.CDLL(path)
    lib.oracle_hash.argtypes = [c_uint32]
    lib.oracle_hash.restype = c_uint32
    lib.oracle_scene_desc_size.restype = ctypes.c_size_t
    lib.oracle_rand_first.argtypes = [c_int32] * 6 + [c_void_p]
    lib.oracle_eval_array.argtypes = [c_int32, c_void_p, c_void_p, c_void_p, c_int64]
    lib.oracle_find_intersection.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int64]
    lib.oracle_find_intersection.restype = ctypes.c_int
    lib.oracle_rand_drct.argtypes = [c_void_p, c_void_p]
    lib.oracle_render.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, POINTER(c_uint64), c_int32,
                                  POINTER(c_uint64), c_void_p]
    lib.oracle_render.restype = ctypes.c_int
    return lib


_lib = None
_native = None


def lib(native=False):
    global _lib, _native
    if native:
        if _native is None:
            _native = load(NATIVE_PATH)
        return _native
    if _lib is None:
        _lib = load()
    return _lib


def hash_u32(x: int) -> int:
    return lib().oracle_hash(x & 0xFFFFFFFF)


def rand_first(W, H, seed, x, y, n):
    out = np.zeros(n, np.float32)
    lib().oracle_rand_first(W, H, seed, x, y, n, out.ctypes.data)
    return out


def eval_array(fn: int, x, native=False):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    aux = np.empty(x.shape, np.int32)
    lib(native).oracle_eval_array(fn, x.ctypes.data, out.ctypes.data, aux.ctypes.data, x.size)
    return out, aux


def find_intersection(scene_desc, rays):
    rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
    out = np.empty((rays.shape[0], 8), np.float32)
    col = np.empty((rays.shape[0], 3), np.float32)
    st = lib().oracle_find_intersection(ctypes.addressof(scene_desc), rays.ctypes.data, out.ctypes.data, col.ctypes.data,
                                        rays.shape[0])
    assert st == 0
    return out, col


def render(scene_desc, uniforms, reg, frame=None, threads=None, count_ops=False, pixel_counts=False, native=False):
    """Renders `reg` into frame (h, w, 4) float32 (zeros if None). Returns (frame, n_inter, ops, counts).
    native=True: the native-math build (glibc built-ins, unfused), for the sensitivity report only."""
    h, w = reg.h, reg.w
    if frame is None:
        frame = np.zeros((h, w, 4), np.float32)
    assert frame.dtype == np.float32 and frame.flags["C_CONTIGUOUS"] and frame.shape[0] >= h
    n = c_uint64()
    ops = c_uint64()
    counts = np.zeros((h, w), np.uint32) if pixel_counts else None
    threads = threads or os.cpu_count() or 1
    st = lib(native).oracle_render(ctypes.addressof(scene_desc), ctypes.addressof(uniforms), ctypes.addressof(reg),
                             frame.ctypes.data, frame.shape[1], threads, ctypes.byref(n), 1 if count_ops else 0,
                             ctypes.byref(ops), counts.ctypes.data if counts is not None else None)
    assert st == 0
    return frame, n.value, ops.value, counts


def count_ops(scene_desc, uniforms, reg, threads=None):
    """Op-counting render of `reg` (oracle_count_ops): (n_intersections, fp32 ops, ops inside the
    w_by_volume Newton loop, which the sampler-table kernel replaces by one load)."""
    lib_ = lib()
    lib_.oracle_count_ops.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int32, POINTER(c_uint64),
                                      POINTER(c_uint64), POINTER(c_uint64)]
    lib_.oracle_count_ops.restype = ctypes.c_int
    frame = np.zeros((reg.h, reg.w, 4), np.float32)
    n, ops, sops = c_uint64(), c_uint64(), c_uint64()
    st = lib_.oracle_count_ops(ctypes.addressof(scene_desc), ctypes.addressof(uniforms), ctypes.addressof(reg),
                               frame.ctypes.data, reg.w, threads or os.cpu_count() or 1, ctypes.byref(n),
                               ctypes.byref(ops), ctypes.byref(sops))
    assert st == 0
    return n.value, ops.value, sops.value


FRAME_DTYPES = {0: np.float32, 1: np.float16, 2: np.uint8}


def render_fmt(scene_desc, uniforms, reg, fmt, frame=None, threads=None):
    """oracle_render_fmt: renders `reg` into frame (h, w, 4) of the format's dtype (zeros if None).
    Returns (frame, n_inter)."""
    lib_ = lib()
    lib_.oracle_render_fmt.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int64, c_int32,
                                       POINTER(c_uint64)]
    lib_.oracle_render_fmt.restype = ctypes.c_int
    dt = FRAME_DTYPES[fmt]
    if frame is None:
        frame = np.zeros((reg.h, reg.w, 4), dt)
    assert frame.dtype == dt and frame.flags["C_CONTIGUOUS"] and frame.shape[0] >= reg.h
    n = c_uint64()
    st = lib_.oracle_render_fmt(ctypes.addressof(scene_desc), ctypes.addressof(uniforms), ctypes.addressof(reg),
                                frame.ctypes.data, fmt, frame.shape[1], threads or os.cpu_count() or 1, ctypes.byref(n))
    assert st == 0
    return frame, n.value


def float_to_half_bits(x):
    lib_ = lib()
    lib_.oracle_float_to_half.argtypes = [c_float]
    lib_.oracle_float_to_half.restype = ctypes.c_uint16
    return np.array([lib_.oracle_float_to_half(float(v)) for v in np.asarray(x, np.float32).ravel()], np.uint16)


def half_bits_to_float(h):
    lib_ = lib()
    lib_.oracle_half_to_float.argtypes = [ctypes.c_uint16]
    lib_.oracle_half_to_float.restype = c_float
    return np.array([lib_.oracle_half_to_float(int(v)) for v in np.asarray(h, np.uint16).ravel()], np.float32)
