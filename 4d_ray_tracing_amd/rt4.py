"""Python host mirror of the reference's host interface, over the C ABI of librt4.so (include/rt4.h).

The reference's host is C++ on SFML; this module gives the same operations to Python callers
(tests, bench.py) without re-implementing any of them: every call goes into librt4.so.

  Properties            <- Properties (inc/properties.h:8-18, src/properties.cpp:12-77)
  Orientation.update    <- Orientation::update (src/controls.cpp:72-86)
  uniforms_from_properties <- initShader/initControls/drawShaderImage uniform producers
                           (src/main.cpp:25-39,86-91, src/controls.cpp:140-159, src/windows/windows.cpp:41-44)
  Scene.load_frag/parse <- pasting scenes/<name>.frag into executable/shader.frag (executable/README.md:9-11)
  Tracer.render_*       <- CellsWindow::drawShaderImage -> texture.draw(sprite, &shader) (windows.cpp:40-47)

There is no fallback: if librt4.so is missing or fails to load, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os
import sys
from ctypes import POINTER, Structure, byref, c_char_p, c_float, c_int, c_int32, c_int64, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RT4_LIB", os.path.join(_HERE, "lib", "librt4.so"))

F4 = c_float * 4
F3 = c_float * 3
F2 = c_float * 2


class Material(Structure):  # shader.frag:163-167
    _fields_ = [("glow", c_float), ("refl_prob", c_float), ("color", F3)]


class Space(Structure):  # visible_space, shader.frag:225-228
    _fields_ = [("point", F4), ("norm", F4), ("material", Material)]


class Sphere(Structure):  # visible_sphere, shader.frag:189-192
    _fields_ = [("center", F4), ("r", c_float), ("material", Material)]


class Cylinder(Structure):  # visible_cylinder, shader.frag:243-247
    _fields_ = [("point", F4), ("axis1", F4), ("axis2", F4), ("r", c_float), ("material", Material)]


class CylindersUnion(Structure):  # shader.frag:279-281
    _fields_ = [("cylinder1", Cylinder), ("cylinder2", Cylinder)]


class Tiger(Structure):  # shader.frag:298-300
    _fields_ = [("inner_cyl1", Cylinder), ("outer_cyl1", Cylinder), ("inner_cyl2", Cylinder), ("outer_cyl2", Cylinder)]


class Cube(Structure):  # visible_cube, shader.frag:345-350
    _fields_ = [("point", F4), ("norm", F4), ("x", F4), ("y", F4), ("z", F4), ("r", c_float), ("material", Material)]


class Hypercube(Structure):  # shader.frag:370-372
    _fields_ = [("cubes", Cube * 8)]


class Sun(Structure):  # sun_properties, shader.frag:404-409
    _fields_ = [("drct", F4), ("angular_size", c_float), ("light", F3), ("sharpness", c_float)]


class Group(Structure):
    _fields_ = [("kind", c_int32), ("first", c_int32), ("count", c_int32), ("outer", c_int32), ("new_first", c_int32)]


MAX_GROUPS, MAX_SPACES, MAX_SPHERES, MAX_CYLINDERS = 16, 32, 32, 16
MAX_UNIONS, MAX_HYPERCUBES, MAX_TIGERS = 4, 4, 4

GROUP_SPACES, GROUP_SPHERES, GROUP_CYLINDERS, GROUP_CYLINDERS_UNION, GROUP_HYPERCUBE, GROUP_TIGER = 1, 2, 3, 4, 5, 6
FINAL_LIGHT_SUN_SKY, FINAL_LIGHT_CONSTANT = 0, 1
SECTION_YXZ, SECTION_YWZ, SECTION_YXW = 0, 1, 2
FLAG_SAMPLER_LUT = 0x1
FLAG_GENERIC_KERNEL = 0x2
FLAG_PRIMARY_REUSE = 0x4
FLAG_SERIAL_FRAMES = 0x8
FLAG_OVERLAP_SHALLOW = 0x10  # rt4.h RT4_FLAG_OVERLAP_SHALLOW: at most 3 overlapped launches in flight
FRAME_RGBA32F, FRAME_RGBA16F, FRAME_RGBA8 = 0, 1, 2
KEY_FORWARD, KEY_BACK, KEY_RIGHT, KEY_LEFT, KEY_UP, KEY_DOWN, KEY_W_POS, KEY_W_NEG = (1 << i for i in range(8))
MAX_SECTIONS = 3
EVAL_ACOS, EVAL_ASIN, EVAL_SIN, EVAL_COS, EVAL_VOLUME_BY_W, EVAL_W_BY_VOLUME, EVAL_HASH, EVAL_SQRT = range(8)


class SceneDesc(Structure):
    _fields_ = [
        ("sky_light", F3),
        ("sun", Sun),
        ("final_light_mode", c_int32),
        ("final_light_const", F3),
        ("n_groups", c_int32),
        ("groups", Group * MAX_GROUPS),
        ("n_spaces", c_int32),
        ("spaces", Space * MAX_SPACES),
        ("n_spheres", c_int32),
        ("spheres", Sphere * MAX_SPHERES),
        ("n_cylinders", c_int32),
        ("cylinders", Cylinder * MAX_CYLINDERS),
        ("n_unions", c_int32),
        ("unions", CylindersUnion * MAX_UNIONS),
        ("n_hypercubes", c_int32),
        ("hypercubes", Hypercube * MAX_HYPERCUBES),
        ("n_tigers", c_int32),
        ("tigers", Tiger * MAX_TIGERS),
    ]


class Uniforms(Structure):  # shader.frag:5-19
    _fields_ = [
        ("seed", c_int32),
        ("samples", c_int32),
        ("reflections_amount", c_int32),
        ("small_indent", c_float),
        ("resolution", F2),
        ("part", c_float),
        ("light_to_color_conversion_coefficient", c_float),
        ("mtr_sizes", F2),
        ("focus", F4),
        ("vec_to_mtr", F4),
        ("top_drct", F4),
        ("right_drct", F4),
    ]


class OrientationStruct(Structure):  # struct Orientation, inc/controls.h:9-14
    _fields_ = [(n, F4) for n in ("forward", "top", "right", "w_drct", "horizontal_forward", "horizontal_right", "vertical_top")]


class CameraStruct(Structure):  # rt4.h rt4_camera (SphOrientation + controls.cpp state)
    _fields_ = [("fi", c_float), ("te", c_float), ("psi", c_float), ("psi_range_center", c_float),
                ("psi_range_radius", c_float), ("constrain_psi_range", c_int32), ("mouse_sensitivity", c_float),
                ("wheel_sensitivity", c_float), ("movement_speed", c_float), ("focus_to_matrix_distance", c_float),
                ("focus", F4), ("frame_number", c_uint32), ("orientation", OrientationStruct)]


class Region(Structure):
    _fields_ = [("x0", c_int32), ("y0", c_int32), ("w", c_int32), ("h", c_int32), ("band_rows", c_int32), ("band_step", c_int32)]


class SectionJob(Structure):  # rt4.h rt4_section_job
    _fields_ = [("u", Uniforms), ("region", Region), ("d_frame", c_void_p), ("row_stride_px", c_int64)]


def _load(path=None):
    path = path or LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"librt4.so not found at {path}: build it first (python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    E = [c_char_p, c_size_t]  # err, errlen
    sig = {
        "rt4_abi_version": ([], c_int),
        "rt4_build_info": ([], c_char_p),
        "rt4_scene_desc_size": ([], c_size_t),
        "rt4_uniforms_size": ([], c_size_t),
        "rt4_properties_load": ([c_char_p, POINTER(c_void_p)] + E, c_int),
        "rt4_properties_parse": ([c_char_p, c_size_t, POINTER(c_void_p)] + E, c_int),
        "rt4_properties_free": ([c_void_p], None),
        "rt4_properties_has": ([c_void_p, c_char_p], c_int),
        "rt4_properties_get_string": ([c_void_p, c_char_p, c_char_p, c_size_t, POINTER(c_size_t)] + E, c_int),
        "rt4_properties_get_int": ([c_void_p, c_char_p, POINTER(c_int32)] + E, c_int),
        "rt4_properties_get_uint": ([c_void_p, c_char_p, POINTER(c_uint32)] + E, c_int),
        "rt4_properties_get_float": ([c_void_p, c_char_p, POINTER(c_float)] + E, c_int),
        "rt4_properties_get_bool": ([c_void_p, c_char_p, POINTER(c_int)] + E, c_int),
        "rt4_orientation_update": ([c_float, c_float, c_float, POINTER(OrientationStruct)], None),
        "rt4_section_basis": ([POINTER(OrientationStruct), c_int, POINTER(c_float), POINTER(c_float)], c_int),
        "rt4_uniforms_from_properties": ([c_void_p, c_int32, c_int32, c_int, POINTER(Uniforms), POINTER(OrientationStruct)] + E, c_int),
        "rt4_window_cells": ([c_void_p, c_char_p, POINTER(c_int32), POINTER(c_int32)] + E, c_int),
        "rt4_scene_load_frag": ([c_char_p, POINTER(SceneDesc)] + E, c_int),
        "rt4_scene_parse_frag": ([c_char_p, c_size_t, POINTER(SceneDesc)] + E, c_int),
        "rt4_scene_validate": ([POINTER(SceneDesc)] + E, c_int),
        "rt4_scene_builtin": ([c_char_p, POINTER(SceneDesc)] + E, c_int),
        "rt4_context_create": ([c_int, c_uint32, POINTER(c_void_p)] + E, c_int),
        "rt4_context_set_scene": ([c_void_p, POINTER(SceneDesc)] + E, c_int),
        "rt4_context_destroy": ([c_void_p], None),
        "rt4_render_device": ([c_void_p, POINTER(Uniforms), POINTER(Region), c_void_p, c_int64, c_void_p, c_void_p] + E, c_int),
        "rt4_render_host": ([c_void_p, POINTER(Uniforms), POINTER(Region), c_void_p, c_int64, POINTER(c_uint64)] + E, c_int),
        "rt4_debug_eval": ([c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64] + E, c_int),
        "rt4_debug_find_intersection": ([c_void_p, c_void_p, c_void_p, c_void_p, c_int64] + E, c_int),
        "rt4_context_kernel_shape": ([c_void_p], c_uint32),
        "rt4_debug_verify_sqrt": ([c_void_p, POINTER(c_uint64)] + E, c_int),
        "rt4_frame_format_bytes": ([c_int32], c_int32),
        "rt4_camera_init": ([c_void_p, POINTER(CameraStruct)] + E, c_int),
        "rt4_camera_rotate": ([POINTER(CameraStruct), c_float, c_float, c_float], None),
        "rt4_camera_mouse_move": ([POINTER(CameraStruct), c_int32, c_int32, c_uint32], c_int),
        "rt4_camera_wheel": ([POINTER(CameraStruct), c_float], None),
        "rt4_camera_move": ([POINTER(CameraStruct), c_uint32, c_float], None),
        "rt4_camera_frame_uniforms": ([POINTER(CameraStruct), POINTER(Uniforms), c_int, c_int32, POINTER(Uniforms)], c_int),
        "rt4_write_ppm": ([c_char_p, c_void_p, c_int32, c_int32, c_int32, c_int64] + E, c_int),
        "rt4_write_png": ([c_char_p, c_void_p, c_int32, c_int32, c_int32, c_int64] + E, c_int),
        "rt4_render_device_ex": ([c_void_p, POINTER(Uniforms), POINTER(Region), c_void_p, c_int32, c_int64, c_void_p,
                                  c_void_p] + E, c_int),
        "rt4_render_host_ex": ([c_void_p, POINTER(Uniforms), POINTER(Region), c_void_p, c_int32, c_int64,
                                POINTER(c_uint64)] + E, c_int),
        "rt4_progressive_uniforms": ([POINTER(Uniforms), c_uint32, POINTER(Uniforms)], c_int),
        "rt4_render_sections_device": ([c_void_p, POINTER(SectionJob), c_int32, c_int32, c_void_p, c_void_p] + E, c_int),
        "rt4_render_frames_device": ([c_void_p, POINTER(Uniforms), c_int32, POINTER(Region), c_void_p, c_int32, c_int64,
                                      c_void_p, c_void_p] + E, c_int),
        "rt4_context_reserve_frames": ([c_void_p, c_int32, c_int32] + E, c_int),
        "rt4_context_frames_per_launch": ([c_void_p, c_int32, c_int32], c_int32),
        "rt4_debug_verify_div": ([c_void_p, c_float, c_int32, POINTER(c_uint64)] + E, c_int),
        "rt4_context_evaluated": ([c_void_p, POINTER(c_uint64), c_int32] + E, c_int),
        "rt4_debug_sky_threshold": ([c_void_p, c_float, c_int32, POINTER(c_float)] + E, c_int),
        "rt4_band_plan": ([c_int32, c_int32, c_int32, c_int32, c_int32, POINTER(Region), POINTER(c_int32)] + E, c_int),
        "rt4_bands_unpermute_device": ([c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                        c_void_p] + E, c_int),
        "rt4_context_frame_scratch_bytes": ([c_void_p], c_uint64),
        "rt4_context_overlap_bytes": ([c_void_p], c_uint64),
        "rt4_context_reserve_overlap": ([c_void_p, c_int32, c_int32] + E, c_int),
        "rt4_accum_save": ([c_char_p, c_void_p, c_int32, c_int32, c_int32, c_int64, c_int64, c_uint32] + E, c_int),
        "rt4_accum_info": ([c_char_p, POINTER(c_int32), POINTER(c_int32), POINTER(c_int32), POINTER(c_int64),
                            POINTER(c_uint32)] + E, c_int),
        "rt4_accum_load": ([c_char_p, c_void_p, c_int32, c_int32, c_int32, c_int64, POINTER(c_int64), POINTER(c_uint32)]
                           + E, c_int),
        "rt4_accum_save_key": ([c_char_p, c_void_p, c_int32, c_int32, c_int32, c_int64, c_int64, c_uint32, c_uint32] + E,
                               c_int),
        "rt4_accum_key": ([c_void_p, c_void_p], c_uint32),
        "rt4_accum_key_of": ([c_char_p, POINTER(c_uint32)] + E, c_int),
    }
    tolerant = os.environ.get("RT4_AB_TOLERANT") == "1"  # tools/abtest.sh: older builds lack newer exports
    for name, (argtypes, restype) in sig.items():
        if tolerant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)  # AttributeError if the library lacks a declared export
        fn.argtypes = argtypes
        fn.restype = restype
    return lib


lib = _load()


def load_variant(path: str):
    """Another build of librt4.so (e.g. the native-math diagnostic build, lib_native/librt4.so) with the
    same C ABI, for Tracer(library=...): two builds side by side in one process."""
    return _load(path)
EXPORTED = (
    "rt4_abi_version rt4_build_info rt4_scene_desc_size rt4_uniforms_size rt4_properties_load rt4_properties_parse "
    "rt4_properties_free rt4_properties_has rt4_properties_get_string rt4_properties_get_int rt4_properties_get_uint "
    "rt4_properties_get_float rt4_properties_get_bool rt4_orientation_update rt4_section_basis "
    "rt4_uniforms_from_properties rt4_window_cells rt4_scene_load_frag rt4_scene_parse_frag rt4_scene_validate "
    "rt4_scene_builtin rt4_context_create rt4_context_set_scene rt4_context_destroy rt4_render_device rt4_render_host "
    "rt4_debug_eval rt4_debug_find_intersection rt4_context_kernel_shape rt4_debug_verify_sqrt "
    "rt4_camera_init rt4_camera_rotate rt4_camera_mouse_move rt4_camera_wheel rt4_camera_move "
    "rt4_camera_frame_uniforms rt4_write_ppm rt4_frame_format_bytes rt4_render_device_ex rt4_render_host_ex rt4_progressive_uniforms rt4_render_sections_device "
    "rt4_debug_verify_div rt4_debug_sky_threshold rt4_context_evaluated rt4_render_frames_device rt4_context_reserve_frames rt4_context_frames_per_launch "
    "rt4_band_plan rt4_bands_unpermute_device rt4_context_frame_scratch_bytes rt4_context_overlap_bytes rt4_context_reserve_overlap rt4_accum_save rt4_accum_info rt4_accum_load rt4_write_png "
    "rt4_accum_save_key rt4_accum_key rt4_accum_key_of"
).split()

if ctypes.sizeof(SceneDesc) != lib.rt4_scene_desc_size() or ctypes.sizeof(Uniforms) != lib.rt4_uniforms_size():
    raise ImportError("rt4.py struct layout does not match librt4.so (rebuild the library)")


class RT4Error(RuntimeError):
    """A non-zero status from librt4.so (the reference aborts on these: src/util/util.cpp:9-12)."""

    def __init__(self, status: int, msg: str):
        super().__init__(f"rt4 status {status}: {msg}")
        self.status = status


def _errbuf():
    return ctypes.create_string_buffer(1024)


def _check(status: int, err) -> None:
    if status != 0:
        raise RT4Error(status, err.value.decode("utf-8", "replace"))


class Properties:
    """properties.txt reader with the reference's getters (inc/properties.h:8-18)."""

    def __init__(self, path: str | None = None, text: str | None = None):
        h = c_void_p()
        err = _errbuf()
        if text is not None:
            raw = text.encode("utf-8")
            _check(lib.rt4_properties_parse(raw, len(raw), byref(h), err, len(err)), err)
        else:
            _check(lib.rt4_properties_load(os.fsencode(path), byref(h), err, len(err)), err)
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib.rt4_properties_free(self._h)
            self._h = None

    def has(self, key: str) -> bool:
        return bool(lib.rt4_properties_has(self._h, key.encode()))

    def getString(self, key: str) -> str:
        need = c_size_t()
        err = _errbuf()
        _check(lib.rt4_properties_get_string(self._h, key.encode(), None, 0, byref(need), err, len(err)), err)
        buf = ctypes.create_string_buffer(need.value + 1)
        _check(lib.rt4_properties_get_string(self._h, key.encode(), buf, len(buf), None, err, len(err)), err)
        return buf.value.decode("utf-8")

    def getStringOrNull(self, key: str) -> str:  # properties.cpp:31-33 (map[key] -> "" when absent)
        return self.getString(key) if self.has(key) else ""

    def _get(self, fn, ctype, key):
        v = ctype()
        err = _errbuf()
        _check(fn(self._h, key.encode(), byref(v), err, len(err)), err)
        return v.value

    def getInt(self, key: str) -> int:
        return self._get(lib.rt4_properties_get_int, c_int32, key)

    def getUnsignedInt(self, key: str) -> int:
        return self._get(lib.rt4_properties_get_uint, c_uint32, key)

    def getFloat(self, key: str) -> float:
        return self._get(lib.rt4_properties_get_float, c_float, key)

    def getBool(self, key: str) -> bool:
        return bool(self._get(lib.rt4_properties_get_bool, c_int, key))


class Orientation:
    """Camera basis from (fi, te, psi) in radians (src/controls.cpp:72-86)."""

    def __init__(self, fi: float = 0.0, te: float = 0.0, psi: float = 0.0):
        self.s = OrientationStruct()
        lib.rt4_orientation_update(fi, te, psi, byref(self.s))

    def __getattr__(self, name):
        return list(getattr(self.s, name))

    def section_basis(self, section: int):
        top, right = F4(), F4()
        if lib.rt4_section_basis(byref(self.s), section, top, right) != 0:
            raise RT4Error(-1, f"bad section {section}")
        return list(top), list(right)


def uniforms_from_properties(props: Properties, cells_w: int, cells_h: int, section: int = SECTION_YXZ):
    u = Uniforms()
    o = OrientationStruct()
    err = _errbuf()
    _check(lib.rt4_uniforms_from_properties(props._h, cells_w, cells_h, section, byref(u), byref(o), err, len(err)), err)
    return u


def window_cells(props: Properties, window_type: str = "main"):
    w, h = c_int32(), c_int32()
    err = _errbuf()
    _check(lib.rt4_window_cells(props._h, window_type.encode(), byref(w), byref(h), err, len(err)), err)
    return w.value, h.value


def make_uniforms(width: int, height: int, samples: int, reflections: int, seed: int = 12345, *, small_indent=0.005,
                  k=1.0, matrix_height=2.0, focus_to_matrix=1.5, focus=(0.0, -2.0, 0.0, 0.0), part=1.0,
                  fi=0.0, te=0.0, psi=0.0, section=SECTION_YXZ):
    """Uniforms of the default camera built through the library's own producers."""
    text = (
        f"ray_tracing.samples = {samples}\nray_tracing.reflections_amount = {reflections}\n"
        f"ray_tracing.small_indent = {small_indent!r}\nlight_to_color_conversion_coefficient = {k!r}\n"
        f"camera.matrix_height = {matrix_height!r}\ncamera.focus_to_matrix_distance = {focus_to_matrix!r}\n"
        f"camera.initial_position.x = {focus[0]!r}\ncamera.initial_position.y = {focus[1]!r}\n"
        f"camera.initial_position.z = {focus[2]!r}\ncamera.initial_position.w = {focus[3]!r}\n"
        f"camera.initial_position.fi = {fi!r}\ncamera.initial_position.te = {te!r}\n"
        f"camera.initial_position.psi = {psi!r}\nconstrain_psi_range = false\n"
    )
    u = uniforms_from_properties(Properties(text=text), width, height, section)
    u.seed = ctypes.c_int32(seed & 0xFFFFFFFF if seed >= 0 else seed).value
    u.part = part
    return u


BUILTIN_SCENES = ("sphere", "room", "tiger", "cylinder4d", "hypercube")
SCENES_DIR = os.path.join(os.path.dirname(_HERE), "scenes")


class Scene:
    """A parsed scene (rt4_scene_desc)."""

    def __init__(self, desc: SceneDesc):
        self.desc = desc

    @classmethod
    def builtin(cls, name: str) -> "Scene":
        d = SceneDesc()
        err = _errbuf()
        _check(lib.rt4_scene_builtin(name.encode(), byref(d), err, len(err)), err)
        return cls(d)

    @classmethod
    def load_frag(cls, path: str) -> "Scene":
        d = SceneDesc()
        err = _errbuf()
        _check(lib.rt4_scene_load_frag(os.fsencode(path), byref(d), err, len(err)), err)
        return cls(d)

    @classmethod
    def parse(cls, text: str) -> "Scene":
        d = SceneDesc()
        err = _errbuf()
        raw = text.encode("utf-8")
        _check(lib.rt4_scene_parse_frag(raw, len(raw), byref(d), err, len(err)), err)
        return cls(d)

    @classmethod
    def named(cls, name: str) -> "Scene":
        """A builtin reference scene, or scenes/<name>.frag of this repository, or a path to a .frag file."""
        if name in BUILTIN_SCENES:
            return cls.builtin(name)
        path = name if name.endswith(".frag") else os.path.join(SCENES_DIR, name + ".frag")
        return cls.load_frag(path)

    def to_bytes(self) -> bytes:
        return bytes(self.desc)

    def groups(self):
        return [(g.kind, g.first, g.count, g.outer, g.new_first) for g in self.desc.groups[: self.desc.n_groups]]


def region(w: int, h: int, x0: int = 0, y0: int = 0, band_rows: int = 0, band_step: int = 0) -> Region:
    return Region(x0, y0, w, h, band_rows, band_step)


def band_plan(width: int, height: int, world: int, rank: int, band: int = 8):
    """(region of `rank`, rows_max) of the C ABI's pixel-band plan (rt4_band_plan; shard.py make_plan)."""
    reg, rows_max = Region(), c_int32()
    err = _errbuf()
    _check(lib.rt4_band_plan(width, height, world, band, rank, byref(reg), byref(rows_max), err, len(err)), err)
    return reg, rows_max.value


def bands_unpermute_device(gathered_ptr: int, image_ptr: int, width: int, height: int, world: int, rows_max: int,
                           fmt: int = FRAME_RGBA32F, band: int = 8, stream: int = 0) -> None:
    """The frame from world x rows_max gathered shard rows on the device (rt4_bands_unpermute_device)."""
    err = _errbuf()
    _check(lib.rt4_bands_unpermute_device(c_void_p(gathered_ptr), c_void_p(image_ptr), width, height, world, band,
                                          rows_max, fmt, c_void_p(stream), err, len(err)), err)


class Camera:
    """The reference's camera controller (src/controls.cpp) over rt4_camera: mouse/wheel rotation,
    WASD/Space/Shift/E/Q motion and per-frame uniforms (main.cpp:86-91)."""

    def __init__(self, props: "Properties"):
        self.s = CameraStruct()
        err = _errbuf()
        _check(lib.rt4_camera_init(props._h, byref(self.s), err, len(err)), err)

    def rotate(self, d_fi=0.0, d_te=0.0, d_psi=0.0):
        lib.rt4_camera_rotate(byref(self.s), d_fi, d_te, d_psi)

    def mouse_move(self, dx: int, dy: int, max_offset: int) -> bool:
        """True when the move only re-centres the cursor (out of the allowed offset)."""
        return bool(lib.rt4_camera_mouse_move(byref(self.s), dx, dy, max_offset))

    def wheel(self, delta: float):
        lib.rt4_camera_wheel(byref(self.s), delta)

    def move(self, keys: int, seconds: float):
        lib.rt4_camera_move(byref(self.s), keys, seconds)

    def frame_uniforms(self, base: Uniforms, section: int = SECTION_YXZ, seed: int = 0) -> Uniforms:
        out = Uniforms()
        seed = ctypes.c_int32(seed & 0xFFFFFFFF).value
        if lib.rt4_camera_frame_uniforms(byref(self.s), byref(base), section, seed, byref(out)) != 0:
            raise RT4Error(-1, "rt4_camera_frame_uniforms failed")
        return out


def write_ppm(path: str, frame, fmt: int | None = None) -> None:
    """Binary PPM of an (h, w, 4) frame (float32 / float16 / uint8), rows top first (rt4_write_ppm)."""
    import numpy as np

    frame = np.ascontiguousarray(frame)
    if fmt is None:
        fmt = {np.dtype("float32"): FRAME_RGBA32F, np.dtype("float16"): FRAME_RGBA16F,
               np.dtype("uint8"): FRAME_RGBA8}[frame.dtype]
    h, w = frame.shape[:2]
    err = _errbuf()
    _check(lib.rt4_write_ppm(os.fsencode(path), c_void_p(frame.ctypes.data), fmt, w, h, w, err, len(err)), err)


def accum_save(path: str, frame, frames_done: int, seed: int, fmt: int | None = None, key: int = 0) -> None:
    """Checkpoint of a progressive accumulator (rt4_accum_save_key): the (h, w, 4) host frame and the number of
    frames already blended into it, with the base seed of its rt4_progressive_uniforms and the run's key
    (accum_key; 0 = not recorded). Written to path + ".tmp" and renamed over path."""
    import numpy as np

    frame = np.ascontiguousarray(frame)
    if fmt is None:
        fmt = {np.dtype("float32"): FRAME_RGBA32F, np.dtype("float16"): FRAME_RGBA16F,
               np.dtype("uint8"): FRAME_RGBA8}[frame.dtype]
    h, w = frame.shape[:2]
    err = _errbuf()
    _check(lib.rt4_accum_save_key(os.fsencode(path), c_void_p(frame.ctypes.data), fmt, w, h, w, frames_done,
                                  seed & 0xFFFFFFFF, key & 0xFFFFFFFF, err, len(err)), err)


def accum_key(scene, u) -> int:
    """The run key a checkpoint records (rt4_accum_key): scene + image-deciding uniforms, not seed or part."""
    return lib.rt4_accum_key(byref(scene.desc if hasattr(scene, "desc") else scene), byref(u))


def accum_key_of(path: str) -> int:
    """The key a checkpoint was saved with (0: not recorded)."""
    k = c_uint32()
    err = _errbuf()
    _check(lib.rt4_accum_key_of(os.fsencode(path), byref(k), err, len(err)), err)
    return k.value


def accum_info(path: str) -> dict:
    """The checkpoint's header (rt4_accum_info): w, h, format, frames_done, seed."""
    w, h, f, n, sd = c_int32(), c_int32(), c_int32(), c_int64(), c_uint32()
    err = _errbuf()
    _check(lib.rt4_accum_info(os.fsencode(path), byref(w), byref(h), byref(f), byref(n), byref(sd), err, len(err)), err)
    return {"w": w.value, "h": h.value, "format": f.value, "frames_done": n.value, "seed": sd.value}


def accum_load(path: str):
    """(frame, frames_done, seed) from a checkpoint (rt4_accum_load); frame is an (h, w, 4) numpy array of the
    checkpoint's format."""
    import numpy as np

    info = accum_info(path)
    frame = np.empty((info["h"], info["w"], 4), dtype=FRAME_NUMPY[info["format"]])
    n, sd = c_int64(), c_uint32()
    err = _errbuf()
    _check(lib.rt4_accum_load(os.fsencode(path), c_void_p(frame.ctypes.data), info["format"], info["w"], info["h"],
                              info["w"], byref(n), byref(sd), err, len(err)), err)
    return frame, n.value, sd.value


def write_png(path: str, frame, fmt: int | None = None) -> None:
    """8-bit RGB PNG of an (h, w, 4) frame, the same pixels as write_ppm (rt4_write_png)."""
    import numpy as np

    frame = np.ascontiguousarray(frame)
    if fmt is None:
        fmt = {np.dtype("float32"): FRAME_RGBA32F, np.dtype("float16"): FRAME_RGBA16F,
               np.dtype("uint8"): FRAME_RGBA8}[frame.dtype]
    h, w = frame.shape[:2]
    err = _errbuf()
    _check(lib.rt4_write_png(os.fsencode(path), c_void_p(frame.ctypes.data), fmt, w, h, w, err, len(err)), err)


def frame_format_bytes(fmt: int) -> int:
    return lib.rt4_frame_format_bytes(fmt)


FRAME_NUMPY = {FRAME_RGBA32F: "float32", FRAME_RGBA16F: "float16", FRAME_RGBA8: "uint8"}


def progressive_uniforms(base: Uniforms, frame_number: int) -> Uniforms:
    """Uniforms of progressive frame n >= 1: part = 1/n, seed_n = seed ^ n*0x9E3779B9 (rt4.h)."""
    out = Uniforms()
    if lib.rt4_progressive_uniforms(byref(base), frame_number, byref(out)) != 0:
        raise RT4Error(-1, f"bad progressive frame number {frame_number}")
    return out


class Tracer:
    """Device context: scene on the device (+ optional sampler table) and the trace kernel."""

    def __init__(self, device: int = 0, flags: int = 0, scene: Scene | None = None, library=None):
        self._lib = library or lib  # library: load_variant(...) of another build (diagnostics)
        # librt4.so links the system HIP runtime; PyTorch-ROCm brings its own copy. In one process the
        # torch runtime must initialise first (torch.cuda reports no GPU when it comes second).
        torch = sys.modules.get("torch")
        if torch is not None and hasattr(torch, "cuda") and not torch.cuda.is_initialized():
            try:
                torch.cuda.init()
            except Exception:  # no GPU for torch: librt4.so reports its own error below
                pass
        h = c_void_p()
        err = _errbuf()
        _check(self._lib.rt4_context_create(device, flags, byref(h), err, len(err)), err)
        self._h = h
        self.device = device
        if scene is not None:
            self.set_scene(scene)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.rt4_context_destroy(self._h)
            self._h = None

    __del__ = close

    def set_scene(self, scene: Scene) -> None:
        err = _errbuf()
        _check(self._lib.rt4_context_set_scene(self._h, byref(scene.desc), err, len(err)), err)

    def render_device(self, u: Uniforms, reg: Region, frame_ptr: int, row_stride_px: int, counter_ptr: int = 0,
                      stream: int = 0) -> None:
        """Asynchronous launch on `stream` into a device float4 framebuffer (e.g. a torch tensor's data_ptr())."""
        err = _errbuf()
        _check(self._lib.rt4_render_device(self._h, byref(u), byref(reg), c_void_p(frame_ptr), row_stride_px,
                                     c_void_p(counter_ptr or None), c_void_p(stream or None), err, len(err)), err)

    def render_device_ex(self, u: Uniforms, reg: Region, frame_ptr: int, fmt: int, row_stride_px: int,
                         counter_ptr: int = 0, stream: int = 0) -> None:
        """render_device into a device frame of any rt4_frame_format."""
        err = _errbuf()
        _check(self._lib.rt4_render_device_ex(self._h, byref(u), byref(reg), c_void_p(frame_ptr), fmt, row_stride_px,
                                        c_void_p(counter_ptr or None), c_void_p(stream or None), err, len(err)), err)

    def render_frames_device(self, us, reg: Region, frame_ptr: int, fmt: int, row_stride_px: int,
                             counter_ptr: int = 0, stream: int = 0) -> None:
        """len(us) consecutive frames into one device frame, pipelined (rt4_render_frames_device): the same
        result as render_device_ex(us[0]), render_device_ex(us[1]), ... in order."""
        arr = (Uniforms * len(us))(*us)
        err = _errbuf()
        _check(self._lib.rt4_render_frames_device(self._h, arr, len(us), byref(reg), c_void_p(frame_ptr), fmt, row_stride_px,
                                            c_void_p(counter_ptr or None), c_void_p(stream or None), err, len(err)), err)

    def frames_per_launch(self, w: int, h: int) -> int:
        """Frames per pipelined launch for a w x h region with the current scene (1: frame by frame)."""
        return int(self._lib.rt4_context_frames_per_launch(self._h, w, h))

    def reserve_frames(self, w: int, h: int) -> None:
        """Allocate the frame-colour scratch of pipelined launches of a w x h region up front."""
        err = _errbuf()
        _check(self._lib.rt4_context_reserve_frames(self._h, w, h, err, len(err)), err)

    def frame_scratch_bytes(self) -> int:
        """Bytes of the context's frame-colour scratch (0: none allocated)."""
        return int(self._lib.rt4_context_frame_scratch_bytes(self._h))

    def overlap_bytes(self) -> int:
        """Bytes of the context's overlap slot buffers (rt4.h rt4_context_overlap_bytes)."""
        return int(self._lib.rt4_context_overlap_bytes(self._h))

    def reserve_overlap(self, w: int, h: int) -> None:
        """Allocate the slot buffers overlapped single-frame launches of a w x h image use, up front."""
        err = _errbuf()
        _check(self._lib.rt4_context_reserve_overlap(self._h, w, h, err, len(err)), err)

    def render_sections_device(self, jobs, fmt: int = FRAME_RGBA32F, counter_ptr: int = 0, stream: int = 0) -> None:
        """One launch over up to three images: jobs = [(uniforms, region, frame_ptr, row_stride_px), ...]."""
        arr = (SectionJob * len(jobs))()
        for q, (u, reg, ptr, stride) in enumerate(jobs):
            arr[q].u = u
            arr[q].region = reg
            arr[q].d_frame = ptr
            arr[q].row_stride_px = stride
        err = _errbuf()
        _check(self._lib.rt4_render_sections_device(self._h, arr, len(jobs), fmt, c_void_p(counter_ptr or None),
                                              c_void_p(stream or None), err, len(err)), err)

    def render_host_ex(self, u: Uniforms, reg: Region, frame, fmt: int, row_stride_px: int | None = None) -> int:
        """Synchronous render into a host array (h, stride, 4) of the format's dtype (FRAME_NUMPY)."""
        import numpy as np

        assert frame.dtype == np.dtype(FRAME_NUMPY[fmt]) and frame.flags["C_CONTIGUOUS"]
        stride = row_stride_px if row_stride_px is not None else frame.shape[1]
        n = c_uint64()
        err = _errbuf()
        _check(self._lib.rt4_render_host_ex(self._h, byref(u), byref(reg), c_void_p(frame.ctypes.data), fmt, stride,
                                      byref(n), err, len(err)), err)
        return n.value

    def render_host(self, u: Uniforms, reg: Region, frame, row_stride_px: int | None = None) -> int:
        """Synchronous render into a host float32 array of shape (h, stride, 4); returns the intersection count."""
        import numpy as np

        assert frame.dtype == np.float32 and frame.flags["C_CONTIGUOUS"]
        stride = row_stride_px if row_stride_px is not None else frame.shape[1]
        n = c_uint64()
        err = _errbuf()
        _check(self._lib.rt4_render_host(self._h, byref(u), byref(reg), c_void_p(frame.ctypes.data), stride, byref(n), err,
                                   len(err)), err)
        return n.value

    @property
    def kernel_shape(self) -> int:
        """Shape code of the trace kernel the scene runs on (rt4.h rt4_context_kernel_shape)."""
        return self._lib.rt4_context_kernel_shape(self._h)

    def debug_eval(self, fn: int, x):
        import numpy as np

        x = np.ascontiguousarray(x, dtype=np.float32)
        out = np.empty_like(x)
        aux = np.empty(x.shape, np.int32)
        err = _errbuf()
        _check(self._lib.rt4_debug_eval(self._h, fn, c_void_p(x.ctypes.data), c_void_p(out.ctypes.data),
                                  c_void_p(aux.ctypes.data), x.size, err, len(err)), err)
        return out, aux

    def debug_verify_sqrt(self) -> int:
        """Mismatches of the kernel's sqrt against IEEE sqrt over all 2^32 inputs (rt4.h)."""
        n = c_uint64(0)
        err = _errbuf()
        _check(self._lib.rt4_debug_verify_sqrt(self._h, ctypes.byref(n), err, len(err)), err)
        return n.value

    def evaluated(self, reset: bool = True) -> int:
        """find_intersection calls evaluated by RT4_FLAG_PRIMARY_REUSE launches since the last reset."""
        n = c_uint64(0)
        err = _errbuf()
        _check(self._lib.rt4_context_evaluated(self._h, ctypes.byref(n), 1 if reset else 0, err, len(err)), err)
        return n.value

    def debug_verify_div(self, b: float, full: bool = False) -> int:
        """Mismatches of the verified-divisor quotient x / b (reduced sweep, or all 2^32 numerators)."""
        n = c_uint64(0)
        err = _errbuf()
        _check(self._lib.rt4_debug_verify_div(self._h, b, 1 if full else 0, ctypes.byref(n), err, len(err)), err)
        return n.value

    def debug_sky_threshold(self, ang: float, full: bool = False) -> float:
        """Smallest float c with acos(c) < ang in the kernel's acos (NaN: none)."""
        c = c_float(0.0)
        err = _errbuf()
        _check(self._lib.rt4_debug_sky_threshold(self._h, ang, 1 if full else 0, ctypes.byref(c), err, len(err)), err)
        return c.value

    def debug_find_intersection(self, rays):
        import numpy as np

        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        out = np.empty((rays.shape[0], 8), np.float32)
        col = np.empty((rays.shape[0], 3), np.float32)
        err = _errbuf()
        _check(self._lib.rt4_debug_find_intersection(self._h, c_void_p(rays.ctypes.data), c_void_p(out.ctypes.data),
                                               c_void_p(col.ctypes.data), rays.shape[0], err, len(err)), err)
        return out, col
