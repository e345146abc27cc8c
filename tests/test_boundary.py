"""The drop-in boundary on the CPU: C-ABI exports, properties.txt grammar, camera / uniform producers
and the scene loader (no GPU needed; nothing here launches a kernel)."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

from conftest import REFERENCE, reference_available

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt4.h")
GOLDEN32 = np.float32(1.61803399)


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt4_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(rt4):
    names = declared_functions()
    assert len(names) >= 25
    lib = ctypes.CDLL(rt4.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(rt4.EXPORTED)  # the Python binding covers exactly the header


def test_layout_matches_binding(rt4):
    assert ctypes.sizeof(rt4.SceneDesc) == rt4.lib.rt4_scene_desc_size()
    assert ctypes.sizeof(rt4.Uniforms) == rt4.lib.rt4_uniforms_size() == 104  # 13 uniforms, 26 words
    assert rt4.lib.rt4_abi_version() == 2
    assert b"gfx950" in rt4.lib.rt4_build_info()


# ------------------------------------------------------------------------------ properties.txt
PROPS = """# comment line
 ray_tracing.samples = 100          # trailing comment
 ray_tracing.reflections_amount = 4
 ray_tracing.small_indent = 0.005
 camera.focus_to_matrix_distance = 1.5
 camera.matrix_height = 2.0
 camera.initial_position.x = 0.0
 camera.initial_position.y = -2.0
 camera.initial_position.z = 0.0
 camera.initial_position.w = 0.0
 camera.initial_position.fi  = 0.0
 camera.initial_position.te  = 0.0
 camera.initial_position.psi = 0.0
 constrain_psi_range = true
 psi_range_radius = 45.0
 light_to_color_conversion_coefficient = 1.0
 window.main.title = Main section
 window.main.width = 850
 window.main.cell_size = 7
 window.additional.width = 600
 window.additional.cell_size = 10
 show_additional_windows = TRUE
 dup = first
 dup = second
 int_garbage = 12abc
 negative = -3
 not_a_number = abc
 huge = 99999999999
 empty_value =
 a = b = c
"""


def test_properties_grammar(rt4):
    p = rt4.Properties(text=PROPS)
    assert p.getUnsignedInt("ray_tracing.samples") == 100
    assert p.getFloat("ray_tracing.small_indent") == np.float32(0.005)
    assert p.getString("window.main.title") == "Main section"
    assert p.getBool("show_additional_windows") is True  # case-insensitive (properties.cpp:70)
    assert p.getString("dup") == "first"  # unordered_map::insert keeps the first (properties.cpp:25)
    assert p.getInt("int_garbage") == 12  # std::stoi stops at the first non-digit
    assert p.getInt("negative") == -3
    assert p.getString("empty_value") == ""
    assert p.getString("a") == "b = c"  # split at the first '='
    assert p.getStringOrNull("no.such.key") == ""
    for key, fn in (("negative", p.getUnsignedInt), ("not_a_number", p.getInt), ("huge", p.getInt),
                    ("not_a_number", p.getFloat), ("not_a_number", p.getBool), ("no.such.key", p.getString)):
        with pytest.raises(rt4.RT4Error):
            fn(key)
    with pytest.raises(rt4.RT4Error, match="Cannot find property"):
        p.getFloat("missing")


def test_properties_errors(rt4, tmp_path):
    with pytest.raises(rt4.RT4Error, match="Cannot parse the line"):
        rt4.Properties(text="key_without_separator\n")
    with pytest.raises(rt4.RT4Error, match="Cannot open file"):
        rt4.Properties(path=str(tmp_path / "nope.txt"))
    f = tmp_path / "crlf.txt"
    f.write_bytes(b"flag = true\r\nn = 3\r\n")  # Windows line endings (the reference ran on Windows)
    p = rt4.Properties(path=str(f))
    assert p.getBool("flag") is True and p.getUnsignedInt("n") == 3


def test_window_cells(rt4):
    p = rt4.Properties(text=PROPS)
    assert rt4.window_cells(p, "main") == (121, 75)  # 850/7, int(850/GOLDEN)/7 (windows.cpp:10-12,25-26)
    assert rt4.window_cells(p, "additional") == (60, 37)


def test_uniforms_default_camera(rt4):
    p = rt4.Properties(text=PROPS)
    u = rt4.uniforms_from_properties(p, 121, 75)
    assert (u.samples, u.reflections_amount) == (100, 4)
    assert u.small_indent == np.float32(0.005) and u.light_to_color_conversion_coefficient == 1.0
    assert list(u.mtr_sizes) == [float(np.float32(2.0) * GOLDEN32), 2.0]  # main.cpp:37-38
    assert list(u.focus) == [0, -2, 0, 0]
    assert list(u.vec_to_mtr) == [0, 1.5, 0, 0]  # forward * focus_to_matrix_distance
    assert list(u.top_drct) == [0, 0, 1, 0] and list(u.right_drct) == [1, 0, 0, 0]
    assert list(u.resolution) == [121, 75] and u.part == 1.0
    u2 = rt4.uniforms_from_properties(p, 60, 37, rt4.SECTION_YWZ)
    assert list(u2.top_drct) == [0, 0, 1, 0] and list(u2.right_drct) == [0, 0, 0, 1]
    u3 = rt4.uniforms_from_properties(p, 60, 37, rt4.SECTION_YXW)
    assert list(u3.top_drct) == [0, 0, 0, 1] and list(u3.right_drct) == [1, 0, 0, 0]


def test_orientation_rotations(rt4):
    o = rt4.Orientation(fi=np.float32(np.pi / 2), te=0.0, psi=0.0)
    np.testing.assert_allclose(o.forward, [1, 0, 0, 0], atol=1e-6)  # (forward, right) rotated by fi
    np.testing.assert_allclose(o.right, [0, -1, 0, 0], atol=1e-6)
    o = rt4.Orientation(0.3, 0.2, 0.1)
    basis = np.array([o.forward, o.top, o.right, o.w_drct], np.float64)
    np.testing.assert_allclose(basis @ basis.T, np.eye(4), atol=1e-6)
    np.testing.assert_allclose(o.vertical_top, rt4.Orientation(0.0, 0.0, 0.1).top, atol=1e-7)


def test_psi_constraint(rt4):
    text = PROPS.replace("camera.initial_position.psi = 0.0", "camera.initial_position.psi = 400.0")
    u = rt4.uniforms_from_properties(rt4.Properties(text=text), 10, 10)
    # SphOrientation::init (controls.cpp:29-39): the range centre is the normalised psi (400 -> 40 deg)
    # but psi itself is then clamped into [centre - 45, centre + 45]: 400 deg -> 85 deg
    psi = np.deg2rad(85.0)
    np.testing.assert_allclose(u.top_drct, [0, 0, np.cos(psi), np.sin(psi)], atol=1e-5)


# ------------------------------------------------------------------------------ scenes
REF_SCENES = {"Шар": "sphere", "Комната": "room", "Фигура": "tiger", "Четырёхмерный": "cylinder4d",
              "Гиперкуб": "hypercube"}


@pytest.mark.skipif(not reference_available(), reason="reference tree not mounted (GPU box)")
def test_reference_scene_files_parse_to_builtins(rt4):
    files = sorted(glob.glob(os.path.join(REFERENCE, "scenes", "*.frag")))
    assert len(files) == 5
    for f in files:
        name = [v for k, v in REF_SCENES.items() if k in os.path.basename(f)][0]
        assert rt4.Scene.load_frag(f).to_bytes() == rt4.Scene.builtin(name).to_bytes(), name
    full = rt4.Scene.load_frag(os.path.join(REFERENCE, "executable", "shader.frag"))
    assert full.to_bytes() == rt4.Scene.builtin("tiger").to_bytes()  # shipped default scene


def test_builtin_scene_values(rt4):
    s = rt4.Scene.builtin("room").desc
    assert s.n_spaces == 8 and s.n_spheres == 2 and s.final_light_mode == rt4.FINAL_LIGHT_CONSTANT
    assert s.spheres[0].center[2] == np.float32(-3.5) / np.float32(5)  # -size/5, fp32 folding
    assert s.spheres[0].r == np.float32(0.35) * np.float32(3.5)
    s = rt4.Scene.builtin("hypercube").desc
    assert s.n_hypercubes == 1 and list(s.hypercubes[0].cubes[4].norm) == [-1, 0, 0, 0]
    assert list(s.hypercubes[0].cubes[4].point) == [-1, 2, 0, 0]
    s = rt4.Scene.builtin("sphere").desc
    assert s.sun.angular_size == np.float32(3.14159265) * np.float32(0.09)
    assert s.groups[1].kind == rt4.GROUP_SPHERES and s.groups[1].outer == 1


def test_authored_scenes_parse(rt4):
    for f in sorted(glob.glob(os.path.join(ROOT, "scenes", "*.frag"))):
        s = rt4.Scene.load_frag(f)
        assert s.desc.n_groups >= 1, f


SNIPPET = """
const float size = 2.0;
const vec3 sky_light = vec3(0.1, 0.2, 0.3);
const sun_properties sun = sun_properties(vec4(0, 0, 1, 0), PI * 0.1, vec3(1), 0.5);
const uint n = 2;
const visible_sphere[n] balls = visible_sphere[n](
  visible_sphere(sphere(vec4(-size/5, 0, 0, 0), 0.5 * size), material(1, 0.25, vec3(1, 0, 0))), /* block */
  visible_sphere(sphere(vec4(1, 2, 3, 4), 0.5), material(0, 0, vec3(0, 1, 0)))
);
visible_cylinder[1] tubes = visible_cylinder[1](visible_cylinder(vec4(0), vec4(1, 0, 0, 0), vec4(0, 1, 0, 0), 0.25, material(0, 0, vec3(0.5))));
intersection find_intersection(ray ray) {
  intersection inter = NOT_INTERSECT;
  inter = closest(sphere_intersection(balls[1], ray, false), inter);
  for (int i = 0; i < tubes.length(); i++) { inter = closest(inter, cylinder_intersection(tubes[i], ray, true)); }
  for (int i = 0; i < n; i++)
    inter = closest(sphere_intersection(balls[i], ray, true), inter);
  return inter;
}
vec3 final_light(vec4 drct) { return vec3(0.5, 0.25, 0.125); }
"""


def test_scene_loader_subset(rt4):
    d = rt4.Scene.parse(SNIPPET).desc
    assert d.n_spheres == 2 and d.n_cylinders == 1
    assert d.spheres[0].center[0] == np.float32(-2.0) / np.float32(5) and d.spheres[0].r == 1.0
    assert d.spheres[0].material.refl_prob == 0.25
    groups = [(g.kind, g.first, g.count, g.outer, g.new_first) for g in d.groups[: d.n_groups]]
    assert groups == [(rt4.GROUP_SPHERES, 1, 1, 0, 1), (rt4.GROUP_CYLINDERS, 0, 1, 1, 0), (rt4.GROUP_SPHERES, 0, 2, 1, 1)]
    assert d.final_light_mode == rt4.FINAL_LIGHT_CONSTANT and list(d.final_light_const) == [0.5, 0.25, 0.125]


@pytest.mark.parametrize("bad, msg", [
    ("intersection find_intersection(ray ray) { inter = closest(foo_intersection(x, ray), inter); }", "unsupported"),
    ("const vec3 sky_light = vec3(1);", "find_intersection"),
    ("visible_sphere s = visible_sphere(sphere(vec4(0), 1), material(0, 0, vec3(1)));\n"
     "intersection find_intersection(ray ray) { inter = closest(sphere_intersection(s, ray, true), inter); }",
     "sky_light"),
    ("const visible_sphere[2] s = visible_sphere[2](visible_sphere(sphere(vec4(0), 1), material(0, 0, vec3(1))));", "size mismatch"),
    ("const float x = vec4(1, 2);", None),  # not a scene object: ignored, so the error is the missing function
    ("visible_sphere s = visible_sphere(sphere(vec4(0, 0), 1), material(0, 0, vec3(1)));", "components"),
    ("/* unterminated", "unterminated"),
])
def test_scene_loader_errors(rt4, bad, msg):
    with pytest.raises(rt4.RT4Error, match=msg or "find_intersection"):
        rt4.Scene.parse(bad)


def test_scene_capacity_error(rt4):
    items = ",".join(["visible_sphere(sphere(vec4(0), 1), material(0, 0, vec3(1)))"] * 33)
    text = (f"const vec3 sky_light = vec3(1); const sun_properties sun = sun_properties(vec4(1), 1, vec3(1), 0);"
            f"visible_sphere[33] s = visible_sphere[33]({items});"
            "intersection find_intersection(ray ray) { for (int i = 0; i < s.length(); i++) "
            "inter = closest(sphere_intersection(s[i], ray, true), inter); }")
    with pytest.raises(rt4.RT4Error, match="too many"):
        rt4.Scene.parse(text)


def test_scene_missing_file(rt4, tmp_path):
    with pytest.raises(rt4.RT4Error, match="cannot open"):
        rt4.Scene.load_frag(str(tmp_path / "Сцена.frag"))  # UTF-8 path
