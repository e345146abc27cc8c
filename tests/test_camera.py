"""Camera model and the image writer (row 4) on the CPU. The expected values
are an independent numpy-float32 restatement of src/controls.cpp / src/util/math.cpp / main.cpp:86-91."""
import math

import numpy as np
import pytest

F = np.float32
PI = F(3.14159265)

# the camera block of executable/properties.txt:25-51 (values only)
PROPS = """
ray_tracing.samples = 2
ray_tracing.reflections_amount = 3
ray_tracing.small_indent = 0.005
light_to_color_conversion_coefficient = 1.0
camera.matrix_height = 2.0
camera.focus_to_matrix_distance = 1.5
camera.initial_position.x = 0.0
camera.initial_position.y = -2.0
camera.initial_position.z = 0.0
camera.initial_position.w = 0.0
camera.initial_position.fi  = {fi}
camera.initial_position.te  = {te}
camera.initial_position.psi = {psi}
mouse_border_width = 15
constrain_psi_range = {constrain}
psi_range_radius = 45.0
mouse_sensitivity = 0.005
wheel_sensitivity = 0.1
movement_speed = 3.0
"""


def normalize_angle(a):  # math.cpp:24-28 (std::remainder on floats)
    a = F(math.remainder(float(F(a)), float(F(2) * PI)))
    if a < -PI:
        a = F(a + F(2) * PI)
    if a > PI:
        a = F(a - F(2) * PI)
    return a


def pull(f, c, r):  # math.cpp:19-22
    f = F(f)
    if f < F(c - r):
        f = F(c - r)
    if f > F(c + r):
        f = F(c + r)
    return f


def rotate(angle, x, y):  # controls.cpp:63-68
    s, c = F(math.sin(float(angle))), F(math.cos(float(angle)))
    return x * c + y * s, x * -s + y * c


def orientation(fi, te, psi):  # Orientation::update, controls.cpp:72-86
    fwd, top, right, w = (np.array(v, F) for v in ([0, 1, 0, 0], [0, 0, 1, 0], [1, 0, 0, 0], [0, 0, 0, 1]))
    top, w = rotate(psi, top, w)
    vtop = top.copy()
    fwd, right = rotate(fi, fwd, right)
    hf, hr = fwd.copy(), right.copy()
    fwd, top = rotate(te, fwd, top)
    return dict(forward=fwd, top=top, right=right, w_drct=w, horizontal_forward=hf, horizontal_right=hr,
                vertical_top=vtop)


def camera(rt4, fi=0.0, te=0.0, psi=0.0, constrain="true"):
    return rt4.Camera(rt4.Properties(text=PROPS.format(fi=fi, te=te, psi=psi, constrain=constrain)))


def vec(a):
    return np.array(a[:], F)


def test_init_and_orientation(rt4):
    cam = camera(rt4, fi=30.0, te=100.0, psi=-20.0)  # te clamps to pi/2
    s = cam.s
    d2r = lambda d: F(F(d) / F(180) * PI)  # noqa: E731
    assert s.fi == normalize_angle(d2r(30.0)) and s.te == pull(d2r(100.0), 0, PI / F(2))
    assert s.psi == d2r(-20.0) and s.psi_range_center == d2r(-20.0) and s.psi_range_radius == d2r(45.0)
    assert s.frame_number == 1 and list(s.focus) == [0.0, -2.0, 0.0, 0.0]
    o = orientation(s.fi, s.te, s.psi)
    for k, v in o.items():
        np.testing.assert_allclose(vec(getattr(s.orientation, k)), v, rtol=0, atol=2e-7)


def test_rotation_normalisation(rt4):
    cam = camera(rt4)
    fi, te, psi = F(0), F(0), F(0)
    for dfi, dte, dpsi in [(1.0, 0.3, 0.2), (2.5, 1.5, 0.5), (3.0, -4.0, -2.0), (-7.0, 0.2, 0.1)]:
        cam.rotate(dfi, dte, dpsi)
        fi = normalize_angle(F(fi + F(dfi)))
        te = pull(F(te + F(dte)), 0, PI / F(2))
        psi = pull(F(psi + F(dpsi)), F(0), F(F(45) / F(180) * PI))  # constrain_psi_range = true
        assert (cam.s.fi, cam.s.te, cam.s.psi) == (fi, te, psi)
        assert cam.s.frame_number == 1
    cam2 = camera(rt4, constrain="false")
    cam2.rotate(0, 0, 4.0)
    assert cam2.s.psi == normalize_angle(F(4.0))


def test_mouse_and_wheel(rt4):
    cam = camera(rt4)
    before = bytes(cam.s)
    assert cam.mouse_move(300, 0, 200) is True and bytes(cam.s) == before  # re-centre only
    assert cam.mouse_move(0, 0, 200) is False and bytes(cam.s) == before
    cam.s.frame_number = 5
    assert cam.mouse_move(40, -10, 200) is False
    assert cam.s.fi == normalize_angle(F(F(40) * F(0.005))) and cam.s.te == pull(F(F(-10) * F(0.005)), 0, PI / F(2))
    assert cam.s.frame_number == 1
    cam.s.frame_number = 3
    cam.wheel(2.0)
    assert cam.s.psi == F(F(2.0) * F(0.1)) and cam.s.frame_number == 1


def test_move(rt4):
    cam = camera(rt4, fi=25.0, te=10.0, psi=5.0)
    o = orientation(cam.s.fi, cam.s.te, cam.s.psi)
    cam.s.frame_number = 9
    cam.move(rt4.KEY_FORWARD | rt4.KEY_RIGHT | rt4.KEY_W_NEG, 0.25)
    d = o["horizontal_forward"] + o["horizontal_right"] - o["w_drct"]
    ln = F(np.sqrt(F(F(F(d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) + d[3] * d[3])))
    k = F(F(F(0.25) * F(3.0)) / ln)
    np.testing.assert_array_equal(vec(cam.s.focus), np.array([0, -2, 0, 0], F) + d * k)
    assert cam.s.frame_number == 1
    cam.s.frame_number = 4
    focus = vec(cam.s.focus)
    cam.move(rt4.KEY_FORWARD | rt4.KEY_BACK, 1.0)  # opposite keys cancel: no move, frame kept
    assert (vec(cam.s.focus) == focus).all() and cam.s.frame_number == 4


def test_frame_uniforms_progressive(rt4):
    cam = camera(rt4, fi=15.0)
    base = rt4.make_uniforms(64, 40, samples=2, reflections=3)
    parts = []
    for n in range(3):
        u = cam.frame_uniforms(base, rt4.SECTION_YWZ, seed=100 + n)
        parts.append(u.part)
        assert u.seed == 100 + n and u.samples == 2 and list(u.resolution) == [64.0, 40.0]
    assert parts == [F(1), F(1) / F(2), F(1) / F(3)]
    o = cam.s.orientation
    np.testing.assert_array_equal(vec(u.vec_to_mtr), vec(o.forward) * F(1.5))
    np.testing.assert_array_equal(vec(u.top_drct), vec(o.top))
    np.testing.assert_array_equal(vec(u.right_drct), vec(o.w_drct))
    cam.move(rt4.KEY_UP, 0.1)  # a move restarts the accumulation
    assert cam.frame_uniforms(base).part == F(1)


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_write_ppm(rt4, tmp_path, fmt):
    rng = np.random.default_rng(fmt)
    f32 = rng.uniform(-0.2, 1.2, (5, 7, 4)).astype(np.float32)
    frame = {0: f32, 1: f32.astype(np.float16), 2: (np.clip(f32, 0, 1) * 255 + 0.5).astype(np.uint8)}[fmt]
    path = str(tmp_path / "out.ppm")
    rt4.write_ppm(path, frame)
    data = open(path, "rb").read()
    assert data.startswith(b"P6\n7 5\n255\n")
    px = np.frombuffer(data[len(b"P6\n7 5\n255\n"):], np.uint8).reshape(5, 7, 3)
    src = frame[..., :3].astype(np.float32)
    want = frame[..., :3] if fmt == 2 else (np.clip(src, 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    assert (px == want).all()


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_write_png_same_pixels_as_ppm(rt4, tmp_path, fmt):
    """rt4_write_png: a valid PNG (signature, IHDR, CRCs, zlib stream with Adler-32) whose decoded pixels
    are byte for byte the PPM's (the same RGBA8 rule), in every frame format; a padded row stride too."""
    import struct
    import zlib

    rng = np.random.default_rng(10 + fmt)
    f32 = rng.uniform(-0.2, 1.2, (6, 9, 4)).astype(np.float32)
    frame = {0: f32, 1: f32.astype(np.float16), 2: (np.clip(f32, 0, 1) * 255 + 0.5).astype(np.uint8)}[fmt]
    rt4.write_ppm(str(tmp_path / "a.ppm"), frame)
    rt4.write_png(str(tmp_path / "a.png"), frame)
    ppm = open(tmp_path / "a.ppm", "rb").read()[len(b"P6\n9 6\n255\n"):]
    data = open(tmp_path / "a.png", "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body)
        chunks[typ] = body
        pos += 12 + n
    assert struct.unpack(">IIBBBBB", chunks[b"IHDR"]) == (9, 6, 8, 2, 0, 0, 0) and b"IEND" in chunks
    raw = zlib.decompress(chunks[b"IDAT"])  # checks the Adler-32 too
    rows = [raw[i * 28:(i + 1) * 28] for i in range(6)]
    assert all(r[0] == 0 for r in rows)
    assert b"".join(r[1:] for r in rows) == ppm
    # a padded buffer through the C ABI: the padding columns are not written
    import ctypes
    import os

    pad = np.zeros((6, 12, 4), dtype=frame.dtype)
    pad[:, :9] = frame
    err = ctypes.create_string_buffer(256)
    assert rt4.lib.rt4_write_png(os.fsencode(str(tmp_path / "b.png")), ctypes.c_void_p(pad.ctypes.data), fmt, 9, 6, 12,
                                 err, len(err)) == 0
    assert open(tmp_path / "b.png", "rb").read() == data
    assert rt4.lib.rt4_write_png(os.fsencode(str(tmp_path / "c.png")), ctypes.c_void_p(pad.ctypes.data), fmt, 30000, 1,
                                 30000, err, len(err)) == -1  # a row over a stored block's 65535 bytes
