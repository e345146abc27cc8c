"""HIP kernel vs CPU oracle parity on the MI355X (run on the GPU box: pytest -m gpu).

Bar: bit-exact. Both sides implement the same fp32 contract, so every float the
kernel produces must have the oracle's bit pattern (NaN == NaN), and intersection counts must match.
All calls go through the C ABI of librt4.so.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCENES = ["sphere", "room", "tiger", "cylinder4d", "hypercube", "tiger_two_mirrors", "all_primitives"]
REF_SCENES = SCENES[:5]
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    same = a.view(np.uint32) == b.view(np.uint32)
    both_nan = np.isnan(a) & np.isnan(b)
    return same | both_nan


def assert_bits(a, b, what):
    eq = bits_equal(a, b)
    if not eq.all():
        idx = np.argwhere(~eq)[:5]
        detail = [(tuple(i), float(np.asarray(a)[tuple(i)]), float(np.asarray(b)[tuple(i)])) for i in idx]
        pytest.fail(f"{what}: {(~eq).sum()} of {eq.size} values differ, e.g. {detail}")


# ------------------------------------------------------------------------------------------ math
def test_device_math_bitwise(tracer, rt4, oracle):
    rng = np.random.default_rng(1)
    special = np.array([0.0, -0.0, 0.5, -0.5, 1.0, -1.0, 1.0000001, -1.0000001, np.nan, np.inf, -np.inf,
                        np.float32(0.49999997), np.float32(0.50000006), 1e-30, -1e-30, 1e-40], np.float32)
    unit = np.concatenate([np.linspace(-1.0, 1.0, 400001, dtype=np.float32), rng.uniform(-1.2, 1.2, 200000).astype(np.float32), special])
    angles = np.concatenate([np.linspace(-10.0, 10.0, 400001, dtype=np.float32),
                             (rng.random(200000, dtype=np.float32) * np.float32(2.0) * np.float32(3.14159265)), special])
    for fn, x in [(rt4.EVAL_ACOS, unit), (rt4.EVAL_ASIN, unit), (rt4.EVAL_SIN, angles), (rt4.EVAL_COS, angles),
                  (rt4.EVAL_VOLUME_BY_W, unit)]:
        g, _ = tracer.debug_eval(fn, x)
        c, _ = oracle.eval_array(fn, x)
        assert_bits(g, c, f"eval fn {fn}")


def test_sqrt_exhaustive(tracer, rt4):
    """The kernel's sqrt (fast path without input scaling, rt4_device_math.h sqrt_) equals the IEEE
    square root on every one of the 2^32 float patterns (device-side sweep)."""
    assert tracer.debug_verify_sqrt() == 0


def test_sqrt_values(tracer, rt4):
    rng = np.random.default_rng(5)
    bits = rng.integers(0, 2**32, 400000, dtype=np.uint64).astype(np.uint32)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, 1e-40, 2.0**-96, 2.0**-97, 3.4e38, -1.0, 2.0, 0.25],
                       np.float32)
    x = np.concatenate([bits.view(np.float32), special])
    g, _ = tracer.debug_eval(rt4.EVAL_SQRT, x)
    with np.errstate(invalid="ignore"):
        ref = np.sqrt(x)
    assert_bits(g, ref, "sqrt_")


def test_hash_bitwise(tracer, rt4, oracle):
    x = np.random.default_rng(2).integers(0, 2**32, 100000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    g, _ = tracer.debug_eval(rt4.EVAL_HASH, x)
    c, _ = oracle.eval_array(rt4.EVAL_HASH, x)
    assert (g.view(np.uint32) == c.view(np.uint32)).all()


def test_w_by_volume_exhaustive(tracer, rt4, oracle):
    """Every value rand() can return (m * 2^-23, shader.frag:111-118): result bits and Newton iterations."""
    v = (np.arange(1 << 23, dtype=np.uint32) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)
    g, gi = tracer.debug_eval(rt4.EVAL_W_BY_VOLUME, v)
    c, ci = oracle.eval_array(rt4.EVAL_W_BY_VOLUME, v)
    assert_bits(g, c, "w_by_volume")
    assert (gi == ci).all()
    assert not np.isnan(g).any() and np.abs(g).max() <= 1.0
    assert gi.max() < 64  # the loop cap is never reached


# --------------------------------------------------------------------------- kernel selection
EXACT_COUNTS = {  # scene -> (group bits, n_spaces, n_spheres, n_cylinders): rt4_trace.hip kVariants
    "sphere": (0x03, 1, 2, 0), "room": (0x03, 8, 2, 0), "tiger": (0x21, 1, 0, 0),
    "tiger_two_mirrors": (0x21, 3, 0, 0), "cylinder4d": (0x09, 1, 0, 0), "hypercube": (0x11, 1, 0, 0),
    "all_primitives": (0x3F, 2, 3, 1),
}


@pytest.mark.parametrize("name", SCENES)
def test_scene_runs_exact_count_kernel(rt4, name):
    """Every reference and authored scene gets the kernel compiled for its exact object counts."""
    k, nsp, nsh, ncy = EXACT_COUNTS[name]
    t = rt4.Tracer(device=0, scene=rt4.Scene.named(name))
    try:
        assert t.kernel_shape == k | (nsp + 1) << 8 | (nsh + 1) << 16 | (ncy + 1) << 24
    finally:
        t.close()
    t = rt4.Tracer(device=0, scene=rt4.Scene.named(name), flags=rt4.FLAG_GENERIC_KERNEL)
    try:
        assert t.kernel_shape == 0xFFFFFFFF
    finally:
        t.close()


def test_untested_objects_keep_primitive_ids(rt4, oracle):
    """A scene that defines a union the group list never tests: the flat primitive table still holds
    its two entries, so the exact-count kernel (compile-time table bases) must not be chosen; the
    runtime-count kernel renders it bit-exactly."""
    base = rt4.Scene.builtin("hypercube")
    d = rt4.SceneDesc.from_buffer_copy(bytes(base.desc))
    d.n_unions = 1
    d.unions[0] = rt4.Scene.builtin("cylinder4d").desc.unions[0]
    scene = rt4.Scene(d)
    t = rt4.Tracer(device=0, scene=scene)
    try:
        k = t.kernel_shape
    finally:
        t.close()
    assert k == (1 | 16)  # spaces + hypercube, counts read at run time
    u = rt4.make_uniforms(64, 40, samples=3, reflections=4, seed=5)
    fg, ng, fc, nc = render_both(rt4, oracle, scene, u, rt4.region(64, 40), flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert_bits(fg, fc, "hypercube + untested union")


# ------------------------------------------------------------------------------- intersections
def random_rays(n, seed):
    rng = np.random.default_rng(seed)
    p = rng.uniform(-4.0, 4.0, (n, 4)).astype(np.float32)
    p[: n // 4] = np.array([0.0, -2.0, 0.0, 0.0], np.float32)  # camera focus
    d = rng.normal(size=(n, 4)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    return np.concatenate([p, d], axis=1).astype(np.float32)


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("generic", [False, True])
def test_find_intersection_bitwise(rt4, oracle, name, generic):
    scene = rt4.Scene.named(name)
    t = rt4.Tracer(device=0, scene=scene, flags=rt4.FLAG_GENERIC_KERNEL if generic else 0)
    try:
        rays = random_rays(100000, 1000 + SCENES.index(name))
        g, gc = t.debug_find_intersection(rays)
        c, cc = oracle.find_intersection(scene.desc, rays)
        assert_bits(g, c, f"{name} find_intersection")
        assert_bits(gc, cc, f"{name} material color")
        assert g[:, 0].sum() > 1000  # the rays do hit things
    finally:
        t.close()


def grazing_rays(centers, radii, n_per, seed):
    """Rays passing sphere i at perpendicular distance r_i (1 + e), |e| from 1e-8 to 1e-1 and both
    signs, from outside (2r..60r away): the boundary of the sphere cull (rt4_aux.h SphereCull)."""
    rng = np.random.default_rng(seed)
    out = []
    for c, r in zip(centers, radii):
        c = np.asarray(c, np.float64)
        u = rng.normal(size=(n_per, 4))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        v = rng.normal(size=(n_per, 4))
        v -= (v * u).sum(1, keepdims=True) * u
        v /= np.linalg.norm(v, axis=1, keepdims=True)
        L = r * np.exp(rng.uniform(np.log(2.0), np.log(60.0), n_per))[:, None]
        e = np.where(rng.random(n_per) < 0.5, -1.0, 1.0) * 10.0 ** rng.uniform(-8, -1, n_per)
        e[: n_per // 16] = 0.0
        sa = np.clip(r * (1.0 + e)[:, None] / L, 0.0, 1.0)
        d = -u * np.sqrt(1.0 - sa * sa) + v * sa
        out.append(np.concatenate([c + L * u, d], axis=1))
    return np.concatenate(out).astype(np.float32)


@pytest.mark.parametrize("name", ["sphere", "room", "all_primitives"])
def test_find_intersection_grazing_spheres(rt4, oracle, name):
    scene = rt4.Scene.named(name)
    d = scene.desc
    centers = [list(d.spheres[i].center) for i in range(d.n_spheres)]
    radii = [d.spheres[i].r for i in range(d.n_spheres)]
    rays = grazing_rays(centers, radii, 40000, 77)
    c, cc = oracle.find_intersection(scene.desc, rays)
    t = rt4.Tracer(device=0, scene=scene)
    try:
        g, gc = t.debug_find_intersection(rays)
    finally:
        t.close()
    assert_bits(g, c, f"{name} grazing find_intersection")
    assert_bits(gc, cc, f"{name} grazing material color")
    # many of the hits are the spheres themselves (normal unlike every space's), near the tangent
    sn = np.array([list(d.spaces[i].norm) for i in range(d.n_spaces)], np.float32)
    on_space = np.zeros(len(c), bool)
    for n in sn:
        on_space |= np.all(np.abs(np.abs(c[:, 2:6]) - np.abs(n)) < 1e-6, axis=1)
    assert ((c[:, 0] > 0) & ~on_space).mean() > 0.05


def on_cylinder_rays(cyls, n, seed):
    """Rays starting on (or within 1e-6 relative of) infinite cylinders (point, axis1, axis2, r), at any
    distance along their axes: the cases where the exact test can report a NaN-distance hit (a negative
    rounding under the sqrt) far from the figure's bounding ball."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        cp, a1, a2, r = cyls[k % len(cyls)]
        cp, a1, a2 = (np.array(v, np.float64) for v in (cp, a1, a2))
        basis = np.linalg.qr(np.stack([a1, a2] + list(rng.normal(size=(2, 4)))).T)[0].T  # a1, a2, b1, b2
        b1, b2 = basis[2], basis[3]
        phi = rng.uniform(0, 2 * np.pi)
        rr = r * (1 + rng.choice([0.0, 1e-7, -1e-7, 1e-6]))
        p = cp + rng.uniform(-6, 6) * a1 + rng.uniform(-6, 6) * a2 + rr * (np.cos(phi) * b1 + np.sin(phi) * b2)
        d = rng.normal(size=4)
        d /= np.linalg.norm(d)
        out.append(np.concatenate([p, d]))
    return np.array(out, np.float32)


@pytest.mark.parametrize("name", ["tiger", "cylinder4d", "all_primitives", "tiger_two_mirrors"])
def test_find_intersection_rays_on_infinite_cylinders(rt4, oracle, name):
    """Bit-exact on rays from the tiger's / union's cylinder surfaces, including NaN-distance hits
    outside the bounding ball that the kernel's bound skip must not drop (rt4_aux.h BoundBall)."""
    d = rt4.Scene.named(name).desc
    cyls = []
    for q in range(d.n_tigers):
        t = d.tigers[q]
        cyls += [(list(c.point), list(c.axis1), list(c.axis2), c.r) for c in (t.inner_cyl1, t.outer_cyl1, t.inner_cyl2,
                                                                          t.outer_cyl2)]
    for q in range(d.n_unions):
        u = d.unions[q]
        cyls += [(list(c.point), list(c.axis1), list(c.axis2), c.r) for c in (u.cylinder1, u.cylinder2)]
    rays = on_cylinder_rays(cyls, 20000, 123)
    c, cc = oracle.find_intersection(d, rays)
    t = rt4.Tracer(device=0, scene=rt4.Scene(d))
    try:
        g, gc = t.debug_find_intersection(rays)
    finally:
        t.close()
    assert_bits(g, c, f"{name} on-cylinder find_intersection")
    assert_bits(gc, cc, f"{name} on-cylinder material color")


def grazing_cylinder_rays(cyls, n_per, seed):
    """Rays whose projection onto a cylinder's circle plane passes the circle at r (1 + e), |e| from 1e-8 to
    1e-1 and both signs, from outside, with a random component along the axes: the boundary of the cylinders'
    sphere cull (rt4_fast.h cyl_cand_cull, rt4_aux.h SphereCull)."""
    rng = np.random.default_rng(seed)
    out = []
    for cp, a1, a2, r in cyls:
        cp, a1, a2 = (np.array(v, np.float64) for v in (cp, a1, a2))
        for _ in range(n_per):
            b1, b2 = np.linalg.qr(np.stack([a1, a2] + list(rng.normal(size=(2, 4)))).T)[0].T[2:]
            th = rng.uniform(0, 2 * np.pi)
            u = np.cos(th) * b1 + np.sin(th) * b2
            v = -np.sin(th) * b1 + np.cos(th) * b2
            L = r * np.exp(rng.uniform(np.log(2.0), np.log(60.0)))
            e = rng.choice([-1.0, 1.0]) * 10.0 ** rng.uniform(-8, -1) if rng.random() > 1 / 16 else 0.0
            sa = min(r * (1.0 + e) / L, 1.0)
            dp = -u * np.sqrt(1.0 - sa * sa) + v * sa
            d = dp * rng.uniform(0.3, 1.0) + rng.normal(0, 0.5) * a1 + rng.normal(0, 0.5) * a2
            p = cp + L * u + rng.uniform(-3, 3) * a1 + rng.uniform(-3, 3) * a2
            out.append(np.concatenate([p, d / np.linalg.norm(d)]))
    return np.array(out, np.float32)


@pytest.mark.parametrize("name", ["cylinder4d", "all_primitives"])
def test_find_intersection_grazing_cylinders(rt4, oracle, name):
    """Bit-exact on rays grazing the cylinders and the union's cylinders, where the cull (r05-v50) decides."""
    d = rt4.Scene.named(name).desc
    cyls = [(list(c.point), list(c.axis1), list(c.axis2), c.r) for c in (d.cylinders[i] for i in range(d.n_cylinders))]
    for q in range(d.n_unions):
        u = d.unions[q]
        cyls += [(list(c.point), list(c.axis1), list(c.axis2), c.r) for c in (u.cylinder1, u.cylinder2)]
    assert cyls
    rays = grazing_cylinder_rays(cyls, 8000, 321)
    c, cc = oracle.find_intersection(d, rays)
    t = rt4.Tracer(device=0, scene=rt4.Scene(d))
    try:
        g, gc = t.debug_find_intersection(rays)
    finally:
        t.close()
    assert_bits(g, c, f"{name} grazing-cylinder find_intersection")
    assert_bits(gc, cc, f"{name} grazing-cylinder material color")
    assert (c[:, 0] > 0).mean() > 0.05


# -------------------------------------------------------------------------------------- images
def render_both(rt4, oracle, scene, u, reg, flags=0, old=None):
    t = rt4.Tracer(device=0, flags=flags, scene=scene)
    try:
        fg = np.zeros((reg.h, reg.w, 4), np.float32) if old is None else old.copy()
        ng = t.render_host(u, reg, fg)
    finally:
        t.close()
    fc = np.zeros((reg.h, reg.w, 4), np.float32) if old is None else old.copy()
    fc, nc, _, _ = oracle.render(scene.desc, u, reg, fc)
    return fg, ng, fc, nc


@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("flags", ["lut", "inline", "generic"])
def test_render_bitwise_small(rt4, oracle, name, flags):
    u = rt4.make_uniforms(96, 60, samples=4, reflections=4, seed=777)
    reg = rt4.region(96, 60)
    f = {"lut": rt4.FLAG_SAMPLER_LUT, "inline": 0, "generic": rt4.FLAG_GENERIC_KERNEL}[flags]
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named(name), u, reg, flags=f)
    assert ng == nc
    assert_bits(fg, fc, f"{name} image")


def test_render_bitwise_config2_rows(rt4, oracle):
    """BASELINE config 2 (sphere, 1920x1080, 16 spp, 8 bounces, seed 12345) on every 32nd row."""
    u = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=12345)
    reg = rt4.region(1920, 34, y0=5, band_rows=1, band_step=32)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named("sphere"), u, reg, flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert_bits(fg, fc, "config2 rows")


def test_render_bitwise_config3_rows(rt4, oracle):
    """BASELINE config 3 (hypercube, 1920x1080, 16 spp, 8 bounces) on every 64th row."""
    u = rt4.make_uniforms(1920, 1080, samples=16, reflections=8, seed=12345)
    reg = rt4.region(1920, 17, y0=11, band_rows=1, band_step=64)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named("hypercube"), u, reg)
    assert ng == nc
    assert_bits(fg, fc, "config3 rows")


def test_render_bitwise_config1_full_frame(rt4, oracle):
    """BASELINE config 1 (sphere, 256x256, 1 spp, 2 bounces, seed 12345): every pixel, and the count
    stays within the nominal bound W*H*spp*(B+1)."""
    u = rt4.make_uniforms(256, 256, samples=1, reflections=2, seed=12345)
    reg = rt4.region(256, 256)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named("sphere"), u, reg, flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert 256 * 256 <= ng <= 256 * 256 * 1 * 3
    assert_bits(fg, fc, "config1 frame")


@pytest.mark.parametrize("name,spp,bounces,flags", [
    ("tiger_two_mirrors", 64, 12, "lut"),  # BASELINE config 4 (3840x2160, 64 spp, 12 bounces)
    ("all_primitives", 16, 8, "inline"),  # BASELINE config 5's frame (3840x2160, 16 spp per frame)
])
def test_render_bitwise_4k_configs_rows(rt4, oracle, name, spp, bounces, flags):
    """The 8-GPU configs at their full 4K resolution and sample counts, on two rows far apart (one
    near the middle, one in the lower half): uniforms and scr_coord bits are those of the 4K frame."""
    u = rt4.make_uniforms(3840, 2160, samples=spp, reflections=bounces, seed=12345)
    reg = rt4.region(3840, 2, y0=1003, band_rows=1, band_step=700)
    f = {"lut": rt4.FLAG_SAMPLER_LUT, "inline": 0}[flags]
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named(name), u, reg, flags=f)
    assert ng == nc
    assert_bits(fg, fc, f"{name} 4k rows")


def test_progressive_blend(rt4, oracle):
    """mix(old_frame, new, part) with part = 1/3 over a non-zero old frame (shader.frag:524-527)."""
    u = rt4.make_uniforms(64, 40, samples=2, reflections=3, seed=99, part=1.0 / 3.0)
    reg = rt4.region(64, 40)
    old = np.random.default_rng(5).random((40, 64, 4), dtype=np.float32)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene.named("tiger"), u, reg, old=old)
    assert ng == nc
    assert_bits(fg, fc, "progressive")


def test_banded_regions_tile_the_image(rt4):
    """Pixel-tile sharding: two interleaved band sets reproduce the full image bit for bit."""
    u = rt4.make_uniforms(80, 64, samples=2, reflections=3, seed=4242)
    scene = rt4.Scene.named("cylinder4d")
    t = rt4.Tracer(device=0, scene=scene)
    try:
        full = np.zeros((64, 80, 4), np.float32)
        n_full = t.render_host(u, rt4.region(80, 64), full)
        parts, n_parts = [], 0
        for r in range(2):
            f = np.zeros((32, 80, 4), np.float32)
            n_parts += t.render_host(u, rt4.region(80, 32, y0=8 * r, band_rows=8, band_step=16), f)
            parts.append(f)
    finally:
        t.close()
    rebuilt = np.zeros_like(full)
    for r in range(2):
        for b in range(4):
            rebuilt[16 * b + 8 * r: 16 * b + 8 * r + 8] = parts[r][8 * b: 8 * b + 8]
    assert n_parts == n_full
    assert_bits(rebuilt, full, "banded")


@pytest.mark.parametrize("name", REF_SCENES)
def test_golden_images(rt4, name):
    """GPU output against the committed oracle images (tests/golden/make_golden.py)."""
    meta = json.load(open(os.path.join(GOLDEN, "images.json")))[name]
    u = rt4.make_uniforms(meta["width"], meta["height"], samples=meta["samples"], reflections=meta["reflections"],
                          seed=meta["seed"])
    t = rt4.Tracer(device=0, scene=rt4.Scene.named(name))
    try:
        f = np.zeros((meta["height"], meta["width"], 4), np.float32)
        n = t.render_host(u, rt4.region(meta["width"], meta["height"]), f)
    finally:
        t.close()
    ref = np.load(os.path.join(GOLDEN, f"image_{name}.npy"))
    assert n == meta["intersections"]
    assert_bits(f, ref, f"golden {name}")


# ------------------------------------------------------------------- scene-constant verification
def test_reduced_divisor_sweep_agrees_with_full(tracer, rt4):
    """rt4_context_set_scene enables the 3-op quotient for a divisor after a REDUCED sweep (positive
    numerators; exponent fields outside the middle band, plus three fields of it: DESIGN.md §4.5). On
    every divisor of the seven scenes and on random ones over the whole exponent range it must decide
    exactly as the sweep over all 2^32 numerators."""
    divs = set()
    for name in SCENES:
        d = rt4.Scene.named(name).desc
        divs |= {d.spheres[i].r for i in range(d.n_spheres)} | {d.cylinders[i].r for i in range(d.n_cylinders)}
        for i in range(d.n_unions):
            divs |= {d.unions[i].cylinder1.r, d.unions[i].cylinder2.r}
        for i in range(d.n_tigers):
            t = d.tigers[i]
            divs |= {t.inner_cyl1.r, t.outer_cyl1.r, t.inner_cyl2.r, t.outer_cyl2.r}
        divs.add(d.sun.angular_size)
    rng = np.random.default_rng(11)
    rand = (rng.uniform(0.5, 1.0, 24) * 2.0 ** rng.integers(-120, 120, 24)).astype(np.float32)
    divs |= {float(x) for x in rand} | {3.0, 0.1, 1.0, 7.0, 1e-30, 3e30}
    divs = {b for b in divs if np.isfinite(b) and b != 0 and np.isfinite(np.float32(1) / np.float32(b))}
    decided = {True: 0, False: 0}
    for b in sorted(divs):
        red, full = tracer.debug_verify_div(b), tracer.debug_verify_div(b, full=True)
        assert (red == 0) == (full == 0), (b, red, full)
        assert red <= full
        decided[full == 0] += 1
    assert decided[True] > 0 and decided[False] > 0  # both outcomes occur: the check has teeth


def test_sky_threshold_sweep_restriction(tracer, rt4):
    """For sun angular sizes <= 1 set_scene searches the acos threshold over c in (0.5, 1] only. The
    full 2^32 search at ang = 1 lands above 0.5, which proves that no c <= 0.5 has acos(c) < 1 (and so
    < any smaller ang); restricted and full searches agree on the scenes' suns and random sizes."""
    c1 = tracer.debug_sky_threshold(1.0, full=True)
    assert c1 > 0.5
    angs = {rt4.Scene.named(n).desc.sun.angular_size for n in SCENES}
    angs |= {float(x) for x in np.random.default_rng(3).uniform(1e-4, 1.0, 6).astype(np.float32)} | {1.0}
    for a in sorted(angs):
        r, f = tracer.debug_sky_threshold(a), tracer.debug_sky_threshold(a, full=True)
        assert (np.isnan(r) and np.isnan(f)) or np.float32(r).view(np.uint32) == np.float32(f).view(np.uint32), (a, r, f)


# ---------------------------------------------------------------------------- primary-ray reuse
@pytest.mark.parametrize("name", SCENES)
@pytest.mark.parametrize("spp,bounces", [(4, 4), (3, 0), (1, 2)])
def test_primary_reuse_bitwise(rt4, oracle, name, spp, bounces):
    """RT4_FLAG_PRIMARY_REUSE: the cached primary candidate gives the same image and the same reference
    count as evaluating it in every sample (bounces = 0: every sample ends at its first bounce; spp = 1:
    nothing to reuse); evaluated calls = count - (spp - 1) per pixel."""
    u = rt4.make_uniforms(96, 60, samples=spp, reflections=bounces, seed=4321)
    reg = rt4.region(96, 60)
    scene = rt4.Scene.named(name)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT | rt4.FLAG_PRIMARY_REUSE, scene=scene)
    try:
        fg = np.zeros((60, 96, 4), np.float32)
        ng = t.render_host(u, reg, fg)
        n_eval = t.evaluated()
    finally:
        t.close()
    fc, nc, _, _ = oracle.render(scene.desc, u, reg)
    assert ng == nc
    assert_bits(fg, fc, f"{name} primary reuse")
    assert n_eval == nc - (spp - 1) * 96 * 60


def test_primary_reuse_progressive_and_sections(rt4, oracle):
    """Reuse across progressive frames (fp16 accumulator) and in a three-section launch."""
    import torch

    scene = rt4.Scene.named("room")
    base = rt4.make_uniforms(72, 44, samples=5, reflections=6, seed=77)
    reg = rt4.region(72, 44)
    t = rt4.Tracer(device=0, flags=rt4.FLAG_SAMPLER_LUT | rt4.FLAG_PRIMARY_REUSE, scene=scene)
    try:
        g = np.zeros((44, 72, 4), np.float16)
        c = np.zeros((44, 72, 4), np.float16)
        for n in range(1, 4):
            u = rt4.progressive_uniforms(base, n)
            ng = t.render_host_ex(u, reg, g, rt4.FRAME_RGBA16F)
            _, nc = oracle.render_fmt(scene.desc, u, reg, rt4.FRAME_RGBA16F, frame=c)
            assert ng == nc
            assert (g.view(np.uint16) == c.view(np.uint16)).all(), n
        jobs, frames, us = [], [], []
        for sec, (w, h) in zip((rt4.SECTION_YXZ, rt4.SECTION_YWZ, rt4.SECTION_YXW), [(50, 31), (30, 19), (30, 19)]):
            u = rt4.make_uniforms(w, h, samples=3, reflections=4, seed=9, section=sec, fi=15.0, te=5.0, psi=20.0)
            fr = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
            frames.append(fr)
            us.append((u, w, h))
            jobs.append((u, rt4.region(w, h), fr.data_ptr(), w))
        t.render_sections_device(jobs)
        torch.cuda.synchronize()
        for (u, w, h), fr in zip(us, frames):
            cc, _, _, _ = oracle.render(scene.desc, u, rt4.region(w, h))
            assert (fr.cpu().numpy().view(np.uint32) == cc.view(np.uint32)).all()
    finally:
        t.close()


def test_find_intersection_hypercube_face_planes(rt4, oracle):
    """The axis-aligned cell test (rt4_fast.h axis2) against the exact one where they could differ:
    rays starting exactly on a cell's face plane (h = +-0, whose sign the full dot may flip), rays
    parallel to a face (cos_dn = 0), zero direction components, and origins on the cell edges."""
    scene = rt4.Scene.named("hypercube")
    d = scene.desc
    rng = np.random.default_rng(17)
    planes = []
    for k in range(8):
        cu = d.hypercubes[0].cubes[k]
        planes.append((k & 3, cu.point[k & 3], cu.r, list(cu.point)))
    rays = []
    for q in range(40000):
        a, c, r, cpt = planes[q % 8]
        p = rng.uniform(-3.0, 3.0, 4).astype(np.float32)
        p[a] = np.float32(c) if q % 3 else -np.float32(c)
        if q % 5 == 0:  # on an edge of the cell: a second coordinate at +-r from the cell point
            b = (a + 1 + q % 3) % 4
            p[b] = np.float32(cpt[b] + (r if q % 2 else -r))
        dv = rng.normal(size=4).astype(np.float32)
        if q % 4 == 0:
            dv[a] = 0.0  # parallel to the face
        if q % 7 == 0:
            dv[(a + 2) % 4] = -0.0
        dv /= np.float32(np.linalg.norm(dv))
        rays.append(np.concatenate([p, dv]))
    rays = np.array(rays, np.float32)
    c, cc = oracle.find_intersection(d, rays)
    t = rt4.Tracer(device=0, scene=scene)
    try:
        g, gc = t.debug_find_intersection(rays)
    finally:
        t.close()
    assert_bits(g, c, "hypercube face-plane find_intersection")
    assert_bits(gc, cc, "hypercube face-plane colour")
    assert c[:, 0].sum() > 1000
