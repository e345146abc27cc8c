"""Randomised scenes: HIP kernel vs CPU oracle, bit-exact (run on the GPU box: pytest -m gpu).

The fixed scenes pin the kernel on the reference's geometry. Here every object of the authored
all-primitives scene (and of the reference scenes) is perturbed from a seed: positions, radii, axes,
normals, the sun, the camera. That exercises the per-scene host work on geometry nobody chose:
verified divisors for arbitrary radii, the sphere-cull thresholds, the bounding-ball skips of the
tiger and the union (including axes that are no longer orthonormal, where the host must refuse the
skip) and the tiger's shared-axes check (broken on purpose in some seeds: generic tiger path).
"""
import numpy as np
import pytest

from test_gpu_parity import assert_bits, random_rays, render_both

pytestmark = pytest.mark.gpu


def _f4(arr):
    return np.array(arr[:4], np.float32)


def _set4(arr, v):
    for i in range(4):
        arr[i] = float(np.float32(v[i]))


def _unit(v):
    v = np.asarray(v, np.float64)
    return (v / np.linalg.norm(v)).astype(np.float32)


def _rotation(rng, angle):
    """A random 4D rotation by a small angle (exp of a skew matrix, in float64)."""
    a = rng.normal(size=(4, 4))
    a = (a - a.T) / 2.0
    a *= angle / np.linalg.norm(a, 2)
    w, v = np.linalg.eig(a)
    return np.real(v @ np.diag(np.exp(w)) @ np.linalg.inv(v))


def _perturb_cylinder(c, rng, rot, shift, rscale):
    _set4(c.point, _f4(c.point) + shift)
    _set4(c.axis1, (rot @ _f4(c.axis1).astype(np.float64)).astype(np.float32))
    _set4(c.axis2, (rot @ _f4(c.axis2).astype(np.float64)).astype(np.float32))
    c.r = float(np.float32(c.r * rscale))


def perturb(rt4, name, seed):
    """Returns a Scene: `name` with every object moved by a seeded amount."""
    rng = np.random.default_rng(seed)
    scene = rt4.Scene.named(name)
    d = rt4.SceneDesc.from_buffer_copy(scene.to_bytes())
    for i in range(d.n_spaces):
        s = d.spaces[i]
        _set4(s.point, _f4(s.point) + rng.normal(0, 0.05, 4).astype(np.float32))
        _set4(s.norm, _unit(_f4(s.norm) + rng.normal(0, 0.05, 4)))
    for i in range(d.n_spheres):
        s = d.spheres[i]
        _set4(s.center, _f4(s.center) + rng.normal(0, 0.3, 4).astype(np.float32))
        s.r = float(np.float32(s.r * rng.uniform(0.5, 1.5)))
    for i in range(d.n_cylinders):
        _perturb_cylinder(d.cylinders[i], rng, _rotation(rng, 0.2), rng.normal(0, 0.2, 4), rng.uniform(0.7, 1.3))
    for i in range(d.n_unions):
        u = d.unions[i]
        rot, shift = _rotation(rng, 0.2), rng.normal(0, 0.2, 4)
        for c in (u.cylinder1, u.cylinder2):
            _perturb_cylinder(c, rng, rot, shift, rng.uniform(0.8, 1.2))
    for i in range(d.n_tigers):
        t = d.tigers[i]
        rot, shift = _rotation(rng, 0.2), rng.normal(0, 0.2, 4)
        for c in (t.inner_cyl1, t.outer_cyl1, t.inner_cyl2, t.outer_cyl2):
            _perturb_cylinder(c, rng, rot, shift, rng.uniform(0.8, 1.2))
        if seed % 3 == 0:  # break init_tiger's shared point: the kernel must fall back to the generic tiger
            _set4(t.inner_cyl2.point, _f4(t.inner_cyl2.point) + np.float32(1e-3))
    for i in range(d.n_hypercubes):
        h = d.hypercubes[i]
        shift = rng.normal(0, 0.2, 4).astype(np.float32)
        for c in h.cubes:
            _set4(c.point, _f4(c.point) + shift)
            c.r = float(np.float32(c.r * rng.uniform(0.9, 1.1)))
    _set4(d.sun.drct, _unit(_f4(d.sun.drct) + rng.normal(0, 0.2, 4)))
    return rt4.Scene(d)


CASES = [(n, s) for n in ("all_primitives", "tiger_two_mirrors", "sphere", "room", "cylinder4d", "hypercube", "tiger")
         for s in range(1, 7)]


@pytest.mark.parametrize("name,seed", CASES)
def test_random_scene_find_intersection(rt4, oracle, name, seed):
    scene = perturb(rt4, name, seed)
    rays = random_rays(20000, 7000 + seed)
    c, cc = oracle.find_intersection(scene.desc, rays)
    for flags in (0, rt4.FLAG_GENERIC_KERNEL):
        t = rt4.Tracer(device=0, scene=scene, flags=flags)
        try:
            g, gc = t.debug_find_intersection(rays)
        finally:
            t.close()
        assert_bits(g, c, f"{name}/{seed} find_intersection flags={flags}")
        assert_bits(gc, cc, f"{name}/{seed} material color flags={flags}")


@pytest.mark.parametrize("name,seed", CASES)
def test_random_scene_render(rt4, oracle, name, seed):
    scene = perturb(rt4, name, seed)
    u = rt4.make_uniforms(64, 40, samples=3, reflections=4, seed=100 + seed)
    rng = np.random.default_rng(seed)
    u.focus[0] += float(np.float32(rng.normal(0, 0.2)))
    u.focus[3] += float(np.float32(rng.normal(0, 0.2)))
    reg = rt4.region(64, 40)
    fg, ng, fc, nc = render_both(rt4, oracle, scene, u, reg, flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert_bits(fg, fc, f"{name}/{seed} image")


@pytest.mark.parametrize("name", ["hypercube", "all_primitives"])
def test_nonfinite_and_huge_rays(rt4, oracle, name):
    """Rays with inf / NaN / |x| >= 1e30 components, one per 16 lanes: the hypercube's axis-aligned
    cull (rt4_fast.h) must fall back to the full dot products for the whole wave."""
    scene = rt4.Scene.named(name)
    rays = random_rays(20000, 99)
    rng = np.random.default_rng(3)
    bad = np.arange(0, len(rays), 16)
    vals = np.array([np.inf, -np.inf, np.nan, 1e30, -3e35, 1e-40], np.float32)
    rays[bad, rng.integers(0, 8, len(bad))] = vals[rng.integers(0, len(vals), len(bad))]
    rays[5000:5064, 4:8] = np.array([0.0, 0.0, 0.0, 1.0], np.float32)  # parallel to 6 of the 8 cells
    rays[6000:6064, 0:4] = np.array([1e20, 2.0, 0.0, 0.0], np.float32)
    c, cc = oracle.find_intersection(scene.desc, rays)
    t = rt4.Tracer(device=0, scene=scene)
    try:
        g, gc = t.debug_find_intersection(rays)
    finally:
        t.close()
    assert_bits(g, c, f"{name} non-finite rays")
    assert_bits(gc, cc, f"{name} non-finite rays colour")


SPECIAL_RADII = [float("nan"), 0.0, -0.5, 1e-20, 2e-4, 1e20, float("inf"), 3e-4]


@pytest.mark.parametrize("name", ["sphere", "tiger", "cylinder4d", "all_primitives"])
@pytest.mark.parametrize("radius", SPECIAL_RADII)
def test_special_radii(rt4, oracle, name, radius):
    """Spheres, union and tiger cylinders with NaN, zero, negative, tiny, SMALL-sized, huge and infinite
    radii: the sphere cull and the bounding-ball skips (rt4_aux.h SphereCull, BoundBall) must
    report exactly what the exact path reports, NaN-distance hits included."""
    d = rt4.SceneDesc.from_buffer_copy(rt4.Scene.named(name).to_bytes())
    if d.n_spheres:
        d.spheres[0].r = radius
    for i in range(d.n_unions):
        d.unions[i].cylinder1.r = radius
    for i in range(d.n_tigers):
        t = d.tigers[i]
        t.inner_cyl1.r = radius  # the inner radius of the first axes pair; the other three stay
        t.outer_cyl2.r = radius if radius != radius else t.outer_cyl2.r
    scene = rt4.Scene(d)
    rays = random_rays(20000, 4242)
    c, cc = oracle.find_intersection(scene.desc, rays)
    for flags in (0, rt4.FLAG_GENERIC_KERNEL):
        t = rt4.Tracer(device=0, scene=scene, flags=flags)
        try:
            g, gc = t.debug_find_intersection(rays)
        finally:
            t.close()
        assert_bits(g, c, f"{name} r={radius} find_intersection flags={flags}")
        assert_bits(gc, cc, f"{name} r={radius} colour flags={flags}")


@pytest.mark.parametrize("radius", SPECIAL_RADII)
def test_special_cube_radii(rt4, oracle, radius):
    """Hypercube cells with special half-sizes: the bounding-ball skip of the faces (rt4_aux.h
    hyper_bound) and the pending-cell pass must agree with the exact first-hit-in-order test."""
    d = rt4.SceneDesc.from_buffer_copy(rt4.Scene.named("hypercube").to_bytes())
    for k in (0, 3, 6):
        d.hypercubes[0].cubes[k].r = radius
    scene = rt4.Scene(d)
    rays = random_rays(20000, 515)
    c, cc = oracle.find_intersection(scene.desc, rays)
    for flags in (0, rt4.FLAG_GENERIC_KERNEL):
        t = rt4.Tracer(device=0, scene=scene, flags=flags)
        try:
            g, gc = t.debug_find_intersection(rays)
        finally:
            t.close()
        assert_bits(g, c, f"hypercube r={radius} flags={flags}")
        assert_bits(gc, cc, f"hypercube r={radius} colour flags={flags}")


@pytest.mark.parametrize("ang", [float("nan"), 0.0, -0.1, 1e-30, 1.0, 1.5, 3.2, 100.0, float("inf")])
def test_special_sun_sizes(rt4, oracle, ang):
    """Sun angular sizes outside the usual range (NaN, 0, negative, tiny, above 1 and pi, inf): the
    verified sky threshold, the sky pre-test and the sun division (rt4_aux.h sky_c_star, sky_pre_k,
    sun_ang) must keep final_light exact. A 64x40 render, 3 spp, 3 bounces."""
    d = rt4.SceneDesc.from_buffer_copy(rt4.Scene.named("sphere").to_bytes())
    d.sun.angular_size = ang
    u = rt4.make_uniforms(64, 40, samples=3, reflections=3, seed=8)
    reg = rt4.region(64, 40)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene(d), u, reg, flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert_bits(fg, fc, f"sun angular size {ang}")


@pytest.mark.parametrize("drct", [(0.0, 0.0, 0.0, 0.0), (float("nan"), 0.0, 1.0, 0.0), (1e30, 0.0, 1e30, 0.0),
                                  (1e-30, 0.0, 0.0, 0.0), (0.0, -1.0, 0.0, 0.0), (float("inf"), 1.0, 0.0, 0.0)])
def test_special_sun_directions(rt4, oracle, drct):
    """Degenerate sun directions (zero, NaN, huge, tiny, straight down, inf): length(sun.drct) is a
    verified scene divisor (rt4_aux.h sun_len) and scales the sky pre-test constant."""
    d = rt4.SceneDesc.from_buffer_copy(rt4.Scene.named("sphere").to_bytes())
    for i in range(4):
        d.sun.drct[i] = drct[i]
    u = rt4.make_uniforms(64, 40, samples=3, reflections=3, seed=9)
    reg = rt4.region(64, 40)
    fg, ng, fc, nc = render_both(rt4, oracle, rt4.Scene(d), u, reg, flags=rt4.FLAG_SAMPLER_LUT)
    assert ng == nc
    assert_bits(fg, fc, f"sun direction {drct}")
