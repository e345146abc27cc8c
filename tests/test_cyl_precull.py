"""The cylinders' pre-normalisation cull (rt4_fast.h cyl_cand_precull, derivation in rt4_aux.h SphereCull) implies
the post-normalisation cull, whose "no hit" the sphere cull's own bound guarantees. Checked here on the kernel's
fp32 op sequence (RN per op; fma emulated in float64, exact for the product) over rays whose projected line passes
just outside the cylinder radius, where the two margins are thinnest: every ray the pre-cull skips must satisfy
the post-normalisation test (or point away)."""
import numpy as np

f32 = np.float32
K = f32(4e-6)          # rt4_aux.h SPHERE_CULL_K
K2 = f32(8e-6)         # rt4_aux.h CYL_PRECULL_K


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def dot(a, b):  # rt4_device_math.h dot: fma(w, fma(z, fma(y, x*x)))
    return fma(a[..., 3], b[..., 3], fma(a[..., 2], b[..., 2], fma(a[..., 1], b[..., 1], (a[..., 0] * b[..., 0]).astype(f32))))


def point_in_space(p, sp, sn):  # mad(sn, dot(sp - p, sn), p)
    t = dot((sp - p).astype(f32), sn)
    return fma(sn, t[..., None], p)


def vec_in_space(v, sn):  # mad(sn, -dot(v, sn), v)
    t = -dot(v, sn)
    return fma(sn, t[..., None], v)


def constants(r):  # rt4_trace.hip cull_of (d2_out only needs to be a lower bound on "outside" here)
    r2m = f32(np.float64(r) * r * (1.0 + 1e-4))
    r2m_pre = np.nextafter(f32(np.float64(r2m) * (1.0 + 1e-6)), f32(np.inf))
    return f32(max(r, 0.0003) ** 2), r2m, r2m_pre


def test_precull_implies_post_cull():
    rng = np.random.default_rng(20260518)
    checked = culled = 0
    for trial in range(40):
        # a cylinder: point cp, orthonormal axes a1, a2; b1, b2 complete the basis (the circle's plane)
        q, _ = np.linalg.qr(rng.normal(size=(4, 4)))
        a1, a2, b1, b2 = (q[:, i].astype(f32) for i in range(4))
        cp = rng.uniform(-8, 8, 4).astype(f32)
        r = f32(rng.uniform(0.05, 3.0))
        d2_out, r2m, r2m_pre = constants(r)
        n = 50000
        # projected line at distance rho = r (1 + t) from the axis plane, t from 1e-7 to 1e-2 (log-uniform)
        t = 10.0 ** rng.uniform(-7, -2, n)
        rho = r * (1.0 + t)
        y0 = rng.uniform(-6 * r, 6 * r, n)
        al, be = rng.uniform(-5, 5, (2, n))
        p = (cp[None] + rho[:, None] * b1 + y0[:, None] * b2 + al[:, None] * a1 + be[:, None] * a2).astype(f32)
        phi = rng.uniform(-np.pi, np.pi, n)
        inplane = np.cos(phi)[:, None] * (-np.sign(y0))[:, None] * b2  # toward the circle (dp >= 0 mostly)
        outplane = np.sin(phi)[:, None] * (rng.normal(size=(n, 1)) * a1 + rng.normal(size=(n, 1)) * a2)
        d = inplane + outplane
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(f32)
        # kernel op sequence (rt4_fast.h cyl_cand_precull)
        r1p = point_in_space(p, cp[None], a1[None])
        r1d = vec_in_space(d, a1[None])
        p12 = point_in_space(r1p, cp[None], a2[None])
        e = vec_in_space(r1d, a2[None])
        po = (cp[None] - p12).astype(f32)
        dd = dot(po, po)
        L = dot(e, e)
        Q = dot(po, e)
        lhs = ((dd * L).astype(f32) - (Q * Q).astype(f32)).astype(f32)
        rhs = (fma(np.full(n, K2), dd, np.full(n, r2m_pre)) * L).astype(f32)
        pre = (dd >= d2_out) & (dd < 1e18) & (L > 1e-30) & (L < 1e18) & (lhs > rhs)
        # post-normalisation cull on the same ray (cyl_project, then sphere_culled)
        ln = np.sqrt(L).astype(f32)
        ok = ln >= f32(1e-4)
        dn = (e / ln[:, None]).astype(f32)
        dp = dot(po, dn)
        post = (dd >= d2_out) & ((dp < 0) | (((dd - (dp * dp).astype(f32)).astype(f32)) > fma(np.full(n, K), dd, np.full(n, r2m))))
        bad = pre & ok & ~post
        assert not bad.any(), (trial, int(bad.sum()), float(t[bad][0]), float(r))
        checked += n
        culled += int(pre.sum())
    # the sample reaches the thin margin: a real share of it is culled, the rest is left to the exact test
    assert 0.05 * checked < culled < 0.95 * checked
