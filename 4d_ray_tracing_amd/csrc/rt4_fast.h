// rt4_fast.h — the specialised find_intersection (shader.frag:434-451) for scenes in canonical form.
//
// Same results as rt4_intersect.h bit for bit; less work, by structure only:
//   * candidates carry {hit, flip, dist, sdist, id}; the normal and the material are computed once,
//     for the winning candidate (resolve()), instead of for every primitive hit along the way;
//   * divisions by scene constants use DivC (rt4_aux.h), verified exhaustively per divisor;
//   * dist_to_axes_plane(..) > r / < r compare the squared length with exact thresholds (no sqrt);
//   * tiger: projection / sphere-core / axes-distance shared inside each axes pair (init_tiger).
#pragma once

#include "rt4_aux.h"
#include "rt4_intersect.h"

#ifndef RT4_SPHERE_CULL
#define RT4_SPHERE_CULL 1
#endif
#ifndef RT4_HYPER_AXIS_TIGER
#define RT4_HYPER_AXIS_TIGER 1  // the axis form in the tiger kernels too: r05-v48, config 5 +4.3 % (r05_ab.txt); it
                                // measured 4.5 % slower before r05-v45's register savings
#endif
#ifndef RT4_HYPER_AXIS
#define RT4_HYPER_AXIS 1  // hypercube cull: one-component form for axis-aligned canonical cells (rt4_aux.h
                          // hyper_axis)
#endif
#ifndef RT4_HYPER_PENDING
#define RT4_HYPER_PENDING 1  // hypercube: per-lane pending-cell loop (hypercube_cand) instead of 8 cells in order
#endif
constexpr int HYPER_CELLS_LDS = 8 * 6;  // float4s of hypercube 0's cells staged ahead of the primitive table
#ifndef RT4_BOUND_SKIP
#define RT4_BOUND_SKIP 1  // bounding-ball skips for tiger / union / hypercube faces (rt4_aux.h BoundBall)
#endif

namespace rt4 {

#ifdef RT4_LANESTATS
__device__ unsigned long long* rt4_ls_counter;  // diagnostic build only: the launch's counter buffer
#endif

// x / b with the verified 3-op form when allowed (uniform branch: c.fast is a scene constant).
__device__ __forceinline__ float div_c(float x, const DivC& c) {
  if (c.fast) {
    const float q = x * c.y;
    const float r = fmaf_(-q, c.b, x);
    const float q2 = fmaf_(r, c.y, q);
    return (r == 0.0f || !__builtin_isfinite(q)) ? q : q2;
  }
  return x / c.b;
}
__device__ __forceinline__ V4 divs_c(V4 a, const DivC& c) {
  return V4{div_c(a.x, c), div_c(a.y, c), div_c(a.z, c), div_c(a.w, c)};
}

struct Cand {
  bool hit;
  bool flip;    // sphere-like: normal negated (outer && len_po > r); space: sign(dot_vn) < 0
  float dist;   // distance along the ray (what closest() compares)
  float sdist;  // cylinder-like: distance inside the projected 2-plane (before /= len)
  uint32_t id;  // flat primitive index into SceneAux::prims (rt4_aux.h)
};

__device__ __forceinline__ Cand no_cand() { return Cand{false, false, 0.0f, 0.0f, 0u}; }

__device__ __forceinline__ Cand closest(const Cand& a, const Cand& b) {  // shader.frag:181-185
  const bool ta = a.hit && (!b.hit || a.dist < b.dist);
  return Cand{ta ? a.hit : b.hit, ta ? a.flip : b.flip, ta ? a.dist : b.dist, ta ? a.sdist : b.sdist,
              ta ? a.id : b.id};
}

// sphere_intersection without the normal (shader.frag:197-217). The early returns matter on a GPU:
// when no lane of the wave needs the rest, the wave skips it (s_cbranch_execz).
__device__ __forceinline__ Cand sphere_cand(V4 center, float r, const DivC& dc, const Ray& ray, bool outer,
                                            uint32_t id) {
  V4 vec_po = sub(center, ray.point);
  const float len_po = length(vec_po);
  float cos_opa = 0.0f;
  if (!(len_po < SMALL_F)) {
    const float dot_pord = dot(vec_po, ray.drct);
    if (len_po >= r && dot_pord < 0.0f) return no_cand();
    cos_opa = rdiv(dot_pord, len_po);
    cos_opa = cos_opa > 1.0f ? 1.0f : cos_opa;
    cos_opa = cos_opa < -1.0f ? -1.0f : cos_opa;
  }
  const float angle_opa = acos_(cos_opa);
  const float sin_oap = div_c(len_po * sin_(angle_opa), dc);
  if (sin_oap >= 1.0f) return no_cand();
  float angle_oap = asin_(sin_oap);
  const bool flip = outer && len_po > r;
  if (flip) angle_oap = PI_F - angle_oap;
  const float angle_aop = PI_F - angle_opa - angle_oap;
  const float dist = sqrt_(r * r + len_po * len_po - 2.0f * r * len_po * cos_(angle_aop));
  return Cand{true, flip, dist, dist, id};
}

// sphere_cand from d2 = dot(vec_po, vec_po) and dp = dot(vec_po, ray.drct), already evaluated by the
// cull pass (find_pre) with the same operands and the same op sequence, so the same bits: the exact
// test then needs neither the centre nor the two dots again.
__device__ __forceinline__ Cand sphere_cand_d(float d2, float dp, float r, const DivC& dc, bool outer, uint32_t id) {
  const float len_po = sqrt_(d2);
  float cos_opa = 0.0f;
  if (!(len_po < SMALL_F)) {
    if (len_po >= r && dp < 0.0f) return no_cand();
    cos_opa = rdiv(dp, len_po);
    cos_opa = cos_opa > 1.0f ? 1.0f : cos_opa;
    cos_opa = cos_opa < -1.0f ? -1.0f : cos_opa;
  }
  const float angle_opa = acos_(cos_opa);
  const float sin_oap = div_c(len_po * sin_(angle_opa), dc);
  if (sin_oap >= 1.0f) return no_cand();
  float angle_oap = asin_(sin_oap);
  const bool flip = outer && len_po > r;
  if (flip) angle_oap = PI_F - angle_oap;
  const float angle_aop = PI_F - angle_opa - angle_oap;
  const float dist = sqrt_(r * r + len_po * len_po - 2.0f * r * len_po * cos_(angle_aop));
  return Cand{true, flip, dist, dist, id};
}

// Sphere-core shared by the outer=true/false variants of one cylinder face pair.
struct SphereCore2 {
  bool miss;
  float len_po, angle_opa, angle_oap;
};
// The cores of the two radii of one tiger axes pair (inner and outer cylinder: same centre, same
// projected ray): vec_po, len_po, cos_opa, acos(cos_opa) and its sine do not depend on r, so they are
// evaluated once; each radius keeps its own early-out, its sin_oap (div_c by r) and its asin. The same
// ops on the same operands as two separate cores, so the same bits.
__device__ __forceinline__ void sphere_core_pair(V4 center, float r0, const DivC& dc0, float r1, const DivC& dc1,
                                                 const Ray& ray, SphereCore2& c0, SphereCore2& c1) {
  const V4 vec_po = sub(center, ray.point);
  const float len_po = length(vec_po);
  float cos_opa = 0.0f;
  bool away = false;
  if (!(len_po < SMALL_F)) {
    const float dot_pord = dot(vec_po, ray.drct);
    away = dot_pord < 0.0f;
    cos_opa = rdiv(dot_pord, len_po);
    cos_opa = cos_opa > 1.0f ? 1.0f : cos_opa;
    cos_opa = cos_opa < -1.0f ? -1.0f : cos_opa;
  }
  c0 = SphereCore2{away && len_po >= r0, len_po, 0.0f, 0.0f};
  c1 = SphereCore2{away && len_po >= r1, len_po, 0.0f, 0.0f};
  if (c0.miss && c1.miss) return;
  const float angle_opa = acos_(cos_opa);
  const float ls = len_po * sin_(angle_opa);
  if (!c0.miss) {
    c0.angle_opa = angle_opa;
    const float sin_oap = div_c(ls, dc0);
    c0.miss = sin_oap >= 1.0f;
    if (!c0.miss) c0.angle_oap = asin_(sin_oap);
  }
  if (!c1.miss) {
    c1.angle_opa = angle_opa;
    const float sin_oap = div_c(ls, dc1);
    c1.miss = sin_oap >= 1.0f;
    if (!c1.miss) c1.angle_oap = asin_(sin_oap);
  }
}
__device__ __forceinline__ void sphere_dist2(const SphereCore2& c, float r, float& d_outer, bool& flip_outer,
                                             float& d_inner) {
  // outer = true
  flip_outer = c.len_po > r;
  {
    const float oap = flip_outer ? PI_F - c.angle_oap : c.angle_oap;
    const float aop = PI_F - c.angle_opa - oap;
    d_outer = sqrt_(r * r + c.len_po * c.len_po - 2.0f * r * c.len_po * cos_(aop));
  }
  if (flip_outer) {  // outer = false never flips
    const float aop = PI_F - c.angle_opa - c.angle_oap;
    d_inner = sqrt_(r * r + c.len_po * c.len_po - 2.0f * r * c.len_po * cos_(aop));
  } else {
    d_inner = d_outer;  // identical op sequence when no flip
  }
}

#ifndef RT4_SPACE_SIGN_DOT
#define RT4_SPACE_SIGN_DOT 1  // space_cand: cos_dh = sgn * dot(norm, drct) (r06-v53, with RT4_BALL_BEHIND)
#endif
__device__ __forceinline__ Cand space_cand(const rt4_scene_desc* __restrict__ S, int i, const Ray& ray) {  // :231-239
  const rt4_space& s = S->spaces[i];
  const V4 sn = ld4(s.norm);
  const float dot_vn = dot(sub(ld4(s.point), ray.point), sn);
  const float sgn = dot_vn > 0.0f ? 1.0f : (dot_vn < 0.0f ? -1.0f : 0.0f);
#if RT4_SPACE_SIGN_DOT
  // dot(sn * sgn, d) as sgn * dot(sn, d) (round 6, A/B knob): for sgn = +-1 the fma chain of the negated vector is the
  // exact negation of the plain one (round-to-nearest-even is symmetric), except that an exact zero keeps +0 where the
  // negation gives -0; for sgn = 0 both are a zero (or the same NaN class from non-finite operands). A zero is below
  // SMALL_F either way, and a nonzero cos_dh is bit-identical, so the candidate is too: 3 VALU fewer per space.
  const float cos_dh = sgn * dot(sn, ray.drct);
#else
  const float cos_dh = dot(mul(sn, sgn), ray.drct);
#endif
  Cand c{true, sgn < 0.0f, 0.0f, 0.0f, static_cast<uint32_t>(i)};
  if (cos_dh < SMALL_F) return no_cand();
  c.dist = rdiv(__builtin_fabsf(dot_vn), cos_dh);
  return c;
}

// 2-axis cylinder candidate (shader.frag:251-267); p = the ray projected onto its 2-plane
__device__ __forceinline__ Cand cyl_cand(const CylProj& p, V4 cp, float r, const DivC& dc, bool outer, uint32_t id) {
  if (p.miss) return no_cand();
  Cand c = sphere_cand(cp, r, dc, p.r12, outer, id);
  c.dist = c.dist / p.len;  // inter.dist /= drct_in_plane_length (:265)
  return c;
}

// cyl_cand with the sphere cull (rt4_aux.h SphereCull) on the projected ray: a lane whose projected line clears
// the circle skips the transcendental part; the exact part reuses the cull's two dots (sphere_cand_d: the same
// ops on the same operands as sphere_cand), so the result is cyl_cand's, bit for bit.
__device__ __forceinline__ bool sphere_culled(float d2, float dp, float d2_out, float r2m) {
  return d2 >= d2_out && (dp < 0.0f || d2 - dp * dp > fmaf_(SPHERE_CULL_K, d2, r2m));
}
__device__ __forceinline__ Cand cyl_cand_cull(const CylProj& p, V4 cp, float r, const DivC& dc, const SphereCull& k,
                                              bool outer, uint32_t id) {
  if (p.miss) return no_cand();
  const V4 po = sub(cp, p.r12.point);
  const float d2 = dot(po, po), dp = dot(po, p.r12.drct);
  if (sphere_culled(d2, dp, k.d2_out, k.r2m)) return no_cand();
  Cand c = sphere_cand_d(d2, dp, r, dc, outer, id);
  c.dist = c.dist / p.len;  // inter.dist /= drct_in_plane_length (:265)
  return c;
}
// cyl_project + cyl_cand_cull with the cull tested first on the unnormalised projected direction (rt4_aux.h
// SphereCull, pre-normalisation form): a culled lane skips the two lengths and four divisions too. The lanes it
// does not cull take cyl_project's remaining steps and cyl_cand_cull's test and exact part, the same ops on the
// same operands, so the result is cyl_cand's, bit for bit.
__device__ __forceinline__ Cand cyl_cand_precull(V4 cp, V4 a1, V4 a2, const Ray& ray, float r, const DivC& dc,
                                                 const SphereCull& k, bool outer, uint32_t id) {
  const V4 r1p = point_in_space(ray.point, cp, a1), r1d = vec_in_space(ray.drct, a1);
  const V4 p12 = point_in_space(r1p, cp, a2), e = vec_in_space(r1d, a2);
  const V4 po = sub(cp, p12);
  const float d2 = dot(po, po);
  const float L = dot(e, e);
  {
    const float Q = dot(po, e);
    if (d2 >= k.d2_out && d2 < 1e18f && L > 1e-30f && L < 1e18f &&
        d2 * L - Q * Q > fmaf_(CYL_PRECULL_K, d2, k.r2m_pre) * L)
      return no_cand();
  }
  // cyl_project (rt4_intersect.h): miss on a short in-plane direction, then the normalisation
  if (length(r1d) < SMALL_F) return no_cand();
  const float len = sqrt_(L);  // length(e)
  if (len < SMALL_F) return no_cand();
  const V4 dn = divs(e, len);
  const float dp = dot(po, dn);
  if (sphere_culled(d2, dp, k.d2_out, k.r2m)) return no_cand();
  Cand c = sphere_cand_d(d2, dp, r, dc, outer, id);
  c.dist = c.dist / len;  // inter.dist /= drct_in_plane_length (:265)
  return c;
}
#ifndef RT4_CYL_CULL
#define RT4_CYL_CULL 1  // the sphere cull for the cylinders and the union's cylinders: 1 after the projection's
                        // normalisation, 2 also before it (config 5 -0.4 %: few waves cull every lane, and the
                        // extra test costs more than the divisions it skips; profiles/r05_ab.txt)
#endif
#ifndef RT4_TIGER_CULL
#define RT4_TIGER_CULL 0  // the sphere cull for the tiger's axes pairs and split quarters: config 4 -1.3 %, config 5
                          // +-0 (r05_ab.txt), off
#endif

// dist_to_axes_plane(..)^2 without the sqrt (shader.frag:270-275)
__device__ __forceinline__ float axes_dist_sq(float dist, const Ray& ray, V4 cp, V4 a1, V4 a2) {
  const V4 p = mad(ray.drct, dist, ray.point);
  const V4 p1 = point_in_space(p, cp, a1);
  const V4 p12 = point_in_space(p1, cp, a2);
  const V4 v = sub(cp, p12);
  return dot(v, v);
}

__device__ __forceinline__ Cand union_cand(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                           int i, uint32_t base, const Ray& ray) {  // :284-294
  const rt4_cylinders_union& u = S->unions[i];
  const V4 p1 = ld4(u.cylinder1.point), a11 = ld4(u.cylinder1.axis1), a12 = ld4(u.cylinder1.axis2);
  const V4 p2 = ld4(u.cylinder2.point), a21 = ld4(u.cylinder2.axis1), a22 = ld4(u.cylinder2.axis2);
  const float gt = X->union_gt[i];
#if RT4_CYL_CULL == 2
  Cand c1 = cyl_cand_precull(p1, a11, a12, ray, u.cylinder1.r, X->union_r[i][0], X->union_cull[i][0], true, base);
#elif RT4_CYL_CULL
  Cand c1 = cyl_cand_cull(cyl_project(p1, a11, a12, ray), p1, u.cylinder1.r, X->union_r[i][0], X->union_cull[i][0], true,
                          base);
#else
  Cand c1 = cyl_cand(cyl_project(p1, a11, a12, ray), p1, u.cylinder1.r, X->union_r[i][0], true, base);
#endif
  if (c1.hit && axes_dist_sq(c1.dist, ray, p2, a21, a22) > gt) c1.hit = false;
#if RT4_CYL_CULL == 2
  Cand c2 = cyl_cand_precull(p2, a21, a22, ray, u.cylinder2.r, X->union_r[i][1], X->union_cull[i][1], true, base + 1);
#elif RT4_CYL_CULL
  Cand c2 = cyl_cand_cull(cyl_project(p2, a21, a22, ray), p2, u.cylinder2.r, X->union_r[i][1], X->union_cull[i][1], true,
                          base + 1);
#else
  Cand c2 = cyl_cand(cyl_project(p2, a21, a22, ray), p2, u.cylinder2.r, X->union_r[i][1], true, base + 1);
#endif
  if (c2.hit && axes_dist_sq(c2.dist, ray, p1, a11, a12) > gt) c2.hit = false;
  return closest(c1, c2);
}

// Four faces of one axes pair of a tiger: cylinders (cp, a1, a2) with radii r_in, r_out, each with
// outer = true/false, kept iff the other pair's axes distance d satisfies lt <= d^2 <= gt.
__device__ __forceinline__ Cand tiger_pair(V4 cp, V4 a1, V4 a2, float r_in, float r_out, const DivC& dc_in,
                                           const DivC& dc_out, V4 op, V4 oa1, V4 oa2, float gt, float lt,
                                           const Ray& ray, uint32_t id_base, const SphereCull& k_in,
                                           const SphereCull& k_out) {
  const CylProj p = cyl_project(cp, a1, a2, ray);
  if (p.miss) return no_cand();
#if RT4_TIGER_CULL
  {  // both radii miss (rt4_aux.h SphereCull): no face of this pair can hit
    const V4 po = sub(cp, p.r12.point);
    const float d2 = dot(po, po), dp = dot(po, p.r12.drct);
    if (sphere_culled(d2, dp, k_in.d2_out, k_in.r2m) && sphere_culled(d2, dp, k_out.d2_out, k_out.r2m)) return no_cand();
  }
#endif
  SphereCore2 c_in, c_out;
  sphere_core_pair(cp, r_in, dc_in, r_out, dc_out, p.r12, c_in, c_out);
  Cand res = no_cand();
  {
    const SphereCore2& c = c_in;
    if (!c.miss) {
      float d_o, d_i;
      bool f_o;
      sphere_dist2(c, r_in, d_o, f_o, d_i);
      Cand c_o{true, f_o, d_o / p.len, d_o, id_base};    // face x11 (outer = true)
      Cand c_i{true, false, d_i / p.len, d_i, id_base};  // face x12 (outer = false)
      float q = axes_dist_sq(c_o.dist, ray, op, oa1, oa2);
      if (q > gt || q < lt) c_o.hit = false;
      q = axes_dist_sq(c_i.dist, ray, op, oa1, oa2);
      if (q > gt || q < lt) c_i.hit = false;
      res = closest(c_o, c_i);
    }
  }
  {
    const SphereCore2& c = c_out;
    if (!c.miss) {
      float d_o, d_i;
      bool f_o;
      sphere_dist2(c, r_out, d_o, f_o, d_i);
      Cand c_o{true, f_o, d_o / p.len, d_o, id_base + 1};   // face x21
      Cand c_i{true, false, d_i / p.len, d_i, id_base + 1};  // face x22
      float q = axes_dist_sq(c_o.dist, ray, op, oa1, oa2);
      if (q > gt || q < lt) c_o.hit = false;
      q = axes_dist_sq(c_i.dist, ray, op, oa1, oa2);
      if (q > gt || q < lt) c_i.hit = false;
      res = closest(res, closest(c_o, c_i));
    }
  }
  return res;
}

__device__ __forceinline__ Cand tiger_cand(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                           int i, uint32_t base, const Ray& ray) {  // :327-341
  const rt4_tiger& t = S->tigers[i];
  const V4 pA = ld4(t.inner_cyl1.point), a1 = ld4(t.inner_cyl1.axis1), a2 = ld4(t.inner_cyl1.axis2);
  const V4 pB = ld4(t.inner_cyl2.point), a3 = ld4(t.inner_cyl2.axis1), a4 = ld4(t.inner_cyl2.axis2);
  const Cand lo = tiger_pair(pA, a1, a2, t.inner_cyl1.r, t.outer_cyl1.r, X->tiger_r[i][0], X->tiger_r[i][1], pB, a3,
                             a4, X->tiger_gt[i][0], X->tiger_lt[i][0], ray, base, X->tiger_cull[i][0], X->tiger_cull[i][1]);
  const Cand hi = tiger_pair(pB, a3, a4, t.inner_cyl2.r, t.outer_cyl2.r, X->tiger_r[i][2], X->tiger_r[i][3], pA, a1,
                             a2, X->tiger_gt[i][1], X->tiger_lt[i][1], ray, base + 2, X->tiger_cull[i][2],
                             X->tiger_cull[i][3]);
  return closest(lo, hi);
}

__device__ __forceinline__ V4 sel4(bool c, V4 a, V4 b) { return V4{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w}; }

// One quarter q = 2 * pair + radius (pair 0: inner_cyl1 / outer_cyl1, pair 1: inner_cyl2 / outer_cyl2; radius 0:
// inner, 1: outer) of tiger_cand, for the in-wave split of the tiger test (rt4_trace.hip TSPLIT): the pair's
// projection and the radius-independent part of its sphere core, then the radius's early-out, asin, two faces and
// their filters, the very ops tiger_pair runs for that radius. So
//   tiger_cand == closest(closest(q0, q1), closest(q2, q3))
// bit for bit (tiger_pair folds its radii the same way; closest(no_cand, x) == x, closest(x, no_cand) == x).
// q may differ from lane to lane: the pair's geometry and the radius are selected per lane from scalar loads.
__device__ __forceinline__ Cand tiger_quarter(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X, int i,
                                              uint32_t base, const Ray& ray, unsigned q) {
  const rt4_tiger& t = S->tigers[i];
  const bool pb = q >= 2u, outer = (q & 1u) != 0u;
  const V4 pA = ld4(t.inner_cyl1.point), a1 = ld4(t.inner_cyl1.axis1), a2 = ld4(t.inner_cyl1.axis2);
  const V4 pB = ld4(t.inner_cyl2.point), a3 = ld4(t.inner_cyl2.axis1), a4 = ld4(t.inner_cyl2.axis2);
  const V4 cp = sel4(pb, pB, pA), ax1 = sel4(pb, a3, a1), ax2 = sel4(pb, a4, a2);
  const V4 op = sel4(pb, pA, pB), oa1 = sel4(pb, a1, a3), oa2 = sel4(pb, a2, a4);
  const float r = pb ? (outer ? t.outer_cyl2.r : t.inner_cyl2.r) : (outer ? t.outer_cyl1.r : t.inner_cyl1.r);
  const DivC& d0 = X->tiger_r[i][0];
  const DivC& d1 = X->tiger_r[i][1];
  const DivC& d2 = X->tiger_r[i][2];
  const DivC& d3 = X->tiger_r[i][3];
  const DivC dc{pb ? (outer ? d3.b : d2.b) : (outer ? d1.b : d0.b), pb ? (outer ? d3.y : d2.y) : (outer ? d1.y : d0.y),
                pb ? (outer ? d3.fast : d2.fast) : (outer ? d1.fast : d0.fast), 0};
  const float gt = pb ? X->tiger_gt[i][1] : X->tiger_gt[i][0], lt = pb ? X->tiger_lt[i][1] : X->tiger_lt[i][0];
  const uint32_t id = base + (pb ? 2u : 0u) + (outer ? 1u : 0u);
  const CylProj p = cyl_project(cp, ax1, ax2, ray);
  if (p.miss) return no_cand();
#if RT4_TIGER_CULL
  {  // this radius misses (rt4_aux.h SphereCull)
    const SphereCull& k0 = X->tiger_cull[i][0];
    const SphereCull& k1 = X->tiger_cull[i][1];
    const SphereCull& k2 = X->tiger_cull[i][2];
    const SphereCull& k3 = X->tiger_cull[i][3];
    const float kd = pb ? (outer ? k3.d2_out : k2.d2_out) : (outer ? k1.d2_out : k0.d2_out);
    const float kr = pb ? (outer ? k3.r2m : k2.r2m) : (outer ? k1.r2m : k0.r2m);
    const V4 po = sub(cp, p.r12.point);
    if (sphere_culled(dot(po, po), dot(po, p.r12.drct), kd, kr)) return no_cand();
  }
#endif
  SphereCore2 c, c_same;
  sphere_core_pair(cp, r, dc, r, dc, p.r12, c, c_same);  // both cores of one radius: the pair's shared part + it
  if (c.miss) return no_cand();
  float d_o, d_i;
  bool f_o;
  sphere_dist2(c, r, d_o, f_o, d_i);
  Cand c_o{true, f_o, d_o / p.len, d_o, id};   // outer = true face
  Cand c_i{true, false, d_i / p.len, d_i, id};  // outer = false face
  float qd = axes_dist_sq(c_o.dist, ray, op, oa1, oa2);
  if (qd > gt || qd < lt) c_o.hit = false;
  qd = axes_dist_sq(c_i.dist, ray, op, oa1, oa2);
  if (qd > gt || qd < lt) c_i.hit = false;
  return closest(c_o, c_i);
}

// far: the ray's line clears the hypercube's ball (rt4_aux.h hyper_bound); l2 = |drct|^2
__device__ __forceinline__ Cand cube_cand(const rt4_cube& c, const Ray& ray, uint32_t id, bool far, float l2) {  // :352-366
  const V4 cpt = ld4(c.point), cn = ld4(c.norm);
  const V4 vec_n = neg(cn);
  const float h = dot(sub(cpt, ray.point), vec_n);
  const float cos_dn = dot(ray.drct, vec_n);
  if (h < 0.0f || cos_dn < 0.0f) return no_cand();
  if (far && cos_dn * cos_dn >= 1e-12f * l2) return no_cand();  // finite hit point, outside the ball
  const float dist = rdiv(h, cos_dn);
  const V4 vec_cp = sub(mad(ray.drct, dist, ray.point), cpt);
  if (__builtin_fabsf(dot(vec_cp, ld4(c.x))) > c.r || __builtin_fabsf(dot(vec_cp, ld4(c.y))) > c.r ||
      __builtin_fabsf(dot(vec_cp, ld4(c.z))) > c.r)
    return no_cand();
  return Cand{true, false, dist, 0.0f, id};
}

__device__ __forceinline__ Cand hypercube_cand_seq(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                                   int i, uint32_t base, const Ray& ray);

// cube_cand's exact test from a cell staged in LDS (rt4_aux.h hyper_cells): the same floats, the same ops
__device__ __forceinline__ bool cell_hit(const float4* cell, const Ray& ray, float& dist) {
  const float4 p4 = cell[0], n4 = cell[1], x4 = cell[2], y4 = cell[3], z4 = cell[4];
  const float r = cell[5].x;
  const V4 cpt{p4.x, p4.y, p4.z, p4.w};
  const V4 vec_n = neg(V4{n4.x, n4.y, n4.z, n4.w});
  const float h = dot(sub(cpt, ray.point), vec_n);
  const float cos_dn = dot(ray.drct, vec_n);
  dist = rdiv(h, cos_dn);
  const V4 vec_cp = sub(mad(ray.drct, dist, ray.point), cpt);
  return !(__builtin_fabsf(dot(vec_cp, V4{x4.x, x4.y, x4.z, x4.w})) > r ||
           __builtin_fabsf(dot(vec_cp, V4{y4.x, y4.y, y4.z, y4.w})) > r ||
           __builtin_fabsf(dot(vec_cp, V4{z4.x, z4.y, z4.z, z4.w})) > r);
}

// hypercube_intersection (shader.frag:394-400) as two passes: every cell's cheap rejection
// (h < 0 || cos_dn < 0, the far-face skip) for all lanes, then each lane's remaining candidate cells
// in cell order until the first hit, read from LDS. Same first-hit-in-order result; a wave pays for
// max-over-lanes(candidates tried) exact tests instead of all 8 cells.
template <bool PENDING, bool AXIS>
__device__ __forceinline__ Cand hypercube_cand(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                               const float4* cells, int i, uint32_t base, const Ray& ray) {
  if constexpr (PENDING) {
    const rt4_hypercube& hc = S->hypercubes[i];
    float l2 = 0.0f;
    bool far = false;
#if RT4_BOUND_SKIP
    {
      const f16v k = *reinterpret_cast<const f16v*>(&X->hyper_bound[i]);
      const V4 pc = sub(V4{k[0], k[1], k[2], k[3]}, ray.point);
      const float a = dot(pc, pc), b = dot(pc, ray.drct);
      l2 = dot(ray.drct, ray.drct);
      far = a < 1e30f && l2 > 1e-30f && l2 < 1e30f && (a - fmaf_(4e-6f, a, k[12])) * l2 > b * b;
    }
#endif
    // Axis-aligned canonical cells (rt4_aux.h hyper_axis) and a finite ray in every lane: vec_n is
    // -+e_(k&3), so h = dot(cpt - p, vec_n) and cos_dn = dot(d, vec_n) are exactly -+(one component)
    // (the other products are +-0, which leave a nonzero sum unchanged); only the sign of a zero
    // result can differ, and the tests below do not see it (cos_dn enters squared).
    bool axis = false;
    if constexpr (AXIS)
      axis = X->hyper_axis[i] != 0 &&
             !__any(!(__builtin_fabsf(ray.point.x) < 1e30f && __builtin_fabsf(ray.point.y) < 1e30f &&
                      __builtin_fabsf(ray.point.z) < 1e30f && __builtin_fabsf(ray.point.w) < 1e30f &&
                      __builtin_fabsf(ray.drct.x) < 1e30f && __builtin_fabsf(ray.drct.y) < 1e30f &&
                      __builtin_fabsf(ray.drct.z) < 1e30f && __builtin_fabsf(ray.drct.w) < 1e30f));
    uint32_t cand = 0;
    if (axis) {
      const float pc[4] = {ray.point.x, ray.point.y, ray.point.z, ray.point.w};
      const float dc[4] = {ray.drct.x, ray.drct.y, ray.drct.z, ray.drct.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const float d = hc.cubes[k].point[k & 3] - pc[k & 3];
        const float h = k < 4 ? -d : d;
        const float cos_dn = k < 4 ? -dc[k & 3] : dc[k & 3];
        const bool rejected = h < 0.0f || cos_dn < 0.0f || (far && cos_dn * cos_dn >= 1e-12f * l2);
        cand |= rejected ? 0u : (1u << k);
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const rt4_cube& c = hc.cubes[k];
        const V4 vec_n = neg(ld4(c.norm));
        const float h = dot(sub(ld4(c.point), ray.point), vec_n);
        const float cos_dn = dot(ray.drct, vec_n);
        const bool rejected = h < 0.0f || cos_dn < 0.0f || (far && cos_dn * cos_dn >= 1e-12f * l2);
        cand |= rejected ? 0u : (1u << k);
      }
    }
    Cand res = no_cand();
    while (cand) {
#ifdef RT4_LANESTATS  // diagnostic: pending-cell trips and their active lanes (counter[58], [59])
      {
        const unsigned long long ex = __builtin_amdgcn_read_exec();
        if (rt4_ls_counter && (threadIdx.x & 63u) == static_cast<unsigned>(__builtin_ctzll(ex))) {
          atomicAdd(rt4_ls_counter + 58, 1ull);
          atomicAdd(rt4_ls_counter + 59, static_cast<unsigned long long>(__popcll(ex)));
        }
      }
#endif
      const int k = __builtin_ctz(cand);
      cand &= cand - 1u;
      float dist;
      if (cell_hit(cells + 6 * k, ray, dist)) {
        res = Cand{true, false, dist, 0.0f, base + static_cast<uint32_t>(k)};
        cand = 0u;
      }
    }
    return res;
  } else {
    return hypercube_cand_seq(S, X, i, base, ray);
  }
}

__device__ __forceinline__ Cand hypercube_cand_seq(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                                   int i, uint32_t base, const Ray& ray) {  // :394-400
  const rt4_hypercube& hc = S->hypercubes[i];
  float l2 = 0.0f;
  bool far = false;
#if RT4_BOUND_SKIP
  {
    const f16v k = *reinterpret_cast<const f16v*>(&X->hyper_bound[i]);  // centre 0-3, r2m 12
    const V4 pc = sub(V4{k[0], k[1], k[2], k[3]}, ray.point);
    const float a = dot(pc, pc), b = dot(pc, ray.drct);
    l2 = dot(ray.drct, ray.drct);
    far = a < 1e30f && l2 > 1e-30f && l2 < 1e30f && (a - fmaf_(4e-6f, a, k[12])) * l2 > b * b;
  }
#endif
  Cand res = no_cand();
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (!res.hit) res = cube_cand(hc.cubes[k], ray, base + k, far, l2);
  }
  return res;
}

// SH = shape bits (low 8 bits, K_*) | (n_spaces+1) << 8 | (n_spheres+1) << 16 | (n_cylinders+1) << 24;
// a zero count field means "read the count from the scene" (runtime loop).
constexpr uint32_t sh_count(uint32_t sh, int field) { return (sh >> (8 * field)) & 0xFFu; }

// Primitive-table entries of a shape (rt4_aux.h SceneAux::prims): exact for exact-count shapes,
// MAX_PRIMS when a count is read at run time. Sizes the kernel's LDS copy of the table.
constexpr int n_prims_of(uint32_t sh) {
  const uint32_t k = sh & 0xFFu;
  if (sh_count(sh, 1) == 0 || sh_count(sh, 2) == 0 || sh_count(sh, 3) == 0) return MAX_PRIMS;
  const int n = static_cast<int>(sh_count(sh, 1) + sh_count(sh, 2) + sh_count(sh, 3)) - 3 + ((k & K_UNION) ? 2 : 0) +
                ((k & K_HYPERCUBE) ? 8 : 0) + ((k & K_TIGER) ? 4 : 0);
  return n > 0 ? n : 1;
}

// for (i < count) body(i): fully unrolled when the count field C is a compile-time count
template <uint32_t C, typename F>
__device__ __forceinline__ void for_count(int runtime_n, F&& body) {
  if constexpr (C != 0) {
#pragma unroll
    for (int i = 0; i < static_cast<int>(C) - 1; i++) body(i);
  } else {
    for (int i = 0; i < runtime_n; i++) body(i);
  }
}

// True when the ray's line stays clear of a bounding ball (rt4_aux.h BoundBall): the group's exact test
// would report no hit. One 32-B scalar load, three dots.
// RT4_BALL_BEHIND (round 6): also when the ball is behind the ray: the origin outside the inflated ball (a > R2m) and
// the centre not ahead (b <= 0). Every forward point p + t d (t >= 0) is then at squared distance a - 2 t b + t^2 l2
// >= a > R2m from the centre, and the exact tests report only forward hits (dist = sqrt(..) >= 0, t = s / |e| in the
// projected plane) inside the ball (the derivation in rt4_aux.h, which R2m's 1e-3 inflation covers); the NaN-distance
// hits of origins near a cylinder keep the exact path through the same band check. So the skip is exact too.
#ifndef RT4_BALL_BEHIND_MAX
#define RT4_BALL_BEHIND_MAX 1  // r06-v54: the behind test as max(b, 0) inside the line test (fits the mirror room's registers)
#endif
#ifndef RT4_BALL_BEHIND
#define RT4_BALL_BEHIND 2  // r06-v53: 1 (not the closed rooms; config 5 +1.5 %); r06-v54: 2, every kernel (config 4 +3.1 %)
#endif
// BEHIND: the kernel's shape takes the second test (RT4_BALL_BEHIND; not in the closed rooms' kernels, >= 3 spaces,
// where it spilled in the loop at their wave bound)
template <uint32_t SH>
constexpr bool ball_behind_of() {
  return RT4_BALL_BEHIND != 0 && (RT4_BALL_BEHIND == 2 || ((SH >> 8) & 0xFFu) < 4);
}
// LINE = false: only the occlusion test (the hypercube's ball: its parallel faces' +inf hits forbid the line skip)
template <bool BEHIND = false, bool OCC = false, bool LINE = true>
__device__ __forceinline__ bool far_from(const BoundBall& bb, const Ray& ray, const Cand* acc = nullptr) {
  const f16v k = *reinterpret_cast<const f16v*>(&bb);  // centre, a1, a2, r2m, band[0..2]
  const f16v m = *(reinterpret_cast<const f16v*>(&bb) + 1);  // band[3..7]
  const V4 pc = sub(V4{k[0], k[1], k[2], k[3]}, ray.point);
  const float a = dot(pc, pc), b = dot(pc, ray.drct), l2 = dot(ray.drct, ray.drct);
  const float u1 = dot(pc, V4{k[4], k[5], k[6], k[7]}), u2 = dot(pc, V4{k[8], k[9], k[10], k[11]});
  const float dB = fmaf_(u1, u1, u2 * u2), dA = a - dB;  // squared distances to plane B and plane A
  const bool near_surface = (dA >= k[13] && dA <= k[14]) || (dA >= k[15] && dA <= m[0]) ||
                            (dB >= m[1] && dB <= m[2]) || (dB >= m[3] && dB <= m[4]);
#if RT4_BALL_BEHIND_MAX
  // the same skip as one v_max: with b clamped at 0 the line test reads a (1 - 4e-6) > R2m when b <= 0, i.e. the origin
  // outside the inflated ball (a finite b: a, l2 < 1e30)
  if constexpr (BEHIND && !OCC && LINE) {
    const float bp = fmaxf(b, 0.0f);
    return !near_surface && a < 1e30f && l2 > 1e-30f && l2 < 1e30f && (a - fmaf_(4e-6f, a, k[12])) * l2 > bp * bp;
  }
#endif
  const bool behind = BEHIND && b <= 0.0f && a > k[12];
  if constexpr (!OCC && LINE)  // r06-v53's expression as it was (the same code in the kernels without the knob)
    return !near_surface && a < 1e30f && l2 > 1e-30f && l2 < 1e30f && ((a - fmaf_(4e-6f, a, k[12])) * l2 > b * b || behind);
  const bool in_range = a < 1e30f && l2 > 1e-30f && l2 < 1e30f;
  bool occ = false;
  if constexpr (OCC) {  // RT4_OCCLUDE_SKIP (below): the ball starts beyond acc's hit
    const float x = b - acc->dist * l2 - 5e-5f * (a + l2);
    occ = acc->hit && x > 0.0f && x * x > k[12] * l2;
  }
  return in_range && ((LINE && !near_surface && ((a - fmaf_(4e-6f, a, k[12])) * l2 > b * b || behind)) || occ);
}

// Hypercube skip behind a hit (round 6, RT4_HYPER_SKIP, A/B knob): the hypercube's finite hits lie on its cells, inside
// hyper_bound's inflated ball; its +inf (parallel face) and NaN hits never replace a hit with a finite distance. So when
// acc already holds such a hit and the ray's line clears the ball, or the ball is behind the ray (the max(b, 0) form),
// the hypercube cannot change acc and its test is skipped.
#ifndef RT4_HYPER_SKIP
#define RT4_HYPER_SKIP 0
#endif
__device__ __forceinline__ bool hyper_skip(const BoundBall& bb, const Ray& ray, const Cand& acc) {
  const f16v k = *reinterpret_cast<const f16v*>(&bb);
  const V4 pc = sub(V4{k[0], k[1], k[2], k[3]}, ray.point);
  const float a = dot(pc, pc), b = dot(pc, ray.drct), l2 = dot(ray.drct, ray.drct);
  const float bp = fmaxf(b, 0.0f);
  return acc.hit && acc.dist < 3.0e38f && a < 1e30f && l2 > 1e-30f && l2 < 1e30f &&
         (a - fmaf_(4e-6f, a, k[12])) * l2 > bp * bp;
}

// Occlusion skip (round 6, RT4_OCCLUDE_SKIP: 1 = tiger and union, 3 = also the hypercube): a group whose bounding ball
// starts beyond the closest hit so far cannot change it. Every hit the group's exact test reports lies in the inflated
// ball (rt4_aux.h BoundBall; the hypercube's finite hits lie on its cells' faces, inside hyper_bound), so its distance
// t satisfies t l2 >= b - sqrt(R2m l2) (b = (c - p).d, l2 = |d|^2), and closest() keeps acc for any t >= acc.dist
// (ties keep acc; NaN and +inf distances never replace a hit). The test skips when
//   x = b - acc.dist l2 - 5e-5 (a + l2) > 0  and  x^2 > R2m l2,
// where 5e-5 (a + l2) >= 1e-4 sqrt(a l2) covers the fp32 rounding of b, of the products and of the hit point itself
// (each ~1e-6 sqrt(a l2)). acc without a hit, or with a NaN or infinite distance, never skips.
#ifndef RT4_OCCLUDE_SKIP
#define RT4_OCCLUDE_SKIP 0
#endif
template <uint32_t SH>
constexpr bool occlude_of(int what) {  // what: 1 = tiger / union, 2 = hypercube; not in the closed rooms' kernels
  return (RT4_OCCLUDE_SKIP & what) != 0 && ((SH >> 8) & 0xFFu) < 4;
}
// Flat primitive-table index of each group's first entry (rt4_aux.h SceneAux::prims order): compile-time
// for exact-count shapes (the scene-shape check pins one union / hypercube / tiger), else read.
struct PrimBases {
  uint32_t sphere, cyl, uni, cube, tiger;
};
template <uint32_t SH>
__device__ __forceinline__ PrimBases prim_bases(const SceneAux* __restrict__ X) {
  constexpr uint32_t K = SH & 0xFFu;
  constexpr uint32_t NSP = sh_count(SH, 1), NSH = sh_count(SH, 2), NCY = sh_count(SH, 3);
  if constexpr (NSP != 0 && NSH != 0 && NCY != 0) {
    constexpr uint32_t sph = NSP - 1, cyl = sph + NSH - 1, uni = cyl + NCY - 1;
    constexpr uint32_t cube = uni + ((K & K_UNION) ? 2u : 0u), tiger = cube + ((K & K_HYPERCUBE) ? 8u : 0u);
    return PrimBases{sph, cyl, uni, cube, tiger};
  } else {
    return PrimBases{static_cast<uint32_t>(X->base_sphere), static_cast<uint32_t>(X->base_cyl),
                     static_cast<uint32_t>(X->base_union), static_cast<uint32_t>(X->base_cube),
                     static_cast<uint32_t>(X->base_tiger)};
  }
}

// find_cand in three parts, so that a kernel can pool the exact sphere tests of several waves between
// them (rt4_trace.hip, POOL): find_pre = the spaces and the sphere cull (pending-sphere bit mask),
// sphere_exact = one pending sphere's exact test, find_rest = the groups after the spheres.
// Exact-count sphere groups of up to GEO_MAX spheres keep the cull's two dots per sphere for the exact
// test (sphere_cand_d); RT4_SPHERE_GEO=0 recomputes them from the centre (A/B knob). Measured
// (profiles/r02_ab.txt): sphere scene (2 spheres) +0.7 %; all_primitives (3 spheres, 4 selects per
// trip, 6 live VGPRs) -0.3 %, so three or more spheres keep the recomputation.
#ifndef RT4_SPHERE_GEO
#define RT4_SPHERE_GEO 1
#endif
#ifndef RT4_CULL_MAX
#define RT4_CULL_MAX 0
#endif
constexpr int GEO_MAX = 2;
template <uint32_t SH>
constexpr int geo_spheres() {
  return (RT4_SPHERE_GEO && ((SH & 0xFFu) & K_SPHERES) && sh_count(SH, 2) != 0 && sh_count(SH, 2) - 1 <= GEO_MAX)
             ? static_cast<int>(sh_count(SH, 2)) - 1
             : 0;
}
struct SphereGeo {
  float d2[GEO_MAX], dp[GEO_MAX];
};

template <uint32_t SH>
__device__ __forceinline__ Cand find_pre(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                         const Ray& ray, uint32_t& pend, SphereGeo* geo = nullptr) {
  constexpr uint32_t K = SH & 0xFFu;
  constexpr uint32_t NSP = sh_count(SH, 1), NSH = sh_count(SH, 2);
  Cand inter = no_cand();
  pend = 0;
  if (K & K_SPACES) for_count<NSP>(S->n_spaces, [&](int i) { inter = closest(space_cand(S, i, ray), inter); });
  if (K & K_SPHERES) {
    // Pass 1 (every sphere, ~20 VALU): the exact early-out (outside and pointing away) plus a
    // conservative "clearly missed" test; only the remaining spheres are marked pending
    // (rt4_aux.h SphereCull for the error bound that makes the cull exact).
    for_count<NSH>(S->n_spheres, [&](int i) {
      const f8v k = *reinterpret_cast<const f8v*>(&X->sphere_cull[i]);  // one 32-B scalar load
      const V4 po = sub(V4{k[0], k[1], k[2], k[3]}, ray.point);
      const float d2 = dot(po, po);  // exactly the dot whose sqrt is len_po in sphere_cand
      const float dp = dot(po, ray.drct);
      if constexpr (geo_spheres<SH>() > 0) {
        if (geo) {
          geo->d2[i] = d2;
          geo->dp[i] = dp;
        }
      }
      const bool outside = d2 >= k[4];  // len_po >= max(r, SMALL)
#ifdef RT4_CULL_BITWISE  // A/B build only: the same predicate without short-circuit branches
      const bool skip = outside & ((dp < 0.0f) | (d2 - dp * dp > fmaf_(SPHERE_CULL_K, d2, k[5])));
#else
      bool skip;
      if constexpr (RT4_CULL_MAX && !(K & K_TIGER)) {
        // round 6 (A/B knob; not next to a tiger, where it spilled): dp clamped at 0 folds the "outside and pointing
        // away" early-out into the one test: for dp < 0 it reads d2 > fma(K, d2, r2m) > r^2 (1 + 1e-4), so len_po >= r
        // and the exact path's own early-out (:205) returns no hit; outside rays nearer the surface than that now run
        // the exact path, which returns the same no hit; inside rays are never culled (d2 < r^2 < the threshold); a NaN
        // dp stays NaN (a select, not max), so such rays are not culled, as before.
        (void)outside;
        const float bp = dp < 0.0f ? 0.0f : dp;
        skip = d2 - bp * bp > fmaf_(SPHERE_CULL_K, d2, k[5]);
      } else {
        skip = outside && (dp < 0.0f || d2 - dp * dp > fmaf_(SPHERE_CULL_K, d2, k[5]));
      }
#endif
      pend |= skip ? 0u : (1u << i);
    });
  }
  return inter;
}

// The exact test of pending sphere i from the cull's dots (geo_spheres<SH>() > 0): the per-lane sphere
// index selects its pair of dots with NSH - 1 selects; the primitive entry supplies r and its divisor.
template <uint32_t SH>
__device__ __forceinline__ Cand sphere_exact_geo(const SceneAux* __restrict__ X, const PrimEntry* P,
                                                 const SphereGeo& g, int i) {
  constexpr int N = geo_spheres<SH>();
  float d2 = g.d2[0], dp = g.dp[0];
#pragma unroll
  for (int k = 1; k < N; k++) {
    d2 = i == k ? g.d2[k] : d2;
    dp = i == k ? g.dp[k] : dp;
  }
  const uint32_t id = prim_bases<SH>(X).sphere + static_cast<uint32_t>(i);
  const PrimEntry& e = P[id];
  const DivC dc{e.r, e.y, e.fast, 0};
  return sphere_cand_d(d2, dp, e.r, dc, true, id);
}

template <uint32_t SH>
__device__ __forceinline__ Cand sphere_exact(const SceneAux* __restrict__ X, const PrimEntry* P, const Ray& ray, int i) {
  const uint32_t id = prim_bases<SH>(X).sphere + static_cast<uint32_t>(i);
  const PrimEntry& e = P[id];
  const DivC dc{e.r, e.y, e.fast, 0};
  return sphere_cand(ld4(e.p), e.r, dc, ray, true, id);
}

template <uint32_t SH, bool WITH_TIGER = true>
__device__ __forceinline__ Cand find_rest(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                          const PrimEntry* P, const Ray& ray, Cand inter) {
  constexpr uint32_t K = SH & 0xFFu;
  constexpr uint32_t NCY = sh_count(SH, 3);
  const PrimBases B = prim_bases<SH>(X);
  if (K & K_CYLINDERS)
    for_count<NCY>(S->n_cylinders, [&](int i) {
      const rt4_cylinder& c = S->cylinders[i];
      const V4 cp = ld4(c.point);
#if RT4_CYL_CULL == 2
      inter = closest(cyl_cand_precull(cp, ld4(c.axis1), ld4(c.axis2), ray, c.r, X->cyl_r[i], X->cyl_cull[i], true,
                                       B.cyl + static_cast<uint32_t>(i)),
                      inter);
#elif RT4_CYL_CULL
      inter = closest(cyl_cand_cull(cyl_project(cp, ld4(c.axis1), ld4(c.axis2), ray), cp, c.r, X->cyl_r[i], X->cyl_cull[i],
                                    true, B.cyl + static_cast<uint32_t>(i)),
                      inter);
#else
      inter = closest(cyl_cand(cyl_project(cp, ld4(c.axis1), ld4(c.axis2), ray), cp, c.r, X->cyl_r[i], true,
                               B.cyl + static_cast<uint32_t>(i)),
                      inter);
#endif
    });
  if (K & K_UNION)
    if (!(RT4_BOUND_SKIP && far_from<ball_behind_of<SH>(), occlude_of<SH>(1)>(X->union_bound[0], ray, &inter)))
      inter = closest(union_cand(S, X, 0, B.uni, ray), inter);
  if (K & K_HYPERCUBE)
    if (!(occlude_of<SH>(2) && far_from<false, true, false>(X->hyper_bound[0], ray, &inter)) &&
        !(RT4_HYPER_SKIP && hyper_skip(X->hyper_bound[0], ray, inter)))
      inter = closest(hypercube_cand<RT4_HYPER_PENDING != 0, RT4_HYPER_AXIS && (RT4_HYPER_AXIS_TIGER || !(K & K_TIGER))>(S, X, reinterpret_cast<const float4*>(P) - HYPER_CELLS_LDS, 0, B.cube, ray), inter);
  if ((K & K_TIGER) && WITH_TIGER)
    if (!(RT4_BOUND_SKIP && far_from<ball_behind_of<SH>(), occlude_of<SH>(1)>(X->tiger_bound[0], ray, &inter))) {
#ifdef RT4_LANESTATS  // diagnostic: tiger tests and their active lanes (counter[60], [61])
      {
        const unsigned long long ex = __builtin_amdgcn_read_exec();
        if (rt4_ls_counter && (threadIdx.x & 63u) == static_cast<unsigned>(__builtin_ctzll(ex))) {
          atomicAdd(rt4_ls_counter + 60, 1ull);
          atomicAdd(rt4_ls_counter + 61, static_cast<unsigned long long>(__popcll(ex)));
        }
      }
#endif
      inter = closest(tiger_cand(S, X, 0, B.tiger, ray), inter);
    }
  return inter;
}

// The exact tests of a lane's pending spheres in index order (pass 2 of find_cand), from the cull's dots
// or the centre.
template <uint32_t SH, bool GEO = true>
__device__ __forceinline__ Cand exact_pending(const SceneAux* __restrict__ X, const PrimEntry* P, const Ray& ray,
                                              const SphereGeo& geo, uint32_t pend, Cand inter) {
  while (pend) {
#ifdef RT4_LANESTATS  // diagnostic: trips and their active lanes (counter[40], [41]), as in find_cand
    {
      const unsigned long long ex = __builtin_amdgcn_read_exec();
      if (rt4_ls_counter && (threadIdx.x & 63u) == static_cast<unsigned>(__builtin_ctzll(ex))) {
        atomicAdd(rt4_ls_counter + 40, 1ull);
        atomicAdd(rt4_ls_counter + 41, static_cast<unsigned long long>(__popcll(ex)));
      }
    }
#endif
    const int i = __builtin_ctz(pend);
    pend &= pend - 1u;
    if constexpr (GEO && geo_spheres<SH>() > 0)
      inter = closest(sphere_exact_geo<SH>(X, P, geo, i), inter);
    else
      inter = closest(sphere_exact<SH>(X, P, ray, i), inter);
  }
  return inter;
}

template <uint32_t SH, bool WITH_TIGER = true>
__device__ __forceinline__ Cand find_cand(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                          const PrimEntry* P, const Ray& ray) {
  constexpr uint32_t K = SH & 0xFFu;
#if RT4_SPHERE_CULL
  uint32_t pend;
  SphereGeo geo;
  Cand inter = find_pre<SH>(S, X, ray, pend, &geo);
  if (K & K_SPHERES) {
#ifdef RT4_LANESTATS  // diagnostic: histogram of the lanes with pending spheres per find (counter[42 + bucket]
                      // wave events, counter[50 + bucket] lanes; buckets 1, 2, 3-4, 5-8, 9-16, 17-32, 33-64)
    {
      const unsigned long long pm = __ballot(pend != 0u);
      const unsigned long long ex = __builtin_amdgcn_read_exec();
      if (pm && rt4_ls_counter && (threadIdx.x & 63u) == static_cast<unsigned>(__builtin_ctzll(ex))) {
        const unsigned n = static_cast<unsigned>(__popcll(pm));
        const unsigned bk = n <= 1u ? 0u : (n <= 2u ? 1u : (n <= 4u ? 2u : (n <= 8u ? 3u : (n <= 16u ? 4u : (n <= 32u ? 5u : 6u)))));
        atomicAdd(rt4_ls_counter + 42 + bk, 1ull);
        atomicAdd(rt4_ls_counter + 50 + bk, static_cast<unsigned long long>(n));
      }
    }
#endif
    // Pass 2: each lane evaluates ITS pending spheres in index order, so a wave pays for
    // max-over-lanes(pending) exact evaluations instead of n_spheres.
    while (pend) {
#ifdef RT4_LANESTATS  // diagnostic: pending-loop trips and their active lanes, per block in LDS
      {
        const unsigned long long ex = __builtin_amdgcn_read_exec();
        // the pointer is set by the trace kernel only: null in the tile-order and find kernels
        if (rt4_ls_counter && (threadIdx.x & 63u) == static_cast<unsigned>(__builtin_ctzll(ex))) {
          atomicAdd(rt4_ls_counter + 40, 1ull);
          atomicAdd(rt4_ls_counter + 41, static_cast<unsigned long long>(__popcll(ex)));
        }
      }
#endif
      const int i = __builtin_ctz(pend);
      pend &= pend - 1u;
      if constexpr (geo_spheres<SH>() > 0)
        inter = closest(sphere_exact_geo<SH>(X, P, geo, i), inter);
      else
        inter = closest(sphere_exact<SH>(X, P, ray, i), inter);
    }
  }
  return find_rest<SH, WITH_TIGER>(S, X, P, ray, inter);
#else
  constexpr uint32_t NSP = sh_count(SH, 1), NSH = sh_count(SH, 2);
  const PrimBases B = prim_bases<SH>(X);
  Cand inter = no_cand();
  if (K & K_SPACES) for_count<NSP>(S->n_spaces, [&](int i) { inter = closest(space_cand(S, i, ray), inter); });
  if (K & K_SPHERES)
    for_count<NSH>(S->n_spheres, [&](int i) {
      const rt4_sphere& sp = S->spheres[i];
      inter = closest(sphere_cand(ld4(sp.center), sp.r, X->sphere_r[i], ray, true, B.sphere + static_cast<uint32_t>(i)),
                      inter);
    });
  return find_rest<SH, WITH_TIGER>(S, X, P, ray, inter);
#endif
}

// Normal + material of the winning candidate (per-lane data: vector loads from the scene).
__device__ __forceinline__ V4 cyl_normal(V4 cp, V4 a1, V4 a2, float r, const DivC& dc, float sdist, bool flip,
                                         const Ray& ray) {
  const CylProj p = cyl_project(cp, a1, a2, ray);
  V4 n = divs_c(sub(cp, mad(p.r12.drct, sdist, p.r12.point)), dc);  // shader.frag:218-219 on the projected ray
  return flip ? neg(n) : n;
}

// Normal of the winning candidate from its LDS primitive entry; Hit.mat = the flat primitive index.
// Only the kinds the scene shape K can produce are compiled in.
template <uint32_t SH>
__device__ __forceinline__ Hit resolve(const PrimEntry* P, const Ray& ray, const Cand& c) {
  constexpr uint32_t K = SH & 0xFFu;
  const PrimEntry& e = P[c.id];
  const int kind = e.kind;
  Hit h;
  h.hit = c.hit;
  h.dist = c.dist;
  h.mat = static_cast<int>(c.id);
  h.norm = ld4(e.p);  // PK_CUBE: the cell's space.norm (shader.frag:365)
  if ((K & K_SPACES) && kind == PK_SPACE) {
    h.norm = neg(mul(ld4(e.p), c.flip ? -1.0f : 1.0f));  // -drct_h (shader.frag:234,238)
  } else if ((K & K_SPHERES) && kind == PK_SPHERE) {
    const DivC dc{e.r, e.y, e.fast, 0};
    const V4 n = divs_c(sub(ld4(e.p), mad(ray.drct, c.sdist, ray.point)), dc);  // :218-219
    h.norm = c.flip ? neg(n) : n;
  } else if ((K & (K_CYLINDERS | K_UNION | K_TIGER)) && kind == PK_CYLINDER) {
    const DivC dc{e.r, e.y, e.fast, 0};
    h.norm = cyl_normal(ld4(e.p), ld4(e.a1), ld4(e.a2), e.r, dc, c.sdist, c.flip, ray);
  }
  return h;
}

}  // namespace rt4
