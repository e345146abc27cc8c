// =====================================================================================================
// rt4 ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A scalar CPU restatement of the reference hot path, executable/shader.frag (BusyginIvan/
// 4D_ray_tracing), one function per shader function, each citing the lines it follows. It is the
// parity checker for the HIP kernel and the timed CPU baseline ("port") in bench.py. Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product (librt4.so)
// never links or calls it.
//
// PARITY STATUS: "parity unpinned" for rendered images — the reference is a GLSL 330 shader that
// cannot run in this environment (no desktop GL) and ships no tests, golden images or
// fixtures. What IS pinned: the integer RNG against the survey's known-answer vectors (hash, first
// rand() of two pixels: SURVEY.md §4), the sampler's domain properties (exhaustive 2^23 sweep), and
// each intersector against closed-form geometry (tests/test_oracle.py).
//
// fp32 semantics (shared with the kernel). GLSL leaves built-in precision to the
// driver, so this restatement fixes one definition both sides follow bit for bit:
//   * IEEE fp32, round-to-nearest-even, denormals kept, NO implicit contraction (-ffp-contract=off).
//   * dot(a,b) = fma(a.w,b.w, fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)));  length(v) = sqrt(dot(v,v)).
//   * vector multiply-add forms written in the shader (p + d*t, v - n*k, sky*(1-k) + light*k, ...)
//     are one fma per component; every scalar expression is evaluated literally, left to right.
//   * division and sqrt are correctly rounded.
//   * acos/asin/sin/cos are the polynomial definitions in rt4m_* below (Cephes-style coefficients,
//     ~1-2 ulp), evaluated with fma; they return NaN outside their domain like libm.
//
// The template parameter F is `float` for rendering and `CF` (an fp32 value that counts its
// arithmetic) for the algorithmic op count: add/sub/mul/div/sqrt/rint = 1, fma = 2, neg/abs/compare = 0.
// =====================================================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "../include/rt4.h"

namespace {

// ---------------------------------------------------------------- op-counting fp32 scalar
thread_local uint64_t g_ops = 0;
// ops spent inside w_by_volume's Newton loop (rand_drct): the sampler table (RT4_FLAG_SAMPLER_LUT)
// replaces exactly these with one load, so "executed" counts for the LUT kernel drop them
thread_local uint64_t g_sampler_ops = 0;

struct CF {
  float v;
  CF() = default;
  constexpr CF(float x) : v(x) {}
};
inline CF operator+(CF a, CF b) { ++g_ops; return CF(a.v + b.v); }
inline CF operator-(CF a, CF b) { ++g_ops; return CF(a.v - b.v); }
inline CF operator*(CF a, CF b) { ++g_ops; return CF(a.v * b.v); }
inline CF operator/(CF a, CF b) { ++g_ops; return CF(a.v / b.v); }
inline CF operator-(CF a) { return CF(-a.v); }
inline bool operator<(CF a, CF b) { return a.v < b.v; }
inline bool operator>(CF a, CF b) { return a.v > b.v; }
inline bool operator<=(CF a, CF b) { return a.v <= b.v; }
inline bool operator>=(CF a, CF b) { return a.v >= b.v; }
inline CF& operator+=(CF& a, CF b) { a = a + b; return a; }
inline CF& operator*=(CF& a, CF b) { a = a * b; return a; }
inline CF& operator/=(CF& a, CF b) { a = a / b; return a; }

#ifdef RT4_NATIVE_MATH
// Native-math mode (librt4_oracle_native.so): the shader's multiply-add forms as written,
// a*b + c with two roundings, and the GLSL built-ins from glibc (acosf, asinf, sinf, cosf) instead of the
// rt4m_* definitions. A sensitivity probe of the images to the built-ins' definition, which the
// unrunnable GL reference leaves open; never the parity checker.
inline float fma_(float a, float b, float c) { return a * b + c; }
constexpr bool kNative = true;
#else
inline float fma_(float a, float b, float c) { return std::fmaf(a, b, c); }
constexpr bool kNative = false;
#endif
inline float sqrt_(float a) { return std::sqrt(a); }
inline float abs_(float a) { return std::fabs(a); }
inline float rint_(float a) { return std::rint(a); }
inline float val(float a) { return a; }
inline CF fma_(CF a, CF b, CF c) { g_ops += 2; return CF(std::fmaf(a.v, b.v, c.v)); }
inline CF sqrt_(CF a) { ++g_ops; return CF(std::sqrt(a.v)); }
inline CF abs_(CF a) { return CF(std::fabs(a.v)); }
inline CF rint_(CF a) { ++g_ops; return CF(std::rint(a.v)); }
inline float val(CF a) { return a.v; }

// ---------------------------------------------------------------- constants (shader.frag:23-24)
constexpr float PI_F = 3.14159265f;   // shader.frag:23
constexpr float SMALL_F = 0.0003f;    // shader.frag:24
constexpr float PIO2_F = 1.57079637050628662109375f;  // float(pi/2)
constexpr float PIO2_LO = -4.37113900018624283e-8f;    // pi/2 - PIO2_F
constexpr float TWO_OVER_PI = 0.636619772367581343f;
constexpr int NEWTON_CAP = 64;  // never reached for rand() inputs (exhaustive sweep: max 8)

// ---------------------------------------------------------------- deterministic transcendentals
// asin core on z = s*s (or z = (1-|x|)/2, s = sqrt(z)): s + s*z*P(z), P from Cephes asinf.
template <class F> F rt4m_asin_core(F s, F z) {
  F p = fma_(fma_(fma_(fma_(F(4.2163199048e-2f), z, F(2.4181311049e-2f)), z, F(4.5470025998e-2f)), z,
                  F(7.4953002686e-2f)), z, F(1.6666752422e-1f));
  return fma_(p, z * s, s);
}

template <class F> F rt4m_asin(F x) {
  if constexpr (kNative && std::is_same<F, float>::value) return std::asin(x);
  F a = abs_(x);
  F r;
  if (a > F(0.5f)) {
    F z = F(0.5f) * (F(1.0f) - a);
    F s = sqrt_(z);
    r = F(PIO2_F) - F(2.0f) * rt4m_asin_core(s, z);
  } else {
    r = rt4m_asin_core(a, a * a);
  }
  return std::signbit(val(x)) ? -r : r;
}

template <class F> F rt4m_acos(F x) {
  if constexpr (kNative && std::is_same<F, float>::value) return std::acos(x);
  F a = abs_(x);
  if (a > F(0.5f)) {
    F z = F(0.5f) * (F(1.0f) - a);
    F s = sqrt_(z);
    F t = F(2.0f) * rt4m_asin_core(s, z);
    return x > F(0.0f) ? t : F(PI_F) - t;
  }
  // |x| <= 0.5, or NaN (NaN propagates through the core)
  return F(PIO2_F) - rt4m_asin_core(x, x * x);
}

// sin/cos: Cody-Waite reduction by pi/2 (two fma steps), Cephes sinf/cosf kernels on |r| <= pi/4.
template <class F> void rt4m_reduce(F x, F& r, int& q) {
  F j = rint_(x * F(TWO_OVER_PI));
  r = fma_(-j, F(PIO2_F), x);
  r = fma_(-j, F(PIO2_LO), r);
  float jv = val(j);
  q = (std::fabs(jv) < 8388608.0f) ? (static_cast<int>(jv) & 3) : 0;
}
template <class F> F rt4m_sin_kernel(F r) {
  F z = r * r;
  F p = fma_(fma_(F(-1.9515295891e-4f), z, F(8.3321608736e-3f)), z, F(-1.6666654611e-1f));
  return fma_(p, z * r, r);
}
template <class F> F rt4m_cos_kernel(F r) {
  F z = r * r;
  F p = fma_(fma_(F(2.443315711809948e-5f), z, F(-1.388731625493765e-3f)), z, F(4.166664568298827e-2f));
  return fma_(p, z * z, fma_(F(-0.5f), z, F(1.0f)));
}
template <class F> F rt4m_sin(F x) {
  if constexpr (kNative && std::is_same<F, float>::value) return std::sin(x);
  F r; int q; rt4m_reduce(x, r, q);
  F s = rt4m_sin_kernel(r), c = rt4m_cos_kernel(r);
  switch (q) { case 0: return s; case 1: return c; case 2: return -s; default: return -c; }
}
template <class F> F rt4m_cos(F x) {
  if constexpr (kNative && std::is_same<F, float>::value) return std::cos(x);
  F r; int q; rt4m_reduce(x, r, q);
  F s = rt4m_sin_kernel(r), c = rt4m_cos_kernel(r);
  switch (q) { case 0: return c; case 1: return -s; case 2: return -c; default: return s; }
}

// ---------------------------------------------------------------- vec4 / vec3 (GLSL built-ins)
template <class F> struct V4 { F x, y, z, w; };
template <class F> struct V3 { F x, y, z; };

template <class F> inline V4<F> v4(const float* p) { return {F(p[0]), F(p[1]), F(p[2]), F(p[3])}; }
template <class F> inline V3<F> v3(const float* p) { return {F(p[0]), F(p[1]), F(p[2])}; }
template <class F> inline V4<F> add(V4<F> a, V4<F> b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
template <class F> inline V4<F> sub(V4<F> a, V4<F> b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
template <class F> inline V4<F> mul(V4<F> a, F s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
template <class F> inline V4<F> divs(V4<F> a, F s) { return {a.x / s, a.y / s, a.z / s, a.w / s}; }
template <class F> inline V4<F> neg(V4<F> a) { return {-a.x, -a.y, -a.z, -a.w}; }
// a*s + c, one fma per component
template <class F> inline V4<F> mad(V4<F> a, F s, V4<F> c) {
  return {fma_(a.x, s, c.x), fma_(a.y, s, c.y), fma_(a.z, s, c.z), fma_(a.w, s, c.w)};
}
template <class F> inline F dot(V4<F> a, V4<F> b) {
  return fma_(a.w, b.w, fma_(a.z, b.z, fma_(a.y, b.y, a.x * b.x)));
}
template <class F> inline F length(V4<F> v) { return sqrt_(dot(v, v)); }

// ---------------------------------------------------------------- geometry helpers (shader.frag:45-85)
template <class F> struct Ray { V4<F> point, drct; };

template <class F> F v_cos(V4<F> v1, V4<F> v2) { return dot(v1, v2) / length(v1) / length(v2); }  // :45-47
template <class F> F angle(V4<F> v1, V4<F> v2) { return rt4m_acos(v_cos(v1, v2)); }               // :50
template <class F> V4<F> vec_in_space(V4<F> vec, V4<F> norm) { return mad(norm, -dot(vec, norm), vec); }  // :53
template <class F> V4<F> point_in_space(V4<F> p, V4<F> sp_point, V4<F> sp_norm) {  // :64-71
  return mad(sp_norm, dot(sub(sp_point, p), sp_norm), p);
}
template <class F> Ray<F> ray_in_space(Ray<F> r, V4<F> sp_point, V4<F> sp_norm) {  // :74-79
  return {point_in_space(r.point, sp_point, sp_norm), vec_in_space(r.drct, sp_norm)};
}
template <class F> V4<F> redirect(V4<F> vec, V4<F> norm) {  // :82-85
  F d = dot(vec, norm);
  return d >= F(0.0f) ? vec : mad(norm, -(F(2.0f) * d), vec);
}
template <class F> V4<F> reflect_(V4<F> i, V4<F> n) {  // GLSL reflect: I - 2*dot(N,I)*N
  F d = dot(n, i);
  return mad(n, -(F(2.0f) * d), i);
}

// ---------------------------------------------------------------- RNG (shader.frag:90-121)
inline uint32_t hash_u32(uint32_t x) {  // :94-102
  x += (x << 10);
  x ^= (x >> 6);
  x += (x << 3);
  x ^= (x >> 11);
  x += (x << 15);
  x ^= (x >> 9);
  return x;
}

struct Rng {  // uint_seed / rand_iter_seed / scr_coord bits: :90-92, :106
  uint32_t uint_seed, iter, bx, by;
  uint32_t random_uint() {  // :104-108
    iter += 0x79A010A9u;
    return hash_u32(bx ^ (by << 9) ^ iter ^ uint_seed);
  }
  float rand() {  // :111-118
    uint32_t bits = random_uint();
    bits &= 0x007FFFFFu;
    bits |= 0x3F800000u;
    float f;
    std::memcpy(&f, &bits, 4);
    return f - 1.0f;
  }
};

inline uint32_t fbits(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

// ---------------------------------------------------------------- S^3 sampler (shader.frag:136-158)
template <class F> F volume_by_w(F w) {  // :136-138
  return (w * sqrt_(F(1.0f) - w * w) - rt4m_acos(w)) / F(PI_F) + F(1.0f);
}
template <class F> F w_by_volume(F v, int* iters) {  // :141-150
  F old_w;
  F new_w = F(0.0f);
  int it = 0;
  do {
    old_w = new_w;
    F old_v = volume_by_w(old_w);
    F df = old_w > F(0.0f) ? old_v - volume_by_w(old_w - F(SMALL_F)) : volume_by_w(old_w + F(SMALL_F)) - old_v;
    new_w = old_w - F(SMALL_F) / df * (old_v - v);
    ++it;
  } while (abs_(new_w - old_w) >= F(SMALL_F) && it < NEWTON_CAP);
  if (iters) *iters = it;
  return new_w;
}
template <class F> V4<F> rand_drct(Rng& rng) {  // :153-158, cyl_vec_to_vec :128-130
  const uint64_t ops0 = g_ops;
  F w = w_by_volume(F(rng.rand()), nullptr);
  g_sampler_ops += g_ops - ops0;
  F r = sqrt_(F(1.0f) - w * w);
  F z = (F(rng.rand()) * F(2.0f) - F(1.0f)) * r;
  F rr = sqrt_(r * r - z * z);
  F fi = F(rng.rand()) * F(2.0f) * F(PI_F);
  return {rr * rt4m_cos(fi), rr * rt4m_sin(fi), z, w};
}

// ---------------------------------------------------------------- intersections (shader.frag:163-400)
template <class F> struct Mat { F glow, refl; V3<F> color; };
template <class F> struct Inter { bool hit; F dist; V4<F> norm; Mat<F> m; };

template <class F> Mat<F> mat_of(const rt4_material& m) { return {F(m.glow), F(m.refl_prob), v3<F>(m.color)}; }
template <class F> Inter<F> not_intersect() {  // :178
  return {false, F(0.0f), {F(0.0f), F(0.0f), F(0.0f), F(0.0f)}, {F(0.0f), F(0.0f), {F(0.0f), F(0.0f), F(0.0f)}}};
}
template <class F> Inter<F> closest(const Inter<F>& a, const Inter<F>& b) {  // :181-185
  if (!a.hit) return b;
  if (!b.hit) return a;
  return a.dist < b.dist ? a : b;
}

template <class F> Inter<F> sphere_intersection(V4<F> center, F r, const Mat<F>& m, Ray<F> ray, bool outer) {  // :197-221
  V4<F> vec_po = sub(center, ray.point);
  F len_po = length(vec_po);
  F cos_opa;
  if (len_po < F(SMALL_F)) {
    cos_opa = F(0.0f);
  } else {
    F dot_pord = dot(vec_po, ray.drct);
    if (len_po >= r && dot_pord < F(0.0f)) return not_intersect<F>();
    cos_opa = dot_pord / len_po;
    if (cos_opa > F(1.0f)) cos_opa = F(1.0f);
    if (cos_opa < F(-1.0f)) cos_opa = F(-1.0f);
  }
  F angle_opa = rt4m_acos(cos_opa);
  F sin_oap = len_po * rt4m_sin(angle_opa) / r;
  if (sin_oap >= F(1.0f)) return not_intersect<F>();
  F angle_oap = rt4m_asin(sin_oap);
  bool flip = outer && len_po > r;
  if (flip) angle_oap = F(PI_F) - angle_oap;
  F angle_aop = F(PI_F) - angle_opa - angle_oap;
  F dist = sqrt_(r * r + len_po * len_po - F(2.0f) * r * len_po * rt4m_cos(angle_aop));
  V4<F> norm = divs(sub(center, mad(ray.drct, dist, ray.point)), r);
  if (flip) norm = neg(norm);  // norm *= -1 : exact sign flip
  return {true, dist, norm, m};
}

template <class F> Inter<F> space_intersection(const rt4_space& s, Ray<F> ray) {  // :231-239
  V4<F> sp = v4<F>(s.point), sn = v4<F>(s.norm);
  V4<F> vec_v = sub(sp, ray.point);
  F dot_vn = dot(vec_v, sn);
  float dv = val(dot_vn);
  F sgn = F(dv > 0.0f ? 1.0f : (dv < 0.0f ? -1.0f : 0.0f));  // GLSL sign()
  V4<F> drct_h = mul(sn, sgn);
  F cos_dh = dot(drct_h, ray.drct);
  if (cos_dh < F(SMALL_F)) return not_intersect<F>();
  F dist = abs_(dot_vn) / cos_dh;
  return {true, dist, neg(drct_h), mat_of<F>(s.material)};
}

template <class F> Inter<F> cylinder_intersection(const rt4_cylinder& c, Ray<F> ray, bool outer) {  // :251-267
  V4<F> cp = v4<F>(c.point), a1 = v4<F>(c.axis1), a2 = v4<F>(c.axis2);
  Ray<F> r1 = ray_in_space(ray, cp, a1);
  if (length(r1.drct) < F(SMALL_F)) return not_intersect<F>();
  Ray<F> r12 = ray_in_space(r1, cp, a2);
  F len = length(r12.drct);
  if (len < F(SMALL_F)) return not_intersect<F>();
  r12.drct = divs(r12.drct, len);
  Inter<F> inter = sphere_intersection(cp, F(c.r), mat_of<F>(c.material), r12, outer);
  inter.dist /= len;
  return inter;
}

template <class F> F dist_to_axes_plane(F dist, Ray<F> ray, const rt4_cylinder& c) {  // :270-275
  V4<F> cp = v4<F>(c.point);
  V4<F> p = mad(ray.drct, dist, ray.point);
  V4<F> p1 = point_in_space(p, cp, v4<F>(c.axis1));
  V4<F> p12 = point_in_space(p1, cp, v4<F>(c.axis2));
  return length(sub(cp, p12));
}

template <class F> Inter<F> cylinders_union_intersection(const rt4_cylinders_union& u, Ray<F> ray) {  // :284-294
  Inter<F> i1 = cylinder_intersection(u.cylinder1, ray, true);
  if (dist_to_axes_plane(i1.dist, ray, u.cylinder2) > F(u.cylinder2.r)) i1 = not_intersect<F>();
  Inter<F> i2 = cylinder_intersection(u.cylinder2, ray, true);
  if (dist_to_axes_plane(i2.dist, ray, u.cylinder1) > F(u.cylinder2.r)) i2 = not_intersect<F>();  // :290 quirk
  return closest(i1, i2);
}

template <class F>
Inter<F> tigers_face_intersection(const rt4_cylinder& cyl, const rt4_cylinder& outer_cyl, const rt4_cylinder& inner_cyl,
                                  Ray<F> ray, bool outer) {  // :317-324
  Inter<F> inter = cylinder_intersection(cyl, ray, outer);
  if (dist_to_axes_plane(inter.dist, ray, outer_cyl) > F(outer_cyl.r)) return not_intersect<F>();
  if (dist_to_axes_plane(inter.dist, ray, inner_cyl) < F(inner_cyl.r)) return not_intersect<F>();
  return inter;
}

template <class F> Inter<F> tiger_intersection(const rt4_tiger& t, Ray<F> ray) {  // :327-341
  Inter<F> i111 = tigers_face_intersection(t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Inter<F> i112 = tigers_face_intersection(t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Inter<F> i121 = tigers_face_intersection(t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Inter<F> i122 = tigers_face_intersection(t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Inter<F> i211 = tigers_face_intersection(t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Inter<F> i212 = tigers_face_intersection(t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  Inter<F> i221 = tigers_face_intersection(t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Inter<F> i222 = tigers_face_intersection(t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  return closest(closest(closest(i111, i112), closest(i121, i122)), closest(closest(i211, i212), closest(i221, i222)));
}

template <class F> Inter<F> cube_intersection(const rt4_cube& c, Ray<F> ray) {  // :352-366
  V4<F> cpt = v4<F>(c.point), cn = v4<F>(c.norm);
  V4<F> vec_n = neg(cn);
  V4<F> vec_c = sub(cpt, ray.point);
  F h = dot(vec_c, vec_n);
  if (h < F(0.0f)) return not_intersect<F>();
  F cos_dn = dot(ray.drct, vec_n);
  if (cos_dn < F(0.0f)) return not_intersect<F>();
  F dist = h / cos_dn;
  V4<F> point = mad(ray.drct, dist, ray.point);
  V4<F> vec_cp = sub(point, cpt);
  F r(c.r);
  if (abs_(dot(vec_cp, v4<F>(c.x))) > r) return not_intersect<F>();
  if (abs_(dot(vec_cp, v4<F>(c.y))) > r) return not_intersect<F>();
  if (abs_(dot(vec_cp, v4<F>(c.z))) > r) return not_intersect<F>();
  return {true, dist, cn, mat_of<F>(c.material)};
}

template <class F> Inter<F> hypercube_intersection(const rt4_hypercube& h, Ray<F> ray) {  // :394-400
  for (int i = 0; i < 8; i++) {
    Inter<F> inter = cube_intersection(h.cubes[i], ray);
    if (inter.hit) return inter;
  }
  return not_intersect<F>();
}

template <class F> Inter<F> find_intersection(const rt4_scene_desc& s, Ray<F> ray) {  // :434-451
  Inter<F> inter = not_intersect<F>();
  for (int g = 0; g < s.n_groups; g++) {
    const rt4_group& gr = s.groups[g];
    for (int k = 0; k < gr.count; k++) {
      const int i = gr.first + k;
      Inter<F> n;
      switch (gr.kind) {
        case RT4_GROUP_SPACES: n = space_intersection(s.spaces[i], ray); break;
        case RT4_GROUP_SPHERES: {
          const rt4_sphere& sp = s.spheres[i];
          n = sphere_intersection(v4<F>(sp.center), F(sp.r), mat_of<F>(sp.material), ray, gr.outer != 0);
        } break;
        case RT4_GROUP_CYLINDERS: n = cylinder_intersection(s.cylinders[i], ray, gr.outer != 0); break;
        case RT4_GROUP_CYLINDERS_UNION: n = cylinders_union_intersection(s.unions[i], ray); break;
        case RT4_GROUP_HYPERCUBE: n = hypercube_intersection(s.hypercubes[i], ray); break;
        case RT4_GROUP_TIGER: n = tiger_intersection(s.tigers[i], ray); break;
        default: continue;
      }
      inter = gr.new_first ? closest(n, inter) : closest(inter, n);
    }
  }
  return inter;
}

// ---------------------------------------------------------------- shading + trace (shader.frag:454-495)
template <class F> V3<F> final_light(const rt4_scene_desc& s, V4<F> drct) {  // :454-468
  if (s.final_light_mode == RT4_FINAL_LIGHT_CONSTANT) return v3<F>(s.final_light_const);
  V3<F> sky = v3<F>(s.sky_light);
  F deviation = angle(drct, v4<F>(s.sun.drct));
  F ang(s.sun.angular_size);
  if (deviation < ang) {
    F k = deviation / ang, sh(s.sun.sharpness);
    k = (sh * sh * k / (F(1.0f) - sh * k) + F(1.0f)) * (F(1.0f) - k);
    F km = F(1.0f) - k;
    return {fma_(F(s.sun.light[0]), k, sky.x * km), fma_(F(s.sun.light[1]), k, sky.y * km),
            fma_(F(s.sun.light[2]), k, sky.z * km)};
  }
  return sky;
}

template <class F>
V3<F> trace(const rt4_scene_desc& s, const rt4_uniforms& u, Ray<F> ray, Rng& rng, uint64_t& n_inter) {  // :471-495
  V3<F> acc = {F(0.0f), F(0.0f), F(0.0f)};
  V3<F> T = {F(1.0f), F(1.0f), F(1.0f)};
  const F indent(u.small_indent);
  for (int i = 0; i <= u.reflections_amount; i++) {
    Inter<F> inter = find_intersection(s, ray);
    ++n_inter;
    if (!inter.hit) {  // :477-479
      V3<F> fl = final_light(s, ray.drct);
      return {fma_(T.x, fl.x, acc.x), fma_(T.y, fl.y, acc.y), fma_(T.z, fl.z, acc.z)};
    }
    const Mat<F>& m = inter.m;  // :481-482
    acc = {fma_(m.color.x * m.glow, T.x, acc.x), fma_(m.color.y * m.glow, T.y, acc.y),
           fma_(m.color.z * m.glow, T.z, acc.z)};
    T = {T.x * m.color.x, T.y * m.color.y, T.z * m.color.z};
    ray.point = add(ray.point, mad(ray.drct, inter.dist, mul(inter.norm, indent)));  // :485
    if (!(F(rng.rand()) > m.refl))  // rand_outcome :121, :488
      ray.drct = reflect_(ray.drct, inter.norm);
    else
      ray.drct = redirect(rand_drct<F>(rng), inter.norm);  // :491
  }
  return acc;  // :494
}

// IEEE binary16 <-> binary32, round-to-nearest-even (what v_cvt_f16_f32 does on gfx950), denormals kept.
inline float half_to_float(uint16_t h) {
  const uint32_t sign = static_cast<uint32_t>(h & 0x8000u) << 16, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) {
      bits = sign;
    } else {  // subnormal half: m * 2^-24, exact in fp32
      float f = static_cast<float>(m) * 5.9604644775390625e-8f;
      std::memcpy(&bits, &f, 4);
      bits |= sign;
    }
  } else if (e == 31) {
    bits = sign | 0x7F800000u | (m << 13);
  } else {
    bits = sign | ((e + 112u) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}
inline uint16_t float_to_half(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint16_t sign = static_cast<uint16_t>((x >> 16) & 0x8000u);
  const uint32_t ax = x & 0x7FFFFFFFu;
  if (ax >= 0x7F800000u) return sign | (ax > 0x7F800000u ? 0x7E00u | ((ax >> 13) & 0x3FFu) : 0x7C00u);  // NaN / inf
  if (ax >= 0x477FF000u) return sign | 0x7C00u;  // rounds to >= 65520: overflow to inf
  if (ax < 0x38800000u) {  // below 2^-14: half subnormal (or zero), value = round(|f| * 2^24) * 2^-24
    if (ax < 0x33000000u) return sign;  // < 2^-25: rounds to 0 (ties at exactly 2^-25 go to even = 0)
    const uint32_t e = ax >> 23, mant = (ax & 0x7FFFFFu) | 0x800000u;
    const uint32_t shift = 126u - e;  // 14..24
    uint32_t q = mant >> shift;
    const uint32_t rem = mant & ((1u << shift) - 1u), half = 1u << (shift - 1u);
    if (rem > half || (rem == half && (q & 1u))) q++;
    return sign | static_cast<uint16_t>(q);
  }
  uint32_t q = ((ax >> 13) - (112u << 10));
  const uint32_t rem = ax & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (q & 1u))) q++;
  return sign | static_cast<uint16_t>(q);
}

// mix(old, new, part) in the frame format (rt4.h rt4_frame_format); the blend is fp32 in every format.
void store_blend(void* px, int32_t fmt, const float c[3], float part) {
  const float keep = 1.0f - part;
  if (fmt == RT4_FRAME_RGBA16F) {
    uint16_t* h = static_cast<uint16_t*>(px);
    for (int q = 0; q < 3; q++) h[q] = float_to_half(fma_(c[q], part, half_to_float(h[q]) * keep));
    h[3] = 0x3C00u;  // 1.0
  } else if (fmt == RT4_FRAME_RGBA8) {
    uint8_t* b = static_cast<uint8_t*>(px);
    for (int q = 0; q < 3; q++) {
      const float old = static_cast<float>(b[q]) / 255.0f;
      const float v = fma_(c[q], part, old * keep);
      b[q] = static_cast<uint8_t>(static_cast<uint32_t>(std::fmin(std::fmax(v, 0.0f), 1.0f) * 255.0f + 0.5f));
    }
    b[3] = 255;
  } else {
    float* f = static_cast<float*>(px);
    for (int q = 0; q < 3; q++) f[q] = fma_(c[q], part, f[q] * keep);
    f[3] = 1.0f;
  }
}

template <class F> void render_pixel(const rt4_scene_desc& s, const rt4_uniforms& u, int x, int y, float* px,
                                     uint64_t& n_inter, int32_t fmt = RT4_FRAME_RGBA32F) {  // main :513-528
  const float sx = (static_cast<float>(x) + 0.5f) / u.resolution[0];  // :515-516 (IEEE division)
  const float sy = (static_cast<float>(y) + 0.5f) / u.resolution[1];
  Rng rng{static_cast<uint32_t>(u.seed), static_cast<uint32_t>(u.seed), fbits(sx), fbits(sy)};
  // ray_drct :501-505
  F mx = (F(sx) - F(0.5f)) * F(u.mtr_sizes[0]);
  F my = (F(0.5f) - F(sy)) * F(u.mtr_sizes[1]);
  V4<F> d = mad(v4<F>(u.right_drct), mx, mad(v4<F>(u.top_drct), my, v4<F>(u.vec_to_mtr)));
  d = divs(d, length(d));  // normalize
  V3<F> light = {F(0.0f), F(0.0f), F(0.0f)};
  for (int i = 0; i < u.samples; i++) {  // :520-521
    V3<F> l = trace(s, u, Ray<F>{v4<F>(u.focus), d}, rng, n_inter);
    light = {light.x + l.x, light.y + l.y, light.z + l.z};
  }
  const F ns(static_cast<float>(u.samples));
  light = {light.x / ns, light.y / ns, light.z / ns};  // :522
  const F k(u.light_to_color_conversion_coefficient);  // light_to_color :509-511
  V3<F> c = {F(1.0f) - F(1.0f) / fma_(k, light.x, F(1.0f)), F(1.0f) - F(1.0f) / fma_(k, light.y, F(1.0f)),
             F(1.0f) - F(1.0f) / fma_(k, light.z, F(1.0f))};
  if (fmt != RT4_FRAME_RGBA32F) {  // other frame formats: the blend of store_blend, in fp32
    const float cc[3] = {val(c.x), val(c.y), val(c.z)};
    store_blend(px, fmt, cc, u.part);
    return;
  }
  const F part(u.part), keep = F(1.0f) - F(u.part);  // mix(old, new, part) :526-527
  px[0] = val(fma_(c.x, part, F(px[0]) * keep));
  px[1] = val(fma_(c.y, part, F(px[1]) * keep));
  px[2] = val(fma_(c.z, part, F(px[2]) * keep));
  px[3] = 1.0f;
}

inline int region_row(const rt4_region& r, int i) {
  return r.band_rows > 0 ? r.y0 + (i / r.band_rows) * r.band_step + (i % r.band_rows) : r.y0 + i;
}

template <class F>
void render_rows(const rt4_scene_desc& s, const rt4_uniforms& u, const rt4_region& reg, float* rgba, int64_t stride,
                 int threads, uint64_t* n_inter, uint64_t* ops, uint32_t* pixel_counts, int32_t fmt = RT4_FRAME_RGBA32F,
                 uint64_t* sampler_ops = nullptr) {
  const int64_t px_bytes = fmt == RT4_FRAME_RGBA16F ? 8 : (fmt == RT4_FRAME_RGBA8 ? 4 : 16);
  std::atomic<uint64_t> total_inter{0}, total_ops{0}, total_sampler{0};
  // work items: 64-pixel pieces of rows, interleaved over the threads (balances sky vs object rows, and
  // keeps every thread busy when the region has fewer rows than threads)
  constexpr int PIECE = 64;
  const int64_t pieces = (reg.w + PIECE - 1) / PIECE, items = pieces * reg.h;
  auto worker = [&](int t) {
    uint64_t my_inter = 0;
    g_ops = 0;
    g_sampler_ops = 0;
    for (int64_t it = t; it < items; it += threads) {
      const int i = static_cast<int>(it / pieces);
      const int y = region_row(reg, i);
      const int j0 = static_cast<int>(it % pieces) * PIECE, j1 = std::min(reg.w, j0 + PIECE);
      for (int j = j0; j < j1; j++) {
        uint64_t before = my_inter;
        render_pixel<F>(s, u, reg.x0 + j, y,
                        reinterpret_cast<float*>(reinterpret_cast<char*>(rgba) + px_bytes * (static_cast<int64_t>(i) * stride + j)),
                        my_inter, fmt);
        if (pixel_counts) pixel_counts[static_cast<int64_t>(i) * reg.w + j] = static_cast<uint32_t>(my_inter - before);
      }
    }
    total_inter += my_inter;
    total_ops += g_ops;
    total_sampler += g_sampler_ops;
  };
  if (threads <= 1) {
    worker(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) pool.emplace_back(worker, t);
    for (auto& th : pool) th.join();
  }
  if (n_inter) *n_inter = total_inter.load();
  if (ops) *ops = total_ops.load();
  if (sampler_ops) *sampler_ops = total_sampler.load();
}

}  // namespace

// ==================================================================================== C exports
extern "C" {

int oracle_abi(void) { return 1; }
size_t oracle_scene_desc_size(void) { return sizeof(rt4_scene_desc); }

uint32_t oracle_hash(uint32_t x) { return hash_u32(x); }

// First n rand() values of pixel (x, y) of a W x H image (scr_coord from shader.frag:515-516).
void oracle_rand_first(int32_t W, int32_t H, int32_t seed, int32_t x, int32_t y, int32_t n, float* out) {
  const float sx = (static_cast<float>(x) + 0.5f) / static_cast<float>(W);
  const float sy = (static_cast<float>(y) + 0.5f) / static_cast<float>(H);
  Rng rng{static_cast<uint32_t>(seed), static_cast<uint32_t>(seed), fbits(sx), fbits(sy)};
  for (int i = 0; i < n; i++) out[i] = rng.rand();
}

// Element-wise evaluation of the math definitions; fn = rt4_eval_fn.
void oracle_eval_array(int32_t fn, const float* in, float* out, int32_t* aux, int64_t n) {
  for (int64_t i = 0; i < n; i++) {
    const float x = in[i];
    int it = 0;
    float r = 0.0f;
    switch (fn) {
      case RT4_EVAL_ACOS: r = rt4m_acos<float>(x); break;
      case RT4_EVAL_ASIN: r = rt4m_asin<float>(x); break;
      case RT4_EVAL_SIN: r = rt4m_sin<float>(x); break;
      case RT4_EVAL_COS: r = rt4m_cos<float>(x); break;
      case RT4_EVAL_VOLUME_BY_W: r = volume_by_w<float>(x); break;
      case RT4_EVAL_W_BY_VOLUME: r = w_by_volume<float>(x, &it); break;
      case RT4_EVAL_HASH: {
        uint32_t h = hash_u32(fbits(x));
        std::memcpy(&r, &h, 4);
      } break;
      default: r = std::nanf(""); break;
    }
    out[i] = r;
    if (aux) aux[i] = it;
  }
}

// find_intersection for n rays; out: n x 8 {hit, dist, norm xyzw, glow, refl}, out_color: n x 3.
int oracle_find_intersection(const rt4_scene_desc* s, const float* rays, float* out, float* out_color, int64_t n) {
  if (!s || !rays || !out) return RT4_ERR_ARG;
  for (int64_t i = 0; i < n; i++) {
    const float* r = rays + 8 * i;
    Ray<float> ray{v4<float>(r), v4<float>(r + 4)};
    Inter<float> h = find_intersection(*s, ray);
    float* o = out + 8 * i;
    o[0] = h.hit ? 1.0f : 0.0f;
    o[1] = h.dist;
    o[2] = h.norm.x; o[3] = h.norm.y; o[4] = h.norm.z; o[5] = h.norm.w;
    o[6] = h.m.glow; o[7] = h.m.refl;
    if (out_color) { out_color[3 * i] = h.m.color.x; out_color[3 * i + 1] = h.m.color.y; out_color[3 * i + 2] = h.m.color.z; }
  }
  return RT4_OK;
}

// One diffuse direction draw from a given RNG state (for sampler tests): returns the direction and
// the advanced counter. state[0]=uint_seed, state[1]=rand_iter_seed, state[2]=bits(sx), state[3]=bits(sy).
void oracle_rand_drct(uint32_t* state, float* out4) {
  Rng rng{state[0], state[1], state[2], state[3]};
  V4<float> d = rand_drct<float>(rng);
  out4[0] = d.x; out4[1] = d.y; out4[2] = d.z; out4[3] = d.w;
  state[1] = rng.iter;
}

// Renders region `reg` exactly like rt4_render_host (same layout). threads <= 1 runs inline.
// count_ops != 0 runs the op-counting instantiation and stores the fp32 op total in *ops.
// pixel_counts (optional, h*w) receives per-pixel find_intersection counts.
int oracle_render(const rt4_scene_desc* s, const rt4_uniforms* u, const rt4_region* reg, float* rgba,
                  int64_t row_stride_px, int32_t threads, uint64_t* n_intersections, int32_t count_ops,
                  uint64_t* ops, uint32_t* pixel_counts) {
  if (!s || !u || !reg || !rgba) return RT4_ERR_ARG;
  if (reg->w < 0 || reg->h < 0 || row_stride_px < reg->w) return RT4_ERR_ARG;
  if (threads < 1) threads = 1;
  if (count_ops)
    render_rows<CF>(*s, *u, *reg, rgba, row_stride_px, threads, n_intersections, ops, pixel_counts);
  else
    render_rows<float>(*s, *u, *reg, rgba, row_stride_px, threads, n_intersections, nullptr, pixel_counts);
  return RT4_OK;
}

// The op-counting render alone: *ops = all fp32 ops (as oracle_render with count_ops), *sampler_ops =
// the part of them inside w_by_volume (shader.frag:141-150), which the sampler-table kernel replaces
// by one load. Executed ops per unit with the table = (ops - sampler_ops) / n_intersections.
int oracle_count_ops(const rt4_scene_desc* s, const rt4_uniforms* u, const rt4_region* reg, float* rgba,
                     int64_t row_stride_px, int32_t threads, uint64_t* n_intersections, uint64_t* ops,
                     uint64_t* sampler_ops) {
  if (!s || !u || !reg || !rgba) return RT4_ERR_ARG;
  if (reg->w < 0 || reg->h < 0 || row_stride_px < reg->w) return RT4_ERR_ARG;
  if (threads < 1) threads = 1;
  render_rows<CF>(*s, *u, *reg, rgba, row_stride_px, threads, n_intersections, ops, nullptr, RT4_FRAME_RGBA32F,
                  sampler_ops);
  return RT4_OK;
}

// oracle_render in a frame format (rt4.h rt4_frame_format): frame holds h rows of row_stride_px pixels.
int oracle_render_fmt(const rt4_scene_desc* s, const rt4_uniforms* u, const rt4_region* reg, void* frame, int32_t fmt,
                      int64_t row_stride_px, int32_t threads, uint64_t* n_intersections) {
  if (!s || !u || !reg || !frame) return RT4_ERR_ARG;
  if (fmt < RT4_FRAME_RGBA32F || fmt > RT4_FRAME_RGBA8) return RT4_ERR_ARG;
  if (reg->w < 0 || reg->h < 0 || row_stride_px < reg->w) return RT4_ERR_ARG;
  if (threads < 1) threads = 1;
  render_rows<float>(*s, *u, *reg, static_cast<float*>(frame), row_stride_px, threads, n_intersections, nullptr, nullptr,
                     fmt);
  return RT4_OK;
}

uint16_t oracle_float_to_half(float f) { return float_to_half(f); }
float oracle_half_to_float(uint16_t h) { return half_to_float(h); }

}  // extern "C"
