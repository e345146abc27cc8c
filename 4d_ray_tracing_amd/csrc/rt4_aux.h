// rt4_aux.h — per-scene constants derived on the host at rt4_context_set_scene, stored on the device
// right after the rt4_scene_desc. They let the specialised kernel replace expensive correctly
// rounded operations by cheaper ones WITHOUT changing a single result bit:
//   DivC       x / b for a scene constant b (a radius, the sun's angular size) as
//              q = x*y, r = fma(-q, b, x), q + r*y with y = RN(1/b). Enabled per divisor only after
//              an exhaustive device check over all 2^32 numerators found no bit difference against
//              the IEEE quotient (rt4_verify_div_kernel); otherwise the kernel divides normally.
//   thresholds sqrt(x) > r  <=>  x > gt(r)   and   sqrt(x) < r  <=>  x < lt(r), exact because
//              RN(sqrt(.)) is monotone; gt/lt found by bisection over float bit patterns.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../../include/rt4.h"

namespace rt4 {

typedef float f8v __attribute__((ext_vector_type(8)));    // one s_load_dwordx8 when wave-uniform
typedef float f16v __attribute__((ext_vector_type(16)));  // one s_load_dwordx16

struct DivC {
  float b;       // divisor
  float y;       // RN(1/b)
  int32_t fast;  // 1: the 3-op quotient was verified bit-exact for every float numerator
  int32_t pad;
};

// One entry per primitive that can be a hit (flat index = Cand.id): what resolve() needs to build
// the normal of the winning hit, and its material. Staged into LDS by every workgroup.
enum PrimKind : int32_t { PK_SPACE = 0, PK_SPHERE = 1, PK_CYLINDER = 2, PK_CUBE = 3 };
struct PrimEntry {
  float p[4];     // space.norm | sphere.center | cylinder.point | cube.norm
  float a1[4];    // cylinder.axis1
  float a2[4];    // cylinder.axis2
  float r;        // sphere / cylinder radius (divisor of the normal)
  float y;        // DivC.y for r
  int32_t fast;   // DivC.fast for r
  int32_t kind;   // PrimKind
  float glow, refl, color[3];  // material (shader.frag:163-167)
  float pad[3];
};
static_assert(sizeof(PrimEntry) == 96, "PrimEntry is 6 x 16 B");
constexpr int MAX_PRIMS = RT4_MAX_SPACES + RT4_MAX_SPHERES + RT4_MAX_CYLINDERS + 2 * RT4_MAX_UNIONS +
                          8 * RT4_MAX_HYPERCUBES + 4 * RT4_MAX_TIGERS;

// Sphere cull (rt4_fast.h find_cand): for a ray outside the sphere (len_po >= r, len_po >= SMALL)
// with dot_pord >= 0, sphere_cand misses iff sin_oap = RN(RN(len_po * sin_(acos_(c))) / r) >= 1,
// c = RN(dot_pord / len_po). With d2 = dot(po,po) (len_po = RN(sqrt(d2))) and
//   P = RN(d2 - RN(dot_pord^2)) > RN(fma(K, d2, r2m)),   K = 4e-6, r2m = RN(r^2 (1 + 1e-4)),
// the exact path is guaranteed to miss: sin_(acos_(c)) is within 1.75e-7 (relative) of
// sqrt(1 - c^2) for every float c in [0, 1) (exhaustive), the rounding of c costs at
// most 2u c^2/(1-c^2) <= 2u d2/P relative in 1 - c^2, and P's own rounding at most 3u d2; together
// P >= r^2 (1 + 7e-7) + 3.1e-7 d2 suffices, which the test exceeds ~13x (d2 term) / ~140x (r^2).
// Culled spheres are exactly the ones the exact path reports as no hit, so results are unchanged.
constexpr float SPHERE_CULL_K = 4e-6f;
// Everything the cull pass reads per sphere, in one 32-B block (one wide scalar load per sphere pair
// instead of one load and one wait per field).
struct alignas(32) SphereCull {
  float center[4];  // spheres[i].center
  float d2_out;     // smallest d2 with RN(sqrt(d2)) >= max(r, SMALL_F)
  float r2m;        // RN(r^2 (1 + 1e-4)); +inf disables the cull (tiny or non-finite r)
  float r2m_pre;    // r2m (1 + 1e-6), rounded up: the cylinders' pre-normalisation cull (below); +inf disables
  float pad;
};

// The same cull for the 2-axis cylinders (rt4_fast.h cyl_cand_cull): their exact test is sphere_cand on the ray
// projected onto the cylinder's 2-plane (shader.frag:251-267), and the derivation above is in terms of d2 and
// dot_pord alone, whatever the ray's direction, so it holds for the projected ray as it is. Only d2_out and r2m
// are used (the centre is the cylinder's point). A tiger's axes pair skips its shared sphere core when both of its
// radii cull; one quarter of the in-wave split when its own radius does.
// Pre-normalisation form (rt4_fast.h cyl_cand_precull): cyl_project normalises the projected direction e (two
// lengths, four divisions) before the test needs dp = dot(po, RN(e / len)). With u = 2^-24, |dp - s| <= 8.1u sqrt(d2)
// for s = dot(po, e) / |e| (the division and sqrt round once each, the two dots by gamma_4), so
//   P = RN(d2 - RN(dp^2)) >= d2 - s^2 - 18.2u d2,   T = RN(fma(K, d2, r2m)) <= (K d2 + r2m)(1 + u),
// and P > T (the cull above, hence the miss) follows from d2 - s^2 > (K + 18.3u) d2 + r2m (1 + u)   (1).
// From Q = dot(po, e), L = dot(e, e) (relative error gamma_4 for L, 4u sqrt(d2) |e| for Q) and M = d2 |e|^2:
//   lhs = RN(RN(d2 L) - RN(Q^2)) <= M - (po.e)^2 + 15.1u M,   rhs = RN(RN(fma(K2, d2, r2m_pre)) L)
//   >= (K2 d2 + r2m_pre) |e|^2 (1 - 6.1u),
// so lhs > rhs gives d2 - s^2 > (K2 (1 - 6.1u) - 15.1u) d2 + r2m_pre (1 - 6.1u), which implies (1) for
// K2 >= K + 33.4u (~6.0e-6; CYL_PRECULL_K = 8e-6) and r2m_pre >= r2m (1 + 7.2u). The operands are kept in range
// (d2, L < 1e18, L > 1e-30; d2 >= d2_out > 9e-8) so that no product overflows or leaves the normal range.
constexpr float CYL_PRECULL_K = 8e-6f;

// Bounding hypersphere of a tiger / cylinders union (rt4_fast.h far_from): every point the exact test
// can report as a hit lies on one cylinder (distance r from its axes plane, up to ~1e-5 relative) and
// passes the other cylinder's axes-distance filter (d^2 <= gt). When the two axes planes are
// orthogonal complements through the same point (init_tiger / the reference's unions), those two
// distances are the point's coordinates in the two planes, so |q - c|^2 <= r^2 + gt = R^2. A ray whose
// LINE keeps its distance^2 to c above R2m = R^2 (1 + 1e-3) (+ 4e-6 |p - c|^2 for the fp32
// evaluation) cannot produce a real hit. The one other way these tests report a hit is a NaN
// distance: sqrt(r^2 + len_po^2 - 2 r len_po cos) of a slightly negative rounding of (len_po - r)^2,
// i.e. a ray starting on (within ~5e-4 r of) one of the infinite cylinders, anywhere; the NaN then
// passes the filters (the reference's comparisons are false on NaN). So the skip also requires the
// origin's squared distance to each axes plane to stay out of [0.99 r^2, 1.01 r^2] for the radii of
// that plane's cylinders (band[]). Then the skipped test's result is exactly "no hit".
// r2m = +inf disables (non-orthonormal axes, different points).
struct alignas(64) BoundBall {
  float center[4];
  float a1[4], a2[4];  // orthonormal axes of plane A (its cylinders: radii bands 0-1); plane B is the complement
  float r2m;
  float band[8];       // [lo, hi] of d_A^2 for up to two plane-A radii, then of d_B^2 for plane-B radii
  float pad[3];
};

// Everything final_light reads on its common paths (constant override, sky pre-test), in one 64-B block.
struct alignas(64) HotSky {
  float sky[3];        // sky_light (shader.frag:405)
  float pre_k;         // sky_pre_k below
  float sun_drct[4];   // sun.drct
  float const_rgb[3];  // final_light_const (RT4_FINAL_LIGHT_CONSTANT)
  int32_t mode;        // final_light_mode
  float pre_a;        // the pre-test's a <= pre_a shortcut: 0 when sky_c_star > 0, else -inf (off; with
                       // pre_k = 0 the whole pre-test is then off: a sun wider than pi/2 reaches a <= 0)
  float pad[3];
};

struct SceneAux {
  // flat primitive ids: spaces, spheres, cylinders, union cylinders (2 per union), cubes (8 per
  // hypercube), tiger cylinders (inner1, outer1, inner2, outer2 per tiger)
  int32_t n_prims;
  int32_t base_sphere, base_cyl, base_union, base_cube, base_tiger;
  int32_t pad_[2];
  DivC sphere_r[RT4_MAX_SPHERES];
  DivC cyl_r[RT4_MAX_CYLINDERS];
  DivC union_r[RT4_MAX_UNIONS][2];
  float union_gt[RT4_MAX_UNIONS];      // gt(cylinder2.r): both union checks use cylinder2.r (shader.frag:286,290)
  DivC tiger_r[RT4_MAX_TIGERS][4];     // inner_cyl1, outer_cyl1, inner_cyl2, outer_cyl2
  float tiger_gt[RT4_MAX_TIGERS][2];   // [0]: gt(outer_cyl2.r) filters faces 1xx; [1]: gt(outer_cyl1.r) filters 2xx
  float tiger_lt[RT4_MAX_TIGERS][2];   // [0]: lt(inner_cyl2.r);                    [1]: lt(inner_cyl1.r)
  DivC sun_ang;
  DivC sun_len;  // length(sun.drct) (fma dot + correctly rounded sqrt, as the kernel would compute it)
  float sky_c_star;  // every v_cos <= this gives acos(v_cos) >= angular_size: plain sky, no acos needed
                     // (largest float below min{c : acos(c) < angular_size}, exhaustive device search)
  float sky_pre_k;   // conservative sky pre-test (trace final_light): a <= 0 || a*a < l2 * sky_pre_k with
                     // a = dot(drct, sun.drct), l2 = dot(drct, drct) in [2^-40, 2^40] implies
                     // v_cos <= sky_c_star. sky_pre_k = RN(c*^2 len(sun)^2 (1 - 1e-5)); 0 disables.
  // 1 when hypercube i's cells are axis-aligned in the canonical order: cell k's norm is +e_(k&3) for
  // k < 4 and -e_(k&3) for k >= 4 (other components +-0), every |point| < 1e30. Then for finite rays
  // (|p|, |d| < 1e30) the cull's dot products are exactly +-one component (rt4_fast.h hypercube_cand).
  int32_t hyper_axis[RT4_MAX_HYPERCUBES];
  int32_t pad2_[2];
  HotSky hot_sky;
  SphereCull sphere_cull[RT4_MAX_SPHERES];
  BoundBall union_bound[RT4_MAX_UNIONS];
  BoundBall tiger_bound[RT4_MAX_TIGERS];
  // Hypercube (rt4_fast.h cube_cand): a face hit needs |q - c|^2 <= |cpt - c|^2 + 3 r^2 for the face
  // square (orthonormal normal + axes); only center and r2m are used. A face that is not nearly
  // parallel to the ray (cos_dn^2 >= 1e-12 |d|^2) has a finite hit point, so for a ray whose line
  // clears the ball its extent test fails: skipped. Nearly parallel faces (the +inf / NaN "hits" of
  // shader.frag:357-365) always run the exact test.
  BoundBall hyper_bound[RT4_MAX_HYPERCUBES];
  // hypercube 0's cells as 6 float4 each {point, norm, x, y, z, {r}}, staged in LDS ahead of the
  // primitive table so the pending-cell loop can read the cell a lane needs (rt4_fast.h)
  float hyper_cells[8][24];  // must directly precede prims (kernels address it as prims - 48 float4)
  PrimEntry prims[MAX_PRIMS];
  // after the table, so that the fields above keep their offsets (r05-v50; the kernels' scalar addressing and so
  // their schedules stay as they were)
  SphereCull cyl_cull[RT4_MAX_CYLINDERS];
  SphereCull union_cull[RT4_MAX_UNIONS][2];
  SphereCull tiger_cull[RT4_MAX_TIGERS][4];  // inner_cyl1, outer_cyl1, inner_cyl2, outer_cyl2 (as tiger_r)
};

static_assert(offsetof(SceneAux, prims) - offsetof(SceneAux, hyper_cells) == sizeof(float) * 8 * 24,
              "hyper_cells must directly precede prims");

}  // namespace rt4
