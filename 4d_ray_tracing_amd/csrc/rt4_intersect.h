// rt4_intersect.h — the 4D intersectors of executable/shader.frag:181-451 for gfx950.
//
// Every function performs exactly the oracle's op sequence (bit-exact contract); the
// speed comes from structure, not from changed arithmetic:
//   * scene data is read through `const __restrict__` pointers with wave-uniform indices -> scalar
//     loads (s_load) into SGPRs, operands of VALU ops without VGPR copies;
//   * find_intersection is specialised per scene shape (FindSpec<K>): straight-line code, hit
//     records stay in registers (the generic group loop spilled them to scratch);
//   * tiger CSE (FindSpec with a tiger built by init_tiger): a face pair that differs only in the
//     `outer` flag shares the ray projection and the sphere-core (acos/sin/asin), and the inner and
//     outer cylinder of one axes-pair share the projection and dist_to_axes_plane. Same ops, same
//     bits, ~2.5x fewer of them.
#pragma once

#include "../../include/rt4.h"
#include "rt4_device_math.h"

namespace rt4 {

struct Hit {
  bool hit;
  float dist;
  V4 norm;
  int mat;  // byte offset of the rt4_material inside the device scene (rt4_scene_desc)
};

__device__ __forceinline__ Hit no_hit() { return Hit{false, 0.0f, V4{0.0f, 0.0f, 0.0f, 0.0f}, 0}; }

// closest(a, b), shader.frag:181-185 (on a tie the second argument wins). Field-wise selects:
// a ternary on the records would select an address and force both into scratch memory.
__device__ __forceinline__ Hit closest(const Hit& a, const Hit& b) {
  const bool ta = a.hit && (!b.hit || a.dist < b.dist);
  Hit r;
  r.hit = ta ? a.hit : b.hit;
  r.dist = ta ? a.dist : b.dist;
  r.norm.x = ta ? a.norm.x : b.norm.x;
  r.norm.y = ta ? a.norm.y : b.norm.y;
  r.norm.z = ta ? a.norm.z : b.norm.z;
  r.norm.w = ta ? a.norm.w : b.norm.w;
  r.mat = ta ? a.mat : b.mat;
  return r;
}

struct Ray {
  V4 point, drct;
};

template <class T>
__device__ __forceinline__ int mat_off(const rt4_scene_desc* S, const T& field) {
  return static_cast<int>(reinterpret_cast<const char*>(&field) - reinterpret_cast<const char*>(S));
}

__device__ __forceinline__ V4 point_in_space(V4 p, V4 sp, V4 sn) { return mad(sn, dot(sub(sp, p), sn), p); }  // :64-71
__device__ __forceinline__ V4 vec_in_space(V4 v, V4 sn) { return mad(sn, -dot(v, sn), v); }                  // :53

// ------------------------------------------------------------------ hypersphere, shader.frag:197-221
// The part of sphere_intersection that does not depend on `outer`.
struct SphereCore {
  bool miss;
  float len_po, angle_opa, angle_oap;
};

__device__ __forceinline__ SphereCore sphere_core(V4 center, float r, const Ray& ray) {
  SphereCore c;
  V4 vec_po = sub(center, ray.point);
  c.len_po = length(vec_po);
  float cos_opa;
  c.miss = false;
  if (c.len_po < SMALL_F) {
    cos_opa = 0.0f;
  } else {
    float dot_pord = dot(vec_po, ray.drct);
    c.miss = c.len_po >= r && dot_pord < 0.0f;
    cos_opa = dot_pord / c.len_po;
    cos_opa = cos_opa > 1.0f ? 1.0f : cos_opa;
    cos_opa = cos_opa < -1.0f ? -1.0f : cos_opa;
  }
  c.angle_opa = acos_(cos_opa);
  float sin_oap = c.len_po * sin_(c.angle_opa) / r;
  c.miss = c.miss || (sin_oap >= 1.0f);  // `if (sin_oap >= 1) return NOT_INTERSECT` (a NaN passes on)
  c.angle_oap = asin_(sin_oap);
  return c;
}

__device__ __forceinline__ Hit sphere_finish(const SphereCore& c, V4 center, float r, int mat, const Ray& ray,
                                             bool outer) {
  const bool flip = outer && c.len_po > r;
  const float angle_oap = flip ? PI_F - c.angle_oap : c.angle_oap;
  const float angle_aop = PI_F - c.angle_opa - angle_oap;
  const float dist = sqrt_(r * r + c.len_po * c.len_po - 2.0f * r * c.len_po * cos_(angle_aop));
  V4 norm = divs(sub(center, mad(ray.drct, dist, ray.point)), r);
  if (flip) norm = neg(norm);
  Hit h{!c.miss, dist, norm, mat};
  if (c.miss) h = no_hit();
  return h;
}

__device__ __forceinline__ Hit sphere_intersection(V4 center, float r, int mat, const Ray& ray, bool outer) {
  SphereCore c = sphere_core(center, r, ray);
  return sphere_finish(c, center, r, mat, ray, outer);
}

// ------------------------------------------------------------------ hyperplane, shader.frag:231-239
__device__ __forceinline__ Hit space_intersection(const rt4_scene_desc* __restrict__ S, int i, const Ray& ray) {
  const rt4_space& s = S->spaces[i];
  V4 sn = ld4(s.norm);
  float dot_vn = dot(sub(ld4(s.point), ray.point), sn);
  float sgn = dot_vn > 0.0f ? 1.0f : (dot_vn < 0.0f ? -1.0f : 0.0f);
  V4 drct_h = mul(sn, sgn);
  float cos_dh = dot(drct_h, ray.drct);
  if (cos_dh < SMALL_F) return no_hit();
  float dist = __builtin_fabsf(dot_vn) / cos_dh;
  return Hit{true, dist, neg(drct_h), mat_off(S, s.material)};
}

// ------------------------------------------------------------------ 2-axis cylinder, shader.frag:251-275
struct CylProj {  // ray projected onto the cylinder's 2-plane, shader.frag:252-258
  bool miss;
  float len;  // drct_in_plane_length
  Ray r12;
};

__device__ __forceinline__ CylProj cyl_project(V4 cp, V4 a1, V4 a2, const Ray& ray) {
  CylProj p;
  Ray r1{point_in_space(ray.point, cp, a1), vec_in_space(ray.drct, a1)};
  p.miss = length(r1.drct) < SMALL_F;
  p.r12 = Ray{point_in_space(r1.point, cp, a2), vec_in_space(r1.drct, a2)};
  p.len = length(p.r12.drct);
  p.miss = p.miss || (p.len < SMALL_F);
  p.r12.drct = divs(p.r12.drct, p.len);
  return p;
}

__device__ __forceinline__ Hit cyl_from_sphere(const CylProj& p, Hit h) {  // inter.dist /= len (:265)
  if (p.miss) return no_hit();
  h.dist = h.dist / p.len;
  return h;
}

__device__ __forceinline__ Hit cylinder_intersection(const rt4_scene_desc* __restrict__ S, const rt4_cylinder& c,
                                                     const Ray& ray, bool outer) {
  V4 cp = ld4(c.point);
  CylProj p = cyl_project(cp, ld4(c.axis1), ld4(c.axis2), ray);
  return cyl_from_sphere(p, sphere_intersection(cp, c.r, mat_off(S, c.material), p.r12, outer));
}

__device__ __forceinline__ float dist_to_axes_plane(float dist, const Ray& ray, V4 cp, V4 a1, V4 a2) {  // :270-275
  V4 p = mad(ray.drct, dist, ray.point);
  V4 p1 = point_in_space(p, cp, a1);
  V4 p12 = point_in_space(p1, cp, a2);
  return length(sub(cp, p12));
}

__device__ __forceinline__ float dist_to_axes_plane(float dist, const Ray& ray, const rt4_cylinder& c) {
  return dist_to_axes_plane(dist, ray, ld4(c.point), ld4(c.axis1), ld4(c.axis2));
}

// ------------------------------------------------------------------ duocylinder, shader.frag:284-294
__device__ __forceinline__ Hit cylinders_union_intersection(const rt4_scene_desc* __restrict__ S, int i,
                                                            const Ray& ray) {
  const rt4_cylinders_union& u = S->unions[i];
  Hit i1 = cylinder_intersection(S, u.cylinder1, ray, true);
  if (dist_to_axes_plane(i1.dist, ray, u.cylinder2) > u.cylinder2.r) i1 = no_hit();
  Hit i2 = cylinder_intersection(S, u.cylinder2, ray, true);
  if (dist_to_axes_plane(i2.dist, ray, u.cylinder1) > u.cylinder2.r) i2 = no_hit();  // :290 (cylinder2.r)
  return closest(i1, i2);
}

// ------------------------------------------------------------------ tiger, shader.frag:317-341
__device__ __forceinline__ Hit tigers_face(const rt4_scene_desc* __restrict__ S, const rt4_cylinder& cyl,
                                           const rt4_cylinder& outer_cyl, const rt4_cylinder& inner_cyl,
                                           const Ray& ray, bool outer) {
  Hit h = cylinder_intersection(S, cyl, ray, outer);
  if (dist_to_axes_plane(h.dist, ray, outer_cyl) > outer_cyl.r) return no_hit();
  if (dist_to_axes_plane(h.dist, ray, inner_cyl) < inner_cyl.r) return no_hit();
  return h;
}

__device__ __forceinline__ Hit tiger_intersection(const rt4_scene_desc* __restrict__ S, int i, const Ray& ray) {
  const rt4_tiger& t = S->tigers[i];
  Hit i111 = tigers_face(S, t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Hit i112 = tigers_face(S, t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Hit c1 = closest(i111, i112);
  Hit i121 = tigers_face(S, t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Hit i122 = tigers_face(S, t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Hit c12 = closest(c1, closest(i121, i122));
  Hit i211 = tigers_face(S, t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Hit i212 = tigers_face(S, t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  Hit c2 = closest(i211, i212);
  Hit i221 = tigers_face(S, t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Hit i222 = tigers_face(S, t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  return closest(c12, closest(c2, closest(i221, i222)));
}

// A face kept iff the other axes-pair's distance d satisfies !(d > outer_r) && !(d < inner_r).
__device__ __forceinline__ Hit face_filter(Hit h, float d, float outer_r, float inner_r) {
  if (d > outer_r || d < inner_r) return no_hit();
  return h;
}

// Tiger with shared axes inside each pair (init_tiger, shader.frag:303-314): inner/outer cylinder
// of a pair have the same point/axes, so the projection and dist_to_axes_plane are common.
__device__ __forceinline__ Hit tiger_intersection_shared(const rt4_scene_desc* __restrict__ S, int i, const Ray& ray) {
  const rt4_tiger& t = S->tigers[i];
  const V4 pA = ld4(t.inner_cyl1.point), a1 = ld4(t.inner_cyl1.axis1), a2 = ld4(t.inner_cyl1.axis2);
  const V4 pB = ld4(t.inner_cyl2.point), a3 = ld4(t.inner_cyl2.axis1), a4 = ld4(t.inner_cyl2.axis2);
  const float rA_in = t.inner_cyl1.r, rA_out = t.outer_cyl1.r, rB_in = t.inner_cyl2.r, rB_out = t.outer_cyl2.r;

  Hit acc_lo, acc_hi;
  {  // faces 111 112 121 122: cylinders of pair A, filtered by pair B
    const CylProj p = cyl_project(pA, a1, a2, ray);
    const SphereCore ci = sphere_core(pA, rA_in, p.r12);
    Hit i111 = cyl_from_sphere(p, sphere_finish(ci, pA, rA_in, mat_off(S, t.inner_cyl1.material), p.r12, true));
    Hit i112 = cyl_from_sphere(p, sphere_finish(ci, pA, rA_in, mat_off(S, t.inner_cyl1.material), p.r12, false));
    i111 = face_filter(i111, dist_to_axes_plane(i111.dist, ray, pB, a3, a4), rB_out, rB_in);
    i112 = face_filter(i112, dist_to_axes_plane(i112.dist, ray, pB, a3, a4), rB_out, rB_in);
    const SphereCore co = sphere_core(pA, rA_out, p.r12);
    Hit i121 = cyl_from_sphere(p, sphere_finish(co, pA, rA_out, mat_off(S, t.outer_cyl1.material), p.r12, true));
    Hit i122 = cyl_from_sphere(p, sphere_finish(co, pA, rA_out, mat_off(S, t.outer_cyl1.material), p.r12, false));
    i121 = face_filter(i121, dist_to_axes_plane(i121.dist, ray, pB, a3, a4), rB_out, rB_in);
    i122 = face_filter(i122, dist_to_axes_plane(i122.dist, ray, pB, a3, a4), rB_out, rB_in);
    acc_lo = closest(closest(i111, i112), closest(i121, i122));
  }
  {  // faces 211 212 221 222: cylinders of pair B, filtered by pair A
    const CylProj p = cyl_project(pB, a3, a4, ray);
    const SphereCore ci = sphere_core(pB, rB_in, p.r12);
    Hit i211 = cyl_from_sphere(p, sphere_finish(ci, pB, rB_in, mat_off(S, t.inner_cyl2.material), p.r12, true));
    Hit i212 = cyl_from_sphere(p, sphere_finish(ci, pB, rB_in, mat_off(S, t.inner_cyl2.material), p.r12, false));
    i211 = face_filter(i211, dist_to_axes_plane(i211.dist, ray, pA, a1, a2), rA_out, rA_in);
    i212 = face_filter(i212, dist_to_axes_plane(i212.dist, ray, pA, a1, a2), rA_out, rA_in);
    const SphereCore co = sphere_core(pB, rB_out, p.r12);
    Hit i221 = cyl_from_sphere(p, sphere_finish(co, pB, rB_out, mat_off(S, t.outer_cyl2.material), p.r12, true));
    Hit i222 = cyl_from_sphere(p, sphere_finish(co, pB, rB_out, mat_off(S, t.outer_cyl2.material), p.r12, false));
    i221 = face_filter(i221, dist_to_axes_plane(i221.dist, ray, pA, a1, a2), rA_out, rA_in);
    i222 = face_filter(i222, dist_to_axes_plane(i222.dist, ray, pA, a1, a2), rA_out, rA_in);
    acc_hi = closest(closest(i211, i212), closest(i221, i222));
  }
  return closest(acc_lo, acc_hi);
}

// ------------------------------------------------------------------ hypercube, shader.frag:352-400
__device__ __forceinline__ Hit cube_intersection(const rt4_scene_desc* __restrict__ S, const rt4_cube& c,
                                                 const Ray& ray) {
  V4 cpt = ld4(c.point), cn = ld4(c.norm);
  V4 vec_n = neg(cn);
  float h = dot(sub(cpt, ray.point), vec_n);
  if (h < 0.0f) return no_hit();
  float cos_dn = dot(ray.drct, vec_n);
  if (cos_dn < 0.0f) return no_hit();
  float dist = h / cos_dn;
  V4 vec_cp = sub(mad(ray.drct, dist, ray.point), cpt);
  if (__builtin_fabsf(dot(vec_cp, ld4(c.x))) > c.r) return no_hit();
  if (__builtin_fabsf(dot(vec_cp, ld4(c.y))) > c.r) return no_hit();
  if (__builtin_fabsf(dot(vec_cp, ld4(c.z))) > c.r) return no_hit();
  return Hit{true, dist, cn, mat_off(S, c.material)};
}

__device__ __forceinline__ Hit hypercube_intersection(const rt4_scene_desc* __restrict__ S, int i, const Ray& ray) {
  const rt4_hypercube& hc = S->hypercubes[i];
  Hit res = no_hit();
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (!res.hit) res = cube_intersection(S, hc.cubes[k], ray);  // first hit in cell order
  }
  return res;
}

// ------------------------------------------------------------------ find_intersection, shader.frag:434-451
// Generic: any group list (order, tie direction, outer flags) of rt4_scene_desc.
__device__ __forceinline__ Hit find_intersection_generic(const rt4_scene_desc* __restrict__ S, const Ray& ray) {
  Hit inter = no_hit();
  const int ng = S->n_groups;
  for (int g = 0; g < ng; g++) {
    const int kind = S->groups[g].kind, first = S->groups[g].first, count = S->groups[g].count;
    const bool outer = S->groups[g].outer != 0, new_first = S->groups[g].new_first != 0;
    for (int k = 0; k < count; k++) {
      const int i = first + k;
      Hit n;
      if (kind == RT4_GROUP_SPACES) {
        n = space_intersection(S, i, ray);
      } else if (kind == RT4_GROUP_SPHERES) {
        const rt4_sphere& sp = S->spheres[i];
        n = sphere_intersection(ld4(sp.center), sp.r, mat_off(S, sp.material), ray, outer);
      } else if (kind == RT4_GROUP_CYLINDERS) {
        n = cylinder_intersection(S, S->cylinders[i], ray, outer);
      } else if (kind == RT4_GROUP_CYLINDERS_UNION) {
        n = cylinders_union_intersection(S, i, ray);
      } else if (kind == RT4_GROUP_HYPERCUBE) {
        n = hypercube_intersection(S, i, ray);
      } else if (kind == RT4_GROUP_TIGER) {
        n = tiger_intersection(S, i, ray);
      } else {
        continue;
      }
      inter = new_first ? closest(n, inter) : closest(inter, n);
    }
  }
  return inter;
}

// Shape bits of a specialised scene: groups appear at most once each, in shader.frag's order
// (:437-448), cover their whole object array, and use the reference form closest(new, inter).
enum : uint32_t {
  K_SPACES = 1u << 0,
  K_SPHERES = 1u << 1,
  K_CYLINDERS = 1u << 2,
  K_UNION = 1u << 3,
  K_HYPERCUBE = 1u << 4,
  K_TIGER = 1u << 5,  // one tiger with shared axes per pair (init_tiger)
};

template <uint32_t K>
__device__ __forceinline__ Hit find_intersection_spec(const rt4_scene_desc* __restrict__ S, const Ray& ray) {
  Hit inter = no_hit();
  if (K & K_SPACES) {
    const int n = S->n_spaces;
    for (int i = 0; i < n; i++) inter = closest(space_intersection(S, i, ray), inter);
  }
  if (K & K_SPHERES) {
    const int n = S->n_spheres;
    for (int i = 0; i < n; i++) {
      const rt4_sphere& sp = S->spheres[i];
      inter = closest(sphere_intersection(ld4(sp.center), sp.r, mat_off(S, sp.material), ray, true), inter);
    }
  }
  if (K & K_CYLINDERS) {
    const int n = S->n_cylinders;
    for (int i = 0; i < n; i++) inter = closest(cylinder_intersection(S, S->cylinders[i], ray, true), inter);
  }
  if (K & K_UNION) inter = closest(cylinders_union_intersection(S, 0, ray), inter);
  if (K & K_HYPERCUBE) inter = closest(hypercube_intersection(S, 0, ray), inter);
  if (K & K_TIGER) inter = closest(tiger_intersection_shared(S, 0, ray), inter);
  return inter;
}

}  // namespace rt4
