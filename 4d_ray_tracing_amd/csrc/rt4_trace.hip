// rt4_trace.hip — the hot path: executable/shader.frag's per-cell trace loop as one gfx950 kernel,
// plus the device context and the C-ABI render / diagnostic entry points of include/rt4.h.
//
// Kernel shape:
//   * one lane per pixel; a 256-thread workgroup renders a 16x16 pixel tile, each wave an 8x8
//     sub-tile (spatially coherent paths inside a wave).
//   * the sample x bounce loops of main()/trace() (shader.frag:474, :520) are FLATTENED into one
//     loop of find_intersection calls: a lane whose path ends starts its next sample in the same
//     iteration, so a wave runs max_lane(sum of path lengths) iterations, not
//     samples * max(path length). The RNG counter keeps running across samples (shader.frag:92).
//   * scene geometry is wave-uniform: read through a const __restrict__ pointer, which the
//     compiler turns into scalar (s_load / K$) loads; materials are fetched per lane at shading.
//   * optional w_by_volume table (RT4_FLAG_SAMPLER_LUT): the Newton loop of shader.frag:141-150
//     is a pure function of rand()'s 23 mantissa bits; a 2^23-entry table built by the same
//     device function replaces the divergent loop by one cached load.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <new>

#include "../../include/rt4.h"
#include "rt4_device_math.h"
#include "rt4_internal.h"

using namespace rt4;

namespace {

// ---------------------------------------------------------------- hit record
struct Hit {
  bool hit;
  float dist;
  V4 norm;
  int mat;  // byte offset of the rt4_material inside the device scene
};

__device__ __forceinline__ Hit no_hit() { return Hit{false, 0.0f, V4{0.0f, 0.0f, 0.0f, 0.0f}, 0}; }

// closest(a, b), shader.frag:181-185 (tie -> b)
__device__ __forceinline__ Hit closest(const Hit& a, const Hit& b) {
  if (!a.hit) return b;
  if (!b.hit) return a;
  return a.dist < b.dist ? a : b;
}

#define MAT_OFF(ptr) (static_cast<int>(reinterpret_cast<const char*>(&(ptr)) - reinterpret_cast<const char*>(S)))

struct Ray { V4 point, drct; };

// ---------------------------------------------------------------- intersectors (shader.frag:189-400)
__device__ __forceinline__ Hit sphere_intersection(V4 center, float r, int mat, Ray ray, bool outer) {  // :197-221
  V4 vec_po = sub(center, ray.point);
  float len_po = length(vec_po);
  float cos_opa;
  if (len_po < SMALL_F) {
    cos_opa = 0.0f;
  } else {
    float dot_pord = dot(vec_po, ray.drct);
    if (len_po >= r && dot_pord < 0.0f) return no_hit();
    cos_opa = dot_pord / len_po;
    cos_opa = cos_opa > 1.0f ? 1.0f : cos_opa;
    cos_opa = cos_opa < -1.0f ? -1.0f : cos_opa;
  }
  float angle_opa = acos_(cos_opa);
  float sin_oap = len_po * sin_(angle_opa) / r;
  if (sin_oap >= 1.0f) return no_hit();
  float angle_oap = asin_(sin_oap);
  bool flip = outer && len_po > r;
  if (flip) angle_oap = PI_F - angle_oap;
  float angle_aop = PI_F - angle_opa - angle_oap;
  float dist = __builtin_sqrtf(r * r + len_po * len_po - 2.0f * r * len_po * cos_(angle_aop));
  V4 norm = divs(sub(center, mad(ray.drct, dist, ray.point)), r);
  if (flip) norm = neg(norm);
  return Hit{true, dist, norm, mat};
}

__device__ __forceinline__ Hit space_intersection(const rt4_scene_desc* __restrict__ S, int i, Ray ray) {  // :231-239
  const rt4_space& s = S->spaces[i];
  V4 sn = ld4(s.norm);
  float dot_vn = dot(sub(ld4(s.point), ray.point), sn);
  float sgn = dot_vn > 0.0f ? 1.0f : (dot_vn < 0.0f ? -1.0f : 0.0f);
  V4 drct_h = mul(sn, sgn);
  float cos_dh = dot(drct_h, ray.drct);
  if (cos_dh < SMALL_F) return no_hit();
  float dist = __builtin_fabsf(dot_vn) / cos_dh;
  return Hit{true, dist, neg(drct_h), MAT_OFF(s.material)};
}

__device__ __forceinline__ V4 point_in_space(V4 p, V4 sp, V4 sn) { return mad(sn, dot(sub(sp, p), sn), p); }
__device__ __forceinline__ V4 vec_in_space(V4 v, V4 sn) { return mad(sn, -dot(v, sn), v); }

__device__ __forceinline__ Hit cylinder_intersection(const rt4_scene_desc* __restrict__ S, const rt4_cylinder& c,
                                                     Ray ray, bool outer) {  // :251-267
  V4 cp = ld4(c.point), a1 = ld4(c.axis1), a2 = ld4(c.axis2);
  Ray r1{point_in_space(ray.point, cp, a1), vec_in_space(ray.drct, a1)};
  if (length(r1.drct) < SMALL_F) return no_hit();
  Ray r12{point_in_space(r1.point, cp, a2), vec_in_space(r1.drct, a2)};
  float len = length(r12.drct);
  if (len < SMALL_F) return no_hit();
  r12.drct = divs(r12.drct, len);
  Hit h = sphere_intersection(cp, c.r, MAT_OFF(c.material), r12, outer);
  h.dist = h.dist / len;
  return h;
}

__device__ __forceinline__ float dist_to_axes_plane(float dist, Ray ray, const rt4_cylinder& c) {  // :270-275
  V4 cp = ld4(c.point);
  V4 p = mad(ray.drct, dist, ray.point);
  V4 p1 = point_in_space(p, cp, ld4(c.axis1));
  V4 p12 = point_in_space(p1, cp, ld4(c.axis2));
  return length(sub(cp, p12));
}

__device__ __forceinline__ Hit cylinders_union_intersection(const rt4_scene_desc* __restrict__ S, int i,
                                                            Ray ray) {  // :284-294
  const rt4_cylinders_union& u = S->unions[i];
  Hit i1 = cylinder_intersection(S, u.cylinder1, ray, true);
  if (dist_to_axes_plane(i1.dist, ray, u.cylinder2) > u.cylinder2.r) i1 = no_hit();
  Hit i2 = cylinder_intersection(S, u.cylinder2, ray, true);
  if (dist_to_axes_plane(i2.dist, ray, u.cylinder1) > u.cylinder2.r) i2 = no_hit();  // :290 (cylinder2.r)
  return closest(i1, i2);
}

__device__ __forceinline__ Hit tigers_face(const rt4_scene_desc* __restrict__ S, const rt4_cylinder& cyl,
                                           const rt4_cylinder& outer_cyl, const rt4_cylinder& inner_cyl, Ray ray,
                                           bool outer) {  // :317-324
  Hit h = cylinder_intersection(S, cyl, ray, outer);
  if (dist_to_axes_plane(h.dist, ray, outer_cyl) > outer_cyl.r) return no_hit();
  if (dist_to_axes_plane(h.dist, ray, inner_cyl) < inner_cyl.r) return no_hit();
  return h;
}

__device__ __forceinline__ Hit tiger_intersection(const rt4_scene_desc* __restrict__ S, int i, Ray ray) {  // :327-341
  const rt4_tiger& t = S->tigers[i];
  Hit i111 = tigers_face(S, t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Hit i112 = tigers_face(S, t.inner_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Hit i121 = tigers_face(S, t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, true);
  Hit i122 = tigers_face(S, t.outer_cyl1, t.outer_cyl2, t.inner_cyl2, ray, false);
  Hit i211 = tigers_face(S, t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Hit i212 = tigers_face(S, t.inner_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  Hit i221 = tigers_face(S, t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, true);
  Hit i222 = tigers_face(S, t.outer_cyl2, t.outer_cyl1, t.inner_cyl1, ray, false);
  return closest(closest(closest(i111, i112), closest(i121, i122)), closest(closest(i211, i212), closest(i221, i222)));
}

__device__ __forceinline__ Hit cube_intersection(const rt4_scene_desc* __restrict__ S, const rt4_cube& c,
                                                 Ray ray) {  // :352-366
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
  return Hit{true, dist, cn, MAT_OFF(c.material)};
}

__device__ __forceinline__ Hit hypercube_intersection(const rt4_scene_desc* __restrict__ S, int i, Ray ray) {  // :394-400
  const rt4_hypercube& hc = S->hypercubes[i];
  Hit res = no_hit();
  for (int k = 0; k < 8; k++) {
    Hit h = cube_intersection(S, hc.cubes[k], ray);
    if (!res.hit && h.hit) res = h;  // first hit in cell order
  }
  return res;
}

__device__ __forceinline__ Hit find_intersection(const rt4_scene_desc* __restrict__ S, Ray ray) {  // :434-451
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
        n = sphere_intersection(ld4(sp.center), sp.r, MAT_OFF(sp.material), ray, outer);
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

// ---------------------------------------------------------------- shading (shader.frag:404-495)
__device__ __forceinline__ V3 final_light(const rt4_scene_desc* __restrict__ S, V4 drct) {  // :454-468
  if (S->final_light_mode == RT4_FINAL_LIGHT_CONSTANT) return ld3(S->final_light_const);
  V3 sky = ld3(S->sky_light);
  V4 sd = ld4(S->sun.drct);
  float deviation = acos_(dot(drct, sd) / length(drct) / length(sd));  // angle(), :45-50
  float ang = S->sun.angular_size;
  if (deviation < ang) {
    float k = deviation / ang, s = S->sun.sharpness;
    k = (s * s * k / (1.0f - s * k) + 1.0f) * (1.0f - k);
    float km = 1.0f - k;
    return V3{fmaf_(S->sun.light[0], k, sky.x * km), fmaf_(S->sun.light[1], k, sky.y * km),
              fmaf_(S->sun.light[2], k, sky.z * km)};
  }
  return sky;
}

struct RngState {
  uint32_t base;  // bits(scr.x) ^ (bits(scr.y) << 9) ^ uint_seed   (shader.frag:106-107)
  uint32_t iter;  // rand_iter_seed                                (shader.frag:92, :105)
};

__device__ __forceinline__ float rand_(RngState& r) {  // :104-118
  r.iter += 0x79A010A9u;
  uint32_t bits = hash_u32(r.base ^ r.iter);
  return __uint_as_float((bits & 0x007FFFFFu) | 0x3F800000u) - 1.0f;
}

template <bool LUT>
__device__ __forceinline__ V4 rand_drct(RngState& rng, const float* __restrict__ wlut) {  // :153-158
  float u1 = rand_(rng);
  float w;
  if (LUT) {
    w = wlut[__float_as_uint(u1 + 1.0f) & 0x007FFFFFu];  // u1 = m * 2^-23 exactly
  } else {
    w = w_by_volume(u1, nullptr);
  }
  float r = __builtin_sqrtf(1.0f - w * w);
  float z = (rand_(rng) * 2.0f - 1.0f) * r;
  float rr = __builtin_sqrtf(r * r - z * z);
  float fi = rand_(rng) * 2.0f * PI_F;
  float sf, cf;
  sincos_(fi, sf, cf);
  return V4{rr * cf, rr * sf, z, w};
}

struct KernelArgs {
  rt4_uniforms u;
  rt4_region reg;
  int64_t row_stride_px;
};

template <bool LUT>
__global__ __launch_bounds__(256) void rt4_trace_kernel(const rt4_scene_desc* __restrict__ S, const KernelArgs a,
                                                        float4* __restrict__ frame,
                                                        unsigned long long* __restrict__ counter,
                                                        const float* __restrict__ wlut) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
  const int i = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
  const bool active = (j < a.reg.w) && (i < a.reg.h);

  const int x = a.reg.x0 + j;
  const int y = a.reg.band_rows > 0 ? a.reg.y0 + (i / a.reg.band_rows) * a.reg.band_step + (i % a.reg.band_rows)
                                    : a.reg.y0 + i;
  // main(): scr_coord = gl_FragCoord.xy / resolution (shader.frag:515-516)
  const float sx = (static_cast<float>(x) + 0.5f) / a.u.resolution[0];
  const float sy = (static_cast<float>(y) + 0.5f) / a.u.resolution[1];
  const uint32_t useed = static_cast<uint32_t>(a.u.seed);
  RngState rng{__float_as_uint(sx) ^ (__float_as_uint(sy) << 9) ^ useed, useed};

  // ray_drct(), shader.frag:501-505
  const float mx = (sx - 0.5f) * a.u.mtr_sizes[0];
  const float my = (0.5f - sy) * a.u.mtr_sizes[1];
  V4 d0 = mad(ld4(a.u.right_drct), mx, mad(ld4(a.u.top_drct), my, ld4(a.u.vec_to_mtr)));
  d0 = divs(d0, length(d0));
  const V4 focus = ld4(a.u.focus);

  // flattened samples x bounces (shader.frag:520-521 around :474-495)
  Ray ray{focus, d0};
  V3 acc{0.0f, 0.0f, 0.0f}, T{1.0f, 1.0f, 1.0f}, light{0.0f, 0.0f, 0.0f};
  int s = active ? 0 : a.u.samples;
  int b = 0;
  uint32_t n_inter = 0;
  const float indent = a.u.small_indent;
  const int R = a.u.reflections_amount;
  const char* Sb = reinterpret_cast<const char*>(S);

  while (s < a.u.samples) {
    Hit h = find_intersection(S, ray);
    ++n_inter;
    bool end;
    if (!h.hit) {  // :477-479
      V3 fl = final_light(S, ray.drct);
      acc = V3{fmaf_(T.x, fl.x, acc.x), fmaf_(T.y, fl.y, acc.y), fmaf_(T.z, fl.z, acc.z)};
      end = true;
    } else {
      const rt4_material* m = reinterpret_cast<const rt4_material*>(Sb + h.mat);
      const float glow = m->glow, refl = m->refl_prob;
      const V3 c{m->color[0], m->color[1], m->color[2]};
      acc = V3{fmaf_(c.x * glow, T.x, acc.x), fmaf_(c.y * glow, T.y, acc.y), fmaf_(c.z * glow, T.z, acc.z)};  // :481
      T = V3{T.x * c.x, T.y * c.y, T.z * c.z};                                                                  // :482
      ray.point = add(ray.point, mad(ray.drct, h.dist, mul(h.norm, indent)));                                  // :485
      if (!(rand_(rng) > refl)) {  // :488 rand_outcome
        float dn = dot(h.norm, ray.drct);
        ray.drct = mad(h.norm, -(2.0f * dn), ray.drct);  // reflect
      } else {
        V4 v = rand_drct<LUT>(rng, wlut);  // :491 redirect(rand_drct(), norm)
        float dv = dot(v, h.norm);
        ray.drct = dv >= 0.0f ? v : mad(h.norm, -(2.0f * dv), v);
      }
      ++b;
      end = b > R;
    }
    if (end) {  // path finished: next sample restarts at the focus
      light = V3{light.x + acc.x, light.y + acc.y, light.z + acc.z};
      ++s;
      b = 0;
      ray = Ray{focus, d0};
      acc = V3{0.0f, 0.0f, 0.0f};
      T = V3{1.0f, 1.0f, 1.0f};
    }
  }

  if (active) {
    const float ns = static_cast<float>(a.u.samples);
    light = V3{light.x / ns, light.y / ns, light.z / ns};  // :522
    const float k = a.u.light_to_color_conversion_coefficient;  // :509-511
    const V3 c{1.0f - 1.0f / fmaf_(k, light.x, 1.0f), 1.0f - 1.0f / fmaf_(k, light.y, 1.0f),
               1.0f - 1.0f / fmaf_(k, light.z, 1.0f)};
    float4* px = frame + static_cast<int64_t>(i) * a.row_stride_px + j;
    const float4 old = *px;  // old_frame (:526)
    const float part = a.u.part, keep = 1.0f - a.u.part;
    *px = make_float4(fmaf_(c.x, part, old.x * keep), fmaf_(c.y, part, old.y * keep),
                      fmaf_(c.z, part, old.z * keep), 1.0f);  // mix, alpha 1 (:527)
  }

  if (counter) {
    // wave-level sum, one atomic per wave
    unsigned long long v = n_inter;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0 && v) atomicAdd(counter, v);
  }
}

__global__ void rt4_build_wlut_kernel(float* __restrict__ lut) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m < (1u << 23)) lut[m] = w_by_volume(__uint_as_float(m | 0x3F800000u) - 1.0f, nullptr);
}

__global__ void rt4_eval_kernel(int fn, const float* __restrict__ in, float* __restrict__ out, int32_t* __restrict__ aux,
                                int64_t n) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float x = in[t];
  int it = 0;
  float r;
  switch (fn) {
    case RT4_EVAL_ACOS: r = acos_(x); break;
    case RT4_EVAL_ASIN: r = asin_(x); break;
    case RT4_EVAL_SIN: r = sin_(x); break;
    case RT4_EVAL_COS: r = cos_(x); break;
    case RT4_EVAL_VOLUME_BY_W: r = volume_by_w(x); break;
    case RT4_EVAL_W_BY_VOLUME: r = w_by_volume(x, &it); break;
    case RT4_EVAL_HASH: r = __uint_as_float(hash_u32(__float_as_uint(x))); break;
    default: r = __builtin_nanf(""); break;
  }
  out[t] = r;
  if (aux) aux[t] = it;
}

__global__ void rt4_find_kernel(const rt4_scene_desc* __restrict__ S, const float* __restrict__ rays,
                                float* __restrict__ out, float* __restrict__ out_color, int64_t n) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const float* r = rays + 8 * t;
  Hit h = find_intersection(S, Ray{ld4(r), ld4(r + 4)});
  float* o = out + 8 * t;
  o[0] = h.hit ? 1.0f : 0.0f;
  o[1] = h.dist;
  o[2] = h.norm.x; o[3] = h.norm.y; o[4] = h.norm.z; o[5] = h.norm.w;
  if (h.hit) {
    const rt4_material* m = reinterpret_cast<const rt4_material*>(reinterpret_cast<const char*>(S) + h.mat);
    o[6] = m->glow; o[7] = m->refl_prob;
    out_color[3 * t] = m->color[0]; out_color[3 * t + 1] = m->color[1]; out_color[3 * t + 2] = m->color[2];
  } else {
    o[6] = 0.0f; o[7] = 0.0f;
    out_color[3 * t] = 0.0f; out_color[3 * t + 1] = 0.0f; out_color[3 * t + 2] = 0.0f;
  }
}

}  // namespace

// ==================================================================================== context
struct rt4_context {
  int device = 0;
  uint32_t flags = 0;
  rt4_scene_desc* d_scene = nullptr;
  bool has_scene = false;
  float* d_wlut = nullptr;
};

#define HIP_TRY(expr)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) {                                                                      \
      rt4_set_err(err, errlen, "%s failed: %s", #expr, hipGetErrorString(e_));                   \
      return RT4_ERR_HIP;                                                                        \
    }                                                                                            \
  } while (0)

extern "C" {

int rt4_context_create(int device, uint32_t flags, rt4_context** out, char* err, size_t errlen) {
  if (!out) return rt4_set_err(err, errlen, "out is NULL"), RT4_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) {
    rt4_set_err(err, errlen, "device %d out of range (have %d HIP devices)", device, ndev);
    return RT4_ERR_HIP;
  }
  HIP_TRY(hipSetDevice(device));
  rt4_context* c = new (std::nothrow) rt4_context();
  if (!c) return rt4_set_err(err, errlen, "out of host memory"), RT4_ERR_ARG;
  c->device = device;
  c->flags = flags;
  hipError_t e = hipMalloc(&c->d_scene, sizeof(rt4_scene_desc));
  if (e == hipSuccess && (flags & RT4_FLAG_SAMPLER_LUT)) {
    e = hipMalloc(&c->d_wlut, sizeof(float) << 23);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(rt4_build_wlut_kernel, dim3((1u << 23) / 256), dim3(256), 0, 0, c->d_wlut);
      e = hipGetLastError();
      if (e == hipSuccess) e = hipDeviceSynchronize();
    }
  }
  if (e != hipSuccess) {
    rt4_set_err(err, errlen, "context allocation failed: %s", hipGetErrorString(e));
    rt4_context_destroy(c);
    return RT4_ERR_HIP;
  }
  *out = c;
  return RT4_OK;
}

void rt4_context_destroy(rt4_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->d_scene) (void)hipFree(ctx->d_scene);
  if (ctx->d_wlut) (void)hipFree(ctx->d_wlut);
  delete ctx;
}

int rt4_context_set_scene(rt4_context* ctx, const rt4_scene_desc* scene, char* err, size_t errlen) {
  if (!ctx || !scene) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  int st = rt4_scene_validate(scene, err, errlen);
  if (st != RT4_OK) return st;
  HIP_TRY(hipSetDevice(ctx->device));
  HIP_TRY(hipMemcpy(ctx->d_scene, scene, sizeof(rt4_scene_desc), hipMemcpyHostToDevice));
  ctx->has_scene = true;
  return RT4_OK;
}

int rt4_render_device(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* d_rgba,
                      int64_t row_stride_px, unsigned long long* d_counter, void* stream, char* err, size_t errlen) {
  if (!ctx || !u || !region || !d_rgba) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (!ctx->has_scene) return rt4_set_err(err, errlen, "context has no scene (rt4_context_set_scene)"), RT4_ERR_ARG;
  int st = rt4_check_render_args(u, region, row_stride_px, err, errlen);
  if (st != RT4_OK) return st;
  if (region->w == 0 || region->h == 0) return RT4_OK;
  KernelArgs a;
  a.u = *u;
  a.reg = *region;
  a.row_stride_px = row_stride_px;
  dim3 grid((region->w + 15) / 16, (region->h + 15) / 16);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (ctx->d_wlut)
    hipLaunchKernelGGL(rt4_trace_kernel<true>, grid, dim3(256), 0, s, ctx->d_scene, a,
                       reinterpret_cast<float4*>(d_rgba), d_counter, ctx->d_wlut);
  else
    hipLaunchKernelGGL(rt4_trace_kernel<false>, grid, dim3(256), 0, s, ctx->d_scene, a,
                       reinterpret_cast<float4*>(d_rgba), d_counter, ctx->d_wlut);
  HIP_TRY(hipGetLastError());
  return RT4_OK;
}

int rt4_render_host(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* rgba,
                    int64_t row_stride_px, uint64_t* n_intersections, char* err, size_t errlen) {
  if (!ctx || !u || !region || !rgba) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  int st = rt4_check_render_args(u, region, row_stride_px, err, errlen);
  if (st != RT4_OK) return st;
  if (n_intersections) *n_intersections = 0;
  if (region->w == 0 || region->h == 0) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t bytes = static_cast<size_t>(region->h - 1) * row_stride_px * 16 + static_cast<size_t>(region->w) * 16;
  float* d = nullptr;
  unsigned long long* dc = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  hipError_t e = hipMalloc(&dc, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpy(d, rgba, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(dc, 0, sizeof(unsigned long long));
  if (e != hipSuccess) {
    (void)hipFree(d);
    if (dc) (void)hipFree(dc);
    rt4_set_err(err, errlen, "render_host staging failed: %s", hipGetErrorString(e));
    return RT4_ERR_HIP;
  }
  st = rt4_render_device(ctx, u, region, d, row_stride_px, dc, nullptr, err, errlen);
  if (st == RT4_OK) {
    e = hipDeviceSynchronize();
    unsigned long long cnt = 0;
    if (e == hipSuccess) e = hipMemcpy(rgba, d, bytes, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&cnt, dc, sizeof(cnt), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      rt4_set_err(err, errlen, "render_host failed: %s", hipGetErrorString(e));
      st = RT4_ERR_HIP;
    } else if (n_intersections) {
      *n_intersections = cnt;
    }
  }
  (void)hipFree(d);
  (void)hipFree(dc);
  return st;
}

int rt4_debug_eval(rt4_context* ctx, int fn, const float* in, float* out, int32_t* aux, int64_t n, char* err,
                   size_t errlen) {
  if (!ctx || !in || !out || n < 0) return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  if (n == 0) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  float *din = nullptr, *dout = nullptr;
  int32_t* daux = nullptr;
  HIP_TRY(hipMalloc(&din, n * sizeof(float)));
  hipError_t e = hipMalloc(&dout, n * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&daux, n * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(din, in, n * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rt4_eval_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, 0, fn, din, dout,
                       daux, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost);
  if (e == hipSuccess && aux) e = hipMemcpy(aux, daux, n * sizeof(int32_t), hipMemcpyDeviceToHost);
  (void)hipFree(din);
  if (dout) (void)hipFree(dout);
  if (daux) (void)hipFree(daux);
  if (e != hipSuccess) {
    rt4_set_err(err, errlen, "debug_eval failed: %s", hipGetErrorString(e));
    return RT4_ERR_HIP;
  }
  return RT4_OK;
}

int rt4_debug_find_intersection(rt4_context* ctx, const float* rays, float* out, float* out_color, int64_t n,
                                char* err, size_t errlen) {
  if (!ctx || !rays || !out || !out_color || n < 0) return rt4_set_err(err, errlen, "bad argument"), RT4_ERR_ARG;
  if (!ctx->has_scene) return rt4_set_err(err, errlen, "context has no scene"), RT4_ERR_ARG;
  if (n == 0) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  float *dr = nullptr, *dout = nullptr, *dcol = nullptr;
  HIP_TRY(hipMalloc(&dr, n * 8 * sizeof(float)));
  hipError_t e = hipMalloc(&dout, n * 8 * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&dcol, n * 3 * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(dr, rays, n * 8 * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rt4_find_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, 0, ctx->d_scene,
                       dr, dout, dcol, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, dout, n * 8 * sizeof(float), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(out_color, dcol, n * 3 * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(dr);
  if (dout) (void)hipFree(dout);
  if (dcol) (void)hipFree(dcol);
  if (e != hipSuccess) {
    rt4_set_err(err, errlen, "debug_find_intersection failed: %s", hipGetErrorString(e));
    return RT4_ERR_HIP;
  }
  return RT4_OK;
}

}  // extern "C"
