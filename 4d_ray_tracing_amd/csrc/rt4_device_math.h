// rt4_device_math.h — fp32 building blocks of the trace kernel (gfx950).
//
// Numerical contract: the GLSL built-ins of executable/shader.frag are given ONE
// definition here, evaluated with explicit v_fma_f32 where the contract says fma and separately
// rounded ops everywhere else. The build uses -ffp-contract=off (no silent fusion) and correctly
// rounded fp32 division/sqrt, so every value is reproducible bit for bit on the host.
//   dot(a,b) = fma(a.w,b.w, fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)))
//   vector multiply-add forms of the shader are one fma per component.
//   acos/asin: Cephes asinf kernel; sin/cos: pi/2 Cody-Waite reduction + Cephes kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rt4 {

constexpr float PI_F = 3.14159265f;   // shader.frag:23
constexpr float SMALL_F = 0.0003f;    // shader.frag:24
constexpr float PIO2_F = 1.57079637050628662109375f;
constexpr float PIO2_LO = -4.37113900018624283e-8f;
constexpr float TWO_OVER_PI = 0.636619772367581343f;
constexpr int NEWTON_CAP = 64;

struct V4 { float x, y, z, w; };
struct V3 { float x, y, z; };

__device__ __forceinline__ float fmaf_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// Native-math mode (-DRT4_NATIVE_MATH, a diagnostic build: DESIGN.md §6): the GLSL built-ins of the
// shader come from ocml (acosf, asinf, sinf, cosf) and the shader's multiply-add forms are evaluated as
// written, a*b + c with two roundings, instead of the fixed deterministic definition below. It measures
// how far the images move with the built-ins' definition, the one thing the unrunnable GL reference
// leaves open. sfma_ is a multiply-add written in the shader; fmaf_ stays an exact fma
// where an algorithm needs one (correctly rounded sqrt and quotient, conservative bounds).
#ifdef RT4_NATIVE_MATH
__device__ __forceinline__ float sfma_(float a, float b, float c) { return a * b + c; }
#else
__device__ __forceinline__ float sfma_(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
#endif

__device__ __forceinline__ V4 make4(float x, float y, float z, float w) { return V4{x, y, z, w}; }
__device__ __forceinline__ V4 ld4(const float* p) { return V4{p[0], p[1], p[2], p[3]}; }
__device__ __forceinline__ V3 ld3(const float* p) { return V3{p[0], p[1], p[2]}; }
__device__ __forceinline__ V4 add(V4 a, V4 b) { return V4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
__device__ __forceinline__ V4 sub(V4 a, V4 b) { return V4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
__device__ __forceinline__ V4 mul(V4 a, float s) { return V4{a.x * s, a.y * s, a.z * s, a.w * s}; }
__device__ __forceinline__ V4 divs(V4 a, float s) { return V4{a.x / s, a.y / s, a.z / s, a.w / s}; }
__device__ __forceinline__ V4 neg(V4 a) { return V4{-a.x, -a.y, -a.z, -a.w}; }
__device__ __forceinline__ V4 mad(V4 a, float s, V4 c) {  // a*s + c
  return V4{sfma_(a.x, s, c.x), sfma_(a.y, s, c.y), sfma_(a.z, s, c.z), sfma_(a.w, s, c.w)};
}
__device__ __forceinline__ float dot(V4 a, V4 b) {
  return sfma_(a.w, b.w, sfma_(a.z, b.z, sfma_(a.y, b.y, a.x * b.x)));
}
#ifndef RT4_FAST_SQRT
#define RT4_FAST_SQRT 1
#endif
// Correctly rounded sqrt: the same value as __builtin_sqrtf under -fhip-fp32-correctly-rounded-divide-sqrt,
// minus the library expansion's input scaling and class fix-up when no lane needs them. For |x|
// outside (0, 2^-96) the hardware estimate v_sqrt_f32 plus the one-ulp residual correction of that expansion is
// already the correctly rounded result (+-0, +inf, NaN and negative inputs included); inside, the
// library path runs. Verified against __builtin_sqrtf on all 2^32 inputs (rt4_debug_verify_sqrt).
__device__ __forceinline__ float sqrt_core(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
  const float sup = __uint_as_float(__float_as_uint(s) + 1u);
  const float rdn = fmaf_(-sdn, s, x);
  const float rup = fmaf_(-sup, s, x);
  const float r = rdn <= 0.0f ? sdn : s;
  return rup > 0.0f ? sup : r;
}
__device__ __forceinline__ float sqrt_(float x) {
#if RT4_FAST_SQRT
  // |x| in (0, 2^-96), denormals included, tested on the bit pattern: float compares may see a
  // denormal as zero
#if RT4_FAST_SQRT == 2  // per-lane branch (exec-mask save/restore around both paths)
  if ((__float_as_uint(x) & 0x7FFFFFFFu) - 1u >= 0x0F7FFFFFu) return sqrt_core(x);
#else  // wave-uniform branch: the library path only when some active lane needs it (scalar branch only)
  if (!__any((__float_as_uint(x) & 0x7FFFFFFFu) - 1u < 0x0F7FFFFFu)) return sqrt_core(x);
#endif
#endif
  return __builtin_sqrtf(x);
}
__device__ __forceinline__ float length(V4 v) { return sqrt_(dot(v, v)); }

// Division by a per-ray divisor (IEEE, correctly rounded: 11 VALU on gfx950). RT4_ABL_FASTDIV is an
// ablation build only (NOT exact): reciprocal + one residual step and no check, to bound what an
// exactness-checked fast quotient could gain at these sites (profiles/r02_ab.txt).
__device__ __forceinline__ float rdiv(float x, float b) {
#ifdef RT4_ABL_FASTDIV
  const float y = __builtin_amdgcn_rcpf(b);
  const float q = x * y;
  return fmaf_(fmaf_(-q, b, x), y, q);
#else
  return x / b;
#endif
}

// ---- transcendentals ------------------------------------------------------------------------
__device__ __forceinline__ float asin_core(float s, float z) {
  float p = fmaf_(fmaf_(fmaf_(fmaf_(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                        7.4953002686e-2f), z, 1.6666752422e-1f);
  return fmaf_(p, z * s, s);
}

#ifdef RT4_NATIVE_MATH
__device__ __forceinline__ float asin_(float x) { return asinf(x); }
__device__ __forceinline__ float acos_(float x) { return acosf(x); }
__device__ __forceinline__ float sin_(float x) { return sinf(x); }
__device__ __forceinline__ float cos_(float x) { return cosf(x); }
__device__ __forceinline__ void sincos_(float x, float& sv, float& cv) {
  sv = sinf(x);
  cv = cosf(x);
}
#else
// Branch-free form of the oracle's rt4m_asin: both arms compute the same op sequence per lane.
__device__ __forceinline__ float asin_(float x) {
  float a = __builtin_fabsf(x);
  bool big = a > 0.5f;
  float zb = 0.5f * (1.0f - a);
  float z = big ? zb : a * a;
  float s = big ? sqrt_(zb) : a;
  float c = asin_core(s, z);
  float r = big ? (PIO2_F - 2.0f * c) : c;
  return __builtin_copysignf(r, x);
}

__device__ __forceinline__ float acos_(float x) {
  float a = __builtin_fabsf(x);
  bool big = a > 0.5f;
  float zb = 0.5f * (1.0f - a);
  float z = big ? zb : x * x;
  float s = big ? sqrt_(zb) : x;
  float c = asin_core(s, z);
  float t = 2.0f * c;
  float rb = x > 0.0f ? t : PI_F - t;
  return big ? rb : PIO2_F - c;
}

__device__ __forceinline__ float sin_kernel(float r) {
  float z = r * r;
  float p = fmaf_(fmaf_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
  return fmaf_(p, z * r, r);
}
__device__ __forceinline__ float cos_kernel(float r) {
  float z = r * r;
  float p = fmaf_(fmaf_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
  return fmaf_(p, z * z, fmaf_(-0.5f, z, 1.0f));
}
__device__ __forceinline__ void reduce_pio2(float x, float& r, int& q) {
  float j = __builtin_rintf(x * TWO_OVER_PI);
  r = fmaf_(-j, PIO2_F, x);
  r = fmaf_(-j, PIO2_LO, r);
  q = (__builtin_fabsf(j) < 8388608.0f) ? (static_cast<int>(j) & 3) : 0;
}
__device__ __forceinline__ float sin_(float x) {
  float r; int q; reduce_pio2(x, r, q);
  float s = sin_kernel(r), c = cos_kernel(r);
  float v = (q & 1) ? c : s;
  return (q & 2) ? -v : v;
}
__device__ __forceinline__ float cos_(float x) {
  float r; int q; reduce_pio2(x, r, q);
  float s = sin_kernel(r), c = cos_kernel(r);
  float v = (q & 1) ? s : c;
  return ((q + 1) & 2) ? -v : v;
}
// sin and cos of the same angle share the reduction and both kernels (rand_drct, shader.frag:129).
__device__ __forceinline__ void sincos_(float x, float& sv, float& cv) {
  float r; int q; reduce_pio2(x, r, q);
  float s = sin_kernel(r), c = cos_kernel(r);
  float vs = (q & 1) ? c : s;
  float vc = (q & 1) ? s : c;
  sv = (q & 2) ? -vs : vs;
  cv = ((q + 1) & 2) ? -vc : vc;
}
#endif  // RT4_NATIVE_MATH

// ---- RNG (shader.frag:90-121) -----------------------------------------------------------------
__device__ __forceinline__ uint32_t hash_u32(uint32_t x) {  // :94-102
  x += (x << 10);
  x ^= (x >> 6);
  x += (x << 3);
  x ^= (x >> 11);
  x += (x << 15);
  x ^= (x >> 9);
  return x;
}

// ---- S^3 sampler (shader.frag:136-150) ------------------------------------------------------------
__device__ __forceinline__ float volume_by_w(float w) {  // :136-138
  return (w * sqrt_(1.0f - w * w) - acos_(w)) / PI_F + 1.0f;
}
__device__ __forceinline__ float w_by_volume(float v, int* iters) {  // :141-150
  float old_w;
  float new_w = 0.0f;
  int it = 0;
  do {
    old_w = new_w;
    float old_v = volume_by_w(old_w);
    // one volume_by_w per iteration for the finite difference: both arms of the shader's ternary
    // evaluate volume_by_w(old_w -/+ SMALL), so the selected argument is computed first.
    bool pos = old_w > 0.0f;
    float probe = volume_by_w(pos ? old_w - SMALL_F : old_w + SMALL_F);
    float df = pos ? old_v - probe : probe - old_v;
    new_w = old_w - SMALL_F / df * (old_v - v);
    ++it;
  } while (__builtin_fabsf(new_w - old_w) >= SMALL_F && it < NEWTON_CAP);
  if (iters) *iters = it;
  return new_w;
}

}  // namespace rt4
