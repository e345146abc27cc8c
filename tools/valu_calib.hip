// valu_calib.hip — issue-rate calibration of the gfx950 VALU (diagnostic, not part of librt4.so).
// Measures wave64 instruction throughput per SIMD for independent v_fma_f32 / v_pk_fma_f32 /
// v_sqrt_f32 / v_add_u32 streams at several waves per SIMD, to read the trace kernel's
// SQ_INSTS_VALU-based issue fraction against the real per-SIMD ceiling.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/valu_calib tools/valu_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int CHAINS = 8;
constexpr int ITERS = 4096;

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void calib(float* out, float seed) {
  float a[CHAINS];
  f2 p[CHAINS];
  unsigned u[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; c++) {
    a[c] = seed + threadIdx.x * 1e-7f + c;
    p[c] = f2{a[c], a[c] + 0.5f};
    u[c] = threadIdx.x + c;
  }
  const float m = 0.999999f, k = 1e-7f;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int c = 0; c < CHAINS; c++) {
      if (MODE == 0) a[c] = __builtin_fmaf(a[c], m, k);                       // v_fma_f32
      if (MODE == 1) p[c] = __builtin_elementwise_fma(p[c], f2{m, m}, f2{k, k});  // v_pk_fma_f32
      if (MODE == 2) a[c] = __builtin_amdgcn_sqrtf(a[c]);                      // v_sqrt_f32
      if (MODE == 3) u[c] = u[c] * 1664525u + 1013904223u;                     // v_mad_u32_u24 / mul_lo
      if (MODE == 4) u[c] = (u[c] ^ (u[c] << 3)) + 7u;                         // v_lshl_xor + v_add
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < CHAINS; c++) s += a[c] + p[c].x + p[c].y + static_cast<float>(u[c]);
  if (s == 12345.678f) out[0] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 4);
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_fma_f32", "v_pk_fma_f32", "v_sqrt_f32", "u32 mul-add (LCG)", "u32 shl-xor-add"};
  const int insts_per_op[] = {1, 1, 1, 0, 0};  // LCG / xorshift: read from the ISA, reported per op
  for (int mode = 0; mode < 5; mode++) {
    for (int waves_per_simd : {1, 2, 4, 8}) {
      const int blocks = ncu * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
      auto fn = mode == 0 ? calib<0> : mode == 1 ? calib<1> : mode == 2 ? calib<2> : mode == 3 ? calib<3> : calib<4>;
      hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      hipEventRecord(e0);
      for (int r = 0; r < 5; r++) hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double ops = 5.0 * blocks * 4.0 * CHAINS * ITERS;  // wave-level ops
      const double per_simd_per_ns = ops / (ncu * 4.0) / (ms * 1e6);
      printf("%-20s waves/SIMD %d: %.3f wave-ops/ns/SIMD (%.2f ns each)%s\n", names[mode], waves_per_simd,
             per_simd_per_ns, 1.0 / per_simd_per_ns, insts_per_op[mode] ? "" : " [several insts per op]");
    }
  }
  return 0;
}
