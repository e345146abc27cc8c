// gather_bits_probe — bytes per request of the sampler table's 4-B gathers (round 6).
//
// The trace kernel's diffuse bounce reads one float of the 2^23-entry (32 MiB) sampler table at a random index; every
// such read leaves L2 as one 64-B fabric request (TCC_EA0_RDREQ_32B = 0 in every profile). This probe replays that
// access pattern (uniformly random 4-B gathers, every CU busy, many in flight per lane) over a 32 MiB table with each
// cache-policy setting a buffer load can carry on gfx950 (cpol: sc0 = 1, nt = 2, sc1 = 16, and their combinations)
// and with the table in coarse-grained, fine-grained and uncached device memory, one dispatch per variant. Under
// rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum the request sizes and L2 hits per
// variant can be put next to the gather rate it prints.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o 4d_ray_tracing_amd/lib/gather_bits_probe tools/gather_bits_probe.hip
// Run:   4d_ray_tracing_amd/lib/gather_bits_probe [gathers_per_lane]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                            \
    }                                                                                          \
  } while (0)

constexpr uint32_t kEntries = 1u << 23;  // the sampler table's size (32 MiB of floats)

template <int CPOL>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ table, int n_per_lane, uint32_t seed,
                                                     float* __restrict__ out) {
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(table), 0, kEntries * 4u, 0x00020000);
  uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u ^ seed;
  float acc = 0.0f;
  for (int k = 0; k < n_per_lane; k++) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    acc += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, (x & (kEntries - 1u)) * 4u, 0, CPOL));
  }
  if (acc == 1234.5f) out[0] = acc;  // keeps the loads alive; never true for the zero table
}

template <int CPOL>
static void run(const char* mem, const float* table, float* out, int blocks, int n_per_lane, hipEvent_t e0,
                hipEvent_t e1) {
  hipLaunchKernelGGL(gather_kernel<CPOL>, dim3(blocks), dim3(256), 0, 0, table, n_per_lane, 1u, out);  // warm
  CK(hipEventRecord(e0));
  hipLaunchKernelGGL(gather_kernel<CPOL>, dim3(blocks), dim3(256), 0, 0, table, n_per_lane, 7u, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.0f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double gathers = static_cast<double>(blocks) * 256.0 * n_per_lane;
  std::printf("{\"memory\": \"%s\", \"cpol\": %d, \"ms\": %.4f, \"G_gathers_per_s\": %.2f}\n", mem, CPOL, ms,
              gathers / (ms * 1e-3) / 1e9);
}

int main(int argc, char** argv) {
  const int n_per_lane = argc > 1 ? std::atoi(argv[1]) : 256;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 32;
  float* out = nullptr;
  CK(hipMalloc(&out, sizeof(float)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[] = {"coarse", "fine", "uncached"};
  const unsigned flags[] = {hipDeviceMallocDefault, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
  for (int m = 0; m < 3; m++) {
    float* table = nullptr;
    CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&table), kEntries * sizeof(float), flags[m]));
    CK(hipMemset(table, 0, kEntries * sizeof(float)));
    CK(hipDeviceSynchronize());
    run<0>(names[m], table, out, blocks, n_per_lane, e0, e1);
    if (m == 0) {  // the load's cache-policy bits on the product's (coarse-grained) table
      run<1>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<2>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<3>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<16>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<17>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<18>(names[m], table, out, blocks, n_per_lane, e0, e1);
      run<19>(names[m], table, out, blocks, n_per_lane, e0, e1);
    }
    CK(hipFree(table));
  }
  CK(hipFree(out));
  return 0;
}
