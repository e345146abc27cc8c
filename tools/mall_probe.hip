// mall_probe — where are random 4-B gathers over a table of S bytes served?
//
// The trace kernel's diffuse bounce reads one float of the 2^23-entry sampler table (32 MiB) at a
// uniformly random index (rt4_trace.hip rand_drct<LUT>; shader.frag:141-158 is what the table replaces).
// gfx950 exposes no MALL (Infinity Cache) counters to rocprofv3, so this probe measures the same access
// pattern over table sizes that fit each level — 2 MiB (L2 share of one XCD), 32 MiB (the sampler
// table: over L2, under the 256 MiB MALL), 128 MiB, and 1-4 GiB (far over the MALL: HBM) — and reports
// the gather rate. Under rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum each size is one
// dispatch, so the fabric read latency per size (LEVEL / RDREQ) can be put next to the trace kernel's
// (the bench-shape PMC summaries, e.g. profiles/r05_v45/pmc_config2.json derived.ea_read_latency_cycles).
//
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/build/mall_probe tools/mall_probe.hip
// Run:   tools/build/mall_probe [gathers_per_lane]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// xorshift-multiply hash per lane; each gather's index depends on the previous value loaded only
// through a data dependency that cannot be elided (sum), not through the address, so many gathers of
// one lane are in flight at once, like the trace kernel's independent lanes.
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ table, uint32_t mask, int n_per_lane,
                                                     uint32_t seed, float* __restrict__ out) {
  uint32_t x = (blockIdx.x * blockDim.x + threadIdx.x) * 0x9E3779B9u ^ seed;
  float acc = 0.0f;
  for (int k = 0; k < n_per_lane; k++) {
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    acc += table[x & mask];
  }
  if (acc == 1234.5f) out[0] = acc;  // keeps the loads alive; never true for the zero table
}

int main(int argc, char** argv) {
  const int n_per_lane = argc > 1 ? std::atoi(argv[1]) : 256;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int blocks = cus * 32;  // 8 waves per SIMD worth of 256-lane blocks
  const uint64_t sizes_mib[] = {2, 8, 32, 64, 128, 256, 512, 1024, 4096};
  const uint64_t max_bytes = sizes_mib[sizeof(sizes_mib) / sizeof(sizes_mib[0]) - 1] << 20;
  float* table = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&table, max_bytes));
  CK(hipMalloc(&out, sizeof(float)));
  CK(hipMemset(table, 0, max_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"probe\": \"uniform random 4-B gathers\", \"blocks\": %d, \"threads\": 256, \"gathers_per_lane\": %d, "
              "\"results\": [\n",
              blocks, n_per_lane);
  bool first = true;
  for (uint64_t mib : sizes_mib) {
    const uint32_t mask = static_cast<uint32_t>((mib << 20) / sizeof(float) - 1);
    // warm (fills whatever cache level the size fits), then timed
    hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, 0, table, mask, n_per_lane, 1u, out);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(gather_kernel, dim3(blocks), dim3(256), 0, 0, table, mask, n_per_lane, 7u, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.0f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double gathers = static_cast<double>(blocks) * 256.0 * n_per_lane;
    std::printf("%s  {\"table_mib\": %llu, \"ms\": %.4f, \"G_gathers_per_s\": %.2f, \"GB_per_s_64B_lines\": %.1f}",
                first ? "" : ",\n", static_cast<unsigned long long>(mib), ms, gathers / (ms * 1e-3) / 1e9,
                gathers * 64.0 / (ms * 1e-3) / 1e9);
    first = false;
  }
  std::printf("\n]}\n");
  CK(hipFree(table));
  CK(hipFree(out));
  return 0;
}
