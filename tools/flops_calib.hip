// Calibration of gfx950's FLOP counters (round 6): do SQ_INSTS_VALU_FLOPS_FP32 and
// SQ_INSTS_VALU_FLOPS_FP32_TRANS count executed lane operations (EXEC-masked) or wave instructions x 64?
// One kernel per (operation, active lanes of 64): each active lane runs ITERS dependent operations of one kind on
// its own value; inactive lanes skip the loop. Known work per dispatch: ITERS x active lanes x waves operations
// (an fma = 2 FLOP). Run under rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS
// SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU
// SQ_THREAD_CYCLES_VALU; tools/flops_calib.py compares. Build: hipcc --offload-arch=gfx950 -O3 -o flops_calib
// tools/flops_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;
constexpr int BLOCKS = 2048, THREADS = 256;

enum Op { FMA = 0, ADD = 1, MUL = 2, SQRT = 3 };

template <int OP, int EVERY>
__global__ __launch_bounds__(THREADS) void calib_kernel(float* out, float a, float b) {
  const unsigned lane = threadIdx.x & 63u;
  float x = static_cast<float>(threadIdx.x) * 1e-3f + 1.0f;
  if (lane % EVERY == 0) {
    for (int i = 0; i < ITERS; i++) {
      if constexpr (OP == FMA) x = __builtin_fmaf(x, a, b);
      else if constexpr (OP == ADD) x = x + b;
      else if constexpr (OP == MUL) x = x * a;
      else x = __builtin_amdgcn_sqrtf(x + b);
    }
  }
  out[blockIdx.x * THREADS + threadIdx.x] = x;
}

template <int OP, int EVERY>
static void run(float* d) {
  hipLaunchKernelGGL((calib_kernel<OP, EVERY>), dim3(BLOCKS), dim3(THREADS), 0, 0, d, 0.999999f, 1e-7f);
  (void)hipDeviceSynchronize();
  const long long lanes = static_cast<long long>(BLOCKS) * THREADS / EVERY;
  std::printf("op %d every %d: %lld active lanes x %d ops = %lld lane-ops\n", OP, EVERY, lanes, ITERS,
              lanes * ITERS);
}

template <int OP>
static void run_op(float* d) {
  run<OP, 1>(d);
  run<OP, 2>(d);
  run<OP, 8>(d);
  run<OP, 64>(d);
}

int main() {
  float* d = nullptr;
  if (hipMalloc(&d, sizeof(float) * BLOCKS * THREADS) != hipSuccess) return 1;
  run_op<FMA>(d);
  run_op<ADD>(d);
  run_op<MUL>(d);
  run_op<SQRT>(d);
  (void)hipFree(d);
  return 0;
}
