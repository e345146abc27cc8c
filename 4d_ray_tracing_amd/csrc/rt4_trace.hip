// rt4_trace.hip — the hot path: executable/shader.frag's per-cell trace loop as one gfx950 kernel,
// plus the device context and the C-ABI render / diagnostic entry points of include/rt4.h.
//
// Kernel shape:
//   * persistent waves over a global pixel queue. One lane traces one pixel at a time. A lane
//     whose pixel has run all its samples goes idle; once >= REFILL_MIN lanes of a wave are idle,
//     the wave writes their pixels out and hands them new pixels (ballot + mbcnt rank) from
//     64-pixel batches (8x8 tiles) claimed with one atomicAdd. Lanes stay busy until the queue
//     drains, instead of idling until the slowest pixel of a fixed 64-pixel wave is done.
//   * within a pixel the sample x bounce loops of main()/trace() (shader.frag:474, :520) are
//     FLATTENED: one loop iteration = one find_intersection + its shading. A finished path starts
//     the pixel's next sample in the next iteration. The RNG counter keeps running across samples
//     (shader.frag:92), exactly as in the shader.
//   * find_intersection is specialised per scene shape (rt4_intersect.h); scene geometry is
//     wave-uniform -> scalar loads; materials are fetched per lane at shading.
//   * optional w_by_volume table (RT4_FLAG_SAMPLER_LUT): the Newton loop of shader.frag:141-150
//     is a pure function of rand()'s 23 mantissa bits; a 2^23-entry table built by the same
//     device function replaces the divergent loop by one cached load.
#ifdef RT4_NATIVE_MATH
// Native-math diagnostic build (rt4_device_math.h): the exact shortcuts whose proofs assume the
// deterministic built-ins are compiled out, so the kernel evaluates the shader's expressions plainly.
#define RT4_SPHERE_CULL 0
#define RT4_SKY_PRETEST 0
#define RT4_SKY_THRESHOLD 0
#define RT4_BOUND_SKIP 0
#endif
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <map>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/rt4.h"
#include "rt4_device_math.h"
#include "rt4_fast.h"
#include "rt4_intersect.h"
#include "rt4_internal.h"

using namespace rt4;

namespace {

#ifndef RT4_REFILL_MIN
#define RT4_REFILL_MIN 1  // refill as soon as one lane is idle (r01 A/B: 8 -> 1 is +4.5 % sphere, +6 % hypercube, +4 % tiger)
#endif
#ifndef RT4_REFILL_MIN_OPEN
// The exact-count kernels without a tiger and without the lockstep rules (sphere, hypercube, cylinder4d): refill once
// this many lanes are idle. Since the inbox (r02), the deferred exact tests (r03) and the one-trip hand-out (r04) the
// refill's fixed cost per execution dominates its lost lanes: r05 A/B 4 / 6 / 8 against 1: config 2 -3.0 / -2.8 /
// -3.2 %, config 3 -2.2 / -2.8 / -2.7 % kernel time; the tiger kernels lose (config 4 +0.6 %, config 5 +2.2 % at 8)
// and keep RT4_REFILL_MIN (profiles/r05_ab.txt)
#define RT4_REFILL_MIN_OPEN 4
#endif
#ifndef RT4_PHASE_REFILL
// Lockstep for closed scenes. In a closed room every path runs all R + 1 bounces, so the
// lanes of a wave that start together stay in lockstep, bounce for bounce, and their rays stay coherent;
// every early miss and every refill off that beat drifts a lane out of phase for good, which over a long
// pipelined launch cost config 4 a third of its lane utilisation (38 % -> 26 %). Two rules, in the kernels
// of scenes with three or more spaces (phase_refill_of):
//   * phase-aligned refill: idle lanes of a wave with active lanes left are refilled only in an iteration
//     where some active lane starts a sample (b == 0);
//   * wave clock (RT4_WAVE_CLOCK): while almost every path of the wave runs full length, samples start only
//     every R + 1 iterations, so lanes pushed off the beat rejoin it.
// Config 4: 110.5 -> 91 ms frame by frame, 123 -> 88 ms pipelined (20 frames); open scenes lose 1-2.5 % to
// the wait (hypercube, tiger, all_primitives), so they keep the immediate refill. 3 = closed rooms (default),
// 1 = also the tiger kernels, 2 = every kernel, 0 = none (A/B knob; profiles/r03_ab.txt).
#define RT4_PHASE_REFILL 3
#endif
#ifndef RT4_LUT_PREFETCH
// When the sampler-table entry of a possible diffuse bounce is fetched: 2 = at a hit, in flight
// during resolve + shading; 0 = in rand_drct. Measured alternatives, all slower (profiles/r01_ab.txt):
// at the top of every iteration; at the top for lanes that can hit; at a hit by LDS-DMA.
#define RT4_LUT_PREFETCH 2
#endif
#ifndef RT4_SKY_THRESHOLD
#define RT4_SKY_THRESHOLD 1
#endif
using WEntry = float;  // a {w, sqrt(1 - w*w)} table was 1 % faster on sphere, 6 % slower on room (rejected)
#ifndef RT4_ABL_WLUT_STRIDE
// A/B build only (RT4_ABL_WLUT_STRIDE=16: one entry per 64-B line, a 512 MiB table that cannot stay in
// the 256 MiB Infinity Cache): where the gathers are served from (profiles/r03_ab.txt)
#define RT4_ABL_WLUT_STRIDE 1
#endif
__device__ __forceinline__ float went_w(WEntry e) { return e; }
#ifndef RT4_ORDER_PREPASS
#define RT4_ORDER_PREPASS 1  // longest-first tile order from a primary-ray pre-pass (rt4_tile_order_kernel)
#endif
#ifndef RT4_LAST_FRAME_ORDER
// The tile order of a pipelined launch's last frame (round 6, A/B knob): 0 = row-major like the other frames; 1 = its
// rows in reverse (bottom-up: in the reference's scenes the sky is at the top, so the cheapest tiles go last); 2 = the
// pre-pass's hit-first order (§4.15) for the last frame only. Only the launch's drain depends on the last frame's
// order; images and counts do not.
#define RT4_LAST_FRAME_ORDER 0
#endif
#ifndef RT4_SKY_PRETEST
#define RT4_SKY_PRETEST 1
#endif
#ifndef RT4_POOL_SPHERES
// Cross-wave pooling of the exact sphere tests (rt4_trace_kernel POOL). Bit-exact, but measured
// slower: sphere -13 %, room -7 %, all_primitives -21 % (profiles/r02_ab.txt): the four waves must
// iterate in step, and two barriers per iteration cost more than the denser tests save. Off.
#define RT4_POOL_SPHERES 0
#endif
#ifndef RT4_CLAIM_TILES
#define RT4_CLAIM_TILES 4  // 8x8 tiles per queue atomic in pipelined launches (rt4_trace_kernel CLAIM_TILES)
#endif
#ifndef RT4_CLAIM_TILES_DEFER
#define RT4_CLAIM_TILES_DEFER 4  // the same for the deferred-sphere kernel (needs its 6-wave register budget)
#endif
#ifndef RT4_WAVE_CLOCK
#define RT4_WAVE_CLOCK 1  // wave clock for the phase-refill kernels (rt4_trace_kernel CLOCK); 0 = off (A/B knob)
#endif
#ifndef RT4_DEFER_TIGER
#define RT4_DEFER_TIGER 32  // deferred tiger tests: the wave's lane threshold (rt4_trace_kernel TDEFER); 0 = off
#endif
#ifndef RT4_TIGER_SPLIT
#define RT4_TIGER_SPLIT 16  // in-wave split of the tiger test in the lockstep kernels: the most lanes split (0 = off)
#endif
#ifndef RT4_REFILL_HYPER
#define RT4_REFILL_HYPER 0  // the refill threshold of the open hypercube kernels (0: RT4_REFILL_MIN_OPEN; A/B knob)
#endif
#ifndef RT4_SAVE_HYPER
#define RT4_SAVE_HYPER 0  // the tiger kernels' register savings (RT4_WAVE_COUNT, RT4_FLUSH_REMAT) in the hypercube kernels
#endif
#ifndef RT4_REFILL_OPEN_TIGER
#define RT4_REFILL_OPEN_TIGER 2  // the refill threshold of the open tiger kernels (0: REFILL_MIN): config 5 +0.6 % at 2
                                 // (3: +0.3 %, 4: +0.25 %; r05-v51, profiles/r05_ab.txt)
#endif
#ifndef RT4_TIGER_SPLIT_REUSE
#define RT4_TIGER_SPLIT_REUSE 1  // the split in the lockstep kernels' primary-reuse instantiations too
#endif
#ifndef RT4_TIGER_SPLIT_OPEN_LDS
// round 6 (A/B knob): the open tiger kernels split through the mirror room's LDS hand-off after the deferral decides
// to run (at most RT4_TIGER_SPLIT_OPEN lanes split, more run the direct test) instead of serving over ds_bpermute
#define RT4_TIGER_SPLIT_OPEN_LDS 0
#endif
#ifndef RT4_TIGER_SPLIT_BPERM_RES
// round 6 (A/B knob): the split's quarter results go back to their owners by ds_bpermute instead of the per-wave LDS
// area (no lds_tres), so the open kernels' split fits the all_primitives kernel's LDS at 6 blocks per CU
#define RT4_TIGER_SPLIT_BPERM_RES 0
#endif
#ifndef RT4_TIGER_SPLIT_OPEN
#define RT4_TIGER_SPLIT_OPEN 0  // the same in the open tiger kernels (tiger, all_primitives)
#endif
#ifndef RT4_BEAT_SLACK
#define RT4_BEAT_SLACK 0  // in-beat tiger deferral in the lockstep kernels: parked iterations per sample (0 = off)
#endif
#ifndef RT4_DEFER_TIGER_WAIT
#define RT4_DEFER_TIGER_WAIT 6  // r05-v52: 6 (config 5 +0.4 % over 4 in 5 rounds; 3 and 12 slower; profiles/r05_ab.txt)
#endif
#ifndef RT4_DEFER_EXACT_TIGER
// Deferred exact sphere tests in the open tiger kernels (round 6; rt4_trace_kernel SDEFER): the
// wave's pending-lane threshold (0 = off) and the most iterations a lane waits. A lane whose sphere cull leaves
// pending spheres parks before any other group and redoes the cull next iteration (no state kept), as in §4.25.
#define RT4_DEFER_EXACT_TIGER 0
#endif
#ifndef RT4_DEFER_WAIT_TIGER
#define RT4_DEFER_WAIT_TIGER 4
#endif
#ifndef RT4_DEFER_EXACT
// Deferred exact sphere tests: a wave runs its pending exact sphere tests only once at
// least RT4_DEFER_EXACT of its lanes have one, or after RT4_DEFER_WAIT iterations; the lanes that wait park
// (config 2 +6 % at 32 / 4). Open scenes only: kernels without a tiger (all_primitives -0.5 %) and
// without the phase-aligned refill (the closed room -3 %); 0 = off.
#define RT4_DEFER_EXACT 32
#endif
#ifndef RT4_DEFER_WAIT
#define RT4_DEFER_WAIT 4
#endif
#ifndef RT4_LSUM_REG
#define RT4_LSUM_REG 1
#endif
#ifndef RT4_FLUSH_REMAT
#define RT4_FLUSH_REMAT 1  // the outbox path recomputes the lane / wave / sample count where it runs (r05)
#endif
#ifndef RT4_WAVE_COUNT
#define RT4_WAVE_COUNT 1  // intersection counts in a scalar register per wave (kernels without primary reuse)
#endif
#ifndef RT4_LSUM_REG_TIGER
#define RT4_LSUM_REG_TIGER 1  // the light sum in VGPRs in the tiger kernels bounded to 5 waves (r05: config 4 +1 % at 5)
#endif
#if defined(RT4_STAMPS) || defined(RT4_LANESTATS) || defined(RT4_TAILSTATS)
#define RT4_OVERLAP_FRAMES 0  // the diagnostic builds write counter[1..]: the caller's buffer, never a count slot
#endif
#ifndef RT4_OVERLAP_FRAMES
#define RT4_OVERLAP_FRAMES 1  // single-frame launches overlap the previous frame's drain
#endif
#ifndef RT4_DEFER_GEO
#define RT4_DEFER_GEO 0  // the deferred-sphere kernel keeps the cull's dots for the exact tests (r03: 1)
#endif
#ifndef RT4_REFILL_ONE_TRIP
#define RT4_REFILL_ONE_TRIP 1
#endif
#ifndef RT4_OVERLAP_GRID_LESS
// Overlapped traces of short frames (at most RT4_OVERLAP_SHORT_WORK pixel samples x (bounces + 1)) run this many
// blocks per CU fewer than the occupancy allows, so that when one frame's trace holds the chip alone the previous
// frame's fold finds free slots at once instead of waiting for that trace's drain (2 measured best: config 2
// -9 %, config 3 -10 %; a long frame, config 4, loses 5 % with it; profiles/r04_ab.txt)
#define RT4_OVERLAP_GRID_LESS 2
#endif
#ifndef RT4_OVERLAP_SHORT_WORK
#define RT4_OVERLAP_SHORT_WORK (1ull << 30)
#endif
#ifndef RT4_SIDE_LOW_PRIORITY
#define RT4_SIDE_LOW_PRIORITY 1  // overlapped traces on streams made with the least priority (measured 2-5 % faster)
#endif
#ifndef RT4_FOLD_PRIO
#define RT4_FOLD_PRIO 3  // wave priority of the fold kernel (s_setprio): overlapped frames -0.5..-0.9 % (r05-v48)
#endif
#ifndef RT4_OVERLAP_SLOTS
// Overlapped launches in flight at once: RT4_OVERLAP_SLOTS (and as many side streams) for frames too small to fill
// the chip, RT4_OVERLAP_BIG for the others (more streams than the process's four hardware queues cost a frame that
// fills the chip 4-10 %; a small frame gains from every launch in flight; profiles/r04_ab.txt)
#define RT4_OVERLAP_SLOTS 8
#endif
#ifndef RT4_OVERLAP_BIG
#define RT4_OVERLAP_BIG 3
#endif
static_assert(RT4_OVERLAP_SLOTS >= 2 && RT4_OVERLAP_SLOTS <= 8, "overlap slots");
static_assert(RT4_OVERLAP_BIG >= 2 && RT4_OVERLAP_BIG <= RT4_OVERLAP_SLOTS, "overlap slots of big frames");
// Wave bounds keep every trace kernel off scratch inside its trace loop (checked on the built
// library by tools/codegen_check.py and tests/test_codegen.py). At 6 waves/SIMD the tiger kernels ran at the
// register limit, spilling path state in the loop, and there the compiler's live-range splitting could put
// register copies ahead of a join block's EXEC restore: the lanes the restore re-enables skip the copy-out but
// run the copy-back, and receive another variable's value (the intersection count, the light sum's pixel word).
// Which build hit it depended on scheduling: the -amdgpu-sched-strategy=iterative-ilp build and a build with the
// sphere cull's && / || written as & / | computed other images and counts; the shipped one did not, by luck.
#ifndef RT4_WAVES_MIRROR
#define RT4_WAVES_MIRROR 6  // the tiger kernel specialised for three or more spaces (config 4's mirror room)
#endif
#ifndef RT4_WAVES_MIRROR_INLINE
#define RT4_WAVES_MIRROR_INLINE 6  // the same with the inline Newton sampler (5 with RT4_TIGER_CULL: one spill at 6)
#endif
#ifndef RT4_WAVES_MIRROR_REUSE
#define RT4_WAVES_MIRROR_REUSE 5  // its primary-reuse instantiations (spilled in the loop at 6)
#endif
#ifndef RT4_WAVES_ALLPRIM
#define RT4_WAVES_ALLPRIM 6  // tiger kernels with other groups (all_primitives: BASELINE config 5), sampler table
#endif
#ifndef RT4_WAVES_ALLPRIM_INLINE
#define RT4_WAVES_ALLPRIM_INLINE 5  // the same with the inline Newton sampler (spilled in the loop at 6)
#endif
#ifndef RT4_WAVES_ALLPRIM_REUSE
#define RT4_WAVES_ALLPRIM_REUSE 4  // their primary-reuse instantiations (96 VGPRs at 5 still spilled)
#endif
#ifndef RT4_WAVES_UNION_REUSE
#define RT4_WAVES_UNION_REUSE 5  // the cylinders-union kernel's primary-reuse instantiation (spilled at 6)
#endif
#ifndef RT4_WAVES_SPHERE
#define RT4_WAVES_SPHERE 7  // r04: 7 with the light sum in LDS and no kept cull dots (RT4_DEFER_GEO 0)
#endif
#ifndef RT4_WAVES_EXACT
#define RT4_WAVES_EXACT 6  // exact-count kernels without a tiger (sphere, room, hypercube, cylinder4d): 6 waves/SIMD
#endif
#ifndef RT4_WAVES_PER_SIMD
#define RT4_WAVES_PER_SIMD 1
#endif
constexpr unsigned BATCH = 64;                   // pixels per queue claim: one 8x8 tile
constexpr unsigned REFILL_MIN = RT4_REFILL_MIN;  // refill a wave once this many of its lanes are idle
constexpr uint32_t GENERIC = 0xFFFFFFFFu;
constexpr int QUEUE_SLOTS = 64;     // rotating per-launch queue words (see rt4_render_device)

// Diagnostic build only (-DRT4_STAMPS, never shipped): s_memtime stamps accumulate per-wave cycles
// per loop phase into counter[1..6] (refill, find, miss, resolve, diffuse, total). Read the shares,
// not the run time: the stamps' own waits change the schedule (cdna_hip_programming.md §7).
#ifdef RT4_STAMPS
#define RT4_STAMP(var)                          \
  do {                                          \
    __builtin_amdgcn_sched_barrier(0);          \
    var = __builtin_amdgcn_s_memtime();         \
    __builtin_amdgcn_sched_barrier(0);          \
  } while (0)
#define RT4_ACC(slot, t0)                                   \
  do {                                                      \
    unsigned long long t1_;                                 \
    RT4_STAMP(t1_);                                         \
    st[slot] += t1_ - (t0);                                 \
  } while (0)
#else
#define RT4_STAMP(var) (void)0
#define RT4_ACC(slot, t0) (void)0
#endif
// Diagnostic build only (-DRT4_LANESTATS, never shipped): per phase, wave executions and active lanes
// (popcount of exec) into counter[16 + 2p], counter[17 + 2p] (tools/lanestats.py).
#ifdef RT4_LANESTATS
#define RT4_LS(p)                                                          \
  do {                                                                     \
    ls[2 * (p)] += 1;                                                      \
    ls[2 * (p) + 1] += __popcll(__builtin_amdgcn_read_exec());             \
  } while (0)
#else
#define RT4_LS(p) (void)0
#endif

// find_intersection front-ends: the generic group loop returns a full Hit; the specialised path
// returns a candidate whose normal/material are resolved only on a hit (rt4_fast.h).
template <uint32_t K>
struct Finder {
  using R = Cand;
  static __device__ __forceinline__ Cand find(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                              const PrimEntry* P, const Ray& ray) {
    return find_cand<K>(S, X, P, ray);
  }
  static __device__ __forceinline__ Hit resolve(const PrimEntry* P, const Ray& ray, const Cand& c) {
    return rt4::resolve<K>(P, ray, c);
  }
  static __device__ __forceinline__ float refl(const rt4_scene_desc* __restrict__, const PrimEntry* P, const Cand& c) {
    return P[c.id].refl;
  }
  static __device__ __forceinline__ void material(const rt4_scene_desc* __restrict__, const PrimEntry* P, const Hit& h,
                                                  float& glow, float& refl, V3& color) {
    const PrimEntry& e = P[h.mat];
    glow = e.glow;
    refl = e.refl;
    color = V3{e.color[0], e.color[1], e.color[2]};
  }
};
template <>
struct Finder<GENERIC> {
  using R = Hit;
  static __device__ __forceinline__ Hit find(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__,
                                             const PrimEntry*, const Ray& ray) {
    return find_intersection_generic(S, ray);
  }
  static __device__ __forceinline__ Hit resolve(const PrimEntry*, const Ray&, const Hit& h) { return h; }
  static __device__ __forceinline__ float refl(const rt4_scene_desc* __restrict__ S, const PrimEntry*, const Hit& h) {
    return reinterpret_cast<const rt4_material*>(reinterpret_cast<const char*>(S) + h.mat)->refl_prob;
  }
  static __device__ __forceinline__ void material(const rt4_scene_desc* __restrict__ S, const PrimEntry*, const Hit& h,
                                                  float& glow, float& refl, V3& color) {
    const rt4_material* m = reinterpret_cast<const rt4_material*>(reinterpret_cast<const char*>(S) + h.mat);
    glow = m->glow;
    refl = m->refl_prob;
    color = V3{m->color[0], m->color[1], m->color[2]};
  }
};

// ---------------------------------------------------------------- shading (shader.frag:404-495)
__device__ __forceinline__ V3 final_light(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                         V4 drct) {  // :454-468
  const f16v h = *reinterpret_cast<const f16v*>(&X->hot_sky);  // rt4_aux.h HotSky: one wide scalar load
  if (__float_as_int(h[11]) == RT4_FINAL_LIGHT_CONSTANT) return V3{h[8], h[9], h[10]};
  const V3 sky{h[0], h[1], h[2]};
  const V4 sd{h[4], h[5], h[6], h[7]};
  const float a_ds = dot(drct, sd), l2 = dot(drct, drct);
#if RT4_SKY_PRETEST
  // clearly away from the sun: the exact v_cos below would be <= sky_c_star (rt4_aux.h sky_pre_k)
  if (l2 >= 0x1p-40f && l2 <= 0x1p40f && (a_ds <= h[12] || a_ds * a_ds < l2 * h[3])) return sky;
#endif
  // angle(), :45-50: (dot / length(drct)) / length(sun.drct); the second length is a scene constant
  const float vcos = div_c(a_ds / sqrt_(l2), X->sun_len);
  float ang = S->sun.angular_size;
#if RT4_SKY_THRESHOLD
  if (!(vcos > X->sky_c_star)) return sky;  // acos(vcos) >= ang (or NaN): the sky branch, exactly
#endif
  float deviation = acos_(vcos);
  if (deviation < ang) {
    float k = div_c(deviation, X->sun_ang), s = S->sun.sharpness;
    k = (s * s * k / (1.0f - s * k) + 1.0f) * (1.0f - k);
    float km = 1.0f - k;
    return V3{sfma_(S->sun.light[0], k, sky.x * km), sfma_(S->sun.light[1], k, sky.y * km),
              sfma_(S->sun.light[2], k, sky.z * km)};
  }
  return sky;
}

// The lane's index in its wave from mbcnt, evaluated where it stands (asm volatile: not merged with another
// evaluation, so no register carries it across the loop body; RT4_FLUSH_REMAT)
__device__ __forceinline__ unsigned rt4_lane_id() {
  unsigned l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

struct RngState {
  uint32_t base;  // bits(scr.x) ^ (bits(scr.y) << 9) ^ uint_seed   (shader.frag:106-107)
  uint32_t iter;  // rand_iter_seed                                (shader.frag:92, :105)
};

__device__ __forceinline__ uint32_t rand_bits(RngState& r) {  // 23 mantissa bits of rand(), :104-116
  r.iter += 0x79A010A9u;
  return hash_u32(r.base ^ r.iter) & 0x007FFFFFu;
}
__device__ __forceinline__ float bits_to_rand(uint32_t m) { return __uint_as_float(m | 0x3F800000u) - 1.0f; }  // :117
__device__ __forceinline__ float rand_(RngState& r) { return bits_to_rand(rand_bits(r)); }

#if RT4_LUT_PREFETCH
// Index of the sampler-table entry a diffuse bounce reads once rand_outcome's draw is consumed: the
// next rand() call (rand_drct's w, shader.frag:154). Pure function of the counter.
__device__ __forceinline__ uint32_t next_w_index(const RngState& r) {
  return hash_u32(r.base ^ (r.iter + 0x79A010A9u)) & 0x007FFFFFu;
}
#endif

// w_pre: wlut[next_diffuse_w_index()] loaded at the top of the iteration (LUT path only)
template <bool LUT>
__device__ __forceinline__ V4 rand_drct(RngState& rng, const WEntry* __restrict__ wlut, WEntry w_pre) {  // :153-158
  float w, r;
  if (LUT) {
#if RT4_LUT_PREFETCH
    rng.iter += 0x79A010A9u;  // the w draw: its value was prefetched
    const WEntry e = w_pre;
#else
    const WEntry e = wlut[rand_bits(rng) * RT4_ABL_WLUT_STRIDE];
#endif
    w = went_w(e);
    r = sqrt_(1.0f - w * w);
  } else {
    w = w_by_volume(rand_(rng), nullptr);
    r = sqrt_(1.0f - w * w);
  }
  const float z = (rand_(rng) * 2.0f - 1.0f) * r;
  const float rr = sqrt_(r * r - z * z);
  const float fi = rand_(rng) * 2.0f * PI_F;
  float sf, cf;
  sincos_(fi, sf, cf);
  return V4{rr * cf, rr * sf, z, w};
}

// One image of a launch: the whole frame, or one section of ThreeWindowGroup (rt4_render_sections_device).
struct JobArgs {
  float resolution[2], mtr_sizes[2];
  float vec_to_mtr[4], top_drct[4], right_drct[4];
  rt4_region reg;
  void* frame;
  int64_t row_stride_px;
  unsigned tile_base;  // first queue tile of the job (8x8 tiles, row-major inside the job)
  unsigned tiles_x;
  unsigned fc_base;    // an overlapped sections launch: the section's first pixel in the frame-colour slot (else 0)
};
struct KernelArgs {
  // uniforms every job shares (one shader, one frame: rt4_check_jobs)
  int32_t seed, samples, reflections_amount;
  float small_indent, part, k;  // k = light_to_color_conversion_coefficient
  float focus[4];
  int32_t format, n_jobs;
  unsigned total;  // 64 x tiles of all jobs
  const unsigned* order;  // queue position -> tile (rt4_tile_order_kernel), or null: row-major
  const unsigned* order_ends;  // the pre-pass's {hit, sky} tile counts (with order)
  unsigned long long* eval_counter;  // evaluated find_intersection calls (primary-reuse launches), or null
  JobArgs jobs[RT4_MAX_SECTIONS];
  // Frames pipelined in one launch (rt4_render_frames_device): n_frames > 1 runs n_frames frames of job 0
  // through one queue (queue item = frame x tile), frame f with seed frame_seed[f]; a finished pixel's
  // tone-mapped colour goes to fcolor[f] and rt4_fold_frames_kernel blends the frames in order
  // (frame_part[f]) into the frame buffer afterwards. Pixel words then pack j | i << 13 | f << 26.
  int32_t n_frames;
  unsigned frame_tiles;  // tiles per frame
  float4* fcolor;        // n_frames x reg.h x reg.w; also set (n_frames 1) for an overlapped launch: one image per section
  int32_t frame_seed[RT4_MAX_FRAMES];
  float frame_part[RT4_MAX_FRAMES];
};

__device__ __forceinline__ int region_row(const rt4_region& r, int i) {
  return r.band_rows > 0 ? r.y0 + (i / r.band_rows) * r.band_step + (i % r.band_rows) : r.y0 + i;
}

// A lane's pixel, packed into one dword of its cold state: region-local j (16 bits) | i (14) | job (2);
// when the pixels go to the frame-colour scratch (KernelArgs::fcolor) j (13) | i (13) | frame (6), where an overlapped
// sections launch puts the section in the frame field.
__device__ __forceinline__ int pack_pixel(int j, int i, int job) { return j | (i << 16) | (job << 30); }
__device__ __forceinline__ int pack_pixel_f(int j, int i, int f) { return j | (i << 13) | (f << 26); }

// A specialised-kernel candidate in one float4 (the primary-ray cache of RT4_FLAG_PRIMARY_REUSE).
__device__ __forceinline__ float4 pack_cand(const Cand& c) {
  return make_float4(c.dist, c.sdist, __uint_as_float((c.hit ? 1u : 0u) | (c.flip ? 2u : 0u) | (c.id << 2)), 0.0f);
}
__device__ __forceinline__ Cand unpack_cand(float4 v) {
  const uint32_t m = __float_as_uint(v.z);
  return Cand{(m & 1u) != 0u, (m & 2u) != 0u, v.x, v.y, m >> 2};
}

typedef _Float16 h4v __attribute__((ext_vector_type(4)));

// light /= samples; light_to_color (shader.frag:522-526)
template <bool REMAT = false>
__device__ __forceinline__ V3 tone_map(const KernelArgs& a, V3 light) {
  int samples = a.samples;
  // converted where it is used: a conversion hoisted out of the trace loop holds a VGPR across it for the once-per-
  // pixel write (spilled in the register-bound kernels; RT4_FLUSH_REMAT)
  if (REMAT) asm volatile("" : "+s"(samples));
  const float ns = static_cast<float>(samples);
  light = V3{light.x / ns, light.y / ns, light.z / ns};
  const float k = a.k;
  return V3{1.0f - 1.0f / sfma_(k, light.x, 1.0f), 1.0f - 1.0f / sfma_(k, light.y, 1.0f),
            1.0f - 1.0f / sfma_(k, light.z, 1.0f)};
}

// mix(old_frame, c, part), alpha 1 (shader.frag:527), per frame format (rt4.h rt4_frame_format; the
// blend is fp32 in every format, then the stored value is rounded). Shared by write_pixel and the
// fold of pipelined frames, so both run the same ops.
__device__ __forceinline__ float4 blend_f32(V3 c, float part, float4 old) {
  const float keep = 1.0f - part;
  return make_float4(sfma_(c.x, part, old.x * keep), sfma_(c.y, part, old.y * keep), sfma_(c.z, part, old.z * keep),
                     1.0f);
}
__device__ __forceinline__ h4v blend_f16(V3 c, float part, h4v o) {
  const float keep = 1.0f - part;
  // the fp32 blend, THEN the rounding to half: the empty asm keeps the backend from fusing the fma
  // and the conversion into v_fma_mixlo_f16, which rounds once (differs from the contract in the
  // last half ulp: seen after 256 progressive frames of BASELINE config 5)
  float b0 = sfma_(c.x, part, static_cast<float>(o[0]) * keep);
  float b1 = sfma_(c.y, part, static_cast<float>(o[1]) * keep);
  float b2 = sfma_(c.z, part, static_cast<float>(o[2]) * keep);
  asm volatile("" : "+v"(b0), "+v"(b1), "+v"(b2));
  h4v v;
  v[0] = static_cast<_Float16>(b0);
  v[1] = static_cast<_Float16>(b1);
  v[2] = static_cast<_Float16>(b2);
  v[3] = static_cast<_Float16>(1.0f);
  return v;
}
__device__ __forceinline__ uint32_t blend_u8(V3 c, float part, uint32_t o) {
  const float keep = 1.0f - part;
  const float oc[3] = {static_cast<float>(o & 0xFFu) / 255.0f, static_cast<float>((o >> 8) & 0xFFu) / 255.0f,
                       static_cast<float>((o >> 16) & 0xFFu) / 255.0f};
  const float nc[3] = {sfma_(c.x, part, oc[0] * keep), sfma_(c.y, part, oc[1] * keep), sfma_(c.z, part, oc[2] * keep)};
  uint32_t v = 0xFF000000u;
  for (int q = 0; q < 3; q++) v |= static_cast<uint32_t>(fminf(fmaxf(nc[q], 0.0f), 1.0f) * 255.0f + 0.5f) << (8 * q);
  return v;
}

// The pixel's light sum, tone-mapped and blended into the launch's frame (shader.frag:522-527).
template <bool REMAT>
__device__ __forceinline__ void write_pixel(const KernelArgs& a, const JobArgs& J, int pk, V3 light) {
  const int j = pk & 0xFFFF, i = (pk >> 16) & 0x3FFF;
  const V3 c = tone_map<REMAT>(a, light);
  const float part = a.part;
  char* base = static_cast<char*>(J.frame);
  const int64_t at = static_cast<int64_t>(i) * J.row_stride_px + j;
  if (a.format == RT4_FRAME_RGBA16F) {
    h4v* px = reinterpret_cast<h4v*>(base) + at;
    *px = blend_f16(c, part, *px);
  } else if (a.format == RT4_FRAME_RGBA8) {
    uint32_t* px = reinterpret_cast<uint32_t*>(base) + at;
    *px = blend_u8(c, part, *px);
  } else {
    float4* px = reinterpret_cast<float4*>(base) + at;
    *px = blend_f32(c, part, *px);
  }
}

// Waves per SIMD the register allocator must leave room for (measured, profiles/r02_ab.txt, r03_ab.txt): the
// tiger kernels with other groups (all_primitives, ~107 VGPRs -> 4 waves) ran faster at 5 with a small
// spill (+3.7 % on config 5), and since the deferred tiger tests at 6 (+2.9 %, r03-v40); the tiger kernel
// specialised for three or more spaces (the mirror room of
// config 4) at 6 (+2.3 %); the one-space tiger kernel and everything else keep the allocator's choice
// (a 6-wave bound costs the one-space tiger 1.2 %).
constexpr int min_waves_of(uint32_t K, bool reuse = false, bool lut = true) {
  if (K == GENERIC) return RT4_WAVES_PER_SIMD;
  if (!(K & K_TIGER)) {
    if ((K >> 8) == 0) return RT4_WAVES_PER_SIMD;  // runtime counts
    // the one-space sphere kernel (BASELINE config 2): 7 waves since r04 (72 VGPRs, no spill in the loop) with
    // its light sum in LDS and the exact tests recomputing the cull's dots: +3-4 % over r03-v40's 6 waves (80
    // VGPRs), which had beaten 7 waves with the light sum in VGPRs (claim state spilled 48 B/lane; r03_ab.txt).
    // The hypercube kernel -1.3 % at 7 (profiles/r02_ab.txt)
    if ((K & 0xFFu) == (K_SPACES | K_SPHERES) && ((K >> 8) & 0xFFu) == 2) return reuse ? 6 : RT4_WAVES_SPHERE;
    if (reuse && (K & K_UNION)) return RT4_WAVES_UNION_REUSE;
    return reuse ? 6 : RT4_WAVES_EXACT;  // exact-count shapes (SH() fields)
  }
  // the tiger kernels: the bound at which each instantiation runs its trace loop without scratch
  if ((K >> 8) == 0) return RT4_WAVES_PER_SIMD;  // runtime counts: the allocator's choice (no spill)
  if (K & (K_SPHERES | K_CYLINDERS | K_UNION | K_HYPERCUBE))
    return reuse ? RT4_WAVES_ALLPRIM_REUSE : (lut ? RT4_WAVES_ALLPRIM : RT4_WAVES_ALLPRIM_INLINE);
  if (((K >> 8) & 0xFFu) >= 4)  // SH(): space count + 1, bits 8..15
    return reuse ? RT4_WAVES_MIRROR_REUSE : (lut ? RT4_WAVES_MIRROR : RT4_WAVES_MIRROR_INLINE);
  return RT4_WAVES_PER_SIMD;
}

// Phase-aligned refill for this kernel (RT4_PHASE_REFILL): scenes with a tiger or >= 3 spaces (closed rooms).
constexpr bool phase_refill_of(uint32_t K) {
  if (RT4_PHASE_REFILL == 0) return false;
  if (RT4_PHASE_REFILL == 2) return true;
  const bool rooms = K != GENERIC && (K & K_SPACES) && ((K >> 8) & 0xFFu) >= 4;  // >= 3 spaces: closed rooms
  return RT4_PHASE_REFILL == 3 ? rooms : rooms || (K != GENERIC && (K & K_TIGER));
}

template <uint32_t K, bool LUT, bool REUSE>
__global__ __launch_bounds__(256, min_waves_of(K, REUSE, LUT)) void rt4_trace_kernel(const rt4_scene_desc* __restrict__ S,
                                                        const SceneAux* __restrict__ X, const KernelArgs a,
                                                        unsigned long long* __restrict__ counter,
                                                        const WEntry* __restrict__ wlut, unsigned* __restrict__ queue,
                                                        unsigned* __restrict__ queue_next) {
  const unsigned lane = threadIdx.x & 63u;
  // the next launch's queue word starts at zero (launches of a context are ordered, launch_jobs):
  // no memset between frames
  if (blockIdx.x == 0 && threadIdx.x == 0) *queue_next = 0u;
  const unsigned total = a.total;
  const V4 focus = ld4(a.focus);
  const float indent = a.small_indent;
  const int R = a.reflections_amount, NS = a.samples;
  const uint32_t useed = static_cast<uint32_t>(a.seed);
  // Longest-first order only when the pre-pass found sky tiles: with every tile a hit, its order is
  // row-major scrambled by the atomics, which cost all_primitives 20 % (row-major kept instead).
  const unsigned* order = a.order && a.order_ends[1] != 0u ? a.order : nullptr;
  // the primitive table (normals + materials of hits) is read per lane: stage it in LDS once
  // (+ hypercube 0's cells ahead of it, rt4_fast.h HYPER_CELLS_LDS)
  constexpr int CELLS4 = (K != GENERIC && (K & K_HYPERCUBE)) ? HYPER_CELLS_LDS : 0;
  __shared__ float4 lds_prims[K == GENERIC ? 1 : CELLS4 + n_prims_of(K) * 6];
  if constexpr (K != GENERIC) {
    const float4* cells = reinterpret_cast<const float4*>(X->hyper_cells);
    for (int t = threadIdx.x; t < CELLS4; t += blockDim.x) lds_prims[t] = cells[t];
    const float4* src = reinterpret_cast<const float4*>(X->prims);
    const int n4 = X->n_prims * 6;
    for (int t = threadIdx.x; t < n4; t += blockDim.x) lds_prims[CELLS4 + t] = src[t];
    __syncthreads();
  }
  const PrimEntry* P = reinterpret_cast<const PrimEntry*>(lds_prims + CELLS4);

  // Cross-wave pooling of the exact sphere tests: in the specialised kernels with
  // spheres, the four waves of a workgroup iterate in step; each iteration every wave publishes the
  // rays of its lanes with pending spheres (find_pre's cull) and the (lane, sphere) pairs, and after a
  // barrier the workgroup's 256 lanes evaluate the pooled pairs densely (one pair per lane) instead
  // of each wave running the ~190-instruction test on the ~14 of its 64 lanes that need it. Results
  // are combined by each ray's own lane in sphere index order (closest(), shader.frag:440-441), so
  // the bits do not change. Up to PCAP lanes per wave are pooled; the rest test their spheres locally.
  constexpr bool POOL = RT4_POOL_SPHERES && K != GENERIC && (K & K_SPHERES) && sh_count(K, 2) != 0;
  constexpr int NSH = POOL ? static_cast<int>(sh_count(K, 2)) - 1 : 1;
  constexpr int PCAP = 32, QCAP = POOL ? PCAP * NSH : 1;
  __shared__ float4 lds_pray[POOL ? 4 * PCAP * 2 : 1];  // pooled rays: {point, drct} per slot
  __shared__ uint16_t lds_pair[POOL ? 4 * QCAP : 1];   // slot | sphere << 6
  __shared__ float2 lds_pres[POOL ? 4 * QCAP : 1];     // {dist, hit | flip << 1}
  __shared__ uint4 lds_pn4;                            // pairs of each wave | busy << 31, one word per wave
  uint32_t* const lds_pn = reinterpret_cast<uint32_t*>(&lds_pn4);
  const unsigned wave = threadIdx.x >> 6;
  // Deferred exact sphere tests (A/B knob RT4_DEFER_EXACT = the wave's pending-lane threshold, 0 = off;
  // RT4_DEFER_WAIT = the most iterations a parked lane waits): DESIGN.md §9, profiles/r03_ab.txt
  // (not in the native-math build: the deferral runs find_pre's cull, whose exactness bound assumes the
  // deterministic fused dot that build un-fuses)
  constexpr bool DEFER = RT4_SPHERE_CULL && RT4_DEFER_EXACT > 0 && !POOL && !REUSE && K != GENERIC && (K & K_SPHERES) && !(K & K_TIGER) &&
                         !phase_refill_of(K) && sh_count(K, 2) != 0;
  constexpr bool PHASE = phase_refill_of(K);
  constexpr unsigned REFILL_K =
      K != GENERIC && (K >> 8) != 0 && !PHASE && !REUSE && (RT4_REFILL_OPEN_TIGER > 0 || !(K & K_TIGER))
          ? static_cast<unsigned>((K & K_TIGER) ? RT4_REFILL_OPEN_TIGER
                                                : ((K & K_HYPERCUBE) && RT4_REFILL_HYPER > 0 ? RT4_REFILL_HYPER
                                                                                              : RT4_REFILL_MIN_OPEN))
                                                                          : REFILL_MIN;
  int defer_age = 0;  // wave-uniform: iterations since the wave's parked lanes were first parked
  // Wave clock (closed scenes): while almost every path of the wave runs all R + 1 bounces
  // (early ends <= 1/32 of the sample ends, a leaky count), samples start only every R + 1 iterations, so
  // the lanes stay in lockstep bounce for bounce however long the launch; otherwise the phase rule above.
  constexpr bool CLOCK = PHASE && RT4_WAVE_CLOCK;
  unsigned wave_it = 0;             // wave-uniform: iteration index mod (R + 1)
  unsigned n_early = 0, n_full = 0;  // wave-uniform: sample ends before / at the bounce limit (leaky)
  bool hold = false;                 // the lane's next sample waits for the next clock boundary
  bool use_cached = false;           // REUSE: the lane's next find is its pixel's cached primary candidate
  // Deferred tiger tests (open scenes with a tiger): a lane whose ray reaches the tiger's
  // bounding ball keeps its candidate of every other group (cold[512], pack_cand) and waits until at least
  // RT4_DEFER_TIGER lanes of the wave need the tiger test, or RT4_DEFER_TIGER_WAIT iterations; then the
  // tiger runs last, as in find_rest (closest(tiger, the rest): the same bits).
  // In-beat deferral (RT4_BEAT_SLACK = D > 0): the lockstep kernels defer too, with the wave
  // clock's period stretched to R + 1 + D iterations and each lane allowed at most D parked iterations per sample,
  // so a lane that parks still ends its sample within the period and keeps the beat.
  constexpr int BEAT_SLACK = PHASE && CLOCK ? RT4_BEAT_SLACK : 0;
  constexpr bool TDEFER = RT4_DEFER_TIGER > 0 && !REUSE && K != GENERIC && (K & K_TIGER) && (!PHASE || BEAT_SLACK > 0);
  int slack = BEAT_SLACK;            // BEAT_SLACK: the lane's parked iterations left in this sample
  // Deferred exact sphere tests next to the deferred tiger (RT4_DEFER_EXACT_TIGER > 0): the open tiger kernels with
  // spheres (all_primitives, BASELINE config 5) split find_cand<K, false> into find_pre (spaces + sphere cull), the
  // pending exact tests and find_rest without the tiger, the same ops in the same order; a lane with pending spheres
  // parks until RT4_DEFER_EXACT_TIGER lanes of the wave have some, or RT4_DEFER_WAIT_TIGER iterations (defer_age).
  constexpr bool SDEFER = RT4_DEFER_EXACT_TIGER > 0 && RT4_SPHERE_CULL && TDEFER && !PHASE && !REUSE && K != GENERIC &&
                          (K & K_SPHERES) && sh_count(K, 2) != 0;
  // In-wave split of the tiger test (RT4_TIGER_SPLIT = the most lanes split, 0 = off): when at
  // most that many lanes of the wave need the tiger test in an iteration, each one's test is cut into its four
  // (axes pair, radius) quarters (rt4_fast.h tiger_quarter), run on four lanes at once through a per-wave LDS
  // hand-off, and folded back in tiger_cand's order: the same bits, on up to 4x the lanes. Lockstep kernels (the
  // mirror room, where lanes may not park for a deferral) and, with RT4_TIGER_SPLIT_OPEN, the open ones.
  // (with primary reuse only in the lockstep kernels: a lane whose bounce 0 comes from the cache takes no part)
  constexpr bool TSPLIT = (!REUSE || (CLOCK && RT4_TIGER_SPLIT_REUSE)) && K != GENERIC && (K & K_TIGER) &&
                          (PHASE ? RT4_TIGER_SPLIT > 0 : RT4_TIGER_SPLIT_OPEN > 0);
  constexpr unsigned TSPLIT_MAX = PHASE ? RT4_TIGER_SPLIT : RT4_TIGER_SPLIT_OPEN;
  // Open tiger kernels (TDEFER and TSPLIT): a run serves at most TSPLIT_MAX lanes, the parked ones first, and the
  // others stay parked, so every test runs split and the direct test is not compiled. Their rays and results move by
  // ds_bpermute (no LDS buffer: the all_primitives kernel's LDS allows no more at 6 blocks per CU). Bit-exact
  // (tools/variant_probe.py) but rejected (profiles/r05_ab.txt, r05-v48 trial): the per-lane pair geometry takes
  // ~40 VGPRs, so the kernel spills at 6 waves and runs 5 (-6.9 % config 5, 20 B spill) or 4 (-12 %, no spill).
  constexpr bool TSERVE = TSPLIT && TDEFER && !PHASE && !RT4_TIGER_SPLIT_OPEN_LDS;
  static_assert(!TSPLIT || TSPLIT_MAX <= 16, "one pass of four quarters per test");
  constexpr bool TRES_LDS = TSPLIT && !TSERVE && !(RT4_TIGER_SPLIT_BPERM_RES && !PHASE);
  __shared__ float4 lds_tray[TSPLIT && !TSERVE ? 4 * 2 * TSPLIT_MAX : 1];  // per wave: up to TSPLIT_MAX rays {point, drct}
  __shared__ float4 lds_tres[TRES_LDS ? 4 * 4 * TSPLIT_MAX : 1];  // per wave: 4 quarter results per test (pack_cand)
  __shared__ uint32_t lds_town[TSERVE ? 4 * 16 : 1];            // per wave: the lane of each served test
  bool tparked = false;              // TDEFER: the lane waits for the tiger test with its candidate in cold[512]
  int tdefer_age = 0;                // TDEFER, wave-uniform
  auto clock_on = [&]() { return n_early * 32u <= n_full; };

  bool exhausted = false;
  bool active = false, pending = false;
  RngState rng{0u, 0u};
  Ray ray{V4{0.0f, 0.0f, 0.0f, 0.0f}, V4{0.0f, 0.0f, 0.0f, 0.0f}};
  V3 acc{0.0f, 0.0f, 0.0f}, T{1.0f, 1.0f, 1.0f};
  // Cold per-lane state in LDS, one float4 column per lane (ds_read/write_b128, conflict-free):
  // [0] the pixel's primary direction d0, [256] {light sum, pack_pixel()}. Touched once per sample,
  // so the VGPRs go to occupancy instead (6 -> 7 waves/SIMD on the sphere scene).
  // [512]: the pixel's primary candidate (RT4_FLAG_PRIMARY_REUSE; pack_cand)
  __shared__ float4 lds_cold[(REUSE || TDEFER ? 3 : 2) * 256];
  float4* const cold = lds_cold + threadIdx.x;
  // RT4_LSUM_REG (specialised kernels without a tiger or a hypercube): {light sum, pack_pixel()} stays
  // in 4 VGPRs instead of cold[256], so the end of a sample is three register adds instead of an LDS
  // round trip. Measured (profiles/r02_ab.txt): sphere scene +1.2 %; the hypercube kernel -2.6 % (same
  // 6 waves/SIMD, worse allocation); the tiger kernels have no VGPRs to spare at their wave bounds.
  // (not in the deferred-sphere kernel since r04: its light sum in LDS and the exact tests recomputing the
  // cull's dots (DEFER_GEO) bring it to 72 VGPRs, 7 waves/SIMD with no spill in the loop: config 2 +3-4 %,
  // profiles/r04_ab.txt)
  constexpr bool LSUM_REG = (RT4_LSUM_REG && K != GENERIC && !(K & (K_TIGER | K_HYPERCUBE)) && !(DEFER && !RT4_DEFER_GEO)) ||
                            (RT4_LSUM_REG_TIGER && K != GENERIC && (K & K_TIGER) && !REUSE && min_waves_of(K, REUSE, LUT) <= 5);
  float4 lsum_reg = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  auto lsum_load = [&]() -> float4 {
    if constexpr (LSUM_REG) return lsum_reg;
    else return cold[256];
  };
  auto lsum_store = [&](float4 v) {
    if constexpr (LSUM_REG) lsum_reg = v;
    else cold[256] = v;
  };
  // Per-wave pixel I/O staged in LDS, 64 entries per wave:
  //   inbox: when the wave claims a 64-pixel batch (one 8x8 tile of one job), all 64 lanes set up the
  //     batch's pixels at once (scr_coord, RNG base, primary direction: shader.frag:501-505, :515-516);
  //     an idle lane starts a pixel by reading its entry ({d0}, {RNG base, pack_pixel or ~0 = none}).
  //   outbox: a lane whose pixel has run all its samples appends {light sum, pack_pixel} to the wave's
  //     ring; the wave writes the ring out 64 pixels at a time (old_frame read, tone map, blend:
  //     shader.frag:522-527), so the old_frame load latency and the write arithmetic are paid once per
  //     64 pixels with every lane busy, instead of per pixel on one or two lanes.
  __shared__ float4 lds_in_d0[256];
  __shared__ uint2 lds_in_px[256];
  __shared__ float4 lds_out[256];
  const unsigned wbase = threadIdx.x & ~63u;
  // RT4_FLUSH_REMAT (the tiger kernels): the outbox (retire, flush_ring: once per finished pixel / per 64) takes the
  // wave's first thread from a scalar register and the lane from mbcnt where it runs, so no VGPR keeps them (or their
  // LDS addresses) live across the tiger test, the loop's register peak; there they were spilled. The sphere and
  // hypercube kernels measured 1.4 % / 5.7 % slower with it (profiles/r05_ab.txt) and keep the plain form.
  constexpr bool REMAT = RT4_FLUSH_REMAT && K != GENERIC && ((K & K_TIGER) || (RT4_SAVE_HYPER && (K & K_HYPERCUBE)));
  const unsigned wave_s = __builtin_amdgcn_readfirstlane(wbase);
  unsigned in_next = 64;  // wave-uniform: next inbox entry to hand out (64: empty)
  // RT4_CLAIM_TILES > 1: one atomic claims that many consecutive tiles; the spare ones are used in turn.
  // A spare position past the end of the queue reports it exhausted like a fresh claim.
  // wave-uniform: the position after the last claimed tile | the claimed tiles not handed out yet (queue
  // positions are multiples of BATCH, so the count fits in the low bits)
  unsigned spare = 0;
  // Tiles per queue atomic: fewer round trips to the one contended queue word. Measured
  // (profiles/r03_ab.txt): hypercube +3.7 % at 2, all_primitives +4.6 % and the mirror room +1.4 % at 4,
  // but the sphere kernel with deferred exact tests -5..-7 %: it keeps one.
  constexpr unsigned CLAIM_TILES = static_cast<unsigned>(DEFER ? RT4_CLAIM_TILES_DEFER : RT4_CLAIM_TILES);
  uint32_t in_seed = useed;  // wave-uniform: the seed of the inbox's frame
  unsigned ring_n = 0;    // wave-uniform: outbox entries waiting to be written
  int s = 0, b = 0;
  uint32_t n_inter = 0, n_eval = 0;  // find_intersection calls of the reference / evaluated here (per lane, REUSE)
  // Without primary reuse every counted call is evaluated and a lane adds at most one per iteration: the wave
  // counts them in a wave-uniform (scalar) register from one ballot per iteration instead of a VGPR per lane,
  // which frees a register in the register-bound tiger kernels (RT4_WAVE_COUNT).
  constexpr bool WAVE_COUNT = RT4_WAVE_COUNT && !REUSE && K != GENERIC && ((K & K_TIGER) || (RT4_SAVE_HYPER && (K & K_HYPERCUBE)));
  unsigned long long w_inter = 0;

#ifdef RT4_LANESTATS
  unsigned long long ls[20] = {};
  rt4_ls_counter = counter;  // every thread stores the same pointer
#endif
#ifdef RT4_STAMPS
  unsigned long long st[6] = {0, 0, 0, 0, 0, 0}, t_loop0, t_ph;
  RT4_STAMP(t_loop0);
#endif
#ifdef RT4_TAILSTATS  // diagnostic build only (tools/tailstats.py): per-wave start / queue-empty / exit times
  const unsigned long long tail_t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long tail_exh = 0;
#endif
  // Writes the outbox ring (lane q takes entry q); one wave-uniform pass per job, so every job's frame
  // pointer and stride stay scalar.
  auto flush_ring = [&]() {
    const unsigned fl = REMAT ? rt4_lane_id() : lane;
    if (fl < ring_n) {
      const float4 lp = lds_out[(REMAT ? wave_s : wbase) + fl];
      const int pk = __float_as_int(lp.w);
#ifdef RT4_GUARD_WRITES  // diagnostic builds only (tools/variant_probe.py): drop a pixel word outside the launch
      const unsigned gj = a.fcolor ? pk & 0x1FFF : pk & 0xFFFF, gi = a.fcolor ? (pk >> 13) & 0x1FFF : (pk >> 16) & 0x3FFF;
      const unsigned gq = a.fcolor ? (pk >> 26) & 0x3F : (pk >> 30) & 3;
      const unsigned gn = a.fcolor && a.n_jobs == 1 ? static_cast<unsigned>(a.n_frames) : static_cast<unsigned>(a.n_jobs);
      const rt4_region& grg = a.jobs[gq < static_cast<unsigned>(a.n_jobs) ? gq : 0].reg;
      if (gq < gn && gj < static_cast<unsigned>(grg.w) && gi < static_cast<unsigned>(grg.h)) {
#endif
      if (a.fcolor) {
        // pipelined or overlapped frames: the light sum of frame f as is; rt4_fold_frames_kernel tone-maps and
        // blends
        const unsigned j = pk & 0x1FFF, i = (pk >> 13) & 0x1FFF, f = (pk >> 26) & 0x3F;  // < 2^28 pixels (4 GiB)
        if (a.n_jobs == 1) {  // f: the frame of a pipelined launch
          const rt4_region& rg = a.jobs[0].reg;
          a.fcolor[(f * static_cast<unsigned>(rg.h) + i) * static_cast<unsigned>(rg.w) + j] = lp;
        } else {  // f: the section of an overlapped sections launch
          for (int jb = 0; jb < a.n_jobs; jb++)
            if (f == static_cast<unsigned>(jb))
              a.fcolor[a.jobs[jb].fc_base + i * static_cast<unsigned>(a.jobs[jb].reg.w) + j] = lp;
        }
      } else {
        for (int jb = 0; jb < a.n_jobs; jb++)
          if (((pk >> 30) & 3) == jb) write_pixel<REMAT>(a, a.jobs[jb], pk, V3{lp.x, lp.y, lp.z});
      }
#ifdef RT4_GUARD_WRITES
      }
#endif
    }
    ring_n = 0;
  };
  // Moves the finished pixels of the pending lanes into the ring (writing the ring out first when they
  // would not fit).
  auto retire = [&]() {
    const unsigned long long pm = __ballot(pending);
    if (pm) {
      const unsigned np = static_cast<unsigned>(__popcll(pm));
      if (ring_n + np > 64u) flush_ring();
      if (pending) {
        const unsigned r = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(pm >> 32),
                                                     __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(pm), 0u));
        lds_out[(REMAT ? wave_s : wbase) + ring_n + r] = lsum_load();
        pending = false;
      }
      ring_n += np;
    }
  };
  // Claims the next 64-pixel batch and fills the inbox (all lanes; wave-uniform control). False when
  // the queue is exhausted.
  auto claim_batch = [&]() -> bool {
    unsigned base = 0;
    if (CLAIM_TILES > 1 && (spare & (BATCH - 1u)) != 0u) {  // the next tile of the last claim: no atomic
      base = spare & ~(BATCH - 1u);
      spare += BATCH - 1u;  // the next position, one tile fewer
    } else {
      // several tiles per claim only in pipelined launches and before their last frame, so the drain at
      // the end of the launch still hands out single tiles
      const unsigned nt =
          (CLAIM_TILES > 1 && a.n_frames > 1 && (spare & ~(BATCH - 1u)) + a.frame_tiles * BATCH < total) ? CLAIM_TILES
                                                                                                         : 1u;
      if (lane == 0) base = atomicAdd(queue, BATCH * nt);
      base = __builtin_amdgcn_readfirstlane(base);
      spare = (base + BATCH) | (nt - 1u);
    }
    if (base >= total) return false;
    // a 64-pixel batch is one tile of one job (of one frame): wave-uniform here (scalar loads)
    unsigned pos = base >> 6, frame = 0;
    if (a.n_frames > 1) {
      frame = pos / a.frame_tiles;
      pos -= frame * a.frame_tiles;
      in_seed = static_cast<uint32_t>(a.frame_seed[frame]);
    }
    const bool last = a.n_frames <= 1 || frame + 1u == static_cast<unsigned>(a.n_frames);  // wave-uniform
    if (RT4_LAST_FRAME_ORDER == 1 && a.n_frames > 1 && last && a.n_jobs == 1) pos = a.frame_tiles - 1u - pos;
    const unsigned btile = order && (RT4_LAST_FRAME_ORDER != 2 || last) ? order[pos] : pos;
    const int job = (a.n_jobs > 1 && btile >= a.jobs[1].tile_base) + (a.n_jobs > 2 && btile >= a.jobs[2].tile_base);
    const JobArgs& J = a.jobs[job];
    const unsigned tile = btile - J.tile_base;
    const int jj = static_cast<int>((tile % J.tiles_x) * 8u + (lane & 7u));
    const int ii = static_cast<int>((tile / J.tiles_x) * 8u + (lane >> 3));
    uint2 px{0u, 0xFFFFFFFFu};
    float4 d0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (jj < J.reg.w && ii < J.reg.h) {
      // main(): scr_coord = gl_FragCoord.xy / resolution (shader.frag:515-516)
      const float sx = (static_cast<float>(J.reg.x0 + jj) + 0.5f) / J.resolution[0];
      const float sy = (static_cast<float>(region_row(J.reg, ii)) + 0.5f) / J.resolution[1];
      // ray_drct(), shader.frag:501-505
      const float mx = (sx - 0.5f) * J.mtr_sizes[0];
      const float my = (0.5f - sy) * J.mtr_sizes[1];
      V4 dd = mad(ld4(J.right_drct), mx, mad(ld4(J.top_drct), my, ld4(J.vec_to_mtr)));
      dd = divs(dd, length(dd));
      d0 = make_float4(dd.x, dd.y, dd.z, dd.w);
      px = uint2{__float_as_uint(sx) ^ (__float_as_uint(sy) << 9) ^ in_seed,
                 static_cast<uint32_t>(a.fcolor ? pack_pixel_f(jj, ii, static_cast<int>(frame) + job) : pack_pixel(jj, ii, job))};
    }
    lds_in_d0[threadIdx.x] = d0;
    lds_in_px[threadIdx.x] = px;
    return true;
  };
  // One bounce of the lane's path from candidate c (shader.frag:475-492): on a miss the sky term, on a
  // hit the emitted light, the attenuation, the offset origin and the new direction. True when the
  // path is finished (a miss, or the bounces ran out: :494).
  auto shade = [&](const typename Finder<K>::R& c) -> bool {
    WEntry w_pre{};  // sampler-table entry for this bounce's diffuse direction (LUT path)
    if (!c.hit) {  // :477-479
      RT4_LS(3);
      RT4_STAMP(t_ph);
      const V3 fl = final_light(S, X, ray.drct);
      RT4_ACC(2, t_ph);
      acc = V3{sfma_(T.x, fl.x, acc.x), sfma_(T.y, fl.y, acc.y), sfma_(T.z, fl.z, acc.z)};
      return true;
    }
    RT4_LS(4);
    // rand_outcome's draw first (shader.frag:488, :121; the same draw, taken earlier): only a
    // diffuse outcome reads the sampler table, so mirrors and reflect outcomes issue no gather
    const bool diffuse = rand_(rng) > Finder<K>::refl(S, P, c);
#if RT4_LUT_PREFETCH == 2
#ifdef RT4_ABL_NOLUT  // ablation only (wrong images): the index arithmetic without the table gather
    if (LUT && diffuse) w_pre = WEntry{static_cast<float>(next_w_index(rng)) * 2.3841858e-7f - 1.0f};
#else
    if (LUT && diffuse) w_pre = wlut[next_w_index(rng) * RT4_ABL_WLUT_STRIDE];  // in flight during resolve + shading
#endif
#endif
    RT4_STAMP(t_ph);
    const Hit h = Finder<K>::resolve(P, ray, c);
    float glow, refl;
    V3 col;
    Finder<K>::material(S, P, h, glow, refl, col);
    RT4_ACC(3, t_ph);
    acc = V3{sfma_(col.x * glow, T.x, acc.x), sfma_(col.y * glow, T.y, acc.y), sfma_(col.z * glow, T.z, acc.z)};  // :481
    T = V3{T.x * col.x, T.y * col.y, T.z * col.z};                                                                  // :482
    ray.point = add(ray.point, mad(ray.drct, h.dist, mul(h.norm, indent)));                                          // :485
    if (!diffuse) {  // :488 rand_outcome -> reflect
      RT4_LS(5);
      const float dn = dot(h.norm, ray.drct);
      ray.drct = mad(h.norm, -(2.0f * dn), ray.drct);
    } else {  // :491 redirect(rand_drct(), norm)
      RT4_LS(6);
      RT4_STAMP(t_ph);
      const V4 v = rand_drct<LUT>(rng, wlut, w_pre);
      RT4_ACC(4, t_ph);
      const float dv = dot(v, h.norm);
      ray.drct = dv >= 0.0f ? v : mad(h.norm, -(2.0f * dv), v);
    }
    ++b;
    return b > R;
  };
  while (true) {
    RT4_STAMP(t_ph);
    // wave clock (CLOCK kernels, while the wave's paths run full length): samples start only at
    // iterations wave_it % (R + 1) == 0; a held lane (its sample ended early) waits for the next one
    bool boundary = true;
    if constexpr (CLOCK) {
      if (clock_on()) {
        if (__ballot(active) == 0ull) wave_it = 0;  // nothing in flight: this iteration starts the period
        boundary = wave_it == 0u;
      }
      wave_it = wave_it + 1u == static_cast<unsigned>(R + 1 + BEAT_SLACK) ? 0u : wave_it + 1u;
      if (boundary) hold = false;
    }
    if (!exhausted) {
      const unsigned long long idle = __ballot(!active);
      bool refill = static_cast<unsigned>(__popcll(idle)) >= REFILL_K;
      if (CLOCK && clock_on()) refill = refill && boundary;
      // phase-aligned: with active lanes left, wait (at most R + 1 iterations) for one of them to start
      // a sample; every active lane finishes a sample within R + 1 iterations, so the wait is bounded.
      // Not with primary reuse: there a sample's bounce 0 is shaded in the iteration that ends the previous
      // sample, so a starting sample is at b == 1 at the top of the loop.
      else if (PHASE && !REUSE && refill && ~idle != 0ull) refill = __ballot(active && b == 0) != 0ull;
      if (refill) {
        RT4_LS(8);
        retire();
        const unsigned rank =
            __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(idle >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(idle), 0u));
        const unsigned nidle = static_cast<unsigned>(__popcll(idle));
        unsigned got = 0;
        while (got < nidle) {
          if (in_next == 64u) {
            if (!claim_batch()) {
              exhausted = true;
#ifdef RT4_TAILSTATS
              tail_exh = __builtin_amdgcn_s_memrealtime();
#endif
              break;
            }
            in_next = 0;
          }
          const unsigned n = min(nidle - got, 64u - in_next);
          if (!active && rank >= got && rank < got + n) {
            const unsigned e = wbase + in_next + (rank - got);
            // both reads before the test: one LDS round trip per hand-out instead of two (RT4_REFILL_ONE_TRIP)
            const uint2 px = lds_in_px[e];
#if RT4_REFILL_ONE_TRIP
            const float4 d0 = lds_in_d0[e];
            asm volatile("" ::"v"(d0.x), "v"(d0.y), "v"(d0.z), "v"(d0.w));  // keep the read here, beside px's
#endif
            if (px.y != 0xFFFFFFFFu) {
#if !RT4_REFILL_ONE_TRIP
              const float4 d0 = lds_in_d0[e];
#endif
              rng = RngState{px.x, in_seed};
              ray = Ray{focus, V4{d0.x, d0.y, d0.z, d0.w}};
              acc = V3{0.0f, 0.0f, 0.0f};
              T = V3{1.0f, 1.0f, 1.0f};
              cold[0] = d0;
              lsum_store(make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(px.y)));
              s = 0;
              b = 0;
              if constexpr (BEAT_SLACK > 0) slack = BEAT_SLACK;
              active = NS > 0;
              pending = !active;
            }
          }
          in_next += n;
          got += n;
        }
      }
    }
    RT4_ACC(0, t_ph);
#ifdef RT4_LANESTATS
    ls[0] += 1;
    ls[1] += __popcll(__ballot(active));
#endif
    typename Finder<K>::R c{};
    bool parked = CLOCK && hold;  // DEFER: the lane's exact sphere tests wait; CLOCK: the lane's next sample
    bool cached = false;          // CLOCK && REUSE: this iteration's candidate came from the primary cache
    if constexpr (POOL) {
      // find part 1 + publish; barrier; pooled exact tests; barrier; combine (find part 2 below)
      RT4_STAMP(t_ph);
      uint32_t pend = 0;
      Cand pre = no_cand();
      if (active) pre = find_pre<K>(S, X, ray, pend);
      const unsigned long long pm = __ballot(pend != 0u);
      const unsigned slot = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(pm >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(pm), 0u));
      const bool pooled = pend != 0u && slot < static_cast<unsigned>(PCAP);
      if (pooled) {
        lds_pray[(wave * PCAP + slot) * 2] = make_float4(ray.point.x, ray.point.y, ray.point.z, ray.point.w);
        lds_pray[(wave * PCAP + slot) * 2 + 1] = make_float4(ray.drct.x, ray.drct.y, ray.drct.z, ray.drct.w);
      }
      unsigned nq = 0;  // wave-uniform
#pragma unroll
      for (int i = 0; i < NSH; i++) {
        const unsigned long long qm = __ballot(pooled && ((pend >> i) & 1u));
        if (pooled && ((pend >> i) & 1u)) {
          const unsigned q = nq + __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(qm >> 32),
                                                            __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(qm), 0u));
          lds_pair[wave * QCAP + q] = static_cast<uint16_t>(slot | (static_cast<unsigned>(i) << 6));
        }
        nq += static_cast<unsigned>(__popcll(qm));
      }
      const bool busy = __any(active) || !exhausted;
      if (lane == 0) lds_pn[wave] = nq | (busy ? 0x80000000u : 0u);
      __syncthreads();
      const uint4 pn = lds_pn4;
      if (((pn.x | pn.y | pn.z | pn.w) & 0x80000000u) == 0u) break;  // every wave of the block is done
      const unsigned c1 = pn.x & 0xFFFFu, c2 = c1 + (pn.y & 0xFFFFu), c3 = c2 + (pn.z & 0xFFFFu);
      const unsigned ntot = c3 + (pn.w & 0xFFFFu);
      for (unsigned p = threadIdx.x; p < ntot; p += 256u) {
        const unsigned w = (p >= c1) + (p >= c2) + (p >= c3);
        const unsigned j = p - (w == 0u ? 0u : (w == 1u ? c1 : (w == 2u ? c2 : c3)));
        const unsigned e = lds_pair[w * QCAP + j];
        const unsigned sl = e & 63u;
        const float4 rp = lds_pray[(w * PCAP + sl) * 2], rd = lds_pray[(w * PCAP + sl) * 2 + 1];
        const Cand q = sphere_exact<K>(X, P, Ray{V4{rp.x, rp.y, rp.z, rp.w}, V4{rd.x, rd.y, rd.z, rd.w}},
                                       static_cast<int>(e >> 6));
        lds_pres[w * QCAP + j] = make_float2(q.dist, __uint_as_float((q.hit ? 1u : 0u) | (q.flip ? 2u : 0u)));
      }
      __syncthreads();
      if (active) {
        Cand inter = pre;
        unsigned nb = 0;  // the pair index of this lane's sphere i: recomputed from the same ballots
#pragma unroll
        for (int i = 0; i < NSH; i++) {
          const bool mine = (pend >> i) & 1u;
          const unsigned long long qm = __ballot(pooled && mine);
          if (mine) {
            Cand q;
            if (pooled) {
              const unsigned at = nb + __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(qm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(qm), 0u));
              const float2 r = lds_pres[wave * QCAP + at];
              const uint32_t f = __float_as_uint(r.y);
              q = Cand{(f & 1u) != 0u, (f & 2u) != 0u, r.x, r.x, prim_bases<K>(X).sphere + static_cast<uint32_t>(i)};
              if (!q.hit) q = no_cand();
            } else {
              q = sphere_exact<K>(X, P, ray, i);
            }
            inter = closest(q, inter);
          }
          nb += static_cast<unsigned>(__popcll(qm));
        }
        c = find_rest<K>(S, X, P, ray, inter);
      }
      RT4_ACC(1, t_ph);
    } else if constexpr (TDEFER || TSPLIT) {
      if (!__any(active)) {
        if (exhausted) break;
        continue;
      }
      RT4_STAMP(t_ph);
      Cand pre = no_cand();
      bool need = false;
      const bool held = CLOCK && parked;  // held for the wave clock (the lockstep kernels)
      bool fresh = false;                 // SDEFER: the lane starts a find this iteration
      if (active && !held) {
        if constexpr (CLOCK && REUSE) {  // as the generic path below: bounce 0 from the cache at the clock boundary
          cached = use_cached;
          use_cached = false;
        }
        if (cached) {
          pre = unpack_cand(cold[512]);
        } else if (tparked) {
          pre = unpack_cand(cold[512]);
          need = true;
        } else if constexpr (SDEFER) {
          fresh = true;
        } else {
          pre = find_cand<K, false>(S, X, P, ray);  // every group but the tiger, in order
          need = !(RT4_BOUND_SKIP && far_from<ball_behind_of<K>(), occlude_of<K>(1)>(X->tiger_bound[0], ray, &pre));
        }
      }
      if constexpr (SDEFER) {
        // find_cand<K, false> in its three parts, the pending exact sphere tests deferred (the same bits)
        uint32_t pend = 0;
        SphereGeo geo;
        Cand inter = no_cand();
        if (fresh) inter = find_pre<K>(S, X, ray, pend, nullptr);
        const unsigned long long pm = __ballot(pend != 0u);
        const bool run = pm != 0ull && (static_cast<unsigned>(__popcll(pm)) >= static_cast<unsigned>(RT4_DEFER_EXACT_TIGER) ||
                                        defer_age >= RT4_DEFER_WAIT_TIGER || pm == __ballot(fresh));
        if (pm != 0ull && !run) {
          if (pend != 0u) {
            parked = true;
            fresh = false;
          }
          ++defer_age;
        } else {
          defer_age = 0;
        }
        if (fresh) {
          pre = find_rest<K, false>(S, X, P, ray, exact_pending<K, false>(X, P, ray, geo, pend, inter));
          need = !(RT4_BOUND_SKIP && far_from<ball_behind_of<K>(), occlude_of<K>(1)>(X->tiger_bound[0], ray, &pre));
        }
      }
      if constexpr (TSERVE) {
        const unsigned long long mp = __ballot(need && tparked), mn = __ballot(need && !tparked);
        const unsigned np = static_cast<unsigned>(__popcll(mp)), nt = np + static_cast<unsigned>(__popcll(mn));
        const bool run = nt != 0u && (nt >= static_cast<unsigned>(RT4_DEFER_TIGER) || tdefer_age >= RT4_DEFER_TIGER_WAIT ||
                                      (mp | mn) == __ballot(active && !held));
        const unsigned slot = tparked ? __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(mp >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(mp), 0u))
                                      : np + __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(mn >> 32),
                                                                       __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(mn), 0u));
        const bool serve = run && need && slot < TSPLIT_MAX;  // the parked lanes first, at most TSPLIT_MAX
        // every lane's candidate waits in cold[512] (no VGPRs held across the split test)
        if (active && !held && !tparked) cold[512] = pack_cand(pre);
        if (need && !serve) {
          tparked = true;
          parked = true;
        }
        // a run that left lanes parked runs again next iteration; otherwise the deferral's clock
        tdefer_age = run ? (nt > TSPLIT_MAX ? RT4_DEFER_TIGER_WAIT : 0) : (nt != 0u ? tdefer_age + 1 : 0);
      } else if constexpr (TDEFER) {
        const unsigned long long tm = __ballot(need);
        // in-beat: a lane with no parked iteration left forces the run (its sample must end within the period)
        const bool forced = BEAT_SLACK > 0 && clock_on() && __ballot(need && slack <= 0) != 0ull;
        // (!parked: as !held, and it leaves out the lanes parked for their exact sphere tests, SDEFER)
        const bool run = tm != 0ull && (static_cast<unsigned>(__popcll(tm)) >= static_cast<unsigned>(RT4_DEFER_TIGER) ||
                                        tdefer_age >= RT4_DEFER_TIGER_WAIT || tm == __ballot(active && !parked) || forced);
        if (tm != 0ull && !run) {
          ++tdefer_age;
          if (need) {
            if (!tparked) cold[512] = pack_cand(pre);
            tparked = true;
            parked = true;
            if (BEAT_SLACK > 0) --slack;
          }
        } else {
          tdefer_age = 0;
        }
      }
      // the tiger test of the lanes that run it now (find_rest's last group: closest(tiger, the rest))
#ifdef RT4_LANESTATS  // diagnostic: tiger tests and their lanes (counter[60], [61], [64..71]), as find_rest counts them
      {
        const unsigned long long gm_ = __ballot(active && !parked && need);
        if (gm_ && lane == static_cast<unsigned>(__builtin_ctzll(__builtin_amdgcn_read_exec()))) {
          atomicAdd(counter + 60, 1ull);
          atomicAdd(counter + 61, static_cast<unsigned long long>(__popcll(gm_)));
          // by lanes: 1-16, 17-32, 33-48, 49-64 (counter[64..67] events, [68..71] lanes; tools/lanestats.py)
          const unsigned bk_ = (static_cast<unsigned>(__popcll(gm_)) - 1u) >> 4;
          atomicAdd(counter + 64 + bk_, 1ull);
          atomicAdd(counter + 68 + bk_, static_cast<unsigned long long>(__popcll(gm_)));
        }
      }
#endif
      if constexpr (TSERVE) {
        // every served test split into its quarters; rays and results by ds_bpermute, the owners' lanes by LDS
        const bool go = active && !parked && need;
        const unsigned long long gm = __ballot(go);
        const unsigned ng = static_cast<unsigned>(__popcll(gm));
        Cand tg = no_cand();
        if (ng != 0u) {
          const unsigned ln = rt4_lane_id(), wv = wave_s >> 6;
          const unsigned rk = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(gm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(gm), 0u));
          if (go) lds_town[wv * 16u + rk] = ln;
          const bool task = ln < 4u * ng;
          const int src = static_cast<int>((task ? lds_town[wv * 16u + (ln >> 2)] : ln) << 2);
          auto pull = [&](float v) { return __int_as_float(__builtin_amdgcn_ds_bpermute(src, __float_as_int(v))); };
          const Ray tr{V4{pull(ray.point.x), pull(ray.point.y), pull(ray.point.z), pull(ray.point.w)},
                       V4{pull(ray.drct.x), pull(ray.drct.y), pull(ray.drct.z), pull(ray.drct.w)}};
          float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          if (task) q = pack_cand(tiger_quarter(S, X, 0, prim_bases<K>(X).tiger, tr, ln & 3u));
          auto part = [&](unsigned j) {  // the owner's quarter j, from lane 4 rk + j
            const int from = static_cast<int>(((go ? 4u * rk + j : ln) & 63u) << 2);
            return unpack_cand(make_float4(__int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.x))),
                                           __int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.y))),
                                           __int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.z))), 0.0f));
          };
          const Cand t01 = closest(part(0u), part(1u));
          tg = closest(t01, closest(part(2u), part(3u)));
        }
        if (active && !parked) {
          c = go ? closest(tg, unpack_cand(cold[512])) : unpack_cand(cold[512]);
          tparked = false;
        }
      } else if constexpr (TSPLIT) {
        const bool go = active && !parked && need;
        Cand tg = no_cand();
        const unsigned long long gm = __ballot(go);
        const unsigned ng = static_cast<unsigned>(__popcll(gm));
        if (ng > TSPLIT_MAX) {
          if (go) tg = tiger_cand(S, X, 0, prim_bases<K>(X).tiger, ray);
        } else if (ng != 0u) {
          // the lanes running the test publish their rays, 4 ng lanes run the quarters, the owners fold their four
          // results (one pass: TSPLIT_MAX <= 16; a loop of passes kept tg live across the quarter and spilled)
          const unsigned ln = rt4_lane_id(), wv = wave_s >> 6;
          float4* const tray = lds_tray + wv * (2u * TSPLIT_MAX);
          float4* const tres = lds_tres + (TRES_LDS ? wv * (4u * TSPLIT_MAX) : 0u);
          const unsigned rk = __builtin_amdgcn_mbcnt_hi(static_cast<unsigned>(gm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo(static_cast<unsigned>(gm), 0u));
          if (go) {
            tray[2u * rk] = make_float4(ray.point.x, ray.point.y, ray.point.z, ray.point.w);
            tray[2u * rk + 1u] = make_float4(ray.drct.x, ray.drct.y, ray.drct.z, ray.drct.w);
          }
          // Cross-lane hand-offs through LDS: a wave's LDS accesses complete in program order, and the wave barrier
          // keeps the compiler from moving one lane's read of another lane's slot above the write.
          __builtin_amdgcn_wave_barrier();
          if constexpr (TRES_LDS) {
            if (ln < 4u * ng) {  // quarter ln & 3 of the test of the lane ranked ln >> 2
              const float4 p4 = tray[2u * (ln >> 2)], d4 = tray[2u * (ln >> 2) + 1u];
              tres[ln] = pack_cand(tiger_quarter(S, X, 0, prim_bases<K>(X).tiger,
                                                 Ray{V4{p4.x, p4.y, p4.z, p4.w}, V4{d4.x, d4.y, d4.z, d4.w}}, ln & 3u));
            }
            __builtin_amdgcn_wave_barrier();
            if (go)
              tg = closest(closest(unpack_cand(tres[4u * rk]), unpack_cand(tres[4u * rk + 1u])),
                           closest(unpack_cand(tres[4u * rk + 2u]), unpack_cand(tres[4u * rk + 3u])));
          } else {
            // the owner of rank rk pulls quarter j from lane 4 rk + j (every lane takes part in the permutes; a lane
            // that owns no test pulls its own value and drops it)
            float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (ln < 4u * ng) {
              const float4 p4 = tray[2u * (ln >> 2)], d4 = tray[2u * (ln >> 2) + 1u];
              q = pack_cand(tiger_quarter(S, X, 0, prim_bases<K>(X).tiger,
                                          Ray{V4{p4.x, p4.y, p4.z, p4.w}, V4{d4.x, d4.y, d4.z, d4.w}}, ln & 3u));
            }
            auto part = [&](unsigned j) {
              const int from = static_cast<int>(((go ? 4u * rk + j : ln) & 63u) << 2);
              return unpack_cand(make_float4(__int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.x))),
                                             __int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.y))),
                                             __int_as_float(__builtin_amdgcn_ds_bpermute(from, __float_as_int(q.z))), 0.0f));
            };
            const Cand t01 = closest(part(0u), part(1u));
            const Cand t = closest(t01, closest(part(2u), part(3u)));
            if (go) tg = t;
          }
        }
        if (active && !parked) {
          c = need ? closest(tg, pre) : pre;
          tparked = false;
        }
      } else if (active && !parked) {
        c = need ? closest(tiger_cand(S, X, 0, prim_bases<K>(X).tiger, ray), pre) : pre;
        tparked = false;
      }
      RT4_ACC(1, t_ph);
    } else if constexpr (DEFER) {
      // find in two parts with the exact sphere tests deferred: lanes whose cull leaves
      // pending spheres park (no shading, no count) until enough lanes of the wave are pending; a parked
      // lane redoes the cull next iteration (same ray, same bits) instead of keeping its state
      if (!__any(active)) {
        if (exhausted) break;
        continue;
      }
      RT4_STAMP(t_ph);
      uint32_t pend = 0;
      SphereGeo geo;
      Cand inter = no_cand();
      if (active) inter = find_pre<K>(S, X, ray, pend, RT4_DEFER_GEO ? &geo : nullptr);
      const unsigned long long pm = __ballot(pend != 0u);
      const bool run = pm != 0ull && (static_cast<unsigned>(__popcll(pm)) >= static_cast<unsigned>(RT4_DEFER_EXACT) ||
                                      defer_age >= RT4_DEFER_WAIT || pm == __ballot(active));
      if (pm != 0ull && !run) {
        parked = pend != 0u;
        ++defer_age;
      } else {
        defer_age = 0;
      }
      if (active && !parked) c = find_rest<K>(S, X, P, ray, exact_pending<K, RT4_DEFER_GEO != 0>(X, P, ray, geo, pend, inter));
      RT4_ACC(1, t_ph);
    } else {
      if (!__any(active)) {
        if (exhausted) break;
        continue;
      }
      if (active && !parked) {
        RT4_STAMP(t_ph);
        if constexpr (CLOCK && REUSE) {
          // with the wave clock a sample's bounce 0 is shaded from the cache at the clock boundary, in its
          // own iteration (the other lanes do the same in lockstep), instead of in the iteration that ended
          // the previous sample
          cached = use_cached;
          if (cached) c = unpack_cand(cold[512]);
          else c = Finder<K>::find(S, X, P, ray);  // :475
          use_cached = false;
        } else {
          c = Finder<K>::find(S, X, P, ray);  // :475
        }
        RT4_ACC(1, t_ph);
      }
    }
    bool end_early = false, end_full = false;  // CLOCK: the lane's sample ended before / at the bounce limit
    if (active && parked) RT4_LS(9);  // lanes waiting (deferred exact tests, or held for the wave clock)
    if constexpr (WAVE_COUNT) w_inter += static_cast<unsigned long long>(__popcll(__ballot(active && !parked)));
    if (active && !parked) {
      RT4_LS(1);
      if constexpr (!WAVE_COUNT) {
        ++n_inter;
        if (!cached) ++n_eval;
      }
      if constexpr (REUSE) {
        if (s == 0 && b == 0) cold[512] = pack_cand(c);  // the pixel's primary candidate
      }
      bool end = shade(c);
      if constexpr (!REUSE) {
        if (end) {  // path finished (:478 or :494): accumulate, next sample restarts at the focus
          RT4_LS(7);
          end_early = b <= R;
          end_full = !end_early;
          const float4 lp = lsum_load();
          lsum_store(make_float4(lp.x + acc.x, lp.y + acc.y, lp.z + acc.z, lp.w));
          const float4 c0 = cold[0];
          ray = Ray{focus, V4{c0.x, c0.y, c0.z, c0.w}};
          ++s;
          b = 0;
          if constexpr (BEAT_SLACK > 0) slack = BEAT_SLACK;
          acc = V3{0.0f, 0.0f, 0.0f};
          T = V3{1.0f, 1.0f, 1.0f};
          if (s >= NS) {
            active = false;
            pending = true;
          }
        }
      }
      while (REUSE && end) {  // path finished (:478 or :494): accumulate, next sample restarts at the focus
        RT4_LS(7);
        if (!end_early && !end_full) {
          end_early = b <= R;
          end_full = !end_early;
        }
        const float4 lp0 = lsum_load();
        float4 lp = make_float4(lp0.x + acc.x, lp0.y + acc.y, lp0.z + acc.z, lp0.w);
        const float4 c0 = cold[0];
        ray = Ray{focus, V4{c0.x, c0.y, c0.z, c0.w}};
        ++s;
        b = 0;
        acc = V3{0.0f, 0.0f, 0.0f};
        T = V3{1.0f, 1.0f, 1.0f};
        end = false;
        if (s >= NS) {
          active = false;
          pending = true;
        } else if constexpr (REUSE) {
          {
            // RT4_FLAG_PRIMARY_REUSE: every sample of a pixel starts with the same primary ray
            // (shader.frag:519-521), so its bounce 0 is the cached candidate, shaded in this same
            // iteration with the sample's own random numbers; no find_intersection is evaluated.
            const Cand pc = unpack_cand(cold[512]);
            if (!pc.hit) {
              ++n_inter;
              // a primary miss: every remaining sample is that same sky ray, acc = fma(T, sky, acc)
              // with T = 1, acc = 0 (:477-479), added to the sum sample by sample
              const V3 fl = final_light(S, X, ray.drct);
              const V3 m{sfma_(1.0f, fl.x, 0.0f), sfma_(1.0f, fl.y, 0.0f), sfma_(1.0f, fl.z, 0.0f)};
              lp = make_float4(lp.x + m.x, lp.y + m.y, lp.z + m.z, lp.w);
              for (++s; s < NS; ++s) {
                lp = make_float4(lp.x + m.x, lp.y + m.y, lp.z + m.z, lp.w);
                ++n_inter;
              }
              active = false;
              pending = true;
            } else if (CLOCK && clock_on()) {
              use_cached = true;  // shaded (and counted) at the next clock boundary
            } else {
              ++n_inter;
              end = shade(pc);  // one bounce; the path goes on next iteration unless bounces ran out
            }
          }
        }
        lsum_store(lp);
      }
    }
    if constexpr (CLOCK) {
      n_early += static_cast<unsigned>(__popcll(__ballot(end_early)));
      n_full += static_cast<unsigned>(__popcll(__ballot(end_full)));
      if (n_early + n_full > 4096u) {  // leaky: the recent paths decide
        n_early >>= 1;
        n_full >>= 1;
      }
      // a lane that starts its next sample off the clock waits for the next boundary
      if (clock_on() && wave_it != 0u && active && (end_early || end_full)) hold = true;
    }
  }
  retire();  // the pixels finished after the queue ran dry, then whatever the ring holds
  if (ring_n) flush_ring();
#ifdef RT4_LANESTATS
  if (counter && lane == 0)
    for (int q = 0; q < 20; q++) atomicAdd(counter + 16 + q, ls[q]);
#endif
#ifdef RT4_STAMPS
  RT4_ACC(5, t_loop0);
  if (counter && lane == 0)
    for (int q = 0; q < 6; q++) atomicAdd(counter + 1 + q, st[q]);
#endif

#ifdef RT4_TAILSTATS
  if (counter && lane == 0) {  // counter[64 + 3 w ...]: the caller allocates 64 + 3 x (grid waves) words
    const unsigned gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    counter[64 + 3 * gw] = tail_t0;
    counter[64 + 3 * gw + 1] = tail_exh;
    counter[64 + 3 * gw + 2] = __builtin_amdgcn_s_memrealtime();
  }
#endif
  if (counter) {  // wave-level sum, one atomic per wave
    unsigned long long v = w_inter;
    if constexpr (!WAVE_COUNT) {
      v = n_inter;
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    }
    if (lane == 0 && v) atomicAdd(counter, v);
  }
  if (a.eval_counter) {  // evaluated find calls (fewer than the count above with primary reuse)
    unsigned long long v = w_inter;
    if constexpr (!WAVE_COUNT) {
      v = n_eval;
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    }
    if (lane == 0 && v) atomicAdd(a.eval_counter, v);
  }
}

__global__ void rt4_build_wlut_kernel(WEntry* __restrict__ lut) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= (1u << 23)) return;
  const float w = w_by_volume(__uint_as_float(m | 0x3F800000u) - 1.0f, nullptr);
  lut[m * RT4_ABL_WLUT_STRIDE] = w;
}

// Checks of the verified-divisor quotient div_c (rt4_fast.h) against the IEEE quotient x / b, one
// divisor per blockIdx.y. Equivalent to all 2^32 numerators at a fraction of the work (DESIGN.md
// §4.5): both quotients are odd in x (RN is symmetric), so only sign-0 patterns are swept; and in the
// middle band of exponent fields [lo, hi] every intermediate (x, q, the exact residual x - q b when
// non-zero, q2, x / b) is a normal number, so scaling x by 2^k scales every rounded step exactly and
// one field stands for the whole band. The band is swept at three representative fields (lo, mid,
// hi); every field outside it, subnormals, zero, inf and NaN included, is swept in full.
// lo > hi: no band, all 256 fields.
struct DivSweep {
  float b, y;
  uint32_t lo, hi;
};
constexpr int MAX_DIV_SWEEPS = 128;
struct DivSweeps {
  DivSweep d[MAX_DIV_SWEEPS];
};
__device__ __forceinline__ uint32_t div_sweep_fields(const DivSweep& d) {
  return d.lo > d.hi ? 256u : d.lo + 3u + (255u - d.hi);
}
__device__ __forceinline__ uint32_t div_sweep_field(const DivSweep& d, uint32_t k) {
  if (d.lo > d.hi || k < d.lo) return k;
  k -= d.lo;
  if (k < 3u) return k == 0u ? d.lo : (k == 1u ? (d.lo + d.hi) / 2u : d.hi);
  return d.hi + 1u + (k - 3u);
}
__global__ void rt4_verify_div_kernel(const DivSweeps sw, unsigned* __restrict__ mismatches) {
  const DivSweep d = sw.d[blockIdx.y];
  if (d.b == 0.0f) return;  // the warm-up launch of rt4_context_create (0 is never a swept divisor)
  const DivC c{d.b, d.y, 1, 0};
  const uint64_t total = static_cast<uint64_t>(div_sweep_fields(d)) << 23;
  unsigned bad = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint32_t f = div_sweep_field(d, static_cast<uint32_t>(i >> 23));
    const float x = __uint_as_float((f << 23) | (static_cast<uint32_t>(i) & 0x007FFFFFu));
    const float q1 = x / d.b;
    const float q2 = div_c(x, c);
    const bool same = __float_as_uint(q1) == __float_as_uint(q2) || (q1 != q1 && q2 != q2);
    bad += same ? 0u : 1u;
  }
  if (bad) atomicAdd(mismatches + blockIdx.y, bad);
}

// Exhaustive check of sqrt_ (rt4_device_math.h) against the IEEE square root for every 32-bit pattern.
__global__ void rt4_verify_sqrt_kernel(unsigned long long* __restrict__ mismatches) {
  unsigned bad = 0;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const float x = __uint_as_float(static_cast<uint32_t>(i));
    const float a = sqrt_(x), b = __builtin_sqrtf(x);
    bad += (__float_as_uint(a) == __float_as_uint(b) || (a != a && b != b)) ? 0u : 1u;
  }
  if (bad) atomicAdd(mismatches, static_cast<unsigned long long>(bad));
}

// min over the float patterns c in [lo, lo + count) with acos_(c) < ang, as an order-preserving key
// (0xFFFFFFFF: none). For ang <= 1 only c in (0.5, 1] can qualify: acos_ of c <= 0.5 is >= pi/3 - tiny
// (rt4_device_math.h acos_: the small branch returns pi/2 - asin_core(c), the big negative one
// pi - 2 asin_core >= pi/2), and NaN for NaN or c > 1. rt4_debug_sky_threshold(1.0, full) > 0.5 proves
// it over all 2^32 patterns (tests/test_gpu_parity.py).
__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__global__ void rt4_sky_threshold_kernel(float ang, uint32_t lo, uint64_t count, uint32_t* __restrict__ best) {
  uint32_t mine = 0xFFFFFFFFu;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count; i += stride) {
    const float c = __uint_as_float(lo + static_cast<uint32_t>(i));
    if (acos_(c) < ang) mine = min(mine, order_key(c));
  }
  if (mine != 0xFFFFFFFFu) atomicMin(best, mine);
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
    case RT4_EVAL_SQRT: r = sqrt_(x); break;
    default: r = __builtin_nanf(""); break;
  }
  out[t] = r;
  if (aux) aux[t] = it;
}

template <uint32_t K>
__global__ void rt4_find_kernel(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                const float* __restrict__ rays, float* __restrict__ out,
                                float* __restrict__ out_color, int64_t n) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
#ifdef RT4_LANESTATS
  rt4_ls_counter = nullptr;  // diagnostic build: only the trace kernel counts
#endif
  if (t >= n) return;
  const float* r = rays + 8 * t;
  const Ray ray{ld4(r), ld4(r + 4)};
  const typename Finder<K>::R c = Finder<K>::find(S, X, X->prims, ray);
  Hit h = c.hit ? Finder<K>::resolve(X->prims, ray, c) : no_hit();
  h.dist = c.dist;
  float* o = out + 8 * t;
  o[0] = h.hit ? 1.0f : 0.0f;
  o[1] = h.dist;
  o[2] = h.norm.x; o[3] = h.norm.y; o[4] = h.norm.z; o[5] = h.norm.w;
  if (h.hit) {
    float glow, refl;
    V3 col;
    Finder<K>::material(S, X->prims, h, glow, refl, col);
    o[6] = glow; o[7] = refl;
    out_color[3 * t] = col.x; out_color[3 * t + 1] = col.y; out_color[3 * t + 2] = col.z;
  } else {
    o[6] = 0.0f; o[7] = 0.0f;
    out_color[3 * t] = 0.0f; out_color[3 * t + 1] = 0.0f; out_color[3 * t + 2] = 0.0f;
  }
}

// Tile order for the pixel queue (longest work first): one thread per 8x8 tile traces the primary ray
// of the tile's centre pixel; tiles whose ray hits something go to the front of `order`, sky tiles to
// the back. The queue hands tiles out in this order, so the slow tiles do not form the drain at the
// end of the launch. Results do not depend on the order (every pixel is independent).
template <uint32_t K>
__global__ void rt4_tile_order_kernel(const rt4_scene_desc* __restrict__ S, const SceneAux* __restrict__ X,
                                      const KernelArgs a, unsigned* __restrict__ order, unsigned* __restrict__ ends) {
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned n = a.total >> 6;
#ifdef RT4_LANESTATS
  rt4_ls_counter = nullptr;  // diagnostic build: only the trace kernel counts
#endif
  if (t >= n) return;
  const int job = (a.n_jobs > 1 && t >= a.jobs[1].tile_base) + (a.n_jobs > 2 && t >= a.jobs[2].tile_base);
  const JobArgs& J = a.jobs[job];
  const unsigned lt = t - J.tile_base;
  const int jj = min(static_cast<int>((lt % J.tiles_x) * 8u + 4u), J.reg.w - 1);
  const int ii = min(static_cast<int>((lt / J.tiles_x) * 8u + 4u), J.reg.h - 1);
  const float sx = (static_cast<float>(J.reg.x0 + jj) + 0.5f) / J.resolution[0];
  const float sy = (static_cast<float>(region_row(J.reg, ii)) + 0.5f) / J.resolution[1];
  const float mx = (sx - 0.5f) * J.mtr_sizes[0];
  const float my = (0.5f - sy) * J.mtr_sizes[1];
  V4 dd = mad(ld4(J.right_drct), mx, mad(ld4(J.top_drct), my, ld4(J.vec_to_mtr)));
  dd = divs(dd, length(dd));
  const typename Finder<K>::R c = Finder<K>::find(S, X, X->prims, Ray{ld4(a.focus), dd});
  const unsigned pos = c.hit ? atomicAdd(ends, 1u) : n - 1u - atomicAdd(ends + 1, 1u);
  order[pos] = t;
}

// The frames of a pipelined launch blended in order into the frame buffer (rt4_render_frames_device):
// per pixel the same blend as write_pixel, frame after frame, each rounded to the frame format.
// count_src (an overlapped single frame): the trace kernel's count, moved into the caller's counter here, on
// the caller's stream, and reset for the slot's next frame
__global__ void rt4_fold_frames_kernel(const KernelArgs a, unsigned long long* count_src, unsigned long long* count_dst) {
#if RT4_FOLD_PRIO > 0
  // the fold's waves win the SIMD's issue arbitration over the co-resident trace waves of later frames
  __builtin_amdgcn_s_setprio(RT4_FOLD_PRIO);
#endif
  const int job = static_cast<int>(blockIdx.y);  // the section of an overlapped sections launch (else 0)
  const JobArgs& J = a.jobs[job];
  const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (count_src && p == 0 && job == 0) {
    if (count_dst) atomicAdd(count_dst, *count_src);
    *count_src = 0ull;
  }
  const int64_t npx = static_cast<int64_t>(J.reg.w) * J.reg.h;
  if (p >= npx) return;
  const int i = static_cast<int>(p / J.reg.w), j = static_cast<int>(p - static_cast<int64_t>(i) * J.reg.w);
  char* base = static_cast<char*>(J.frame);
  const int64_t at = static_cast<int64_t>(i) * J.row_stride_px + j;
  auto color = [&](int f) {  // frame f's light sum, tone-mapped as write_pixel does
    const float4 l = a.fcolor[J.fc_base + f * npx + p];
    return tone_map(a, V3{l.x, l.y, l.z});
  };
  if (a.format == RT4_FRAME_RGBA16F) {
    h4v* px = reinterpret_cast<h4v*>(base) + at;
    h4v v = *px;
    for (int f = 0; f < a.n_frames; f++) v = blend_f16(color(f), a.frame_part[f], v);
    *px = v;
  } else if (a.format == RT4_FRAME_RGBA8) {
    uint32_t* px = reinterpret_cast<uint32_t*>(base) + at;
    uint32_t v = *px;
    for (int f = 0; f < a.n_frames; f++) v = blend_u8(color(f), a.frame_part[f], v);
    *px = v;
  } else {
    float4* px = reinterpret_cast<float4*>(base) + at;
    float4 v = *px;
    for (int f = 0; f < a.n_frames; f++) v = blend_f32(color(f), a.frame_part[f], v);
    *px = v;
  }
}

// The frame from the gathered band shards (rt4_bands_unpermute_device): one block per image row copies
// the row from its place in the gather, in 16-B words when rows allow it, else 4-B words (every format's
// pixel is a multiple of 4 B).
template <typename W>
__global__ void rt4_unpermute_kernel(const W* __restrict__ gathered, W* __restrict__ image, int32_t words_per_row,
                                     int32_t world, int32_t band, int32_t rows_max) {
  const int64_t y = blockIdx.x;
  const int64_t b = y / band;
  const int64_t src = (b % world) * rows_max + (b / world) * band + y % band;  // shard.py gather_index
  const W* in = gathered + src * words_per_row;
  W* out = image + y * words_per_row;
  for (int32_t k = threadIdx.x; k < words_per_row; k += blockDim.x) out[k] = in[k];
}

// ---------------------------------------------------------------- kernel table
typedef void (*TraceFn)(const rt4_scene_desc*, const SceneAux*, const KernelArgs, unsigned long long*,
                        const WEntry*, unsigned*, unsigned*);
typedef void (*FindFn)(const rt4_scene_desc*, const SceneAux*, const float*, float*, float*, int64_t);
typedef void (*OrderFn)(const rt4_scene_desc*, const SceneAux*, const KernelArgs, unsigned*, unsigned*);

struct Variant {
  uint32_t shape;
  TraceFn trace[2][2];  // [lut][primary reuse]
  FindFn find;
  OrderFn order;
};

#define RT4_VARIANT(K)                                                                                  \
  {K,                                                                                                   \
   {{rt4_trace_kernel<K, false, false>, rt4_trace_kernel<K, false, (K) != GENERIC>},                    \
    {rt4_trace_kernel<K, true, false>, rt4_trace_kernel<K, true, (K) != GENERIC>}},                     \
   rt4_find_kernel<K>, rt4_tile_order_kernel<K>}
// shape | (n_spaces+1) << 8 | (n_spheres+1) << 16 | (n_cylinders+1) << 24 (rt4_fast.h sh_count),
// from the scene's object counts (the same encoding scene_shape() computes)
#define SH(K, nsp, nsh, ncy) \
  ((K) | (uint32_t((nsp) + 1) << 8) | (uint32_t((nsh) + 1) << 16) | (uint32_t((ncy) + 1) << 24))
const Variant kVariants[] = {
    RT4_VARIANT(GENERIC),
    RT4_VARIANT(K_SPACES),
    RT4_VARIANT(K_SPACES | K_SPHERES),
    RT4_VARIANT(K_SPACES | K_UNION),
    RT4_VARIANT(K_SPACES | K_HYPERCUBE),
    RT4_VARIANT(K_SPACES | K_TIGER),
    RT4_VARIANT(K_SPACES | K_SPHERES | K_CYLINDERS | K_UNION | K_HYPERCUBE | K_TIGER),
    // exact object counts of the reference scenes and the authored ones: fully unrolled
    RT4_VARIANT(SH(K_SPACES | K_SPHERES, 1, 2, 0)),      // sphere
    RT4_VARIANT(SH(K_SPACES | K_SPHERES, 8, 2, 0)),      // room
    RT4_VARIANT(SH(K_SPACES | K_TIGER, 1, 0, 0)),        // tiger
    RT4_VARIANT(SH(K_SPACES | K_TIGER, 3, 0, 0)),        // tiger_two_mirrors
    RT4_VARIANT(SH(K_SPACES | K_UNION, 1, 0, 0)),        // cylinder4d
    RT4_VARIANT(SH(K_SPACES | K_HYPERCUBE, 1, 0, 0)),    // hypercube
    RT4_VARIANT(SH(K_SPACES | K_SPHERES | K_CYLINDERS | K_UNION | K_HYPERCUBE | K_TIGER, 2, 3, 1)),  // all_primitives
};
#undef RT4_VARIANT
#undef SH

bool same4(const float* a, const float* b) { return std::memcmp(a, b, 4 * sizeof(float)) == 0; }

// Same primary rays for every tile (rt4_tile_order_kernel's inputs, the scene aside)?
bool same_primary_rays(const KernelArgs& x, const KernelArgs& y) {
  if (!same4(x.focus, y.focus) || x.n_jobs != y.n_jobs || x.total != y.total) return false;
  for (int i = 0; i < x.n_jobs; i++) {
    const JobArgs &p = x.jobs[i], &q = y.jobs[i];
    if (std::memcmp(p.resolution, q.resolution, sizeof p.resolution) || std::memcmp(p.mtr_sizes, q.mtr_sizes, sizeof p.mtr_sizes) ||
        !same4(p.vec_to_mtr, q.vec_to_mtr) || !same4(p.top_drct, q.top_drct) || !same4(p.right_drct, q.right_drct) ||
        std::memcmp(&p.reg, &q.reg, sizeof p.reg) || p.tile_base != q.tile_base || p.tiles_x != q.tiles_x)
      return false;
  }
  return true;
}

// Shape of a scene for the specialised kernels (rt4_intersect.h: find_intersection_spec); GENERIC
// when the group list is anything other than shader.frag's canonical form.
uint32_t scene_shape(const rt4_scene_desc& s) {
  static const uint32_t bit[7] = {0, K_SPACES, K_SPHERES, K_CYLINDERS, K_UNION, K_HYPERCUBE, K_TIGER};
  uint32_t k = 0;
  int last = 0;
  for (int g = 0; g < s.n_groups; g++) {
    const rt4_group& gr = s.groups[g];
    if (gr.kind <= last || gr.kind > RT4_GROUP_TIGER || !gr.new_first || gr.first != 0) return GENERIC;
    last = gr.kind;
    int n = 0;
    switch (gr.kind) {
      case RT4_GROUP_SPACES: n = s.n_spaces; break;
      case RT4_GROUP_SPHERES: n = s.n_spheres; if (!gr.outer) return GENERIC; break;
      case RT4_GROUP_CYLINDERS: n = s.n_cylinders; if (!gr.outer) return GENERIC; break;
      case RT4_GROUP_CYLINDERS_UNION: n = s.n_unions; if (n != 1) return GENERIC; break;
      case RT4_GROUP_HYPERCUBE: n = s.n_hypercubes; if (n != 1) return GENERIC; break;
      case RT4_GROUP_TIGER: {
        n = s.n_tigers;
        if (n != 1) return GENERIC;
        const rt4_tiger& t = s.tigers[0];
        if (!same4(t.inner_cyl1.point, t.outer_cyl1.point) || !same4(t.inner_cyl1.axis1, t.outer_cyl1.axis1) ||
            !same4(t.inner_cyl1.axis2, t.outer_cyl1.axis2) || !same4(t.inner_cyl2.point, t.outer_cyl2.point) ||
            !same4(t.inner_cyl2.axis1, t.outer_cyl2.axis1) || !same4(t.inner_cyl2.axis2, t.outer_cyl2.axis2))
          return GENERIC;
      } break;
    }
    if (gr.count != n) return GENERIC;
    k |= bit[gr.kind];
  }
  const uint32_t counted = k | (static_cast<uint32_t>(s.n_spaces + 1) << 8) |
                           (static_cast<uint32_t>(s.n_spheres + 1) << 16) |
                           (static_cast<uint32_t>(s.n_cylinders + 1) << 24);
#ifndef RT4_NO_EXACT_COUNTS  // A/B knob: -DRT4_NO_EXACT_COUNTS runs every scene on its runtime-count kernel
  // exact counts first (unrolled; primitive-table bases compile-time, rt4_fast.h prim_bases: objects of
  // an untested group would shift them), then the runtime-count kernel
  const bool bases_fixed = s.n_unions == ((k & K_UNION) ? 1 : 0) && s.n_hypercubes == ((k & K_HYPERCUBE) ? 1 : 0) &&
                           s.n_tigers == ((k & K_TIGER) ? 1 : 0);
  for (const Variant& v : kVariants)
    if (bases_fixed && v.shape == counted) return counted;
#endif
  for (const Variant& v : kVariants)
    if (v.shape == k) return k;
  return GENERIC;
}

const Variant& variant_for(uint32_t shape) {
  for (const Variant& v : kVariants)
    if (v.shape == shape) return v;
  return kVariants[0];
}

}  // namespace

// ==================================================================================== context
struct rt4_context {
  int device = 0;
  uint32_t flags = 0;
  rt4_scene_desc* d_scene = nullptr;  // followed by its SceneAux (scene_aux())
  SceneAux aux{};
  unsigned* d_scratch = nullptr;      // verification counters (MAX_DIV_SWEEPS + 1 words)
  bool has_scene = false;
  uint32_t shape = GENERIC;
  WEntry* d_wlut = nullptr;
  unsigned* d_queue = nullptr;  // QUEUE_SLOTS words
  unsigned* d_order = nullptr;  // tile order (rt4_tile_order_kernel) + 2 end counters
  void* d_fcolor = nullptr;     // frame colours of pipelined launches (rt4_render_frames_device)
  size_t fcolor_bytes = 0;
  size_t order_cap = 0;         // tiles it holds
  bool order_valid = false;     // d_order holds the order for order_args (same scene)
  KernelArgs order_args{};
  hipEvent_t done = nullptr;    // recorded after each launch: launches on another stream wait for it
  hipStream_t last_stream = nullptr;
  bool launched = false;
  unsigned launch_seq = 0;
  bool q_dirty[QUEUE_SLOTS] = {};  // a launch failed before zeroing this queue word: its next user zeroes it
  unsigned long long* d_eval = nullptr;  // evaluated find calls (RT4_FLAG_PRIMARY_REUSE), rt4_context_evaluated
  int n_cu = 0;
  TraceFn occ_fn = nullptr;  // blocks per CU of the last trace kernel launched (occupancy query cache)
  int occ_per_cu = 0;
  // Overlapped single frames: launch s traces on a side stream into a slot buffer while the
  // launches before it drain; its fold runs on the caller's stream. A frame too small to fill the chip ("deep")
  // runs up to S = RT4_OVERLAP_SLOTS in flight (side stream and buffer s % S), any other frame up to
  // B = RT4_OVERLAP_BIG (side stream and buffer s % B), so a frame that fills the chip allocates only B buffers.
  // seq_done[s % S]: recorded when launch s is complete (launch s + S, and for a big frame s + B, waits for it:
  // queue word, frame-colour buffer and count slot). Switching between deep and big frames first drains every
  // launch in flight (the two buffer rotations share buffers 0 .. B - 1).
  hipStream_t side[RT4_OVERLAP_SLOTS] = {};
  hipEvent_t traced[RT4_OVERLAP_SLOTS] = {};
  hipEvent_t seq_done[RT4_OVERLAP_SLOTS] = {};
  void* d_ofcolor[RT4_OVERLAP_SLOTS] = {};
  size_t ofcolor_cap[RT4_OVERLAP_SLOTS] = {};  // bytes of each slot buffer (grown to the largest launch it served)
  bool overlapped = false, last_deep = false;  // the last overlapped launch's rotation
  unsigned long long* d_ocount = nullptr;  // one counter per slot
};

#define HIP_TRY(expr)                                                                            \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) {                                                                      \
      rt4_set_err(err, errlen, "%s failed: %s", #expr, hipGetErrorString(e_));                   \
      return RT4_ERR_HIP;                                                                        \
    }                                                                                            \
  } while (0)

namespace {

constexpr size_t kAuxOffset = (sizeof(rt4_scene_desc) + 255) & ~size_t(255);
constexpr size_t kSceneBytes = kAuxOffset + sizeof(SceneAux);

const SceneAux* scene_aux(const rt4_context* c) {
  return reinterpret_cast<const SceneAux*>(reinterpret_cast<const char*>(c->d_scene) + kAuxOffset);
}

float fbits(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

// Largest x >= 0 with RN(sqrt(x)) <= r: then sqrt(x) > r  <=>  x > gt.
float sqrt_gt_threshold(float r) {
  uint32_t lo = 0, hi = 0x7F800000u;  // predicate true at lo (sqrt(0) = 0 <= r), false at +inf
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (std::sqrt(fbits(mid)) <= r) lo = mid; else hi = mid;
  }
  return fbits(lo);
}
// Smallest x >= 0 with RN(sqrt(x)) >= r: then sqrt(x) < r  <=>  x < lt.
float sqrt_lt_threshold(float r) {
  if (!(r > 0.0f)) return 0.0f;
  uint32_t lo = 0, hi = 0x7F800000u;  // false at lo (sqrt(0) < r), true at +inf
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (std::sqrt(fbits(mid)) >= r) hi = mid; else lo = mid;
  }
  return fbits(hi);
}

// Verified scene constants, process-wide (a pure function of the fp32 bit patterns and of this
// library's device code, the same on every gfx950): divisor bits -> div_c exact for all numerators;
// sun angular-size bits -> the sky-threshold search result (order key, 0xFFFFFFFF: none).
std::mutex g_verify_mu;
std::map<uint32_t, bool> g_div_ok;
std::map<uint32_t, uint32_t> g_sky_best;

uint32_t fkey(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

bool divisor_candidate(float b) { return std::isfinite(b) && b != 0.0f && std::isfinite(1.0f / b); }

// The middle band of exponent fields of rt4_verify_div_kernel for divisor b (lo > hi: none). x = m 2^e
// (field e + 127): the exact residual x - q b is a multiple of 2^(e - 47), so it is zero or normal for
// e >= -79; q, q2 and x / b (exponent e - eb + {-1, 0, 1}) stay normal and finite for
// -125 + eb <= e <= 126 + eb. Four fields of margin on each side; fields 251-255 always swept.
DivSweep div_sweep(float b, bool full) {
  DivSweep d{b, 1.0f / b, 1u, 0u};
  if (full) return d;
  int eb = 0;
  std::frexp(b, &eb);
  eb -= 1;  // b = 1.m * 2^eb
  const int e_lo = std::max(-79, -125 + eb) + 4, e_hi = std::min(122, 126 + eb) - 4;
  if (e_lo <= e_hi) {
    d.lo = static_cast<uint32_t>(e_lo + 127);
    d.hi = static_cast<uint32_t>(e_hi + 127);
  }
  return d;
}

// Verifies the divisors and the sky threshold not yet in the caches: one launch for all divisors, one
// for the threshold, one copy back.
int verify_constants(rt4_context* ctx, const std::vector<float>& divisors, bool need_sky, float ang, char* err,
                     size_t errlen) {
  std::lock_guard<std::mutex> lock(g_verify_mu);
#ifdef RT4_SETUP_TIMING
  const auto t0 = std::chrono::steady_clock::now();
#endif
  DivSweeps sw;
  std::memset(&sw, 0, sizeof sw);
  std::vector<uint32_t> todo;
  for (float b : divisors) {
    const uint32_t k = fkey(b);
    if (!divisor_candidate(b) || g_div_ok.count(k) || std::find(todo.begin(), todo.end(), k) != todo.end()) continue;
    if (todo.size() == static_cast<size_t>(MAX_DIV_SWEEPS)) break;  // the rest stays on IEEE division
    sw.d[todo.size()] = div_sweep(b, false);
    todo.push_back(k);
  }
  const bool sky = need_sky && !g_sky_best.count(fkey(ang));
  if (todo.empty() && !sky) return RT4_OK;
  const size_t n = todo.size();
  std::vector<uint32_t> res(n + 1, 0u);
  res[n] = 0xFFFFFFFFu;
  HIP_TRY(hipMemcpy(ctx->d_scratch, res.data(), (n + 1) * sizeof(uint32_t), hipMemcpyHostToDevice));
  if (n) {
    hipLaunchKernelGGL(rt4_verify_div_kernel, dim3(2048, static_cast<unsigned>(n)), dim3(256), 0, 0, sw, ctx->d_scratch);
    HIP_TRY(hipGetLastError());
  }
  if (sky) {
    const bool small = ang <= 1.0f;  // only c in (0.5, 1] can have acos_(c) < ang (rt4_sky_threshold_kernel)
    const uint32_t lo = small ? 0x3F000001u : 0u;
    const uint64_t count = small ? (0x3F800000ull - 0x3F000001ull + 1ull) : (1ull << 32);
    hipLaunchKernelGGL(rt4_sky_threshold_kernel, dim3(small ? 512 : 65536), dim3(256), 0, 0, ang, lo, count,
                       ctx->d_scratch + n);
    HIP_TRY(hipGetLastError());
  }
  HIP_TRY(hipMemcpy(res.data(), ctx->d_scratch, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost));
#ifdef RT4_SETUP_TIMING
  std::fprintf(stderr, "[rt4 set_scene] verify: %zu divisors%s, %.3f ms\n", n, sky ? " + sky threshold" : "",
               std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
#endif
  for (size_t i = 0; i < n; i++) g_div_ok[todo[i]] = res[i] == 0u;
  if (sky) g_sky_best[fkey(ang)] = res[n];
  return RT4_OK;
}

DivC make_divc(float b) {
  DivC d{b, 1.0f / b, 0, 0};
  if (divisor_candidate(b)) {
    std::lock_guard<std::mutex> lock(g_verify_mu);
    auto it = g_div_ok.find(fkey(b));
    d.fast = (it != g_div_ok.end() && it->second) ? 1 : 0;
  }
  return d;
}

// length(sun.drct) exactly as the device computes it (rt4_device_math.h dot/length)
float sun_length(const rt4_scene_desc& s) {
  const float* d = s.sun.drct;
  return std::sqrt(std::fmaf(d[3], d[3], std::fmaf(d[2], d[2], std::fmaf(d[1], d[1], d[0] * d[0]))));
}

int build_aux(rt4_context* ctx, const rt4_scene_desc& s, SceneAux* a, char* err, size_t errlen) {
  std::memset(a, 0, sizeof *a);
  {
    std::vector<float> divs;
    for (int i = 0; i < s.n_spheres; i++) divs.push_back(s.spheres[i].r);
    for (int i = 0; i < s.n_cylinders; i++) divs.push_back(s.cylinders[i].r);
    for (int i = 0; i < s.n_unions; i++) {
      divs.push_back(s.unions[i].cylinder1.r);
      divs.push_back(s.unions[i].cylinder2.r);
    }
    for (int i = 0; i < s.n_tigers; i++) {
      const rt4_tiger& t = s.tigers[i];
      for (float r : {t.inner_cyl1.r, t.outer_cyl1.r, t.inner_cyl2.r, t.outer_cyl2.r}) divs.push_back(r);
    }
    divs.push_back(s.sun.angular_size);
    divs.push_back(sun_length(s));
    const int vs = verify_constants(ctx, divs, s.final_light_mode == RT4_FINAL_LIGHT_SUN_SKY, s.sun.angular_size, err,
                                    errlen);
    if (vs != RT4_OK) return vs;
  }
  int st = RT4_OK;
  for (int i = 0; i < s.n_spheres; i++) a->sphere_r[i] = make_divc(s.spheres[i].r);
  auto cull_of = [](float r, const float* center, SphereCull* k) {  // rt4_aux.h SphereCull
    std::memset(k, 0, sizeof *k);
    std::memcpy(k->center, center, sizeof k->center);
    // SMALL_F, shader.frag:24; a NaN radius never takes the exact early-out (len_po >= NaN is false)
    k->d2_out = std::isnan(r) ? NAN : sqrt_lt_threshold(std::max(r, 0.0003f));
    const bool ok = r >= 1e-15f && r <= 1e15f;  // r <= 0: sin_oap < 1 always, never cull
    k->r2m = ok ? static_cast<float>(static_cast<double>(r) * r * (1.0 + 1e-4)) : INFINITY;
    k->r2m_pre = ok ? std::nextafter(static_cast<float>(static_cast<double>(k->r2m) * (1.0 + 1e-6)), INFINITY) : INFINITY;
  };
  for (int i = 0; i < s.n_spheres; i++) cull_of(s.spheres[i].r, s.spheres[i].center, &a->sphere_cull[i]);
  for (int i = 0; i < s.n_cylinders; i++) {
    a->cyl_r[i] = make_divc(s.cylinders[i].r);
    cull_of(s.cylinders[i].r, s.cylinders[i].point, &a->cyl_cull[i]);
  }
  for (int i = 0; i < s.n_unions; i++) {
    a->union_r[i][0] = make_divc(s.unions[i].cylinder1.r);
    a->union_r[i][1] = make_divc(s.unions[i].cylinder2.r);
    cull_of(s.unions[i].cylinder1.r, s.unions[i].cylinder1.point, &a->union_cull[i][0]);
    cull_of(s.unions[i].cylinder2.r, s.unions[i].cylinder2.point, &a->union_cull[i][1]);
    a->union_gt[i] = sqrt_gt_threshold(s.unions[i].cylinder2.r);
  }
  // bounding balls (rt4_aux.h BoundBall): R^2 = max over faces (r_self^2 + gt of the filter)
  // rA / rB: the radii of the cylinders around plane A (c1's axes) / plane B (c2's axes)
  auto bound = [](const rt4_cylinder& c1, const rt4_cylinder& c2, double r2, const float rA[2], const float rB[2],
                  BoundBall* b) {
    std::memset(b, 0, sizeof *b);
    std::memcpy(b->center, c1.point, sizeof b->center);
    std::memcpy(b->a1, c1.axis1, sizeof b->a1);
    std::memcpy(b->a2, c1.axis2, sizeof b->a2);
    const float rr[4] = {rA[0], rA[1], rB[0], rB[1]};
    for (int q = 0; q < 4; q++) {
      const double r2q = static_cast<double>(rr[q]) * rr[q];
      b->band[2 * q] = static_cast<float>(r2q * 0.99);
      b->band[2 * q + 1] = static_cast<float>(r2q * 1.01);
    }
    b->r2m = INFINITY;
    const float* ax[4] = {c1.axis1, c1.axis2, c2.axis1, c2.axis2};
    bool ok = same4(c1.point, c2.point) && std::isfinite(r2);
    // radii in [1e-15, 1e15]: a zero, negative or NaN radius makes sin_oap < -1 possible (a NaN hit
    // anywhere, found by tests/test_gpu_random_scenes.py test_special_radii), and for tiny radii the
    // fp32 rounding of r^2 is no longer within the band's 1 %
    for (int q = 0; q < 4; q++) ok = ok && rr[q] >= 1e-15f && rr[q] <= 1e15f;
    for (int i = 0; i < 4 && ok; i++)
      for (int j = i; j < 4 && ok; j++) {
        double d = 0;
        for (int k = 0; k < 4; k++) d += static_cast<double>(ax[i][k]) * ax[j][k];
        ok = std::isfinite(d) && (i == j ? std::fabs(d - 1.0) <= 1e-6 : std::fabs(d) <= 1e-6);
      }
    for (int k = 0; k < 4 && ok; k++) ok = std::isfinite(c1.point[k]) && std::fabs(c1.point[k]) < 1e15f;
    if (ok && r2 < 1e30) b->r2m = std::nextafter(static_cast<float>(r2 * (1.0 + 1e-3)), INFINITY);
  };
  for (int i = 0; i < s.n_unions; i++) {  // both filters use gt(cylinder2.r) (shader.frag:286,290)
    const rt4_cylinders_union& u = s.unions[i];
    const double g = sqrt_gt_threshold(u.cylinder2.r);
    const double r1 = u.cylinder1.r, r2 = u.cylinder2.r;
    const float rA[2] = {u.cylinder1.r, u.cylinder1.r}, rB[2] = {u.cylinder2.r, u.cylinder2.r};
    bound(u.cylinder1, u.cylinder2, std::max(r1 * r1, r2 * r2) + g, rA, rB, &a->union_bound[i]);
  }
  for (int i = 0; i < s.n_tigers; i++) {
    const rt4_tiger& t = s.tigers[i];
    const double g1 = sqrt_gt_threshold(t.outer_cyl2.r), g2 = sqrt_gt_threshold(t.outer_cyl1.r);
    const double o1 = std::max(std::fabs(t.inner_cyl1.r), std::fabs(t.outer_cyl1.r));
    const double o2 = std::max(std::fabs(t.inner_cyl2.r), std::fabs(t.outer_cyl2.r));
    const float rA[2] = {t.inner_cyl1.r, t.outer_cyl1.r}, rB[2] = {t.inner_cyl2.r, t.outer_cyl2.r};
    bound(t.inner_cyl1, t.inner_cyl2, std::max(o1 * o1 + g1, o2 * o2 + g2), rA, rB, &a->tiger_bound[i]);
  }
  for (int i = 0; i < 1 && i < s.n_hypercubes; i++)  // rt4_aux.h hyper_cells
    for (int k = 0; k < 8; k++) {
      const rt4_cube& cu = s.hypercubes[i].cubes[k];
      float* d = a->hyper_cells[k];
      std::memcpy(d, cu.point, 16);
      std::memcpy(d + 4, cu.norm, 16);
      std::memcpy(d + 8, cu.x, 16);
      std::memcpy(d + 12, cu.y, 16);
      std::memcpy(d + 16, cu.z, 16);
      d[20] = cu.r;
    }
  for (int i = 0; i < s.n_hypercubes; i++) {  // rt4_aux.h hyper_axis
    bool canon = true;
    for (int k = 0; k < 8; k++) {
      const rt4_cube& cu = s.hypercubes[i].cubes[k];
      for (int q = 0; q < 4; q++) {
        const float want = q != (k & 3) ? 0.0f : (k < 4 ? 1.0f : -1.0f);
        canon = canon && cu.norm[q] == want && std::fabs(cu.point[q]) < 1e30f;  // -0 == 0
      }
    }
    a->hyper_axis[i] = canon ? 1 : 0;
  }
  for (int i = 0; i < s.n_hypercubes; i++) {  // rt4_aux.h hyper_bound
    BoundBall& b = a->hyper_bound[i];
    std::memset(&b, 0, sizeof b);
    b.r2m = INFINITY;
    double c[4] = {0, 0, 0, 0};
    for (int k = 0; k < 8; k++)
      for (int q = 0; q < 4; q++) c[q] += s.hypercubes[i].cubes[k].point[q] / 8.0;
    double r2 = 0, cmax = 0;
    bool ok = true;
    for (int k = 0; k < 8 && ok; k++) {
      const rt4_cube& cu = s.hypercubes[i].cubes[k];
      const float* v[4] = {cu.norm, cu.x, cu.y, cu.z};
      for (int p = 0; p < 4 && ok; p++)
        for (int q = p; q < 4 && ok; q++) {
          double d = 0;
          for (int m = 0; m < 4; m++) d += static_cast<double>(v[p][m]) * v[q][m];
          ok = std::isfinite(d) && (p == q ? std::fabs(d - 1.0) <= 1e-6 : std::fabs(d) <= 1e-6);
        }
      double e = 0;
      for (int q = 0; q < 4; q++) e += (cu.point[q] - c[q]) * (cu.point[q] - c[q]);
      r2 = std::max(r2, e + 3.0 * cu.r * cu.r);
      for (int q = 0; q < 4; q++) cmax = std::max(cmax, std::fabs(static_cast<double>(cu.point[q])));
      ok = ok && std::isfinite(cu.r) && cu.r >= 0.0f && cmax < 1e15;
    }
    for (int q = 0; q < 4; q++) b.center[q] = static_cast<float>(c[q]);
    // absolute coordinates round too: + (1e-5 max|coord|)^2
    if (ok) b.r2m = std::nextafter(static_cast<float>(r2 * (1.0 + 1e-3) + 1e-10 * cmax * cmax), INFINITY);
  }
  for (int i = 0; i < s.n_tigers; i++) {
    const rt4_tiger& t = s.tigers[i];
    const float rs[4] = {t.inner_cyl1.r, t.outer_cyl1.r, t.inner_cyl2.r, t.outer_cyl2.r};
    for (int k = 0; k < 4; k++) a->tiger_r[i][k] = make_divc(rs[k]);
    const float* cps[4] = {t.inner_cyl1.point, t.outer_cyl1.point, t.inner_cyl2.point, t.outer_cyl2.point};
    for (int k = 0; k < 4; k++) cull_of(rs[k], cps[k], &a->tiger_cull[i][k]);
    a->tiger_gt[i][0] = sqrt_gt_threshold(t.outer_cyl2.r);
    a->tiger_lt[i][0] = sqrt_lt_threshold(t.inner_cyl2.r);
    a->tiger_gt[i][1] = sqrt_gt_threshold(t.outer_cyl1.r);
    a->tiger_lt[i][1] = sqrt_lt_threshold(t.inner_cyl1.r);
  }
  a->sun_ang = make_divc(s.sun.angular_size);
  if (s.final_light_mode == RT4_FINAL_LIGHT_SUN_SKY) {  // sky threshold (rt4_aux.h), verify_constants
    uint32_t best;
    {
      std::lock_guard<std::mutex> lock(g_verify_mu);
      best = g_sky_best.at(fkey(s.sun.angular_size));
    }
    if (best == 0xFFFFFFFFu) {
      a->sky_c_star = INFINITY;  // acos never below the angular size: always sky
    } else {
      const uint32_t bits = (best & 0x80000000u) ? (best & 0x7FFFFFFFu) : ~best;
      float m;
      std::memcpy(&m, &bits, 4);
      a->sky_c_star = std::nextafter(m, -INFINITY);
    }
  } else {
    a->sky_c_star = -INFINITY;
  }
  if (st == RT4_OK) {
    const float len = sun_length(s);
    a->sun_len = make_divc(len);
    // Sky pre-test constant (rt4_aux.h sky_pre_k). With a*a < l2*K computed in fp32 (3 roundings) the
    // exact ratio a / (sqrt(l2) len) is below c* (1 - 4.9e-6); the kernel's v_cos (3 more roundings)
    // stays below c* (1 - 4.6e-6) <= c*, i.e. the sky branch. Needs c* > 0 and K well inside the
    // normal range so that the two products cannot underflow or overflow for l2 in [2^-40, 2^40].
    a->sky_pre_k = 0.0f;
    const double c = a->sky_c_star;
    if (s.final_light_mode == RT4_FINAL_LIGHT_SUN_SKY && std::isfinite(c) && c > 0.0 && std::isfinite(len) && len > 0.0f) {
      const double k = c * c * static_cast<double>(len) * len * (1.0 - 1e-5);
      if (k >= 0x1p-40 && k <= 0x1p40) a->sky_pre_k = static_cast<float>(k);
    }
  }
  if (st != RT4_OK) return st;
  HotSky& hs = a->hot_sky;  // rt4_aux.h HotSky
  std::memcpy(hs.sky, s.sky_light, sizeof hs.sky);
  hs.pre_k = a->sky_pre_k;
  std::memcpy(hs.sun_drct, s.sun.drct, sizeof hs.sun_drct);
  std::memcpy(hs.const_rgb, s.final_light_const, sizeof hs.const_rgb);
  hs.mode = s.final_light_mode;
  const bool pre_ok = s.final_light_mode == RT4_FINAL_LIGHT_SUN_SKY && a->sky_c_star > 0.0f;  // finite or +inf
  hs.pre_a = pre_ok ? 0.0f : -INFINITY;
  if (!pre_ok) hs.pre_k = 0.0f;
  // flat primitive table (rt4_aux.h)
  int n = 0;
  auto add = [&](int kind, const float* p, const float* a1, const float* a2, float r, const DivC& dc,
                 const rt4_material& m) {
    PrimEntry& e = a->prims[n++];
    std::memcpy(e.p, p, sizeof e.p);
    if (a1) std::memcpy(e.a1, a1, sizeof e.a1);
    if (a2) std::memcpy(e.a2, a2, sizeof e.a2);
    e.r = r;
    e.y = dc.y;
    e.fast = dc.fast;
    e.kind = kind;
    e.glow = m.glow;
    e.refl = m.refl_prob;
    std::memcpy(e.color, m.color, sizeof e.color);
  };
  const DivC none{0.0f, 0.0f, 0, 0};
  for (int i = 0; i < s.n_spaces; i++) add(PK_SPACE, s.spaces[i].norm, nullptr, nullptr, 0.0f, none, s.spaces[i].material);
  a->base_sphere = n;
  for (int i = 0; i < s.n_spheres; i++)
    add(PK_SPHERE, s.spheres[i].center, nullptr, nullptr, s.spheres[i].r, a->sphere_r[i], s.spheres[i].material);
  a->base_cyl = n;
  for (int i = 0; i < s.n_cylinders; i++) {
    const rt4_cylinder& c = s.cylinders[i];
    add(PK_CYLINDER, c.point, c.axis1, c.axis2, c.r, a->cyl_r[i], c.material);
  }
  a->base_union = n;
  for (int i = 0; i < s.n_unions; i++) {
    const rt4_cylinder* cs[2] = {&s.unions[i].cylinder1, &s.unions[i].cylinder2};
    for (int k = 0; k < 2; k++) add(PK_CYLINDER, cs[k]->point, cs[k]->axis1, cs[k]->axis2, cs[k]->r, a->union_r[i][k], cs[k]->material);
  }
  a->base_cube = n;
  for (int i = 0; i < s.n_hypercubes; i++)
    for (int k = 0; k < 8; k++) {
      const rt4_cube& c = s.hypercubes[i].cubes[k];
      add(PK_CUBE, c.norm, nullptr, nullptr, 0.0f, none, c.material);
    }
  a->base_tiger = n;
  for (int i = 0; i < s.n_tigers; i++) {
    const rt4_tiger& t = s.tigers[i];
    const rt4_cylinder* cs[4] = {&t.inner_cyl1, &t.outer_cyl1, &t.inner_cyl2, &t.outer_cyl2};
    for (int k = 0; k < 4; k++) add(PK_CYLINDER, cs[k]->point, cs[k]->axis1, cs[k]->axis2, cs[k]->r, a->tiger_r[i][k], cs[k]->material);
  }
  a->n_prims = n;
  return RT4_OK;
}

}  // namespace

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
  hipError_t e = hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device);
  if (e == hipSuccess) e = hipMalloc(&c->d_scene, kSceneBytes);
  if (e == hipSuccess) e = hipMalloc(&c->d_scratch, (MAX_DIV_SWEEPS + 1) * sizeof(unsigned));
  if (e == hipSuccess) e = hipMalloc(&c->d_queue, QUEUE_SLOTS * sizeof(unsigned));
  if (e == hipSuccess) e = hipMalloc(&c->d_eval, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->d_eval, 0, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->d_queue, 0, QUEUE_SLOTS * sizeof(unsigned));
  if (e == hipSuccess) e = hipDeviceSynchronize();  // zeroed before any stream's first launch
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  for (int k = 0; k < RT4_OVERLAP_SLOTS && e == hipSuccess; k++) {
    e = hipEventCreateWithFlags(&c->seq_done[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->traced[k], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventRecord(c->seq_done[k], nullptr);  // "launches -S .. -1" are complete
  }
  if (e == hipSuccess) e = hipMalloc(&c->d_ocount, RT4_OVERLAP_SLOTS * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->d_ocount, 0, RT4_OVERLAP_SLOTS * sizeof(unsigned long long));
  if (e == hipSuccess) {  // tile order for frames up to 2^18 tiles (16.7 M pixels); larger ones grow it once
    e = hipMalloc(&c->d_order, ((size_t(1) << 18) + 2) * sizeof(unsigned));
    if (e == hipSuccess) c->order_cap = size_t(1) << 18;
  }
  if (e == hipSuccess) {
    // The first host<->device copies of the process (the runtime sets up its staging buffers: ~7 ms,
    // tools/setscene_probe.py) and first launches of the two scene-verification kernels, with no
    // work, so that one-time runtime set-up is paid here instead of in the first set_scene.
    std::vector<char> zeros(kSceneBytes, 0);  // the sizes set_scene copies (pageable host memory)
    e = hipMemcpy(c->d_scene, zeros.data(), kSceneBytes, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(zeros.data(), c->d_scratch, (MAX_DIV_SWEEPS + 1) * sizeof(unsigned), hipMemcpyDeviceToHost);
    DivSweeps sw;
    std::memset(&sw, 0, sizeof sw);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(rt4_verify_div_kernel, dim3(1, 1), dim3(64), 0, 0, sw, c->d_scratch);
      hipLaunchKernelGGL(rt4_sky_threshold_kernel, dim3(1), dim3(64), 0, 0, 1.0f, 0u, 0ull, c->d_scratch);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
  }
  if (e == hipSuccess && (flags & RT4_FLAG_SAMPLER_LUT)) {
    // Diagnostic (round 6): RT4_WLUT_ALLOC=fine|uncached places the table in fine-grained or
    // uncached device memory, to measure whether a 4-B gather then leaves L2 as a smaller fabric request. The
    // default (coarse-grained hipMalloc) is what every product launch uses; images do not depend on it.
    const char* wa = std::getenv("RT4_WLUT_ALLOC");
    unsigned wflags = !wa ? hipDeviceMallocDefault
                          : !std::strcmp(wa, "fine")     ? hipDeviceMallocFinegrained
                          : !std::strcmp(wa, "uncached") ? hipDeviceMallocUncached
                                                         : hipDeviceMallocDefault;
    e = wflags == hipDeviceMallocDefault
            ? hipMalloc(&c->d_wlut, (sizeof(WEntry) << 23) * RT4_ABL_WLUT_STRIDE)
            : hipExtMallocWithFlags(reinterpret_cast<void**>(&c->d_wlut),(sizeof(WEntry) << 23) * RT4_ABL_WLUT_STRIDE, wflags);
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
  if (ctx->launched) (void)hipEventSynchronize(ctx->done);  // frames in flight (side streams included)
  if (ctx->d_scene) (void)hipFree(ctx->d_scene);
  if (ctx->d_wlut) (void)hipFree(ctx->d_wlut);
  if (ctx->d_queue) (void)hipFree(ctx->d_queue);
  if (ctx->d_order) (void)hipFree(ctx->d_order);
  if (ctx->d_fcolor) (void)hipFree(ctx->d_fcolor);
  if (ctx->done) (void)hipEventDestroy(ctx->done);
  for (int k = 0; k < RT4_OVERLAP_SLOTS; k++) {
    if (ctx->side[k]) {
      (void)hipStreamSynchronize(ctx->side[k]);
      (void)hipStreamDestroy(ctx->side[k]);
    }
    if (ctx->traced[k]) (void)hipEventDestroy(ctx->traced[k]);
    if (ctx->seq_done[k]) (void)hipEventDestroy(ctx->seq_done[k]);
    if (ctx->d_ofcolor[k]) (void)hipFree(ctx->d_ofcolor[k]);
  }
  if (ctx->d_ocount) (void)hipFree(ctx->d_ocount);
  if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
  if (ctx->d_eval) (void)hipFree(ctx->d_eval);
  delete ctx;
}

int rt4_context_set_scene(rt4_context* ctx, const rt4_scene_desc* scene, char* err, size_t errlen) {
  if (!ctx || !scene) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  int st = rt4_scene_validate(scene, err, errlen);
  if (st != RT4_OK) return st;
  HIP_TRY(hipSetDevice(ctx->device));
#ifdef RT4_SETUP_TIMING  // diagnostic build only (tools/setscene_probe.py): host time of each phase
  const auto t0 = std::chrono::steady_clock::now();
#endif
  st = build_aux(ctx, *scene, &ctx->aux, err, errlen);
  if (st != RT4_OK) return st;
#ifdef RT4_SETUP_TIMING
  const auto t1 = std::chrono::steady_clock::now();
#endif
  // A frame still in flight on a caller's (non-blocking) stream reads d_scene: let it finish first.
  if (ctx->launched) HIP_TRY(hipEventSynchronize(ctx->done));
  HIP_TRY(hipMemcpy(ctx->d_scene, scene, sizeof(rt4_scene_desc), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(reinterpret_cast<char*>(ctx->d_scene) + kAuxOffset, &ctx->aux, sizeof(SceneAux),
                    hipMemcpyHostToDevice));
#ifdef RT4_SETUP_TIMING
  const auto t2 = std::chrono::steady_clock::now();
  std::fprintf(stderr, "[rt4 set_scene] build_aux+verify %.3f ms, upload %.3f ms\n",
               std::chrono::duration<double, std::milli>(t1 - t0).count(),
               std::chrono::duration<double, std::milli>(t2 - t1).count());
#endif
  ctx->shape = (ctx->flags & RT4_FLAG_GENERIC_KERNEL) ? GENERIC : scene_shape(*scene);
  ctx->has_scene = true;
  ctx->order_valid = false;  // the tile order was for the previous scene
  return RT4_OK;
}

uint32_t rt4_context_kernel_shape(const rt4_context* ctx) { return ctx && ctx->has_scene ? ctx->shape : 0u; }

}  // extern "C"

namespace {

// The uniforms every job of one launch shares (KernelArgs), compared bit for bit.
bool same_shared_uniforms(const rt4_uniforms& a, const rt4_uniforms& b) {
  return a.seed == b.seed && a.samples == b.samples && a.reflections_amount == b.reflections_amount &&
         std::memcmp(&a.small_indent, &b.small_indent, 4) == 0 && std::memcmp(&a.part, &b.part, 4) == 0 &&
         std::memcmp(&a.light_to_color_conversion_coefficient, &b.light_to_color_conversion_coefficient, 4) == 0 &&
         std::memcmp(a.focus, b.focus, sizeof a.focus) == 0;
}

// Frames pipelined in one launch (rt4_render_frames_device): per-frame seed and part of job 0.
struct FramePlan {
  int32_t n;
  const int32_t* seeds;
  const float* parts;
};

// The trace kernel a launch of the context runs: its scene's shape, the sampler table, primary reuse.
TraceFn trace_fn_of(const rt4_context* ctx) {
  const bool reuse = (ctx->flags & RT4_FLAG_PRIMARY_REUSE) && ctx->shape != GENERIC;
  return variant_for(ctx->shape).trace[ctx->d_wlut ? 1 : 0][reuse ? 1 : 0];
}

// Blocks per CU the trace kernel fn holds (occupancy query, cached per kernel).
int occupancy_of(rt4_context* ctx, TraceFn fn, int* per_cu, char* err, size_t errlen) {
  if (ctx->occ_fn != fn) {
    int n = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(fn), 256, 0));
    ctx->occ_fn = fn;
    ctx->occ_per_cu = n;
  }
  *per_cu = ctx->occ_per_cu;
  return RT4_OK;
}

// An overlapped launch of `items` 8x8 tiles runs deep (RT4_OVERLAP_SLOTS in flight) when it has fewer tiles than
// the chip holds waves, unless the context caps the overlap (RT4_FLAG_OVERLAP_SHALLOW).
bool overlap_deep(const rt4_context* ctx, long long items, int per_cu) {
  if (ctx->flags & RT4_FLAG_OVERLAP_SHALLOW) return false;
  return items < static_cast<long long>(ctx->n_cu) * (per_cu > 0 ? per_cu : 1) * 4;
}

// Slot buffer k holds at least `need` bytes. Growing it first waits for every launch in flight (a buffer may be
// in use by any of them). kSlotNoMem when the allocation fails (the caller then runs the frame serially).
constexpr int kSlotNoMem = 1;
int ensure_overlap_buffer(rt4_context* ctx, unsigned k, size_t need, char* err, size_t errlen) {
  if (ctx->ofcolor_cap[k] >= need) return RT4_OK;
  if (ctx->launched) HIP_TRY(hipEventSynchronize(ctx->done));
  for (int q = 0; q < RT4_OVERLAP_SLOTS; q++)
    if (ctx->side[q]) HIP_TRY(hipStreamSynchronize(ctx->side[q]));
  if (ctx->d_ofcolor[k]) (void)hipFree(ctx->d_ofcolor[k]);
  ctx->d_ofcolor[k] = nullptr;
  ctx->ofcolor_cap[k] = 0;
  if (hipMalloc(&ctx->d_ofcolor[k], need) != hipSuccess) {
    (void)hipGetLastError();  // not sticky for the launch that follows
    ctx->d_ofcolor[k] = nullptr;
    return kSlotNoMem;
  }
  ctx->ofcolor_cap[k] = need;
  return RT4_OK;
}

int launch_jobs(rt4_context* ctx, const rt4_section_job* jobs, int32_t n_jobs, int32_t format,
                unsigned long long* d_counter, void* stream, char* err, size_t errlen, const FramePlan* fp = nullptr) {
  if (!ctx || !jobs) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (!ctx->has_scene) return rt4_set_err(err, errlen, "context has no scene (rt4_context_set_scene)"), RT4_ERR_ARG;
  if (n_jobs < 1 || n_jobs > RT4_MAX_SECTIONS)
    return rt4_set_err(err, errlen, "n_jobs %d not in [1, %d]", n_jobs, RT4_MAX_SECTIONS), RT4_ERR_ARG;
  if (rt4_frame_format_bytes(format) == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  KernelArgs a;
  std::memset(&a, 0, sizeof a);
  const rt4_uniforms& u0 = jobs[0].u;
  a.seed = u0.seed;
  a.samples = u0.samples;
  a.reflections_amount = u0.reflections_amount;
  a.small_indent = u0.small_indent;
  a.part = u0.part;
  a.k = u0.light_to_color_conversion_coefficient;
  std::memcpy(a.focus, u0.focus, sizeof a.focus);
  a.format = format;
  a.n_jobs = n_jobs;
  unsigned tiles = 0;
  for (int q = 0; q < RT4_MAX_SECTIONS; q++) a.jobs[q].tile_base = 0xFFFFFFFFu;
  for (int q = 0; q < n_jobs; q++) {
    const rt4_section_job& jb = jobs[q];
    int st = rt4_check_render_args(&jb.u, &jb.region, jb.row_stride_px, err, errlen);
    if (st != RT4_OK) return st;
    if (!same_shared_uniforms(jb.u, u0))
      return rt4_set_err(err, errlen, "job %d: seed/samples/reflections/small_indent/part/k/focus differ from job 0", q),
             RT4_ERR_ARG;
    const bool empty = jb.region.w == 0 || jb.region.h == 0;
    if (!empty && !jb.d_frame) return rt4_set_err(err, errlen, "job %d: NULL frame", q), RT4_ERR_ARG;
    JobArgs& J = a.jobs[q];
    std::memcpy(J.resolution, jb.u.resolution, sizeof J.resolution);
    std::memcpy(J.mtr_sizes, jb.u.mtr_sizes, sizeof J.mtr_sizes);
    std::memcpy(J.vec_to_mtr, jb.u.vec_to_mtr, sizeof J.vec_to_mtr);
    std::memcpy(J.top_drct, jb.u.top_drct, sizeof J.top_drct);
    std::memcpy(J.right_drct, jb.u.right_drct, sizeof J.right_drct);
    J.reg = jb.region;
    J.frame = jb.d_frame;
    J.row_stride_px = jb.row_stride_px;
    J.tiles_x = empty ? 1u : static_cast<unsigned>((jb.region.w + 7) / 8);
    const unsigned t = empty ? 0u : J.tiles_x * static_cast<unsigned>((jb.region.h + 7) / 8);
    J.tile_base = tiles;
    tiles += t;
  }
  if (tiles == 0) return RT4_OK;
  a.total = tiles * 64u;
  a.n_frames = 1;
  const bool frames = fp && fp->n > 1;
  if (frames) {
    if (n_jobs != 1 || fp->n > RT4_MAX_FRAMES || a.jobs[0].reg.w > 8191 || a.jobs[0].reg.h > 8191 ||
        static_cast<uint64_t>(tiles) * 64u * static_cast<uint64_t>(fp->n) >= (1ull << 31))
      return rt4_set_err(err, errlen, "pipelined frames: bad frame plan"), RT4_ERR_ARG;
    a.n_frames = fp->n;
    a.frame_tiles = tiles;
    a.total = tiles * 64u * static_cast<unsigned>(fp->n);
    for (int f = 0; f < fp->n; f++) {
      a.frame_seed[f] = fp->seeds[f];
      a.frame_part[f] = fp->parts[f];
    }
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // Overlapped single frames: one image, one frame, a region the frame-colour pixel word
  // holds; the trace goes to a side stream and its frame colours to a slot buffer, the fold to the caller's
  // stream, so this frame's trace fills the GPU while the previous one drains.
  // Sections (rt4_render_sections_device, three_window_group.cpp:42-46) overlap too: the pixel word's frame field
  // then names the section, and the slot buffer holds the sections' images one after another (JobArgs::fc_base).
  bool small_regions = true;
  size_t npx_all = 0;
  for (int q = 0; q < n_jobs; q++) {
    small_regions = small_regions && a.jobs[q].reg.w <= 8191 && a.jobs[q].reg.h <= 8191;
    npx_all += static_cast<size_t>(a.jobs[q].reg.w) * static_cast<size_t>(a.jobs[q].reg.h);
  }
  bool overlap = RT4_OVERLAP_FRAMES && !(ctx->flags & RT4_FLAG_SERIAL_FRAMES) && !frames && small_regions &&
                 npx_all < (size_t(1) << 31);
  const unsigned slot = ctx->launch_seq % RT4_OVERLAP_SLOTS;
  const Variant& v = variant_for(ctx->shape);
  const bool reuse = (ctx->flags & RT4_FLAG_PRIMARY_REUSE) && ctx->shape != GENERIC;
  const TraceFn fn = trace_fn_of(ctx);
  // grid: what the device holds at once; later blocks would only find the queue empty
  int per_cu = 0;
  {
    const int st = occupancy_of(ctx, fn, &per_cu, err, errlen);
    if (st != RT4_OK) return st;
  }
  const long long items = static_cast<long long>(a.total >> 6);  // tiles of all jobs (and frames)
  // an overlapped frame with fewer tiles than the chip holds waves runs deep: up to RT4_OVERLAP_SLOTS in flight
  const bool deep = overlap && overlap_deep(ctx, items, per_cu);
  if (overlap) {
    const int st = ensure_overlap_buffer(ctx, deep ? slot : ctx->launch_seq % RT4_OVERLAP_BIG, npx_all * sizeof(float4),
                                         err, errlen);
    if (st == kSlotNoMem) overlap = false;  // no memory for the slot buffer: this frame runs serially
    else if (st != RT4_OK) return st;
  }
  hipStream_t ts = s;  // the trace kernel's stream
  if (overlap) {
    for (int q = 1; q < n_jobs; q++)
      a.jobs[q].fc_base = a.jobs[q - 1].fc_base + static_cast<unsigned>(a.jobs[q - 1].reg.w) * static_cast<unsigned>(a.jobs[q - 1].reg.h);
    a.fcolor = static_cast<float4*>(ctx->d_ofcolor[deep ? slot : ctx->launch_seq % RT4_OVERLAP_BIG]);
    a.frame_part[0] = a.part;
  }
  int bpc = per_cu > 0 ? per_cu : 1;
  const unsigned long long frame_work = static_cast<unsigned long long>(a.total) * static_cast<unsigned>(a.samples) *
                                       static_cast<unsigned>(a.reflections_amount + 1);
  if (overlap && frame_work <= RT4_OVERLAP_SHORT_WORK) bpc = bpc > RT4_OVERLAP_GRID_LESS ? bpc - RT4_OVERLAP_GRID_LESS : 1;
  long long blocks = static_cast<long long>(ctx->n_cu) * bpc;
  if (overlap) {
    const unsigned sidx = ctx->launch_seq % (deep ? RT4_OVERLAP_SLOTS : RT4_OVERLAP_BIG);
    if (!ctx->side[sidx]) {
      if (RT4_SIDE_LOW_PRIORITY) {
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&ctx->side[sidx], hipStreamNonBlocking, least));
      } else {
        HIP_TRY(hipStreamCreateWithFlags(&ctx->side[sidx], hipStreamNonBlocking));
      }
    }
    ts = ctx->side[sidx];
  }
  if (blocks > (items + 3) / 4) blocks = (items + 3) / 4;  // >= one tile per wave
  if (blocks < 1) blocks = 1;
  a.order = nullptr;
  a.order_ends = nullptr;
  if (reuse) a.eval_counter = ctx->d_eval;
  // The tile order buffer is one per context: a launch on another stream than the previous one
  // waits for it (launches of one context run in submission order). So does an overlapped launch that
  // switches between the deep and the big rotation (they share slot buffers 0 .. RT4_OVERLAP_BIG - 1).
  if (ctx->launched && (s != ctx->last_stream || (overlap && ctx->overlapped && deep != ctx->last_deep)))
    HIP_TRY(hipStreamWaitEvent(ts, ctx->done, 0));
  // launch s - S is complete before launch s starts: its queue word, frame-colour slot and count slot are
  // free again (launches s - S + 1 .. s - 1 may still be draining: that is the overlap)
  HIP_TRY(hipStreamWaitEvent(ts, ctx->seq_done[slot], 0));
  if (!deep && RT4_OVERLAP_BIG < RT4_OVERLAP_SLOTS)  // and launch s - RT4_OVERLAP_BIG (a frame that fills the chip)
    HIP_TRY(hipStreamWaitEvent(ts, ctx->seq_done[(ctx->launch_seq + RT4_OVERLAP_SLOTS - RT4_OVERLAP_BIG) % RT4_OVERLAP_SLOTS], 0));
  if (frames) {  // the frame colours of a pipelined launch: one scratch buffer per context, grown to the
    // launch's frames (rt4_context_reserve_frames sizes it for a whole chunk ahead of time)
    const size_t need = static_cast<size_t>(fp->n) * static_cast<size_t>(a.jobs[0].reg.w) *
                        static_cast<size_t>(a.jobs[0].reg.h) * sizeof(float4);
    if (ctx->fcolor_bytes < need) {
      HIP_TRY(hipStreamSynchronize(s));
      if (ctx->d_fcolor) (void)hipFree(ctx->d_fcolor);
      ctx->d_fcolor = nullptr;
      ctx->fcolor_bytes = 0;
      HIP_TRY(hipMalloc(&ctx->d_fcolor, need));
      ctx->fcolor_bytes = need;
    }
    a.fcolor = static_cast<float4*>(ctx->d_fcolor);
  }
#if RT4_ORDER_PREPASS
  // Pipelined frames keep row-major order: the longest-first order only shortens the drain at the end
  // of a launch, which a pipelined launch pays once, and in the main phase row-major measured faster
  // (config 2 +1.5 %, config 3 +2 %; profiles/r02_ab.txt).
  if ((!frames || RT4_LAST_FRAME_ORDER == 2) && !overlap) {
  if (ctx->order_cap < tiles) {  // a frame larger than any before: grow once (allocates)
    HIP_TRY(hipStreamSynchronize(s));
    if (ctx->d_order) (void)hipFree(ctx->d_order);
    ctx->d_order = nullptr;
    ctx->order_cap = 0;
    ctx->order_valid = false;
    HIP_TRY(hipMalloc(&ctx->d_order, (static_cast<size_t>(tiles) + 2) * sizeof(unsigned)));
    ctx->order_cap = tiles;
  }
  unsigned* ends = ctx->d_order + ctx->order_cap;
  // The order depends only on the scene and the primary rays (camera, regions, resolution): a frame
  // that repeats them (progressive accumulation, a benchmark loop) reuses the previous order.
  KernelArgs ao = a;  // the order is per frame: one frame's tiles
  ao.total = tiles * 64u;
  ao.n_frames = 1;
  if (!(ctx->order_valid && same_primary_rays(ctx->order_args, ao))) {
    ctx->order_valid = false;
    HIP_TRY(hipMemsetAsync(ends, 0, 2 * sizeof(unsigned), s));
    hipLaunchKernelGGL(v.order, dim3((tiles + 255u) / 256u), dim3(256), 0, s, ctx->d_scene, scene_aux(ctx), ao,
                       ctx->d_order, ends);
    HIP_TRY(hipGetLastError());
    ctx->order_args = ao;
    ctx->order_valid = true;
  }
  a.order = ctx->d_order;
  a.order_ends = ends;
  }
#endif
  // Queue words rotate; launch s zeroes launch s + S's word (launches up to s + S - 1 may already be running,
  // s + S starts only after s is complete): no memset between frames.
  unsigned* q = ctx->d_queue + (ctx->launch_seq % QUEUE_SLOTS);
  unsigned* q_next = ctx->d_queue + ((ctx->launch_seq + RT4_OVERLAP_SLOTS) % QUEUE_SLOTS);  // zeroed by this launch
  const unsigned seq = ctx->launch_seq++;
  if (ctx->q_dirty[seq % QUEUE_SLOTS]) {
    HIP_TRY(hipMemsetAsync(q, 0, sizeof(unsigned), ts));
    ctx->q_dirty[seq % QUEUE_SLOTS] = false;
  }
  if (overlap) {
    ctx->overlapped = true;
    ctx->last_deep = deep;
  }
  unsigned long long* count = overlap ? ctx->d_ocount + slot : d_counter;
  (void)hipGetLastError();  // a sticky error of an earlier, unrelated call must not be taken for this launch's
  hipLaunchKernelGGL(fn, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, ts, ctx->d_scene, scene_aux(ctx), a, count,
                     ctx->d_wlut, q, q_next);
  hipError_t le = hipGetLastError();
  const bool trace_enqueued = le == hipSuccess;
  if (le == hipSuccess && overlap) {
    le = hipEventRecord(ctx->traced[slot], ts);
    if (le == hipSuccess) le = hipStreamWaitEvent(s, ctx->traced[slot], 0);
  }
  if (le == hipSuccess && (frames || overlap)) {
    long long npx = 0;  // the largest image's pixels (blockIdx.y: the section)
    for (int q = 0; q < n_jobs; q++) npx = std::max(npx, static_cast<long long>(a.jobs[q].reg.w) * a.jobs[q].reg.h);
    hipLaunchKernelGGL(rt4_fold_frames_kernel, dim3(static_cast<unsigned>((npx + 255) / 256), static_cast<unsigned>(n_jobs)),
                       dim3(256), 0, s, a,
                       overlap ? count : nullptr, overlap ? d_counter : nullptr);
    le = hipGetLastError();
  }
  // Record the events whatever happened: a launch that may have been enqueued still orders the next
  // launch on another stream behind it (they share d_order / the queue words).
  const hipError_t re2 = hipEventRecord(ctx->seq_done[slot], s);
  hipError_t re = hipEventRecord(ctx->done, s);
  if (re == hipSuccess) re = re2;
  ctx->last_stream = s;
  ctx->launched = true;
  if (le != hipSuccess) {
    ctx->q_dirty[(seq + RT4_OVERLAP_SLOTS) % QUEUE_SLOTS] = true;  // q_next may not be zeroed: its next user does it
    if (overlap && trace_enqueued) {
      // the trace runs on the side stream but no fold on the caller's stream covers it: wait for it here (the
      // scene, the slot buffer and the queue words stay valid), then clear the count it left in its slot
      (void)hipStreamSynchronize(ts);
      (void)hipMemsetAsync(count, 0, sizeof(unsigned long long), s);
      // the launch that reuses this count slot waits on seq_done[slot]: record it (and done) again behind the
      // memset, so that launch's trace cannot add to the slot before it is cleared
      (void)hipEventRecord(ctx->seq_done[slot], s);
      (void)hipEventRecord(ctx->done, s);
    }
    rt4_set_err(err, errlen, "trace kernel launch failed: %s", hipGetErrorString(le));
    return RT4_ERR_HIP;
  }
  if (re != hipSuccess) {
    rt4_set_err(err, errlen, "hipEventRecord failed: %s", hipGetErrorString(re));
    return RT4_ERR_HIP;
  }
  return RT4_OK;
}

}  // namespace

extern "C" {

int rt4_render_device_ex(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, void* d_frame,
                         int32_t format, int64_t row_stride_px, unsigned long long* d_counter, void* stream,
                         char* err, size_t errlen) {
  if (!ctx || !u || !region || !d_frame) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  rt4_section_job job;
  job.u = *u;
  job.region = *region;
  job.d_frame = d_frame;
  job.row_stride_px = row_stride_px;
  return launch_jobs(ctx, &job, 1, format, d_counter, stream, err, errlen);
}

}  // extern "C"

namespace {

// Frames per pipelined launch for a w x h region (1: run frame by frame): RT4_MAX_FRAMES, the 4 GiB
// frame-colour scratch, and queue words below 2^31.
int32_t frames_per_launch(int32_t w, int32_t h) {
  if (w <= 0 || h <= 0 || w > 8191 || h > 8191) return 1;
  const size_t frame_bytes = static_cast<size_t>(w) * static_cast<size_t>(h) * 16u;
  const size_t tiles = static_cast<size_t>((w + 7) / 8) * static_cast<size_t>((h + 7) / 8);
  const size_t n = std::min<size_t>({static_cast<size_t>(RT4_MAX_FRAMES), (size_t(4) << 30) / frame_bytes,
                                     ((size_t(1) << 31) - 1) / (tiles * 64u)});
  return n < 2 ? 1 : static_cast<int32_t>(n);
}

}  // namespace

extern "C" {

int32_t rt4_context_frames_per_launch(const rt4_context* ctx, int32_t w, int32_t h) {
  // Every scene pipelines since r03-v34: the mirror-room tiger kernel (config 4) ran 17 % slower pipelined
  // until the phase-aligned refill kept its lanes in lockstep across frames.
  return ctx ? frames_per_launch(w, h) : 1;
}

int rt4_context_reserve_frames(rt4_context* ctx, int32_t w, int32_t h, char* err, size_t errlen) {
  if (!ctx) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  // the scene's own chunk size (a scene that runs frame by frame needs no scratch)
  const int32_t cap = rt4_context_frames_per_launch(ctx, w, h);
  if (cap < 2) return RT4_OK;
  const size_t need = static_cast<size_t>(cap) * static_cast<size_t>(w) * static_cast<size_t>(h) * sizeof(float4);
  if (ctx->fcolor_bytes >= need) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->launched) HIP_TRY(hipEventSynchronize(ctx->done));
  if (ctx->d_fcolor) (void)hipFree(ctx->d_fcolor);
  ctx->d_fcolor = nullptr;
  ctx->fcolor_bytes = 0;
  HIP_TRY(hipMalloc(&ctx->d_fcolor, need));
  HIP_TRY(hipMemset(ctx->d_fcolor, 0, need));  // first touch here, not in the first pipelined launch
  ctx->fcolor_bytes = need;
  return RT4_OK;
}

int rt4_context_reserve_overlap(rt4_context* ctx, int32_t w, int32_t h, char* err, size_t errlen) {
  if (!ctx) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (w < 1 || h < 1) return rt4_set_err(err, errlen, "bad size %d x %d", w, h), RT4_ERR_ARG;
  if (!RT4_OVERLAP_FRAMES || (ctx->flags & RT4_FLAG_SERIAL_FRAMES)) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  int per_cu = 0;
  const int st = occupancy_of(ctx, trace_fn_of(ctx), &per_cu, err, errlen);
  if (st != RT4_OK) return st;
  const long long items = static_cast<long long>((w + 7) / 8) * ((h + 7) / 8);
  const bool deep = overlap_deep(ctx, items, per_cu);
  const size_t need = static_cast<size_t>(w) * static_cast<size_t>(h) * sizeof(float4);
  for (int k = 0; k < (deep ? RT4_OVERLAP_SLOTS : RT4_OVERLAP_BIG); k++) {
    const int r = ensure_overlap_buffer(ctx, static_cast<unsigned>(k), need, err, errlen);
    if (r == kSlotNoMem) return rt4_set_err(err, errlen, "slot buffer allocation of %zu bytes failed", need), RT4_ERR_HIP;
    if (r != RT4_OK) return r;
  }
  return RT4_OK;
}

uint64_t rt4_context_overlap_bytes(const rt4_context* ctx) {
  uint64_t n = 0;
  if (ctx)
    for (int k = 0; k < RT4_OVERLAP_SLOTS; k++) n += ctx->ofcolor_cap[k];
  return n;
}

int rt4_render_frames_device(rt4_context* ctx, const rt4_uniforms* u, int32_t n_frames, const rt4_region* region,
                             void* d_frame, int32_t format, int64_t row_stride_px, unsigned long long* d_counter,
                             void* stream, char* err, size_t errlen) {
  if (!ctx || !u || !region || !d_frame) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (n_frames < 1) return rt4_set_err(err, errlen, "n_frames %d < 1", n_frames), RT4_ERR_ARG;
  for (int32_t f = 1; f < n_frames; f++) {  // only seed and part may change from frame to frame
    rt4_uniforms x = u[f];
    x.seed = u[0].seed;
    x.part = u[0].part;
    if (std::memcmp(&x, &u[0], sizeof x) != 0)
      return rt4_set_err(err, errlen, "frame %d: uniforms other than seed/part differ from frame 0", f), RT4_ERR_ARG;
  }
  rt4_section_job job;
  job.u = u[0];
  job.region = *region;
  job.d_frame = d_frame;
  job.row_stride_px = row_stride_px;
  const int32_t chunk = rt4_context_frames_per_launch(ctx, region->w, region->h);
  int32_t seeds[RT4_MAX_FRAMES];
  float parts[RT4_MAX_FRAMES];
  for (int32_t f0 = 0; f0 < n_frames; f0 += chunk) {
    const int32_t n = std::min(chunk, n_frames - f0);
    int st;
    if (n == 1) {
      job.u = u[f0];
      st = launch_jobs(ctx, &job, 1, format, d_counter, stream, err, errlen);
    } else {
      for (int32_t f = 0; f < n; f++) {
        seeds[f] = u[f0 + f].seed;
        parts[f] = u[f0 + f].part;
      }
      const FramePlan fp{n, seeds, parts};
      st = launch_jobs(ctx, &job, 1, format, d_counter, stream, err, errlen, &fp);
    }
    if (st != RT4_OK) return st;
  }
  return RT4_OK;
}

int rt4_render_device(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* d_rgba,
                      int64_t row_stride_px, unsigned long long* d_counter, void* stream, char* err, size_t errlen) {
  return rt4_render_device_ex(ctx, u, region, d_rgba, RT4_FRAME_RGBA32F, row_stride_px, d_counter, stream, err,
                              errlen);
}

int rt4_render_sections_device(rt4_context* ctx, const rt4_section_job* jobs, int32_t n_jobs, int32_t format,
                               unsigned long long* d_counter, void* stream, char* err, size_t errlen) {
  return launch_jobs(ctx, jobs, n_jobs, format, d_counter, stream, err, errlen);
}

int rt4_render_host_ex(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, void* frame,
                       int32_t format, int64_t row_stride_px, uint64_t* n_intersections, char* err,
                       size_t errlen) {
  if (!ctx || !u || !region || !frame) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  int st = rt4_check_render_args(u, region, row_stride_px, err, errlen);
  if (st != RT4_OK) return st;
  const int32_t px_bytes = rt4_frame_format_bytes(format);
  if (px_bytes == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  if (n_intersections) *n_intersections = 0;
  if (region->w == 0 || region->h == 0) return RT4_OK;
  HIP_TRY(hipSetDevice(ctx->device));
  const size_t bytes = (static_cast<size_t>(region->h - 1) * row_stride_px + static_cast<size_t>(region->w)) * px_bytes;
  void* d = nullptr;
  unsigned long long* dc = nullptr;
  HIP_TRY(hipMalloc(&d, bytes));
  hipError_t e = hipMalloc(&dc, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemcpy(d, frame, bytes, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(dc, 0, sizeof(unsigned long long));
  if (e != hipSuccess) {
    (void)hipFree(d);
    if (dc) (void)hipFree(dc);
    rt4_set_err(err, errlen, "render_host staging failed: %s", hipGetErrorString(e));
    return RT4_ERR_HIP;
  }
  st = rt4_render_device_ex(ctx, u, region, d, format, row_stride_px, dc, nullptr, err, errlen);
  if (st == RT4_OK) {
    e = hipDeviceSynchronize();
    unsigned long long cnt = 0;
    if (e == hipSuccess) e = hipMemcpy(frame, d, bytes, hipMemcpyDeviceToHost);
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

int rt4_render_host(rt4_context* ctx, const rt4_uniforms* u, const rt4_region* region, float* rgba,
                    int64_t row_stride_px, uint64_t* n_intersections, char* err, size_t errlen) {
  return rt4_render_host_ex(ctx, u, region, rgba, RT4_FRAME_RGBA32F, row_stride_px, n_intersections, err, errlen);
}

uint64_t rt4_context_frame_scratch_bytes(const rt4_context* ctx) { return ctx ? ctx->fcolor_bytes : 0u; }

int rt4_bands_unpermute_device(const void* d_gathered, void* d_image, int32_t width, int32_t height, int32_t world,
                               int32_t band, int32_t rows_max, int32_t format, void* stream, char* err, size_t errlen) {
  if (!d_gathered || !d_image) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  const int32_t px = rt4_frame_format_bytes(format);
  if (px == 0) return rt4_set_err(err, errlen, "unknown frame format %d", format), RT4_ERR_ARG;
  if (width < 1 || height < 1 || world < 1 || band < 1 || rows_max < 1)
    return rt4_set_err(err, errlen, "unpermute: width, height, world, band and rows_max must be >= 1"), RT4_ERR_ARG;
  // every image row's source must lie inside the gather: the plan's rows_max (rt4_band_plan) or more
  const int64_t need = rt4_band_rows_max(height, world, band);
  if (static_cast<int64_t>(rows_max) < need)
    return rt4_set_err(err, errlen, "unpermute: rows_max %d below the plan's %lld", rows_max, static_cast<long long>(need)),
           RT4_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t row_bytes = static_cast<int64_t>(width) * px;
  const bool wide = row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(d_gathered) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(d_image) % 16 == 0;
  if (wide)
    hipLaunchKernelGGL(rt4_unpermute_kernel<uint4>, dim3(static_cast<unsigned>(height)), dim3(256), 0, s,
                       static_cast<const uint4*>(d_gathered), static_cast<uint4*>(d_image),
                       static_cast<int32_t>(row_bytes / 16), world, band, rows_max);
  else
    hipLaunchKernelGGL(rt4_unpermute_kernel<uint32_t>, dim3(static_cast<unsigned>(height)), dim3(256), 0, s,
                       static_cast<const uint32_t*>(d_gathered), static_cast<uint32_t*>(d_image),
                       static_cast<int32_t>(row_bytes / 4), world, band, rows_max);
  HIP_TRY(hipGetLastError());
  return RT4_OK;
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

int rt4_debug_verify_sqrt(rt4_context* ctx, uint64_t* mismatches, char* err, size_t errlen) {
  if (!ctx || !mismatches) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  HIP_TRY(hipSetDevice(ctx->device));
  unsigned long long* d = nullptr;
  HIP_TRY(hipMalloc(&d, sizeof(unsigned long long)));
  hipError_t e = hipMemset(d, 0, sizeof(unsigned long long));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(rt4_verify_sqrt_kernel, dim3(65536), dim3(256), 0, 0, d);
    e = hipGetLastError();
  }
  unsigned long long v = 0;
  if (e == hipSuccess) e = hipMemcpy(&v, d, sizeof v, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return rt4_set_err(err, errlen, "verify_sqrt failed: %s", hipGetErrorString(e)), RT4_ERR_HIP;
  *mismatches = v;
  return RT4_OK;
}

int rt4_context_evaluated(rt4_context* ctx, uint64_t* n, int32_t reset, char* err, size_t errlen) {
  if (!ctx || !n) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  HIP_TRY(hipSetDevice(ctx->device));
  if (ctx->launched) HIP_TRY(hipEventSynchronize(ctx->done));
  unsigned long long v = 0;
  HIP_TRY(hipMemcpy(&v, ctx->d_eval, sizeof v, hipMemcpyDeviceToHost));
  if (reset) HIP_TRY(hipMemset(ctx->d_eval, 0, sizeof v));
  *n = v;
  return RT4_OK;
}

int rt4_debug_verify_div(rt4_context* ctx, float b, int32_t full, uint64_t* mismatches, char* err, size_t errlen) {
  if (!ctx || !mismatches) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  if (!divisor_candidate(b)) return rt4_set_err(err, errlen, "divisor %g has no finite reciprocal", b), RT4_ERR_ARG;
  HIP_TRY(hipSetDevice(ctx->device));
  std::lock_guard<std::mutex> lock(g_verify_mu);  // d_scratch is shared with verify_constants
  DivSweeps sw;
  std::memset(&sw, 0, sizeof sw);
  sw.d[0] = div_sweep(b, full != 0);
  HIP_TRY(hipMemset(ctx->d_scratch, 0, sizeof(unsigned)));
  hipLaunchKernelGGL(rt4_verify_div_kernel, dim3(8192, 1), dim3(256), 0, 0, sw, ctx->d_scratch);
  HIP_TRY(hipGetLastError());
  unsigned v = 0;
  HIP_TRY(hipMemcpy(&v, ctx->d_scratch, sizeof v, hipMemcpyDeviceToHost));
  *mismatches = v;
  return RT4_OK;
}

int rt4_debug_sky_threshold(rt4_context* ctx, float ang, int32_t full, float* c_min, char* err, size_t errlen) {
  if (!ctx || !c_min) return rt4_set_err(err, errlen, "NULL argument"), RT4_ERR_ARG;
  HIP_TRY(hipSetDevice(ctx->device));
  std::lock_guard<std::mutex> lock(g_verify_mu);
  const bool small = !full && ang <= 1.0f;
  const uint32_t init = 0xFFFFFFFFu, lo = small ? 0x3F000001u : 0u;
  const uint64_t count = small ? (0x3F800000ull - 0x3F000001ull + 1ull) : (1ull << 32);
  HIP_TRY(hipMemcpy(ctx->d_scratch, &init, sizeof init, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(rt4_sky_threshold_kernel, dim3(small ? 512 : 65536), dim3(256), 0, 0, ang, lo, count, ctx->d_scratch);
  HIP_TRY(hipGetLastError());
  uint32_t best = 0;
  HIP_TRY(hipMemcpy(&best, ctx->d_scratch, sizeof best, hipMemcpyDeviceToHost));
  if (best == 0xFFFFFFFFu) {
    *c_min = NAN;
  } else {
    const uint32_t bits = (best & 0x80000000u) ? (best & 0x7FFFFFFFu) : ~best;
    std::memcpy(c_min, &bits, 4);
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
    hipLaunchKernelGGL(variant_for(ctx->shape).find, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, 0, ctx->d_scene, scene_aux(ctx),
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
