// rt4_internal.h — helpers shared by the host-side translation units of librt4.so.
#pragma once

#include <cstdarg>
#include <cstddef>
#include <cstdint>
#include <cstdio>

#include "../../include/rt4.h"

// Version of the trace kernel (the third word of rt4_build_info): bench.py records it and takes
// roofline.traffic only from a rocprofv3 profile of the same version (profiles/). Bump on every
// change to the device code.
#define RT4_KERNEL_VERSION "r06-v54"

// Writes a formatted message into err (if non-NULL); returns 0 so it composes in expressions.
inline int rt4_set_err(char* err, size_t errlen, const char* fmt, ...) {
  if (!err || errlen == 0) return 0;
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(err, errlen, fmt, ap);
  va_end(ap);
  return 0;
}

// Validates uniforms + region + stride shared by the device and host render entry points.
int rt4_check_render_args(const rt4_uniforms* u, const rt4_region* r, long long row_stride_px, char* err,
                          size_t errlen);

// Rows owned by `rank` when bands of `band` rows of a height-row frame are dealt round-robin over
// `world` ranks (rt4_band_plan; shard.py BandPlan.rows), and the largest of them (>= 1).
inline int64_t rt4_band_rows(int64_t height, int64_t world, int64_t band, int64_t rank) {
  const int64_t nb = (height + band - 1) / band;    // bands of the frame
  const int64_t k = rank >= nb ? 0 : (nb - rank + world - 1) / world;  // bands rank, rank + world, ...
  if (k == 0) return 0;
  return k * band - ((nb - 1) % world == rank ? nb * band - height : 0);  // the last band may be short
}
inline int64_t rt4_band_rows_max(int64_t height, int64_t world, int64_t band) {
  int64_t mx = 1;
  for (int64_t r = 0; r < world && r * band < height; r++) {
    const int64_t n = rt4_band_rows(height, world, band, r);
    mx = n > mx ? n : mx;
  }
  return mx;
}
