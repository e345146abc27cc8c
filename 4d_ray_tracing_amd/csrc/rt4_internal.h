// rt4_internal.h — helpers shared by the host-side translation units of librt4.so.
#pragma once

#include <cstdarg>
#include <cstddef>
#include <cstdio>

#include "../../include/rt4.h"

// Version of the trace kernel (the third word of rt4_build_info): bench.py records it and takes
// roofline.traffic only from a rocprofv3 profile of the same version (profiles/). Bump on every
// change to the device code.
#define RT4_KERNEL_VERSION "r02-v32"

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
