// kd_capi.hpp -- error state of the C ABI (thread-local message + status codes).
#pragma once

#include <stdarg.h>
#include <stdio.h>

#include <hip/hip_runtime.h>

#include "../../include/kaolin_dibr.h"

namespace kd {

char *error_buffer();  // thread-local, 512 bytes

enum KernelId {
  K_BIN_COUNT = 0,
  K_BIN_SCAN,
  K_BIN_SCATTER,
  K_RASTER_FWD,
  K_SOFT_FWD,
  K_RASTER_BWD_TILE,
  K_SOFT_BWD_TILE,
  K_RASTER_BWD_ATOMIC,
  K_SOFT_BWD_ATOMIC,
  K_ZERO,
  K_SOFT_PAIRS,
  K_SOFT_MATH,
  K_SOFT_REDUCE,
  K_SOFT_BWD_PAIRS,
  K_PREPARE_FWD,
  K_PREPARE_BWD,
  K_TILE_ORDER,
  K_IOU_FWD,
  K_IOU_BWD,
  K_TEX_FWD,
  K_TEX_BWD,
  K_RAST_INTERP,
  K_DT_BIN,
  K_DT_FWD,
  K_DIBR_BWD,
  K_DIBR_FWD,
  K_SOFT_OVF_FWD,
  K_SOFT_OVF_BWD,
  K_DT_BWD,
  K_NUM_KERNELS
};

// Records a HIP event pair around the launches in its scope when profiling is enabled.
struct ProfScope {
  ProfScope(int id, hipStream_t s);
  ~ProfScope();
  int id;
  hipStream_t stream;
  hipEvent_t start, stop;
  bool on;
};

inline int set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(error_buffer(), 512, fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace kd

#define KD_CHECK_ARG(cond, msg)                                                \
  do {                                                                         \
    if (!(cond)) return kd::set_error(KD_ERR_INVALID_ARGUMENT, "%s", (msg));   \
  } while (0)
