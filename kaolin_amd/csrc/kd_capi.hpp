// kd_capi.hpp -- error state of the C ABI (thread-local message + status codes).
#pragma once

#include <stdarg.h>
#include <stdio.h>

#include "../../include/kaolin_dibr.h"

namespace kd {

char *error_buffer();  // thread-local, 512 bytes

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
