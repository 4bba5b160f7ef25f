// common.h — error reporting shared by the libmhppo.so translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

namespace mhppo {
int set_error(int code, const char *fmt, ...);
}
using mhppo::set_error;

#define CHECK_HIP(expr)                                                                     \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return set_error(MHPPO_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                       __FILE__, __LINE__);                                                 \
  } while (0)
