// common.h — error reporting shared by the libmhppo.so translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

namespace mhppo {
int set_error(int code, const char *fmt, ...);

// Makes `dev` the calling thread's current HIP device for the scope of one ABI call and
// restores the caller's device afterwards (a handle is bound to the device it was created
// on, include/mhppo.h; the caller's current device is never changed by a call).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    int cur = -1;
    err = hipGetDevice(&cur);
    if (err == hipSuccess && cur != dev) {
      err = hipSetDevice(dev);
      if (err == hipSuccess) prev = cur;
    }
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};
// per-device tables (workspaces, CU counts) hold this many devices
constexpr int MAX_DEVICES = 16;
}  // namespace mhppo
using mhppo::set_error;

#define GUARD_DEVICE(dev)                                                                  \
  mhppo::DeviceGuard _dg(dev);                                                              \
  if (_dg.err != hipSuccess)                                                                \
    return set_error(MHPPO_EHIP, "hipSetDevice(%d) failed: %s", (int)(dev), hipGetErrorString(_dg.err))

#define CHECK_HIP(expr)                                                                     \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      return set_error(MHPPO_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                       __FILE__, __LINE__);                                                 \
  } while (0)
