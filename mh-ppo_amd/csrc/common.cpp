// common.cpp — thread-local last-error message and version string.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/mhppo.h"

namespace mhppo {
static thread_local char g_err[512] = "";
int set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace mhppo

extern "C" const char *mhppo_last_error(void) { return mhppo::g_err; }
extern "C" const char *mhppo_version(void) { return "mhppo-mi355x 0.1 gfx950"; }
