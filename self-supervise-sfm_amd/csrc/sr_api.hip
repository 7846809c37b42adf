// Host-side ABI plumbing: error reporting and version.
#include <cstdarg>
#include <cstdio>

#include "sr_common.h"

namespace {
thread_local char g_err[512] = "";
}

namespace sr {

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return SR_ELAUNCH;
  }
  return SR_OK;
}

}  // namespace sr

extern "C" const char* sr_last_error(void) { return g_err; }
extern "C" int sr_version(void) { return (0 << 16) | 2; }
