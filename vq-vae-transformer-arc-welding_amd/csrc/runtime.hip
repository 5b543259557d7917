// Status / error plumbing of the C ABI (thread-local last error, launch checks).
#include <stdarg.h>

#include "common.h"

namespace aw {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return AW_ERR_LAUNCH;
  }
  return AW_OK;
}
}  // namespace aw

extern "C" const char* aw_last_error(void) { return aw::g_err; }
extern "C" int aw_version(void) { return 1; }
