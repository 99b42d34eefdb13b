// Host-side error plumbing of the C ABI (include/statecatcher.h).
#include <stdarg.h>
#include <stdio.h>

#include "sc_common.h"

namespace sc {

static thread_local char g_err[512];

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

}  // namespace sc

extern "C" int sc_abi_version(void) { return 14; }
extern "C" const char* sc_last_error(void) { return sc::g_err; }
