// Host-side pieces of the C ABI shared by every kernel file: version and error reporting.
#include <stdarg.h>
#include <stdio.h>
#include "sqr_common.h"

namespace sqr {
static thread_local char g_err[512] = "no error";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace sqr

extern "C" int sqr_version(void) { return 1; }
extern "C" const char* sqr_last_error_string(void) { return sqr::g_err; }
