// Error reporting and version for the grk C ABI (host code).
#include <stdarg.h>
#include <stdio.h>

#include "../../include/grk.h"

namespace grk {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace grk

extern "C" const char* grk_last_error(void) { return grk::g_err; }

extern "C" const char* grk_version(void) { return "grk 0.1 (gfx950)"; }
