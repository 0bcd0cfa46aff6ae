// Error reporting for the C ABI (host only).
#include <stdarg.h>
#include <stdio.h>

#include "../../include/hvit.h"

static thread_local char g_err[1024] = "";

void hvit_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* hvit_last_error(void) { return g_err; }

extern "C" const char* hvit_version(void) { return "hvit 0.1 gfx950"; }
