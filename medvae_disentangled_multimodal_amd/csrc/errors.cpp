// C-ABI error string plumbing shared by every entry point.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

namespace mvae {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mvae

extern "C" const char* mvae_last_error(void) { return mvae::g_err; }
extern "C" int mvae_abi_version(void) { return 1; }
