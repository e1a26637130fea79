// C-ABI error string plumbing and process-wide settings shared by every entry point.
#include <atomic>
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
static std::atomic<int> g_math{0};
int math_mode() { return g_math.load(std::memory_order_relaxed); }
}  // namespace mvae

extern "C" const char* mvae_last_error(void) { return mvae::g_err; }
extern "C" int mvae_abi_version(void) { return 1; }

// GEMM arithmetic of every subsequent convolution / GEMM launch: 0 = 3xBF16 fp32 emulation
// (default, fp32 training), 1 = bf16 operands with fp32 accumulation (bf16-mixed training).
extern "C" int mvae_set_math_mode(int mode) {
  if (mode != 0 && mode != 1 && mode != 2) {
    mvae::set_error("set_math_mode: mode must be 0 (3xbf16), 1 (bf16) or 2 (exact fp32)");
    return -1;
  }
  mvae::g_math.store(mode, std::memory_order_relaxed);
  return 0;
}
extern "C" int mvae_get_math_mode(void) { return mvae::g_math.load(std::memory_order_relaxed); }
