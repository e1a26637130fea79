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
static std::atomic<const unsigned long long*> g_salt{nullptr};
const unsigned long long* dropout_salt() { return g_salt.load(std::memory_order_relaxed); }
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

// Dropout salt: a uint64 in device memory mixed into every dropout seed of the following GroupNorm(+Dropout)
// launches (their masks are hashes of seed and element index). A captured HIP graph freezes the per-launch
// seeds; advancing the salt on the device once per replay gives each replayed step fresh, reproducible masks.
// nullptr (the default) = plain seeds, as before.
extern "C" int mvae_set_dropout_salt(const void* salt_dev) {
  mvae::g_salt.store((const unsigned long long*)salt_dev, std::memory_order_relaxed);
  return 0;
}
