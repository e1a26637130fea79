// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of the conv-VAE training path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

#define MVAE_WAVE 64

namespace mvae {

// Error reporting across the C ABI: every entry point returns 0 on success, a negative code for
// an argument error and the positive hipError_t value for a launch error.
enum { MVAE_OK = 0, MVAE_EINVAL = -1, MVAE_EWORKSPACE = -2 };
void set_error(const char* fmt, ...);

inline int launch_status() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("HIP launch error: %s", hipGetErrorString(e));
    return (int)e;
  }
  return MVAE_OK;
}

__device__ __forceinline__ float silu_f(float v) { return v / (1.0f + __expf(-v)); }
__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + __expf(-v)); }

// wave64 reductions
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace mvae
