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

// descriptor of mvae_conv_weight_transpose_batched (same layout as include/medvae_hip.h)
typedef struct {
  const float* w;
  float* wt;
  int cout, rs, cin, split;
  int block0, pad0;
} mvae_wt_desc;
static_assert(sizeof(mvae_wt_desc) == 40, "mvae_wt_desc layout");

namespace mvae {

// Error reporting across the C ABI: every entry point returns 0 on success, a negative code for
// an argument error and the positive hipError_t value for a launch error.
enum { MVAE_OK = 0, MVAE_EINVAL = -1, MVAE_EWORKSPACE = -2 };
void set_error(const char* fmt, ...);
// device pointer of the process-wide dropout salt (mvae_set_dropout_salt), or nullptr
const unsigned long long* dropout_salt();

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

// 3xBF16 operand pre-split of 4 fp32 values (the GEMM staging's split done once, in HBM):
// {hi0..hi3, lo0..lo3} as bf16, hi = bf16(x) (RNE), lo = bf16(x - hi); 16 B like the fp32 group
__device__ __forceinline__ unsigned pk_bf16x2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) float f2;
  typedef __attribute__((ext_vector_type(2))) __bf16 h2;
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f2{a, b}, h2));
}
__device__ __forceinline__ uint4 split4_bf16(float4 v) {
  const unsigned h01 = pk_bf16x2(v.x, v.y), h23 = pk_bf16x2(v.z, v.w);
  return uint4{h01, h23, pk_bf16x2(v.x - __uint_as_float(h01 << 16), v.y - __uint_as_float(h01 & 0xFFFF0000u)),
               pk_bf16x2(v.z - __uint_as_float(h23 << 16), v.w - __uint_as_float(h23 & 0xFFFF0000u))};
}

// the exact-fp32 arithmetic's pre-split layout (gemm_core.h st_split<0>): the same 16-B group shape as split4_bf16, but
// a BIT split -- the upper 16 bits of x0..x3 in the first 8 B, the lower 16 bits in the last 8 B -- so the GEMM's exact
// MMA step reassembles each fp32 operand bit for bit
__device__ __forceinline__ uint4 split4_bits(float4 v) {
  const unsigned bx = __float_as_uint(v.x), by = __float_as_uint(v.y), bz = __float_as_uint(v.z), bw = __float_as_uint(v.w);
  return uint4{(bx >> 16) | (by & 0xFFFF0000u), (bz >> 16) | (bw & 0xFFFF0000u), (bx & 0xFFFFu) | (by << 16),
               (bz & 0xFFFFu) | (bw << 16)};
}
// pre-split group of format SF: 0 = split4_bf16 (3xBF16 value split; its hi half is the bf16 operand), 1 = split4_bits
template <int SF>
__device__ __forceinline__ uint4 split4_fmt(float4 v) {
  if constexpr (SF == 1) return split4_bits(v);
  else return split4_bf16(v);
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace mvae
