// Weight gradient of a 3x3 / stride-1 / pad-1 convolution with very few output channels (Decoder.conv_out:
// cout = out_ch = 3, src/models/encoder_decoder.py:418-419, :449-451).
//
// As an implicit GEMM this is M = cout (3) x N = 9*cin x K = pixels: every im2col element of x is used for
// only cout MACs, so the GEMM form streams the 9x tap-redundant im2col (9 GB at 64x64x256, bs 256) through
// L2 for 3 useful rows. Here each input pixel of x is read ONCE and scattered into its 9 tap
// contributions: dW[co][r][s][c] += dy[p - (r-1, s-1)][co] * x[p][c], with the image's dy (cout floats per
// pixel) staged once in LDS and re-read per tap. HBM-bound on x (4 B per element) + the small partials.
//
// Deterministic: block (image n, 64-channel chunk) accumulates in registers over a fixed pixel walk, a
// fixed-order LDS reduction over the block's 16 pixel lanes writes one partial per (n, chunk); a second
// kernel sums the nb partials of every output element in order (and the bias gradient = sum of dy).
#include "common.h"

namespace mvae {

constexpr int SC_MAXC = 4;  // cout <= 4
constexpr int SC_PIX = 16;  // pixel lanes per block (x 16 channel groups of 4 = 256 threads)

// part layout: [nb][cin/64 chunks][9 taps][SC_MAXC][64] (+ bias partials [nb][SC_MAXC])
// LDS: the image's dy as [hw][4] (one ds_read_b128 per tap) when it fits (DY_LDS), else dy from global.
__device__ __forceinline__ float4 xval(const float4 v, bool xsplit) {
  if (!xsplit) return v;
  // split4_bf16 group {hi0..hi3, lo0..lo3}: x = hi + lo
  const unsigned u0 = __float_as_uint(v.x), u1 = __float_as_uint(v.y), u2 = __float_as_uint(v.z),
                 u3 = __float_as_uint(v.w);
  return float4{__uint_as_float(u0 << 16) + __uint_as_float(u2 << 16),
                __uint_as_float(u0 & 0xFFFF0000u) + __uint_as_float(u2 & 0xFFFF0000u),
                __uint_as_float(u1 << 16) + __uint_as_float(u3 << 16),
                __uint_as_float(u1 & 0xFFFF0000u) + __uint_as_float(u3 & 0xFFFF0000u)};
}

template <bool XSPLIT, bool DY_LDS>
__global__ void __launch_bounds__(256) wgrad_small_cout_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                               float* __restrict__ part, float* __restrict__ bpart,
                                                               int h, int w, int cin, int cout) {
  extern __shared__ float4 dys[];  // [hw] (DY_LDS), then the reduction scratch
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int cg = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c0 = chunk * 64 + cg * 4;
  const bool cact = c0 < cin;
  const int hw = h * w;
  const float* dyn = dy + (long long)n * hw * cout;
  const float* xn = x + (long long)n * hw * cin;
  if constexpr (DY_LDS) {
    for (int p = threadIdx.x; p < hw; p += 256) {
      float4 v{0.f, 0.f, 0.f, 0.f};
      v.x = dyn[(long long)p * cout];
      if (cout > 1) v.y = dyn[(long long)p * cout + 1];
      if (cout > 2) v.z = dyn[(long long)p * cout + 2];
      if (cout > 3) v.w = dyn[(long long)p * cout + 3];
      dys[p] = v;
    }
    __syncthreads();
  }
  auto dyat = [&](int q) -> float4 {
    if constexpr (DY_LDS) {
      return dys[q];
    } else {
      float4 v{0.f, 0.f, 0.f, 0.f};
      v.x = dyn[(long long)q * cout];
      if (cout > 1) v.y = dyn[(long long)q * cout + 1];
      if (cout > 2) v.z = dyn[(long long)q * cout + 2];
      if (cout > 3) v.w = dyn[(long long)q * cout + 3];
      return v;
    }
  };
  float acc[9][SC_MAXC][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 0; o < SC_MAXC; ++o)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[t][o][e] = 0.f;
  float4 bacc{0.f, 0.f, 0.f, 0.f};
  const float4 zero{0.f, 0.f, 0.f, 0.f};
  int p = pl;
  float4 xnext = (cact && p < hw) ? *(const float4*)(xn + (long long)p * cin + c0) : zero;
  for (; p < hw; p += SC_PIX) {
    const float4 xv = xval(xnext, XSPLIT);
    const int pn = p + SC_PIX;  // prefetch the next pixel's x while this one is scattered
    xnext = (cact && pn < hw) ? *(const float4*)(xn + (long long)pn * cin + c0) : zero;
    const int ph = p / w, pw = p - ph * w;
    // x[p] feeds output pixel q = p - (r-1, s-1) through tap (r, s)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int qh = ph + 1 - r;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int qw = pw + 1 - s;
        const bool ok = (unsigned)qh < (unsigned)h && (unsigned)qw < (unsigned)w;
        const float4 d = ok ? dyat(qh * w + qw) : zero;
        const float dv[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int o = 0; o < SC_MAXC; ++o) {
          acc[r * 3 + s][o][0] += dv[o] * xv.x;
          acc[r * 3 + s][o][1] += dv[o] * xv.y;
          acc[r * 3 + s][o][2] += dv[o] * xv.z;
          acc[r * 3 + s][o][3] += dv[o] * xv.w;
        }
      }
    }
    if (chunk == 0 && cg == 0) {
      const float4 d = dyat(p);
      bacc.x += d.x; bacc.y += d.y; bacc.z += d.z; bacc.w += d.w;
    }
  }
  // fixed-order reduction over the 16 pixel lanes, one tap at a time through LDS
  float* red = (float*)(dys + (DY_LDS ? hw : 0));  // [SC_PIX][SC_MAXC * 64]
  __syncthreads();
  float* out = part + (((long long)n * gridDim.x + chunk) * 9) * SC_MAXC * 64;
  for (int t = 0; t < 9; ++t) {
#pragma unroll
    for (int o = 0; o < SC_MAXC; ++o)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[pl * SC_MAXC * 64 + o * 64 + cg * 4 + e] = acc[t][o][e];
    __syncthreads();
    {
      const int i = threadIdx.x;  // 256 = SC_MAXC * 64 outputs of this tap
      float sum = 0.f;
      for (int q = 0; q < SC_PIX; ++q) sum += red[q * SC_MAXC * 64 + i];
      out[t * SC_MAXC * 64 + i] = sum;
    }
    __syncthreads();
  }
  if (chunk == 0) {
    if (cg == 0) {
      red[pl * 4 + 0] = bacc.x; red[pl * 4 + 1] = bacc.y; red[pl * 4 + 2] = bacc.z; red[pl * 4 + 3] = bacc.w;
    }
    __syncthreads();
    if (threadIdx.x < SC_MAXC) {
      float sum = 0.f;
      for (int q = 0; q < SC_PIX; ++q) sum += red[q * 4 + threadIdx.x];
      bpart[(long long)n * SC_MAXC + threadIdx.x] = sum;
    }
  }
}

// dw[co][r][s][c] = beta*dw + sum_n part[n][c/64][tap][co][c%64]; dbias[co] = beta*dbias + sum_n bpart[n][co].
// One wave per output element (the last cout waves: the bias), lanes over the images, then the fixed wave
// tree: deterministic, and the nb loads of an element are in flight together.
__global__ void __launch_bounds__(256) wgrad_small_cout_final_kernel(const float* __restrict__ part,
                                                                     const float* __restrict__ bpart, float* dw,
                                                                     float* dbias, float beta, int nb, int cin,
                                                                     int cout, int chunks) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;  // over cout * 9 * cin (+ cout)
  const int total = cout * 9 * cin;
  if (i < total) {
    const int c = i % cin, t = (i / cin) % 9, o = i / (9 * cin);
    const int ch = c >> 6, cl = c & 63;
    float s = 0.f;
    for (int n = lane; n < nb; n += 64) s += part[((((long long)n * chunks + ch) * 9 + t) * SC_MAXC + o) * 64 + cl];
    s = wave_sum_f(s);
    if (lane == 0) dw[i] = beta == 0.f ? s : beta * dw[i] + s;
  } else if (dbias != nullptr && i < total + cout) {
    const int o = i - total;
    float s = 0.f;
    for (int n = lane; n < nb; n += 64) s += bpart[(long long)n * SC_MAXC + o];
    s = wave_sum_f(s);
    if (lane == 0) dbias[o] = beta == 0.f ? s : beta * dbias[o] + s;
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_conv2d_wgrad_small_cout_workspace_bytes(int nb, int cin) {
  const int chunks = (cin + 63) / 64;
  return (size_t)nb * chunks * 9 * SC_MAXC * 64 * sizeof(float) + (size_t)nb * SC_MAXC * sizeof(float) + 512;
}

int mvae_conv2d_wgrad_small_cout_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb,
                                      int h, int w, int cin, int cout, int x_split, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  if (nb <= 0 || h <= 0 || w <= 0 || cin <= 0 || (cin & 3) || cout <= 0 || cout > SC_MAXC) {
    set_error("wgrad_small_cout: needs cin %% 4 == 0 and 1 <= cout <= %d", SC_MAXC);
    return MVAE_EINVAL;
  }
  if (((uintptr_t)x & 15) != 0) {
    set_error("wgrad_small_cout: x must be 16-B aligned");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_conv2d_wgrad_small_cout_workspace_bytes(nb, cin)) {
    set_error("wgrad_small_cout: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const int chunks = (cin + 63) / 64;
  float* part = (float*)workspace;
  float* bpart = (float*)(((uintptr_t)(part + (size_t)nb * chunks * 9 * SC_MAXC * 64) + 255) & ~(uintptr_t)255);
  const size_t red_bytes = (size_t)SC_PIX * SC_MAXC * 64 * sizeof(float);
  const bool dy_lds = (size_t)h * w * 16 + red_bytes <= 96 * 1024;  // whole image's dy in LDS (64x64: 64 KB)
  const size_t lds = (dy_lds ? (size_t)h * w * 16 : 0) + red_bytes;
  const dim3 grid(chunks, nb);
  static bool attr_set = false;  // dynamic LDS above 64 KB must be allowed per kernel
  if (!attr_set) {
    const int mx = 160 * 1024;
    (void)hipFuncSetAttribute((const void*)wgrad_small_cout_kernel<true, true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void*)wgrad_small_cout_kernel<true, false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void*)wgrad_small_cout_kernel<false, true>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    (void)hipFuncSetAttribute((const void*)wgrad_small_cout_kernel<false, false>, hipFuncAttributeMaxDynamicSharedMemorySize, mx);
    attr_set = true;
  }
  if (x_split && dy_lds)
    hipLaunchKernelGGL((wgrad_small_cout_kernel<true, true>), grid, dim3(256), lds, st, dy, x, part, bpart, h, w, cin, cout);
  else if (x_split)
    hipLaunchKernelGGL((wgrad_small_cout_kernel<true, false>), grid, dim3(256), lds, st, dy, x, part, bpart, h, w, cin, cout);
  else if (dy_lds)
    hipLaunchKernelGGL((wgrad_small_cout_kernel<false, true>), grid, dim3(256), lds, st, dy, x, part, bpart, h, w, cin, cout);
  else
    hipLaunchKernelGGL((wgrad_small_cout_kernel<false, false>), grid, dim3(256), lds, st, dy, x, part, bpart, h, w, cin, cout);
  hipLaunchKernelGGL(wgrad_small_cout_final_kernel, dim3(cdiv((long long)cout * 9 * cin + cout, 4)), dim3(256), 0, st,
                     (const float*)part, (const float*)bpart, dw, dbias, beta, nb, cin, cout, chunks);
  return launch_status();
}

}  // extern "C"
