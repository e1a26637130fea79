// ConditionalVAE concat conditioning (src/models/conditional_vae.py:65-69 condition_proj, :107-127
// create_condition_map, :131-136 concat) as two launches per direction instead of torch's Linear (a BLAS GEMM),
// ReLU, bilinear interpolate and cat:
//   pre[b,o]  = bias[o] + sum_j cond[b,j] * W[o,j]           nn.Linear(condition_dim -> C*64)
//   m[b,o]    = relu(pre[b,o])                                viewed as [C][8][8] (nn.Unflatten)
//   cmap      = bilinear(m, (H, W)), align_corners=False      F.interpolate
//   xcond     = [x | cmap] written NHWC [B][H][W][2C]         torch.cat(dim=1)
// Index path bit-exact: the projection accumulates cond[b,j]*W[o,j] with fmaf from 0 in j order and adds the bias
// last, so for a one-hot condition (0/1 entries) pre = fl(W[o,idx] + bias[o]) exactly -- torch's addmm result.
// The interpolation restates torch's CPU bilinear kernel for this case bit for bit (measured against torch 2.10,
// tests/test_condition_cpu.py): src = fma(scale, dst + 0.5, -0.5) clamped at 0, i0 = floor, lambdas as
// in UpSample.h (compute_source_index_and_lambda), corner weights w00 = hl0*wl0 ..., and the corner sum
// fma(w11, v11, fma(w10, v10, fma(w00, v00, w01 * v01))). (Torch takes that path whenever H + W <= 128 or one
// thread runs; larger maps in multi-threaded torch go through its generic kernel, which rounds differently.)
// Backward: the adjoint of the interpolation per (sample, channel) in one workgroup (separable, fixed order),
// the ReLU mask, then dW[o,j] += sum_b dpre[b,o] cond[b,j] and dbias[o] += sum_b dpre[b,o] in batch order.
#include "common.h"

namespace mvae {

struct Lerp {
  int i0, i1;
  float l0, l1;
};

// UpSample.h: area_pixel_compute_scale / area_pixel_compute_source_index / compute_source_index_and_lambda
__device__ __forceinline__ Lerp lerp_of(int dst, int in, int out) {
  Lerp r;
  if (in == out) {
    r.i0 = r.i1 = dst;
    r.l0 = 1.f;
    r.l1 = 0.f;
    return r;
  }
  const float scale = (float)in / (float)out;
  float src = __builtin_fmaf(scale, (float)dst + 0.5f, -0.5f);
  src = src < 0.f ? 0.f : src;
  r.i0 = min((int)floorf(src), in - 1);
  r.l1 = fminf(fmaxf(src - (float)r.i0, 0.f), 1.f);
  r.i1 = r.i0 + (r.i0 < in - 1 ? 1 : 0);
  r.l0 = 1.f - r.l1;
  return r;
}

// one thread per projection output (b, o); K = condition_dim
__global__ void __launch_bounds__(256) cond_proj_kernel(const float* __restrict__ cond, const float* __restrict__ w,
                                                        const float* __restrict__ bias, float* __restrict__ m, int B,
                                                        int O, int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * O) return;
  const int b = t / O, o = t - b * O;
  float acc = 0.f;
  for (int j = 0; j < K; ++j) acc = __builtin_fmaf(cond[b * K + j], w[o * K + j], acc);
  const float pre = acc + bias[o];
  m[t] = pre > 0.f ? pre : 0.f;  // relu (torch: NaN propagates; a NaN pre stays NaN below)
  if (pre != pre) m[t] = pre;
}

// one thread per output pixel (b, h, w): copies x's C channels and writes the C interpolated map channels
__global__ void __launch_bounds__(256) cond_concat_kernel(const float* __restrict__ x, const float* __restrict__ m,
                                                          float* __restrict__ xc, int B, int C, int H, int W) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)B * H * W) return;
  const int b = (int)(t / (H * W));
  const int p = (int)(t - (long long)b * H * W);
  const int h = p / W, w = p - (p / W) * W;
  const Lerp lh = lerp_of(h, 8, H), lw = lerp_of(w, 8, W);
  const float w00 = lh.l0 * lw.l0, w01 = lh.l0 * lw.l1, w10 = lh.l1 * lw.l0, w11 = lh.l1 * lw.l1;
  float* out = xc + t * (2 * C);
  const float* xi = x + t * C;
  for (int c = 0; c < C; ++c) out[c] = xi[c];
  for (int c = 0; c < C; ++c) {
    const float* mc = m + ((long long)b * C + c) * 64;
    const float v00 = mc[lh.i0 * 8 + lw.i0], v01 = mc[lh.i0 * 8 + lw.i1];
    const float v10 = mc[lh.i1 * 8 + lw.i0], v11 = mc[lh.i1 * 8 + lw.i1];
    out[C + c] = __builtin_fmaf(w11, v11, __builtin_fmaf(w10, v10, __builtin_fmaf(w00, v00, w01 * v01)));
  }
}

// adjoint of the interpolation for one (b, c) per workgroup, times the relu mask -> dpre[b][c*64 + i*8 + j]
// dm[i][j] = sum_h wh(h, i) * sum_w ww(w, j) * dcmap[h][w]   (separable, fixed order)
constexpr int COND_BWD_THREADS = 256;
constexpr int COND_MAX_HW = 256;  // H, W <= 256 (the LDS row buffer)
__global__ void __launch_bounds__(COND_BWD_THREADS) cond_map_bwd_kernel(const float* __restrict__ dxc,
                                                                        const float* __restrict__ m,
                                                                        float* __restrict__ dpre, int C, int H, int W) {
  __shared__ float rows[COND_MAX_HW][8];  // t[h][j] = sum_w ww(w, j) dcmap[h][w]
  const int b = blockIdx.x / C, c = blockIdx.x - (blockIdx.x / C) * C;
  for (int e = threadIdx.x; e < H * 8; e += blockDim.x) {
    const int h = e >> 3, j = e & 7;
    float s = 0.f;
    const float* row = dxc + (((long long)b * H + h) * W) * (2 * C) + C + c;
    for (int w = 0; w < W; ++w) {
      const Lerp lw = lerp_of(w, 8, W);
      const float g = row[(long long)w * 2 * C];
      if (lw.i0 == j) s += lw.l0 * g;
      if (lw.i1 == j) s += lw.l1 * g;
    }
    rows[h][j] = s;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int i = threadIdx.x >> 3, j = threadIdx.x & 7;
    float s = 0.f;
    for (int h = 0; h < H; ++h) {
      const Lerp lh = lerp_of(h, 8, H);
      if (lh.i0 == i) s += lh.l0 * rows[h][j];
      if (lh.i1 == i) s += lh.l1 * rows[h][j];
    }
    const long long o = ((long long)b * C + c) * 64 + threadIdx.x;
    dpre[o] = m[o] > 0.f ? s : 0.f;
  }
}

// dW[o][j] += sum_b dpre[b][o] * cond[b][j] ; dbias[o] += sum_b dpre[b][o]  (batch order, one thread per output)
__global__ void __launch_bounds__(256) cond_param_grad_kernel(const float* __restrict__ dpre,
                                                              const float* __restrict__ cond, float* __restrict__ dw,
                                                              float* __restrict__ dbias, int B, int O, int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * (K + 1)) return;
  const int o = t / (K + 1), j = t - o * (K + 1);
  float s = 0.f;
  if (j < K)
    for (int b = 0; b < B; ++b) s += dpre[(long long)b * O + o] * cond[b * K + j];
  else
    for (int b = 0; b < B; ++b) s += dpre[(long long)b * O + o];
  if (j < K) {
    if (dw) dw[o * K + j] += s;
  } else if (dbias) {
    dbias[o] += s;
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

// x: [B][H][W][C] (NHWC), cond: [B][K], w: [C*64][K], bias: [C*64] -> m: [B][C*64] (relu(pre), saved for the
// backward), xcond: [B][H][W][2C]
int mvae_condition_concat_fwd(const float* x, const float* cond, const float* w, const float* bias, float* m,
                              float* xcond, int B, int C, int H, int W, int K, hipStream_t st) {
  if (!x || !cond || !w || !bias || !m || !xcond || B <= 0 || C <= 0 || H <= 0 || W <= 0 || K <= 0 ||
      H > COND_MAX_HW || W > COND_MAX_HW) {
    set_error("mvae_condition_concat_fwd: bad arguments (B=%d C=%d H=%d W=%d K=%d)", B, C, H, W, K);
    return MVAE_EINVAL;
  }
  const int O = C * 64;
  hipLaunchKernelGGL(cond_proj_kernel, dim3(cdiv((long long)B * O, 256)), dim3(256), 0, st, cond, w, bias, m, B, O,
                     K);
  hipLaunchKernelGGL(cond_concat_kernel, dim3(cdiv((long long)B * H * W, 256)), dim3(256), 0, st, x, m, xcond, B, C,
                     H, W);
  return launch_status();
}

// dxcond: [B][H][W][2C] gradient of the concatenated input; m from the forward; accumulates dw [C*64][K] and
// dbias [C*64] (either may be null); dpre: workspace of B*C*64 floats
int mvae_condition_concat_bwd(const float* dxcond, const float* cond, const float* m, float* dw, float* dbias,
                              float* dpre, int B, int C, int H, int W, int K, hipStream_t st) {
  if (!dxcond || !cond || !m || !dpre || B <= 0 || C <= 0 || H <= 0 || W <= 0 || K <= 0 || H > COND_MAX_HW ||
      W > COND_MAX_HW) {
    set_error("mvae_condition_concat_bwd: bad arguments (B=%d C=%d H=%d W=%d K=%d)", B, C, H, W, K);
    return MVAE_EINVAL;
  }
  const int O = C * 64;
  hipLaunchKernelGGL(cond_map_bwd_kernel, dim3(B * C), dim3(COND_BWD_THREADS), 0, st, dxcond, m, dpre, C, H, W);
  hipLaunchKernelGGL(cond_param_grad_kernel, dim3(cdiv((long long)O * (K + 1), 256)), dim3(256), 0, st, dpre, cond,
                     dw, dbias, B, O, K);
  return launch_status();
}

}  // extern "C"
