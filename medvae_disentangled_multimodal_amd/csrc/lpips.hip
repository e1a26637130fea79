// Perceptual-loss (LPIPS, net="alex") pieces around the implicit-GEMM convolutions
// (LPIPSLoss, src/losses/vae_losses.py:67-94, backed by the third-party `lpips` 0.1.4 package):
//   * input transform  y = ((a*x + b) - shift[c]) / scale[c]   (`inputs*2-1`, then lpips' ScalingLayer)
//   * ReLU forward / backward (AlexNet feature slices)
//   * k x k stride-s max pool (AlexNet 3/2, VGG 2/2) forward (argmax kept as a window index) /
//     deterministic gather backward
//   * per-layer distance  score[b] += mean_p sum_c w[c] (f0/|f0| - f1/|f1|)^2  and its gradient
// All tensors are NHWC fp32; per-pixel channel vectors are contiguous, one wave per pixel.
#include "common.h"
#include <algorithm>

namespace mvae {

static int egrid(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }

__global__ void lpips_scale_kernel(const float* __restrict__ x, float* __restrict__ y, long long n, int c, float a,
                                   float b, const float* __restrict__ shift, const float* __restrict__ inv_scale) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    y[e] = (a * x[e] + b - shift[ch]) * inv_scale[ch];
  }
}

__global__ void lpips_scale_bwd_kernel(const float* __restrict__ dy, float* __restrict__ dx, long long n, int c,
                                       float a, const float* __restrict__ inv_scale) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    dx[e] = dy[e] * a * inv_scale[e % c];
}

__global__ void relu_kernel(const float* __restrict__ x, float* __restrict__ y, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    y[e] = fmaxf(x[e], 0.f);
}

// torch's threshold_backward: grad passes where the (relu) output is > 0
__global__ void relu_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy, float* __restrict__ dx,
                                long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    dx[e] = y[e] > 0.f ? dy[e] : 0.f;
}

// max over the k x k window at (st*oh, st*ow); ties -> first in (r, s) scan order (torch's rule)
__global__ void maxpool_kernel(const float* __restrict__ x, float* __restrict__ y, unsigned char* __restrict__ arg,
                               int nb, int h, int w, int c, int ho, int wo, int k, int st) {
  const long long n = (long long)nb * ho * wo * c;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    long long q = e / c;
    const int ow = (int)(q % wo);
    q /= wo;
    const int oh = (int)(q % ho);
    const int b = (int)(q / ho);
    float m = -INFINITY;
    int best = 0;
    for (int r = 0; r < k; ++r)
      for (int s = 0; s < k; ++s) {
        const float v = x[(((long long)b * h + st * oh + r) * w + st * ow + s) * c + ch];
        if (v > m || v != v) {
          m = v;
          best = r * k + s;
        }
      }
    y[e] = m;
    arg[e] = (unsigned char)best;
  }
}

// dx[ih][iw] = sum of dy over the windows whose argmax is (ih, iw): gather, no atomics
__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, const unsigned char* __restrict__ arg,
                                   float* __restrict__ dx, int nb, int h, int w, int c, int ho, int wo, int k, int st) {
  const long long n = (long long)nb * h * w * c;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    long long q = e / c;
    const int iw = (int)(q % w);
    q /= w;
    const int ih = (int)(q % h);
    const int b = (int)(q / h);
    float s = 0.f;
    for (int oh = std::max(0, (ih - k + st) / st); oh <= std::min(ho - 1, ih / st); ++oh) {
      const int r = ih - st * oh;
      if (r < 0 || r >= k) continue;
      for (int ow = std::max(0, (iw - k + st) / st); ow <= std::min(wo - 1, iw / st); ++ow) {
        const int t = iw - st * ow;
        if (t < 0 || t >= k) continue;
        const long long o = (((long long)b * ho + oh) * wo + ow) * c + ch;
        if (arg[o] == r * k + t) s += dy[o];
      }
    }
    dx[e] = s;
  }
}

constexpr int LP_MAXC = 512;      // channels per pixel held in registers: <= 8 per lane
constexpr float LP_EPS = 1e-10f;  // lpips normalize_tensor eps

// One workgroup per image, one wave per pixel (strided): d_p = sum_c w_c (f0_c/n0 - f1_c/n1)^2 with
// n = sqrt(sum_c f^2) + eps; score[b] = beta*score[b] + (1/P) sum_p d_p (fixed-order reduction).
__global__ void __launch_bounds__(256) lpips_dist_kernel(const float* __restrict__ f0, const float* __restrict__ f1,
                                                         const float* __restrict__ wl, float* __restrict__ score,
                                                         int npix, int c, float beta) {
  __shared__ float part[4];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float acc = 0.f;
  for (int p = wv; p < npix; p += 4) {
    const float* a0 = f0 + ((long long)b * npix + p) * c;
    const float* a1 = f1 + ((long long)b * npix + p) * c;
    float v0[LP_MAXC / 64], v1[LP_MAXC / 64];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < LP_MAXC / 64; ++i) {
      const int ch = lane + 64 * i;
      v0[i] = ch < c ? a0[ch] : 0.f;
      v1[i] = ch < c ? a1[ch] : 0.f;
      s0 += v0[i] * v0[i];
      s1 += v1[i] * v1[i];
    }
    const float n0 = sqrtf(wave_sum_f(s0)) + LP_EPS, n1 = sqrtf(wave_sum_f(s1)) + LP_EPS;
    float d = 0.f;
#pragma unroll
    for (int i = 0; i < LP_MAXC / 64; ++i) {
      const int ch = lane + 64 * i;
      const float u = v0[i] / n0 - v1[i] / n1;
      if (ch < c) d += wl[ch] * u * u;
    }
    acc += wave_sum_f(d);
  }
  if (lane == 0) part[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float v = (part[0] + part[1] + part[2] + part[3]) / (float)npix;
    score[b] = (beta != 0.f ? beta * score[b] : 0.f) + v;
  }
}

// Gradient of score[b] (upstream gscore[b]) w.r.t. f0 (and f1 when df1 != nullptr):
//   a_c = 2 w_c (u0_c - u1_c) * g / P,  df0_j = a_j/n0 - (sum_c a_c f0_c) f0_j / (n0^2 (n0 - eps))
// and symmetrically with -a for f1. A zero feature vector gets a zero gradient (torch: NaN).
__global__ void __launch_bounds__(256) lpips_dist_bwd_kernel(const float* __restrict__ f0,
                                                             const float* __restrict__ f1,
                                                             const float* __restrict__ wl,
                                                             const float* __restrict__ gscore, float* __restrict__ df0,
                                                             float* __restrict__ df1, int nb, int npix, int c) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  for (long long pp = blockIdx.x * 4LL + (threadIdx.x >> 6); pp < (long long)nb * npix; pp += nw) {
    const int b = (int)(pp / npix);
    const float g = gscore[b] / (float)npix;
    const float* a0 = f0 + pp * c;
    const float* a1 = f1 + pp * c;
    float v0[LP_MAXC / 64], v1[LP_MAXC / 64], av[LP_MAXC / 64];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < LP_MAXC / 64; ++i) {
      const int ch = lane + 64 * i;
      v0[i] = ch < c ? a0[ch] : 0.f;
      v1[i] = ch < c ? a1[ch] : 0.f;
      s0 += v0[i] * v0[i];
      s1 += v1[i] * v1[i];
    }
    const float r0 = sqrtf(wave_sum_f(s0)), r1 = sqrtf(wave_sum_f(s1));
    const float n0 = r0 + LP_EPS, n1 = r1 + LP_EPS;
    float t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int i = 0; i < LP_MAXC / 64; ++i) {
      const int ch = lane + 64 * i;
      av[i] = ch < c ? 2.f * wl[ch] * (v0[i] / n0 - v1[i] / n1) * g : 0.f;
      t0 += av[i] * v0[i];
      t1 += av[i] * v1[i];
    }
    t0 = wave_sum_f(t0);
    t1 = wave_sum_f(t1);
    const float k0 = r0 > 0.f ? t0 / (n0 * n0 * r0) : 0.f;
    const float k1 = r1 > 0.f ? t1 / (n1 * n1 * r1) : 0.f;
#pragma unroll
    for (int i = 0; i < LP_MAXC / 64; ++i) {
      const int ch = lane + 64 * i;
      if (ch >= c) continue;
      df0[pp * c + ch] = r0 > 0.f ? av[i] / n0 - k0 * v0[i] : 0.f;
      if (df1) df1[pp * c + ch] = r1 > 0.f ? -av[i] / n1 + k1 * v1[i] : 0.f;
    }
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_lpips_scale(const float* x, float* y, long long n, int c, float a, float b, const float* shift,
                     const float* inv_scale, void* stream) {
  if (n < 0 || c <= 0) { set_error("lpips_scale: bad sizes"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(lpips_scale_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, x, y, n, c, a, b, shift,
                     inv_scale);
  return launch_status();
}

int mvae_lpips_scale_bwd(const float* dy, float* dx, long long n, int c, float a, const float* inv_scale,
                         void* stream) {
  if (n < 0 || c <= 0) { set_error("lpips_scale_bwd: bad sizes"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(lpips_scale_bwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, dy, dx, n, c, a,
                     inv_scale);
  return launch_status();
}

int mvae_relu_fwd(const float* x, float* y, long long n, void* stream) {
  if (n < 0) { set_error("relu: bad size"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(relu_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, x, y, n);
  return launch_status();
}

int mvae_relu_bwd(const float* y, const float* dy, float* dx, long long n, void* stream) {
  if (n < 0) { set_error("relu_bwd: bad size"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, y, dy, dx, n);
  return launch_status();
}

int mvae_maxpool_fwd(const float* x, float* y, unsigned char* argmax, int nb, int h, int w, int c, int k, int stride,
                     void* stream) {
  if (nb <= 0 || k < 1 || k > 15 || stride < 1 || h < k || w < k || c <= 0) {
    set_error("maxpool: bad sizes");
    return MVAE_EINVAL;
  }
  const int ho = (h - k) / stride + 1, wo = (w - k) / stride + 1;
  hipLaunchKernelGGL(maxpool_kernel, dim3(egrid((long long)nb * ho * wo * c)), dim3(256), 0, (hipStream_t)stream, x, y,
                     argmax, nb, h, w, c, ho, wo, k, stride);
  return launch_status();
}

int mvae_maxpool_bwd(const float* dy, const unsigned char* argmax, float* dx, int nb, int h, int w, int c, int k,
                     int stride, void* stream) {
  if (nb <= 0 || k < 1 || k > 15 || stride < 1 || h < k || w < k || c <= 0) {
    set_error("maxpool_bwd: bad sizes");
    return MVAE_EINVAL;
  }
  const int ho = (h - k) / stride + 1, wo = (w - k) / stride + 1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(egrid((long long)nb * h * w * c)), dim3(256), 0, (hipStream_t)stream, dy,
                     argmax, dx, nb, h, w, c, ho, wo, k, stride);
  return launch_status();
}

int mvae_lpips_dist(const float* f0, const float* f1, const float* w, float* score, int nb, int npix, int c,
                    float beta, void* stream) {
  if (nb <= 0 || npix <= 0 || c <= 0 || c > LP_MAXC) { set_error("lpips_dist: bad sizes (c <= 512)"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(lpips_dist_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, f0, f1, w, score, npix, c, beta);
  return launch_status();
}

int mvae_lpips_dist_bwd(const float* f0, const float* f1, const float* w, const float* gscore, float* df0, float* df1,
                        int nb, int npix, int c, void* stream) {
  if (nb <= 0 || npix <= 0 || c <= 0 || c > LP_MAXC) { set_error("lpips_dist_bwd: bad sizes"); return MVAE_EINVAL; }
  const long long waves = (long long)nb * npix;
  const int blocks = (int)std::max<long long>(1, std::min<long long>((waves + 3) / 4, 16384));
  hipLaunchKernelGGL(lpips_dist_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, f0, f1, w, gscore, df0,
                     df1, nb, npix, c);
  return launch_status();
}

}  // extern "C"
