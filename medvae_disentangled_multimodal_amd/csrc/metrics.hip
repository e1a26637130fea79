// On-device validation metrics (VAELightningModule.validation_step, src/lightning_module.py:220-300,
// via src/utils/metrics.py:14-73):
//   * SSIM as torchmetrics 1.7.4 structural_similarity_index_measure(preds, target, data_range):
//     11x11 Gaussian window (sigma 1.5), c1 = (0.01 R)^2, c2 = (0.03 R)^2, the map cropped by the
//     5-pixel reflect pad -- so only windows lying fully inside the image are evaluated and the
//     padding never contributes; per-image mean over (C, H-10, W-10).
//   * KL statistics of compute_kl_metrics on [B, z, h, w] (NHWC here): kl = 0.5(mu^2 + e^lv - lv - 1),
//     total, per-"sample" sums over dim 1 (the channel dim of a 4-D latent) -> their mean and
//     unbiased std, and the mean over all elements.
// Reductions are fixed-order (double accumulation): results are reproducible run to run.
#include "common.h"
#include <algorithm>

namespace mvae {

constexpr int SSIM_K = 11, SSIM_PAD = 5;

// one workgroup per image; x, y NHWC [nb][h][w][c]
__global__ void __launch_bounds__(256) ssim_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                   int h, int w, int c, float c1, float c2,
                                                   float* __restrict__ per_image) {
  __shared__ float g[SSIM_K];
  __shared__ double part[256];
  if (threadIdx.x == 0) {  // torchmetrics _gaussian: exp(-(d/sigma)^2/2) normalised, d = -5..5 (fp32)
    float s = 0.f, t[SSIM_K];
    for (int i = 0; i < SSIM_K; ++i) {
      const float d = (float)(i - SSIM_PAD) / 1.5f;
      t[i] = expf(-(d * d) / 2.f);
      s += t[i];
    }
    for (int i = 0; i < SSIM_K; ++i) g[i] = t[i] / s;
  }
  __syncthreads();
  const int b = blockIdx.x;
  const int ho = h - 2 * SSIM_PAD, wo = w - 2 * SSIM_PAD;
  const long long img = (long long)b * h * w * c;
  const long long n = (long long)ho * wo * c;
  double acc = 0.0;
  for (long long e = threadIdx.x; e < n; e += blockDim.x) {
    const int ch = (int)(e % c);
    const long long q = e / c;
    const int j = (int)(q % wo) + SSIM_PAD, i = (int)(q / wo) + SSIM_PAD;
    float mx = 0.f, my = 0.f, sxx = 0.f, syy = 0.f, sxy = 0.f;
    for (int r = 0; r < SSIM_K; ++r) {
      const float* xr = x + img + ((long long)(i - SSIM_PAD + r) * w + (j - SSIM_PAD)) * c + ch;
      const float* yr = y + img + ((long long)(i - SSIM_PAD + r) * w + (j - SSIM_PAD)) * c + ch;
      for (int s = 0; s < SSIM_K; ++s) {
        const float wt = g[r] * g[s];
        const float a = xr[s * c], bb = yr[s * c];
        mx += wt * a;
        my += wt * bb;
        sxx += wt * a * a;
        syy += wt * bb * bb;
        sxy += wt * a * bb;
      }
    }
    const float vx = fmaxf(sxx - mx * mx, 0.f), vy = fmaxf(syy - my * my, 0.f);
    const float cxy = sxy - mx * my;
    const float v = ((2.f * mx * my + c1) * (2.f * cxy + c2)) / ((mx * mx + my * my + c1) * (vx + vy + c2));
    acc += (double)v;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) per_image[b] = (float)(part[0] / (double)n);
}

// per-pixel channel sums of the KL terms (mu/lv rows have stride ld >= zc)
__global__ void kl_pixel_sums_kernel(const float* __restrict__ mu, const float* __restrict__ lv, long long ld,
                                     long long npix, int zc, double* __restrict__ sums) {
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < npix; p += (long long)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int k = 0; k < zc; ++k) {
      const float m = mu[p * ld + k], l = lv[p * ld + k];
      s += 0.5 * ((double)m * m + exp((double)l) - l - 1.0);
    }
    sums[p] = s;
  }
}

// out = {kl_total, kl_mean (over pixel sums), kl_std (unbiased), kl_per_dim_mean}
__global__ void __launch_bounds__(256) kl_stats_kernel(const double* __restrict__ sums, long long npix, int zc,
                                                       float* __restrict__ out) {
  __shared__ double part[256];
  double s = 0.0;
  for (long long p = threadIdx.x; p < npix; p += blockDim.x) s += sums[p];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  const double total = part[0];
  const double mean = total / (double)npix;
  __syncthreads();
  double v = 0.0;
  for (long long p = threadIdx.x; p < npix; p += blockDim.x) {
    const double d = sums[p] - mean;
    v += d * d;
  }
  part[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (float)total;
    out[1] = (float)mean;
    out[2] = npix > 1 ? (float)sqrt(part[0] / (double)(npix - 1)) : NAN;
    out[3] = (float)(total / ((double)npix * zc));
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_ssim(const float* x, const float* y, int nb, int h, int w, int c, float data_range, float* per_image,
              void* stream) {
  if (nb <= 0 || c <= 0 || h < SSIM_K || w < SSIM_K) { set_error("ssim: images must be >= 11x11"); return MVAE_EINVAL; }
  const float c1 = (0.01f * data_range) * (0.01f * data_range), c2 = (0.03f * data_range) * (0.03f * data_range);
  hipLaunchKernelGGL(ssim_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, x, y, h, w, c, c1, c2, per_image);
  return launch_status();
}

size_t mvae_kl_stats_workspace_bytes(long long npix) { return (size_t)std::max<long long>(npix, 1) * sizeof(double); }

int mvae_kl_stats(const float* mu, const float* logvar, long long ld, long long npix, int zc, float* out,
                  void* workspace, size_t workspace_bytes, void* stream) {
  if (npix <= 0 || zc <= 0 || ld < zc) { set_error("kl_stats: bad sizes"); return MVAE_EINVAL; }
  if (workspace_bytes < (size_t)npix * sizeof(double)) { set_error("kl_stats: workspace"); return MVAE_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)std::min<long long>((npix + 255) / 256, 4096);
  hipLaunchKernelGGL(kl_pixel_sums_kernel, dim3(blocks), dim3(256), 0, st, mu, logvar, ld, npix, zc, (double*)workspace);
  hipLaunchKernelGGL(kl_stats_kernel, dim3(1), dim3(256), 0, st, (const double*)workspace, npix, zc, out);
  return launch_status();
}

}  // extern "C"
