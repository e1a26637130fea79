// Adversarial branch (row (f)2): the NLayerDiscriminator's non-GEMM layers (src/models/discriminator.py:
// 11-82) -- BatchNorm2d (training-mode batch statistics with running-stat update, or eval mode)
// fused with LeakyReLU(0.2), a standalone LeakyReLU -- over NHWC activations. The 4x4 convolutions
// are the implicit-GEMM kernel. Per-channel statistics are column reductions over N*H*W rows:
// fixed-order two-stage (fp64 partials), bitwise reproducible.
#include "common.h"
#include <algorithm>

namespace mvae {

constexpr int BN_COLS = 64;  // channels per workgroup (one per lane of a wave row)

static int bn_chunks(long long rows, int c) {
  const long long colblocks = (c + BN_COLS - 1) / BN_COLS;
  long long ch = std::max<long long>(1, 2048 / colblocks);
  return (int)std::min<long long>(ch, std::max<long long>(1, rows / 64));
}

// part[k][chunk][c]: k=0 sum x, k=1 sum x^2 (fwd) | k=0 sum g, k=1 sum g*xhat (bwd)
// mode 0: x statistics; mode 1: g = dy * leaky'(y) and g * xhat with xhat = (x - mean) * rstd
__global__ void __launch_bounds__(256) bn_partial_kernel(int mode, const float* __restrict__ x,
                                                         const float* __restrict__ y, const float* __restrict__ dy,
                                                         const float* __restrict__ mean, const float* __restrict__ rstd,
                                                         float slope, long long rows, int c, int rows_per_chunk,
                                                         double* __restrict__ part) {
  __shared__ double s0[256], s1[256];
  const int col = blockIdx.x * BN_COLS + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = std::min<long long>(rows, r0 + rows_per_chunk);
  double a = 0, b = 0;
  if (col < c) {
    if (mode == 0) {
      for (long long r = r0 + rg; r < r1; r += 4) {
        const double v = x[r * c + col];
        a += v;
        b += v * v;
      }
    } else {
      const float m = mean[col], rs = rstd[col];
      for (long long r = r0 + rg; r < r1; r += 4) {
        const long long e = r * c + col;
        float g = dy[e];
        if (slope >= 0.f && y[e] < 0.f) g *= slope;
        a += g;
        b += (double)g * ((x[e] - m) * rs);
      }
    }
  }
  s0[threadIdx.x] = a;
  s1[threadIdx.x] = b;
  __syncthreads();
  if (rg == 0 && col < c) {
    const long long nchunk = gridDim.y;
    const int t = threadIdx.x;
    part[(long long)blockIdx.y * c + col] = s0[t] + s0[t + 64] + s0[t + 128] + s0[t + 192];
    part[(nchunk + blockIdx.y) * (long long)c + col] = s1[t] + s1[t + 64] + s1[t + 128] + s1[t + 192];
  }
}

// fwd finalize: mean, biased var -> rstd; running stats (momentum, unbiased var) when given
__global__ void bn_stats_kernel(const double* __restrict__ part, int chunks, int c, long long rows, float eps,
                                float momentum, float* __restrict__ mean, float* __restrict__ rstd,
                                float* __restrict__ run_mean, float* __restrict__ run_var) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= c) return;
  double s = 0, q = 0;
  for (int k = 0; k < chunks; ++k) {
    s += part[(long long)k * c + col];
    q += part[((long long)chunks + k) * c + col];
  }
  const double m = s / (double)rows;
  const double var = std::max(q / (double)rows - m * m, 0.0);
  mean[col] = (float)m;
  rstd[col] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    const double unb = rows > 1 ? var * (double)rows / (double)(rows - 1) : var;
    run_mean[col] = (float)((1.0 - momentum) * run_mean[col] + momentum * m);
    run_var[col] = (float)((1.0 - momentum) * run_var[col] + momentum * unb);
  }
}

__global__ void bn_eval_stats_kernel(const float* __restrict__ run_mean, const float* __restrict__ run_var, float eps,
                                     int c, float* __restrict__ mean, float* __restrict__ rstd) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= c) return;
  mean[col] = run_mean[col];
  rstd[col] = (float)(1.0 / sqrt((double)run_var[col] + (double)eps));
}

// y = leaky((x - mean) * rstd * gamma + beta)   (slope < 0: no activation)
__global__ void bn_apply_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                const float* __restrict__ rstd, const float* __restrict__ gamma,
                                const float* __restrict__ beta, float slope, float* __restrict__ y, long long n, int c) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    float v = (x[e] - mean[ch]) * rstd[ch] * gamma[ch] + beta[ch];
    if (slope >= 0.f && v < 0.f) v *= slope;
    y[e] = v;
  }
}

// bwd finalize: dgamma += sum g*xhat, dbeta += sum g; coefficients for dx
__global__ void bn_bwd_stats_kernel(const double* __restrict__ part, int chunks, int c,
                                    float* __restrict__ sum_g, float* __restrict__ sum_gx,
                                    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= c) return;
  double s = 0, q = 0;
  for (int k = 0; k < chunks; ++k) {
    s += part[(long long)k * c + col];
    q += part[((long long)chunks + k) * c + col];
  }
  sum_g[col] = (float)s;
  sum_gx[col] = (float)q;
  if (dgamma) dgamma[col] += (float)q;
  if (dbeta) dbeta[col] += (float)s;
}

// dx = gamma*rstd/N * (N*g - sum_g - xhat*sum_gx)   (training mode)
__global__ void bn_dx_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ dy,
                             const float* __restrict__ mean, const float* __restrict__ rstd,
                             const float* __restrict__ gamma, const float* __restrict__ sum_g,
                             const float* __restrict__ sum_gx, float slope, long long rows, float* __restrict__ dx,
                             long long n, int c) {
  const float inv_n = 1.f / (float)rows;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % c);
    float g = dy[e];
    if (slope >= 0.f && y[e] < 0.f) g *= slope;
    const float xh = (x[e] - mean[ch]) * rstd[ch];
    dx[e] = gamma[ch] * rstd[ch] * (g - inv_n * sum_g[ch] - xh * inv_n * sum_gx[ch]);
  }
}

__global__ void leaky_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, float slope, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float v = x[e];
    y[e] = v < 0.f ? v * slope : v;
  }
}

// grad through the in-place LeakyReLU: the mask comes from the output (same sign as the input)
__global__ void leaky_bwd_kernel(const float* __restrict__ y, const float* __restrict__ dy, float* __restrict__ dx,
                                 float slope, long long n) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x)
    dx[e] = y[e] < 0.f ? dy[e] * slope : dy[e];
}

static int egrid(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_batch_norm_workspace_bytes(long long rows, int c) {
  return (size_t)2 * bn_chunks(rows, c) * c * sizeof(double) + (size_t)2 * c * sizeof(float) + 256;
}

// training: batch statistics (mean/rstd written out), running stats updated when run_mean != NULL;
// eval (training == 0): normalise with the running statistics.
int mvae_batch_norm_fwd_nhwc(const float* x, const float* gamma, const float* beta, float* y, float* mean, float* rstd,
                             float* run_mean, float* run_var, long long rows, int c, float eps, float momentum,
                             int training, float slope, void* workspace, size_t workspace_bytes, void* stream) {
  if (rows <= 0 || c <= 0) { set_error("batch_norm: bad sizes"); return MVAE_EINVAL; }
  hipStream_t st = (hipStream_t)stream;
  const long long n = rows * c;
  if (training) {
    const int chunks = bn_chunks(rows, c);
    if (workspace_bytes < (size_t)2 * chunks * c * sizeof(double)) { set_error("batch_norm: workspace"); return MVAE_EWORKSPACE; }
    const int rpc = (int)((rows + chunks - 1) / chunks);
    hipLaunchKernelGGL(bn_partial_kernel, dim3((c + BN_COLS - 1) / BN_COLS, chunks), dim3(256), 0, st, 0, x, nullptr,
                       nullptr, nullptr, nullptr, 0.f, rows, c, rpc, (double*)workspace);
    hipLaunchKernelGGL(bn_stats_kernel, dim3((c + 255) / 256), dim3(256), 0, st, (const double*)workspace, chunks, c,
                       rows, eps, momentum, mean, rstd, run_mean, run_var);
  } else {
    // eval: mean/rstd from the running statistics
    if (!run_mean || !run_var) { set_error("batch_norm: eval mode needs running stats"); return MVAE_EINVAL; }
    hipLaunchKernelGGL(bn_eval_stats_kernel, dim3((c + 255) / 256), dim3(256), 0, st, run_mean, run_var, eps, c, mean,
                       rstd);
  }
  hipLaunchKernelGGL(bn_apply_kernel, dim3(egrid(n)), dim3(256), 0, st, x, mean, rstd, gamma, beta, slope, y, n, c);
  return launch_status();
}

int mvae_batch_norm_bwd_nhwc(const float* x, const float* y, const float* dy, const float* gamma, const float* mean,
                             const float* rstd, float* dx, float* dgamma, float* dbeta, long long rows, int c,
                             float slope, void* workspace, size_t workspace_bytes, void* stream) {
  if (rows <= 0 || c <= 0) { set_error("batch_norm_bwd: bad sizes"); return MVAE_EINVAL; }
  const int chunks = bn_chunks(rows, c);
  const size_t need = (size_t)2 * chunks * c * sizeof(double) + (size_t)2 * c * sizeof(float);
  if (workspace_bytes < need) { set_error("batch_norm_bwd: workspace"); return MVAE_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
  float* sums = (float*)((char*)workspace + (size_t)2 * chunks * c * sizeof(double));
  const int rpc = (int)((rows + chunks - 1) / chunks);
  hipLaunchKernelGGL(bn_partial_kernel, dim3((c + BN_COLS - 1) / BN_COLS, chunks), dim3(256), 0, st, 1, x, y, dy, mean,
                     rstd, slope, rows, c, rpc, part);
  hipLaunchKernelGGL(bn_bwd_stats_kernel, dim3((c + 255) / 256), dim3(256), 0, st, (const double*)part, chunks, c, sums,
                     sums + c, dgamma, dbeta);
  const long long n = rows * c;
  hipLaunchKernelGGL(bn_dx_kernel, dim3(egrid(n)), dim3(256), 0, st, x, y, dy, mean, rstd, gamma, sums, sums + c, slope,
                     rows, dx, n, c);
  return launch_status();
}

int mvae_leaky_relu_fwd(const float* x, float* y, float slope, long long n, void* stream) {
  if (n < 0) { set_error("leaky_relu: bad size"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(leaky_fwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, x, y, slope, n);
  return launch_status();
}

int mvae_leaky_relu_bwd(const float* y, const float* dy, float* dx, float slope, long long n, void* stream) {
  if (n < 0) { set_error("leaky_relu_bwd: bad size"); return MVAE_EINVAL; }
  if (n == 0) return MVAE_OK;
  hipLaunchKernelGGL(leaky_bwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, y, dy, dx, slope, n);
  return launch_status();
}

}  // extern "C"
