// GroupNorm (+ SiLU, + inverted dropout) forward/backward over NHWC activations, and the
// attention row-softmax. Reference: Normalize = nn.GroupNorm(min(32,C), C, eps=1e-6, affine)
// (encoder_decoder.py:28-33), nonlinearity = x*sigmoid(x) (:13-15), nn.Dropout in ResnetBlock
// (:160-163), softmax(dim=2) in AttnBlock (:96-97).
//
// Layout: x is [nb][HW][C] (C contiguous). Statistics are per (sample, group) over HW x C/G.
// Every reduction is two-stage and fixed-order (per-block partials in fp64 -> finalize), so the
// results are bitwise reproducible run to run.
#include "common.h"
#include <algorithm>
#include <stdlib.h>

namespace mvae {

#ifndef GN_UNROLL
#define GN_UNROLL 4  // rows in flight per thread in the streaming GroupNorm kernels
#endif

// streaming 16-B load of an activation / gradient read once per pass, non-temporal policy (the stream does not
// displace the consumer GEMM's working set): GroupNorm bwd chain -5 %, fwd -3 % on c4 (same-box A/B);
// GN_TEMPORAL=1 builds the plain loads
__device__ __forceinline__ float4 gn_ld4(const float* p) {
#ifndef GN_TEMPORAL
  const f32x4 v = __builtin_nontemporal_load((const f32x4*)p);
  return float4{v[0], v[1], v[2], v[3]};
#else
  return *(const float4*)p;
#endif
}

// counter-based hash -> uniform [0,1) for the dropout mask (recomputed in backward, never stored)
__device__ __forceinline__ float hash_uniform(unsigned long long seed, unsigned long long idx) {
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(unsigned)(z >> 40) * (1.0f / 16777216.0f);
}

// Per-channel partial sums over a chunk of rows of one sample.
//   kind 0 (stats):  s0 = sum x,          s1 = sum x^2
//   kind 1 (bwd):    s0 = sum dyn,        s1 = sum dyn * xhat
// where dyn is the gradient w.r.t. the GroupNorm output (through SiLU / dropout if fused).
struct GnArgs {
  const float* x;
  const float* dy;
  const float* mean;   // [nb*G]
  const float* rstd;   // [nb*G]
  const float* gamma;
  const float* beta;
  int nb, hw, C, G, rows_per_chunk, chunks;
  int silu;
  float drop_p;
  unsigned long long seed;
  double* ws;  // [nb][chunks][C][2]
  int y_split;  // forward apply: write y as split4_bf16 groups (the 3xBF16 GEMM operand format)
  const float* dx_add;  // backward: optional gradient of the same tensor from another branch, summed into dx
};

// Thread mapping shared by the NHWC GroupNorm kernels: a block owns (sample b, chunk of rows); a
// thread owns one 4-channel column group c4 and walks rows row_lo + rph, + rpar, ... (rpar rows in
// flight per block), unrolled 4x so every thread keeps 4 independent 16-B loads in flight.
struct GnMap {
  int C4, rpar, c4, rph, row_lo, row_hi;
  bool act;
  __device__ GnMap(const GnArgs& a, int cg0) {
    C4 = a.C >> 2;
    const int tid = threadIdx.x;
    rpar = C4 >= 256 ? 1 : 256 / C4;
    c4 = C4 >= 256 ? cg0 + tid : tid % C4;
    rph = C4 >= 256 ? 0 : tid / C4;
    act = C4 >= 256 ? (c4 < C4) : (tid < rpar * C4);
    row_lo = blockIdx.x * a.rows_per_chunk;
    row_hi = min(a.hw, row_lo + a.rows_per_chunk);
  }
};

template <int KIND>
__global__ void __launch_bounds__(256) gn_partial_kernel(GnArgs a) {
  const int b = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
  const int cpg = a.C / a.G;
  __shared__ double red[256 * 8];
  const long long sbase = (long long)b * a.hw * a.C;
  for (int cg0 = 0; cg0 < (a.C >> 2); cg0 += 256) {
    GnMap mp(a, cg0);
    double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
    if (mp.act) {
      float m[4] = {0, 0, 0, 0}, rs[4] = {0, 0, 0, 0}, gm[4] = {0, 0, 0, 0}, bt[4] = {0, 0, 0, 0};
      if (KIND == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = mp.c4 * 4 + e, g = c / cpg;
          m[e] = a.mean[b * a.G + g];
          rs[e] = a.rstd[b * a.G + g];
          gm[e] = a.gamma[c];
          bt[e] = a.beta[c];
        }
      }
      const float* xp = a.x + sbase + mp.c4 * 4;
      const float* dp = a.dy + sbase + mp.c4 * 4;
      int row = mp.row_lo + mp.rph;
      for (; row < mp.row_hi; row += GN_UNROLL * mp.rpar) {
        float4 xv[GN_UNROLL], dv[GN_UNROLL];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const int r = row + u * mp.rpar;
          const bool ok = r < mp.row_hi;
          xv[u] = ok ? gn_ld4(xp + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
          if (KIND == 1) dv[u] = ok ? gn_ld4(dp + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
          if (KIND == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              s0[e] += xs[e];
              s1[e] += (double)xs[e] * xs[e];
            }
          } else {
            const int r = row + u * mp.rpar;
            if (r >= mp.row_hi) continue;
            const float ds[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
            const long long off = sbase + (long long)r * a.C + mp.c4 * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float d = ds[e];
              if (a.drop_p > 0.f) {
                const float uu = hash_uniform(a.seed, (unsigned long long)(off + e));
                d = (uu >= a.drop_p) ? d / (1.f - a.drop_p) : 0.f;
              }
              const float xh = (xs[e] - m[e]) * rs[e];
              if (a.silu) {
                const float yn = xh * gm[e] + bt[e];
                const float sg = sigmoid_f(yn);
                d = d * sg * (1.f + yn * (1.f - sg));
              }
              s0[e] += d;
              s1[e] += (double)d * xh;
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[tid * 8 + e] = s0[e];
      red[tid * 8 + 4 + e] = s1[e];
    }
    __syncthreads();
    if (mp.act && mp.rph == 0) {
      for (int p = 1; p < mp.rpar; ++p) {  // fixed order: deterministic
        const int t2 = tid + p * mp.C4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] += red[t2 * 8 + e];
          s1[e] += red[t2 * 8 + 4 + e];
        }
      }
      double* w = a.ws + (((long long)b * a.chunks + chunk) * a.C + mp.c4 * 4) * 2;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        w[2 * e] = s0[e];
        w[2 * e + 1] = s1[e];
      }
    }
    __syncthreads();
    if ((a.C >> 2) < 256) break;
  }
}

// one wave per (b, g): fixed-order wave reduction of the chunk x channel partials
__device__ __forceinline__ void gn_group_sums(const GnArgs& a, int b, int g, double& S0, double& S1) {
  const int lane = threadIdx.x & 63, cpg = a.C / a.G;
  double s0 = 0, s1 = 0;
  for (int i = lane; i < a.chunks * cpg; i += 64) {
    const int ch = i / cpg, c = g * cpg + (i - ch * cpg);
    const double* w = a.ws + (((long long)b * a.chunks + ch) * a.C + c) * 2;
    s0 += w[0];
    s1 += w[1];
  }
  S0 = wave_sum_d(s0);
  S1 = wave_sum_d(s1);
}

__global__ void __launch_bounds__(256) gn_stats_finalize_kernel(GnArgs a, float* mean, float* rstd, float* scale,
                                                                float* shift, float eps) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= a.nb * a.G) return;
  const int b = i / a.G, g = i - b * a.G;
  const int cpg = a.C / a.G;
  double s0, s1;
  gn_group_sums(a, b, g, s0, s1);
  const double n = (double)a.hw * cpg;
  const double mu = s0 / n;
  double var = s1 / n - mu * mu;
  if (var < 0) var = 0;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  if (lane == 0) {
    mean[i] = (float)mu;
    rstd[i] = rs;
  }
  for (int c = g * cpg + lane; c < (g + 1) * cpg; c += 64) {
    const float sc = rs * a.gamma[c];
    scale[b * a.C + c] = sc;
    shift[b * a.C + c] = a.beta[c] - (float)mu * sc;
  }
}

// Same finalize from the statistics the producing convolution's epilogue emitted
// (mvae_conv2d_gnstats_nhwc: part[(row/32) * (C/4) + c/4] = {sum, sum sq} over 32 rows x 4 channels)
__global__ void __launch_bounds__(256) gn_stats_finalize_part_kernel(GnArgs a, const double* __restrict__ part,
                                                                     float* mean, float* rstd, float* scale,
                                                                     float* shift, float eps) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= a.nb * a.G) return;
  const int b = i / a.G, g = i - b * a.G;
  const int cpg = a.C / a.G, q4 = cpg >> 2, c4n = a.C >> 2, sbn = a.hw >> 5;
  double s0 = 0, s1 = 0;
  for (int j = lane; j < sbn * q4; j += 64) {  // fixed order per lane, then a fixed wave tree
    const int sb = j / q4, c4 = g * q4 + (j - sb * q4);
    const double* w = part + ((long long)(b * sbn + sb) * c4n + c4) * 2;
    s0 += w[0];
    s1 += w[1];
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  const double n = (double)a.hw * cpg;
  const double mu = s0 / n;
  double var = s1 / n - mu * mu;
  if (var < 0) var = 0;
  const float rs = (float)(1.0 / sqrt(var + (double)eps));
  if (lane == 0) {
    mean[i] = (float)mu;
    rstd[i] = rs;
  }
  for (int c = g * cpg + lane; c < (g + 1) * cpg; c += 64) {
    const float sc = rs * a.gamma[c];
    scale[b * a.C + c] = sc;
    shift[b * a.C + c] = a.beta[c] - (float)mu * sc;
  }
}

// y = [dropout](silu?(x*scale + shift))
__global__ void __launch_bounds__(256) gn_apply_kernel(GnArgs a, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, float* __restrict__ y) {
  const int b = blockIdx.y;
  const long long sbase = (long long)b * a.hw * a.C;
  for (int cg0 = 0; cg0 < (a.C >> 2); cg0 += 256) {
    GnMap mp(a, cg0);
    if (mp.act) {
      const float4 sc = *(const float4*)(scale + (long long)b * a.C + mp.c4 * 4);
      const float4 sh = *(const float4*)(shift + (long long)b * a.C + mp.c4 * 4);
      const float* xp = a.x + sbase + mp.c4 * 4;
      float* yp = y + sbase + mp.c4 * 4;
      for (int row = mp.row_lo + mp.rph; row < mp.row_hi; row += GN_UNROLL * mp.rpar) {
        float4 xv[GN_UNROLL];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const int r = row + u * mp.rpar;
          xv[u] = r < mp.row_hi ? gn_ld4(xp + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const int r = row + u * mp.rpar;
          if (r >= mp.row_hi) continue;
          float o[4] = {xv[u].x * sc.x + sh.x, xv[u].y * sc.y + sh.y, xv[u].z * sc.z + sh.z, xv[u].w * sc.w + sh.w};
          const long long off = sbase + (long long)r * a.C + mp.c4 * 4;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (a.silu) o[k] = o[k] * sigmoid_f(o[k]);
            if (a.drop_p > 0.f) {
              const float uu = hash_uniform(a.seed, (unsigned long long)(off + k));
              o[k] = (uu >= a.drop_p) ? o[k] / (1.f - a.drop_p) : 0.f;
            }
          }
          const float4 ov{o[0], o[1], o[2], o[3]};
          if (a.y_split)
            *(uint4*)(yp + (long long)r * a.C) = split4_bf16(ov);
          else
            *(float4*)(yp + (long long)r * a.C) = ov;
        }
      }
    }
    if ((a.C >> 2) < 256) break;
  }
}

// backward finalize: per (b,g) coefficients so that dx = dyn*k1[b,c] + x*k2[b,g] + k3[b,g]
__global__ void __launch_bounds__(256) gn_bwd_finalize_kernel(GnArgs a, float* k1, float* k2, float* k3) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= a.nb * a.G) return;
  const int b = i / a.G, g = i - b * a.G;
  const int cpg = a.C / a.G;
  double A1 = 0, A2 = 0;
  for (int j = lane; j < a.chunks * cpg; j += 64) {
    const int ch = j / cpg, c = g * cpg + (j - ch * cpg);
    const double* w = a.ws + (((long long)b * a.chunks + ch) * a.C + c) * 2;
    A1 += (double)a.gamma[c] * w[0];
    A2 += (double)a.gamma[c] * w[1];
  }
  A1 = wave_sum_d(A1);
  A2 = wave_sum_d(A2);
  const float rsf = a.rstd[i];
  for (int c = g * cpg + lane; c < (g + 1) * cpg; c += 64) k1[b * a.C + c] = rsf * a.gamma[c];
  if (lane == 0) {
    const double n = (double)a.hw * cpg;
    const double rs = rsf, mu = a.mean[i];
    k2[i] = (float)(-rs * rs * A2 / n);
    k3[i] = (float)(-rs * A1 / n + mu * rs * rs * A2 / n);
  }
}

// dgamma[c] += sum_{b,chunks} s1 ; dbeta[c] += sum s0. Two fixed-order stages so the reduction over the
// nb*chunks partial rows runs on many blocks: stage 1, block (channel tile, slice) sums its slice of rows
// (64 channels x 4 row lanes per block) into part[slice][C][2]; stage 2 sums the slices per channel.
constexpr int GN_PG_SLICES = 64;
__global__ void __launch_bounds__(256) gn_param_grad_kernel(GnArgs a, double* __restrict__ part) {
  __shared__ double sh[2][256];
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sl = blockIdx.y;
  const int n = a.nb * a.chunks;
  const int lo = (int)((long long)n * sl / GN_PG_SLICES), hi = (int)((long long)n * (sl + 1) / GN_PG_SLICES);
  double s0 = 0, s1 = 0;
  if (c < a.C) {
    for (int i = lo + rg; i < hi; i += 4) {
      const double* w = a.ws + ((long long)i * a.C + c) * 2;
      s0 += w[0];
      s1 += w[1];
    }
  }
  sh[0][threadIdx.x] = s0;
  sh[1][threadIdx.x] = s1;
  __syncthreads();
  if (rg == 0 && c < a.C) {
    double* o = part + ((long long)sl * a.C + c) * 2;
    o[0] = sh[0][cl] + sh[0][cl + 64] + sh[0][cl + 128] + sh[0][cl + 192];
    o[1] = sh[1][cl] + sh[1][cl + 64] + sh[1][cl + 128] + sh[1][cl + 192];
  }
}

__global__ void __launch_bounds__(256) gn_param_final_kernel(int C, const double* __restrict__ part,
                                                              float* dgamma, float* dbeta) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  double s0 = 0, s1 = 0;
  for (int sl = 0; sl < GN_PG_SLICES; ++sl) {
    s0 += part[((long long)sl * C + c) * 2];
    s1 += part[((long long)sl * C + c) * 2 + 1];
  }
  if (dgamma) dgamma[c] += (float)s1;
  if (dbeta) dbeta[c] += (float)s0;
}

__global__ void __launch_bounds__(256) gn_dx_kernel(GnArgs a, const float* __restrict__ k1,
                                                    const float* __restrict__ k2, const float* __restrict__ k3,
                                                    float* __restrict__ dx) {
  const int b = blockIdx.y;
  const int cpg = a.C / a.G;
  const long long sbase = (long long)b * a.hw * a.C;
  for (int cg0 = 0; cg0 < (a.C >> 2); cg0 += 256) {
    GnMap mp(a, cg0);
    if (mp.act) {
      float m[4], rs[4], gm[4], bt[4], q1[4], q2[4], q3[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = mp.c4 * 4 + e, bg = b * a.G + c / cpg;
        m[e] = a.mean[bg];
        rs[e] = a.rstd[bg];
        gm[e] = a.gamma[c];
        bt[e] = a.beta[c];
        q1[e] = k1[(long long)b * a.C + c];
        q2[e] = k2[bg];
        q3[e] = k3[bg];
      }
      const float* xp = a.x + sbase + mp.c4 * 4;
      const float* dp = a.dy + sbase + mp.c4 * 4;
      float* op = dx + sbase + mp.c4 * 4;
      const float* ap = a.dx_add ? a.dx_add + sbase + mp.c4 * 4 : nullptr;
      for (int row = mp.row_lo + mp.rph; row < mp.row_hi; row += GN_UNROLL * mp.rpar) {
        float4 xv[GN_UNROLL], dv[GN_UNROLL], av[GN_UNROLL];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const int r = row + u * mp.rpar;
          const bool ok = r < mp.row_hi;
          xv[u] = ok ? gn_ld4(xp + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
          dv[u] = ok ? gn_ld4(dp + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
          // the residual branch's gradient is loaded with the other streams (not behind the arithmetic)
          av[u] = (ap != nullptr && ok) ? gn_ld4(ap + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
          const int r = row + u * mp.rpar;
          if (r >= mp.row_hi) continue;
          const float xs[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
          const float ds[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w};
          const long long off = sbase + (long long)r * a.C + mp.c4 * 4;
          float o[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float d = ds[e];
            if (a.drop_p > 0.f) {
              const float uu = hash_uniform(a.seed, (unsigned long long)(off + e));
              d = (uu >= a.drop_p) ? d / (1.f - a.drop_p) : 0.f;
            }
            if (a.silu) {
              const float yn = (xs[e] - m[e]) * rs[e] * gm[e] + bt[e];
              const float sg = sigmoid_f(yn);
              d = d * sg * (1.f + yn * (1.f - sg));
            }
            o[e] = d * q1[e] + xs[e] * q2[e] + q3[e];
          }
          if (ap != nullptr) {  // the other branch's gradient of x (ResnetBlock / AttnBlock residual): summed here
            o[0] += av[u].x; o[1] += av[u].y; o[2] += av[u].z; o[3] += av[u].w;
          }
          *(float4*)(op + (long long)r * a.C) = float4{o[0], o[1], o[2], o[3]};
        }
      }
    }
    if ((a.C >> 2) < 256) break;
  }
}

// ------------------------------------------------------------------------------------------
// Resident GroupNorm for small per-sample tensors (the 28x28 / 14x14 / 7x7 levels of c2 / c3, where the
// producing conv cannot emit the statistics: h*w % 32 != 0). A workgroup owns (sample b, slab of SC
// channels = whole groups) and holds the slab in registers (IT float4 per thread), so x is read from HBM
// ONCE per pass: forward = statistics (two-pass: mean, then centred variance, on the resident values) +
// apply in one launch (8 B/elem); backward = partial sums + finalize + dx in one launch (12 B/elem, +4 with
// the residual-branch add) and a per-channel parameter-gradient reduction. Cross-thread sums: a fixed wave
// butterfly, then a fixed-order LDS combine -- bitwise reproducible.
// Thread map: C4 = SC/4 (a power of two <= 256) channel quads, rpar = 256 / C4 row phases, thread (rph, c4)
// walks rows rph, rph + rpar, ... (at most IT of them).
// ------------------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ void gn_slab_reduce(float (&s)[K], int C4, float* red /*[K][256]*/, float* out /*[C4][K]*/) {
  const int tid = threadIdx.x;
  if (C4 < 64) {
    for (int m = C4; m < 64; m <<= 1) {  // lanes with the same c4 differ by multiples of C4
#pragma unroll
      for (int k = 0; k < K; ++k) s[k] += __shfl_xor(s[k], m, 64);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) red[k * 256 + tid] = s[k];
  __syncthreads();
  if (tid < C4) {
    const int stride = C4 < 64 ? 64 : C4;  // one representative per (wave, c4)
    float t[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = 0.f;
    for (int j = tid; j < 256; j += stride)
#pragma unroll
      for (int k = 0; k < K; ++k) t[k] += red[k * 256 + j];
#pragma unroll
    for (int k = 0; k < K; ++k) out[tid * K + k] = t[k];
  }
  __syncthreads();
}

constexpr int GN_RES_MAXC = 1024;  // slab channels (C4 <= 256)

template <int IT>
__global__ void __launch_bounds__(256) gn_fwd_resident_kernel(GnArgs a, int SC, float* __restrict__ y,
                                                              float* __restrict__ mean, float* __restrict__ rstd,
                                                              float eps) {
  __shared__ float red[4 * 256];
  __shared__ float chs[GN_RES_MAXC];
  __shared__ float gmu[GN_RES_MAXC], grs[GN_RES_MAXC];  // per slab channel: its group's mean / rstd
  const int tid = threadIdx.x, b = blockIdx.y, c0 = blockIdx.x * SC;
  const int C4 = SC >> 2, rpar = 256 / C4, c4 = tid & (C4 - 1), rph = tid / C4;
  const int cpg = a.C / a.G, ngl = SC / cpg;
  const double n = (double)a.hw * cpg;
  const long long sbase = (long long)b * a.hw * a.C + c0 + c4 * 4;
  float4 v[IT];
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rph + i * rpar;
    v[i] = r < a.hw ? gn_ld4(a.x + sbase + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
    s[0] += v[i].x; s[1] += v[i].y; s[2] += v[i].z; s[3] += v[i].w;
  }
  gn_slab_reduce<4>(s, C4, red, chs);
  for (int gl = tid; gl < ngl; gl += 256) {
    float t = 0.f;
    for (int j = 0; j < cpg; ++j) t += chs[gl * cpg + j];
    const float mu = (float)((double)t / n);
    for (int j = 0; j < cpg; ++j) gmu[gl * cpg + j] = mu;
  }
  __syncthreads();
  float mu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    mu[e] = gmu[c4 * 4 + e];
    s[e] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    if (rph + i * rpar < a.hw) {
      const float d0 = v[i].x - mu[0], d1 = v[i].y - mu[1], d2 = v[i].z - mu[2], d3 = v[i].w - mu[3];
      s[0] = fmaf(d0, d0, s[0]); s[1] = fmaf(d1, d1, s[1]); s[2] = fmaf(d2, d2, s[2]); s[3] = fmaf(d3, d3, s[3]);
    }
  }
  gn_slab_reduce<4>(s, C4, red, chs);
  for (int gl = tid; gl < ngl; gl += 256) {
    float t = 0.f;
    for (int j = 0; j < cpg; ++j) t += chs[gl * cpg + j];
    const float rs = (float)(1.0 / sqrt((double)t / n + (double)eps));
    for (int j = 0; j < cpg; ++j) grs[gl * cpg + j] = rs;
    const int gi = b * a.G + c0 / cpg + gl;
    mean[gi] = gmu[gl * cpg];
    rstd[gi] = rs;
  }
  __syncthreads();
  float sc[4], sh[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + c4 * 4 + e;
    sc[e] = grs[c4 * 4 + e] * a.gamma[c];
    sh[e] = a.beta[c] - mu[e] * sc[e];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rph + i * rpar;
    if (r >= a.hw) continue;
    float o[4] = {v[i].x * sc[0] + sh[0], v[i].y * sc[1] + sh[1], v[i].z * sc[2] + sh[2], v[i].w * sc[3] + sh[3]};
    const long long off = sbase + (long long)r * a.C;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (a.silu) o[k] = o[k] * sigmoid_f(o[k]);
      if (a.drop_p > 0.f) {
        const float uu = hash_uniform(a.seed, (unsigned long long)(off + k));
        o[k] = (uu >= a.drop_p) ? o[k] / (1.f - a.drop_p) : 0.f;
      }
    }
    const float4 ov{o[0], o[1], o[2], o[3]};
    if (a.y_split)
      *(uint4*)(y + off) = split4_bf16(ov);
    else
      *(float4*)(y + off) = ov;
  }
}

// backward; pws = [2][C][nb] fp64 per-sample channel sums {sum dyn, sum dyn*xhat} for the parameter gradients
template <int IT>
__global__ void __launch_bounds__(256) gn_bwd_resident_kernel(GnArgs a, int SC, double* __restrict__ pws,
                                                              float* __restrict__ dx) {
  __shared__ float red[8 * 256];
  __shared__ float chs[GN_RES_MAXC * 2];
  __shared__ float gk2[GN_RES_MAXC], gk3[GN_RES_MAXC];
  const int tid = threadIdx.x, b = blockIdx.y, c0 = blockIdx.x * SC;
  const int C4 = SC >> 2, rpar = 256 / C4, c4 = tid & (C4 - 1), rph = tid / C4;
  const int cpg = a.C / a.G, ngl = SC / cpg;
  const long long sbase = (long long)b * a.hw * a.C + c0 + c4 * 4;
  float m[4], rs[4], gm[4], bt[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = c0 + c4 * 4 + e, bg = b * a.G + c / cpg;
    m[e] = a.mean[bg];
    rs[e] = a.rstd[bg];
    gm[e] = a.gamma[c];
    bt[e] = a.beta[c];
  }
  float4 xv[IT], dv[IT], av[IT];
  const bool add = a.dx_add != nullptr;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rph + i * rpar;
    const bool ok = r < a.hw;
    const long long off = sbase + (long long)r * a.C;
    xv[i] = ok ? gn_ld4(a.x + off) : float4{0.f, 0.f, 0.f, 0.f};
    dv[i] = ok ? gn_ld4(a.dy + off) : float4{0.f, 0.f, 0.f, 0.f};
    av[i] = (add && ok) ? gn_ld4(a.dx_add + off) : float4{0.f, 0.f, 0.f, 0.f};
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const long long off = sbase + (long long)(rph + i * rpar) * a.C;
    float xs[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
    float ds[4] = {dv[i].x, dv[i].y, dv[i].z, dv[i].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = ds[e];  // rows past hw hold d = 0: they add nothing
      if (a.drop_p > 0.f) {
        const float uu = hash_uniform(a.seed, (unsigned long long)(off + e));
        d = (uu >= a.drop_p) ? d / (1.f - a.drop_p) : 0.f;
      }
      const float xh = (xs[e] - m[e]) * rs[e];
      if (a.silu) {
        const float yn = xh * gm[e] + bt[e];
        const float sg = sigmoid_f(yn);
        d = d * sg * (1.f + yn * (1.f - sg));
      }
      ds[e] = d;
      s[e] += d;
      s[4 + e] = fmaf(d, xh, s[4 + e]);
    }
    dv[i] = float4{ds[0], ds[1], ds[2], ds[3]};
  }
  // chs[(c4*8) + k]: k 0-3 = sum dyn of channels c4*4+k, k 4-7 = sum dyn*xhat
  gn_slab_reduce<8>(s, C4, red, chs);
  for (int t = tid; t < SC; t += 256) {
    const int q = t >> 2, e = t & 3, c = c0 + t;
    pws[(long long)c * a.nb + b] = chs[q * 8 + e];
    pws[((long long)a.C + c) * a.nb + b] = chs[q * 8 + 4 + e];
  }
  for (int gl = tid; gl < ngl; gl += 256) {
    double A1 = 0.0, A2 = 0.0;
    for (int j = 0; j < cpg; ++j) {
      const int cl = gl * cpg + j;
      const double g = a.gamma[c0 + cl];
      A1 += g * chs[(cl >> 2) * 8 + (cl & 3)];
      A2 += g * chs[(cl >> 2) * 8 + 4 + (cl & 3)];
    }
    const int gi = b * a.G + c0 / cpg + gl;
    const double n = (double)a.hw * cpg, r = a.rstd[gi], mu = a.mean[gi];
    const float k2 = (float)(-r * r * A2 / n), k3 = (float)(-r * A1 / n + mu * r * r * A2 / n);
    for (int j = 0; j < cpg; ++j) {
      gk2[gl * cpg + j] = k2;
      gk3[gl * cpg + j] = k3;
    }
  }
  __syncthreads();
  float q1[4], q2[4], q3[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    q1[e] = rs[e] * gm[e];
    q2[e] = gk2[c4 * 4 + e];
    q3[e] = gk3[c4 * 4 + e];
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int r = rph + i * rpar;
    if (r >= a.hw) continue;
    float4 o{dv[i].x * q1[0] + xv[i].x * q2[0] + q3[0], dv[i].y * q1[1] + xv[i].y * q2[1] + q3[1],
             dv[i].z * q1[2] + xv[i].z * q2[2] + q3[2], dv[i].w * q1[3] + xv[i].w * q2[3] + q3[3]};
    if (add) {
      o.x += av[i].x; o.y += av[i].y; o.z += av[i].z; o.w += av[i].w;
    }
    *(float4*)(dx + sbase + (long long)r * a.C) = o;
  }
}

// dgamma[c] += sum_b pws[1][c][b], dbeta[c] += sum_b pws[0][c][b]: one block per channel, fixed order
__global__ void __launch_bounds__(256) gn_param_reduce_kernel(const double* __restrict__ pws, int nb, int C,
                                                              float* dgamma, float* dbeta) {
  __shared__ double sh[2][4];
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double s0 = 0.0, s1 = 0.0;
  for (int i = tid; i < nb; i += 256) {
    s0 += pws[(long long)c * nb + i];
    s1 += pws[((long long)C + c) * nb + i];
  }
  s0 = wave_sum_d(s0);
  s1 = wave_sum_d(s1);
  if (lane == 0) {
    sh[0][wv] = s0;
    sh[1][wv] = s1;
  }
  __syncthreads();
  if (tid == 0) {
    if (dbeta) dbeta[c] += (float)(((sh[0][0] + sh[0][1]) + sh[0][2]) + sh[0][3]);
    if (dgamma) dgamma[c] += (float)(((sh[1][0] + sh[1][1]) + sh[1][2]) + sh[1][3]);
  }
}

// Largest slab (of >= 16 channels: 64-B row segments) with <= 16 rows per thread that still gives >= 512
// workgroups; else the feasible slab with the most workgroups.
// slab width for the resident path (0: not eligible). Path selection: mvae_set_group_norm_path (0 auto,
// 1 streaming only); before any call, MVAE_GN_RESIDENT=0 selects streaming only.
static int g_gn_path = -1;
static int gn_resident_slab(int nb, int hw, int C, int G, int* items) {
  if (g_gn_path < 0) {
    const char* e = getenv("MVAE_GN_RESIDENT");
    g_gn_path = (e != nullptr && e[0] == '0') ? 1 : 0;
  }
  if (g_gn_path == 1 || C % G) return 0;
  const int cpg = C / G;
  int best = 0, best_it = 0;
  for (int sc = std::min(C, GN_RES_MAXC); sc >= 16; sc >>= 1) {
    const int c4 = sc >> 2;
    if ((c4 & (c4 - 1)) || C % sc || sc % cpg) continue;
    const int it = (hw + 256 / c4 - 1) / (256 / c4);
    if (it > 16) continue;
    best = sc;
    best_it = it;
    if ((long long)nb * (C / sc) >= 512) break;
  }
  *items = best_it <= 4 ? 4 : best_it <= 8 ? 8 : 16;
  return best;
}

static int gn_target_blocks() {
  static int v = [] {
    const char* e = getenv("MVAE_GN_BLOCKS");  // experiment knob: target grid size of the streaming kernels
    return e ? std::max(64, atoi(e)) : 1024;
  }();
  return v;
}
static int gn_chunks(int nb, int hw) {
  int chunks = 1;
  while ((long long)nb * chunks < gn_target_blocks() && hw / (chunks * 2) >= 16) chunks *= 2;
  return chunks;
}

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_set_group_norm_path(int mode) {
  if (mode != 0 && mode != 1) {
    set_error("group_norm path: 0 (auto: resident for small per-sample tensors) or 1 (streaming only)");
    return MVAE_EINVAL;
  }
  g_gn_path = mode;
  return MVAE_OK;
}

size_t mvae_group_norm_workspace_bytes(int nb, int hw, int c) {
  const int ch = gn_chunks(nb, hw);
  // fp64 partials + 3 float arrays of nb*C (scale/shift or k1) + 2 of nb*C (k2/k3 upper bound)
  // + the parameter-gradient slice partials [GN_PG_SLICES][C][2] fp64
  return (size_t)nb * ch * c * 2 * sizeof(double) + (size_t)nb * c * 5 * sizeof(float) + 256 +
         (size_t)GN_PG_SLICES * c * 2 * sizeof(double) + 256;
}

// y = [dropout](silu?(GroupNorm(x)))  ; saves mean/rstd [nb*groups]
int mvae_group_norm_fwd_nhwc(const float* x, const float* gamma, const float* beta, float* y, float* mean,
                             float* rstd, int nb, int hw, int c, int groups, float eps, int silu,
                             float drop_p, unsigned long long seed, int y_split, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups) {
    set_error("group_norm: C must be a multiple of 4 and of groups");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.gamma = gamma; a.beta = beta; a.nb = nb; a.hw = hw; a.C = c; a.G = groups;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.ws = (double*)workspace;
  int it = 0;
  if (const int sc = gn_resident_slab(nb, hw, c, groups, &it)) {
    a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split;
    const dim3 grid(c / sc, nb);
    if (it == 4) hipLaunchKernelGGL(gn_fwd_resident_kernel<4>, grid, dim3(256), 0, st, a, sc, y, mean, rstd, eps);
    else if (it == 8) hipLaunchKernelGGL(gn_fwd_resident_kernel<8>, grid, dim3(256), 0, st, a, sc, y, mean, rstd, eps);
    else hipLaunchKernelGGL(gn_fwd_resident_kernel<16>, grid, dim3(256), 0, st, a, sc, y, mean, rstd, eps);
    return launch_status();
  }
  float* scale = (float*)((char*)workspace + (size_t)nb * a.chunks * c * 2 * sizeof(double));
  float* shift = scale + (size_t)nb * c;
  hipLaunchKernelGGL(gn_partial_kernel<0>, dim3(a.chunks, nb), dim3(256), 0, st, a);
  hipLaunchKernelGGL(gn_stats_finalize_kernel, dim3(cdiv((long long)nb * groups, 4)), dim3(256), 0, st, a,
                     mean, rstd, scale, shift, eps);
  a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(a.chunks, nb), dim3(256), 0, st, a, scale, shift, y);
  return launch_status();
}

// Forward from the statistics emitted by the producing convolution (mvae_conv2d_gnstats_nhwc): no
// statistics pass over x.
int mvae_group_norm_fwd_part_nhwc(const float* x, const double* part, const float* gamma, const float* beta, float* y,
                                  float* mean, float* rstd, int nb, int hw, int c, int groups, float eps, int silu,
                                  float drop_p, unsigned long long seed, int y_split, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups || (c / groups) % 4 || hw % 32) {
    set_error("group_norm_part: needs hw %% 32 == 0 and channels per group %% 4 == 0");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_part: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.gamma = gamma; a.beta = beta; a.nb = nb; a.hw = hw; a.C = c; a.G = groups;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.ws = (double*)workspace;
  float* scale = (float*)((char*)workspace + (size_t)nb * a.chunks * c * 2 * sizeof(double));
  float* shift = scale + (size_t)nb * c;
  hipLaunchKernelGGL(gn_stats_finalize_part_kernel, dim3(cdiv((long long)nb * groups, 4)), dim3(256), 0, st, a, part,
                     mean, rstd, scale, shift, eps);
  a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split;
  hipLaunchKernelGGL(gn_apply_kernel, dim3(a.chunks, nb), dim3(256), 0, st, a, scale, shift, y);
  return launch_status();
}

// dx = d/dx of the fused forward [+ dx_add when non-null]; dgamma/dbeta are ACCUMULATED (+=) when non-null.
int mvae_group_norm_bwd_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                             const float* mean, const float* rstd, float* dx, const float* dx_add,
                             float* dgamma, float* dbeta,
                             int nb, int hw, int c, int groups, int silu, float drop_p,
                             unsigned long long seed, void* workspace, size_t workspace_bytes, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups) {
    set_error("group_norm_bwd: bad geometry");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.dy = dy; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta; a.dx_add = dx_add;
  a.nb = nb; a.hw = hw; a.C = c; a.G = groups; a.silu = silu; a.drop_p = drop_p; a.seed = seed;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.ws = (double*)workspace;
  int it = 0;
  if (const int sc = gn_resident_slab(nb, hw, c, groups, &it)) {
    double* pws = (double*)workspace;  // [2][C][nb] fp64 (within the [nb][chunks][C][2] partial area)
    const dim3 grid(c / sc, nb);
    if (it == 4) hipLaunchKernelGGL(gn_bwd_resident_kernel<4>, grid, dim3(256), 0, st, a, sc, pws, dx);
    else if (it == 8) hipLaunchKernelGGL(gn_bwd_resident_kernel<8>, grid, dim3(256), 0, st, a, sc, pws, dx);
    else hipLaunchKernelGGL(gn_bwd_resident_kernel<16>, grid, dim3(256), 0, st, a, sc, pws, dx);
    if (dgamma || dbeta)
      hipLaunchKernelGGL(gn_param_reduce_kernel, dim3(c), dim3(256), 0, st, (const double*)pws, nb, c, dgamma, dbeta);
    return launch_status();
  }
  float* k1 = (float*)((char*)workspace + (size_t)nb * a.chunks * c * 2 * sizeof(double));
  float* k2 = k1 + (size_t)nb * c;
  float* k3 = k2 + (size_t)nb * c;
  hipLaunchKernelGGL(gn_partial_kernel<1>, dim3(a.chunks, nb), dim3(256), 0, st, a);
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(cdiv((long long)nb * groups, 4)), dim3(256), 0, st, a, k1,
                     k2, k3);
  if (dgamma || dbeta) {
    double* part = (double*)(((uintptr_t)(k3 + (size_t)nb * c) + 255) & ~(uintptr_t)255);
    hipLaunchKernelGGL(gn_param_grad_kernel, dim3(cdiv(c, 64), GN_PG_SLICES), dim3(256), 0, st, a, part);
    hipLaunchKernelGGL(gn_param_final_kernel, dim3(cdiv(c, 256)), dim3(256), 0, st, c, (const double*)part, dgamma,
                       dbeta);
  }
  hipLaunchKernelGGL(gn_dx_kernel, dim3(a.chunks, nb), dim3(256), 0, st, a, k1, k2, k3, dx);
  return launch_status();
}

// Backward from the partials emitted by the input-gradient conv that consumed this GroupNorm's output
// (mvae_conv2d_dgrad_gnbwd_nhwc, part = [nb*hw/32][c][2] fp64 {sum dyn, sum dyn*xhat}): no partial pass over
// x and dy. No dropout (the fused conv epilogue does not apply a mask).
int mvae_group_norm_bwd_part_nhwc(const float* x, const float* dy, const double* part, const float* gamma,
                                  const float* beta, const float* mean, const float* rstd, float* dx,
                                  const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c, int groups,
                                  int silu, void* workspace, size_t workspace_bytes, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups || hw % 32 || part == nullptr) {
    set_error("group_norm_bwd_part: needs hw %% 32 == 0 and C %% 4 == 0");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd_part: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.dy = dy; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta; a.dx_add = dx_add;
  a.nb = nb; a.hw = hw; a.C = c; a.G = groups; a.silu = silu; a.drop_p = 0.f; a.seed = 0;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  float* k1 = (float*)((char*)workspace + (size_t)nb * a.chunks * c * 2 * sizeof(double));
  float* k2 = k1 + (size_t)nb * c;
  float* k3 = k2 + (size_t)nb * c;
  GnArgs ap = a;  // the reductions run over the conv's 32-row blocks
  ap.ws = const_cast<double*>(part);
  ap.chunks = hw / 32;
  ap.rows_per_chunk = 32;
  hipLaunchKernelGGL(gn_bwd_finalize_kernel, dim3(cdiv((long long)nb * groups, 4)), dim3(256), 0, st, ap, k1,
                     k2, k3);
  if (dgamma || dbeta) {
    double* pg = (double*)(((uintptr_t)(k3 + (size_t)nb * c) + 255) & ~(uintptr_t)255);
    hipLaunchKernelGGL(gn_param_grad_kernel, dim3(cdiv(c, 64), GN_PG_SLICES), dim3(256), 0, st, ap, pg);
    hipLaunchKernelGGL(gn_param_final_kernel, dim3(cdiv(c, 256)), dim3(256), 0, st, c, (const double*)pg, dgamma,
                       dbeta);
  }
  hipLaunchKernelGGL(gn_dx_kernel, dim3(a.chunks, nb), dim3(256), 0, st, a, k1, k2, k3, dx);
  return launch_status();
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// row softmax (attention probabilities): one wave per row
// ------------------------------------------------------------------------------------------
namespace mvae {
__global__ void __launch_bounds__(256) softmax_rows_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                           long long rows, int n) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + row * n;
  float* yr = y + row * n;
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) m = fmaxf(m, xr[j]);
  m = wave_max_f(m);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += __expf(xr[j] - m);
  s = wave_sum_f(s);
  const float inv = 1.f / s;
  for (int j = lane; j < n; j += 64) yr[j] = __expf(xr[j] - m) * inv;
}

__global__ void __launch_bounds__(256) softmax_rows_bwd_kernel(const float* __restrict__ y,
                                                               const float* __restrict__ dy,
                                                               float* __restrict__ dx, long long rows, int n) {
  const long long row = blockIdx.x * 4LL + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* yr = y + row * n;
  const float* dr = dy + row * n;
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += yr[j] * dr[j];
  s = wave_sum_f(s);
  for (int j = lane; j < n; j += 64) dx[row * n + j] = yr[j] * (dr[j] - s);
}
}  // namespace mvae

extern "C" {
int mvae_softmax_rows(const float* x, float* y, long long rows, int n, void* stream) {
  if (rows <= 0 || n <= 0) { set_error("softmax: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x,
                     y, rows, n);
  return launch_status();
}
int mvae_softmax_rows_bwd(const float* y, const float* dy, float* dx, long long rows, int n, void* stream) {
  if (rows <= 0 || n <= 0) { set_error("softmax_bwd: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(softmax_rows_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     y, dy, dx, rows, n);
  return launch_status();
}
}  // extern "C"
