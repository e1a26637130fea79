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
  int y_split;  // forward apply: write y as split4_bf16 groups (1), packed bf16 (2) or planar 3xBF16 (3: bf16 hi plane
                // of nb*hw*C elements, then the lo plane) -- the GEMM operand formats
  const float* dx_add;  // backward: optional gradient of the same tensor from another branch, summed into dx
  // process-wide dropout salt in device memory (mvae_set_dropout_salt): mixed into the seed, so a replayed HIP
  // graph -- whose kernel arguments, seeds included, are frozen -- still draws a fresh mask once the salt advances
  const unsigned long long* salt;
  // backward, optional (mvae_group_norm_bwd_pack_nhwc): dx also written as packed bf16 (RNE, 2 B per element at the
  // element offsets: the bf16-mixed GEMMs' operand format) and its per-channel column sums as fp64 partials
  // (streaming kernel: [nb * chunks][C], resident kernel: [nb][C]) -- the consuming conv's output gradient and bias
  // gradient, without a separate pass over dx
  uint2* dxp;
  double* csp;
  int dxp_split;  // dxp format: 0 = packed bf16 (bf16-mixed), 1 = split4_bf16 groups (3xBF16: 4 B per element at the
                  // fp32 element offsets, mvae_split_bf16's layout -- the pre-split dY operand of the fp32-class GEMMs)
};
__device__ __forceinline__ unsigned long long drop_seed(const GnArgs& a) {
  return a.salt ? a.seed ^ (*a.salt * 0xD1B54A32D192ED03ull) : a.seed;
}

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
                const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + e));
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
              const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + k));
              o[k] = (uu >= a.drop_p) ? o[k] / (1.f - a.drop_p) : 0.f;
            }
          }
          const float4 ov{o[0], o[1], o[2], o[3]};
          if (a.y_split >= 2) {  // packed bf16 / planar 3xBF16 hi plane: element offset * 2 B
            const unsigned h01 = pk_bf16x2(ov.x, ov.y), h23 = pk_bf16x2(ov.z, ov.w);
            *(uint2*)((__bf16*)y + off) = uint2{h01, h23};
            if (a.y_split == 3)
              *(uint2*)((__bf16*)y + (long long)a.nb * a.hw * a.C + off) =
                  uint2{pk_bf16x2(ov.x - __uint_as_float(h01 << 16), ov.y - __uint_as_float(h01 & 0xFFFF0000u)),
                        pk_bf16x2(ov.z - __uint_as_float(h23 << 16), ov.w - __uint_as_float(h23 & 0xFFFF0000u))};
          } else if (a.y_split)
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
  __shared__ double csr[256][4];  // (a.csp) per-thread column sums, combined over the row phases in fixed order
  for (int cg0 = 0; cg0 < (a.C >> 2); cg0 += 256) {
    GnMap mp(a, cg0);
    double cs[4] = {0.0, 0.0, 0.0, 0.0};
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
              const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + e));
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
          // (dx null: the producing conv, dx's only consumer, reads the split / packed copy alone -- uniform)
          if (dx != nullptr) *(float4*)(op + (long long)r * a.C) = float4{o[0], o[1], o[2], o[3]};
          if (a.dxp != nullptr) {
            if (a.dxp_split)
              ((uint4*)a.dxp)[off >> 2] = split4_bf16(float4{o[0], o[1], o[2], o[3]});
            else
              a.dxp[off >> 2] = uint2{pk_bf16x2(o[0], o[1]), pk_bf16x2(o[2], o[3])};
          }
          if (a.csp != nullptr) {  // (uniform) the producing conv's bias gradient
            cs[0] += o[0]; cs[1] += o[1]; cs[2] += o[2]; cs[3] += o[3];
          }
        }
      }
    }
    if (a.csp != nullptr) {  // (uniform) one partial row per (sample, chunk): the row phases summed in order
      const int tid = threadIdx.x;
#pragma unroll
      for (int e = 0; e < 4; ++e) csr[tid][e] = cs[e];
      __syncthreads();
      if (mp.act && mp.rph == 0) {
        double t[4] = {0.0, 0.0, 0.0, 0.0};
        const int C4l = (a.C >> 2) >= 256 ? 256 : (a.C >> 2);
        for (int q = 0; q < mp.rpar; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] += csr[q * C4l + (tid % C4l)][e];
        double* o = a.csp + ((long long)b * gridDim.x + blockIdx.x) * a.C + mp.c4 * 4;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = t[e];
      }
      __syncthreads();
    }
    if ((a.C >> 2) < 256) break;
  }
}

// out[c] = beta * out[c] + sum over nparts partial rows: the bias gradient from the column-sum partials. A block owns 16
// columns; its 16 partial slices (thread (slice, column)) each sum partials slice, slice + 16, ... in order, then the
// slices are added in slice order (fixed order: deterministic; 128-B coalesced rows instead of one serial column walk)
__global__ void __launch_bounds__(256) gn_colsum_final_kernel(const double* __restrict__ part, int nparts, int C,
                                                              float* __restrict__ out, float beta) {
  __shared__ double red[16][17];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s = 0.0;
  if (c < C) {
    int q = sl;
    for (; q + 48 < nparts; q += 64) {  // 4 partial loads in flight, summed in order
      const double v0 = part[(long long)q * C + c], v1 = part[(long long)(q + 16) * C + c];
      const double v2 = part[(long long)(q + 32) * C + c], v3 = part[(long long)(q + 48) * C + c];
      s += v0; s += v1; s += v2; s += v3;
    }
    for (; q < nparts; q += 16) s += part[(long long)q * C + c];
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    out[c] = (beta != 0.f ? beta * out[c] : 0.f) + (float)t;
  }
}

// ------------------------------------------------------------------------------------------
// Resident GroupNorm for small per-sample tensors (the 28x28 / 14x14 / 7x7 levels of c2 / c3, where the
// producing conv cannot emit the statistics: h*w % 32 != 0). The work is cut into UNITS = (sample b, slab of
// SC channels = whole groups); a unit is held in registers (IT float4 per thread), so x is read from HBM ONCE
// per pass: forward = statistics (two-pass: mean, then centred variance, on the resident values) + apply in
// one launch (8 B/elem); backward = partial sums + finalize + dx in one launch (12 B/elem, +4 with the
// residual-branch add) plus a per-channel parameter-gradient reduction.
// Persistent workgroups walk units u = blockIdx.x, + gridDim.x, ... with a one-unit-deep register prefetch:
// the next unit's loads are in flight while this unit reduces and stores, so the read and write phases of
// consecutive units overlap (a one-shot grid would serialize them chip-wide).
// Cross-thread sums: a fixed wave butterfly, then a fixed-order LDS combine -- bitwise reproducible.
// Thread map: C4 = SC/4 (a power of two <= NT) channel quads, rpar = NT / C4 row phases; thread (rph, c4)
// walks rows rph, rph + rpar, ... (at most IT of them).
// ------------------------------------------------------------------------------------------
constexpr int GN_RES_NT = 512;
static int g_gn_path = -1;  // mvae_set_group_norm_path: 0 auto, 1 streaming only (-1: not yet read from the env)
constexpr int GN_RES_MAXC = 2048;  // slab channels (C4 <= GN_RES_NT)

template <int K>
__device__ __forceinline__ void gn_slab_reduce(float (&s)[K], int C4, float* red /*[K][NT]*/, float* out /*[C4][K]*/) {
  const int tid = threadIdx.x;
  if (C4 < 64) {
    for (int m = C4; m < 64; m <<= 1) {  // lanes with the same c4 differ by multiples of C4
#pragma unroll
      for (int k = 0; k < K; ++k) s[k] += __shfl_xor(s[k], m, 64);
    }
  }
#pragma unroll
  for (int k = 0; k < K; ++k) red[k * GN_RES_NT + tid] = s[k];
  __syncthreads();
  if (tid < C4) {
    const int stride = C4 < 64 ? 64 : C4;  // one representative per (wave, c4)
    float t[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = 0.f;
    for (int j = tid; j < GN_RES_NT; j += stride)
#pragma unroll
      for (int k = 0; k < K; ++k) t[k] += red[k * GN_RES_NT + j];
#pragma unroll
    for (int k = 0; k < K; ++k) out[tid * K + k] = t[k];
  }
  __syncthreads();
}

// Unit geometry (uniform across the workgroup). Every access of a unit goes through a buffer descriptor based
// at (b, row 0, channel c0) whose range ends at the sample's end: the thread's lane offset is one VGPR and the
// row step i*rpar*C*4 an SGPR, and rows past hw fall outside the range (loads read 0, stores are dropped).
typedef __attribute__((ext_vector_type(4))) unsigned gn_u32x4;
struct GnUnit {
  int b, c0;
  long long ubase;  // element offset of (b, row 0, channel c0)
  unsigned bytes;   // descriptor range: from ubase to the end of sample b
  __device__ GnUnit(const GnArgs& a, int SC, int u) {
    const int nsl = a.C / SC;
    b = u / nsl;
    c0 = (u - b * nsl) * SC;
    ubase = (long long)b * a.hw * a.C + c0;
    bytes = (unsigned)(((long long)a.hw * a.C - c0) * 4);
  }
  __device__ __amdgpu_buffer_rsrc_t rsrc(const float* p) const {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p + ubase), (short)0, (int)bytes, 0x00020000);
  }
};

template <int IT>
__device__ __forceinline__ void gn_res_load(const float* p, const GnArgs& a, int SC, int u, unsigned vo, int rstep,
                                            bool on, float4 (&v)[IT]) {
  if (!on) {  // uniform
#pragma unroll
    for (int i = 0; i < IT; ++i) v[i] = float4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const __amdgpu_buffer_rsrc_t r = GnUnit(a, SC, u).rsrc(p);
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const gn_u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(r, vo, i * rstep, 0);
    v[i] = float4{__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z), __uint_as_float(t.w)};
  }
}
// Stores take the row step in the VGPR offset with soffset = 0: gfx950 has the "VALU overwrites the data VGPRs
// of a just-issued >8-byte VMEM store" hazard also for buffer stores with an SGPR soffset, which the compiler
// does not guard (it inserts the wait state only without an SGPR soffset). Measured: with the row step in
// soffset, a few % of the dx stores of this kernel landed corrupted (tools/gn_stress.py, 14 of 80 runs).
__device__ __forceinline__ void gn_res_store(__amdgpu_buffer_rsrc_t r, unsigned off, gn_u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}
__device__ __forceinline__ gn_u32x4 gn_bits(float4 v) {
  return gn_u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
}

struct GnFwdSmem {
  float red[4 * GN_RES_NT];
  float chs[GN_RES_MAXC];
  float gmu[GN_RES_MAXC], grs[GN_RES_MAXC];  // per slab channel: its group's mean / rstd
};

template <int IT>
__device__ __forceinline__ void gn_fwd_unit(const GnArgs& a, int SC, int u, const float4 (&v)[IT], GnFwdSmem& sm,
                                            float* __restrict__ y, float* __restrict__ mean, float* __restrict__ rstd,
                                            float eps) {
  const int tid = threadIdx.x;
  const int C4 = SC >> 2, rpar = GN_RES_NT / C4, c4 = tid & (C4 - 1), rph = tid / C4;
  const int cpg = a.C / a.G, ngl = SC / cpg;
  const double n = (double)a.hw * cpg;
  const GnUnit un(a, SC, u);
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    s[0] += v[i].x; s[1] += v[i].y; s[2] += v[i].z; s[3] += v[i].w;
  }
  gn_slab_reduce<4>(s, C4, sm.red, sm.chs);
  for (int gl = tid; gl < ngl; gl += GN_RES_NT) {
    float t = 0.f;
    for (int j = 0; j < cpg; ++j) t += sm.chs[gl * cpg + j];
    const float mu = (float)((double)t / n);
    for (int j = 0; j < cpg; ++j) sm.gmu[gl * cpg + j] = mu;
  }
  __syncthreads();
  float mu[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    mu[e] = sm.gmu[c4 * 4 + e];
    s[e] = 0.f;
  }
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    if (rph + i * rpar < a.hw) {
      const float d0 = v[i].x - mu[0], d1 = v[i].y - mu[1], d2 = v[i].z - mu[2], d3 = v[i].w - mu[3];
      s[0] = fmaf(d0, d0, s[0]); s[1] = fmaf(d1, d1, s[1]); s[2] = fmaf(d2, d2, s[2]); s[3] = fmaf(d3, d3, s[3]);
    }
  }
  gn_slab_reduce<4>(s, C4, sm.red, sm.chs);
  for (int gl = tid; gl < ngl; gl += GN_RES_NT) {
    float t = 0.f;
    for (int j = 0; j < cpg; ++j) t += sm.chs[gl * cpg + j];
    const float rs = (float)(1.0 / sqrt((double)t / n + (double)eps));
    for (int j = 0; j < cpg; ++j) sm.grs[gl * cpg + j] = rs;
    const int gi = un.b * a.G + un.c0 / cpg + gl;
    mean[gi] = sm.gmu[gl * cpg];
    rstd[gi] = rs;
  }
  __syncthreads();
  float sc[4], sh[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = un.c0 + c4 * 4 + e;
    sc[e] = sm.grs[c4 * 4 + e] * a.gamma[c];
    sh[e] = a.beta[c] - mu[e] * sc[e];
  }
  const __amdgpu_buffer_rsrc_t yr = un.rsrc(y);
  const __amdgpu_buffer_rsrc_t ybr =
      __builtin_amdgcn_make_buffer_rsrc((void*)((__bf16*)y + un.ubase), (short)0, (int)(un.bytes >> 1), 0x00020000);
  const __amdgpu_buffer_rsrc_t ylr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)((__bf16*)y + (long long)a.nb * a.hw * a.C + un.ubase), (short)0, (int)(un.bytes >> 1), 0x00020000);
  const unsigned vo = (unsigned)(rph * a.C + c4 * 4) * 4u;
  const int rstep = rpar * a.C * 4;
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    float o[4] = {v[i].x * sc[0] + sh[0], v[i].y * sc[1] + sh[1], v[i].z * sc[2] + sh[2], v[i].w * sc[3] + sh[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (a.silu) o[k] = o[k] * sigmoid_f(o[k]);
      if (a.drop_p > 0.f) {
        const long long off = un.ubase + (long long)(rph + i * rpar) * a.C + c4 * 4;
        const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + k));
        o[k] = (uu >= a.drop_p) ? o[k] / (1.f - a.drop_p) : 0.f;
      }
    }
    const float4 ov{o[0], o[1], o[2], o[3]};
    if (a.y_split >= 2) {  // packed bf16 / planar hi plane: half the byte offsets, 8-B stores (rows past hw: dropped)
      typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
      const unsigned h01 = pk_bf16x2(ov.x, ov.y), h23 = pk_bf16x2(ov.z, ov.w);
      const unsigned o2 = (vo >> 1) + (unsigned)(i * (rstep >> 1));
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{h01, h23}, ybr, o2, 0, 0);
      if (a.y_split == 3)  // lo plane
        __builtin_amdgcn_raw_buffer_store_b64(
            u32x2{pk_bf16x2(ov.x - __uint_as_float(h01 << 16), ov.y - __uint_as_float(h01 & 0xFFFF0000u)),
                  pk_bf16x2(ov.z - __uint_as_float(h23 << 16), ov.w - __uint_as_float(h23 & 0xFFFF0000u))},
            ylr, o2, 0, 0);
      continue;
    }
    const uint4 sp = a.y_split ? split4_bf16(ov) : uint4{0u, 0u, 0u, 0u};
    gn_res_store(yr, vo + (unsigned)(i * rstep), a.y_split ? gn_u32x4{sp.x, sp.y, sp.z, sp.w} : gn_bits(ov));  // rows past hw: dropped
  }
}

template <int IT>
__global__ void __launch_bounds__(GN_RES_NT) gn_fwd_resident_kernel(GnArgs a, int SC, int units, float* __restrict__ y,
                                                                    float* __restrict__ mean, float* __restrict__ rstd,
                                                                    float eps) {
  __shared__ GnFwdSmem sm;
  const int C4 = SC >> 2, rpar = GN_RES_NT / C4, c4 = threadIdx.x & (C4 - 1), rph = threadIdx.x / C4;
  const int G = gridDim.x;
  const unsigned vo = (unsigned)(rph * a.C + c4 * 4) * 4u;
  const int rstep = rpar * a.C * 4;
  float4 va[IT], vb[IT];
  int u = blockIdx.x;
  gn_res_load<IT>(a.x, a, SC, u, vo, rstep, u < units, va);
  while (u < units) {  // ping-pong: the next unit's loads fly while this one reduces and stores
    gn_res_load<IT>(a.x, a, SC, u + G, vo, rstep, u + G < units, vb);
    gn_fwd_unit<IT>(a, SC, u, va, sm, y, mean, rstd, eps);
    u += G;
    if (u >= units) break;
    gn_res_load<IT>(a.x, a, SC, u + G, vo, rstep, u + G < units, va);
    gn_fwd_unit<IT>(a, SC, u, vb, sm, y, mean, rstd, eps);
    u += G;
  }
}

struct GnBwdSmem {
  float red[8 * GN_RES_NT];
  float chs[GN_RES_MAXC * 2];
  float gk2[GN_RES_MAXC], gk3[GN_RES_MAXC];
};

// backward of one unit; pws = [2][C][nb] fp64 per-sample channel sums {sum dyn, sum dyn*xhat}
template <int IT>
__device__ __forceinline__ void gn_bwd_unit(const GnArgs& a, int SC, int u, const float4 (&xv)[IT], float4 (&dv)[IT],
                                            GnBwdSmem& sm, double* __restrict__ pws, float* __restrict__ dx) {
  const int tid = threadIdx.x;
  const int C4 = SC >> 2, rpar = GN_RES_NT / C4, c4 = tid & (C4 - 1), rph = tid / C4;
  const int cpg = a.C / a.G, ngl = SC / cpg;
  const GnUnit un(a, SC, u);
  const unsigned vo = (unsigned)(rph * a.C + c4 * 4) * 4u;
  const int rstep = rpar * a.C * 4;
  float m[4], rs[4], gm[4], bt[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int c = un.c0 + c4 * 4 + e, bg = un.b * a.G + c / cpg;
    m[e] = a.mean[bg];
    rs[e] = a.rstd[bg];
    gm[e] = a.gamma[c];
    bt[e] = a.beta[c];
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const long long off = un.ubase + (long long)(rph + i * rpar) * a.C + c4 * 4;
    const float xs[4] = {xv[i].x, xv[i].y, xv[i].z, xv[i].w};
    float ds[4] = {dv[i].x, dv[i].y, dv[i].z, dv[i].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = ds[e];  // rows past hw hold d = 0: they add nothing
      if (a.drop_p > 0.f) {
        const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + e));
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
    dv[i] = float4{ds[0], ds[1], ds[2], ds[3]};  // now the gradient at the normalized output (dropout / SiLU)
  }
  // chs[(c4*8) + k]: k 0-3 = sum dyn of channels c4*4+k, k 4-7 = sum dyn*xhat
  gn_slab_reduce<8>(s, C4, sm.red, sm.chs);
  for (int t = tid; t < SC; t += GN_RES_NT) {
    const int q = t >> 2, e = t & 3, c = un.c0 + t;
    pws[(long long)c * a.nb + un.b] = sm.chs[q * 8 + e];
    pws[((long long)a.C + c) * a.nb + un.b] = sm.chs[q * 8 + 4 + e];
  }
  for (int gl = tid; gl < ngl; gl += GN_RES_NT) {
    double A1 = 0.0, A2 = 0.0;
    for (int j = 0; j < cpg; ++j) {
      const int cl = gl * cpg + j;
      const double g = a.gamma[un.c0 + cl];
      A1 += g * sm.chs[(cl >> 2) * 8 + (cl & 3)];
      A2 += g * sm.chs[(cl >> 2) * 8 + 4 + (cl & 3)];
    }
    const int gi = un.b * a.G + un.c0 / cpg + gl;
    const double n = (double)a.hw * cpg, r = a.rstd[gi], mu = a.mean[gi];
    const float k2 = (float)(-r * r * A2 / n), k3 = (float)(-r * A1 / n + mu * r * r * A2 / n);
    for (int j = 0; j < cpg; ++j) {
      sm.gk2[gl * cpg + j] = k2;
      sm.gk3[gl * cpg + j] = k3;
    }
  }
  // the residual branch's gradient: loaded here, its latency behind the finalize barrier (IT = 16: in batches of 4
  // rows in the store loop -- 16 more rows would not fit the registers)
  constexpr int AV = IT > 8 ? 4 : IT;
  float4 av[AV];
  if constexpr (IT <= 8) gn_res_load<IT>(a.dx_add, a, SC, u, vo, rstep, a.dx_add != nullptr, av);
  __syncthreads();
  float q1[4], q2[4], q3[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    q1[e] = rs[e] * gm[e];
    q2[e] = sm.gk2[c4 * 4 + e];
    q3[e] = sm.gk3[c4 * 4 + e];
  }
  // (dx null: an empty range, the fp32 stores are dropped -- the conv reads the split / packed copy alone)
  const __amdgpu_buffer_rsrc_t dr = dx ? un.rsrc(dx) : __builtin_amdgcn_make_buffer_rsrc(nullptr, (short)0, 0, 0x00020000);
  const __amdgpu_buffer_rsrc_t pr = a.dxp_split  // split4: fp32 offsets; packed bf16: half of them
      ? __builtin_amdgcn_make_buffer_rsrc((void*)((float*)a.dxp + un.ubase), (short)0, (int)un.bytes, 0x00020000)
      : __builtin_amdgcn_make_buffer_rsrc((void*)((__bf16*)a.dxp + un.ubase), (short)0, (int)(un.bytes >> 1), 0x00020000);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t ar = un.rsrc(a.dx_add);
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    if constexpr (IT > 8) {
      if (i % AV == 0) {
#pragma unroll
        for (int j = 0; j < AV; ++j) {
          if (a.dx_add != nullptr) {
            const gn_u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(ar, vo, (i + j) * rstep, 0);
            av[j] = float4{__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z), __uint_as_float(t.w)};
          } else {
            av[j] = float4{0.f, 0.f, 0.f, 0.f};
          }
        }
      }
    }
    const float4 w = av[i % AV];
    // av is zero when there is no residual-branch gradient; rows past hw: the store is dropped
    const float4 o{dv[i].x * q1[0] + xv[i].x * q2[0] + q3[0] + w.x, dv[i].y * q1[1] + xv[i].y * q2[1] + q3[1] + w.y,
                   dv[i].z * q1[2] + xv[i].z * q2[2] + q3[2] + w.z, dv[i].w * q1[3] + xv[i].w * q2[3] + q3[3] + w.w};
    gn_res_store(dr, vo + (unsigned)(i * rstep), gn_bits(o));
    if (a.dxp != nullptr) {  // packed bf16 at half the byte offsets (8-B stores) or split4 at the fp32 offsets (16-B
      typedef __attribute__((ext_vector_type(2))) unsigned u32x2;  // stores); rows past hw: dropped
      if (a.dxp_split) {
        const uint4 q = split4_bf16(o);
        gn_res_store(pr, vo + (unsigned)(i * rstep), gn_u32x4{q.x, q.y, q.z, q.w});
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{pk_bf16x2(o.x, o.y), pk_bf16x2(o.z, o.w)}, pr,
                                              (vo >> 1) + (unsigned)(i * (rstep >> 1)), 0, 0);
      }
    }
    if (a.csp != nullptr && rph + i * rpar < a.hw) {  // (uniform) the producing conv's bias gradient
      cs[0] += o.x; cs[1] += o.y; cs[2] += o.z; cs[3] += o.w;
    }
  }
  if (a.csp != nullptr) {  // (uniform) per-unit column sums -> csp[b][c0 .. c0 + SC)
    gn_slab_reduce<4>(cs, C4, sm.red, sm.chs);
    for (int t = tid; t < SC; t += GN_RES_NT) a.csp[(long long)un.b * a.C + un.c0 + t] = (double)sm.chs[t];
  }
}

// IT = 13 (a whole 128-B row segment per unit at the 28x28 levels' 32-channel slabs): no next-unit prefetch -- its
// registers would not fit
template <int IT>
__global__ void __launch_bounds__(GN_RES_NT) gn_bwd_resident_kernel(GnArgs a, int SC, int units, double* __restrict__ pws,
                                                                    float* __restrict__ dx) {
  __shared__ GnBwdSmem sm;
  const int C4 = SC >> 2, rpar = GN_RES_NT / C4, c4 = threadIdx.x & (C4 - 1), rph = threadIdx.x / C4;
  const int G = gridDim.x;
  const unsigned vo = (unsigned)(rph * a.C + c4 * 4) * 4u;
  const int rstep = rpar * a.C * 4;
  int u = blockIdx.x;
  if constexpr (IT > 8) {
    float4 xa[IT], da[IT];
    for (; u < units; u += G) {
      gn_res_load<IT>(a.x, a, SC, u, vo, rstep, true, xa);
      gn_res_load<IT>(a.dy, a, SC, u, vo, rstep, true, da);
      gn_bwd_unit<IT>(a, SC, u, xa, da, sm, pws, dx);
    }
    return;
  }
  float4 xa[IT], da[IT], xb[IT], db[IT];
  gn_res_load<IT>(a.x, a, SC, u, vo, rstep, u < units, xa);
  gn_res_load<IT>(a.dy, a, SC, u, vo, rstep, u < units, da);
  while (u < units) {  // ping-pong prefetch of x and dy, as in the forward
    gn_res_load<IT>(a.x, a, SC, u + G, vo, rstep, u + G < units, xb);
    gn_res_load<IT>(a.dy, a, SC, u + G, vo, rstep, u + G < units, db);
    gn_bwd_unit<IT>(a, SC, u, xa, da, sm, pws, dx);
    u += G;
    if (u >= units) break;
    gn_res_load<IT>(a.x, a, SC, u + G, vo, rstep, u + G < units, xa);
    gn_res_load<IT>(a.dy, a, SC, u + G, vo, rstep, u + G < units, da);
    gn_bwd_unit<IT>(a, SC, u, xb, db, sm, pws, dx);
    u += G;
  }
}

// Backward of a large per-sample tensor (c4's 64x64 / 32x32 levels) as units too: a workgroup owns
// (sample, slab of whole groups) and streams it TWICE -- pass 1 (temporal loads) accumulates the partial sums,
// the finalize runs in the workgroup, pass 2 re-reads x and dy (non-temporal, last use) and writes dx. With one
// workgroup per CU the units in flight (256 x <= 128 KB) stay cached between the passes, so HBM sees x and dy
// once (16 B/elem with the residual add) instead of the streaming chain's 24.
template <int U>
__global__ void __launch_bounds__(GN_RES_NT) gn_bwd_unit2_kernel(GnArgs a, int SC, int units, double* __restrict__ pws,
                                                                 float* __restrict__ dx) {
  __shared__ GnBwdSmem sm;
  const int tid = threadIdx.x;
  const int C4 = SC >> 2, rpar = GN_RES_NT / C4, c4 = tid & (C4 - 1), rph = tid / C4;
  const int cpg = a.C / a.G, ngl = SC / cpg;
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const GnUnit un(a, SC, u);
    const long long tb = un.ubase + c4 * 4;  // this thread's channel quad, row 0
    float m[4], rs[4], gm[4], bt[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = un.c0 + c4 * 4 + e, bg = un.b * a.G + c / cpg;
      m[e] = a.mean[bg];
      rs[e] = a.rstd[bg];
      gm[e] = a.gamma[c];
      bt[e] = a.beta[c];
    }
    auto dyn = [&](float4 xv, float4 dv, long long off, float (&d)[4], float (&xh)[4]) {
      const float xs[4] = {xv.x, xv.y, xv.z, xv.w};
      const float ds[4] = {dv.x, dv.y, dv.z, dv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float g = ds[e];
        if (a.drop_p > 0.f) {
          const float uu = hash_uniform(drop_seed(a), (unsigned long long)(off + e));
          g = (uu >= a.drop_p) ? g / (1.f - a.drop_p) : 0.f;
        }
        xh[e] = (xs[e] - m[e]) * rs[e];
        if (a.silu) {
          const float yn = xh[e] * gm[e] + bt[e];
          const float sg = sigmoid_f(yn);
          g = g * sg * (1.f + yn * (1.f - sg));
        }
        d[e] = g;
      }
    };
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r0 = rph; r0 < a.hw; r0 += U * rpar) {  // pass 1: partial sums (loads keep the lines cached)
      float4 xv[U], dv[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int r = r0 + q * rpar;
        const bool ok = r < a.hw;
        xv[q] = ok ? *(const float4*)(a.x + tb + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
        dv[q] = ok ? *(const float4*)(a.dy + tb + (long long)r * a.C) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        float d[4], xh[4];
        dyn(xv[q], dv[q], tb + (long long)(r0 + q * rpar) * a.C, d, xh);  // rows past hw: dv = 0 -> d = 0
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[e] += d[e];
          s[4 + e] = fmaf(d[e], xh[e], s[4 + e]);
        }
      }
    }
    gn_slab_reduce<8>(s, C4, sm.red, sm.chs);
    for (int t = tid; t < SC; t += GN_RES_NT) {
      const int q = t >> 2, e = t & 3, c = un.c0 + t;
      pws[(long long)c * a.nb + un.b] = sm.chs[q * 8 + e];
      pws[((long long)a.C + c) * a.nb + un.b] = sm.chs[q * 8 + 4 + e];
    }
    for (int gl = tid; gl < ngl; gl += GN_RES_NT) {
      double A1 = 0.0, A2 = 0.0;
      for (int j = 0; j < cpg; ++j) {
        const int cl = gl * cpg + j;
        const double g = a.gamma[un.c0 + cl];
        A1 += g * sm.chs[(cl >> 2) * 8 + (cl & 3)];
        A2 += g * sm.chs[(cl >> 2) * 8 + 4 + (cl & 3)];
      }
      const int gi = un.b * a.G + un.c0 / cpg + gl;
      const double n = (double)a.hw * cpg, r = a.rstd[gi], mu = a.mean[gi];
      const float k2 = (float)(-r * r * A2 / n), k3 = (float)(-r * A1 / n + mu * r * r * A2 / n);
      for (int j = 0; j < cpg; ++j) {
        sm.gk2[gl * cpg + j] = k2;
        sm.gk3[gl * cpg + j] = k3;
      }
    }
    __syncthreads();
    float q1[4], q2[4], q3[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q1[e] = rs[e] * gm[e];
      q2[e] = sm.gk2[c4 * 4 + e];
      q3[e] = sm.gk3[c4 * 4 + e];
    }
    __syncthreads();  // gk2 / gk3 are rewritten by the next unit
    const bool add = a.dx_add != nullptr;
    for (int r0 = rph; r0 < a.hw; r0 += U * rpar) {  // pass 2: dx (last use of x and dy: non-temporal)
      float4 xv[U], dv[U], av[U];
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int r = r0 + q * rpar;
        const bool ok = r < a.hw;
        const long long off = tb + (long long)r * a.C;
        xv[q] = ok ? gn_ld4(a.x + off) : float4{0.f, 0.f, 0.f, 0.f};
        dv[q] = ok ? gn_ld4(a.dy + off) : float4{0.f, 0.f, 0.f, 0.f};
        av[q] = (add && ok) ? gn_ld4(a.dx_add + off) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int q = 0; q < U; ++q) {
        const int r = r0 + q * rpar;
        if (r >= a.hw) continue;
        const long long off = tb + (long long)r * a.C;
        float d[4], xh[4];
        dyn(xv[q], dv[q], off, d, xh);
        const float xs[4] = {xv[q].x, xv[q].y, xv[q].z, xv[q].w};
        *(float4*)(dx + off) = float4{d[0] * q1[0] + xs[0] * q2[0] + q3[0] + av[q].x,
                                      d[1] * q1[1] + xs[1] * q2[1] + q3[1] + av[q].y,
                                      d[2] * q1[2] + xs[2] * q2[2] + q3[2] + av[q].z,
                                      d[3] * q1[3] + xs[3] * q2[3] + q3[3] + av[q].w};
      }
    }
  }
}

// slab of the two-pass unit backward: >= 16 channels (64-B row segments), whole groups, <= 128 KB of x + dy
// per unit. Opt-in (MVAE_GN_UNIT=1): whether the second pass hits in cache is not stable -- c4's 32x32x512
// level measured 533 us in one run and 1068 us in another against the streaming chain's 600 (512-KB units at
// 64x64: 1.9x slower every time).
static int gn_unit2_slab(int hw, int C, int G) {
  static const bool off = [] {  // opt-in: MVAE_GN_UNIT=1
    const char* e = getenv("MVAE_GN_UNIT");
    return e == nullptr || e[0] != '1';
  }();
  if (off || g_gn_path == 1 || C % G) return 0;
  const int cpg = C / G;
  for (int sc = 64; sc >= 16; sc >>= 1) {
    if (C % sc || sc % cpg) continue;
    if ((long long)hw * sc * 8 <= (128LL << 10)) return sc;
  }
  return 0;
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

// Slab width for the resident path (0: not eligible). Path selection: mvae_set_group_norm_path (0 auto,
// 1 streaming only); before any call, MVAE_GN_RESIDENT=0 selects streaming only.
// Largest slab (of >= 16 channels: 64-B row segments) with <= max_it rows per thread (forward 16: one 128-B
// row segment per 8 lanes at the 28x28x32 level, 41 -> 33 us; backward 8: two units of x and dy in registers).
static bool gn_fwd_it13() {
  static const int v = getenv("MVAE_GN_FWD_IT16") == nullptr;  // experiment knob: the forward's 28x28 levels on 16 rows
  return v != 0;
}
static int gn_resident_slab(int nb, int hw, int C, int G, int* items, int max_it) {
  if (g_gn_path < 0) {
    const char* e = getenv("MVAE_GN_RESIDENT");
    g_gn_path = (e != nullptr && e[0] == '0') ? 1 : 0;
  }
  if (g_gn_path == 1 || C % G) return 0;
  const int cpg = C / G;
  for (int sc = std::min(C, GN_RES_MAXC); sc >= 16; sc >>= 1) {
    const int c4 = sc >> 2;
    if ((c4 & (c4 - 1)) || c4 > GN_RES_NT || C % sc || sc % cpg) continue;
    const int rpar = GN_RES_NT / c4, it = (hw + rpar - 1) / rpar;
    if (it > max_it) continue;
    *items = it <= 4 ? 4 : it <= 8 ? 8 : (it <= 13 && (max_it < 16 || gn_fwd_it13())) ? 13 : 16;  // 13: 28x28 at 32-ch slabs
    return sc;
  }
  return 0;
}

// persistent grid: as many workgroups as fit on the chip at once (occupancy query, cached per kernel/device)
static int gn_res_grid(const void* kernel, int units) {
  struct Entry { const void* k; int dev, slots; };
  static Entry cache[16];
  static int n_cache = 0;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int slots = 0;
  for (int i = 0; i < n_cache; ++i)
    if (cache[i].k == kernel && cache[i].dev == dev) slots = cache[i].slots;
  if (slots == 0) {
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, GN_RES_NT, 0);
    slots = std::max(1, cus) * std::max(1, per_cu);
    if (n_cache < 16) cache[n_cache++] = Entry{kernel, dev, slots};
  }
  // experiment knob: MVAE_GN_RES_GRID = k > 0: k x the resident slots; 0: one workgroup per unit (no persistence)
  if (const char* e = getenv("MVAE_GN_RES_GRID")) {
    const int k = atoi(e);
    return k <= 0 ? units : std::max(1, std::min(units, slots * k));
  }
  return std::max(1, std::min(units, slots));
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
  static const int fwd_max_it = [] {
    const char* e = getenv("MVAE_GN_RES_FWD_IT");  // experiment knob: rows per thread allowed in the forward
    return e ? atoi(e) : 16;
  }();
  if (const int sc = gn_resident_slab(nb, hw, c, groups, &it, fwd_max_it)) {
    a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split; a.salt = dropout_salt();
    const int units = nb * (c / sc);
    const void* k = it == 4 ? (const void*)gn_fwd_resident_kernel<4>
                  : it == 8 ? (const void*)gn_fwd_resident_kernel<8>
                  : it == 13 ? (const void*)gn_fwd_resident_kernel<13> : (const void*)gn_fwd_resident_kernel<16>;
    const dim3 grid(gn_res_grid(k, units));
    if (it == 4) hipLaunchKernelGGL(gn_fwd_resident_kernel<4>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, y, mean, rstd, eps);
    else if (it == 8) hipLaunchKernelGGL(gn_fwd_resident_kernel<8>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, y, mean, rstd, eps);
    else if (it == 13) hipLaunchKernelGGL(gn_fwd_resident_kernel<13>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, y, mean, rstd, eps);
    else hipLaunchKernelGGL(gn_fwd_resident_kernel<16>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, y, mean, rstd, eps);
    return launch_status();
  }
  float* scale = (float*)((char*)workspace + (size_t)nb * a.chunks * c * 2 * sizeof(double));
  float* shift = scale + (size_t)nb * c;
  hipLaunchKernelGGL(gn_partial_kernel<0>, dim3(a.chunks, nb), dim3(256), 0, st, a);
  hipLaunchKernelGGL(gn_stats_finalize_kernel, dim3(cdiv((long long)nb * groups, 4)), dim3(256), 0, st, a,
                     mean, rstd, scale, shift, eps);
  a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split; a.salt = dropout_salt();
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
  a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.y_split = y_split; a.salt = dropout_salt();
  hipLaunchKernelGGL(gn_apply_kernel, dim3(a.chunks, nb), dim3(256), 0, st, a, scale, shift, y);
  return launch_status();
}

// Statistics only (the consumer applies the normalization itself: the Winograd input transform of the following conv,
// mvae_winograd_input_transform_gn): mean / rstd [nb * groups] and the per-(sample, channel) affine of the apply,
// scale = rstd * gamma, shift = beta - mean * scale ([nb][c] fp32 each, the bytes gn_apply uses). part (nullable): the
// producing conv's epilogue statistics (mvae_conv2d_gnstats_nhwc layout; hw % 32 == 0, channels per group % 4 == 0);
// without it one fp64 partial pass over x.
int mvae_group_norm_stats_nhwc(const float* x, const double* part, const float* gamma, const float* beta, float* mean,
                               float* rstd, float* scale, float* shift, int nb, int hw, int c, int groups, float eps,
                               void* workspace, size_t workspace_bytes, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups || !scale || !shift || !mean || !rstd ||
      (part && ((c / groups) % 4 || hw % 32))) {
    set_error("group_norm_stats: C %% 4 == 0 and %% groups (with part: hw %% 32 == 0, channels per group %% 4 == 0)");
    return MVAE_EINVAL;
  }
  if (!part && workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_stats: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.gamma = gamma; a.beta = beta; a.nb = nb; a.hw = hw; a.C = c; a.G = groups;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.ws = (double*)workspace;
  const dim3 fg(cdiv((long long)nb * groups, 4));
  if (part) {
    hipLaunchKernelGGL(gn_stats_finalize_part_kernel, fg, dim3(256), 0, st, a, part, mean, rstd, scale, shift, eps);
  } else {
    hipLaunchKernelGGL(gn_partial_kernel<0>, dim3(a.chunks, nb), dim3(256), 0, st, a);
    hipLaunchKernelGGL(gn_stats_finalize_kernel, fg, dim3(256), 0, st, a, mean, rstd, scale, shift, eps);
  }
  return launch_status();
}

// y = silu?(x * scale + shift) from mvae_group_norm_stats_nhwc's affine (y_split as mvae_group_norm_fwd_nhwc; no
// dropout): the normalization a deferred GroupNorm output needs when its consumer cannot apply it itself
int mvae_group_norm_apply_nhwc(const float* x, const float* scale, const float* shift, float* y, int nb, int hw, int c,
                               int silu, int y_split, void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || !x || !scale || !shift || !y) {
    set_error("group_norm_apply: C %% 4 == 0");
    return MVAE_EINVAL;
  }
  GnArgs a{};
  a.x = x; a.nb = nb; a.hw = hw; a.C = c; a.G = 1;
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.silu = silu; a.drop_p = 0.f; a.y_split = y_split; a.salt = dropout_salt();
  hipLaunchKernelGGL(gn_apply_kernel, dim3(a.chunks, nb), dim3(256), 0, (hipStream_t)stream, a, scale, shift, y);
  return launch_status();
}

// dx = d/dx of the fused forward [+ dx_add when non-null]; dgamma/dbeta are ACCUMULATED (+=) when non-null.
// pack (non-null dxp): also dxp = packed bf16 of dx and dbias = bias_beta * dbias + column sums of dx (the consuming
// conv's bf16 output gradient and bias gradient; partials in cs_ws)
static int gn_bwd(const float* x, const float* dy, const float* gamma, const float* beta, const float* mean,
                  const float* rstd, float* dx, const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c,
                  int groups, int silu, float drop_p, unsigned long long seed, void* workspace, size_t workspace_bytes,
                  void* dxp, float* dbias, float bias_beta, void* cs_ws, void* stream, int dxp_split = 0);
int mvae_group_norm_bwd_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                             const float* mean, const float* rstd, float* dx, const float* dx_add,
                             float* dgamma, float* dbeta,
                             int nb, int hw, int c, int groups, int silu, float drop_p,
                             unsigned long long seed, void* workspace, size_t workspace_bytes, void* stream) {
  return gn_bwd(x, dy, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu, drop_p, seed,
                workspace, workspace_bytes, nullptr, nullptr, 0.f, nullptr, stream);
}

// column-sum partials of mvae_group_norm_bwd_pack_nhwc: [nb * chunks][C] fp64 (streaming) or [nb][C] (resident)
size_t mvae_group_norm_colsum_workspace_bytes(int nb, int hw, int c) {
  return (size_t)nb * std::max(1, gn_chunks(nb, hw)) * c * sizeof(double);
}

int mvae_group_norm_bwd_pack_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                  const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                  float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                  unsigned long long seed, void* workspace, size_t workspace_bytes, void* dx_packed,
                                  float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                  void* stream) {
  if (dx_packed == nullptr || ((uintptr_t)dx_packed & 7) || ((uintptr_t)dx & 15) || ((uintptr_t)x & 15) ||
      ((uintptr_t)dy & 15) || (dx_add && ((uintptr_t)dx_add & 15)) || (dbias && cs_workspace == nullptr)) {
    set_error("group_norm_bwd_pack: 16-B aligned x / dy / dx, 8-B aligned packed output, a column-sum workspace");
    return MVAE_EINVAL;
  }
  if (dbias && cs_workspace_bytes < mvae_group_norm_colsum_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd_pack: column-sum workspace too small");
    return MVAE_EWORKSPACE;
  }
  return gn_bwd(x, dy, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu, drop_p, seed,
                workspace, workspace_bytes, dx_packed, dbias, bias_beta, cs_workspace, stream);
}

// as mvae_group_norm_bwd_pack_nhwc without the second dx copy: dx and the producing conv's bias gradient (dbias =
// bias_beta * dbias + column sums of dx) -- for a conv that takes its dy in fp32 (the exact-fp32 arithmetic; the Upsample
// conv's Winograd form), in place of a separate column-sum pass over dy
int mvae_group_norm_bwd_colsum_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                    const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                    float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                    unsigned long long seed, void* workspace, size_t workspace_bytes, float* dbias,
                                    float bias_beta, void* cs_workspace, size_t cs_workspace_bytes, void* stream) {
  if (dbias == nullptr || cs_workspace == nullptr || ((uintptr_t)dx & 15) || ((uintptr_t)x & 15) ||
      ((uintptr_t)dy & 15) || (dx_add && ((uintptr_t)dx_add & 15))) {
    set_error("group_norm_bwd_colsum: 16-B aligned x / dy / dx, a bias gradient and a column-sum workspace");
    return MVAE_EINVAL;
  }
  if (cs_workspace_bytes < mvae_group_norm_colsum_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd_colsum: column-sum workspace too small");
    return MVAE_EWORKSPACE;
  }
  return gn_bwd(x, dy, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu, drop_p, seed,
                workspace, workspace_bytes, nullptr, dbias, bias_beta, cs_workspace, stream);
}

// as mvae_group_norm_bwd_pack_nhwc, with dx also written as split4_bf16 groups (the 3xBF16 GEMMs' pre-split operand,
// 4 B per element at dx's element offsets; 16-B aligned) instead of packed bf16
int mvae_group_norm_bwd_split_nhwc(const float* x, const float* dy, const float* gamma, const float* beta,
                                   const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                                   float* dbeta, int nb, int hw, int c, int groups, int silu, float drop_p,
                                   unsigned long long seed, void* workspace, size_t workspace_bytes, void* dx_split,
                                   float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                   void* stream) {
  if (dx_split == nullptr || ((uintptr_t)dx_split & 15) || ((uintptr_t)dx & 15) || ((uintptr_t)x & 15) ||
      ((uintptr_t)dy & 15) || (dx_add && ((uintptr_t)dx_add & 15)) || (dbias && cs_workspace == nullptr)) {
    set_error("group_norm_bwd_split: 16-B aligned x / dy / dx / split output, a column-sum workspace");
    return MVAE_EINVAL;
  }
  if (dbias && cs_workspace_bytes < mvae_group_norm_colsum_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd_split: column-sum workspace too small");
    return MVAE_EWORKSPACE;
  }
  return gn_bwd(x, dy, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu, drop_p, seed,
                workspace, workspace_bytes, dx_split, dbias, bias_beta, cs_workspace, stream, 1);
}

static int gn_bwd(const float* x, const float* dy, const float* gamma, const float* beta, const float* mean,
                  const float* rstd, float* dx, const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c,
                  int groups, int silu, float drop_p, unsigned long long seed, void* workspace, size_t workspace_bytes,
                  void* dxp, float* dbias, float bias_beta, void* cs_ws, void* stream, int dxp_split) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups) {
    set_error("group_norm_bwd: bad geometry");
    return MVAE_EINVAL;
  }
  if (dx == nullptr && dxp == nullptr) {
    set_error("group_norm_bwd: dx may be null only when the split / packed copy is written");
    return MVAE_EINVAL;
  }
  if (workspace_bytes < mvae_group_norm_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  GnArgs a{};
  a.x = x; a.dy = dy; a.mean = mean; a.rstd = rstd; a.gamma = gamma; a.beta = beta; a.dx_add = dx_add;
  a.nb = nb; a.hw = hw; a.C = c; a.G = groups; a.silu = silu; a.drop_p = drop_p; a.seed = seed; a.salt = dropout_salt();
  a.chunks = gn_chunks(nb, hw);
  a.rows_per_chunk = (hw + a.chunks - 1) / a.chunks;
  a.ws = (double*)workspace;
  a.dxp = (uint2*)dxp;
  a.dxp_split = dxp_split;
  a.csp = dbias ? (double*)cs_ws : nullptr;
  int it = 0;
  static const int bwd_max_it = [] {
    const char* e = getenv("MVAE_GN_RES_BWD_IT");  // rows per thread allowed in the resident backward (8 or 13)
    return e ? std::min(13, atoi(e)) : 13;
  }();
  int sc = gn_resident_slab(nb, hw, c, groups, &it, bwd_max_it);
  // the backward holds x and dy of two units (2 waves/SIMD): with 64-B row segments (sc < 32) it streams at
  // ~3.1 TB/s, below the streaming kernels on tensors past ~64 MB (c2's 28x28x128 level: 140 vs 124 us)
  if (sc > 0 && sc < 32 && (long long)nb * hw * c * 4 > (64LL << 20)) sc = 0;
  if (sc) {
    double* pws = (double*)workspace;  // [2][C][nb] fp64 (within the [nb][chunks][C][2] partial area)
    const int units = nb * (c / sc);
    const void* k = it == 4 ? (const void*)gn_bwd_resident_kernel<4>
                  : it == 8 ? (const void*)gn_bwd_resident_kernel<8> : (const void*)gn_bwd_resident_kernel<13>;
    const dim3 grid(gn_res_grid(k, units));
    if (it == 4) hipLaunchKernelGGL(gn_bwd_resident_kernel<4>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, pws, dx);
    else if (it == 8) hipLaunchKernelGGL(gn_bwd_resident_kernel<8>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, pws, dx);
    else hipLaunchKernelGGL(gn_bwd_resident_kernel<13>, grid, dim3(GN_RES_NT), 0, st, a, sc, units, pws, dx);
    if (dgamma || dbeta)
      hipLaunchKernelGGL(gn_param_reduce_kernel, dim3(c), dim3(256), 0, st, (const double*)pws, nb, c, dgamma, dbeta);
    if (dbias)
      hipLaunchKernelGGL(gn_colsum_final_kernel, dim3(cdiv(c, 16)), dim3(256), 0, st, (const double*)a.csp, nb, c,
                         dbias, bias_beta);
    return launch_status();
  }
  // (the packed output, or the column sums: streaming chain -- the unit kernel writes neither)
  if (const int sc2 = (dxp || dbias) ? 0 : gn_unit2_slab(hw, c, groups)) {
    double* pws = (double*)workspace;
    const int units = nb * (c / sc2);
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    static const int per_cu = [] {
      const char* e = getenv("MVAE_GN_UNIT_PER_CU");  // experiment knob: workgroups per CU
      return e ? std::max(1, atoi(e)) : 1;
    }();
    const dim3 grid(std::max(1, std::min(units, std::max(1, cus) * per_cu)));
    hipLaunchKernelGGL(gn_bwd_unit2_kernel<4>, grid, dim3(GN_RES_NT), 0, st, a, sc2, units, pws, dx);
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
  if (dbias)
    hipLaunchKernelGGL(gn_colsum_final_kernel, dim3(cdiv(c, 16)), dim3(256), 0, st, (const double*)a.csp,
                       nb * a.chunks, c, dbias, bias_beta);
  return launch_status();
}

// Backward from the partials emitted by the input-gradient conv that consumed this GroupNorm's output
// (mvae_conv2d_dgrad_gnbwd_nhwc, part = [nb*hw/32][c][2] fp64 {sum dyn, sum dyn*xhat}): no partial pass over
// x and dy. No dropout (the fused conv epilogue does not apply a mask).
static int gn_bwd_part(const float* x, const float* dy, const double* part, const float* gamma, const float* beta,
                       const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                       float* dbeta, int nb, int hw, int c, int groups, int silu, void* workspace,
                       size_t workspace_bytes, void* dx_split, float* dbias, float bias_beta, void* cs_ws,
                       void* stream);

int mvae_group_norm_bwd_part_nhwc(const float* x, const float* dy, const double* part, const float* gamma,
                                  const float* beta, const float* mean, const float* rstd, float* dx,
                                  const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c, int groups,
                                  int silu, void* workspace, size_t workspace_bytes, void* stream) {
  return gn_bwd_part(x, dy, part, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu,
                     workspace, workspace_bytes, nullptr, nullptr, 0.f, nullptr, stream);
}

// as mvae_group_norm_bwd_part_nhwc, with dx also written as split4_bf16 groups and the producing conv's bias gradient
// (dbias = bias_beta * dbias + column sums of dx) -- mvae_group_norm_bwd_split_nhwc's outputs without its partial pass
int mvae_group_norm_bwd_part_split_nhwc(const float* x, const float* dy, const double* part, const float* gamma,
                                        const float* beta, const float* mean, const float* rstd, float* dx,
                                        const float* dx_add, float* dgamma, float* dbeta, int nb, int hw, int c,
                                        int groups, int silu, void* workspace, size_t workspace_bytes, void* dx_split,
                                        float* dbias, float bias_beta, void* cs_workspace, size_t cs_workspace_bytes,
                                        void* stream) {
  // (dx_split null: the bias column sums only -- the exact-fp32 arithmetic's convs read dy in fp32)
  if ((dx_split == nullptr && dbias == nullptr) || ((uintptr_t)dx_split & 15) || ((uintptr_t)dx & 15) ||
      ((uintptr_t)x & 15) || ((uintptr_t)dy & 15) || (dx_add && ((uintptr_t)dx_add & 15)) ||
      (dbias && cs_workspace == nullptr)) {
    set_error("group_norm_bwd_part_split: 16-B aligned x / dy / dx / split output (or a bias gradient), a column-sum "
              "workspace");
    return MVAE_EINVAL;
  }
  if (dbias && cs_workspace_bytes < mvae_group_norm_colsum_workspace_bytes(nb, hw, c)) {
    set_error("group_norm_bwd_part_split: column-sum workspace too small");
    return MVAE_EWORKSPACE;
  }
  return gn_bwd_part(x, dy, part, gamma, beta, mean, rstd, dx, dx_add, dgamma, dbeta, nb, hw, c, groups, silu,
                     workspace, workspace_bytes, dx_split, dbias, bias_beta, cs_workspace, stream);
}

// 1 when mvae_group_norm_bwd_nhwc (with_dxp = 0) or its split / pack forms (with_dxp = 1) run the two-pass streaming
// chain (a partial pass over x and dy, then the dx pass) -- the chain whose partial pass the consuming conv's
// input-gradient epilogue can supply (mvae_group_norm_bwd_part*_nhwc); 0 for the one-pass resident / unit kernels
int mvae_group_norm_bwd_streaming(int nb, int hw, int c, int groups, int with_dxp) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups) return 0;
  static const int bwd_max_it = [] {
    const char* e = getenv("MVAE_GN_RES_BWD_IT");
    return e ? std::min(13, atoi(e)) : 13;
  }();
  int it = 0;
  int sc = gn_resident_slab(nb, hw, c, groups, &it, bwd_max_it);
  if (sc > 0 && sc < 32 && (long long)nb * hw * c * 4 > (64LL << 20)) sc = 0;
  if (sc) return 0;
  return (with_dxp || !gn_unit2_slab(hw, c, groups)) ? 1 : 0;
}

static int gn_bwd_part(const float* x, const float* dy, const double* part, const float* gamma, const float* beta,
                       const float* mean, const float* rstd, float* dx, const float* dx_add, float* dgamma,
                       float* dbeta, int nb, int hw, int c, int groups, int silu, void* workspace,
                       size_t workspace_bytes, void* dx_split, float* dbias, float bias_beta, void* cs_ws,
                       void* stream) {
  if (nb <= 0 || hw <= 0 || c <= 0 || (c & 3) || groups <= 0 || c % groups || hw % 32 || part == nullptr) {
    set_error("group_norm_bwd_part: needs hw %% 32 == 0 and C %% 4 == 0");
    return MVAE_EINVAL;
  }
  if (dx == nullptr && dx_split == nullptr) {
    set_error("group_norm_bwd_part: dx may be null only when the split copy is written");
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
  a.dxp = (uint2*)dx_split;
  a.dxp_split = 1;
  a.csp = dbias ? (double*)cs_ws : nullptr;
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
  if (dbias)
    hipLaunchKernelGGL(gn_colsum_final_kernel, dim3(cdiv(c, 16)), dim3(256), 0, st, (const double*)a.csp,
                       nb * a.chunks, c, dbias, bias_beta);
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
