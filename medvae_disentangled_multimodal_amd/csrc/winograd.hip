// Winograd F(2x2, 3x3) convolution for the 3x3 / stride-1 / pad-1 convs of the low-resolution, wide levels (c4 / c5's
// 8x8 x 2048 and 16x16 x 1024: ResnetBlock conv1 / conv2, the mid blocks -- src/models/encoder_decoder.py:123-170) in the
// fp32-class (3xBF16) arithmetic: forward, input gradient and weight gradient (F(3x3, 2x2), below).
//
// Per 2x2 output tile t and channel c the 4x4 input patch d is transformed to V = B^T d B, the 3x3 filter g of (k, c) to
// U = G g G^T, the 16 transformed positions xi are independent GEMMs M_xi[t][k] = sum_c V_xi[t][c] U_xi[k][c], and the
// tile's outputs are A^T M A:
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1],  G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1],
//   A^T = [1 1 1 0; 0 1 -1 -1]
// 16 multiplies per output tile instead of 36: the GEMM work is 4/9 of the direct conv's. The transforms are additions
// (and halvings) of fp32 values; V and U are written in the 3xBF16 pre-split layout (split4_bf16) so the batched GEMM
// (gemm3x_kernel, A_ROWK_SPLIT x B_ROWK_SPLIT, 16 batch entries) stages them without split arithmetic. Its cost against
// the direct conv is the traffic of V (16 / 4 = 4x the input) and M (4x the output) -- small next to the GEMM when the
// channel count is large and the image small, which is where the dispatcher (ops.py) uses it.
//
// The input gradient of the same conv is a 3x3 / stride-1 / pad-1 conv of dy with the flipped, transposed filters
// g'(c, k)[r][s] = g(k, c)[2-r][2-s]: the same four stages with U' (mvae_winograd_weight_transform's dgrad form).
// The output transform can add the conv bias and the ResnetBlock residual and emits the following GroupNorm's
// statistics in the GEMM epilogue's layout (per 32-pixel block and 4-channel group, fp64 {sum y, sum y^2}).
#include "gemm_core.h"

namespace mvae {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return float4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
__device__ __forceinline__ float4 f4sub(float4 a, float4 b) { return float4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
__device__ __forceinline__ float4 f4scale(float4 a, float s) { return float4{a.x * s, a.y * s, a.z * s, a.w * s}; }

// B^T d B of a 4x4 patch of float4 channel groups, in place: rows, then columns
__device__ __forceinline__ void wino_bt(float4 (&d)[4][4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float4 r0 = f4sub(d[0][j], d[2][j]), r1 = f4add(d[1][j], d[2][j]);
    const float4 r2 = f4sub(d[2][j], d[1][j]), r3 = f4sub(d[1][j], d[3][j]);
    d[0][j] = r0; d[1][j] = r1; d[2][j] = r2; d[3][j] = r3;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 c0 = f4sub(d[i][0], d[i][2]), c1 = f4add(d[i][1], d[i][2]);
    const float4 c2 = f4sub(d[i][2], d[i][1]), c3 = f4sub(d[i][1], d[i][3]);
    d[i][0] = c0; d[i][1] = c1; d[i][2] = c2; d[i][3] = c3;
  }
}

// x [nb][H][W][C] (fp32, or split4_bf16 groups when XS) -> V [16][T][C] split4_bf16, T = nb (H/2) (W/2)
// one thread per (tile, 4-channel group): 16 coalesced 16-B loads (zeros outside the image), 16 16-B stores
template <bool XS>
__global__ void __launch_bounds__(256) wino_in_kernel(const float* __restrict__ x, uint4* __restrict__ v, int nb, int H,
                                                      int W, int C) {
  const int C4 = C >> 2, th = H >> 1, tw = W >> 1;
  const long long T = (long long)nb * th * tw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * C4) return;
  const long long t = idx / C4;
  const int c4 = (int)(idx - t * C4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  float4 d[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int h = 2 * ti - 1 + i, w = 2 * tj - 1 + j;
      float4 val{0.f, 0.f, 0.f, 0.f};
      if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
        const float4 r = *(const float4*)(x + (((long long)b * H + h) * W + w) * C + c4 * 4);
        if constexpr (XS) {  // split4: hi0..hi3 then lo0..lo3 as bf16 -> fp32 hi + lo
          const unsigned h01 = __float_as_uint(r.x), h23 = __float_as_uint(r.y);
          const unsigned l01 = __float_as_uint(r.z), l23 = __float_as_uint(r.w);
          val = float4{__uint_as_float(h01 << 16) + __uint_as_float(l01 << 16),
                       __uint_as_float(h01 & 0xFFFF0000u) + __uint_as_float(l01 & 0xFFFF0000u),
                       __uint_as_float(h23 << 16) + __uint_as_float(l23 << 16),
                       __uint_as_float(h23 & 0xFFFF0000u) + __uint_as_float(l23 & 0xFFFF0000u)};
        } else {
          val = r;
        }
      }
      d[i][j] = val;
    }
  wino_bt(d);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[((long long)(i * 4 + j) * T + t) * C4 + c4] = split4_bf16(d[i][j]);
}

// Weight gradient (F(3x3, 2x2) on the same tiles): with D_t the 2x2 output-gradient tile and X_t the input patch of
// tile t, dW[r][s] = sum_t sum_{a,e} D_t[a][e] X_t[a+r][e+s] = G^T [ sum_t (A D_t A^T) (.) (B^T X_t B) ] G -- the bilinear
// form of the forward identity differentiated by the filter. So dW = G^T M G with M_xi[k][c] = sum_t D'_xi[t][k]
// V_xi[t][c]: 16 GEMMs over the tiles (K = T) of the transformed output gradient D' = A D A^T (A = (A^T)^T, rows
// [1 0; 1 1; 1 -1; 0 -1]) and the forward's V.

// dy [nb][H][W][K] (fp32, or split4_bf16 groups when XS) -> D' [16][T][K] split4_bf16: one thread per (tile, 4-group)
template <bool XS>
__global__ void __launch_bounds__(256) wino_dy_kernel(const float* __restrict__ dy, uint4* __restrict__ d, int nb, int H,
                                                      int W, int K) {
  const int K4 = K >> 2, th = H >> 1, tw = W >> 1;
  const long long T = (long long)nb * th * tw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * K4) return;
  const long long t = idx / K4;
  const int k4 = (int)(idx - t * K4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  float4 v[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float4 r = *(const float4*)(dy + (((long long)b * H + 2 * ti + a) * W + 2 * tj + e) * K + k4 * 4);
      if constexpr (XS) {
        const unsigned h01 = __float_as_uint(r.x), h23 = __float_as_uint(r.y);
        const unsigned l01 = __float_as_uint(r.z), l23 = __float_as_uint(r.w);
        v[a][e] = float4{__uint_as_float(h01 << 16) + __uint_as_float(l01 << 16),
                         __uint_as_float(h01 & 0xFFFF0000u) + __uint_as_float(l01 & 0xFFFF0000u),
                         __uint_as_float(h23 << 16) + __uint_as_float(l23 << 16),
                         __uint_as_float(h23 & 0xFFFF0000u) + __uint_as_float(l23 & 0xFFFF0000u)};
      } else {
        v[a][e] = r;
      }
    }
  float4 c[4][2];  // A D: rows
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    c[0][e] = v[0][e];
    c[1][e] = f4add(v[0][e], v[1][e]);
    c[2][e] = f4sub(v[0][e], v[1][e]);
    c[3][e] = f4scale(v[1][e], -1.f);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 o[4] = {c[i][0], f4add(c[i][0], c[i][1]), f4sub(c[i][0], c[i][1]), f4scale(c[i][1], -1.f)};
#pragma unroll
    for (int j = 0; j < 4; ++j) d[((long long)(i * 4 + j) * T + t) * K4 + k4] = split4_bf16(o[j]);
  }
}

// dw [cout][3][3][cin] = beta * dw + G^T M G, M [16][cout][cin] fp32: one thread per (k, 4-group of c)
__global__ void __launch_bounds__(256) wino_wout_kernel(const float* __restrict__ m, float* __restrict__ dw, float beta,
                                                        int cout, int cin) {
  const int C4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * C4) return;
  const long long mn = (long long)cout * cin;
  float4 mv[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) mv[i][j] = *(const float4*)(m + (i * 4 + j) * mn + idx * 4);
  float4 r[3][4];  // G^T M
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[0][j] = f4add(mv[0][j], f4scale(f4add(mv[1][j], mv[2][j]), 0.5f));
    r[1][j] = f4scale(f4sub(mv[1][j], mv[2][j]), 0.5f);
    r[2][j] = f4add(f4scale(f4add(mv[1][j], mv[2][j]), 0.5f), mv[3][j]);
  }
  const int k = (int)(idx / C4), c4 = (int)(idx - (long long)k * C4);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const float4 o[3] = {f4add(r[i][0], f4scale(f4add(r[i][1], r[i][2]), 0.5f)), f4scale(f4sub(r[i][1], r[i][2]), 0.5f),
                         f4add(f4scale(f4add(r[i][1], r[i][2]), 0.5f), r[i][3])};
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float4* p = (float4*)(dw + (((long long)k * 3 + i) * 3 + j) * cin + c4 * 4);
      float4 v = o[j];
      if (beta != 0.f) v = f4add(v, f4scale(*p, beta));
      *p = v;
    }
  }
}

// G g G^T of a 3x3 filter of float4 groups
__device__ __forceinline__ void wino_g(const float4 (&g)[3][3], float4 (&o)[4][4]) {
  float4 t[4][3];
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    t[0][s] = g[0][s];
    t[1][s] = f4scale(f4add(f4add(g[0][s], g[1][s]), g[2][s]), 0.5f);
    t[2][s] = f4scale(f4add(f4sub(g[0][s], g[1][s]), g[2][s]), 0.5f);
    t[3][s] = g[2][s];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i][0] = t[i][0];
    o[i][1] = f4scale(f4add(f4add(t[i][0], t[i][1]), t[i][2]), 0.5f);
    o[i][2] = f4scale(f4add(f4sub(t[i][0], t[i][1]), t[i][2]), 0.5f);
    o[i][3] = t[i][2];
  }
}

// forward filters U[16][cout][cin] split4_bf16 from KRSC weights w [cout][3][3][cin], g(n, k) = w[n][.][.][k]:
// one thread per (cout n, 4-group of cin k), 9 coalesced 16-B loads, 16 coalesced 16-B stores
__global__ void __launch_bounds__(256) wino_wt_fwd_kernel(const float* __restrict__ w, uint4* __restrict__ u, int cout,
                                                          int cin) {
  const int K4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * K4) return;
  const int n = (int)(idx / K4), k4 = (int)(idx - (long long)n * K4);
  float4 g[3][3], o[4][4];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) g[r][s] = *(const float4*)(w + (((long long)n * 3 + r) * 3 + s) * cin + k4 * 4);
  wino_g(g, o);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) u[((long long)(i * 4 + j) * cout + n) * K4 + k4] = split4_bf16(o[i][j]);
}

// input-gradient filters U'[16][cin][cout] split4_bf16, g'(n = cin, k = cout)[r][s] = w[k][2-r][2-s][n]: the source
// is contiguous along n and the destination along k, so a workgroup transposes a 32 (n) x 8 (k groups of 4) block
// through LDS: loads coalesced over n (32 lanes), stores in 128-B runs over k
constexpr int WDG_N = 32, WDG_K4 = 8;
__global__ void __launch_bounds__(256) wino_wt_dgrad_kernel(const float* __restrict__ w, uint4* __restrict__ u,
                                                            int cout, int cin) {
  __shared__ uint4 lds[16][WDG_N][WDG_K4];  // 64 KB
  const int K4 = cout >> 2;
  const int n0 = blockIdx.x * WDG_N, kb = blockIdx.y * WDG_K4;
  const int nl = threadIdx.x & (WDG_N - 1), kq = threadIdx.x / WDG_N;
  const int n = n0 + nl, k4 = kb + kq;
  if (n < cin && k4 < K4) {
    float4 g[3][3], o[4][4];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = w[(((long long)(k4 * 4 + q) * 3 + (2 - r)) * 3 + (2 - s)) * cin + n];
        g[r][s] = float4{e[0], e[1], e[2], e[3]};
      }
    wino_g(g, o);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) lds[i * 4 + j][nl][kq] = split4_bf16(o[i][j]);
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 16 * WDG_N * WDG_K4 / 256; ++it) {
    const int e = it * 256 + threadIdx.x;
    const int xi = e / (WDG_N * WDG_K4), rem = e % (WDG_N * WDG_K4);
    const int nn = n0 + rem / WDG_K4, kk = kb + rem % WDG_K4;
    if (nn < cin && kk < K4) u[((long long)xi * cin + nn) * K4 + kk] = lds[xi][rem / WDG_K4][rem % WDG_K4];
  }
}

// output transform operands
struct WinoOut {
  const float* m;      // [16][T][N] fp32 GEMM results
  const float* bias;   // [N] or null
  const float* res;    // residual [nb][H][W][N] or null
  float* y;            // [nb][H][W][N]
  double* gn_part;     // GroupNorm statistics of y (forward), or null
  // GroupNorm backward partials (input gradient of a conv whose input was silu?(GroupNorm(x))): per channel and 32-pixel
  // block {sum dyn, sum dyn * xhat} at gnb_part[(block * N + col) * 2], dyn = y * silu'(.) -- the implicit-GEMM epilogue's
  // GemmArgs::gnb_part, same float arithmetic
  double* gnb_part;
  const float* gx;
  const float *mean, *rstd, *gamma, *beta;
  int groups, silu;
  int nb, H, W, N;
};

// M -> y = A^T M A (+ bias) (+ residual) for W in {8, 16}: 8 consecutive tiles are one 32-pixel block of the row-major
// pixel order (2 tile rows of an 8-wide image, 1 of a 16-wide one). One thread per (block of 8 tiles, 4-channel group);
// the channel groups of a block are consecutive threads (coalesced 16-B loads / stores).
template <bool GNB>
__global__ void __launch_bounds__(256) wino_out_kernel(WinoOut p) {
  const int N = p.N, N4 = N >> 2, th = p.H >> 1, tw = p.W >> 1;
  const long long T = (long long)p.nb * th * tw, nblk = T / 8;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= nblk * N4) return;
  const long long blk = idx / N4;
  const int c4 = (int)(idx - blk * N4);
  const float4 bv = p.bias ? *(const float4*)(p.bias + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
  double s0 = 0.0, s1 = 0.0;
  double g0[4] = {0.0, 0.0, 0.0, 0.0}, g1[4] = {0.0, 0.0, 0.0, 0.0};
  float ggm[4], gbt[4];
  if constexpr (GNB) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ggm[e] = p.gamma[c4 * 4 + e];
      gbt[e] = p.beta[c4 * 4 + e];
    }
  }
  const int cpg = GNB ? N / p.groups : 1;
  for (int q = 0; q < 8; ++q) {
    const long long t = blk * 8 + q;
    const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
    float4 mv[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) mv[i][j] = *(const float4*)(p.m + ((long long)(i * 4 + j) * T + t) * N + c4 * 4);
    float4 r[2][4];  // A^T M: rows
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r[0][j] = f4add(f4add(mv[0][j], mv[1][j]), mv[2][j]);
      r[1][j] = f4sub(f4sub(mv[1][j], mv[2][j]), mv[3][j]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const float4 o0 = f4add(f4add(r[a][0], r[a][1]), r[a][2]);
      const float4 o1 = f4sub(f4sub(r[a][1], r[a][2]), r[a][3]);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const long long pix = ((long long)b * p.H + 2 * ti + a) * p.W + 2 * tj + e;
        const long long off = pix * N + c4 * 4;
        float4 o = f4add(e == 0 ? o0 : o1, bv);
        if (p.res) o = f4add(o, *(const float4*)(p.res + off));
        *(float4*)(p.y + off) = o;
        if (p.gn_part) {
          s0 += ((double)o.x + (double)o.y) + ((double)o.z + (double)o.w);
          s1 += ((double)o.x * o.x + (double)o.y * o.y) + ((double)o.z * o.z + (double)o.w * o.w);
        }
        if constexpr (GNB) {
          const float4 x4 = *(const float4*)(p.gx + off);
          const int bg = b * p.groups + (c4 * 4) / cpg;  // (a 4-channel group never straddles a GroupNorm group)
          const float mu = p.mean[bg], rs = p.rstd[bg];
          const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, vs[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float d = vs[u];
            const float xh = (xs[u] - mu) * rs;
            if (p.silu) {
              const float yn = xh * ggm[u] + gbt[u];
              const float sg = sigmoid_f(yn);
              d = d * sg * (1.f + yn * (1.f - sg));
            }
            g0[u] += d;
            g1[u] += (double)d * xh;
          }
        }
      }
    }
  }
  if (p.gn_part) *(double2*)(p.gn_part + (blk * N4 + c4) * 2) = double2{s0, s1};
  if constexpr (GNB) {
    double* gp = p.gnb_part + (blk * N + c4 * 4) * 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) *(double2*)(gp + 2 * u) = double2{g0[u], g1[u]};
  }
}

static long long wino_tiles(int nb, int h, int w) { return (long long)nb * (h / 2) * (w / 2); }

static bool wino_geom_ok(int nb, int h, int w, int cin, int cout) {
  // (h w % 32 == 0: the output transform's 8-tile blocks are the 32-pixel blocks of the statistics layouts)
  return nb > 0 && h >= 2 && (h % 2) == 0 && (w == 8 || w == 16) && (h * w) % 32 == 0 && cin > 0 && cout > 0 &&
         cin % 4 == 0 && cout % 4 == 0 && wino_tiles(nb, h, w) * std::max(cin, cout) * 4 <= MAX_DESC_BYTES;
}

static int egrid256(long long n) { return (int)std::min<long long>((n + 255) / 256, 1LL << 30); }

}  // namespace mvae

using namespace mvae;

extern "C" {

// U = the 16 transformed filters in split4_bf16 ([16][cout][cin] forward, [16][cin][cout] for the input gradient when
// dgrad != 0) of KRSC 3x3 weights w [cout][3][3][cin]
int mvae_winograd_weight_transform(const float* w, void* u, int cin, int cout, int dgrad, void* stream) {
  if (!w || !u || cin <= 0 || cout <= 0 || cin % 4 || cout % 4 || !al16(w) || !al16(u)) {
    set_error("winograd_weight_transform: cin, cout multiples of 4, 16-B aligned w / u");
    return MVAE_EINVAL;
  }
  if (math_mode() != MATH_3XBF16) {
    set_error("winograd: the 3xBF16 (fp32-class) arithmetic only");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  if (dgrad)
    hipLaunchKernelGGL(wino_wt_dgrad_kernel, dim3(cdiv(cin, WDG_N), cdiv(cout / 4, WDG_K4)), dim3(256), 0, st, w,
                       (uint4*)u, cout, cin);
  else
    hipLaunchKernelGGL(wino_wt_fwd_kernel, dim3(egrid256((long long)cout * (cin / 4))), dim3(256), 0, st, w, (uint4*)u,
                       cout, cin);
  return launch_status();
}

// V [16][T][c] split4_bf16 of x [nb][h][w][c] (fp32, or split4_bf16 groups when x_split), T = nb (h/2) (w/2)
int mvae_winograd_input_transform(const float* x, void* v, int nb, int h, int w, int c, int x_split, void* stream) {
  if (!x || !v || !wino_geom_ok(nb, h, w, c, c) || !al16(x) || !al16(v)) {
    set_error("winograd_input_transform: even h, w in {8, 16}, h w %% 32 == 0, c %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const long long n = wino_tiles(nb, h, w) * (c / 4);
  if (x_split)
    hipLaunchKernelGGL(wino_in_kernel<true>, dim3(egrid256(n)), dim3(256), 0, st, x, (uint4*)v, nb, h, w, c);
  else
    hipLaunchKernelGGL(wino_in_kernel<false>, dim3(egrid256(n)), dim3(256), 0, st, x, (uint4*)v, nb, h, w, c);
  return launch_status();
}

// M [16][T][n_out] fp32 = V_xi [T][k_in] . U_xi [n_out][k_in]^T for the 16 positions xi: one batched launch of the
// implicit-GEMM core on pre-split operands
int mvae_winograd_gemm(const void* v, const void* u, float* m, long long tiles, int k_in, int n_out, void* stream) {
  if (!v || !u || !m || tiles <= 0 || k_in <= 0 || n_out <= 0 || k_in % 4 || n_out % 4 || !al16(v) || !al16(u) ||
      !al16(m) || tiles * std::max(k_in, n_out) * 4 > MAX_DESC_BYTES || tiles > (1LL << 30)) {
    set_error("winograd_gemm: k_in, n_out multiples of 4, 16-B aligned, one position < 4 GiB");
    return MVAE_EINVAL;
  }
  if (math_mode() != MATH_3XBF16) {
    set_error("winograd: the 3xBF16 (fp32-class) arithmetic only");
    return MVAE_EINVAL;
  }
  GemmArgs a{};
  a.M = (int)tiles; a.N = n_out; a.K = k_in; a.batch = 16;
  a.A = (const float*)v; a.lda = k_in; a.sA = tiles * k_in;
  a.B = (const float*)u; a.ldb = k_in; a.sB = (long long)n_out * k_in;
  a.C = m; a.ldc = n_out; a.sC = tiles * n_out;
  a.alpha = 1.f; a.beta = 0.f;
  a.a_bytes = (unsigned)(tiles * k_in * 4); a.b_bytes = (unsigned)((long long)n_out * k_in * 4);
  a.c_bytes = (unsigned)(tiles * n_out * 4);
  set_splits(a, 1);
  const int cfg = choose_tile(a, true, false);
  launch_big<A_ROWK_SPLIT, 4, B_ROWK_SPLIT, 4>(a, (hipStream_t)stream, cfg);
  return launch_status();
}

// y [nb][h][w][n] = A^T M A (+ bias[n]) (+ residual, same layout as y); gn_part (nullable): the GroupNorm statistics of
// y per 32-pixel block and 4-channel group (fp64 pairs, [nb*h*w/32][n/4][2], the mvae_conv2d_gnstats_nhwc layout)
int mvae_winograd_output_transform(const float* m, const float* bias, const float* residual, float* y, double* gn_part,
                                   int nb, int h, int w, int n, void* stream) {
  if (!m || !y || !wino_geom_ok(nb, h, w, n, n) || !al16(m) || !al16(y) || (bias && !al16(bias)) ||
      (residual && !al16(residual))) {
    set_error("winograd_output_transform: even h, w in {8, 16}, h w %% 32 == 0, n %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  WinoOut p{};
  p.m = m; p.bias = bias; p.res = residual; p.y = y; p.gn_part = gn_part;
  p.groups = 1; p.nb = nb; p.H = h; p.W = w; p.N = n;
  const long long nblk = wino_tiles(nb, h, w) / 8;
  hipLaunchKernelGGL(wino_out_kernel<false>, dim3(egrid256(nblk * (n / 4))), dim3(256), 0, (hipStream_t)stream, p);
  return launch_status();
}

// Input-gradient output transform dx = A^T M A that also emits the backward partials of the GroupNorm whose
// (silu'd) output was the conv's input -- mvae_conv2d_dgrad_gnbwd_nhwc's epilogue: per channel and 32-pixel block
// {sum dyn, sum dyn * xhat} (fp64) at part[((pixel / 32) * n + channel) * 2], x / mean / rstd / gamma / beta the
// GroupNorm's input and statistics ([nb][h][w][n], [nb * groups] x 2, [n] x 2)
int mvae_winograd_output_gnbwd(const float* m, float* dx, const float* x, const float* mean, const float* rstd,
                               const float* gamma, const float* beta, int groups, int silu, double* part, int nb, int h,
                               int w, int n, void* stream) {
  if (!m || !dx || !x || !mean || !rstd || !gamma || !beta || !part || groups <= 0 || n % groups ||
      (n / groups) % 4 || !wino_geom_ok(nb, h, w, n, n) || !al16(m) || !al16(dx) || !al16(x)) {
    set_error("winograd_output_gnbwd: even h, w in {8, 16}, h w %% 32 == 0, channels per group %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  WinoOut p{};
  p.m = m; p.y = dx; p.gnb_part = part; p.gx = x; p.mean = mean; p.rstd = rstd; p.gamma = gamma; p.beta = beta;
  p.groups = groups; p.silu = silu; p.nb = nb; p.H = h; p.W = w; p.N = n;
  const long long nblk = wino_tiles(nb, h, w) / 8;
  hipLaunchKernelGGL(wino_out_kernel<true>, dim3(egrid256(nblk * (n / 4))), dim3(256), 0, (hipStream_t)stream, p);
  return launch_status();
}

// D' [16][T][k] split4_bf16 of the output gradient dy [nb][h][w][k] (fp32, or split4_bf16 groups when dy_split)
int mvae_winograd_dy_transform(const float* dy, void* d, int nb, int h, int w, int k, int dy_split, void* stream) {
  if (!dy || !d || !wino_geom_ok(nb, h, w, k, k) || !al16(dy) || !al16(d)) {
    set_error("winograd_dy_transform: even h, w in {8, 16}, h w %% 32 == 0, k %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const long long n = wino_tiles(nb, h, w) * (k / 4);
  if (dy_split)
    hipLaunchKernelGGL(wino_dy_kernel<true>, dim3(egrid256(n)), dim3(256), 0, st, dy, (uint4*)d, nb, h, w, k);
  else
    hipLaunchKernelGGL(wino_dy_kernel<false>, dim3(egrid256(n)), dim3(256), 0, st, dy, (uint4*)d, nb, h, w, k);
  return launch_status();
}

// M [16][cout][cin] fp32 = sum over the tiles of D'_xi [T][cout] (x) V_xi [T][cin]: one batched launch (COL x COL
// images of pre-split operands), split over the tiles when the 16 products leave the chip under-filled and the
// workspace (mvae_gemm_workspace_bytes(cout, cin, tiles, 16)) allows
int mvae_winograd_wgrad_gemm(const void* d, const void* v, float* m, long long tiles, int cout, int cin, float* workspace,
                             size_t workspace_bytes, void* stream) {
  if (!d || !v || !m || tiles <= 0 || cout <= 0 || cin <= 0 || cout % 4 || cin % 4 || !al16(d) || !al16(v) || !al16(m) ||
      tiles * std::max(cout, cin) * 4 > MAX_DESC_BYTES || tiles > (1LL << 30)) {
    set_error("winograd_wgrad_gemm: cout, cin multiples of 4, 16-B aligned, one position < 4 GiB");
    return MVAE_EINVAL;
  }
  if (math_mode() != MATH_3XBF16) {
    set_error("winograd: the 3xBF16 (fp32-class) arithmetic only");
    return MVAE_EINVAL;
  }
  GemmArgs a{};
  a.M = cout; a.N = cin; a.K = (int)tiles; a.batch = 16;
  a.A = (const float*)d; a.lda = cout; a.sA = tiles * cout;
  a.B = (const float*)v; a.ldb = cin; a.sB = tiles * cin;
  a.C = m; a.ldc = cin; a.sC = (long long)cout * cin;
  a.alpha = 1.f; a.beta = 0.f;
  a.a_bytes = (unsigned)(tiles * cout * 4); a.b_bytes = (unsigned)(tiles * cin * 4);
  a.c_bytes = (unsigned)((long long)cout * cin * 4);
  const int cfg = choose_tile(a, true, workspace != nullptr);
  plan_splits(a, cfg, workspace, workspace_bytes);
  launch_big<A_COLM_SPLIT, 4, B_COLN_SPLIT, 4>(a, (hipStream_t)stream, cfg);
  return gemm_finish(a, (hipStream_t)stream);
}

// dw [cout][3][3][cin] = beta * dw + G^T M G
int mvae_winograd_wgrad_output(const float* m, float* dw, float beta, int cout, int cin, void* stream) {
  if (!m || !dw || cout <= 0 || cin <= 0 || cin % 4 || !al16(m) || !al16(dw)) {
    set_error("winograd_wgrad_output: cin %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(wino_wout_kernel, dim3(egrid256((long long)cout * (cin / 4))), dim3(256), 0, (hipStream_t)stream, m,
                     dw, beta, cout, cin);
  return launch_status();
}

// workspace of the Winograd form of a conv: V (16 T cin), M (16 T cout) and U (16 cin cout), 4 B each, 256-B aligned
size_t mvae_winograd_workspace_bytes(int nb, int h, int w, int cin, int cout) {
  const long long t = wino_tiles(nb, h, w);
  auto al = [](long long b) { return (size_t)((b + 255) / 256 * 256); };
  return al(64LL * t * cin) + al(64LL * t * cout) + al(64LL * cin * cout);
}

}  // extern "C"
