// Winograd convolution F(m x m, 3x3), m = 2 or 4, for the 3x3 / stride-1 / pad-1 convs of the low-resolution, wide levels
// (c4 / c5's 8x8 x 2048 and 16x16 x 1024: ResnetBlock conv1 / conv2, the mid blocks -- src/models/encoder_decoder.py:
// 123-170) in the fp32-class (3xBF16) arithmetic: forward, input gradient and weight gradient.
//
// Per m x m output tile t and channel c the a x a input patch d (a = m + 2) is transformed to V = B^T d B, the 3x3 filter
// g of (k, c) to U = G g G^T, the a^2 transformed positions xi are independent GEMMs M_xi[t][k] = sum_c V_xi[t][c]
// U_xi[k][c], and the tile's outputs are A^T M A. a^2 multiplies per output tile instead of 9 m^2: the GEMM work is
// 16/36 = 4/9 (m = 2) or 36/144 = 1/4 (m = 4) of the direct conv's.
//   m = 2: B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1], G = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1],
//          A^T = [1 1 1 0; 0 1 -1 -1]
//   m = 4: points 0, +-1, +-2, inf (wino_bt / wino_g / wino_at below)
// The transforms run in fp32; V and U are written pre-split so the batched GEMM (gemm3x_kernel, A_ROWK_SPLIT x
// B_ROWK_SPLIT, a^2 batch entries) stages them without split arithmetic, in the layout of the process's GEMM arithmetic:
// 3xBF16 and bf16 -- split4_bf16 (the bf16 GEMM stages the hi halves: V and U rounded to bf16); exact fp32 -- split4_bits
// (a bit split the f32-input MFMA reassembles exactly). Error against float64 (tests/test_gpu_winograd.py): 3xBF16 m = 2
// ~1e-5, m = 4 ~5e-5 norm-wise relative (the larger m = 4 coefficients amplify the operand rounding; the north_star bar
// is 1e-3); exact fp32 m = 4 ~5e-7; bf16 m = 2 ~4e-3 (1.7x the direct bf16 conv; m = 4 would be ~11x, so the bf16 mode
// uses m = 2 -- ops.py). The cost against the direct conv is the transform
// traffic -- V is a^2 / m^2 times the input (4x for m = 2, 2.25x for m = 4), M as much of the output -- small next to
// the GEMM when the channel count is large and the image small, which is where the dispatcher (ops.py) uses it.
//
// The input gradient is a 3x3 / stride-1 / pad-1 conv of dy with the flipped, transposed filters g'(c, k)[r][s] =
// g(k, c)[2-r][2-s]: the same stages with U' (mvae_winograd_weight_transform's dgrad form). The output transform can add
// the conv bias and the ResnetBlock residual and emits the following GroupNorm's statistics in the GEMM epilogue's
// layout (per 32-pixel block and 4-channel group, fp64 {sum y, sum y^2}), or, for an input gradient, the GroupNorm
// backward partials of mvae_conv2d_dgrad_gnbwd_nhwc.
//
// Weight gradient: with D_t the m x m output-gradient tile and X_t the input patch of tile t, dW[r][s] =
// sum_t sum_{u,e} D_t[u][e] X_t[u+r][e+s] = G^T [ sum_t (A D_t A^T) (.) (B^T X_t B) ] G -- the bilinear form of the
// forward identity differentiated by the filter. So dW = G^T M G with M_xi[k][c] = sum_t D'_xi[t][k] V_xi[t][c]: a^2
// GEMMs over the tiles (K = T) of the transformed output gradient D' = A D A^T and the forward's V.
#include "gemm_core.h"

namespace mvae {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) { return float4{a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

// transform coefficients (compile-time after unrolling: zero terms vanish, +-1 terms are adds / subtracts)
template <int MT>
__host__ __device__ constexpr float wino_bt(int i, int j) {  // B^T [a][a]
  if constexpr (MT == 2) {
    constexpr float m[4][4] = {{1, 0, -1, 0}, {0, 1, 1, 0}, {0, -1, 1, 0}, {0, 1, 0, -1}};
    return m[i][j];
  } else {
    constexpr float m[6][6] = {{4, 0, -5, 0, 1, 0},  {0, -4, -4, 1, 1, 0}, {0, 4, -4, -1, 1, 0},
                               {0, -2, -1, 2, 1, 0}, {0, 2, -1, -2, 1, 0}, {0, 4, 0, -5, 0, 1}};
    return m[i][j];
  }
}
template <int MT>
__host__ __device__ constexpr float wino_g(int i, int j) {  // G [a][3]
  if constexpr (MT == 2) {
    constexpr float m[4][3] = {{1, 0, 0}, {0.5f, 0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {0, 0, 1}};
    return m[i][j];
  } else {
    constexpr float m[6][3] = {{0.25f, 0, 0},
                               {-1.f / 6, -1.f / 6, -1.f / 6},
                               {-1.f / 6, 1.f / 6, -1.f / 6},
                               {1.f / 24, 1.f / 12, 1.f / 6},
                               {1.f / 24, -1.f / 12, 1.f / 6},
                               {0, 0, 1}};
    return m[i][j];
  }
}
template <int MT>
__host__ __device__ constexpr float wino_at(int i, int j) {  // A^T [m][a]
  if constexpr (MT == 2) {
    constexpr float m[2][4] = {{1, 1, 1, 0}, {0, 1, -1, -1}};
    return m[i][j];
  } else {
    constexpr float m[4][6] = {{1, 1, 1, 1, 1, 0}, {0, 1, -1, 2, -2, 0}, {0, 1, 1, 4, 4, 0}, {0, 1, -1, 8, -8, 1}};
    return m[i][j];
  }
}

// acc (+)= c * v, with `first` a compile-time flag after unrolling
__device__ __forceinline__ void wmadd(float4& acc, bool& first, float c, float4 v) {
  if (c == 0.f) return;
  float4 t;
  if (c == 1.f) t = v;
  else if (c == -1.f) t = float4{-v.x, -v.y, -v.z, -v.w};
  else t = float4{c * v.x, c * v.y, c * v.z, c * v.w};
  if (first) {
    acc = t;
    first = false;
  } else if (c == -1.f) {
    acc = float4{acc.x - v.x, acc.y - v.y, acc.z - v.z, acc.w - v.w};
  } else {
    acc = f4add(acc, t);
  }
}

// y[i] = sum_k C(i, k) x[k] for i < RO, k < RI, over float4 vectors with strides (x, y may alias only if RO == RI and
// the caller copies); COEF(i, k) is a constexpr coefficient function
template <int RO, int RI, typename F>
__device__ __forceinline__ void wlin(float4* y, int ys, const float4* x, int xs, F coef) {
  float4 t[RO];
#pragma unroll
  for (int i = 0; i < RO; ++i) {
    bool first = true;
    t[i] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < RI; ++k) wmadd(t[i], first, coef(i, k), x[k * xs]);
  }
#pragma unroll
  for (int i = 0; i < RO; ++i) y[i * ys] = t[i];
}

// 16-B buffer store of a split4_bf16 group: plane xi of a [P][rows][16 B] array is `base + xi * plane` bytes (the
// whole array < 4 GiB, checked by the entry points): 32-bit offset adds instead of a 64-bit multiply per store
__device__ __forceinline__ void wstore(__amdgpu_buffer_rsrc_t r, unsigned off, uint4 u) {
  bstore4(r, off, float4{__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)});
}

// a 4-channel group of a transformed operand in format SF (0 split4_bf16, 1 split4_bits: 16 B; 2 packed bf16 -- the
// bf16-mixed mode's LDS-DMA GEMM operand, round to nearest even: 8 B)
template <int SF>
constexpr unsigned wgb() { return SF == 2 ? 8u : 16u; }
template <int SF>
struct WGroup {
  using T = uint4;
};
template <>
struct WGroup<2> {
  using T = uint2;
};
template <int SF>
__device__ __forceinline__ typename WGroup<SF>::T wgroup(float4 v) {
  if constexpr (SF == 2) return uint2{pk_bf16x2(v.x, v.y), pk_bf16x2(v.z, v.w)};
  else return split4_fmt<SF>(v);
}
template <int SF>
__device__ __forceinline__ void wstore_f(__amdgpu_buffer_rsrc_t r, unsigned off, float4 v) {
  if constexpr (SF == 2) {
    typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
    const uint2 g = wgroup<2>(v);
    __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{g.x, g.y}, r, off, 0, 0);
  } else {
    wstore(r, off, split4_fmt<SF>(v));
  }
}

__device__ __forceinline__ float4 split4_to_f32(float4 r) {  // split4_bf16 group (hi0..hi3 lo0..lo3) -> hi + lo
  const unsigned h01 = __float_as_uint(r.x), h23 = __float_as_uint(r.y);
  const unsigned l01 = __float_as_uint(r.z), l23 = __float_as_uint(r.w);
  return float4{__uint_as_float(h01 << 16) + __uint_as_float(l01 << 16),
                __uint_as_float(h01 & 0xFFFF0000u) + __uint_as_float(l01 & 0xFFFF0000u),
                __uint_as_float(h23 << 16) + __uint_as_float(l23 << 16),
                __uint_as_float(h23 & 0xFFFF0000u) + __uint_as_float(l23 & 0xFFFF0000u)};
}

// x [nb][H][W][C] (fp32, or split4_bf16 groups when XS) -> V [a^2][T][C] split4_bf16, T = nb (H/m) (W/m)
// one thread per (tile, 4-channel group): a^2 coalesced 16-B loads (zeros outside the image), a^2 16-B stores
// GN (nullable): x is a GroupNorm INPUT -- each in-image element is normalized on load, y = silu?(x * scale[b][c] +
// shift[b][c]) (mvae_group_norm_stats_nhwc's affine; the apply pass's arithmetic), so the GroupNorm output feeding this
// conv is never written (zero padding stays zero: it pads y)
struct WinoGn {
  const float* scale;
  const float* shift;
  int silu;
};

template <int MT, bool XS, int GN = 0, int SF = 0>  // GN: 0 none, 1 GroupNorm affine on load, 2 affine + SiLU
__global__ void __launch_bounds__(256) wino_in_kernel(const float* __restrict__ x, uint4* __restrict__ v, int nb, int H,
                                                      int W, int C, WinoGn gn) {
  constexpr int AL = MT + 2;
  const int C4 = C >> 2, th = (H + MT - 1) / MT, tw = (W + MT - 1) / MT;  // (edge tiles zero-filled)
  const long long T = (long long)nb * th * tw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * C4) return;
  const long long t = idx / C4;
  const int c4 = (int)(idx - t * C4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  // buffer loads, zero beyond the image (the descriptor's range check): all 36 loads issue back to back instead of
  // one exec-masked branch -- and one wait -- per patch element
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(x, (unsigned)((long long)nb * H * W * C * 4));
  const unsigned cb = (unsigned)c4 * 16u;
  const unsigned plane = (unsigned)(T * C4) * wgb<SF>(), base = (unsigned)(t * C4 + c4) * wgb<SF>();
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(v, plane * (unsigned)(AL * AL));
  float4 d[AL][AL];
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) {
      const int h = MT * ti - 1 + i, w = MT * tj - 1 + j;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const float4 r = bload4(xr, ok ? ((unsigned)((b * H + h) * W + w) * (unsigned)C) * 4u + cb : OOB);
      d[i][j] = XS ? split4_to_f32(r) : r;
    }
  if constexpr (GN != 0) {
    // normalized after all 36 loads are in flight, in branch-free code (SiLU a template choice: a per-element branch
    // on a runtime flag split the load sequence into one load-wait-compute chain per element, 1.7x the plain
    // transform's time); the hardware reciprocal (1 ulp) instead of an IEEE division. Padding stays zero (it pads
    // the normalized output).
    const float4 sc = *(const float4*)(gn.scale + (long long)b * C + c4 * 4);
    const float4 sh = *(const float4*)(gn.shift + (long long)b * C + c4 * 4);
#pragma unroll
    for (int i = 0; i < AL; ++i)
#pragma unroll
      for (int j = 0; j < AL; ++j) {
        const int h = MT * ti - 1 + i, w = MT * tj - 1 + j;
        const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        float o[4] = {fmaf(d[i][j].x, sc.x, sh.x), fmaf(d[i][j].y, sc.y, sh.y), fmaf(d[i][j].z, sc.z, sh.z),
                      fmaf(d[i][j].w, sc.w, sh.w)};
        if constexpr (GN == 2) {
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = o[k] * __builtin_amdgcn_rcpf(1.f + __expf(-o[k]));
        }
        d[i][j] = ok ? float4{o[0], o[1], o[2], o[3]} : float4{0.f, 0.f, 0.f, 0.f};
      }
  }
  constexpr auto bt = [](int i, int k) { return wino_bt<MT>(i, k); };
#pragma unroll
  for (int j = 0; j < AL; ++j) wlin<AL, AL>(&d[0][j], AL, &d[0][j], AL, bt);  // columns: B^T d
#pragma unroll
  for (int i = 0; i < AL; ++i) wlin<AL, AL>(&d[i][0], 1, &d[i][0], 1, bt);    // rows: (B^T d) B
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) wstore_f<SF>(vr, base + (unsigned)(i * AL + j) * plane, d[i][j]);
}

// G g G^T of a 3x3 filter of float4 groups
template <int MT>
__device__ __forceinline__ void wino_filter(const float4 (&g)[3][3], float4 (&o)[MT + 2][MT + 2]) {
  constexpr int AL = MT + 2;
  constexpr auto gc = [](int i, int k) { return wino_g<MT>(i, k); };
  float4 t[AL][3];
#pragma unroll
  for (int s = 0; s < 3; ++s) wlin<AL, 3>(&t[0][s], 3, &g[0][s], 3, gc);
#pragma unroll
  for (int i = 0; i < AL; ++i) wlin<AL, 3>(&o[i][0], 1, &t[i][0], 1, gc);
}

// forward filters U[a^2][cout][cin] split4_bf16 from KRSC weights w [cout][3][3][cin], g(n, k) = w[n][.][.][k]:
// one thread per (cout n, 4-group of cin k), 9 coalesced 16-B loads, a^2 coalesced 16-B stores
template <int MT, int SF>
__global__ void __launch_bounds__(256) wino_wt_fwd_kernel(const float* __restrict__ w, uint4* __restrict__ u, int cout,
                                                          int cin) {
  constexpr int AL = MT + 2;
  const int K4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * K4) return;
  const int n = (int)(idx / K4), k4 = (int)(idx - (long long)n * K4);
  float4 g[3][3], o[AL][AL];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) g[r][s] = *(const float4*)(w + (((long long)n * 3 + r) * 3 + s) * cin + k4 * 4);
  wino_filter<MT>(g, o);
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j)
      ((typename WGroup<SF>::T*)u)[((long long)(i * AL + j) * cout + n) * K4 + k4] = wgroup<SF>(o[i][j]);
}

// input-gradient filters U'[a^2][cin][cout] split4_bf16, g'(n = cin, k = cout)[r][s] = w[k][2-r][2-s][n]: the source is
// contiguous along n and the destination along k, so a workgroup transposes a 32 (n) x KQ (k groups of 4) block through
// LDS: loads coalesced over n (32 lanes), stores in KQ * 16-B runs over k
constexpr int WDG_N = 32;
// KQ k-groups per workgroup (store runs of KQ x 16 B), the a^2 positions staged through LDS in passes of PP (the stage
// is PP x 32 x KQ x 16 B): m = 4 large filters (cin x cout >= 2^20: c4's 16x16 / 8x8 levels) take 8 x 16 B runs in two
// passes of 18 positions (72 KB, 256 threads; 8x8x2048: 274 -> 205 us), the small ones one pass of 4 x 16 B (fewer
// barriers: the two-pass form measured 30-40 % slower on them); m = 2 one pass of 8
template <int MT, bool BIG>
constexpr int wdg_kq() { return (MT == 2 || BIG) ? 8 : 4; }
template <int MT, bool BIG>
constexpr int wdg_pp() { return MT == 2 ? 16 : BIG ? 18 : 36; }
template <int MT, bool BIG, int SF>
__global__ void __launch_bounds__(256) wino_wt_dgrad_kernel(const float* __restrict__ w, uint4* __restrict__ u,
                                                            int cout, int cin) {
  constexpr int AL = MT + 2, KQ = wdg_kq<MT, BIG>(), NT = WDG_N * KQ, PP = wdg_pp<MT, BIG>();
  static_assert((AL * AL) % PP == 0, "position passes");
  using GT = typename WGroup<SF>::T;
  __shared__ GT lds[PP][WDG_N][KQ];
  const int K4 = cout >> 2;
  const int n0 = blockIdx.x * WDG_N, kb = blockIdx.y * KQ;
  const int nl = threadIdx.x % WDG_N, kq = threadIdx.x / WDG_N;
  const int n = n0 + nl, k4 = kb + kq;
  const bool act = n < cin && k4 < K4;
  float4 o[AL][AL];
  if (act) {
    float4 g[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) e[q] = w[(((long long)(k4 * 4 + q) * 3 + (2 - r)) * 3 + (2 - s)) * cin + n];
        g[r][s] = float4{e[0], e[1], e[2], e[3]};
      }
    wino_filter<MT>(g, o);
  }
#pragma unroll
  for (int p0 = 0; p0 < AL * AL; p0 += PP) {
    if (act) {
#pragma unroll
      for (int i = 0; i < AL; ++i)
#pragma unroll
        for (int j = 0; j < AL; ++j)
          if (i * AL + j >= p0 && i * AL + j < p0 + PP) lds[i * AL + j - p0][nl][kq] = wgroup<SF>(o[i][j]);
    }
    __syncthreads();
    for (int e = threadIdx.x; e < PP * WDG_N * KQ; e += NT) {
      const int xi = e / (WDG_N * KQ), rem = e % (WDG_N * KQ);
      const int nn = n0 + rem / KQ, kk = kb + rem % KQ;
      if (nn < cin && kk < K4) ((GT*)u)[((long long)(p0 + xi) * cin + nn) * K4 + kk] = lds[xi][rem / KQ][rem % KQ];
    }
    __syncthreads();
  }
}

// output transform operands
struct WinoOut {
  const float* m;      // [a^2][T][N] fp32 GEMM results
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

// M -> y = A^T M A (+ bias) (+ residual). A thread covers whole 32-pixel blocks of the statistics layouts: TR tile rows
// x CT tiles of one image, i.e. an (TR m) x WSEG pixel window with WSEG = min(W, 32) (W in {8, 16}: the full width, TR
// = 32 / (m W) tile rows when that is > 1; W a multiple of 32: one tile row of a 32-pixel column segment) -- NBK = TR m
// WSEG / 32 blocks, each block's sums in registers (compile-time index). Threads of a group are consecutive 4-channel
// groups (coalesced 16-B loads / stores).
template <int MT, int WSEG>
struct WinoOutGeo {
  static constexpr int TR = MT * WSEG >= 32 ? 1 : 32 / (MT * WSEG);
  static constexpr int CT = WSEG / MT;
  static constexpr int NBK = TR * MT * WSEG / 32;
};

template <int MT, int WSEG, bool GNB, bool ST>
__global__ void __launch_bounds__(256) wino_out_kernel(WinoOut p) {
  constexpr int AL = MT + 2;
  using Geo = WinoOutGeo<MT, WSEG>;
  constexpr int TR = Geo::TR, CT = Geo::CT, NBK = Geo::NBK;
  const int N = p.N, N4 = N >> 2, th = p.H / MT, tw = p.W / MT, nseg = p.W / WSEG;
  const long long T = (long long)p.nb * th * tw;
  const unsigned mplane = (unsigned)(T * N4 * 16);
  const __amdgpu_buffer_rsrc_t mr = make_rsrc(p.m, mplane * (unsigned)(AL * AL));
  const long long ngrp = (long long)p.nb * (th / TR) * nseg;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= ngrp * N4) return;
  const long long grp = idx / N4;
  const int c4 = (int)(idx - grp * N4);
  const int seg = (int)(grp % nseg);
  const long long rg = grp / nseg;
  const int b = (int)(rg / (th / TR)), ti0 = (int)(rg % (th / TR)) * TR, tj0 = seg * CT;
  const float4 bv = p.bias ? *(const float4*)(p.bias + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
  // y / residual / GroupNorm input through buffer descriptors (32-bit offsets; a null residual is an empty range,
  // whose loads return zeros: no branch and no wait per pixel)
  const unsigned ybytes = (unsigned)((long long)p.nb * p.H * p.W * N * 4);
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, ybytes);
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(p.res ? p.res : p.y, p.res ? ybytes : 0u);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(GNB ? p.gx : p.y, GNB ? ybytes : 0u);
  // (the GroupNorm-backward partials of one 32-pixel block are summed in fp32 -- 32 terms -- and stored as fp64: half
  // the accumulator registers of fp64 sums, which with the full M tile in registers held this variant to one wave per
  // SIMD)
  double s0[NBK], s1[NBK];
  float g0[GNB ? NBK : 1][4], g1[GNB ? NBK : 1][4];
#pragma unroll
  for (int q = 0; q < NBK; ++q) s0[q] = s1[q] = 0.0;
#pragma unroll
  for (int q = 0; q < (GNB ? NBK : 1); ++q)
#pragma unroll
    for (int u = 0; u < 4; ++u) g0[q][u] = g1[q][u] = 0.f;
  float ggm[4] = {0.f, 0.f, 0.f, 0.f}, gbt[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (GNB) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      ggm[e] = p.gamma[c4 * 4 + e];
      gbt[e] = p.beta[c4 * 4 + e];
    }
  }
  const int cpg = GNB ? N / p.groups : 1;
  const bool silu = GNB && p.silu != 0;
#pragma unroll
  for (int tr = 0; tr < TR; ++tr)
#pragma unroll 1
    for (int tq = 0; tq < CT; ++tq) {
      const int ti = ti0 + tr, tj = tj0 + tq;
      const long long t = ((long long)b * th + ti) * tw + tj;
      const unsigned mbase = (unsigned)(t * N4 + c4) * 16u;
      constexpr auto at = [](int i, int k) { return wino_at<MT>(i, k); };
      float4 r[MT][AL];
      float4 mv[AL][AL];
#pragma unroll
      for (int i = 0; i < AL; ++i)
#pragma unroll
        for (int j = 0; j < AL; ++j) mv[i][j] = bload4(mr, mbase + (unsigned)(i * AL + j) * mplane);
#pragma unroll
      for (int j = 0; j < AL; ++j) wlin<MT, AL>(&r[0][j], AL, &mv[0][j], AL, at);  // A^T M
#pragma unroll
      for (int a = 0; a < MT; ++a) {
        float4 o[MT];
        wlin<MT, AL>(o, 1, &r[a][0], 1, at);  // (A^T M) A
        const int row = ti * MT + a;
        const int q = ((tr * MT + a) * WSEG) / 32;  // block within the group (compile-time: tr, a unrolled)
#pragma unroll
        for (int e = 0; e < MT; ++e) {
          const unsigned off = ((unsigned)((b * p.H + row) * p.W + tj * MT + e) * (unsigned)N + (unsigned)c4 * 4u) * 4u;
          // (the input-gradient transform with GroupNorm partials has no bias / residual: mvae_winograd_output_gnbwd)
          float4 val = GNB ? o[e] : f4add(f4add(o[e], bv), bload4(rr, off));
          bstore4(yr, off, val);
          if constexpr (ST) {
            s0[q] += ((double)val.x + (double)val.y) + ((double)val.z + (double)val.w);
            s1[q] += ((double)val.x * val.x + (double)val.y * val.y) + ((double)val.z * val.z + (double)val.w * val.w);
          }
          if constexpr (GNB) {
            const float4 x4 = bload4(xr, off);
            const int bg = b * p.groups + (c4 * 4) / cpg;  // (a 4-channel group never straddles a GroupNorm group)
            const float mu = p.mean[bg], rs = p.rstd[bg];
            const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, vs[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              float d = vs[u];
              const float xh = (xs[u] - mu) * rs;
              // (branch-free: a per-element branch on the uniform silu flag held this variant to one wave per SIMD)
              const float yn = xh * ggm[u] + gbt[u];
              const float sg = sigmoid_f(yn);
              const float ds = d * sg * (1.f + yn * (1.f - sg));
              d = silu ? ds : d;
              g0[q][u] += d;
              g1[q][u] += d * xh;
            }
          }
        }
      }
    }
#pragma unroll
  for (int q = 0; q < NBK; ++q) {
    // first pixel of local block q: (q 32 / WSEG) rows down, at the group's column segment
    const long long blk = (((long long)b * p.H + ti0 * MT + (q * 32) / WSEG) * p.W + seg * WSEG) >> 5;
    if constexpr (ST) *(double2*)(p.gn_part + (blk * N4 + c4) * 2) = double2{s0[q], s1[q]};
    if constexpr (GNB) {
      double* gp = p.gnb_part + (blk * N + c4 * 4) * 2;
#pragma unroll
      for (int u = 0; u < 4; ++u) *(double2*)(gp + 2 * u) = double2{(double)g0[q][u], (double)g1[q][u]};
    }
  }
}

// M -> y = A^T M A (+ bias) (+ residual) for any H, W (edge tiles cut at the image border): one thread per (tile,
// 4-channel group), no statistics (the GroupNorm after such a conv computes its own)
template <int MT>
__global__ void __launch_bounds__(256) wino_out_any_kernel(WinoOut p) {
  constexpr int AL = MT + 2;
  const int N = p.N, N4 = N >> 2, th = (p.H + MT - 1) / MT, tw = (p.W + MT - 1) / MT;
  const long long T = (long long)p.nb * th * tw;
  const unsigned mplane = (unsigned)(T * N4 * 16);
  const __amdgpu_buffer_rsrc_t mr = make_rsrc(p.m, mplane * (unsigned)(AL * AL));
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * N4) return;
  const long long t = idx / N4;
  const int c4 = (int)(idx - t * N4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  const float4 bv = p.bias ? *(const float4*)(p.bias + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
  float4 mv[AL][AL];
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) mv[i][j] = bload4(mr, (unsigned)(t * N4 + c4) * 16u + (unsigned)(i * AL + j) * mplane);
  constexpr auto at = [](int i, int k) { return wino_at<MT>(i, k); };
  float4 r[MT][AL];
#pragma unroll
  for (int j = 0; j < AL; ++j) wlin<MT, AL>(&r[0][j], AL, &mv[0][j], AL, at);
#pragma unroll
  for (int a = 0; a < MT; ++a) {
    float4 o[MT];
    wlin<MT, AL>(o, 1, &r[a][0], 1, at);
    const int row = ti * MT + a;
#pragma unroll
    for (int e = 0; e < MT; ++e) {
      const int col = tj * MT + e;
      if (row < p.H && col < p.W) {
        const long long off = (((long long)b * p.H + row) * p.W + col) * N + c4 * 4;
        float4 val = f4add(o[e], bv);
        if (p.res) val = f4add(val, *(const float4*)(p.res + off));
        *(float4*)(p.y + off) = val;
      }
    }
  }
}

// Where the output-gradient 4-group k4 of low-resolution pixel (h, w) of image b lives (byte offset): the dy [nb][H][W][K]
// of a conv; or, UPS (the Upsample conv run as 4 class convs on its low-resolution input, K = 4 cout, k4 = class pq x
// cout / 4 + c4), the class-pq sub-image of the full-resolution dy [nb][2H][2W][cout] -- pixel (2h + p, 2w + q)
template <bool UPS>
struct DySrc {
  unsigned pix0, chan, rowb;  // per image / class: base pixel, byte offset of the 4-group, bytes per pixel
  int H, W;
  __device__ DySrc(int b, int k4, int H_, int W_, int K) : H(H_), W(W_) {
    if constexpr (UPS) {
      const int cq4 = K >> 4, pq = k4 / cq4, c4 = k4 - pq * cq4;  // (K / 4 = cout: 4-groups per class = K / 16)
      pix0 = (unsigned)((b * 2 * H + (pq >> 1)) * 2 * W + (pq & 1));
      chan = (unsigned)c4 * 16u;
      rowb = (unsigned)(K >> 2) * 4u;
    } else {
      pix0 = (unsigned)(b * H * W);
      chan = (unsigned)k4 * 16u;
      rowb = (unsigned)K * 4u;
    }
  }
  __device__ unsigned off(int h, int w) const {  // (h, w) inside the low-resolution image
    if constexpr (UPS) return (pix0 + (unsigned)(2 * h * 2 * W + 2 * w)) * rowb + chan;
    else return (pix0 + (unsigned)(h * W + w)) * rowb + chan;
  }
};

// dy [nb][H][W][K] (fp32, or split4_bf16 groups when XS; UPS: the Upsample conv's class sub-images, DySrc) -> D' =
// A D A^T [a^2][T][K] split4_bf16: one thread per (tile, 4-group)
template <int MT, bool XS, int SF = 0, bool UPS = false>
__global__ void __launch_bounds__(256) wino_dy_kernel(const float* __restrict__ dy, uint4* __restrict__ d, int nb, int H,
                                                      int W, int K) {
  constexpr int AL = MT + 2;
  const int K4 = K >> 2, th = (H + MT - 1) / MT, tw = (W + MT - 1) / MT;
  const long long T = (long long)nb * th * tw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * K4) return;
  const long long t = idx / K4;
  const int k4 = (int)(idx - t * K4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(dy, (unsigned)((long long)nb * H * W * K * 4));
  const DySrc<UPS> src(b, k4, H, W, K);
  const unsigned plane = (unsigned)(T * K4) * wgb<SF>(), base = (unsigned)(t * K4 + k4) * wgb<SF>();
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(d, plane * (unsigned)(AL * AL));
  float4 v[MT][MT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int e = 0; e < MT; ++e) {
      const int h = MT * ti + a, w = MT * tj + e;  // (pixels past the image edge carry no gradient: zero)
      const float4 r = bload4(dr, (h < H && w < W) ? src.off(h, w) : OOB);
      v[a][e] = XS ? split4_to_f32(r) : r;
    }
  constexpr auto ac = [](int i, int k) { return wino_at<MT>(k, i); };  // A = (A^T)^T
  float4 c[AL][MT], o[AL][AL];
#pragma unroll
  for (int e = 0; e < MT; ++e) wlin<AL, MT>(&c[0][e], MT, &v[0][e], MT, ac);
#pragma unroll
  for (int i = 0; i < AL; ++i) wlin<AL, MT>(&o[i][0], 1, &c[i][0], 1, ac);
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) wstore_f<SF>(vr, base + (unsigned)(i * AL + j) * plane, o[i][j]);
}

// dy -> both backward operands in one pass over dy (a conv whose input and weight gradients both run the Winograd
// form): V' = B^T P B of the a x a patch P (the input gradient's transformed input, as wino_in_kernel on dy) and
// D' = A D A^T of the m x m tile D = P[1..m][1..m] inside it (the weight gradient's transformed output gradient, as
// wino_dy_kernel) -- the separate kernels each read all of dy. One thread per (tile, 4-group); D' one output row at a
// time (181-215 VGPRs: the patch plus one row; 2 waves per SIMD, as the input transform).
template <int MT, bool XS, int SF = 0, bool UPS = false>
__global__ void __launch_bounds__(256) wino_dy2_kernel(const float* __restrict__ dy, uint4* __restrict__ v,
                                                       uint4* __restrict__ d, int nb, int H, int W, int K) {
  constexpr int AL = MT + 2;
  const int K4 = K >> 2, th = (H + MT - 1) / MT, tw = (W + MT - 1) / MT;
  const long long T = (long long)nb * th * tw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * K4) return;
  const long long t = idx / K4;
  const int k4 = (int)(idx - t * K4);
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(dy, (unsigned)((long long)nb * H * W * K * 4));
  const DySrc<UPS> src(b, k4, H, W, K);
  const unsigned plane = (unsigned)(T * K4) * wgb<SF>(), base = (unsigned)(t * K4 + k4) * wgb<SF>();
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(v, plane * (unsigned)(AL * AL));
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(d, plane * (unsigned)(AL * AL));
  float4 p[AL][AL];
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) {
      const int h = MT * ti - 1 + i, w = MT * tj - 1 + j;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const float4 r = bload4(xr, ok ? src.off(h, w) : OOB);
      p[i][j] = XS ? split4_to_f32(r) : r;
    }
#pragma unroll
  for (int i = 0; i < AL; ++i) {  // D' row i = (A D)[i] A^T, A[i][u] = A^T[u][i]
    float4 ci[MT], o[AL];
#pragma unroll
    for (int e = 0; e < MT; ++e) {
      bool first = true;
      ci[e] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < MT; ++u) wmadd(ci[e], first, wino_at<MT>(u, i), p[1 + u][1 + e]);
    }
#pragma unroll
    for (int j = 0; j < AL; ++j) {
      bool first = true;
      o[j] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < MT; ++e) wmadd(o[j], first, wino_at<MT>(e, j), ci[e]);
    }
#pragma unroll
    for (int j = 0; j < AL; ++j) wstore_f<SF>(dr, base + (unsigned)(i * AL + j) * plane, o[j]);
  }
  constexpr auto bt = [](int i, int k) { return wino_bt<MT>(i, k); };
#pragma unroll
  for (int j = 0; j < AL; ++j) wlin<AL, AL>(&p[0][j], AL, &p[0][j], AL, bt);
#pragma unroll
  for (int i = 0; i < AL; ++i) wlin<AL, AL>(&p[i][0], 1, &p[i][0], 1, bt);
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) wstore_f<SF>(vr, base + (unsigned)(i * AL + j) * plane, p[i][j]);
}

// The Upsample conv (nearest x2, then a 3x3 / pad-1 conv: encoder_decoder.py:194-209) as four 3x3 / pad-1 convs on the
// LOW-resolution input, one per output parity class (p, q): output pixel (2i + p, 2j + q) = sum over taps (r, s) of
// w[r][s] x[i + floor((p + r - 1) / 2)][j + floor((q + s - 1) / 2)], i.e. class kernel K_pq[a][b] = sum of the taps
// (r, s) with e_p(r) = a, e_q(s) = b, e_0 = (0, 1, 1), e_1 = (1, 1, 2) (the sub-pixel form's tap sums, embedded in a
// 3x3 support). The four classes share the input transform V of x: one position GEMM over N = 4 cout, (m+2)^2 / (4 m^2)
// MACs per output pixel per channel pair instead of the sub-pixel form's 4 (0.56x at m = 4).
__host__ __device__ constexpr int ups_tap(int p, int r) { return p == 0 ? (r == 0 ? 0 : 1) : (r == 2 ? 2 : 1); }

// kc [4 cout][3][3][cin] (row pq * cout + k) from w [cout][3][3][cin]: one thread per (class, k, 4-group of cin)
__global__ void __launch_bounds__(256) wino_ups_weights_kernel(const float* __restrict__ w, float* __restrict__ kc,
                                                               int cout, int cin) {
  const int C4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 4LL * cout * C4) return;
  const int c4 = (int)(idx % C4);
  const long long kq = idx / C4;
  const int k = (int)(kq % cout), pq = (int)(kq / cout), p = pq >> 1, q = pq & 1;
  float4 o[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int bb = 0; bb < 3; ++bb) o[a][bb] = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      const float4 v = *(const float4*)(w + (((long long)k * 3 + r) * 3 + s2) * cin + c4 * 4);
      o[ups_tap(p, r)][ups_tap(q, s2)] = f4add(o[ups_tap(p, r)][ups_tap(q, s2)], v);
    }
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int bb = 0; bb < 3; ++bb) *(float4*)(kc + ((kq * 3 + a) * 3 + bb) * cin + c4 * 4) = o[a][bb];
}

// dw [cout][3][3][cin] = beta * dw + sum over the classes of the class kernels' gradients dkc [4 cout][3][3][cin] at the
// taps each original tap feeds (the transpose of wino_ups_weights_kernel), fixed class order
__global__ void __launch_bounds__(256) wino_ups_fold_kernel(const float* __restrict__ dkc, float* __restrict__ dw,
                                                            float beta, int cout, int cin) {
  const int C4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * C4) return;
  const int k = (int)(idx / C4), c4 = (int)(idx - (long long)k * C4);
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s2 = 0; s2 < 3; ++s2) {
      float4 acc = float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int pq = 0; pq < 4; ++pq) {
        const long long row = (long long)pq * cout + k;
        acc = f4add(acc, *(const float4*)(dkc + ((row * 3 + ups_tap(pq >> 1, r)) * 3 + ups_tap(pq & 1, s2)) * cin +
                                          c4 * 4));
      }
      float4* q = (float4*)(dw + (((long long)k * 3 + r) * 3 + s2) * cin + c4 * 4);
      if (beta != 0.f) {
        const float4 old = *q;
        acc = float4{fmaf(beta, old.x, acc.x), fmaf(beta, old.y, acc.y), fmaf(beta, old.z, acc.z),
                     fmaf(beta, old.w, acc.w)};
      }
      *q = acc;
    }
}

// M [a^2][T][4 cout] (class-major columns) -> y [nb][2H][2W][cout] = A^T M_pq A at pixels (2i + p, 2j + q) (+ bias):
// one thread per (low-resolution tile, class, 4-channel group)
template <int MT>
__global__ void __launch_bounds__(256) wino_out_ups_kernel(WinoOut p) {
  constexpr int AL = MT + 2;
  const int N = p.N, N4 = N >> 2, K4 = N, th = (p.H + MT - 1) / MT, tw = (p.W + MT - 1) / MT;  // (K4: 4 N / 4)
  const long long T = (long long)p.nb * th * tw;
  const unsigned mplane = (unsigned)(T * K4 * 16);
  const __amdgpu_buffer_rsrc_t mr = make_rsrc(p.m, mplane * (unsigned)(AL * AL));
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= T * K4) return;
  const long long t = idx / K4;
  const int k4 = (int)(idx - t * K4), pq = k4 / N4, c4 = k4 - pq * N4;
  const int tj = (int)(t % tw), ti = (int)((t / tw) % th), b = (int)(t / ((long long)tw * th));
  const float4 bv = p.bias ? *(const float4*)(p.bias + c4 * 4) : float4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t yr = make_rsrc(p.y, (unsigned)((long long)p.nb * 4 * p.H * p.W * N * 4));
  float4 mv[AL][AL];
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) mv[i][j] = bload4(mr, (unsigned)(t * K4 + k4) * 16u + (unsigned)(i * AL + j) * mplane);
  constexpr auto at = [](int i, int k) { return wino_at<MT>(i, k); };
  float4 r[MT][AL];
#pragma unroll
  for (int j = 0; j < AL; ++j) wlin<MT, AL>(&r[0][j], AL, &mv[0][j], AL, at);
#pragma unroll
  for (int a = 0; a < MT; ++a) {
    float4 o[MT];
    wlin<MT, AL>(o, 1, &r[a][0], 1, at);
    const int row = ti * MT + a;
#pragma unroll
    for (int e = 0; e < MT; ++e) {
      const int col = tj * MT + e;
      const unsigned off =
          ((unsigned)((b * 2 * p.H + 2 * row + (pq >> 1)) * 2 * p.W + 2 * col + (pq & 1)) * (unsigned)N + c4 * 4) * 4u;
      bstore4(yr, (row < p.H && col < p.W) ? off : OOB, f4add(o[e], bv));
    }
  }
}

// dw [cout][3][3][cin] = beta * dw + G^T M G, M [a^2][cout][cin] fp32: one thread per (k, 4-group of c)
template <int MT>
__global__ void __launch_bounds__(256) wino_wout_kernel(const float* __restrict__ m, float* __restrict__ dw, float beta,
                                                        int cout, int cin) {
  constexpr int AL = MT + 2;
  const int C4 = cin >> 2;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * C4) return;
  const long long mn = (long long)cout * cin;
  float4 mv[AL][AL];
#pragma unroll
  for (int i = 0; i < AL; ++i)
#pragma unroll
    for (int j = 0; j < AL; ++j) mv[i][j] = *(const float4*)(m + (i * AL + j) * mn + idx * 4);
  constexpr auto gt = [](int r, int i) { return wino_g<MT>(i, r); };  // G^T
  float4 r[3][AL], o[3][3];
#pragma unroll
  for (int j = 0; j < AL; ++j) wlin<3, AL>(&r[0][j], AL, &mv[0][j], AL, gt);
#pragma unroll
  for (int i = 0; i < 3; ++i) wlin<3, AL>(&o[i][0], 1, &r[i][0], 1, gt);
  const int k = (int)(idx / C4), c4 = (int)(idx - (long long)k * C4);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float4* q = (float4*)(dw + (((long long)k * 3 + i) * 3 + j) * cin + c4 * 4);
      float4 val = o[i][j];
      if (beta != 0.f) {
        const float4 old = *q;
        val = float4{fmaf(beta, old.x, val.x), fmaf(beta, old.y, val.y), fmaf(beta, old.z, val.z),
                     fmaf(beta, old.w, val.w)};
      }
      *q = val;
    }
}

static long long wino_tiles(int nb, int h, int w, int mt) {
  return (long long)nb * ((h + mt - 1) / mt) * ((w + mt - 1) / mt);
}

// any image size (edge tiles zero-filled / cut), channel counts % 4, every operand < 4 GiB
static bool wino_geom_ok(int mt, int nb, int h, int w, int cin, int cout) {
  // (the transforms address the whole [P][T][c] array through one buffer descriptor: < 4 GiB)
  return (mt == 2 || mt == 4) && nb > 0 && h > 0 && w > 0 && cin > 0 && cout > 0 && cin % 4 == 0 && cout % 4 == 0 &&
         (long long)nb * h * w * std::max(cin, cout) * 4 <= MAX_DESC_BYTES &&
         (long long)(mt + 2) * (mt + 2) * wino_tiles(nb, h, w, mt) * std::max(cin, cout) * 4 <= MAX_DESC_BYTES;
}

// the blocked output transform (statistics in the 32-pixel-block layouts): whole tiles, and thread groups that are
// whole 32-pixel blocks -- h % 4 == 0 covers every (m, w) pair (m = 2 at w = 8 takes 2 tile rows per group)
static bool wino_blocks_ok(int h, int w) { return h % 4 == 0 && (w == 8 || w == 16 || (w >= 32 && w % 32 == 0)); }

static int egrid256(long long n) { return (int)std::min<long long>((n + 255) / 256, 1LL << 30); }

// every GEMM arithmetic: 3xBF16 (V / U value-split into split4_bf16), bf16 (the same groups; the GEMM stages the hi
// halves) and exact fp32 (bit split, split4_bits: the f32-input MFMA reassembles the transforms' fp32 words exactly)
static int wino_sf() { return math_mode() == MATH_FP32 ? 1 : math_mode() == MATH_BF16 ? 2 : 0; }
// a pre-split INPUT is a 3xBF16 value split: there is none in the exact mode
static bool wino_split_in_ok(int split) {
  if (!split || wino_sf() != 1) return true;
  set_error("winograd: pre-split (3xBF16) inputs are not used in the exact fp32 arithmetic");
  return false;
}

// FN<MT, SF>(args...) for the transform layout of the current arithmetic (sf: wino_sf())
#define WINO_GO(FN, MT, ...)                        \
  do {                                              \
    if (sf == 1) FN<MT, 1>(__VA_ARGS__);            \
    else if (sf == 2) FN<MT, 2>(__VA_ARGS__);       \
    else FN<MT, 0>(__VA_ARGS__);                    \
  } while (0)

template <int MT, int SF>
static void wt_go(const float* w, void* u, int cin, int cout, int dgrad, hipStream_t st) {
  if (dgrad) {
    if constexpr (MT == 4) {
      if ((long long)cin * cout >= (1LL << 20)) {
        hipLaunchKernelGGL((wino_wt_dgrad_kernel<4, true, SF>), dim3(cdiv(cin, WDG_N), cdiv(cout / 4, wdg_kq<4, true>())),
                           dim3(WDG_N * wdg_kq<4, true>()), 0, st, w, (uint4*)u, cout, cin);
        return;
      }
    }
    hipLaunchKernelGGL((wino_wt_dgrad_kernel<MT, false, SF>), dim3(cdiv(cin, WDG_N), cdiv(cout / 4, wdg_kq<MT, false>())),
                       dim3(WDG_N * wdg_kq<MT, false>()), 0, st, w, (uint4*)u, cout, cin);
  } else {
    hipLaunchKernelGGL((wino_wt_fwd_kernel<MT, SF>), dim3(egrid256((long long)cout * (cin / 4))), dim3(256), 0, st, w,
                       (uint4*)u, cout, cin);
  }
}

// gn: 0 plain (xs: x pre-split), 1 GroupNorm affine on load, 2 affine + SiLU
template <int MT, int SF>
static void in_go(const float* x, void* v, int nb, int h, int w, int c, int xs, int gn, WinoGn p, hipStream_t st) {
  const dim3 g(egrid256(wino_tiles(nb, h, w, MT) * (c / 4)));
  if constexpr (SF != 1) {
    if (xs) {
      hipLaunchKernelGGL((wino_in_kernel<MT, true, 0, SF>), g, dim3(256), 0, st, x, (uint4*)v, nb, h, w, c, p);
      return;
    }
  }
  if (gn == 2) hipLaunchKernelGGL((wino_in_kernel<MT, false, 2, SF>), g, dim3(256), 0, st, x, (uint4*)v, nb, h, w, c, p);
  else if (gn == 1) hipLaunchKernelGGL((wino_in_kernel<MT, false, 1, SF>), g, dim3(256), 0, st, x, (uint4*)v, nb, h, w, c, p);
  else hipLaunchKernelGGL((wino_in_kernel<MT, false, 0, SF>), g, dim3(256), 0, st, x, (uint4*)v, nb, h, w, c, p);
}

// both = 0: D' only (wino_dy_kernel); 1: V' and D' in one pass (wino_dy2_kernel); ups: the Upsample conv's class
// sub-images of the full-resolution dy (k = 4 cout)
template <int MT, int SF>
static void dy_go(const float* dy, void* v, void* d, int nb, int h, int w, int k, int xs, bool both, hipStream_t st,
                  bool ups = false) {
  const dim3 g(egrid256(wino_tiles(nb, h, w, MT) * (k / 4)));
  uint4 *vv = (uint4*)v, *dd = (uint4*)d;
  if (ups) {  // (no pre-split form: the Upsample conv's dy is never split)
    if (both) hipLaunchKernelGGL((wino_dy2_kernel<MT, false, SF, true>), g, dim3(256), 0, st, dy, vv, dd, nb, h, w, k);
    else hipLaunchKernelGGL((wino_dy_kernel<MT, false, SF, true>), g, dim3(256), 0, st, dy, dd, nb, h, w, k);
    return;
  }
  if constexpr (SF != 1) {
    if (xs) {
      if (both) hipLaunchKernelGGL((wino_dy2_kernel<MT, true, SF>), g, dim3(256), 0, st, dy, vv, dd, nb, h, w, k);
      else hipLaunchKernelGGL((wino_dy_kernel<MT, true, SF>), g, dim3(256), 0, st, dy, dd, nb, h, w, k);
      return;
    }
  }
  if (both) hipLaunchKernelGGL((wino_dy2_kernel<MT, false, SF>), g, dim3(256), 0, st, dy, vv, dd, nb, h, w, k);
  else hipLaunchKernelGGL((wino_dy_kernel<MT, false, SF>), g, dim3(256), 0, st, dy, dd, nb, h, w, k);
}

template <int MT, int WSEG>
static void wino_out_go(WinoOut& p, bool gnb, hipStream_t st) {
  using Geo = WinoOutGeo<MT, WSEG>;
  const long long groups = (long long)p.nb * (p.H / MT / Geo::TR) * (p.W / WSEG);
  const dim3 g(egrid256(groups * (p.N / 4)));
  if (gnb) hipLaunchKernelGGL((wino_out_kernel<MT, WSEG, true, false>), g, dim3(256), 0, st, p);
  else if (p.gn_part) hipLaunchKernelGGL((wino_out_kernel<MT, WSEG, false, true>), g, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((wino_out_kernel<MT, WSEG, false, false>), g, dim3(256), 0, st, p);
}

static int wino_out_launch(WinoOut& p, int tile, bool gnb, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!wino_blocks_ok(p.H, p.W)) {  // (callers reject statistics here)
    const dim3 g(egrid256(wino_tiles(p.nb, p.H, p.W, tile) * (p.N / 4)));
    if (tile == 2) hipLaunchKernelGGL(wino_out_any_kernel<2>, g, dim3(256), 0, st, p);
    else hipLaunchKernelGGL(wino_out_any_kernel<4>, g, dim3(256), 0, st, p);
    return launch_status();
  }
  const int wseg = std::min(p.W, 32);
  if (tile == 2) {
    if (wseg == 8) wino_out_go<2, 8>(p, gnb, st);
    else if (wseg == 16) wino_out_go<2, 16>(p, gnb, st);
    else wino_out_go<2, 32>(p, gnb, st);
  } else {
    if (wseg == 8) wino_out_go<4, 8>(p, gnb, st);
    else if (wseg == 16) wino_out_go<4, 16>(p, gnb, st);
    else wino_out_go<4, 32>(p, gnb, st);
  }
  return launch_status();
}

}  // namespace mvae

using namespace mvae;

extern "C" {

// U = the a^2 transformed filters in split4_bf16 ([a^2][cout][cin] forward, [a^2][cin][cout] for the input gradient
// when dgrad != 0) of KRSC 3x3 weights w [cout][3][3][cin]; tile = m (2 or 4)
int mvae_winograd_weight_transform(const float* w, void* u, int cin, int cout, int dgrad, int tile, void* stream) {
  if (!w || !u || cin <= 0 || cout <= 0 || cin % 4 || cout % 4 || !al16(w) || !al16(u) || (tile != 2 && tile != 4)) {
    set_error("winograd_weight_transform: cin, cout multiples of 4, 16-B aligned w / u, tile 2 or 4");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const int sf = wino_sf();
  if (tile == 2) WINO_GO(wt_go, 2, w, u, cin, cout, dgrad, st);
  else WINO_GO(wt_go, 4, w, u, cin, cout, dgrad, st);
  return launch_status();
}

// V [a^2][T][c] split4_bf16 of x [nb][h][w][c] (fp32, or split4_bf16 groups when x_split), T = nb (h/m) (w/m)
int mvae_winograd_input_transform(const float* x, void* v, int nb, int h, int w, int c, int x_split, int tile,
                                  void* stream) {
  if (!x || !v || !wino_geom_ok(tile, nb, h, w, c, c) || !al16(x) || !al16(v)) {
    set_error("winograd_input_transform: tile 2 or 4, c %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  if (!wino_split_in_ok(x_split)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int sf = wino_sf();
  if (tile == 2) WINO_GO(in_go, 2, x, v, nb, h, w, c, x_split, 0, WinoGn{}, st);
  else WINO_GO(in_go, 4, x, v, nb, h, w, c, x_split, 0, WinoGn{}, st);
  return launch_status();
}

// V of silu?(GroupNorm(x)) without that GroupNorm output ever written: x the GroupNorm's input, scale / shift [nb][c]
// from mvae_group_norm_stats_nhwc
int mvae_winograd_input_transform_gn(const float* x, const float* scale, const float* shift, int silu, void* v, int nb,
                                     int h, int w, int c, int tile, void* stream) {
  if (!x || !v || !scale || !shift || !wino_geom_ok(tile, nb, h, w, c, c) || !al16(x) || !al16(v) || !al16(scale) ||
      !al16(shift)) {
    set_error("winograd_input_transform_gn: tile 2 or 4, c %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const WinoGn gn{scale, shift, silu};
  const int sf = wino_sf(), mode = silu ? 2 : 1;
  if (tile == 2) WINO_GO(in_go, 2, x, v, nb, h, w, c, 0, mode, gn, st);
  else WINO_GO(in_go, 4, x, v, nb, h, w, c, 0, mode, gn, st);
  return launch_status();
}

// M [a^2][T][n_out] fp32 = V_xi [T][k_in] . U_xi [n_out][k_in]^T for the a^2 positions xi: one batched launch of the
// implicit-GEMM core on pre-split operands
int mvae_winograd_gemm(const void* v, const void* u, float* m, long long tiles, int k_in, int n_out, int tile,
                       void* stream) {
  if (!v || !u || !m || tiles <= 0 || k_in <= 0 || n_out <= 0 || k_in % 4 || n_out % 4 || !al16(v) || !al16(u) ||
      !al16(m) || tiles * std::max(k_in, n_out) * 4 > MAX_DESC_BYTES || tiles > (1LL << 30) ||
      (tile != 2 && tile != 4)) {
    set_error("winograd_gemm: k_in, n_out multiples of 4, 16-B aligned, one position < 4 GiB, tile 2 or 4");
    return MVAE_EINVAL;
  }
  // (bf16-mixed: V and U packed bf16, 2 B per element, through the LDS-DMA main loop -- 16-B rows need k_in % 8)
  const bool pk = wino_sf() == 2;
  if (pk && k_in % 8) {
    set_error("winograd_gemm: the bf16 (packed) operands need k_in %% 8 == 0");
    return MVAE_EINVAL;
  }
  const unsigned eb = pk ? 2u : 4u;
  GemmArgs a{};
  a.M = (int)tiles; a.N = n_out; a.K = k_in; a.batch = (tile + 2) * (tile + 2);
  a.A = (const float*)v; a.lda = k_in; a.sA = tiles * k_in;
  a.B = (const float*)u; a.ldb = k_in; a.sB = (long long)n_out * k_in;
  a.C = m; a.ldc = n_out; a.sC = tiles * n_out;
  a.alpha = 1.f; a.beta = 0.f;
  a.a_bytes = (unsigned)(tiles * k_in * eb); a.b_bytes = (unsigned)((long long)n_out * k_in * eb);
  a.c_bytes = (unsigned)(tiles * n_out * 4);
  set_splits(a, 1);
  auto go = [&](GemmArgs& g, int c) {
    if (pk) conv_dma(A_ROWK, g, (hipStream_t)stream, c, 4);
    else launch_big<A_ROWK_SPLIT, 4, B_ROWK_SPLIT, 4>(g, (hipStream_t)stream, c);
  };
  const int cfg = choose_tile(a, true, false);
  // wave-quantization tail (as conv2d_impl's): positions whose tiles would leave a nearly empty last round (c2's 7x7x512
  // level: 16 tiles of 256x128 per position x 36 = 2.25 rounds) go in a second launch the cost model tiles finely
  static const bool no_tail = getenv("MVAE_NO_TAIL_SPLIT") != nullptr;
  int b_main = a.batch;
  if (!no_tail && cfg >= T256x256 && cfg <= T64x64) {
    GemmArgs one = a;
    one.batch = 1;
    const long long tp = tiles_of(cfg, one), slots = 256LL * resident_of(cfg), tot = tp * a.batch;
    const long long full = tot / slots, rem = tot - full * slots;
    // (up to half a round: c4's 8x8x2048 level is 32 tiles x 36 = 4.5 rounds of 256x256)
    if (full >= 1 && rem > 0 && rem * 2 <= slots) b_main = (int)std::max<long long>(1, full * slots / tp);
  }
  if (b_main >= a.batch) {
    go(a, cfg);
    return launch_status();
  }
  GemmArgs t = a;
  a.batch = b_main;
  go(a, cfg);
  t.batch -= b_main;
  // (the A / B pointers are float-typed: a packed operand's element offset is half as many floats)
  t.A = (const float*)((const char*)t.A + (long long)b_main * t.sA * eb);
  t.B = (const float*)((const char*)t.B + (long long)b_main * t.sB * eb);
  t.C += (long long)b_main * t.sC;
  go(t, choose_tile(t, true, false));
  return launch_status();
}

// y [nb][h][w][n] = A^T M A (+ bias[n]) (+ residual, same layout as y); gn_part (nullable): the GroupNorm statistics of
// y per 32-pixel block and 4-channel group (fp64 pairs, [nb*h*w/32][n/4][2], the mvae_conv2d_gnstats_nhwc layout)
int mvae_winograd_output_transform(const float* m, const float* bias, const float* residual, float* y, double* gn_part,
                                   int nb, int h, int w, int n, int tile, void* stream) {
  if (!m || !y || !wino_geom_ok(tile, nb, h, w, n, n) || !al16(m) || !al16(y) || (bias && !al16(bias)) ||
      (residual && !al16(residual)) || (gn_part && !wino_blocks_ok(h, w))) {
    set_error("winograd_output_transform: tile 2 or 4, n %% 4 == 0, 16-B aligned; statistics need h %% 4 == 0 and w in "
              "{8, 16} or a multiple of 32");
    return MVAE_EINVAL;
  }
  WinoOut p{};
  p.m = m; p.bias = bias; p.res = residual; p.y = y; p.gn_part = gn_part;
  p.groups = 1; p.nb = nb; p.H = h; p.W = w; p.N = n;
  return wino_out_launch(p, tile, false, stream);
}

// Input-gradient output transform dx = A^T M A that also emits the backward partials of the GroupNorm whose
// (silu'd) output was the conv's input -- mvae_conv2d_dgrad_gnbwd_nhwc's epilogue: per channel and 32-pixel block
// {sum dyn, sum dyn * xhat} (fp64) at part[((pixel / 32) * n + channel) * 2], x / mean / rstd / gamma / beta the
// GroupNorm's input and statistics ([nb][h][w][n], [nb * groups] x 2, [n] x 2)
int mvae_winograd_output_gnbwd(const float* m, float* dx, const float* x, const float* mean, const float* rstd,
                               const float* gamma, const float* beta, int groups, int silu, double* part, int nb, int h,
                               int w, int n, int tile, void* stream) {
  if (!m || !dx || !x || !mean || !rstd || !gamma || !beta || !part || groups <= 0 || n % groups ||
      (n / groups) % 4 || !wino_geom_ok(tile, nb, h, w, n, n) || !wino_blocks_ok(h, w) || !al16(m) || !al16(dx) ||
      !al16(x)) {
    set_error("winograd_output_gnbwd: tile 2 or 4, h %% 4 == 0, w in {8, 16} or a multiple of 32, channels per "
              "group %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  WinoOut p{};
  p.m = m; p.y = dx; p.gnb_part = part; p.gx = x; p.mean = mean; p.rstd = rstd; p.gamma = gamma; p.beta = beta;
  p.groups = groups; p.silu = silu; p.nb = nb; p.H = h; p.W = w; p.N = n;
  return wino_out_launch(p, tile, true, stream);
}

// D' [a^2][T][k] split4_bf16 of the output gradient dy [nb][h][w][k] (fp32, or split4_bf16 groups when dy_split)
int mvae_winograd_dy_transform(const float* dy, void* d, int nb, int h, int w, int k, int dy_split, int tile,
                               void* stream) {
  if (!dy || !d || !wino_geom_ok(tile, nb, h, w, k, k) || !al16(dy) || !al16(d)) {
    set_error("winograd_dy_transform: tile 2 or 4, k %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  if (!wino_split_in_ok(dy_split)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int sf = wino_sf();
  if (tile == 2) WINO_GO(dy_go, 2, dy, nullptr, d, nb, h, w, k, dy_split, false, st);
  else WINO_GO(dy_go, 4, dy, nullptr, d, nb, h, w, k, dy_split, false, st);
  return launch_status();
}

// Both backward transforms of dy in one pass: v = the input gradient's V' (as mvae_winograd_input_transform on dy) and
// d = the weight gradient's D' (as mvae_winograd_dy_transform), each [a^2][T][k] split4_bf16
int mvae_winograd_dy_transforms(const float* dy, void* v, void* d, int nb, int h, int w, int k, int dy_split, int tile,
                                void* stream) {
  if (!dy || !v || !d || !wino_geom_ok(tile, nb, h, w, k, k) || !al16(dy) || !al16(v) || !al16(d)) {
    set_error("winograd_dy_transforms: tile 2 or 4, k %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  if (!wino_split_in_ok(dy_split)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int sf = wino_sf();
  if (tile == 2) WINO_GO(dy_go, 2, dy, v, d, nb, h, w, k, dy_split, true, st);
  else WINO_GO(dy_go, 4, dy, v, d, nb, h, w, k, dy_split, true, st);
  return launch_status();
}

// M [a^2][cout][cin] fp32 = sum over the tiles of D'_xi [T][cout] (x) V_xi [T][cin]: one batched launch (COL x COL
// images of pre-split operands), split over the tiles when the a^2 products leave the chip under-filled and the
// workspace (mvae_gemm_workspace_bytes(cout, cin, tiles, a^2)) allows
int mvae_winograd_wgrad_gemm(const void* d, const void* v, float* m, long long tiles, int cout, int cin, int tile,
                             float* workspace, size_t workspace_bytes, void* stream) {
  if (!d || !v || !m || tiles <= 0 || cout <= 0 || cin <= 0 || cout % 4 || cin % 4 || !al16(d) || !al16(v) || !al16(m) ||
      tiles * std::max(cout, cin) * 4 > MAX_DESC_BYTES || tiles > (1LL << 30) || (tile != 2 && tile != 4)) {
    set_error("winograd_wgrad_gemm: cout, cin multiples of 4, 16-B aligned, one position < 4 GiB, tile 2 or 4");
    return MVAE_EINVAL;
  }
  const bool pk = wino_sf() == 2;  // (bf16-mixed: packed D' / V through the LDS-DMA COL x COL loop)
  if (pk && (cout % 8 || cin % 8)) {
    set_error("winograd_wgrad_gemm: the bf16 (packed) operands need cout, cin %% 8 == 0");
    return MVAE_EINVAL;
  }
  const unsigned eb = pk ? 2u : 4u;
  GemmArgs a{};
  a.M = cout; a.N = cin; a.K = (int)tiles; a.batch = (tile + 2) * (tile + 2);
  a.A = (const float*)d; a.lda = cout; a.sA = tiles * cout;
  a.B = (const float*)v; a.ldb = cin; a.sB = tiles * cin;
  a.C = m; a.ldc = cin; a.sC = (long long)cout * cin;
  a.alpha = 1.f; a.beta = 0.f;
  a.a_bytes = (unsigned)(tiles * cout * eb); a.b_bytes = (unsigned)(tiles * cin * eb);
  a.c_bytes = (unsigned)((long long)cout * cin * 4);
  const int cfg = choose_tile(a, true, workspace != nullptr);
  plan_splits(a, cfg, workspace, workspace_bytes);
  if (pk) wgrad_dma(B_COLN, a, (hipStream_t)stream, cfg, 4);
  else launch_big<A_COLM_SPLIT, 4, B_COLN_SPLIT, 4>(a, (hipStream_t)stream, cfg);
  return gemm_finish(a, (hipStream_t)stream);
}

// The Upsample conv on the Winograd form (see wino_ups_weights_kernel): kc [4 cout][3][3][cin] = the four class kernels
// of w [cout][3][3][cin], row pq * cout + k -- the forward / input-gradient "weights" of a 3x3 conv with 4 cout outputs
int mvae_winograd_upsample_weights(const float* w, float* kc, int cin, int cout, void* stream) {
  if (!w || !kc || cin <= 0 || cout <= 0 || cin % 4 || !al16(w) || !al16(kc)) {
    set_error("winograd_upsample_weights: cin %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(wino_ups_weights_kernel, dim3(egrid256(4LL * cout * (cin / 4))), dim3(256), 0, (hipStream_t)stream,
                     w, kc, cout, cin);
  return launch_status();
}

// dw = beta * dw + the class kernels' gradients dkc [4 cout][3][3][cin] folded back onto the 3x3 taps
int mvae_winograd_upsample_fold(const float* dkc, float* dw, float beta, int cin, int cout, void* stream) {
  if (!dkc || !dw || cin <= 0 || cout <= 0 || cin % 4 || !al16(dkc) || !al16(dw)) {
    set_error("winograd_upsample_fold: cin %% 4 == 0, 16-B aligned");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(wino_ups_fold_kernel, dim3(egrid256((long long)cout * (cin / 4))), dim3(256), 0,
                     (hipStream_t)stream, dkc, dw, beta, cout, cin);
  return launch_status();
}

// m [a^2][T][4 cout] (the position GEMM of V of the low-resolution x [nb][h][w][cin] with the class kernels' U) ->
// y [nb][2h][2w][cout] (+ bias)
int mvae_winograd_output_transform_upsample(const float* m, const float* bias, float* y, int nb, int h, int w, int cout,
                                            int tile, void* stream) {
  if (!m || !y || cout % 4 || !wino_geom_ok(tile, nb, h, w, 4 * cout, 4 * cout) || !al16(m) || !al16(y) ||
      (bias && !al16(bias)) || (long long)nb * 4 * h * w * cout * 4 > MAX_DESC_BYTES) {
    set_error("winograd_output_transform_upsample: tile 2 or 4, cout %% 4 == 0, 16-B aligned, operands < 4 GiB");
    return MVAE_EINVAL;
  }
  WinoOut p{};
  p.m = m; p.bias = bias; p.y = y;
  p.groups = 1; p.nb = nb; p.H = h; p.W = w; p.N = cout;
  const dim3 g(egrid256(wino_tiles(nb, h, w, tile) * cout));
  if (tile == 2) hipLaunchKernelGGL(wino_out_ups_kernel<2>, g, dim3(256), 0, (hipStream_t)stream, p);
  else hipLaunchKernelGGL(wino_out_ups_kernel<4>, g, dim3(256), 0, (hipStream_t)stream, p);
  return launch_status();
}

// The Upsample conv's backward transforms of its full-resolution dy [nb][2h][2w][cout]: for each class pq the sub-image
// dy[2i + p][2j + q] (an h x w image) -> v = V' [a^2][T][4 cout] (the input gradient's transformed input; null: not
// wanted) and d = D' [a^2][T][4 cout] (the weight gradient's), columns class-major as the class kernels' rows
int mvae_winograd_dy_transforms_upsample(const float* dy, void* v, void* d, int nb, int h, int w, int cout, int tile,
                                         void* stream) {
  if (!dy || !d || cout % 4 || !wino_geom_ok(tile, nb, h, w, 4 * cout, 4 * cout) || !al16(dy) || !al16(d) ||
      (v && !al16(v))) {
    set_error("winograd_dy_transforms_upsample: tile 2 or 4, cout %% 4 == 0, 16-B aligned, operands < 4 GiB");
    return MVAE_EINVAL;
  }
  hipStream_t st = (hipStream_t)stream;
  const int sf = wino_sf(), k = 4 * cout;
  if (tile == 2) WINO_GO(dy_go, 2, dy, v, d, nb, h, w, k, 0, v != nullptr, st, true);
  else WINO_GO(dy_go, 4, dy, v, d, nb, h, w, k, 0, v != nullptr, st, true);
  return launch_status();
}

// dw [cout][3][3][cin] = beta * dw + G^T M G
int mvae_winograd_wgrad_output(const float* m, float* dw, float beta, int cout, int cin, int tile, void* stream) {
  if (!m || !dw || cout <= 0 || cin <= 0 || cin % 4 || !al16(m) || !al16(dw) || (tile != 2 && tile != 4)) {
    set_error("winograd_wgrad_output: cin %% 4 == 0, 16-B aligned, tile 2 or 4");
    return MVAE_EINVAL;
  }
  const dim3 g(egrid256((long long)cout * (cin / 4)));
  if (tile == 2)
    hipLaunchKernelGGL(wino_wout_kernel<2>, g, dim3(256), 0, (hipStream_t)stream, m, dw, beta, cout, cin);
  else
    hipLaunchKernelGGL(wino_wout_kernel<4>, g, dim3(256), 0, (hipStream_t)stream, m, dw, beta, cout, cin);
  return launch_status();
}

}  // extern "C"
