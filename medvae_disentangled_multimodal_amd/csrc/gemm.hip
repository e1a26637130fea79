// Implicit-GEMM convolution / strided-batched GEMM on gfx950 MFMA (fp32 in HBM, "3xBF16" math).
//
// One kernel template serves every matrix product of the conv-VAE training step:
//   conv fwd   (A = NHWC im2col gather incl. stride-2 + asymmetric pad and nearest-x2 upsample,
//               B = KRSC weights)                                   encoder_decoder.py:148-209
//   conv dgrad (A = transposed gather of dY, B = [Cin][R][S][Cout] weights)
//   conv wgrad (A = dY^T, B = im2col gather of X; K = pixels, deterministic split-K)
//   attention  (Q.K^T, P.V and their backward products; batched)     encoder_decoder.py:83-107
//
// Numerics ("3xBF16"): every fp32 operand x is split into hi = bf16(x), lo = bf16(x - hi) when it
// is staged into LDS; a product is hi*hi + hi*lo + lo*hi accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16. Relative error per product ~1e-5 (vs 6e-8 for fp32), far inside the
// 1e-3 parity budget, at 3/16 of the bf16 MFMA cost = 5.3x the fp32-MFMA rate.
//
// Tile: BM x BN x 32, 256 threads = 4 waves in 2x2, each wave owns (BM/2)x(BN/2) = 32x32 MFMA tiles.
// LDS: hi/lo bf16 planes of A[BM][32] and B[BN][32], rows padded to 40 elements (80 B) so the
// ds_read_b128 fragment reads are bank-conflict free; double-buffered, register-staged loads
// (global loads for tile t+1 are in flight while tile t is multiplied), one barrier per K-tile.
#include "common.h"
#include <algorithm>

namespace mvae {

enum { A_ROWK = 0, A_COLM = 1, A_CONV = 2 };
enum { B_ROWK = 0, B_COLN = 1, B_WGRADX = 2 };
enum { CONV_FWD = 0, CONV_UPS = 1, CONV_DGRAD = 2 };

struct GemmArgs {
  int M, N, K;
  int batch, splits, k_split;  // split z covers K range [z*k_split, min(K,(z+1)*k_split))
  const float* A; long long lda, sA;
  const float* B; long long ldb, sB;
  float* C; long long ldc, sC;
  const float* bias;
  const float* res; long long ldr, sR;
  float alpha, beta;
  float* ws;  // split partials [batch][splits][M][N]
  // gather geometry: source X is [nb][H][W][Cx]; output pixels are [nb][Ho][Wo]
  int H, W, Cx, Ho, Wo, R, S, stride, pad_t, pad_l, conv_mode;
  int tiles_m, tiles_n;
};

constexpr int BK = 32;
constexpr int PITCH = 40;  // bf16 elements per LDS row

__device__ __forceinline__ void split4(const float4& v, bf16x4& hi, bf16x4& lo) {
  __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
  hi = bf16x4{h0, h1, h2, h3};
  lo = bf16x4{(__bf16)(v.x - (float)h0), (__bf16)(v.y - (float)h1), (__bf16)(v.z - (float)h2),
              (__bf16)(v.w - (float)h3)};
}

__device__ __forceinline__ void st_split(__bf16* hi_plane, __bf16* lo_plane, int off, const float4& v) {
  bf16x4 h, l;
  split4(v, h, l);
  *(bf16x4*)(hi_plane + off) = h;
  *(bf16x4*)(lo_plane + off) = l;
}

// ------------------------------------------------------------------------------------------
// operand loaders. Each stages a ROWS x 32 tile of the logical operand (rows = M or N, k
// contiguous in LDS). Interface: init(args, row0, k_begin, tid), load() (tile at the current k),
// advance() (k += 32), store(hi_plane, lo_plane).
// ------------------------------------------------------------------------------------------

// K-contiguous rows: element (row, k) at P[row*ld + k].
template <int ROWS, int VEC>
struct LoadRowK {
  static constexpr int NR = ROWS / 32;
  const float* P;
  long long ld;
  int rows, K, row0, k, kc, r0;
  float4 v[NR];
  __device__ void init(const float* p, long long ld_, int rows_, int K_, int row0_, int kb, int tid) {
    P = p; ld = ld_; rows = rows_; K = K_; row0 = row0_; k = kb; kc = tid & 7; r0 = tid >> 3;
  }
  __device__ void load() {
    const int kk = k + kc * 4;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = row0 + r0 + 32 * i;
      const float* src = P + (long long)row * ld + kk;
      if (VEC == 4) {
        v[i] = (row < rows && kk < K) ? *(const float4*)src : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        const bool rv = row < rows;
        v[i].x = (rv && kk + 0 < K) ? src[0] : 0.f;
        v[i].y = (rv && kk + 1 < K) ? src[1] : 0.f;
        v[i].z = (rv && kk + 2 < K) ? src[2] : 0.f;
        v[i].w = (rv && kk + 3 < K) ? src[3] : 0.f;
      }
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void store(__bf16* hi, __bf16* lo) {
#pragma unroll
    for (int i = 0; i < NR; ++i) st_split(hi, lo, (r0 + 32 * i) * PITCH + kc * 4, v[i]);
  }
};

// Row-dim contiguous: element (row, k) at P[k*ld + row]. Each thread loads a 4(k) x 4(row) block
// and transposes it into the k-contiguous LDS image.
template <int ROWS, int VEC>
struct LoadColK {
  static constexpr int NC4 = ROWS / 4;       // 4-wide column groups
  static constexpr int NT = NC4 * (BK / 4);  // active threads
  const float* P;
  long long ld;
  int rows, K, row0, k, c4, k4;
  bool active;
  float4 v[4];
  __device__ void init(const float* p, long long ld_, int rows_, int K_, int row0_, int kb, int tid) {
    P = p; ld = ld_; rows = rows_; K = K_; row0 = row0_; k = kb;
    active = tid < NT; c4 = tid % NC4; k4 = tid / NC4;
  }
  __device__ void load() {
    const int col = row0 + c4 * 4;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int kr = k + k4 * 4 + kk;
      const float* src = P + (long long)kr * ld + col;
      const bool kv = active && kr < K;
      if (VEC == 4) {
        v[kk] = (kv && col < rows) ? *(const float4*)src : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        v[kk].x = (kv && col + 0 < rows) ? src[0] : 0.f;
        v[kk].y = (kv && col + 1 < rows) ? src[1] : 0.f;
        v[kk].z = (kv && col + 2 < rows) ? src[2] : 0.f;
        v[kk].w = (kv && col + 3 < rows) ? src[3] : 0.f;
      }
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void store(__bf16* hi, __bf16* lo) {
    if (!active) return;
    const int base = (c4 * 4) * PITCH + k4 * 4;
    st_split(hi, lo, base + 0 * PITCH, float4{v[0].x, v[1].x, v[2].x, v[3].x});
    st_split(hi, lo, base + 1 * PITCH, float4{v[0].y, v[1].y, v[2].y, v[3].y});
    st_split(hi, lo, base + 2 * PITCH, float4{v[0].z, v[1].z, v[2].z, v[3].z});
    st_split(hi, lo, base + 3 * PITCH, float4{v[0].w, v[1].w, v[2].w, v[3].w});
  }
};

// Gather-position helper: source pixel of output pixel (oh,ow) for filter tap (r,s).
struct TapPos {
  __device__ static __forceinline__ bool src(const GemmArgs& a, int oh, int ow, int r, int s,
                                             int& ih, int& iw) {
    if (a.conv_mode == CONV_FWD) {
      ih = oh * a.stride - a.pad_t + r;
      iw = ow * a.stride - a.pad_l + s;
      return ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
    } else if (a.conv_mode == CONV_UPS) {  // nearest x2 upsample, then conv (stride 1)
      const int uh = oh - a.pad_t + r, uw = ow - a.pad_l + s;
      ih = uh >> 1;
      iw = uw >> 1;
      return uh >= 0 && uh < 2 * a.H && uw >= 0 && uw < 2 * a.W;
    } else {  // transposed gather (dgrad of a strided conv)
      const int nh = oh + a.pad_t - r, nw = ow + a.pad_l - s;
      if (nh < 0 || nw < 0) return false;
      if (a.stride == 1) {
        ih = nh; iw = nw;
      } else {
        if ((nh % a.stride) | (nw % a.stride)) return false;
        ih = nh / a.stride; iw = nw / a.stride;
      }
      return ih < a.H && iw < a.W;
    }
  }
};

// Implicit im2col of an NHWC tensor: element (pixel m, k = (r*S+s)*Cx + c).
template <int ROWS, int VEC>
struct LoadConvA {
  static constexpr int NR = ROWS / 32;
  const float* X;
  int kc, r0, k;
  int cc[4], rr[4], ss[4];  // (c, r, s) of element kc*4+e of the current k-tile
  long long base[NR];
  int oh[NR], ow[NR];
  bool mv[NR];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid) {
    X = x; kc = tid & 7; r0 = tid >> 3; k = kb;
    const int hw = a.Ho * a.Wo;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = row0 + r0 + 32 * i;
      mv[i] = m < a.M;
      const int mm = mv[i] ? m : 0;
      const int b = mm / hw;
      const int rem = mm - b * hw;
      oh[i] = rem / a.Wo;
      ow[i] = rem - oh[i] * a.Wo;
      base[i] = (long long)b * a.H * a.W * a.Cx;
    }
    const int nE = VEC == 4 ? 1 : 4;
    for (int e = 0; e < nE; ++e) {
      const int kk = k + kc * 4 + e;
      const int tap = kk / a.Cx;
      cc[e] = kk - tap * a.Cx;
      rr[e] = tap / a.S;
      ss[e] = tap - rr[e] * a.S;
    }
  }
  __device__ void advance(const GemmArgs& a) {
    k += BK;
    const int nE = VEC == 4 ? 1 : 4;
    for (int e = 0; e < nE; ++e) {
      cc[e] += BK;
      while (cc[e] >= a.Cx) {
        cc[e] -= a.Cx;
        if (++ss[e] == a.S) { ss[e] = 0; ++rr[e]; }
      }
    }
  }
  float4 v[NR];
  __device__ void load(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      if (VEC == 4) {
        int ih, iw;
        const bool ok = mv[i] && (k + kc * 4 < a.K) && TapPos::src(a, oh[i], ow[i], rr[0], ss[0], ih, iw);
        v[i] = ok ? *(const float4*)(X + base[i] + ((long long)ih * a.W + iw) * a.Cx + cc[0])
                  : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int ih, iw;
          const bool ok = mv[i] && (k + kc * 4 + e < a.K) && TapPos::src(a, oh[i], ow[i], rr[e], ss[e], ih, iw);
          t[e] = ok ? X[base[i] + ((long long)ih * a.W + iw) * a.Cx + cc[e]] : 0.f;
        }
        v[i] = float4{t[0], t[1], t[2], t[3]};
      }
    }
  }
  __device__ void store(__bf16* hi, __bf16* lo) {
#pragma unroll
    for (int i = 0; i < NR; ++i) st_split(hi, lo, (r0 + 32 * i) * PITCH + kc * 4, v[i]);
  }
};

// wgrad B operand: rows n' = (r*S+s)*Cx + c (filter element), k = output pixel m.
// element = X[b][src(oh,ow,r,s)][c]; contiguous along c. 4(k) x 4(n') block per thread.
template <int ROWS, int VEC>
struct LoadWgradX {
  static constexpr int NC4 = ROWS / 4;
  static constexpr int NT = NC4 * (BK / 4);
  const float* X;
  bool active;
  int c4, k4, k;
  int cc[4], rr[4], ss[4];
  bool nv[4];
  int pb, poh, pow_;  // decomposition of pixel k + k4*4
  float4 v[4];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid) {
    X = x; k = kb;
    active = tid < NT; c4 = tid % NC4; k4 = tid / NC4;
    const int nE = VEC == 4 ? 1 : 4;
    const int Nn = a.N;
    for (int e = 0; e < 4; ++e) {
      const int n = row0 + c4 * 4 + e;
      nv[e] = n < Nn;
      if (e < nE || VEC == 1) {
        const int nn = nv[e] ? n : 0;
        const int tap = nn / a.Cx;
        cc[e] = nn - tap * a.Cx;
        rr[e] = tap / a.S;
        ss[e] = tap - rr[e] * a.S;
      }
    }
    const int p = kb + k4 * 4;
    const int hw = a.Ho * a.Wo;
    pb = p / hw;
    const int rem = p - pb * hw;
    poh = rem / a.Wo;
    pow_ = rem - poh * a.Wo;
  }
  __device__ void advance(const GemmArgs& a) {
    k += BK;
    pow_ += BK;
    while (pow_ >= a.Wo) {
      pow_ -= a.Wo;
      if (++poh == a.Ho) { poh = 0; ++pb; }
    }
  }
  __device__ void load(const GemmArgs& a) {
    int b = pb, oh = poh, ow = pow_;
    const long long img = (long long)a.H * a.W * a.Cx;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bool kv = active && (k + k4 * 4 + kk < a.K);
      if (VEC == 4) {
        int ih, iw;
        const bool ok = kv && nv[0] && TapPos::src(a, oh, ow, rr[0], ss[0], ih, iw);
        v[kk] = ok ? *(const float4*)(X + b * img + ((long long)ih * a.W + iw) * a.Cx + cc[0])
                   : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int ih, iw;
          const bool ok = kv && nv[e] && TapPos::src(a, oh, ow, rr[e], ss[e], ih, iw);
          t[e] = ok ? X[b * img + ((long long)ih * a.W + iw) * a.Cx + cc[e]] : 0.f;
        }
        v[kk] = float4{t[0], t[1], t[2], t[3]};
      }
      if (++ow == a.Wo) { ow = 0; if (++oh == a.Ho) { oh = 0; ++b; } }
    }
  }
  __device__ void store(__bf16* hi, __bf16* lo) {
    if (!active) return;
    const int base = (c4 * 4) * PITCH + k4 * 4;
    st_split(hi, lo, base + 0 * PITCH, float4{v[0].x, v[1].x, v[2].x, v[3].x});
    st_split(hi, lo, base + 1 * PITCH, float4{v[0].y, v[1].y, v[2].y, v[3].y});
    st_split(hi, lo, base + 2 * PITCH, float4{v[0].z, v[1].z, v[2].z, v[3].z});
    st_split(hi, lo, base + 3 * PITCH, float4{v[0].w, v[1].w, v[2].w, v[3].w});
  }
};

// Uniform wrappers so the kernel body can treat all loaders alike.
template <int KIND, int ROWS, int VEC, bool IS_A>
struct Operand;

template <int ROWS, int VEC, bool IS_A>
struct Operand<0, ROWS, VEC, IS_A> {  // row-k
  LoadRowK<ROWS, VEC> L;
  __device__ void init(const GemmArgs& a, const float* p, int row0, int kb, int tid) {
    L.init(p, IS_A ? a.lda : a.ldb, IS_A ? a.M : a.N, a.K, row0, kb, tid);
  }
  __device__ void load(const GemmArgs&) { L.load(); }
  __device__ void advance(const GemmArgs&) { L.advance(); }
  __device__ void store(__bf16* h, __bf16* l) { L.store(h, l); }
};
template <int ROWS, int VEC, bool IS_A>
struct Operand<1, ROWS, VEC, IS_A> {  // col
  LoadColK<ROWS, VEC> L;
  __device__ void init(const GemmArgs& a, const float* p, int row0, int kb, int tid) {
    L.init(p, IS_A ? a.lda : a.ldb, IS_A ? a.M : a.N, a.K, row0, kb, tid);
  }
  __device__ void load(const GemmArgs&) { L.load(); }
  __device__ void advance(const GemmArgs&) { L.advance(); }
  __device__ void store(__bf16* h, __bf16* l) { L.store(h, l); }
};
template <int ROWS, int VEC>
struct Operand<2, ROWS, VEC, true> {  // conv gather (A)
  LoadConvA<ROWS, VEC> L;
  __device__ void init(const GemmArgs& a, const float* p, int row0, int kb, int tid) { L.init(a, p, row0, kb, tid); }
  __device__ void load(const GemmArgs& a) { L.load(a); }
  __device__ void advance(const GemmArgs& a) { L.advance(a); }
  __device__ void store(__bf16* h, __bf16* l) { L.store(h, l); }
};
template <int ROWS, int VEC>
struct Operand<2, ROWS, VEC, false> {  // wgrad gather (B)
  LoadWgradX<ROWS, VEC> L;
  __device__ void init(const GemmArgs& a, const float* p, int row0, int kb, int tid) { L.init(a, p, row0, kb, tid); }
  __device__ void load(const GemmArgs& a) { L.load(a); }
  __device__ void advance(const GemmArgs& a) { L.advance(a); }
  __device__ void store(__bf16* h, __bf16* l) { L.store(h, l); }
};

template <int BM, int BN, int AK, int VA, int BKIND, int VB>
__global__ void __launch_bounds__(256) gemm3x_kernel(GemmArgs a) {
  constexpr int A_PL = BM * PITCH, B_PL = BN * PITCH;
  constexpr int BUF = 2 * A_PL + 2 * B_PL;
  constexpr int WM = BM / 64, WN = BN / 64;  // 32x32 MFMA tiles per wave (2x2 waves)
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tile = blockIdx.x;
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;
  const int bidx = z / a.splits, split = z - bidx * a.splits;
  const int kb = split * a.k_split;
  const int ke = min(a.K, kb + a.k_split);
  const float* Ap = a.A + bidx * a.sA;
  const float* Bp = a.B + bidx * a.sB;

  Operand<AK, BM, VA, true> la;
  Operand<BKIND, BN, VB, false> lb;
  la.init(a, Ap, m0, kb, tid);
  lb.init(a, Bp, n0, kb, tid);

  f32x16 acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nt = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  if (nt > 0) {
    la.load(a);
    lb.load(a);
    la.store(lds, lds + A_PL);
    lb.store(lds + 2 * A_PL, lds + 2 * A_PL + B_PL);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      la.advance(a);
      lb.advance(a);
      la.load(a);
      lb.load(a);
    }
    const __bf16* Ahi = lds + cur * BUF;
    const __bf16* Alo = Ahi + A_PL;
    const __bf16* Bhi = Ahi + 2 * A_PL;
    const __bf16* Blo = Bhi + B_PL;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 ah[WM], al[WM], bh[WN], bl[WN];
      const int koff = ks * 16 + (lane >> 5) * 8;
#pragma unroll
      for (int i = 0; i < WM; ++i) {
        const int off = (wm * (BM / 2) + i * 32 + (lane & 31)) * PITCH + koff;
        ah[i] = *(const bf16x8*)(Ahi + off);
        al[i] = *(const bf16x8*)(Alo + off);
      }
#pragma unroll
      for (int j = 0; j < WN; ++j) {
        const int off = (wn * (BN / 2) + j * 32 + (lane & 31)) * PITCH + koff;
        bh[j] = *(const bf16x8*)(Bhi + off);
        bl[j] = *(const bf16x8*)(Blo + off);
      }
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
    }
    if (t + 1 < nt) {
      __bf16* nb = lds + (cur ^ 1) * BUF;
      la.store(nb, nb + A_PL);
      lb.store(nb + 2 * A_PL, nb + 2 * A_PL + B_PL);
    }
    __syncthreads();
  }

  // epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool partial = a.splits > 1;
  float* Cp = a.C + bidx * a.sC;
  const float* Rp = a.res ? a.res + bidx * a.sR : nullptr;
  float* Wp = partial ? a.ws + ((long long)bidx * a.splits + split) * a.M * a.N : nullptr;
#pragma unroll
  for (int j = 0; j < WN; ++j) {
    const int col = n0 + wn * (BN / 2) + j * 32 + (lane & 31);
    if (col >= a.N) continue;
    const float bv = (!partial && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < WM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * (BM / 2) + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= a.M) continue;
        if (partial) {
          Wp[(long long)row * a.N + col] = acc[i][j][r];
        } else {
          float v = a.alpha * acc[i][j][r] + bv;
          if (Rp) v += Rp[(long long)row * a.ldr + col];
          float* cp = Cp + (long long)row * a.ldc + col;
          if (a.beta != 0.f) v += a.beta * *cp;
          *cp = v;
        }
      }
    }
  }
}

// Fixed-order reduction of split-K partials + the same epilogue.
__global__ void splitk_reduce_kernel(GemmArgs a) {
  const long long mn = (long long)a.M * a.N;
  const long long total = mn * a.batch;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int bidx = (int)(e / mn);
    const long long rc = e - bidx * mn;
    const int row = (int)(rc / a.N), col = (int)(rc - (long long)row * a.N);
    const float* w = a.ws + (long long)bidx * a.splits * mn + rc;
    float s = 0.f;
    for (int z = 0; z < a.splits; ++z) s += w[z * mn];
    float v = a.alpha * s + (a.bias ? a.bias[col] : 0.f);
    if (a.res) v += a.res[bidx * a.sR + (long long)row * a.ldr + col];
    float* cp = a.C + bidx * a.sC + (long long)row * a.ldc + col;
    if (a.beta != 0.f) v += a.beta * *cp;
    *cp = v;
  }
}

// ------------------------------------------------------------------------------------------
// host-side dispatch
// ------------------------------------------------------------------------------------------
template <int BM, int BN, int AK, int VA, int BKIND, int VB>
static void launch_t(GemmArgs& a, hipStream_t st) {
  a.tiles_m = cdiv(a.M, BM);
  a.tiles_n = cdiv(a.N, BN);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splits);
  hipLaunchKernelGGL((gemm3x_kernel<BM, BN, AK, VA, BKIND, VB>), grid, dim3(256), 0, st, a);
}

template <int AK, int VA, int BKIND, int VB>
static void launch_sz(GemmArgs& a, hipStream_t st) {
  // 128x128 tiles when the problem fills the chip, otherwise 64x64 (more blocks)
  const long long t128 = (long long)cdiv(a.M, 128) * cdiv(a.N, 128) * a.batch * a.splits;
  if (t128 >= 512 || (a.M >= 128 && a.N >= 128 && t128 >= 256))
    launch_t<128, 128, AK, VA, BKIND, VB>(a, st);
  else
    launch_t<64, 64, AK, VA, BKIND, VB>(a, st);
}

static size_t splitk_ws_bytes(const GemmArgs& a) {
  return a.splits > 1 ? (size_t)a.batch * a.splits * a.M * a.N * sizeof(float) : 0;
}

// choose split-K so that a small-MN / huge-K product (wgrad) still fills 256 CUs
static int choose_splits(int M, int N, int K, int batch) {
  const long long tiles = (long long)cdiv(M, 128) * cdiv(N, 128) * batch;
  int s = 1;
  while (tiles * s < 512 && (long long)K / (s * 2) >= 512 && s < 64) s *= 2;
  return s;
}

static int finish(GemmArgs& a, hipStream_t st) {
  if (a.splits > 1) {
    const long long total = (long long)a.M * a.N * a.batch;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, a);
  }
  return launch_status();
}

static void set_splits(GemmArgs& a, int splits) {
  a.splits = splits;
  a.k_split = ((cdiv(a.K, splits) + BK - 1) / BK) * BK;
  a.splits = cdiv(a.K, a.k_split);
  if (a.splits < 1) a.splits = 1;
}

}  // namespace mvae

using namespace mvae;

static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" {

// C[b] = alpha * op(A[b]) op(B[b]) + bias + residual[b] + beta*C[b]   (row-major, fp32)
//   op(A) is [M][K]: trans_a=0 -> A stored [M][K] (lda); trans_a=1 -> A stored [K][M]
//   op(B) is [K][N]: trans_b=0 -> B stored [K][N] (ldb); trans_b=1 -> B stored [N][K]
int mvae_gemm_strided_batched(int trans_a, int trans_b, int m, int n, int k, float alpha,
                              const float* A, long long lda, long long stride_a,
                              const float* B, long long ldb, long long stride_b, float beta,
                              float* C, long long ldc, long long stride_c, int batch,
                              const float* bias, const float* residual, long long ldr,
                              long long stride_r, float* workspace, size_t workspace_bytes,
                              void* stream) {
  if (m <= 0 || n <= 0 || k < 0 || batch <= 0) { set_error("gemm: bad sizes"); return MVAE_EINVAL; }
  GemmArgs a{};
  a.M = m; a.N = n; a.K = k; a.batch = batch;
  a.A = A; a.lda = lda; a.sA = stride_a;
  a.B = B; a.ldb = ldb; a.sB = stride_b;
  a.C = C; a.ldc = ldc; a.sC = stride_c;
  a.bias = bias; a.res = residual; a.ldr = ldr; a.sR = stride_r;
  a.alpha = alpha; a.beta = beta;
  set_splits(a, workspace ? choose_splits(m, n, k, batch) : 1);
  while (a.splits > 1 && splitk_ws_bytes(a) > workspace_bytes) set_splits(a, a.splits / 2);
  a.ws = workspace;
  hipStream_t st = (hipStream_t)stream;
  const bool va = (trans_a ? (m % 4 == 0) : (k % 4 == 0)) && (lda % 4 == 0) && (stride_a % 4 == 0) && al16(A);
  const bool vb = (trans_b ? (k % 4 == 0) : (n % 4 == 0)) && (ldb % 4 == 0) && (stride_b % 4 == 0) && al16(B);
  const int ak = trans_a ? A_COLM : A_ROWK;
  const int bk = trans_b ? B_ROWK : B_COLN;
#define MVAE_G(AKk, BKk)                                                        \
  if (va && vb) launch_sz<AKk, 4, BKk, 4>(a, st);                              \
  else if (va) launch_sz<AKk, 4, BKk, 1>(a, st);                               \
  else if (vb) launch_sz<AKk, 1, BKk, 4>(a, st);                               \
  else launch_sz<AKk, 1, BKk, 1>(a, st);
  if (ak == A_ROWK && bk == B_ROWK) { MVAE_G(A_ROWK, B_ROWK) }
  else if (ak == A_ROWK && bk == B_COLN) { MVAE_G(A_ROWK, B_COLN) }
  else if (ak == A_COLM && bk == B_ROWK) { MVAE_G(A_COLM, B_ROWK) }
  else { MVAE_G(A_COLM, B_COLN) }
#undef MVAE_G
  return finish(a, st);
}

size_t mvae_gemm_workspace_bytes(int m, int n, int k, int batch) {
  GemmArgs a{};
  a.M = m; a.N = n; a.K = k; a.batch = batch;
  set_splits(a, choose_splits(m, n, k, batch));
  return splitk_ws_bytes(a);
}

// Implicit-GEMM convolution over NHWC activations and KRSC ([Cout][R][S][Cin]) weights.
//   mode 0: y = conv(x, stride, pad_t/pad_l; zero padding outside [0,H)x[0,W))
//   mode 1: y = conv(upsample_nearest_x2(x), stride 1, pad_t/pad_l)
//   mode 2: transposed gather: y[oh] += x[(oh + pad - r)/stride] * w[r] (dgrad of a strided conv)
// y[n][ho][wo][cout] = sum + bias[cout] + residual[n][ho][wo][cout]
int mvae_conv2d_nhwc(const float* x, const float* w, const float* bias, const float* residual,
                     float* y, int nb, int h, int wd, int cin, int cout, int kh, int kw,
                     int stride, int pad_t, int pad_l, int ho, int wo, int mode, void* stream) {
  if (nb <= 0 || h <= 0 || wd <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || ho <= 0 || wo <= 0 ||
      stride <= 0 || mode < 0 || mode > 2) {
    set_error("conv2d: bad geometry");
    return MVAE_EINVAL;
  }
  GemmArgs a{};
  a.M = nb * ho * wo; a.N = cout; a.K = kh * kw * cin; a.batch = 1; a.splits = 1; a.k_split = a.K;
  a.A = x; a.B = w; a.ldb = a.K;
  a.C = y; a.ldc = cout; a.bias = bias; a.res = residual; a.ldr = cout;
  a.alpha = 1.f; a.beta = 0.f;
  a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
  a.stride = stride; a.pad_t = pad_t; a.pad_l = pad_l; a.conv_mode = mode;
  hipStream_t st = (hipStream_t)stream;
  const bool v = (cin % 4 == 0) && al16(x) && al16(w);
  if (v) launch_sz<A_CONV, 4, B_ROWK, 4>(a, st);
  else launch_sz<A_CONV, 1, B_ROWK, 1>(a, st);
  return finish(a, st);
}

// Weight gradient of mvae_conv2d_nhwc (modes 0 and 1):
//   dw[cout][r][s][cin] = beta*dw + sum_pixels dy[pix][cout] * x[src(pix, r, s)][cin]
// K = nb*ho*wo pixels, split deterministically across blocks (partials in `workspace`).
int mvae_conv2d_wgrad_nhwc(const float* dy, const float* x, float* dw, float beta, int nb, int h,
                           int wd, int cin, int cout, int kh, int kw, int stride, int pad_t,
                           int pad_l, int ho, int wo, int mode, float* workspace,
                           size_t workspace_bytes, void* stream) {
  if (mode != 0 && mode != 1) { set_error("wgrad: mode must be 0 or 1"); return MVAE_EINVAL; }
  GemmArgs a{};
  a.M = cout; a.N = kh * kw * cin; a.K = nb * ho * wo; a.batch = 1;
  a.A = dy; a.lda = cout;
  a.B = x;
  a.C = dw; a.ldc = a.N; a.alpha = 1.f; a.beta = beta;
  a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
  a.stride = stride; a.pad_t = pad_t; a.pad_l = pad_l; a.conv_mode = mode;
  set_splits(a, workspace ? choose_splits(a.M, a.N, a.K, 1) : 1);
  while (a.splits > 1 && splitk_ws_bytes(a) > workspace_bytes) set_splits(a, a.splits / 2);
  a.ws = workspace;
  hipStream_t st = (hipStream_t)stream;
  const bool va = (cout % 4 == 0) && al16(dy);
  const bool vb = (cin % 4 == 0) && al16(x);
  if (va && vb) launch_sz<A_COLM, 4, B_WGRADX, 4>(a, st);
  else if (va) launch_sz<A_COLM, 4, B_WGRADX, 1>(a, st);
  else if (vb) launch_sz<A_COLM, 1, B_WGRADX, 4>(a, st);
  else launch_sz<A_COLM, 1, B_WGRADX, 1>(a, st);
  return finish(a, st);
}

size_t mvae_conv2d_wgrad_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  GemmArgs a{};
  a.M = cout; a.N = kh * kw * cin; a.K = nb * ho * wo; a.batch = 1;
  set_splits(a, choose_splits(a.M, a.N, a.K, 1));
  return splitk_ws_bytes(a);
}

}  // extern "C"
