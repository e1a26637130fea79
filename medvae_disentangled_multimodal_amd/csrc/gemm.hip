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
// is staged into LDS; a product is lo*hi + hi*lo + hi*hi accumulated in fp32 by
// v_mfma_f32_32x32x16_bf16. Relative error per product ~1e-5 (vs 6e-8 for fp32), far inside the
// 1e-3 parity budget, at 3/16 of the bf16 MFMA cost = 5.3x the fp32-MFMA rate.
//
// Tiles: BM x BN x 32 per workgroup of WGM x WGN waves; each wave owns a (BM/WGM) x (BN/WGN) block of
// 32x32 MFMA tiles. Register-staged, double-buffered LDS: global loads of K-tile t+1 are in flight
// while tile t is multiplied; one barrier per K-tile.
// LDS images (hi and lo bf16 planes per operand):
//   ROW image [ROWS][40]      for k-contiguous sources (weights, im2col rows); 80-B rows make the
//                             ds_read_b128 fragment reads bank-conflict free
//   COL image [32][ROWS+32]   for row-contiguous sources (dY^T, im2col columns of wgrad, P/V of the
//                             attention backward): stored as loaded (coalesced, conflict-free 8-B
//                             writes) and read k-contiguous with the gfx950 transpose read
//                             ds_read_b64_tr_b16; the +32 pad puts the 4 k-rows of a read in 4
//                             distinct 16-bank windows.
// Workgroup -> tile mapping is XCD-aware: consecutive tiles (which share operand panels) are dealt to
// the same XCD so they hit the same L2.
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
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

template <int ROWS, bool COL>
struct Img {
  static constexpr int PITCH = COL ? ROWS + 32 : 40;
  static constexpr int PLANE = COL ? BK * PITCH : ROWS * PITCH;
  static constexpr int SIZE = 2 * PLANE;
};

__device__ __forceinline__ void split4(const float4& v, bf16x4& hi, bf16x4& lo) {
  const __bf16 h0 = (__bf16)v.x, h1 = (__bf16)v.y, h2 = (__bf16)v.z, h3 = (__bf16)v.w;
  hi = bf16x4{h0, h1, h2, h3};
  lo = bf16x4{(__bf16)(v.x - (float)h0), (__bf16)(v.y - (float)h1), (__bf16)(v.z - (float)h2),
              (__bf16)(v.w - (float)h3)};
}

__device__ __forceinline__ void st_split(__bf16* img, int plane, int off, const float4& v) {
  bf16x4 h, l;
  split4(v, h, l);
  *(bf16x4*)(img + off) = h;
  *(bf16x4*)(img + plane + off) = l;
}

// fragment of a 32x32x16 MFMA operand: lane l holds element [row0 + (l&31)][ks*16 + 8*(l>>5) + j]
template <int ROWS, bool COL>
__device__ __forceinline__ bf16x8 read_frag(const __bf16* plane, int row0, int ks, int lane) {
  if constexpr (!COL) {
    return *(const bf16x8*)(plane + (row0 + (lane & 31)) * 40 + ks * 16 + (lane >> 5) * 8);
  } else {
    constexpr int P = Img<ROWS, true>::PITCH;
    const int g = lane >> 4, li = lane & 15;
    const __bf16* p = plane + (ks * 16 + (g >> 1) * 8 + (li >> 2)) * P + row0 + (g & 1) * 16 + 4 * (li & 3);
    const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)p);
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p + 4 * P));
    return __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// Gather-position helper: source pixel of output pixel (oh,ow) for filter tap (r,s).
__device__ __forceinline__ bool tap_src(const GemmArgs& a, int oh, int ow, int r, int s, int& ih, int& iw) {
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

// ------------------------------------------------------------------------------------------
// operand loaders: init(args, base, row0, k_begin, tid); load(args) (the tile at the current k);
// advance(args) (k += 32); store(img) into the operand's LDS image.
// ------------------------------------------------------------------------------------------

// ROW image, source element (row, k) at P[row*ld + k]
template <int ROWS, int VEC, int NT, bool IS_A>
struct LoadRowK {
  static constexpr int RP = NT / 8;     // rows per pass (8 float4 per 32-wide row)
  static constexpr int NR = ROWS / RP;  // rows per thread
  const float* P;
  long long ld;
  int rows, K, row0, k, kc, r0;
  float4 v[NR];
  __device__ void init(const GemmArgs& a, const float* p, int row0_, int kb, int tid) {
    P = p; ld = IS_A ? a.lda : a.ldb; rows = IS_A ? a.M : a.N; K = a.K;
    row0 = row0_; k = kb; kc = tid & 7; r0 = tid >> 3;
  }
  __device__ void load(const GemmArgs&) {
    const int kk = k + kc * 4;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int row = row0 + r0 + RP * i;
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
  __device__ void advance(const GemmArgs&) { k += BK; }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NR; ++i) st_split(img, Img<ROWS, false>::PLANE, (r0 + RP * i) * 40 + kc * 4, v[i]);
  }
};

// ROW image, implicit im2col of an NHWC tensor: element (pixel m, k = (r*S+s)*Cx + c)
template <int ROWS, int VEC, int NT>
struct LoadConvA {
  static constexpr int RP = NT / 8;
  static constexpr int NR = ROWS / RP;
  const float* X;
  int kc, r0, k;
  int cc[4], rr[4], ss[4];  // (c, r, s) of element kc*4+e of the current k-tile
  long long base[NR];
  int oh[NR], ow[NR];
  bool mv[NR];
  float4 v[NR];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid) {
    X = x; kc = tid & 7; r0 = tid >> 3; k = kb;
    const int hw = a.Ho * a.Wo;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int m = row0 + r0 + RP * i;
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
  __device__ void load(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      if (VEC == 4) {
        int ih, iw;
        const bool ok = mv[i] && (k + kc * 4 < a.K) && tap_src(a, oh[i], ow[i], rr[0], ss[0], ih, iw);
        v[i] = ok ? *(const float4*)(X + base[i] + ((long long)ih * a.W + iw) * a.Cx + cc[0])
                  : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int ih, iw;
          const bool ok = mv[i] && (k + kc * 4 + e < a.K) && tap_src(a, oh[i], ow[i], rr[e], ss[e], ih, iw);
          t[e] = ok ? X[base[i] + ((long long)ih * a.W + iw) * a.Cx + cc[e]] : 0.f;
        }
        v[i] = float4{t[0], t[1], t[2], t[3]};
      }
    }
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NR; ++i) st_split(img, Img<ROWS, false>::PLANE, (r0 + RP * i) * 40 + kc * 4, v[i]);
  }
};

// COL image, source element (row, k) at P[k*ld + row] (rows contiguous)
template <int ROWS, int VEC, int NT, bool IS_A>
struct LoadColK {
  static constexpr int C4 = ROWS / 4;           // float4 per k-row
  static constexpr int NF = (BK * C4 + NT - 1) / NT;  // float4 per thread
  const float* P;
  long long ld;
  int rows, K, row0, k, c4, kr;
  float4 v[NF];
  __device__ void init(const GemmArgs& a, const float* p, int row0_, int kb, int tid) {
    P = p; ld = IS_A ? a.lda : a.ldb; rows = IS_A ? a.M : a.N; K = a.K;
    row0 = row0_; k = kb; c4 = tid % C4; kr = tid / C4;
  }
  __device__ void load(const GemmArgs&) {
    const int col = row0 + c4 * 4;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int krow = kr + i * (NT / C4);
      const int kk = k + krow;
      const bool kv = krow < BK && kk < K;
      const float* src = P + (long long)kk * ld + col;
      if (VEC == 4) {
        v[i] = (kv && col < rows) ? *(const float4*)src : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        v[i].x = (kv && col + 0 < rows) ? src[0] : 0.f;
        v[i].y = (kv && col + 1 < rows) ? src[1] : 0.f;
        v[i].z = (kv && col + 2 < rows) ? src[2] : 0.f;
        v[i].w = (kv && col + 3 < rows) ? src[3] : 0.f;
      }
    }
  }
  __device__ void advance(const GemmArgs&) { k += BK; }
  __device__ void store(__bf16* img) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int krow = kr + i * (NT / C4);
      if (krow < BK) st_split(img, Img<ROWS, true>::PLANE, krow * P_ + c4 * 4, v[i]);
    }
  }
};

// COL image for the wgrad B operand: rows n' = (r*S+s)*Cx + c (filter element), k = output pixel.
// element = X[b][src(oh,ow,r,s)][c], contiguous along c.
template <int ROWS, int VEC, int NT>
struct LoadWgradX {
  static constexpr int C4 = ROWS / 4;
  static constexpr int NF = (BK * C4 + NT - 1) / NT;
  const float* X;
  int c4, kr, k;
  int cc[4], rr[4], ss[4];
  bool nv[4];
  int pb[NF], poh[NF], pow_[NF];  // pixel decomposition of this thread's k-rows
  float4 v[NF];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid) {
    X = x; k = kb; c4 = tid % C4; kr = tid / C4;
    for (int e = 0; e < 4; ++e) {
      const int n = row0 + c4 * 4 + e;
      nv[e] = n < a.N;
      const int nn = nv[e] ? n : 0;
      const int tap = nn / a.Cx;
      cc[e] = nn - tap * a.Cx;
      rr[e] = tap / a.S;
      ss[e] = tap - rr[e] * a.S;
    }
    const int hw = a.Ho * a.Wo;
    // with 64 column groups the k-row is wave-uniform: keep the pixel walk in scalar registers
    const int krw = (C4 % 64 == 0) ? __builtin_amdgcn_readfirstlane(kr) : kr;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int p = kb + krw + i * (NT / C4);
      pb[i] = p / hw;
      const int rem = p - pb[i] * hw;
      poh[i] = rem / a.Wo;
      pow_[i] = rem - poh[i] * a.Wo;
    }
  }
  __device__ void advance(const GemmArgs& a) {
    k += BK;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      pow_[i] += BK;
      while (pow_[i] >= a.Wo) {
        pow_[i] -= a.Wo;
        if (++poh[i] == a.Ho) { poh[i] = 0; ++pb[i]; }
      }
    }
  }
  __device__ void load(const GemmArgs& a) {
    const long long img = (long long)a.H * a.W * a.Cx;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int krow = kr + i * (NT / C4);
      const bool kv = krow < BK && (k + krow < a.K);
      if (VEC == 4) {
        int ih, iw;
        const bool ok = kv && nv[0] && tap_src(a, poh[i], pow_[i], rr[0], ss[0], ih, iw);
        v[i] = ok ? *(const float4*)(X + pb[i] * img + ((long long)ih * a.W + iw) * a.Cx + cc[0])
                  : float4{0.f, 0.f, 0.f, 0.f};
      } else {
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          int ih, iw;
          const bool ok = kv && nv[e] && tap_src(a, poh[i], pow_[i], rr[e], ss[e], ih, iw);
          t[e] = ok ? X[pb[i] * img + ((long long)ih * a.W + iw) * a.Cx + cc[e]] : 0.f;
        }
        v[i] = float4{t[0], t[1], t[2], t[3]};
      }
    }
  }
  __device__ void store(__bf16* img) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int krow = kr + i * (NT / C4);
      if (krow < BK) st_split(img, Img<ROWS, true>::PLANE, krow * P_ + c4 * 4, v[i]);
    }
  }
};

template <int KIND, int ROWS, int VEC, int NT, bool IS_A>
struct Loader;
template <int ROWS, int VEC, int NT, bool IS_A>
struct Loader<0, ROWS, VEC, NT, IS_A> : LoadRowK<ROWS, VEC, NT, IS_A> { static constexpr bool COL = false; };
template <int ROWS, int VEC, int NT, bool IS_A>
struct Loader<1, ROWS, VEC, NT, IS_A> : LoadColK<ROWS, VEC, NT, IS_A> { static constexpr bool COL = true; };
template <int ROWS, int VEC, int NT>
struct Loader<2, ROWS, VEC, NT, true> : LoadConvA<ROWS, VEC, NT> { static constexpr bool COL = false; };
template <int ROWS, int VEC, int NT>
struct Loader<2, ROWS, VEC, NT, false> : LoadWgradX<ROWS, VEC, NT> { static constexpr bool COL = true; };

template <int BM, int BN, int WGM, int WGN, int AK, int VA, int BKIND, int VB>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm3x_kernel(GemmArgs a) {
  constexpr int NT = 64 * WGM * WGN;
  using LA = Loader<AK, BM, VA, NT, true>;
  using LB = Loader<BKIND, BN, VB, NT, false>;
  using IA = Img<BM, LA::COL>;
  using IB = Img<BN, LB::COL>;
  constexpr int BUF = IA::SIZE + IB::SIZE;
  constexpr int TM = BM / WGM / 32, TN = BN / WGN / 32;  // 32x32 MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) __bf16 lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid - wm * WGN;
  // XCD-aware remap (bijective): blocks b and b+8 share an XCD, so hand each XCD a contiguous run
  // of tiles (row-major over (m, n): neighbours share A rows and the same weight panel).
  const int nwg = a.tiles_m * a.tiles_n;
  const int orig = blockIdx.x;
  int tile = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int tm = tile / a.tiles_n, tn = tile - tm * a.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int z = blockIdx.z;
  const int bidx = z / a.splits, split = z - bidx * a.splits;
  const int kb = split * a.k_split;
  const int ke = min(a.K, kb + a.k_split);

  LA la;
  LB lb;
  la.init(a, a.A + bidx * a.sA, m0, kb, tid);
  lb.init(a, a.B + bidx * a.sB, n0, kb, tid);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nt = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  if (nt > 0) {
    la.load(a);
    lb.load(a);
    la.store(lds);
    lb.store(lds + IA::SIZE);
  }
  __syncthreads();
  const int arow = wm * (BM / WGM), brow = wn * (BN / WGN);
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      la.advance(a);
      lb.advance(a);
      la.load(a);
      lb.load(a);
    }
    const __bf16* Ai = lds + cur * BUF;
    const __bf16* Bi = Ai + IA::SIZE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = read_frag<BN, LB::COL>(Bi, brow + j * 32, ks, lane);
        bl[j] = read_frag<BN, LB::COL>(Bi + IB::PLANE, brow + j * 32, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 ah = read_frag<BM, LA::COL>(Ai, arow + i * 32, ks, lane);
        const bf16x8 al = read_frag<BM, LA::COL>(Ai + IA::PLANE, arow + i * 32, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    if (t + 1 < nt) {
      __bf16* nb = lds + (cur ^ 1) * BUF;
      la.store(nb);
      lb.store(nb + IA::SIZE);
    }
    __syncthreads();
  }

  // epilogue: C/D layout of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const bool partial = a.splits > 1;
  float* Cp = a.C + bidx * a.sC;
  const float* Rp = a.res ? a.res + bidx * a.sR : nullptr;
  float* Wp = partial ? a.ws + ((long long)bidx * a.splits + split) * a.M * a.N : nullptr;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + brow + j * 32 + (lane & 31);
    if (col >= a.N) continue;
    const float bv = (!partial && a.bias) ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + arow + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
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
enum { T256x256 = 0, T256x128 = 1, T128x256 = 2, T128x128 = 3, T64x64 = 4 };
static const int TILE_M[] = {256, 256, 128, 128, 64};
static const int TILE_N[] = {256, 128, 256, 128, 64};

static long long tiles_of(int cfg, const GemmArgs& a) {
  return (long long)cdiv(a.M, TILE_M[cfg]) * cdiv(a.N, TILE_N[cfg]) * a.batch;
}

// largest useful split-K factor (>= 16 K-tiles per split)
static int max_splits_of(const GemmArgs& a, bool can_split) {
  if (!can_split) return 1;
  int s = 1;
  while (s < 64 && (long long)a.K / (s * 2) >= 512) s *= 2;
  return s;
}

// pick the largest tile that still gives >= 1 full wave of the 256 CUs, counting the blocks that
// split-K adds when a workspace is available (wgrad: small M x N, huge K)
static int choose_tile(const GemmArgs& a, bool allow_big, bool can_split) {
  const long long ms = max_splits_of(a, can_split);
  if (allow_big) {
    if (tiles_of(T256x256, a) * ms >= 240 && a.M > 128 && a.N > 128) return T256x256;
    if (a.N <= 128 && tiles_of(T256x128, a) * ms >= 240 && a.M > 128) return T256x128;
    if (a.M <= 128 && tiles_of(T128x256, a) * ms >= 240 && a.N > 128) return T128x256;
  }
  if (tiles_of(T128x128, a) * ms >= 200 && a.M > 64 && a.N > 64) return T128x128;
  return T64x64;
}

template <int CFG, int AK, int VA, int BKIND, int VB>
static void launch_cfg(GemmArgs& a, hipStream_t st) {
  constexpr int BM = CFG == T256x256 || CFG == T256x128 ? 256 : CFG == T64x64 ? 64 : 128;
  constexpr int BN = CFG == T256x256 || CFG == T128x256 ? 256 : CFG == T64x64 ? 64 : 128;
  constexpr int WGM = CFG == T256x128 ? 4 : 2;
  constexpr int WGN = (CFG == T256x256 || CFG == T128x256) ? 4 : 2;
  a.tiles_m = cdiv(a.M, BM);
  a.tiles_n = cdiv(a.N, BN);
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splits);
  hipLaunchKernelGGL((gemm3x_kernel<BM, BN, WGM, WGN, AK, VA, BKIND, VB>), grid, dim3(64 * WGM * WGN), 0, st, a);
}

template <int AK, int VA, int BKIND, int VB>
static void launch_big(GemmArgs& a, hipStream_t st, int cfg) {
  switch (cfg) {
    case T256x256: launch_cfg<T256x256, AK, VA, BKIND, VB>(a, st); break;
    case T256x128: launch_cfg<T256x128, AK, VA, BKIND, VB>(a, st); break;
    case T128x256: launch_cfg<T128x256, AK, VA, BKIND, VB>(a, st); break;
    case T128x128: launch_cfg<T128x128, AK, VA, BKIND, VB>(a, st); break;
    default: launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st); break;
  }
}

template <int AK, int VA, int BKIND, int VB>
static void launch_small(GemmArgs& a, hipStream_t st, int cfg) {
  if (cfg == T128x128) launch_cfg<T128x128, AK, VA, BKIND, VB>(a, st);
  else launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st);
}

static size_t splitk_ws_bytes(const GemmArgs& a) {
  return a.splits > 1 ? (size_t)a.batch * a.splits * a.M * a.N * sizeof(float) : 0;
}

static void set_splits(GemmArgs& a, int splits) {
  a.splits = std::max(1, splits);
  a.k_split = ((cdiv(a.K, a.splits) + BK - 1) / BK) * BK;
  a.splits = std::max(1, cdiv(a.K, a.k_split));
}

// split K so that a small-MN / huge-K product (wgrad) still fills the chip; >= 16 K-tiles per split
static int choose_splits(const GemmArgs& a, int cfg) {
  const long long tiles = tiles_of(cfg, a);
  const int ms = max_splits_of(a, true);
  int s = 1;
  while (tiles * s < 400 && s < ms) s *= 2;
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

static void plan_splits(GemmArgs& a, int cfg, float* ws, size_t ws_bytes) {
  set_splits(a, ws ? choose_splits(a, cfg) : 1);
  while (a.splits > 1 && splitk_ws_bytes(a) > ws_bytes) set_splits(a, a.splits / 2);
  a.ws = ws;
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
  hipStream_t st = (hipStream_t)stream;
  const bool va = (trans_a ? (m % 4 == 0) : (k % 4 == 0)) && (lda % 4 == 0) && (stride_a % 4 == 0) && al16(A);
  const bool vb = (trans_b ? (k % 4 == 0) : (n % 4 == 0)) && (ldb % 4 == 0) && (stride_b % 4 == 0) && al16(B);
  const int cfg = choose_tile(a, va && vb, workspace != nullptr);
  plan_splits(a, cfg, workspace, workspace_bytes);
  const int ak = trans_a ? A_COLM : A_ROWK;
  const int bk = trans_b ? B_ROWK : B_COLN;
#define MVAE_G(AKk, BKk)                                                        \
  if (va && vb) launch_big<AKk, 4, BKk, 4>(a, st, cfg);                        \
  else if (va) launch_small<AKk, 4, BKk, 1>(a, st, cfg);                       \
  else if (vb) launch_small<AKk, 1, BKk, 4>(a, st, cfg);                       \
  else launch_small<AKk, 1, BKk, 1>(a, st, cfg);
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
  set_splits(a, choose_splits(a, choose_tile(a, true, true)));
  size_t b1 = splitk_ws_bytes(a);
  set_splits(a, choose_splits(a, choose_tile(a, false, true)));
  return std::max(b1, splitk_ws_bytes(a));
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
  const int cfg = choose_tile(a, v, false);
  if (v) launch_big<A_CONV, 4, B_ROWK, 4>(a, st, cfg);
  else launch_small<A_CONV, 1, B_ROWK, 1>(a, st, cfg);
  return finish(a, st);
}

// Weight gradient of mvae_conv2d_nhwc (modes 0 and 1):
//   dw[cout][r][s][cin] = beta*dw + sum_pixels dy[pix][cout] * x[src(pix, r, s)][cin]
// K = nb*ho*wo pixels, split deterministically across blocks (partials in `workspace`).
static void wgrad_args(GemmArgs& a, int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  a.M = cout; a.N = kh * kw * cin; a.K = nb * ho * wo; a.batch = 1;
}

int mvae_conv2d_wgrad_nhwc(const float* dy, const float* x, float* dw, float beta, int nb, int h,
                           int wd, int cin, int cout, int kh, int kw, int stride, int pad_t,
                           int pad_l, int ho, int wo, int mode, float* workspace,
                           size_t workspace_bytes, void* stream) {
  if (mode != 0 && mode != 1) { set_error("wgrad: mode must be 0 or 1"); return MVAE_EINVAL; }
  GemmArgs a{};
  wgrad_args(a, nb, cin, cout, kh, kw, ho, wo);
  a.A = dy; a.lda = cout;
  a.B = x;
  a.C = dw; a.ldc = a.N; a.alpha = 1.f; a.beta = beta;
  a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
  a.stride = stride; a.pad_t = pad_t; a.pad_l = pad_l; a.conv_mode = mode;
  hipStream_t st = (hipStream_t)stream;
  const bool va = (cout % 4 == 0) && al16(dy);
  const bool vb = (cin % 4 == 0) && al16(x);
  const int cfg = choose_tile(a, va && vb, workspace != nullptr);
  plan_splits(a, cfg, workspace, workspace_bytes);
  if (va && vb) launch_big<A_COLM, 4, B_WGRADX, 4>(a, st, cfg);
  else if (va) launch_small<A_COLM, 4, B_WGRADX, 1>(a, st, cfg);
  else if (vb) launch_small<A_COLM, 1, B_WGRADX, 4>(a, st, cfg);
  else launch_small<A_COLM, 1, B_WGRADX, 1>(a, st, cfg);
  return finish(a, st);
}

size_t mvae_conv2d_wgrad_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  GemmArgs a{};
  wgrad_args(a, nb, cin, cout, kh, kw, ho, wo);
  set_splits(a, choose_splits(a, choose_tile(a, true, true)));
  size_t b1 = splitk_ws_bytes(a);
  set_splits(a, choose_splits(a, choose_tile(a, false, true)));
  return std::max(b1, splitk_ws_bytes(a));
}

}  // extern "C"
