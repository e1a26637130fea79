// Implicit-GEMM convolution / strided-batched GEMM core on gfx950 MFMA (fp32 in HBM, "3xBF16" math).
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
// Global memory is read and written through buffer descriptors: an out-of-bounds element (padding,
// tile tails, gather holes) gets a byte offset past the descriptor's range and the hardware returns
// 0 / drops the store -- no exec-masked branches around loads, so loads stay pipelined.
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
#pragma once
#include "common.h"
#include <algorithm>
#include <stdlib.h>
#include <type_traits>

namespace mvae {

// operand kinds
// *_SPLIT kinds read operands already split into 3xBF16 hi/lo groups in HBM (split4_bf16 layout)
enum { A_ROWK = 0, A_COLM = 1, A_CONV_FWD = 2, A_CONV_UPS = 3, A_CONV_DGRAD = 4, A_CONV_SUBPIX = 5, A_COLM_PIX = 6,
       A_CONV_FWD_SPLIT = 7, A_CONV_DGRAD_SPLIT = 8, A_COLM_SPLIT = 9, A_ROWK_SPLIT = 10 };
enum { B_ROWK = 0, B_COLN = 1, B_WGRAD_FWD = 2, B_WGRAD_UPS = 3, B_WGRAD_SUBPIX = 4, B_ROWK_SPLIT = 5,
       B_WGRAD_FWD_SPLIT = 6, B_WGRAD_P2 = 7, B_WGRAD_P2_SPLIT = 8, B_COLN_SPLIT = 9 };
// B_WGRAD_P2(_SPLIT): the weight gradient's im2col gather of a stride-1 conv whose output is the input's size and whose
// H and W are powers of two (the c4 / c5 levels 64, 32, 16, 8): the source pixel of output pixel p through tap (r, s) is
// p + (r - pad_t) W + (s - pad_l), valid where h + r - pad_t and w + s - pad_l stay inside the image, and h, w come from p
// by shift and mask -- no per-K-tile division or stepping (GemmArgs::lw = log2 W)
// MODE_SUBPIX: one parity class (ph, pw) of "nearest-x2 upsample then 3x3 conv" as a stride-1 2x2 conv
// on the low-resolution input whose padding shifts with the parity: pad = pad_t - ph (batch entry
// bidx = 2*ph + pw carries the class)
enum { MODE_FWD = 0, MODE_UPS = 1, MODE_DGRAD = 2, MODE_SUBPIX = 3 };

constexpr int BK = 32;
// MFMA shape per kernel (template MF): v_mfma_f32_16x16x32_bf16 (MF 16) or v_mfma_f32_32x32x16_bf16
// (MF 32). Both take the same cycles per FLOP, but on random data the chip holds a higher clock under
// the 16x16x32 loop: +8-11 % bf16 FLOP/s in this kernel's per-wave structure (tools/micro/mfma_shape.hip),
// +3-5 % on the conv fwd/dgrad GEMMs. The wgrad / attention GEMMs, whose A operand is a transposed
// (COL) image, measured 5-7 % faster with 32x32x16 and keep it (mf_of).
template <int MF> using acc_of = typename std::conditional<MF == 32, f32x16, f32x4>::type;
template <int MF> constexpr int ks_of() { return BK / (MF == 32 ? 16 : 32); }  // MFMA k-steps per K-tile
template <int MF> constexpr int nr_of() { return MF == 32 ? 16 : 4; }          // accumulator registers per tile
// LDS swizzles, conflict-free for the fragment reads of both MFMA shapes:
//  ROW image: 16-B k-chunk c of row r sits at chunk position c ^ row_swz(r) (the 16x16x32 ds_read_b128
//             lane groups then hit 16 distinct 4-bank windows; 80-B pitch alone leaves them 2-way)
//  COL image: column col of k-row kr sits at col ^ col_swz(kr) (the two 16-lane halves of a 16x16x32
//             ds_read_b64_tr_b16, k-rows 8 apart, land in disjoint bank windows)
__device__ __forceinline__ int row_swz(int r) { return ((r >> 2) ^ (r >> 3) ^ (r >> 4)) & 1; }
__device__ __forceinline__ int col_swz(int kr) { return ((kr >> 3) & 1) << 4; }
// element offset of the 4-element group kc (0..7) of ROW-image row r
__device__ __forceinline__ int row_off(int r, int kc) { return r * 40 + (((kc >> 1) ^ row_swz(r)) << 3) + ((kc & 1) << 2); }
constexpr int MVAE_CONV_WSPLIT = 16;  // conv mode flag: weights hold split4_bf16 groups
constexpr int MVAE_CONV_XSPLIT = 32;  // conv mode flag: the input activation x holds split4_bf16 groups
constexpr int MVAE_CONV_DYSPLIT = 64;  // wgrad mode flag: the output gradient dy holds split4_bf16 groups
constexpr int MVAE_CONV_BF16 = 128;    // conv mode flag: the gathered operand and the weights are packed bf16 (PREC 4)
constexpr int MVAE_CONV_PLANAR = 256;  // conv mode flag: ... are planar 3xBF16 (bf16 hi plane, then lo plane; PREC 5)
constexpr int MVAE_CONV_DGRAD_DIRECT = 512;  // mvae_conv2d_direct32_nhwc: the input gradient (transposed conv of dy)

// Exact division by a runtime constant d for 0 <= n < 2^31 (Granlund-Montgomery, N = 31):
// q = (n * m) >> (31 + l), l = ceil(log2 d), m = floor(2^(31+l) / d) + 1 (< 2^32).
struct Magic {
  unsigned m;
  int sh;
};
inline Magic make_magic(int d) {
  int l = 0;
  while ((1LL << l) < d) ++l;
  return Magic{(unsigned)(((1ULL << (31 + l)) / (unsigned long long)d) + 1ULL), 31 + l};
}
__device__ __forceinline__ int mdiv(int n, Magic mg) {
  return (int)(((unsigned long long)(unsigned)n * mg.m) >> mg.sh);
}

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
  float* bias_ws;  // wgrad only: per-split row sums of A = dY^T (the conv bias gradient) [splits][M]
  unsigned a_bytes, b_bytes, c_bytes, r_bytes;  // descriptor ranges (per batch entry)
  unsigned a_lo = 0, b_lo = 0;  // PREC 5: byte offset of the operand's lo plane from its hi plane
  // gather geometry: source X is [nb][H][W][Cx]; output pixels are [nb][Ho][Wo]
  int H, W, Cx, Ho, Wo, R, S, stride, stride_shift, pad_t, pad_l;
  int lw = 0;  // log2 W (B_WGRAD_P2 gathers)
  int tiles_m, tiles_n;
  Magic mg_cx, mg_s, mg_hw, mg_wo;  // divisions by Cx, S, Ho*Wo, Wo (gather index decomposition)
  // conv K-order permutation (perm_rs = R*S, 1 = identity; needs Cx % 32 == 0): K-tile t covers channel
  // chunk t / RS of tap t % RS, so while the 32 CUs of an XCD sweep K their gathered input
  // footprint is one 32-channel slice of the image rows (L2-resident) instead of all channels of a
  // tap (which overflows L2 and re-fetches the input once per tap)
  int perm_rs = 1;
  Magic mg_rs = {0x80000001u, 31};  // make_magic(1)
  // parity-class output/pixel remap (sub-pixel decompositions): when sub_w2 > 0 the GEMM's pixel index
  // m = (n, i, j) over an [Ho][Wo] class grid maps to the full-resolution pixel (n, 2i+ph, 2j+pw) of a
  // [2Ho][2Wo = sub_w2] image: 4m - 2j + ph*sub_w2 + pw, class (ph, pw) = bidx + sub_par
  int sub_w2 = 0, sub_par = 0;
  int out_remap = 0;  // epilogue writes C row sub_pixel(m) (conv outputs); else row m
  int vec_epi = 0;    // set by launch_cfg: 16-B epilogue through LDS is legal (see gemm3x_kernel)
  // tile order within one split: the N tiles are cut into xcd_groups column groups and the tiles ordered (group, m,
  // n in group), so the contiguous run of tiles an XCD gets spans fewer B panels (1 = plain row-major order; set by
  // launch_cfg from MVAE_XCD_GROUPS when 0)
  int xcd_groups = 0;
  // GroupNorm statistics of the output for the following Normalize (16-B epilogue only): per 32-row block
  // and 4-channel group, {sum y, sum y^2} in fp64 at gn_part[((row/32) * (N/4) + col/4) * 2]
  double* gn_part = nullptr;
  // GroupNorm BACKWARD partials (16-B epilogue only): when C is the input gradient of a conv whose input was
  // y = silu?(GroupNorm(x)), emit per 32-row block and channel {sum dyn, sum dyn * xhat} (fp64) at
  // gnb_part[((row/32) * N + col) * 2], dyn = C * silu'(.) -- the sums the GroupNorm backward would
  // otherwise re-read C and x for (norm.hip gn_partial_kernel<1>, no dropout). x is [M][N] like C.
  double* gnb_part = nullptr;
  const float* gnb_x = nullptr;
  const float *gnb_mean = nullptr, *gnb_rstd = nullptr;  // [nb * G]
  const float *gnb_gamma = nullptr, *gnb_beta = nullptr;  // [N]
  int gnb_hw = 1, gnb_cpg = 1, gnb_G = 1, gnb_silu = 0;
};

// full-resolution pixel of class-grid pixel m (see GemmArgs::sub_w2)
__device__ __forceinline__ int sub_pixel(const GemmArgs& a, int m, int par_off) {
  const int j = m - mdiv(m, a.mg_wo) * a.Wo;
  return 4 * m - 2 * j + par_off;
}
__device__ __forceinline__ int sub_par_off(const GemmArgs& a, int bidx) {
  const int par = bidx + a.sub_par;
  return (par >> 1) * a.sub_w2 + (par & 1);
}

// column of the reference K order where (permuted) K-tile starting at k begins; k % 32 == 0
// (branch-free: perm_rs = 1 gives chunk = t, tap = 0, i.e. the identity)
__device__ __forceinline__ int kperm(const GemmArgs& a, int k) {
  const int t = k >> 5;
  const int chunk = mdiv(t, a.mg_rs);
  return (t - chunk * a.perm_rs) * a.Cx + chunk * BK;
}

inline void set_gather_magic(GemmArgs& a) {
  a.perm_rs = std::max(1, a.perm_rs);
  a.mg_rs = make_magic(a.perm_rs);
  a.mg_cx = make_magic(a.Cx);
  a.mg_s = make_magic(a.S);
  a.mg_hw = make_magic(a.Ho * a.Wo);
  a.mg_wo = make_magic(a.Wo);
}

constexpr unsigned OOB = 0xFFFFFFF0u;  // byte offset beyond every descriptor range
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return float4{__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}
__device__ __forceinline__ float bload1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void bstore1(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, unsigned off, const float4& v) {
  __builtin_amdgcn_raw_buffer_store_b128(
      u32x4_t{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)}, r, off, 0, 0);
}

template <int ROWS, bool COL>
struct Img {
  static constexpr int PITCH = COL ? ROWS + 32 : 40;
  static constexpr int PLANE = COL ? BK * PITCH : ROWS * PITCH;
  static constexpr int SIZE = 2 * PLANE;
};

// PREC 3: hi and lo planes (3xBF16); PREC 1: hi plane only (bf16 operands, fp32 accumulate).
// hi = bf16(x), lo = bf16(x - hi); per element pair: 2 cvt_pk, 1 shift + 1 and (hi back to fp32), 2 sub
// PREC 0 (exact fp32, f32-input MFMA): the planes hold the upper / lower 16 BITS of the fp32 word (a bit split,
// not a value split), so the fragment reads and swizzles of the bf16 images serve unchanged and mma<0>
// reassembles the exact fp32 operand
template <int PREC>
__device__ __forceinline__ void st_split(__bf16* img, int plane, int off, const float4& v) {
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
  if constexpr (PREC == 0) {
    const unsigned bx = __float_as_uint(v.x), by = __float_as_uint(v.y);
    const unsigned bz = __float_as_uint(v.z), bw = __float_as_uint(v.w);
    *(u32x2_t*)(img + off) = u32x2_t{(bx >> 16) | (by & 0xFFFF0000u), (bz >> 16) | (bw & 0xFFFF0000u)};
    *(u32x2_t*)(img + plane + off) = u32x2_t{(bx & 0xFFFFu) | (by << 16), (bz & 0xFFFFu) | (bw << 16)};
    return;
  }
  const unsigned h01 = pk_bf16x2(v.x, v.y), h23 = pk_bf16x2(v.z, v.w);
  *(u32x2_t*)(img + off) = u32x2_t{h01, h23};
  if constexpr (PREC == 3) {
    const unsigned l01 = pk_bf16x2(v.x - __uint_as_float(h01 << 16), v.y - __uint_as_float(h01 & 0xFFFF0000u));
    const unsigned l23 = pk_bf16x2(v.z - __uint_as_float(h23 << 16), v.w - __uint_as_float(h23 & 0xFFFF0000u));
    *(u32x2_t*)(img + plane + off) = u32x2_t{l01, l23};
  }
}

// slot already split in HBM (split4_bf16 layout: per 4 elements hi0..hi3 then lo0..lo3, 16 B; in the exact fp32
// arithmetic, PREC 0, the split4_bits bit split of the same shape -- st_split<0>'s planes)
template <int PREC>
__device__ __forceinline__ void st_presplit(__bf16* img, int plane, int off, const float4& v) {
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2_t;
  *(u32x2_t*)(img + off) = u32x2_t{__float_as_uint(v.x), __float_as_uint(v.y)};
  if constexpr (PREC == 3 || PREC == 0)
    *(u32x2_t*)(img + plane + off) = u32x2_t{__float_as_uint(v.z), __float_as_uint(v.w)};
}

// MFMA operand fragment, k-step ks of the K-tile.
//  32x32x16: lane l holds element [row0 + (l&31)][ks*16 + 8*(l>>5) + j]
//  16x16x32: lane l holds element [row0 + (l&15)][8*(l>>4) + j]
template <int ROWS, bool COL, int MF>
__device__ __forceinline__ bf16x8 read_frag(const __bf16* plane, int row0, int ks, int lane) {
  if constexpr (!COL) {
    if constexpr (MF == 32) {
      const int r = row0 + (lane & 31);
      return *(const bf16x8*)(plane + r * 40 + (((2 * ks + (lane >> 5)) ^ row_swz(r)) << 3));
    } else {
      const int r = row0 + (lane & 15);
      return *(const bf16x8*)(plane + r * 40 + (((lane >> 4) ^ row_swz(r)) << 3));
    }
  } else {
    constexpr int P = Img<ROWS, true>::PITCH;
    const int g = lane >> 4, li = lane & 15;
    const __bf16* p;
    if constexpr (MF == 32) {
      const int kr = ks * 16 + (g >> 1) * 8 + (li >> 2);
      p = plane + kr * P + ((row0 + (g & 1) * 16 + 4 * (li & 3)) ^ col_swz(kr));
    } else {
      const int kr = g * 8 + (li >> 2);
      p = plane + kr * P + ((row0 + 4 * (li & 3)) ^ col_swz(kr));
    }
    const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)p);
    const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(p + 4 * P));
    return __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// source pixel of output pixel (oh,ow) for filter tap (r,s); MODE is a compile-time constant
template <int MODE>
__device__ __forceinline__ bool tap_src(const GemmArgs& a, int pt, int pl, int oh, int ow, int r, int s, int& ih,
                                        int& iw) {
  if constexpr (MODE == MODE_FWD) {
    ih = oh * a.stride - a.pad_t + r;
    iw = ow * a.stride - a.pad_l + s;
    return ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
  } else if constexpr (MODE == MODE_SUBPIX) {  // stride 1, class-dependent padding pt / pl
    ih = oh - pt + r;
    iw = ow - pl + s;
    return ((unsigned)ih < (unsigned)a.H) & ((unsigned)iw < (unsigned)a.W);
  } else if constexpr (MODE == MODE_UPS) {  // nearest x2 upsample, then conv (stride 1)
    const int uh = oh - a.pad_t + r, uw = ow - a.pad_l + s;
    ih = uh >> 1;
    iw = uw >> 1;
    return ((unsigned)uh < (unsigned)(2 * a.H)) & ((unsigned)uw < (unsigned)(2 * a.W));
  } else {  // transposed gather (dgrad of a strided conv); stride is a power of two
    const int nh = oh + a.pad_t - r, nw = ow + a.pad_l - s;
    const int msk = a.stride - 1;
    ih = nh >> a.stride_shift;
    iw = nw >> a.stride_shift;
    return (nh >= 0) & (nw >= 0) & (((nh | nw) & msk) == 0) & (ih < a.H) & (iw < a.W);
  }
}

// Row of the ROW-image store pattern for thread tid: a wave stages 8 rows x 32 k (8 lanes per row).
// ds_write_b64 serves 16 lanes (2 rows) per LDS cycle; with the 80-B row pitch rows r and r+1 overlap
// in 4 banks, rows r and r+4 are 16 banks apart -- so lane groups pair rows (0,4),(1,5),(2,6),(3,7).
__device__ __forceinline__ int row_of_tid(int tid) {
#ifdef MVAE_NO_ROW_SWIZZLE
  return tid >> 3;
#else
  const int g = (tid >> 3) & 7;
  return (tid >> 6) * 8 + ((g >> 1) | ((g & 1) << 2));
#endif
}

// ------------------------------------------------------------------------------------------
// operand loaders. Each thread stages NS float4 "slots" of a BK-deep K-tile:
//   init(args, base, row0, k_begin, tid)
//   prep(args)          per-tile index math for the tile at the current k (before load_slot)
//   load_slot(args, i)  issue the global load of slot i
//   store_slot(img, i)  split slot i into hi/lo bf16 and write it into the operand's LDS image
//   advance()           k += BK
// load() / store() run every slot. Slots let the main loop interleave the staging of tile t+1 with
// the MFMAs of tile t, one slot at a time.
// ------------------------------------------------------------------------------------------

// ROW image, source element (row, k) at P[row*ld + k]
template <int ROWS, int VEC, int NT, bool IS_A, int PREC, bool PRESPLIT = false>
struct LoadRowK {
  static constexpr bool COL = false;
  static constexpr int RP = NT / 8;     // rows per pass (8 float4 per 32-wide row)
  static constexpr int NS = ROWS / RP;  // rows per thread
  __amdgpu_buffer_rsrc_t rs;
  unsigned ld;
  int rows, K, row0, k, kc, r0, kk;
  float4 v[NS];
  __device__ void init(const GemmArgs& a, const float* p, int row0_, int kb, int tid, int) {
    rs = make_rsrc(p, IS_A ? a.a_bytes : a.b_bytes);
    ld = (unsigned)(IS_A ? a.lda : a.ldb); rows = IS_A ? a.M : a.N; K = a.K;
    row0 = row0_; k = kb; kc = tid & 7; r0 = row_of_tid(tid);
  }
  __device__ void prep(const GemmArgs& a) { kk = kperm(a, k) + kc * 4; }
  __device__ void load_slot(const GemmArgs&, int i) {
    const int row = row0 + r0 + RP * i;
    const unsigned base = ((unsigned)row * ld + (unsigned)kk) * 4u;
    const bool rv = row < rows;
    if (VEC == 4) {
      v[i] = bload4(rs, (rv & (kk < K)) ? base : OOB);
    } else {
      v[i].x = bload1(rs, (rv & (kk + 0 < K)) ? base : OOB);
      v[i].y = bload1(rs, (rv & (kk + 1 < K)) ? base + 4 : OOB);
      v[i].z = bload1(rs, (rv & (kk + 2 < K)) ? base + 8 : OOB);
      v[i].w = bload1(rs, (rv & (kk + 3 < K)) ? base + 12 : OOB);
    }
  }
  __device__ void store_slot(__bf16* img, int i) {
    if constexpr (PRESPLIT)
      st_presplit<PREC>(img, Img<ROWS, false>::PLANE, row_off(r0 + RP * i, kc), v[i]);
    else
      st_split<PREC>(img, Img<ROWS, false>::PLANE, row_off(r0 + RP * i, kc), v[i]);
  }
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
    prep(a);
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// ROW image, implicit im2col of an NHWC tensor: element (pixel m, k = (r*S+s)*Cx + c)
// Vector path (VEC 4, every mode but MODE_UPS): the source pixel of row m through tap (r, s) is an affine function
// base(m) + delta(r, s) in every gather mode -- MODE_FWD: (oh*stride + r - pad_t, ...); MODE_SUBPIX: (oh + r - pt,
// ...); MODE_DGRAD (stride 2^q): ((oh + pad_t) >> q) - (r >> q) where (oh + pad_t - r) is a multiple of the stride.
// So init() keeps per row one byte offset of base(m) and a bit mask of the taps whose source pixel exists (tap_src
// evaluated once per tap), prep() turns the lane's k column into (tap bit, delta bytes) once per K-tile, and a slot
// load is an AND, a compare, an add and a select -- instead of the per-slot tap decomposition, bounds checks and
// multiplies of the scalar path.
template <int ROWS, int VEC, int NT, int MODE, int PREC, bool PRESPLIT = false>
struct LoadConvA {
  static constexpr bool COL = false;
  static constexpr bool FAST = VEC == 4 && MODE != MODE_UPS;
  static constexpr int RP = NT / 8;
  static constexpr int NS = ROWS / RP;
  static constexpr int NE = VEC == 4 ? 1 : 4;  // (c, r, s) decompositions per thread (scalar path)
  __amdgpu_buffer_rsrc_t rs;
  int kc, r0, k;
  float4 v[NS];
  int pt, pl;  // MODE_SUBPIX: padding of this batch entry's parity class
  // vector path
  unsigned rowbase[NS], vmask[NS];
  unsigned tbit;
  int delta;
  // scalar path
  unsigned base[NS];
  int oh[NS], ow[NS];
  bool mv[NS];
  int cc[NE], rr[NE], ss[NE];
  bool kv[NE];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid, int bidx) {
    rs = make_rsrc(x, a.a_bytes);
    kc = tid & 7; r0 = row_of_tid(tid); k = kb;
    pt = a.pad_t - ((bidx + a.sub_par) >> 1);
    pl = a.pad_l - ((bidx + a.sub_par) & 1);
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      const int m = row0 + r0 + RP * i;
      const bool valid = m < a.M;
      const int mm = valid ? m : 0;
      const int b = mdiv(mm, a.mg_hw);
      const int rem = mm - b * (a.Ho * a.Wo);
      const int h_ = mdiv(rem, a.mg_wo);
      const int w_ = rem - h_ * a.Wo;
      if constexpr (FAST) {
        int bh, bw;
        if constexpr (MODE == MODE_FWD) {
          bh = h_ * a.stride;
          bw = w_ * a.stride;
        } else if constexpr (MODE == MODE_SUBPIX) {
          bh = h_;
          bw = w_;
        } else {  // MODE_DGRAD
          bh = (h_ + a.pad_t) >> a.stride_shift;
          bw = (w_ + a.pad_l) >> a.stride_shift;
        }
        rowbase[i] = (((unsigned)b * (unsigned)a.H + (unsigned)bh) * (unsigned)a.W + (unsigned)bw) * (unsigned)a.Cx * 4u;
        unsigned msk = 0;
        for (int r = 0; r < a.R; ++r)
          for (int s_ = 0; s_ < a.S; ++s_) {
            int ih = 0, iw = 0;
            if (tap_src<MODE>(a, pt, pl, h_, w_, r, s_, ih, iw)) msk |= 1u << (r * a.S + s_);
          }
        vmask[i] = valid ? msk : 0u;
      } else {
        mv[i] = valid;
        oh[i] = h_;
        ow[i] = w_;
        base[i] = (unsigned)b * (unsigned)(a.H * a.W);
      }
    }
  }
  // (c, r, s) of this thread's k columns, by exact multiply-shift division: branch-free, so the
  // steady-state loop stays one basic block
  __device__ void prep(const GemmArgs& a) {
    const int kp = kperm(a, k);
    if constexpr (FAST) {
      const int kk = kp + kc * 4;
      const int tap = mdiv(kk, a.mg_cx);
      const int c = kk - tap * a.Cx;
      const int r = mdiv(tap, a.mg_s);
      const int s_ = tap - r * a.S;
      int dh, dw;
      if constexpr (MODE == MODE_FWD) {
        dh = r - a.pad_t;
        dw = s_ - a.pad_l;
      } else if constexpr (MODE == MODE_SUBPIX) {
        dh = r - pt;
        dw = s_ - pl;
      } else {
        dh = -(r >> a.stride_shift);
        dw = -(s_ >> a.stride_shift);
      }
      delta = ((dh * a.W + dw) * a.Cx + c) * 4;
      tbit = kk < a.K ? 1u << tap : 0u;
    } else {
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int kk = kp + kc * 4 + e;
        const int tap = mdiv(kk, a.mg_cx);
        cc[e] = kk - tap * a.Cx;
        rr[e] = mdiv(tap, a.mg_s);
        ss[e] = tap - rr[e] * a.S;
        kv[e] = kk < a.K;
      }
    }
  }
  __device__ void load_slot(const GemmArgs& a, int i) {
    if constexpr (FAST) {
      const unsigned off = rowbase[i] + (unsigned)delta;
      v[i] = bload4(rs, (vmask[i] & tbit) ? off : OOB);
    } else if (VEC == 4) {
      int ih = 0, iw = 0;
      const bool tv = tap_src<MODE>(a, pt, pl, oh[i], ow[i], rr[0], ss[0], ih, iw);
      const bool ok = mv[i] & kv[0] & tv;
      const unsigned off = ((base[i] + (unsigned)(ih * a.W + iw)) * (unsigned)a.Cx + (unsigned)cc[0]) * 4u;
      v[i] = bload4(rs, ok ? off : OOB);
    } else {
      float t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int ih = 0, iw = 0;
        const bool tv = tap_src<MODE>(a, pt, pl, oh[i], ow[i], rr[e], ss[e], ih, iw);
        const bool ok = mv[i] & kv[e] & tv;
        const unsigned off = ((base[i] + (unsigned)(ih * a.W + iw)) * (unsigned)a.Cx + (unsigned)cc[e]) * 4u;
        t[e] = bload1(rs, ok ? off : OOB);
      }
      v[i] = float4{t[0], t[1], t[2], t[3]};
    }
  }
  __device__ void store_slot(__bf16* img, int i) {
    if constexpr (PRESPLIT)
      st_presplit<PREC>(img, Img<ROWS, false>::PLANE, row_off(r0 + RP * i, kc), v[i]);
    else
      st_split<PREC>(img, Img<ROWS, false>::PLANE, row_off(r0 + RP * i, kc), v[i]);
  }
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
    prep(a);
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// COL image, source element (row, k) at P[k*ld + row] (rows contiguous); PRESPLIT: the source holds
// split4_bf16 groups of 4 consecutive rows (the wgrad dY^T operand split once per conv, not per workgroup)
template <int ROWS, int VEC, int NT, bool IS_A, int PREC, bool PRESPLIT = false>
struct LoadColK {
  static constexpr bool COL = true;
  static constexpr int C4 = ROWS / 4;                 // float4 per k-row
  static constexpr int NS = (BK * C4 + NT - 1) / NT;  // float4 per thread
  static constexpr bool KROW_CHECK = NS * (NT / C4) != BK;  // false: every thread's k-rows are < BK
  __amdgpu_buffer_rsrc_t rs;
  unsigned ld;
  int rows, K, row0, k, c4, kr;
  float4 v[NS];
  float bs[4] = {0.f, 0.f, 0.f, 0.f};  // A side: running row sums of every staged element
  __device__ void init(const GemmArgs& a, const float* p, int row0_, int kb, int tid, int) {
    rs = make_rsrc(p, IS_A ? a.a_bytes : a.b_bytes);
    ld = (unsigned)(IS_A ? a.lda : a.ldb); rows = IS_A ? a.M : a.N; K = a.K;
    row0 = row0_; k = kb; c4 = tid % C4; kr = tid / C4;
  }
  __device__ void prep(const GemmArgs&) {}
  __device__ void load_slot(const GemmArgs&, int i) {
    const int col = row0 + c4 * 4;
    const int krow = kr + i * (NT / C4);
    const int kk = k + krow;
    const bool kv = (!KROW_CHECK || krow < BK) & (kk < K);
    const unsigned base = ((unsigned)kk * ld + (unsigned)col) * 4u;
    if (VEC == 4) {
      v[i] = bload4(rs, (kv & (col < rows)) ? base : OOB);
    } else {
      v[i].x = bload1(rs, (kv & (col + 0 < rows)) ? base : OOB);
      v[i].y = bload1(rs, (kv & (col + 1 < rows)) ? base + 4 : OOB);
      v[i].z = bload1(rs, (kv & (col + 2 < rows)) ? base + 8 : OOB);
      v[i].w = bload1(rs, (kv & (col + 3 < rows)) ? base + 12 : OOB);
    }
  }
  bool want_bs = true;  // A side: accumulate the row sums (conv bias gradient) -- wave-uniform
  __device__ void store_slot(__bf16* img, int i) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
    const int krow = kr + i * (NT / C4);
    if (!KROW_CHECK || krow < BK) {
      if constexpr (PRESPLIT) {
        st_presplit<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
        // (a pre-split A = dY^T carries no bias sums: its producer -- the GroupNorm backward, or the host's bias pass
        // over the fp32 dy -- sums the conv bias gradient; mvae_conv2d_wgrad_nhwc rejects dbias with MVAE_CONV_DYSPLIT)
      } else {
        st_split<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
        if constexpr (IS_A) {  // (masked, not branched: a uniform branch here splits the pipelined K loop)
          const float wm = want_bs ? 1.f : 0.f;
          bs[0] = fmaf(wm, v[i].x, bs[0]); bs[1] = fmaf(wm, v[i].y, bs[1]);
          bs[2] = fmaf(wm, v[i].z, bs[2]); bs[3] = fmaf(wm, v[i].w, bs[3]);
        }
      }
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// COL image of A = dY^T whose k (pixel) index walks one parity class of a full-resolution image:
// element (row, k) at P[sub_pixel(k)*ld + row] (the wgrad of the sub-pixel Upsample conv)
template <int ROWS, int VEC, int NT, int PREC>
struct LoadColPix {
  static constexpr bool COL = true;
  static constexpr int C4 = ROWS / 4;
  static constexpr int NS = (BK * C4 + NT - 1) / NT;
  static constexpr bool KROW_CHECK = NS * (NT / C4) != BK;
  __amdgpu_buffer_rsrc_t rs;
  unsigned ld;
  int rows, K, row0, k, c4, kr, krw, par_off;
  unsigned pix[NS];
  float4 v[NS];
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  __device__ void init(const GemmArgs& a, const float* p, int row0_, int kb, int tid, int bidx) {
    rs = make_rsrc(p, a.a_bytes);
    ld = (unsigned)a.lda; rows = a.M; K = a.K;
    row0 = row0_; k = kb; c4 = tid % C4; kr = tid / C4;
    krw = (C4 % 64 == 0) ? __builtin_amdgcn_readfirstlane(kr) : kr;
    par_off = sub_par_off(a, bidx);
  }
  __device__ void prep(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < NS; ++i) pix[i] = (unsigned)sub_pixel(a, min(k + krw + i * (NT / C4), K - 1), par_off);
  }
  __device__ void load_slot(const GemmArgs&, int i) {
    const int col = row0 + c4 * 4;
    const int krow = kr + i * (NT / C4);
    const bool kv = (!KROW_CHECK || krow < BK) & (k + krow < K);
    const unsigned base = (pix[i] * ld + (unsigned)col) * 4u;
    if (VEC == 4) {
      v[i] = bload4(rs, (kv & (col < rows)) ? base : OOB);
    } else {
      v[i].x = bload1(rs, (kv & (col + 0 < rows)) ? base : OOB);
      v[i].y = bload1(rs, (kv & (col + 1 < rows)) ? base + 4 : OOB);
      v[i].z = bload1(rs, (kv & (col + 2 < rows)) ? base + 8 : OOB);
      v[i].w = bload1(rs, (kv & (col + 3 < rows)) ? base + 12 : OOB);
    }
  }
  __device__ void store_slot(__bf16* img, int i) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
    const int krow = kr + i * (NT / C4);
    if (!KROW_CHECK || krow < BK) {
      st_split<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
      const float wm = want_bs ? 1.f : 0.f;  // (masked, not branched)
      bs[0] = fmaf(wm, v[i].x, bs[0]); bs[1] = fmaf(wm, v[i].y, bs[1]);
      bs[2] = fmaf(wm, v[i].z, bs[2]); bs[3] = fmaf(wm, v[i].w, bs[3]);
    }
  }
  bool want_bs = true;
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
    prep(a);
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// COL image for the wgrad B operand: rows n' = (r*S+s)*Cx + c (filter element), k = output pixel.
// element = X[b][src(oh,ow,r,s)][c], contiguous along c.
// Affine variant (FAST): a lane's 4 columns are one tap (r, s) and 4 channels, fixed for the launch, so init() keeps
// the lane's tap offset ((r*W + s)*Cx + c) * 4 and prep() reduces each k-row (pixel) to wave-uniform values -- the
// byte offset of its shifted origin (oh*stride - pad, ow*stride - pad) and those two coordinates.
template <int ROWS, int VEC, int NT, int MODE, int PREC, bool PRESPLIT = false>
struct LoadWgradX {
  static constexpr bool COL = true;
  // (measured: the affine form moves index math from the VALU to the SALU here -- the k-rows are wave-uniform --
  // and ran the c4 wgrad GEMMs 3 % slower; kept off)
  static constexpr bool FAST = false;
  static constexpr int C4 = ROWS / 4;
  static constexpr int NS = (BK * C4 + NT - 1) / NT;
  static constexpr bool KROW_CHECK = NS * (NT / C4) != BK;
  __amdgpu_buffer_rsrc_t rs;
  int c4, kr, krw, k;
  int cc[4], rr[4], ss[4];
  bool nv[4];
  int pb[NS], poh[NS], pow_[NS];  // pixel decomposition of this thread's k-rows (current tile)
  // vector path: lane-fixed tap offset, per k-row origin (uniform when C4 % 64 == 0)
  unsigned ldelta;
  unsigned sbase[NS];
  int sh[NS], sw[NS];
  float4 v[NS];
  int pt, pl;
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid, int bidx) {
    rs = make_rsrc(x, a.b_bytes);
    k = kb; c4 = tid % C4; kr = tid / C4;
    pt = a.pad_t - ((bidx + a.sub_par) >> 1);
    pl = a.pad_l - ((bidx + a.sub_par) & 1);
    for (int e = 0; e < 4; ++e) {
      const int n = row0 + c4 * 4 + e;
      nv[e] = n < a.N;
      const int nn = nv[e] ? n : 0;
      const int tap = nn / a.Cx;
      cc[e] = nn - tap * a.Cx;
      rr[e] = tap / a.S;
      ss[e] = tap - rr[e] * a.S;
    }
    if constexpr (FAST) ldelta = (unsigned)(((rr[0] * a.W + ss[0]) * a.Cx + cc[0]) * 4);
    // with 64 column groups the k-row is wave-uniform: keep the pixel walk in scalar registers
    krw = (C4 % 64 == 0) ? __builtin_amdgcn_readfirstlane(kr) : kr;
  }
  __device__ void prep(const GemmArgs& a) {
#ifdef MVAE_WGRAD_XFAKE  // timing-only build: no gather index math (wrong results)
    return;
#endif
    // slot 0's pixel by division; the others step from it (pixels NT / C4 apart: usually the same or the next image
    // row), so each K-tile costs one decomposition instead of NS -- the k-rows are wave-uniform, this is scalar work
    // on every wave of the workgroup, and the wgrad loop is short of scalar issue (PMC: 16 % of wave cycles in the
    // bf16 mode)
    const int p0 = min(k + krw, a.K - 1);  // clamp: rows past K are masked
    pb[0] = mdiv(p0, a.mg_hw);
    {
      const int rem = p0 - pb[0] * (a.Ho * a.Wo);
      poh[0] = mdiv(rem, a.mg_wo);
      pow_[0] = rem - poh[0] * a.Wo;
    }
#pragma unroll
    for (int i = 1; i < NS; ++i) {
      int w_ = pow_[i - 1] + NT / C4, h_ = poh[i - 1], b_ = pb[i - 1];
      while (w_ >= a.Wo) {
        w_ -= a.Wo;
        ++h_;
      }
      while (h_ >= a.Ho) {
        h_ -= a.Ho;
        ++b_;
      }
      pb[i] = b_;  // (past K only for masked rows: any in-range decomposition will do)
      poh[i] = h_;
      pow_[i] = w_;
    }
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      if constexpr (FAST) {
        if constexpr (MODE == MODE_FWD) {
          sh[i] = poh[i] * a.stride - a.pad_t;
          sw[i] = pow_[i] * a.stride - a.pad_l;
        } else {
          sh[i] = poh[i] - pt;
          sw[i] = pow_[i] - pl;
        }
        sbase[i] = (unsigned)((pb[i] * a.H + sh[i]) * a.W + sw[i]) * (unsigned)a.Cx * 4u;
      }
    }
  }
  __device__ void load_slot(const GemmArgs& a, int i) {
    const unsigned img = (unsigned)(a.H * a.W);
    const int krow = kr + i * (NT / C4);
    const bool kv = (!KROW_CHECK || krow < BK) & (k + krow < a.K);
#ifdef MVAE_WGRAD_XFAKE
    if (VEC == 4) {
      v[i] = bload4(rs, (kv & nv[0]) ? (unsigned)(((k + krow) * a.Cx + cc[0]) * 4) : OOB);
      return;
    }
#endif
    if constexpr (FAST) {
      const bool ok = kv & nv[0] & ((unsigned)(sh[i] + rr[0]) < (unsigned)a.H) & ((unsigned)(sw[i] + ss[0]) < (unsigned)a.W);
      v[i] = bload4(rs, ok ? sbase[i] + ldelta : OOB);
    } else if (VEC == 4) {
      int ih = 0, iw = 0;
      const bool tv = tap_src<MODE>(a, pt, pl, poh[i], pow_[i], rr[0], ss[0], ih, iw);
      const bool ok = kv & nv[0] & tv;
      const unsigned off = (((unsigned)pb[i] * img + (unsigned)(ih * a.W + iw)) * (unsigned)a.Cx + (unsigned)cc[0]) * 4u;
      v[i] = bload4(rs, ok ? off : OOB);
    } else {
      float t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int ih = 0, iw = 0;
        const bool tv = tap_src<MODE>(a, pt, pl, poh[i], pow_[i], rr[e], ss[e], ih, iw);
        const bool ok = kv & nv[e] & tv;
        const unsigned off =
            (((unsigned)pb[i] * img + (unsigned)(ih * a.W + iw)) * (unsigned)a.Cx + (unsigned)cc[e]) * 4u;
        t[e] = bload1(rs, ok ? off : OOB);
      }
      v[i] = float4{t[0], t[1], t[2], t[3]};
    }
  }
  __device__ void store_slot(__bf16* img, int i) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
    const int krow = kr + i * (NT / C4);
    if (!KROW_CHECK || krow < BK) {
      if constexpr (PRESPLIT)
        st_presplit<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
      else
        st_split<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
    prep(a);
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// COL image of the weight gradient's B operand for B_WGRAD_P2(_SPLIT) (see the enum): element (n = (r*S+s)*Cx + c,
// k = pixel p) = X[p + (r - pad_t) W + (s - pad_l)][c] where the shifted pixel stays in the image. A lane's 4 columns
// are one tap and 4 channels for the whole launch (tap offset `ldelta` fixed at init); a k-row (pixel) needs only a mask
// and a shift for its (h, w) -- wave-uniform when C4 % 64 == 0 -- instead of LoadWgradX's division and row stepping
template <int ROWS, int NT, int PREC, bool PRESPLIT>
struct LoadWgradXP2 {
  static constexpr bool COL = true;
  static constexpr int C4 = ROWS / 4;
  static constexpr int NS = (BK * C4 + NT - 1) / NT;
  static constexpr bool KROW_CHECK = NS * (NT / C4) != BK;
  __amdgpu_buffer_rsrc_t rs;
  int c4, kr, krw, k, dr, ds;
  unsigned ldelta, cx4;
  bool nv;
  float4 v[NS];
  __device__ void init(const GemmArgs& a, const float* x, int row0, int kb, int tid, int) {
    rs = make_rsrc(x, a.b_bytes);
    k = kb; c4 = tid % C4; kr = tid / C4;
    const int n = row0 + c4 * 4;
    nv = n < a.N;
    const int nn = nv ? n : 0;
    const int tap = nn / a.Cx, c = nn - tap * a.Cx;
    const int r = tap / a.S, s = tap - r * a.S;
    dr = r - a.pad_t;
    ds = s - a.pad_l;
    ldelta = (unsigned)(((dr * a.W + ds) * a.Cx + c) * 4);  // (wraps for negative shifts; used only when valid)
    cx4 = (unsigned)a.Cx * 4u;
    krw = (C4 % 64 == 0) ? __builtin_amdgcn_readfirstlane(kr) : kr;
  }
  __device__ void prep(const GemmArgs&) {}
  __device__ void load_slot(const GemmArgs& a, int i) {
    const int krow = kr + i * (NT / C4);
    const int p = k + krw + i * (NT / C4);
    const int w = p & (a.W - 1), h = (p >> a.lw) & (a.H - 1);
    const bool ok = (!KROW_CHECK || krow < BK) & (p < a.K) & nv & ((unsigned)(h + dr) < (unsigned)a.H) &
                    ((unsigned)(w + ds) < (unsigned)a.W);
    v[i] = bload4(rs, ok ? (unsigned)p * cx4 + ldelta : OOB);
  }
  __device__ void store_slot(__bf16* img, int i) {
    constexpr int P_ = Img<ROWS, true>::PITCH;
    const int krow = kr + i * (NT / C4);
    if (!KROW_CHECK || krow < BK) {
      if constexpr (PRESPLIT)
        st_presplit<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
      else
        st_split<PREC>(img, Img<ROWS, true>::PLANE, krow * P_ + ((c4 * 4) ^ col_swz(krow)), v[i]);
    }
  }
  __device__ void advance() { k += BK; }
  __device__ void load(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < NS; ++i) load_slot(a, i);
  }
  __device__ void store(__bf16* img) {
#pragma unroll
    for (int i = 0; i < NS; ++i) store_slot(img, i);
  }
};

// ------------------------------------------------------------------------------------------
// LDS-DMA operand staging (buffer_load_dwordx4 ... lds): no staging registers, no VALU split, no ds_write.
//   PREC 4 (bf16-mixed): operands STORED as packed bf16 by their producers; 64-deep stages.
//   PREC 5 (3xBF16): operands stored PLANAR -- a bf16 hi plane (hi = bf16(x)) followed, GemmArgs::a_lo / b_lo bytes
//          later, by the lo plane (lo = bf16(x - hi)) -- each plane DMA'd into its own LDS image; 32-deep stages.
// ROW images [ROWS][KT] bf16, filled lane-linearly (one DMA instruction = 1 KB = 1024 / (2 KT) rows, lane l -> row
// l / (KT/8), 16-B slot l % (KT/8)) and swizzled on the SOURCE side: physical slot p of row r holds the row's logical
// 8-element chunk p ^ dswz(r), and fragment reads apply the same involution (ds_read_b128 lane groups {0-3,12-15,
// 20-27}, {4-11,16-19,28-31}, ... then hit 16 distinct 16-B bank windows: 128-B rows use (r >> 1) & 7, 64-B rows
// [0,3,2,1][(r >> 2) & 3]).
// ------------------------------------------------------------------------------------------
constexpr int DBK = 64;  // split-K granularity (whole stages of either loop)
#ifndef MVAE_DMA_SPREAD  // 1: COL (weight-gradient) loops spread their DMA issue over the k-steps; 2: every loop
#define MVAE_DMA_SPREAD 1
#endif
template <int KT>
__device__ __forceinline__ int dswz(int r) { return KT == 64 ? (r >> 1) & 7 : (4 - ((r >> 2) & 3)) & 3; }
typedef __attribute__((address_space(3))) void lds_void_t;

// (permuted) stage starting at k (k % KT == 0): channel chunk t / RS of tap t % RS, KT channels wide
template <int KT>
__device__ __forceinline__ int kperm_dma(const GemmArgs& a, int k) {
  const int t = k / KT;
  const int chunk = mdiv(t, a.mg_rs);
  return (t - chunk * a.perm_rs) * a.Cx + chunk * KT;
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, __bf16* dst, unsigned off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)dst, 16, off, 0, 0, 0);
}

// Piece q of a ROWS-row image (1 KB) is filled by wave (q % (NT/64)) as its instruction q / (NT/64); with an even
// wave count a lane's logical chunk (slot ^ dswz(row)) is the same for all its pieces.
template <int ROWS, int NT, int KT>
struct DmaShape {
  static constexpr int NW = NT / 64;
  static constexpr int CH = KT / 8;    // 16-B chunks per row
  static constexpr int PR = 64 / CH;   // rows per piece
  static constexpr int NI = ROWS * KT / (NT * 8);  // DMA instructions per thread per stage and plane
  static_assert(NI >= 1 && NI * NT * 8 == ROWS * KT && NW % 2 == 0, "DMA image shape");
};
template <int KT>
__device__ __forceinline__ int dma_chunk(int lane, int w) {
  const int row = w * (512 / KT) + lane / (KT / 8);  // any of the lane's rows: the swizzle is the same
  return (lane % (KT / 8)) ^ dswz<KT>(row);
}
// descriptors of the hi plane (or the packed bf16 operand) and of the lo plane lo_off bytes later
__device__ __forceinline__ void plane_rsrc(__amdgpu_buffer_rsrc_t (&rs)[2], const __bf16* p, unsigned bytes,
                                           unsigned lo_off) {
  rs[0] = make_rsrc(p, bytes);
  rs[1] = make_rsrc((const char*)p + lo_off, bytes);
}

// ROW image of a row-major bf16 matrix: element (row, k) at P[row*ld + kperm(k)]
template <int ROWS, int NT, bool IS_A, int KT>
struct DmaRowK {
  using S = DmaShape<ROWS, NT, KT>;
  __amdgpu_buffer_rsrc_t rs[2];
  unsigned rowoff[S::NI];
  bool rv[S::NI];
  int cb, k, K, w;
  unsigned kb2;
  bool kv;
  __device__ void init(const GemmArgs& a, const __bf16* p, int row0, int kb, int tid, int) {
    plane_rsrc(rs, p, IS_A ? a.a_bytes : a.b_bytes, IS_A ? a.a_lo : a.b_lo);
    const int lane = tid & 63;
    w = tid >> 6;
    cb = dma_chunk<KT>(lane, w);
    const unsigned ld = (unsigned)(IS_A ? a.lda : a.ldb);
    const int rows = IS_A ? a.M : a.N;
    K = a.K; k = kb;
#pragma unroll
    for (int i = 0; i < S::NI; ++i) {
      const int row = row0 + (i * S::NW + w) * S::PR + lane / S::CH;
      rv[i] = row < rows;
      rowoff[i] = (unsigned)row * ld * 2u;
    }
  }
  __device__ void prep(const GemmArgs& a) {
    const int kk = kperm_dma<KT>(a, k) + cb * 8;
    kv = kk < K;
    kb2 = (unsigned)kk * 2u;
  }
  __device__ unsigned src(int i) const { return (rv[i] & kv) ? rowoff[i] + kb2 : OOB; }  // source of piece i
  __device__ void issue(const GemmArgs&, __bf16* img, int i, int pl) { dma16(rs[pl], img + (i * S::NW + w) * 512, src(i)); }
  __device__ void advance() { k += KT; }
};

// ROW image of the implicit im2col of a bf16 NHWC tensor (affine gather of LoadConvA's vector path, in bf16
// bytes); needs Cx % 8 == 0 (a 16-B chunk never straddles two taps) and <= 32 taps
template <int ROWS, int NT, int MODE, int KT>
struct DmaConvA {
  using S = DmaShape<ROWS, NT, KT>;
  __amdgpu_buffer_rsrc_t rs[2];
  unsigned rowbase[S::NI], vmask[S::NI];
  unsigned tbit;
  int delta;
  int cb, k, w, pt, pl;
  __device__ void init(const GemmArgs& a, const __bf16* x, int row0, int kb, int tid, int bidx) {
    plane_rsrc(rs, x, a.a_bytes, a.a_lo);
    const int lane = tid & 63;
    w = tid >> 6;
    cb = dma_chunk<KT>(lane, w);
    k = kb;
    pt = a.pad_t - ((bidx + a.sub_par) >> 1);
    pl = a.pad_l - ((bidx + a.sub_par) & 1);
#pragma unroll
    for (int i = 0; i < S::NI; ++i) {
      const int m = row0 + (i * S::NW + w) * S::PR + lane / S::CH;
      const bool valid = m < a.M;
      const int mm = valid ? m : 0;
      const int b = mdiv(mm, a.mg_hw);
      const int rem = mm - b * (a.Ho * a.Wo);
      const int h_ = mdiv(rem, a.mg_wo);
      const int w_ = rem - h_ * a.Wo;
      int bh, bw;
      if constexpr (MODE == MODE_FWD) {
        bh = h_ * a.stride;
        bw = w_ * a.stride;
      } else if constexpr (MODE == MODE_SUBPIX) {
        bh = h_;
        bw = w_;
      } else {  // MODE_DGRAD
        bh = (h_ + a.pad_t) >> a.stride_shift;
        bw = (w_ + a.pad_l) >> a.stride_shift;
      }
      rowbase[i] = (((unsigned)b * (unsigned)a.H + (unsigned)bh) * (unsigned)a.W + (unsigned)bw) * (unsigned)a.Cx * 2u;
      unsigned msk = 0;
      for (int r = 0; r < a.R; ++r)
        for (int s_ = 0; s_ < a.S; ++s_) {
          int ih = 0, iw = 0;
          if (tap_src<MODE>(a, pt, pl, h_, w_, r, s_, ih, iw)) msk |= 1u << (r * a.S + s_);
        }
      vmask[i] = valid ? msk : 0u;
    }
  }
  __device__ void prep(const GemmArgs& a) {
    const int kk = kperm_dma<KT>(a, k) + cb * 8;
    const int tap = mdiv(kk, a.mg_cx);
    const int c = kk - tap * a.Cx;
    const int r = mdiv(tap, a.mg_s);
    const int s_ = tap - r * a.S;
    int dh, dw;
    if constexpr (MODE == MODE_FWD) {
      dh = r - a.pad_t;
      dw = s_ - a.pad_l;
    } else if constexpr (MODE == MODE_SUBPIX) {
      dh = r - pt;
      dw = s_ - pl;
    } else {
      dh = -(r >> a.stride_shift);
      dw = -(s_ >> a.stride_shift);
    }
    delta = ((dh * a.W + dw) * a.Cx + c) * 2;
    tbit = kk < a.K ? 1u << tap : 0u;
  }
  __device__ unsigned src(int i) const { return (vmask[i] & tbit) ? rowbase[i] + (unsigned)delta : OOB; }
  __device__ void issue(const GemmArgs&, __bf16* img, int i, int pl_) {
    dma16(rs[pl_], img + (i * S::NW + w) * 512, src(i));
  }
  __device__ void advance() { k += KT; }
};

// COL images (weight gradient: K = pixels, both operands contiguous along their rows): [KT k-rows][ROWS] bf16, k-row
// pitch ROWS, element (kr, col) at kr * ROWS + (col ^ dcswz(kr)). The 32x32x16 transpose reads (ds_read_b64_tr_b16)
// of a lane group touch 4 consecutive k-rows x 32 columns: the XOR moves the 4 k-rows' 64-B runs into the 4 quarters
// of a 256-B bank row (conflict-free for ROWS >= 128; 2-way at ROWS 64). One DMA instruction fills KPI k-rows; a
// lane's 16-B slot holds the logical chunk slot ^ (dcswz(kr) / 8), the same chunk in every instruction of the lane.
template <int ROWS>
__device__ __forceinline__ int dcswz(int kr) {
  return ROWS >= 128 ? (kr & 3) << 5 : (kr & 1) << 5;
}
template <int ROWS, int NT, int KT>
struct DmaColShape {
  static constexpr int CPR = ROWS / 8;  // 16-B chunks per k-row
  static constexpr int KPI = 64 / CPR;  // k-rows per DMA instruction
  static constexpr int NW = NT / 64;
  static constexpr int NI = ROWS * KT / (NT * 8);  // DMA instructions per thread per stage and plane
  static_assert(ROWS >= 64 && NI >= 1 && NI * NT * 8 == ROWS * KT, "DMA COL image shape");
};

// A = dY^T: element (m, k) at P[k * lda + m]; IS_A false: a k-major B operand, element (n, k) at P[k * ldb + n] (the
// Winograd weight gradient's transformed input V, [tiles][cin])
template <int ROWS, int NT, int KT, bool IS_A = true>
struct DmaColK {
  using S = DmaColShape<ROWS, NT, KT>;
  __amdgpu_buffer_rsrc_t rs[2];
  unsigned colb, ld2;
  bool cv;
  int kr0, k, K, w;
  __device__ void init(const GemmArgs& a, const __bf16* p, int row0, int kb, int tid, int) {
    plane_rsrc(rs, p, IS_A ? a.a_bytes : a.b_bytes, IS_A ? a.a_lo : a.b_lo);
    const int lane = tid & 63;
    w = tid >> 6;
    kr0 = w * S::KPI + lane / S::CPR;
    const int lc = (lane % S::CPR) ^ (dcswz<ROWS>(kr0) >> 3);
    const int col = row0 + lc * 8;
    cv = col < (IS_A ? a.M : a.N);
    colb = (unsigned)col * 2u;
    ld2 = (unsigned)(IS_A ? a.lda : a.ldb) * 2u;
    k = kb; K = a.K;
  }
  __device__ void prep(const GemmArgs&) {}
  __device__ unsigned src(int i) const {
    const int kk = k + kr0 + i * S::NW * S::KPI;
    return (cv & (kk < K)) ? (unsigned)kk * ld2 + colb : OOB;
  }
  __device__ void issue(const GemmArgs&, __bf16* img, int i, int pl) { dma16(rs[pl], img + (i * S::NW + w) * 512, src(i)); }
  __device__ void advance() { k += KT; }
};

// B = im2col of the bf16 NHWC input X: element (n = (r*S+s)*Cx + c, k = output pixel) = X[b][src(oh, ow, r, s)][c]
template <int ROWS, int NT, int MODE, int KT>
struct DmaWgradX {
  using S = DmaColShape<ROWS, NT, KT>;
  __amdgpu_buffer_rsrc_t rs[2];
  int kr0, k, K, w;
  int rr, ss, pt, pl;
  unsigned cb;
  bool nv;
  unsigned off_[S::NI];
  bool ok_[S::NI];
  __device__ void init(const GemmArgs& a, const __bf16* x, int row0, int kb, int tid, int bidx) {
    plane_rsrc(rs, x, a.b_bytes, a.b_lo);
    const int lane = tid & 63;
    w = tid >> 6;
    kr0 = w * S::KPI + lane / S::CPR;
    const int lc = (lane % S::CPR) ^ (dcswz<ROWS>(kr0) >> 3);
    const int n = row0 + lc * 8;
    nv = n < a.N;
    const int nn = nv ? n : 0;
    const int tap = nn / a.Cx;
    cb = (unsigned)(nn - tap * a.Cx) * 2u;
    rr = tap / a.S;
    ss = tap - rr * a.S;
    pt = a.pad_t - ((bidx + a.sub_par) >> 1);
    pl = a.pad_l - ((bidx + a.sub_par) & 1);
    k = kb; K = a.K;
  }
  // the source pixel of instruction i's k-row (computed once per stage, shared by both planes)
  __device__ void prep(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < S::NI; ++i) {
      const int kk = k + kr0 + i * S::NW * S::KPI;
      const int p = min(kk, K - 1);
#ifdef MVAE_WGRAD_XFAKE  // timing-only build: no gather index math (wrong results)
      ok_[i] = nv & (kk < K);
      off_[i] = (unsigned)p * (unsigned)a.Cx * 2u + cb;
      continue;
#endif
      const int b = mdiv(p, a.mg_hw);
      const int rem = p - b * (a.Ho * a.Wo);
      const int oh = mdiv(rem, a.mg_wo);
      const int ow = rem - oh * a.Wo;
      int ih = 0, iw = 0;
      ok_[i] = nv & (kk < K) & tap_src<MODE>(a, pt, pl, oh, ow, rr, ss, ih, iw);
      off_[i] = (((unsigned)b * (unsigned)a.H + (unsigned)ih) * (unsigned)a.W + (unsigned)iw) * (unsigned)a.Cx * 2u + cb;
    }
  }
  __device__ unsigned src(int i) const { return ok_[i] ? off_[i] : OOB; }
  __device__ void issue(const GemmArgs&, __bf16* img, int i, int pl_) { dma16(rs[pl_], img + (i * S::NW + w) * 512, src(i)); }
  __device__ void advance() { k += KT; }
};

// DmaWgradX for B_WGRAD_P2 (stride 1, output = input size, H and W powers of two): a k-row's source is its own pixel
// shifted by the lane's fixed tap offset, valid by a mask-and-shift test of (h, w) -- no divisions per stage
template <int ROWS, int NT, int KT>
struct DmaWgradXP2 {
  using S = DmaColShape<ROWS, NT, KT>;
  __amdgpu_buffer_rsrc_t rs[2];
  int kr0, k, K, w, dr, ds;
  unsigned ldelta, cx2;
  bool nv;
  unsigned off_[S::NI];
  bool ok_[S::NI];
  __device__ void init(const GemmArgs& a, const __bf16* x, int row0, int kb, int tid, int) {
    plane_rsrc(rs, x, a.b_bytes, a.b_lo);
    const int lane = tid & 63;
    w = tid >> 6;
    kr0 = w * S::KPI + lane / S::CPR;
    const int lc = (lane % S::CPR) ^ (dcswz<ROWS>(kr0) >> 3);
    const int n = row0 + lc * 8;
    nv = n < a.N;
    const int nn = nv ? n : 0;
    const int tap = nn / a.Cx, c = nn - tap * a.Cx;
    const int r = tap / a.S, s = tap - r * a.S;
    dr = r - a.pad_t;
    ds = s - a.pad_l;
    ldelta = (unsigned)(((dr * a.W + ds) * a.Cx + c) * 2);
    cx2 = (unsigned)a.Cx * 2u;
    k = kb; K = a.K;
  }
  __device__ void prep(const GemmArgs& a) {
#pragma unroll
    for (int i = 0; i < S::NI; ++i) {
      const int p = k + kr0 + i * S::NW * S::KPI;
      const int ww = p & (a.W - 1), h = (p >> a.lw) & (a.H - 1);
      ok_[i] = nv & (p < K) & ((unsigned)(h + dr) < (unsigned)a.H) & ((unsigned)(ww + ds) < (unsigned)a.W);
      off_[i] = (unsigned)p * cx2 + ldelta;
    }
  }
  __device__ unsigned src(int i) const { return ok_[i] ? off_[i] : OOB; }
  __device__ void issue(const GemmArgs&, __bf16* img, int i, int pl_) { dma16(rs[pl_], img + (i * S::NW + w) * 512, src(i)); }
  __device__ void advance() { k += KT; }
};

// Fragment reads of the DMA main loop as inline asm: the compiler then neither sinks them to just ahead of their
// MFMAs nor waits for the in-flight LDS-DMA before them (it cannot tell a transpose read of stage t from the DMA
// writing stage t+1); the loop places its own counted lgkmcnt waits (LDS reads return in order).
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)(const lds_void_t*)p; }
__device__ __forceinline__ bf16x8 ads_b128(const __bf16* p) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}
__device__ __forceinline__ bf16x4 ads_tr(const __bf16* p) {
  bf16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
  return v;
}
// 16x16x32 fragment (8 consecutive k of one row) of k-step ks from a DMA ROW image
template <int KT>
__device__ __forceinline__ bf16x8 dfrag_asm(const __bf16* img, int row0, int ks, int lane) {
  const int r = row0 + (lane & 15);
  const int c = 4 * ks + (lane >> 4);
  return ads_b128(img + r * KT + ((c ^ dswz<KT>(r)) << 3));
}
// 32x32x16 fragment (k-step ks of 16) from a DMA COL image: two transpose reads, k-rows kr and kr + 4
template <int ROWS>
__device__ __forceinline__ bf16x8 dcfrag_asm(const __bf16* img, int row0, int ks, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int kr = ks * 16 + (g >> 1) * 8 + (li >> 2);
  const int col = row0 + (g & 1) * 16 + 4 * (li & 3);
  const __bf16* p = img + kr * ROWS + (col ^ dcswz<ROWS>(kr));
  const bf16x4 v0 = ads_tr(p), v1 = ads_tr(p + 4 * ROWS);
  return __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N > 15 ? 15 : N));
}

template <int KIND, int ROWS, int NT, bool IS_A, int KT>
struct DmaLoader;
template <int ROWS, int NT, bool IS_A, int KT>
struct DmaLoader<0, ROWS, NT, IS_A, KT> : DmaRowK<ROWS, NT, IS_A, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<A_CONV_FWD, ROWS, NT, true, KT> : DmaConvA<ROWS, NT, MODE_FWD, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<A_CONV_DGRAD, ROWS, NT, true, KT> : DmaConvA<ROWS, NT, MODE_DGRAD, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<A_CONV_SUBPIX, ROWS, NT, true, KT> : DmaConvA<ROWS, NT, MODE_SUBPIX, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<A_COLM, ROWS, NT, true, KT> : DmaColK<ROWS, NT, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<B_COLN, ROWS, NT, false, KT> : DmaColK<ROWS, NT, KT, false> {};
// B operands (IS_A false): weights (ROW) and the weight gradient's im2col gathers (COL)
template <int ROWS, int NT, int KT>
struct DmaLoader<B_WGRAD_FWD, ROWS, NT, false, KT> : DmaWgradX<ROWS, NT, MODE_FWD, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<B_WGRAD_SUBPIX, ROWS, NT, false, KT> : DmaWgradX<ROWS, NT, MODE_SUBPIX, KT> {};
template <int ROWS, int NT, int KT>
struct DmaLoader<B_WGRAD_P2, ROWS, NT, false, KT> : DmaWgradXP2<ROWS, NT, KT> {};

// one MFMA product step: 3xBF16 (lo*hi + hi*lo + hi*hi, small terms first) or plain bf16
__device__ __forceinline__ f32x16 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma_f32(float a, float b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma_f32(float a, float b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
template <int PREC, typename ACC>
__device__ __forceinline__ void mma(ACC& acc, const bf16x8& ah, const bf16x8& al, const bf16x8& bh,
                                    const bf16x8& bl) {
  if constexpr (PREC == 0) {
    // exact fp32: element j of every lane's 8-element fragment is one f32-input MFMA (k-group g of the bf16
    // fragment layout supplies k = 8g + j: the 8 MFMAs cover the fragment's k range once, in the same lanes)
    typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;
    const u16x8 a1 = __builtin_bit_cast(u16x8, ah), a0 = __builtin_bit_cast(u16x8, al);
    const u16x8 b1 = __builtin_bit_cast(u16x8, bh), b0 = __builtin_bit_cast(u16x8, bl);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc = mfma_f32(__uint_as_float(((unsigned)a1[j] << 16) | a0[j]), __uint_as_float(((unsigned)b1[j] << 16) | b0[j]),
                     acc);
    return;
  }
  if constexpr (PREC == 3) {
    acc = mfma_bf16(al, bh, acc);
    acc = mfma_bf16(ah, bl, acc);
  }
  acc = mfma_bf16(ah, bh, acc);
}
// row of accumulator register r (lane's column: lane & (MF-1)) within an MF x MF tile
template <int MF>
__device__ __forceinline__ int acc_row(int r, int lane) {
  if constexpr (MF == 32) return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
  else return 4 * (lane >> 4) + r;
}
// MFMA shape of a kernel: 32x32x16 when A is a transposed (COL) image (wgrad, attention backward)
constexpr int mf_of(int ak) { return (ak == A_COLM || ak == A_COLM_PIX || ak == A_COLM_SPLIT) ? 32 : 16; }

template <int KIND, int ROWS, int VEC, int NT, bool IS_A, int PREC>
struct Loader;
template <int ROWS, int VEC, int NT, bool IS_A, int PREC>
struct Loader<0, ROWS, VEC, NT, IS_A, PREC> : LoadRowK<ROWS, VEC, NT, IS_A, PREC> {};
template <int ROWS, int VEC, int NT, bool IS_A, int PREC>
struct Loader<1, ROWS, VEC, NT, IS_A, PREC> : LoadColK<ROWS, VEC, NT, IS_A, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<2, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_FWD, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<3, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_UPS, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<4, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_DGRAD, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<2, ROWS, VEC, NT, false, PREC> : LoadWgradX<ROWS, VEC, NT, MODE_FWD, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<3, ROWS, VEC, NT, false, PREC> : LoadWgradX<ROWS, VEC, NT, MODE_UPS, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<5, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_SUBPIX, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<6, ROWS, VEC, NT, true, PREC> : LoadColPix<ROWS, VEC, NT, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<4, ROWS, VEC, NT, false, PREC> : LoadWgradX<ROWS, VEC, NT, MODE_SUBPIX, PREC> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<5, ROWS, VEC, NT, false, PREC> : LoadRowK<ROWS, VEC, NT, false, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<7, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_FWD, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<6, ROWS, VEC, NT, false, PREC> : LoadWgradX<ROWS, VEC, NT, MODE_FWD, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<8, ROWS, VEC, NT, true, PREC> : LoadConvA<ROWS, VEC, NT, MODE_DGRAD, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<9, ROWS, VEC, NT, true, PREC> : LoadColK<ROWS, VEC, NT, true, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<A_ROWK_SPLIT, ROWS, VEC, NT, true, PREC> : LoadRowK<ROWS, VEC, NT, true, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<B_COLN_SPLIT, ROWS, VEC, NT, false, PREC> : LoadColK<ROWS, VEC, NT, false, PREC, true> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<B_WGRAD_P2, ROWS, VEC, NT, false, PREC> : LoadWgradXP2<ROWS, NT, PREC, false> {};
template <int ROWS, int VEC, int NT, int PREC>
struct Loader<B_WGRAD_P2_SPLIT, ROWS, VEC, NT, false, PREC> : LoadWgradXP2<ROWS, NT, PREC, true> {};

template <int BM, int BN, int WGM, int WGN, int AK, int VA, int BKIND, int VB, int PREC>
__global__ void __launch_bounds__(64 * WGM * WGN) gemm3x_kernel(GemmArgs a) {
  constexpr int NT = 64 * WGM * WGN;
#ifndef MVAE_COL_MF16  // COL-image (weight-gradient) register-staged loops on 16x16x32 MFMAs (-DMVAE_COL_MF16=0: 32x32x16)
#define MVAE_COL_MF16 1
#endif
  constexpr int MF = (MVAE_COL_MF16 && PREC < 4 && mf_of(AK) == 32) ? 16 : mf_of(AK);
  constexpr int KS = ks_of<MF>(), NR = nr_of<MF>();
  using acc_t = acc_of<MF>;
  constexpr int LP = PREC == 4 ? 1 : PREC == 5 ? 3 : PREC;  // arithmetic of the register-staged loaders
  using LA = Loader<AK, BM, VA, NT, true, LP>;
  using LB = Loader<BKIND, BN, VB, NT, false, LP>;
  using IA = Img<BM, LA::COL>;
  using IB = Img<BN, LB::COL>;
  constexpr int BUF = IA::SIZE + IB::SIZE;
  constexpr int DBUF = (PREC == 5 ? 2 : 1) * (BM + BN) * (PREC == 5 ? 32 : 64);  // PREC 4/5: one DMA stage
  constexpr int TM = BM / WGM / MF, TN = BN / WGN / MF;  // MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) __bf16 lds[(PREC >= 4 && 2 * DBUF > 2 * BUF) ? 2 * DBUF : 2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid - wm * WGN;
  // XCD-aware remap (bijective): blocks b and b+8 share an XCD, so hand each XCD a contiguous run
  // of tiles (row-major over (m, n): neighbours share A rows and the same weight panel).
  // The remap runs over the whole grid (tiles x batch x splits, split-major) since workgroups are
  // dealt to XCDs round-robin by their linear id: the blocks of one split (same K range) share an L2.
  const int ntile = a.tiles_m * a.tiles_n;
  const int nwg = ntile * gridDim.z;
  const int orig = blockIdx.x + ntile * blockIdx.z;
  int lin = orig;
  if (nwg >= 16) {
    const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
    lin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  }
  const int z = lin / ntile;
  const int tile = lin - z * ntile;
  int tm, tn;
  if (a.xcd_groups > 1 && a.tiles_n > 1) {  // grouped order (GemmArgs::xcd_groups), bijective on [0, ntile)
    const int gw = (a.tiles_n + a.xcd_groups - 1) / a.xcd_groups;
    const int ng = (a.tiles_n + gw - 1) / gw;
    const int g = min(tile / (a.tiles_m * gw), ng - 1);
    const int rem = tile - g * a.tiles_m * gw;
    const int width = g == ng - 1 ? a.tiles_n - g * gw : gw;
    tm = rem / width;
    tn = g * gw + (rem - tm * width);
  } else {
    tm = tile / a.tiles_n;
    tn = tile - tm * a.tiles_n;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int bidx = z / a.splits, split = z - bidx * a.splits;
  const int kb = split * a.k_split;
  const int ke = min(a.K, kb + a.k_split);

  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;
  const int arow = wm * (BM / WGM), brow = wn * (BN / WGN);

  if constexpr (PREC >= 4) {
    // LDS-DMA main loop, two stages: at the top of iteration t each wave waits for its own DMA of stage t (vmcnt 0),
    // the barrier makes every wave's DMA of stage t visible and guarantees that every wave has finished reading stage
    // t-1, then the DMA of stage t+1 is issued into that slot and stage t is multiplied: the DMA has one phase to
    // land. Only LDS-DMA loads are in flight in the loop (no VGPR-destination load the compiler would drain with
    // them); fragment reads are inline asm with counted lgkmcnt waits. ROW images (fwd / dgrad) feed 16x16x32 MFMAs,
    // COL images (weight gradient) 32x32x16 MFMAs. PREC 4: bf16 operands, 64-deep stages, the fragments of k-step
    // ks+1 read during k-step ks. PREC 5: planar 3xBF16 operands (hi and lo images), 32-deep stages, per k-step the
    // B fragments then the A fragments streamed one MF-row ahead of their 3 x TN MFMAs.
    // (Measured and removed: a 4-stage ring of 32-deep bf16 stages with fragment reads one stage ahead, 5-10 %
    // slower -- twice the barriers; with no DMA in the loop at all the bf16 loop runs 40-50 % faster, at a higher
    // clock, which no issue order recovers.)
    constexpr int KT = PREC == 5 ? 32 : 64;
    constexpr int NPL = PREC == 5 ? 2 : 1;  // LDS images per operand (hi, lo)
    constexpr bool ACOL = AK == A_COLM,
                   BCOL = BKIND == B_WGRAD_FWD || BKIND == B_WGRAD_SUBPIX || BKIND == B_WGRAD_P2 || BKIND == B_COLN;
    static_assert(ACOL == BCOL && MF == (ACOL ? 32 : 16), "DMA main loop: ROW x ROW (MF 16) or COL x COL (MF 32)");
    using DA = DmaLoader<AK == A_ROWK ? 0 : AK, BM, NT, true, KT>;
    using DB = DmaLoader<BKIND == B_ROWK ? 0 : BKIND, BN, NT, false, KT>;
    constexpr int PA = BM * KT, PB = BN * KT;  // plane sizes (elements)
    constexpr int SBUF = NPL * (PA + PB);      // one stage
    static_assert(2 * SBUF * 2 <= 163840, "DMA stages exceed the LDS");
    DA da;
    DB db;
    da.init(a, (const __bf16*)a.A + bidx * a.sA, m0, kb, tid, bidx);
    db.init(a, (const __bf16*)a.B + bidx * a.sB, n0, kb, tid, bidx);
    const int nt = ke > kb ? (ke - kb + KT - 1) / KT : 0;
    constexpr int NID = NPL * (DA::S::NI + DB::S::NI);  // DMA instructions per thread per stage
    auto issue_q = [&](__bf16* stage, int q) {  // DMA instruction q of the stage (A planes first, then B planes)
      constexpr int QA = NPL * DA::S::NI;
      if (q < QA) da.issue(a, stage + (q / DA::S::NI) * PA, q % DA::S::NI, q / DA::S::NI);
      else db.issue(a, stage + NPL * PA + ((q - QA) / DB::S::NI) * PB, (q - QA) % DB::S::NI, (q - QA) / DB::S::NI);
    };
    auto issue = [&](__bf16* stage) {
      da.prep(a);
      db.prep(a);
#pragma unroll
      for (int q = 0; q < NID; ++q) issue_q(stage, q);
      da.advance();
      db.advance();
    };
    auto frag_a = [&](const __bf16* img, int row0, int ks) {
      if constexpr (ACOL) return dcfrag_asm<BM>(img, row0, ks, lane);
      else return dfrag_asm<KT>(img, row0, ks, lane);
    };
    auto frag_b = [&](const __bf16* img, int row0, int ks) {
      if constexpr (BCOL) return dcfrag_asm<BN>(img, row0, ks, lane);
      else return dfrag_asm<KT>(img, row0, ks, lane);
    };
    constexpr int DKS = KT / (MF == 32 ? 16 : 32);   // MFMA k-steps per stage
    constexpr int RPF = ACOL ? 2 : 1;                // LDS read instructions per fragment
    // (measured, c5 shapes: the spread issue gains 3-6 % on the weight-gradient loops and loses 0-3 % on fwd / dgrad)
    constexpr bool SPREAD = MVAE_DMA_SPREAD == 2 || (MVAE_DMA_SPREAD == 1 && ACOL);
    if (nt > 0) issue(lds);
    for (int t = 0; t < nt; ++t) {
      __bf16* cur = lds + (t & 1) * SBUF;
      __bf16* nxt = lds + ((t + 1) & 1) * SBUF;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const bool more = t + 1 < nt;
      // SPREAD: the stage's DMA instructions are issued in DKS slices, one ahead of each k-step's MFMAs, instead of
      // in one burst after the barrier
      if (SPREAD && more) {
        da.prep(a);
        db.prep(a);
      }
      if (!SPREAD && more) issue(nxt);
      auto dma_slice = [&](int ks) {
        if (SPREAD && more) {
#pragma unroll
          for (int q = ks * NID / DKS; q < (ks + 1) * NID / DKS; ++q) issue_q(nxt, q);
        }
      };
      const __bf16* Ah = cur;
      const __bf16* Bh = cur + NPL * PA;
      if constexpr (PREC == 4) {
        constexpr int RPS = RPF * (TM + TN);  // LDS read instructions per k-step
        bf16x8 fa[2][TM], fb[2][TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[0][j] = frag_b(Bh, brow + j * MF, 0);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[0][i] = frag_a(Ah, arow + i * MF, 0);
#pragma unroll
        for (int ks = 0; ks < DKS; ++ks) {
          const int c = ks & 1;
          if (ks + 1 < DKS) {
#pragma unroll
            for (int j = 0; j < TN; ++j) fb[c ^ 1][j] = frag_b(Bh, brow + j * MF, ks + 1);
#pragma unroll
            for (int i = 0; i < TM; ++i) fa[c ^ 1][i] = frag_a(Ah, arow + i * MF, ks + 1);
          }
          if (ks + 1 < DKS) wait_lgkm<RPS>();  // k-step ks's reads are done; ks+1's stay in flight
          else wait_lgkm<0>();
          __builtin_amdgcn_sched_barrier(0);
          dma_slice(ks);
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma_bf16(fa[c][i], fb[c][j], acc[i][j]);
          __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        const __bf16* Al = Ah + PA;
        const __bf16* Bl = Bh + PB;
        constexpr int RA = 2 * RPF;  // reads per A fragment pair (hi, lo)
#pragma unroll
        for (int ks = 0; ks < DKS; ++ks) {
          bf16x8 bh[TN], bl[TN], ah[2], al[2];
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            bh[j] = frag_b(Bh, brow + j * MF, ks);
            bl[j] = frag_b(Bl, brow + j * MF, ks);
          }
          ah[0] = frag_a(Ah, arow, ks);
          al[0] = frag_a(Al, arow, ks);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            if (i + 1 < TM) {
              ah[(i + 1) & 1] = frag_a(Ah, arow + (i + 1) * MF, ks);
              al[(i + 1) & 1] = frag_a(Al, arow + (i + 1) * MF, ks);
              wait_lgkm<RA>();  // everything but the pair just issued
            } else {
              wait_lgkm<0>();
            }
            __builtin_amdgcn_sched_barrier(0);
            if (i == 0) dma_slice(ks);
#pragma unroll
            for (int j = 0; j < TN; ++j) mma<3>(acc[i][j], ah[i & 1], al[i & 1], bh[j], bl[j]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      if (SPREAD && more) {
        da.advance();
        db.advance();
      }
    }
  } else {
  LA la;
  LB lb;
  // wgrad: only the first column of tiles publishes the bias gradient (row sums of dY^T): the others skip the sums
  if constexpr (AK == A_COLM || AK == A_COLM_PIX || AK == A_COLM_SPLIT) la.want_bs = a.bias_ws != nullptr && tn == 0;
  la.init(a, a.A + bidx * a.sA, m0, kb, tid, bidx);
  lb.init(a, a.B + bidx * a.sB, n0, kb, tid, bidx);

  const int nt = ke > kb ? (ke - kb + BK - 1) / BK : 0;
  // (Measured and removed: in bf16 mode, two K-tiles per stage in the free lo planes -- twice the MFMAs per barrier
  // and twice the load-latency budget -- ran the c5 fwd / dgrad GEMMs 3 % slower: the single-tile bf16 loop is not
  // bound by the barrier count or the global-load latency.)
  {
  // Prologue: tile 0 -> LDS buffer 0, tile 1 -> registers.
  if (nt > 0) {
    la.load(a);
    lb.load(a);
    la.store(lds);
    lb.store(lds + IA::SIZE);
  }
  if (nt > 1) {
    la.advance();
    lb.advance();
    la.load(a);
    lb.load(a);
  }
  __syncthreads();
  // Steady state ("write after barrier"): at iteration t the registers hold tile t+1 (loaded one
  // full compute phase earlier). Right after the barrier each wave splits/writes them into the
  // free buffer, immediately re-issues the global loads of tile t+2 into the same registers, and
  // multiplies tile t -- whose buffer was completed before the barrier -- so the LDS writes and the
  // VALU split overlap the wave's own MFMAs and the global loads have a whole phase to land.
  auto compute = [&](const __bf16* Ai) {
    const __bf16* Bi = Ai + IA::SIZE;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = read_frag<BN, LB::COL, MF>(Bi, brow + j * MF, ks, lane);
        if constexpr (PREC != 1) bl[j] = read_frag<BN, LB::COL, MF>(Bi + IB::PLANE, brow + j * MF, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 ah = read_frag<BM, LA::COL, MF>(Ai, arow + i * MF, ks, lane);
        bf16x8 al{};
        if constexpr (PREC != 1) al = read_frag<BM, LA::COL, MF>(Ai + IA::PLANE, arow + i * MF, ks, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          mma<PREC>(acc[i][j], ah, al, bh[j], bl[j]);
        }
      }
    }
  };
  int t = 0;
  {
#ifndef MVAE_BLOCK_STAGING
  // steady state, software-pipelined by hand: the K-tile's KS*TM MFMA steps (one MF-row A fragment
  // x TN B fragments x 3 split products each) each carry a share of the staging work -- split +
  // LDS write of one slot of tile t+1, then the global load of the same slot of tile t+2 -- and
  // prefetch the next step's A fragment. sched_barrier pins that order (the scheduler would
  // otherwise hoist all staging VALU into one block ahead of the MFMAs, idling the MFMA pipe).
  constexpr int STEPS = KS * TM;
  constexpr int NSL = LA::NS + LB::NS;
  // STAG: the wave runs each step's staging share BEFORE its MFMAs instead of after. Given to the
  // second half of the workgroup (waves 4-7 share SIMDs with waves 0-3), it staggers the two waves of
  // every SIMD: one issues VALU/LDS staging while its partner's MFMAs occupy the matrix pipe.
  auto kloop = [&](auto stag) {
    constexpr bool STAG = decltype(stag)::value;
    for (; t + 2 < nt; ++t) {
      __bf16* nb = lds + ((t & 1) ^ 1) * BUF;
      const __bf16* Ai = lds + (t & 1) * BUF;
      const __bf16* Bi = Ai + IA::SIZE;
      la.advance();
      lb.advance();
      la.prep(a);
      lb.prep(a);
      bf16x8 bh[TN], bl[TN], ah[2], al[2];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = read_frag<BN, LB::COL, MF>(Bi, brow + j * MF, 0, lane);
        if constexpr (PREC != 1) bl[j] = read_frag<BN, LB::COL, MF>(Bi + IB::PLANE, brow + j * MF, 0, lane);
      }
      ah[0] = read_frag<BM, LA::COL, MF>(Ai, arow, 0, lane);
      if constexpr (PREC != 1) al[0] = read_frag<BM, LA::COL, MF>(Ai + IA::PLANE, arow, 0, lane);
      auto stage = [&](int st) {
#pragma unroll
        for (int q = st * NSL / STEPS; q < (st + 1) * NSL / STEPS; ++q) {
          if (q < LA::NS) {
            la.store_slot(nb, q);
            la.load_slot(a, q);
          } else {
            lb.store_slot(nb + IA::SIZE, q - LA::NS);
            lb.load_slot(a, q - LA::NS);
          }
        }
      };
#pragma unroll
      for (int st = 0; st < STEPS; ++st) {
        const int i = st % TM, cur = st & 1;
        if constexpr (STAG) {
          stage(st);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (st + 1 < STEPS) {
          const int ks1 = (st + 1) / TM, i1 = (st + 1) % TM;
          ah[cur ^ 1] = read_frag<BM, LA::COL, MF>(Ai, arow + i1 * MF, ks1, lane);
          if constexpr (PREC != 1) al[cur ^ 1] = read_frag<BM, LA::COL, MF>(Ai + IA::PLANE, arow + i1 * MF, ks1, lane);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          mma<PREC>(acc[i][j], ah[cur], al[cur], bh[j], bl[j]);
        }
        if (KS == 2 && st == TM - 1) {  // B fragments of the second k-half
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            bh[j] = read_frag<BN, LB::COL, MF>(Bi, brow + j * MF, 1, lane);
            if constexpr (PREC != 1) bl[j] = read_frag<BN, LB::COL, MF>(Bi + IB::PLANE, brow + j * MF, 1, lane);
          }
        }
        if constexpr (!STAG) stage(st);
        __builtin_amdgcn_sched_barrier(0);
      }
      __syncthreads();
    }
  };
#ifndef MVAE_NO_PRIO
  // the second-dispatched half of the workgroup loses every VALU arbitration to its SIMD partner: one static
  // priority raise for it (no per-segment flips): wgrad +1-3 %, fwd / dgrad within noise (tools/ab.sh)
  if (NT >= 512 && wid >= (NT / 64) / 2) __builtin_amdgcn_s_setprio(1);
#endif
#ifdef MVAE_STAG
  if (NT >= 512 && wid >= (NT / 64) / 2)
    kloop(std::true_type{});
  else
    kloop(std::false_type{});
#else
    kloop(std::false_type{});
#endif
#ifndef MVAE_NO_PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
#else
  for (; t + 2 < nt; ++t) {  // block staging: all of tile t+1's staging, then tile t's MFMAs
    __bf16* nb = lds + ((t & 1) ^ 1) * BUF;
    la.store(nb);
    lb.store(nb + IA::SIZE);
    la.advance();
    lb.advance();
    la.load(a);
    lb.load(a);
    compute(lds + (t & 1) * BUF);
    __syncthreads();
  }
#endif
  }
  if (t + 1 < nt) {  // last staged tile: write it, nothing left to load
    __bf16* nb = lds + ((t & 1) ^ 1) * BUF;
    la.store(nb);
    lb.store(nb + IA::SIZE);
    compute(lds + (t & 1) * BUF);
    __syncthreads();
    ++t;
  }
  if (t < nt) compute(lds + (t & 1) * BUF);
  }

  // wgrad: the conv bias gradient (row sums of A = dY^T over this split's pixels) falls out of the
  // A staging for free; one column of tiles (tn == 0) publishes it, fixed-order reduction in LDS.
  if constexpr (AK == A_COLM || AK == A_COLM_PIX || AK == A_COLM_SPLIT) {
    if (a.bias_ws != nullptr && tn == 0) {
      constexpr int KRN = NT / (BM / 4);
      float* red = (float*)lds;
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 4; ++e) red[la.kr * BM + la.c4 * 4 + e] = la.bs[e];
      __syncthreads();
      if (la.kr == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sum = 0.f;
          for (int q = 0; q < KRN; ++q) sum += red[q * BM + la.c4 * 4 + e];
          const int row = m0 + la.c4 * 4 + e;
          if (row < a.M) a.bias_ws[((long long)bidx * a.splits + split) * a.M + row] = sum;
        }
      }
    }
  }
  }  // register-staged main loop

  // 16-B epilogue (16x16x32 kernels, one split, plain row order, N / ldc / ldr multiples of 4): each wave
  // stages half of its accumulator block at a time in LDS (free after the main loop) as fp32 rows and
  // re-reads them as float4 runs of the row, so bias / residual / beta*C / the store move whole 16-B
  // groups along C's contiguous channel dimension instead of 4-B scalars in 64-B pieces.
  if constexpr (MF == 16 && TM % 2 == 0) {
    if (a.vec_epi) {
      constexpr int WR = BM / WGM, WC = BN / WGN, HR = WR / 2, PE = WC + 4;
      static_assert((NT / 64) * HR * PE * 4 <= 4 * BUF, "epilogue staging exceeds the LDS");
      constexpr int C4 = WC / 4, RPI = 64 / C4;  // float4 per staged row, rows per wave instruction
      float* stg = (float*)lds + wid * HR * PE;
      const __amdgpu_buffer_rsrc_t cr = make_rsrc(a.C + bidx * a.sC, a.c_bytes);
      const bool has_res = a.res != nullptr;
      const __amdgpu_buffer_rsrc_t rr = make_rsrc(has_res ? a.res + bidx * a.sR : a.C, has_res ? a.r_bytes : 0u);
      const int c4 = lane % C4, rsub = lane / C4;
      const int col = n0 + brow + c4 * 4;
      float4 bv{0.f, 0.f, 0.f, 0.f};
      if (a.bias != nullptr && col < a.N) bv = *(const float4*)(a.bias + col);
      constexpr int NSB = WR / 32;  // 32-row blocks of the wave's rows (GroupNorm statistics)
      double st0[NSB], st1[NSB];
#pragma unroll
      for (int q = 0; q < NSB; ++q) st0[q] = st1[q] = 0.0;
      const bool want_stats = a.gn_part != nullptr;
      // GroupNorm backward partials (GemmArgs::gnb_part): per-channel, per 32-row block; a pass holds whole
      // blocks when HR >= 32 (flushed per pass), else one block spans both passes (flushed at the end)
      const bool want_gnb = a.gnb_part != nullptr;
      constexpr int QP = HR >= 32 ? HR / 32 : 1;
      double gs0[QP][4], gs1[QP][4];
      float ggm[4] = {0.f, 0.f, 0.f, 0.f}, gbt[4] = {0.f, 0.f, 0.f, 0.f};
      const __amdgpu_buffer_rsrc_t xr = make_rsrc(want_gnb ? a.gnb_x + bidx * a.sC : a.C, want_gnb ? a.c_bytes : 0u);
      if (want_gnb && col < a.N) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ggm[e] = a.gnb_gamma[col + e];
          gbt[e] = a.gnb_beta[col + e];
        }
      }
      auto gnb_reset = [&]() {
#pragma unroll
        for (int q = 0; q < QP; ++q)
#pragma unroll
          for (int e = 0; e < 4; ++e) gs0[q][e] = gs1[q][e] = 0.0;
      };
      auto gnb_flush = [&](int q, int row0) {  // fixed xor-tree over the RPI row lanes of one column group
        double s0[4], s1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[e] = gs0[q][e];
          s1[e] = gs1[q][e];
#pragma unroll
          for (int o = C4; o < 64; o <<= 1) {
            s0[e] += __shfl_xor(s0[e], o, 64);
            s1[e] += __shfl_xor(s1[e], o, 64);
          }
        }
        if (rsub == 0 && row0 < a.M && col < a.N) {
          double* gp = a.gnb_part + ((long long)(row0 >> 5) * a.N + col) * 2;
#pragma unroll
          for (int e = 0; e < 4; ++e) *(double2*)(gp + 2 * e) = double2{s0[e], s1[e]};
        }
      };
      gnb_reset();
      __syncthreads();  // every wave's last fragment reads are done: the LDS is free
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int i = 0; i < TM / 2; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < NR; ++r)
              stg[(i * 16 + acc_row<MF>(r, lane)) * PE + j * 16 + (lane & 15)] = acc[pass * (TM / 2) + i][j][r];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < HR / RPI; ++k) {
          const int lr = k * RPI + rsub;
          const float4 s4 = *(const float4*)(stg + lr * PE + c4 * 4);
          const int row = m0 + arow + pass * HR + lr;
          const bool ok = row < a.M && col < a.N;
          const unsigned co = ok ? ((unsigned)row * (unsigned)a.ldc + col) * 4u : OOB;
          float4 v{a.alpha * s4.x + bv.x, a.alpha * s4.y + bv.y, a.alpha * s4.z + bv.z, a.alpha * s4.w + bv.w};
          if (has_res) {
            const float4 r4 = bload4(rr, ok ? ((unsigned)row * (unsigned)a.ldr + col) * 4u : OOB);
            v.x += r4.x; v.y += r4.y; v.z += r4.z; v.w += r4.w;
          }
          if (a.beta != 0.f) {
            const float4 c4v = bload4(cr, co);
            v.x += a.beta * c4v.x; v.y += a.beta * c4v.y; v.z += a.beta * c4v.z; v.w += a.beta * c4v.w;
          }
          bstore4(cr, co, v);
          if (want_stats && ok) {
            const int q = (pass * HR + k * RPI) / 32;  // compile-time: RPI divides 32
            st0[q] += ((double)v.x + (double)v.y) + ((double)v.z + (double)v.w);
            st1[q] += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
          }
          if (want_gnb && ok) {  // same float arithmetic as gn_partial_kernel<1>
            const int q = HR >= 32 ? (k * RPI) / 32 : 0;
            const float4 x4 = bload4(xr, co);
            const int bg = (row / a.gnb_hw) * a.gnb_G + col / a.gnb_cpg;
            const float mu = a.gnb_mean[bg], rs = a.gnb_rstd[bg];
            const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
            const float vs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float d = vs[e];
              const float xh = (xs[e] - mu) * rs;
              if (a.gnb_silu) {
                const float yn = xh * ggm[e] + gbt[e];
                const float sg = sigmoid_f(yn);
                d = d * sg * (1.f + yn * (1.f - sg));
              }
              gs0[q][e] += d;
              gs1[q][e] += (double)d * xh;
            }
          }
        }
        if (want_gnb && (HR >= 32 || pass == 1)) {
#pragma unroll
          for (int q = 0; q < QP; ++q) gnb_flush(q, m0 + arow + (HR >= 32 ? pass * HR + q * 32 : 0));
          gnb_reset();
        }
        __syncthreads();
      }
      if (want_stats) {  // fixed xor-tree over the lanes of one column group (the RPI row lanes)
#pragma unroll
        for (int q = 0; q < NSB; ++q) {
          double s0 = st0[q], s1 = st1[q];
#pragma unroll
          for (int o = C4; o < 64; o <<= 1) {
            s0 += __shfl_xor(s0, o, 64);
            s1 += __shfl_xor(s1, o, 64);
          }
          const int row0 = m0 + arow + q * 32;
          if (rsub == 0 && row0 < a.M && col < a.N) {
            double* gp = a.gn_part + ((long long)(row0 >> 5) * (a.N >> 2) + (col >> 2)) * 2;
            gp[0] = s0;
            gp[1] = s1;
          }
        }
      }
      return;
    }
  }

  // epilogue: C/D layout of the MFMA tile: col = lane & (MF-1), row = acc_row<MF>(r, lane).
  // Stores go through buffer descriptors: rows/cols outside the matrix are dropped by the hardware.
  if (a.splits > 1) {
    const __amdgpu_buffer_rsrc_t ws =
        make_rsrc(a.ws + ((long long)bidx * a.splits + split) * a.M * a.N, (unsigned)(a.M * a.N * 4u));
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + brow + j * MF + (lane & (MF - 1));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int row = m0 + arow + i * MF + acc_row<MF>(r, lane);
          const bool ok = row < a.M && col < a.N;
          bstore1(ws, ok ? ((unsigned)row * a.N + col) * 4u : OOB, acc[i][j][r]);
        }
    }
    return;
  }
  const __amdgpu_buffer_rsrc_t cr = make_rsrc(a.C + bidx * a.sC, a.c_bytes);
  const bool has_res = a.res != nullptr;
  const __amdgpu_buffer_rsrc_t rr = make_rsrc(has_res ? a.res + bidx * a.sR : a.C, has_res ? a.r_bytes : 0u);
  const __amdgpu_buffer_rsrc_t br = make_rsrc(a.bias ? a.bias : a.C, a.bias ? (unsigned)(a.N * 4) : 0u);
  const bool remap = a.out_remap != 0;
  const int par_off = sub_par_off(a, bidx);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + brow + j * MF + (lane & (MF - 1));
    const float bv = bload1(br, col < a.N ? (unsigned)col * 4u : OOB);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        const int row = m0 + arow + i * MF + acc_row<MF>(r, lane);
        const bool ok = row < a.M && col < a.N;
        const int orow = remap ? sub_pixel(a, ok ? row : 0, par_off) : row;
        float v = a.alpha * acc[i][j][r] + bv;
        if (has_res) v += bload1(rr, ok ? ((unsigned)orow * (unsigned)a.ldr + col) * 4u : OOB);
        const unsigned co = ok ? ((unsigned)orow * (unsigned)a.ldc + col) * 4u : OOB;
        if (a.beta != 0.f) v += a.beta * bload1(cr, co);
        bstore1(cr, co, v);
      }
    }
  }
}

// Fixed-order reduction of split-K partials + the same epilogue.
__global__ void splitk_reduce_kernel(GemmArgs a);
// Split-K reduction, 4 columns per thread (N, ldc, ldr multiples of 4; 16-B aligned C / residual / bias): column
// group bx * 256 + thread, output rows y0, y0 + ystep, ...; the split partials are loaded 4 at a time and summed in
// split order (deterministic). Body of splitk_reduce4_kernel and of the weight-gradient finish kernel.
__device__ __forceinline__ void splitk_reduce4_rows(const GemmArgs& a, int bx, int y0, int ystep) {
  const int c4 = bx * 256 + threadIdx.x;
  if (c4 >= (a.N >> 2)) return;
  const int col = c4 * 4;
  const long long mn = (long long)a.M * a.N;
  const float4 zero{0.f, 0.f, 0.f, 0.f};
  const float4 bv = a.bias ? *(const float4*)(a.bias + col) : zero;
  for (int rb = y0; rb < a.M * a.batch; rb += ystep) {
    const int bidx = rb / a.M, row = rb - bidx * a.M;
    const float* w = a.ws + (long long)bidx * a.splits * mn + (long long)row * a.N + col;
    float4 s = zero;
    int z = 0;
    // 16 partial loads in flight per thread (the split loop is a latency chain, not a bandwidth one: a few thousand
    // threads each walk up to 256 splits), summed strictly in split order (the result does not depend on the depth)
    for (; z + 16 <= a.splits; z += 16) {
      float4 wv[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) wv[j] = *(const float4*)(w + (z + j) * mn);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        s.x += wv[j].x; s.y += wv[j].y; s.z += wv[j].z; s.w += wv[j].w;
      }
    }
    for (; z + 4 <= a.splits; z += 4) {
      const float4 w0 = *(const float4*)(w + z * mn), w1 = *(const float4*)(w + (z + 1) * mn);
      const float4 w2 = *(const float4*)(w + (z + 2) * mn), w3 = *(const float4*)(w + (z + 3) * mn);
      s.x = (((s.x + w0.x) + w1.x) + w2.x) + w3.x;
      s.y = (((s.y + w0.y) + w1.y) + w2.y) + w3.y;
      s.z = (((s.z + w0.z) + w1.z) + w2.z) + w3.z;
      s.w = (((s.w + w0.w) + w1.w) + w2.w) + w3.w;
    }
    for (; z < a.splits; ++z) {
      const float4 w0 = *(const float4*)(w + z * mn);
      s.x += w0.x; s.y += w0.y; s.z += w0.z; s.w += w0.w;
    }
    float4 v{a.alpha * s.x + bv.x, a.alpha * s.y + bv.y, a.alpha * s.z + bv.z, a.alpha * s.w + bv.w};
    if (a.res) {
      const float4 r = *(const float4*)(a.res + bidx * a.sR + (long long)row * a.ldr + col);
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    float* cp = a.C + bidx * a.sC + (long long)row * a.ldc + col;
    if (a.beta != 0.f) {
      const float4 c = *(const float4*)cp;
      v.x += a.beta * c.x; v.y += a.beta * c.y; v.z += a.beta * c.z; v.w += a.beta * c.w;
    }
    *(float4*)cp = v;
  }
}


// ------------------------------------------------------------------------------------------
// host-side dispatch
// ------------------------------------------------------------------------------------------
enum { T256x256 = 0, T256x128 = 1, T128x256 = 2, T128x128 = 3, T64x64 = 4, T128x16 = 5, T128x32 = 6 };

// process-wide GEMM arithmetic (mvae_set_math_mode): 3xBF16 fp32 emulation (default), bf16, or exact fp32
// on the f32-input MFMA (v_mfma_f32_{16x16x4,32x32x2}_f32: 1/16 of the bf16 rate)
enum { MATH_3XBF16 = 0, MATH_BF16 = 1, MATH_FP32 = 2 };
int math_mode();

// workgroups of a tile config resident per CU at once (LDS-bound: 160, 120, 120, 80, 40 KB per workgroup; the skinny
// tiles 4 / 3): a "round" of a launch is 256 CUs x this many tiles
inline int resident_of(int cfg) {
  static const int r[7] = {1, 1, 1, 2, 4, 4, 3};
  return (cfg >= 0 && cfg < 7) ? r[cfg] : 1;
}
// tile edge lengths of a config (rows of M, columns of N)
inline int tile_m_of(int cfg) {
  static const int m[7] = {256, 256, 128, 128, 64, 128, 128};
  return (cfg >= 0 && cfg < 7) ? m[cfg] : 64;
}
inline int tile_n_of(int cfg) {
  static const int n[7] = {256, 128, 256, 128, 64, 16, 32};
  return (cfg >= 0 && cfg < 7) ? n[cfg] : 64;
}

inline long long tiles_of(int cfg, const GemmArgs& a) {
  static const int TM_[] = {256, 256, 128, 128, 64, 128, 128};
  static const int TN_[] = {256, 128, 256, 128, 64, 16, 32};
  return (long long)cdiv(a.M, TM_[cfg]) * cdiv(a.N, TN_[cfg]) * a.batch;
}

// largest useful split-K factor (>= 16 K-tiles per split)
inline int max_splits_of(const GemmArgs& a, bool can_split) {
  if (!can_split) return 1;
  int s = 1;
  while (s < 64 && (long long)a.K / (s * 2) >= 512) s *= 2;
  return s;
}

// pick the largest tile that still gives >= 1 full wave of the 256 CUs, counting the blocks that
// split-K adds when a workspace is available (wgrad: small M x N, huge K)
inline int tile_override() {
  static int v = [] {
    const char* e = getenv("MVAE_GEMM_TILE");  // experiment knob: force a tile config (0..4)
    return e ? atoi(e) : -1;
  }();
  return v;
}

inline bool tile_rule_legacy() {  // experiment knob: MVAE_TILE_LEGACY=1 restores the >= 240-tiles rule
  static int v = getenv("MVAE_TILE_LEGACY") != nullptr;
  return v != 0;
}

inline int choose_tile(const GemmArgs& a, bool allow_big, bool can_split) {
  const int ov = tile_override();
  if (ov >= 0 && ov <= 4 && (allow_big || ov >= T128x128)) return ov;
  const long long ms = max_splits_of(a, can_split);
  // skinny N (Decoder.conv_out forward, cout 3; Encoder.conv_in input gradient, cin 6): 128x16 tiles on
  // 2 waves instead of 64-wide tiles that are 95 % padding
  if (allow_big && a.N <= 16 && tiles_of(T128x16, a) >= 512) return T128x16;
  // 32-wide N (the 28x28 level of the c3 model at 32 channels, fwd and input gradient): 128x32 tiles on 4 waves
  // (32x32 per wave) instead of 64x64 tiles whose second half of N is padding. Opt-in (MVAE_T128X32=1): measured on c3
  // (same box) the forward launches ran 17 % slower (2.24 -> 2.62 ms per step), the input gradient unchanged.
  static const bool t128x32 = getenv("MVAE_T128X32") != nullptr;
  if (t128x32 && allow_big && !can_split && a.N > 16 && a.N <= 32 && tiles_of(T128x32, a) >= 512 && !tile_rule_legacy())
    return T128x32;
  if (allow_big && !can_split && !tile_rule_legacy()) {
    // Cost model over the tile configs (fwd / dgrad / batched GEMMs; split-K GEMMs keep the rule below):
    // time ~ rounds x (tiles resident per CU) x tile area / per-tile efficiency, with rounds =
    // ceil(tiles / (256 CUs x tiles resident per CU)). Efficiencies are the measured full-chip rates of each
    // tile relative to 256x256 (tools/tile_sweep.py, c4 shapes: 256x256 1.0, 256x128 / 128x256 0.82,
    // 128x128 0.70, 64x64 0.50); residency from LDS (160, 120, 120, 80, 40 KB per workgroup). The rule it
    // replaces (largest tile with >= 240 tiles) lost 18-65 % on the c2 / c3 layers (7x7 and 14x14 at 256-512
    // channels; 32-64 channels at 14x14-28x28).
    static const double eff[5] = {1.0, 0.82, 0.82, 0.70, 0.50};
    static const int res[5] = {1, 1, 1, 2, 4};
    static const int area[5] = {65536, 32768, 32768, 16384, 4096};
    int best = T64x64;
    double best_t = 1e300;
    for (int c = T256x256; c <= T64x64; ++c) {
      const long long t = tiles_of(c, a);
      const double rounds = (double)((t + 256LL * res[c] - 1) / (256LL * res[c]));
      const double cost = rounds * res[c] * area[c] / eff[c];
      if (cost < best_t * 0.999) { best_t = cost; best = c; }
    }
    return best;
  }
  if (allow_big) {
    if (tiles_of(T256x256, a) * ms >= 240 && a.M > 128 && a.N > 128) return T256x256;
    if (a.N <= 128 && tiles_of(T256x128, a) * ms >= 240 && a.M > 128) return T256x128;
    if (a.M <= 128 && tiles_of(T128x256, a) * ms >= 240 && a.N > 128) return T128x256;
  }
  if (tiles_of(T128x128, a) * ms >= 200 && a.M > 64 && a.N > 64) return T128x128;
  return T64x64;
}

inline bool al16(const void* p);
inline int xcd_groups_env() {  // experiment knob: MVAE_XCD_GROUPS=G orders the tiles in G column groups
  static int v = [] {
    const char* e = getenv("MVAE_XCD_GROUPS");
    return e ? std::max(1, atoi(e)) : 1;
  }();
  return v;
}
// pre-split (3xBF16 value-split) operands cannot feed the exact-fp32 GEMM
inline bool split_forbidden() { return math_mode() == MATH_FP32; }
inline bool vec_epi_disabled() {
  static int v = getenv("MVAE_NO_VEC_EPI") != nullptr;  // experiment knob: scalar epilogue everywhere
  return v != 0;
}

// PO >= 0 forces the kernel arithmetic (PREC 4: bf16-stored operands through the LDS-DMA main loop)
template <int CFG, int AK, int VA, int BKIND, int VB, int PO = -1>
void launch_cfg(GemmArgs& a, hipStream_t st) {
  constexpr int BM = CFG == T256x256 || CFG == T256x128 ? 256 : CFG == T64x64 ? 64 : 128;
  constexpr int BN = CFG == T256x256 || CFG == T128x256 ? 256 : CFG == T64x64 ? 64 : CFG == T128x16 ? 16
                   : CFG == T128x32 ? 32 : 128;
  constexpr int WGM = CFG == T256x128 || CFG == T128x32 ? 4 : 2;
#ifdef MVAE_W4
  constexpr int WGN = CFG == T128x256 ? 4 : (CFG == T128x16 || CFG == T128x32) ? 1 : 2;  // 256x256 on 4 waves
#else
  constexpr int WGN = (CFG == T256x256 || CFG == T128x256) ? 4 : (CFG == T128x16 || CFG == T128x32) ? 1 : 2;
#endif
  a.tiles_m = cdiv(a.M, BM);
  a.tiles_n = cdiv(a.N, BN);
  if (a.xcd_groups <= 0) a.xcd_groups = xcd_groups_env();
  a.vec_epi = a.splits == 1 && !a.out_remap && (a.N & 3) == 0 && (a.ldc & 3) == 0 && (a.sC & 3) == 0 && al16(a.C) &&
              (!a.res || ((a.ldr & 3) == 0 && (a.sR & 3) == 0 && al16(a.res))) && (!a.bias || al16(a.bias)) &&
              !vec_epi_disabled();
  dim3 grid(a.tiles_m * a.tiles_n, 1, a.batch * a.splits);
  constexpr bool presplit = AK == A_CONV_FWD_SPLIT || AK == A_CONV_DGRAD_SPLIT || AK == A_COLM_SPLIT || AK == A_ROWK_SPLIT ||
                            BKIND == B_ROWK_SPLIT || BKIND == B_WGRAD_FWD_SPLIT || BKIND == B_WGRAD_P2_SPLIT ||
                            BKIND == B_COLN_SPLIT;
  // the Winograd position / weight-gradient GEMMs: their pre-split operands come in the arithmetic's own layout (a bit
  // split in the exact mode, csrc/winograd.hip); every other pre-split operand is a 3xBF16 value split, never launched
  // in the exact mode
  constexpr bool wino = (AK == A_ROWK_SPLIT && BKIND == B_ROWK_SPLIT) || (AK == A_COLM_SPLIT && BKIND == B_COLN_SPLIT);
  const int mm = math_mode();
  if constexpr (PO >= 0)
    hipLaunchKernelGGL((gemm3x_kernel<BM, BN, WGM, WGN, AK, VA, BKIND, VB, PO>), grid, dim3(64 * WGM * WGN), 0, st, a);
  else if (mm == MATH_BF16)
    hipLaunchKernelGGL((gemm3x_kernel<BM, BN, WGM, WGN, AK, VA, BKIND, VB, 1>), grid, dim3(64 * WGM * WGN), 0, st, a);
  else if (mm == MATH_FP32 && (!presplit || wino))
    hipLaunchKernelGGL((gemm3x_kernel<BM, BN, WGM, WGN, AK, VA, BKIND, VB, 0>), grid, dim3(64 * WGM * WGN), 0, st, a);
  else
    hipLaunchKernelGGL((gemm3x_kernel<BM, BN, WGM, WGN, AK, VA, BKIND, VB, 3>), grid, dim3(64 * WGM * WGN), 0, st, a);
}

template <int AK, int VA, int BKIND, int VB>
void launch_big(GemmArgs& a, hipStream_t st, int cfg) {
  switch (cfg) {
    case T256x256: launch_cfg<T256x256, AK, VA, BKIND, VB>(a, st); break;
    case T256x128: launch_cfg<T256x128, AK, VA, BKIND, VB>(a, st); break;
    case T128x256: launch_cfg<T128x256, AK, VA, BKIND, VB>(a, st); break;
    case T128x128: launch_cfg<T128x128, AK, VA, BKIND, VB>(a, st); break;
    case T128x16:  // 16-wide tiles need the 16x16x32 MFMA shape
      if constexpr (mf_of(AK) == 16) launch_cfg<T128x16, AK, VA, BKIND, VB>(a, st);
      else launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st);
      break;
    case T128x32:  // (the same)
      if constexpr (mf_of(AK) == 16 && VA == 4 && VB == 4) launch_cfg<T128x32, AK, VA, BKIND, VB>(a, st);
      else launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st);
      break;
    default: launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st); break;
  }
}

// DMA-staged operands (MVAE_CONV_BF16: PREC 4, MVAE_CONV_PLANAR: PREC 5): every tile config on the LDS-DMA main loop
template <int AK, int P>
void launch_dma(GemmArgs& a, hipStream_t st, int cfg) {
  switch (cfg) {
    case T256x256: launch_cfg<T256x256, AK, 4, B_ROWK, 4, P>(a, st); break;
    case T256x128: launch_cfg<T256x128, AK, 4, B_ROWK, 4, P>(a, st); break;
    case T128x256: launch_cfg<T128x256, AK, 4, B_ROWK, 4, P>(a, st); break;
    case T128x128: launch_cfg<T128x128, AK, 4, B_ROWK, 4, P>(a, st); break;
    default: launch_cfg<T64x64, AK, 4, B_ROWK, 4, P>(a, st); break;  // (and the skinny-N 128x16 choice)
  }
}

// gemm_dma.hip: launch_dma for AK in {A_ROWK, A_CONV_FWD, A_CONV_DGRAD, A_CONV_SUBPIX} (own translation unit)
// prec 4: packed bf16 operands; prec 5: planar 3xBF16 operands (hi plane, lo plane a_lo / b_lo bytes later)
void conv_dma(int ak, GemmArgs& a, hipStream_t st, int cfg, int prec);
// weight gradient on DMA-staged dY^T (COL) x im2col of X (B_WGRAD_FWD / B_WGRAD_SUBPIX / B_WGRAD_P2), or x a k-major
// packed operand (B_COLN: the Winograd weight gradient's V)
void wgrad_dma(int bkind, GemmArgs& a, hipStream_t st, int cfg, int prec);

template <int AK, int VA, int BKIND, int VB>
void launch_small(GemmArgs& a, hipStream_t st, int cfg) {
  if (cfg == T128x128) launch_cfg<T128x128, AK, VA, BKIND, VB>(a, st);
  else launch_cfg<T64x64, AK, VA, BKIND, VB>(a, st);
}

inline size_t splitk_ws_bytes(const GemmArgs& a) {
  return a.splits > 1 ? (size_t)a.batch * a.splits * a.M * a.N * sizeof(float) : 0;
}

inline void set_splits(GemmArgs& a, int splits) {
  a.splits = std::max(1, splits);
  a.k_split = ((cdiv(a.K, a.splits) + DBK - 1) / DBK) * DBK;  // whole K-tiles of either main loop
  a.splits = std::max(1, cdiv(a.K, a.k_split));
}

// Split-K factor: fill the chip AND avoid wave quantisation (a last round of blocks that leaves
// most CUs idle): the smallest s whose tiles*s blocks make >= 1 round of 256 CUs at >= 95 % round
// efficiency (fewer splits = less partial-sum traffic); otherwise the most efficient s.
// A "round" counts the workgroups resident per CU at once (1 for the 256-wide tiles, 2 for 128x128, 4 for
// 64x64 / 128x16): a small-tile split-K GEMM (c3's wgrad of 32-128 channels: M x N = 32 x 288 .. 128 x 1152,
// K = 25k-400k pixels) with one workgroup per CU runs its K loop latency-bound (one tile in flight per CU).
constexpr int MAX_SPLITS = 256;
inline bool split_res_legacy() {  // experiment knob: MVAE_SPLIT_LEGACY=1 restores one-workgroup-per-CU rounds
  static int v = getenv("MVAE_SPLIT_LEGACY") != nullptr;
  return v != 0;
}
inline int choose_splits(const GemmArgs& a, int cfg) {
  static const int res_of[7] = {1, 1, 1, 2, 4, 4, 3};
  const bool legacy = split_res_legacy();
  const int res = legacy ? 1 : res_of[cfg];
  const long long slots = 256LL * res;
  const long long tiles = tiles_of(cfg, a);
  const int ms = legacy ? std::max(1, (int)std::min<long long>(64, a.K / 512))
                        : std::max(1, (int)std::min<long long>(MAX_SPLITS, a.K / 256));
  if (tiles >= 4 * slots) return 1;
  int best = 1;
  double best_eff = -1.0;
  for (int s = 1; s <= ms; ++s) {
    const long long blocks = tiles * s;
    const long long rounds = (blocks + slots - 1) / slots;
    const double eff = (double)blocks / (double)(rounds * slots);
    const bool full = blocks * 100 >= slots * 94;  // >= 240 of 256 slots
    if (full && eff >= 0.95) return s;
    const double score = eff - (full ? 0.0 : 0.5);
    if (score > best_eff + 1e-9) { best_eff = score; best = s; }
  }
  return best;
}

// Split-K for an under-filled implicit-GEMM conv (fwd / dgrad of the small-spatial layers: c2's 7x7 level at 512
// channels is 98-196 tiles of any shape for 256 CUs, i.e. one partial round): the unsplit tile the cost model chose
// (cfg0) against 256-wide tiles over K split s ways plus the fixed-order reducer, by a time model -- GEMM: rounds x
// tiles resident per CU x tile area x K / s / (per-tile efficiency x MAC rate per CU); reducer: (s + 2) x M x N x 4 B
// at HBM speed + one launch. Returns the tile config with *splits set, or -1 to stay unsplit. Splits keep >= 16
// K-tiles each and must fit ws_bytes.
inline int conv_split_cfg(const GemmArgs& a, int cfg0, size_t ws_bytes, int* splits_out) {
  static const double eff[5] = {1.0, 0.82, 0.82, 0.70, 0.50};
  static const int res[5] = {1, 1, 1, 2, 4};
  static const int area[5] = {65536, 32768, 32768, 16384, 4096};
  if (cfg0 < T256x256 || cfg0 > T64x64 || ws_bytes == 0 || a.batch != 1) return -1;
  const double mac_rate = 0.9e12;  // MAC/s per CU at 256x256 (efficiency 1.0): ~470 TF/s chip-wide, 3xBF16
  auto gemm_s = [&](int c, long long blocks, double k) {
    const long long slots = 256LL * res[c];
    const double rounds = (double)((blocks + slots - 1) / slots);
    return rounds * res[c] * area[c] * k / eff[c] / mac_rate;
  };
  const double t0 = gemm_s(cfg0, tiles_of(cfg0, a), (double)a.K);
  const double mn4 = 4.0 * (double)a.M * (double)a.N;
  int best = -1, best_s = 1;
  double best_t = t0 * 0.92;  // demand a clear gain: the model ignores prologue / epilogue per split
  for (int c = T256x256; c <= T128x256; ++c) {
    if ((c == T256x256 && (a.M <= 128 || a.N <= 128)) || (c == T256x128 && a.M <= 128) || (c == T128x256 && a.N <= 128))
      continue;
    const long long tiles = tiles_of(c, a);
    for (int s = 2; s <= 32 && (long long)a.K / s >= 16 * BK; ++s) {
      GemmArgs b = a;
      set_splits(b, s);
      if (b.splits < 2 || splitk_ws_bytes(b) > ws_bytes) continue;
      const double t = gemm_s(c, tiles * b.splits, (double)b.k_split) + (b.splits + 2.0) * mn4 / 5.0e12 + 4.0e-6;
      if (t < best_t) {
        best_t = t;
        best = c;
        best_s = b.splits;
      }
    }
  }
  *splits_out = best_s;
  return best;
}

inline void plan_splits(GemmArgs& a, int cfg, float* ws, size_t ws_bytes) {
  set_splits(a, ws ? choose_splits(a, cfg) : 1);
  while (a.splits > 1 && splitk_ws_bytes(a) > ws_bytes) set_splits(a, a.splits / 2);
  a.ws = ws;
}

int gemm_finish(GemmArgs& a, hipStream_t st);
bool splitk_vec_ok(const GemmArgs& a);                  // splitk_reduce4_rows applies
void splitk_vec_grid(const GemmArgs& a, int& gx, int& gy);  // its (column groups, row blocks) grid

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
constexpr long long MAX_DESC_BYTES = 0xFFFFFF00LL;  // one buffer descriptor covers < 4 GiB

}  // namespace mvae
