// Query-block fused attention for 64 <= n <= 256 tokens (n % 64 == 0): AttnBlock's core softmax(q k^T * C^-1/2, dim=2) v
// (src/models/encoder_decoder.py:83-107) at the 16x16 level of c4 / c5 (n = 256, C = 1024) and the 8x8 mid blocks
// (n = 64, C = 2048). One workgroup per (64-query block, image), 8 waves as 2 (query rows) x 4:
//   forward : S = Q_blk K^T over C (register-staged, double-buffered LDS, one barrier per K-tile) -> scaled row softmax
//             in registers (row max / sum across the 4 column waves through LDS, fixed order) -> P written to HBM (the
//             backward's saved tensor, n x n per image) and staged as COL images -> O_blk = P V over 128-channel chunks.
//             Replaces two batched GEMM launches and a softmax pass; the scores never leave the workgroup.
//   backward: dP = dO_blk V^T -> D = rowsum(P o dP) -> dS = scale * P o (dP - D) written to HBM and staged -> dQ_blk =
//             dS K. dV = P^T dO and dK = dS^T Q sum over every query block and stay batched GEMMs (ops.AttnCoreFn).
// Same loaders, LDS images, fragment reads and mma<PREC> as the implicit-GEMM core (3xBF16, bf16 or exact fp32).
#include "gemm_core.h"

namespace mvae {

constexpr int AQ_NT = 512;  // 8 waves
constexpr int AQ_BQ = 64;   // queries per workgroup
constexpr int AQ_CB = 128;  // output channels per chunk of the P-products

template <int TNS>  // TNS = n / 64: 16-column MFMA tiles per wave in the score block
struct AqShape {
  static constexpr int NTOK = 64 * TNS;
  using IA = Img<AQ_BQ, false>;  // Q / dO K-tile (ROW)
  using IB = Img<NTOK, false>;   // K / V K-tile (ROW)
  using IP = Img<AQ_BQ, true>;   // P / dS K-tile (COL: [key][query])
  using IV = Img<AQ_CB, true>;   // V / K chunk K-tile (COL: [key][channel])
  static constexpr int S_ELEMS = 2 * (IA::SIZE + IB::SIZE);
  static constexpr int O_ELEMS = (NTOK / 32) * IP::SIZE + 2 * IV::SIZE;
  static constexpr int ELEMS = S_ELEMS > O_ELEMS ? S_ELEMS : O_ELEMS;
  static constexpr int RED_FLOATS = 2 * 4 * AQ_BQ;  // row max / row sum partials of the 4 column waves
  static constexpr int BYTES = ELEMS * 2 + RED_FLOATS * 4;
  static_assert(BYTES <= 163840, "attn_tile: LDS");
};

// acc[i][j] (i: 16-row tile of the wave's 32 rows, j: 16-column tile) of the [64 x n] block A_blk B^T over K = C, both
// operands row-major [rows][C] (Q or dO against K or V)
template <int PREC, int TNS>
__device__ void aq_scores(const float* A, const float* B, int n, int C, __bf16* sm, f32x4 (&acc)[2][TNS], int tid,
                          int lane, int wm, int wn) {
  using S = AqShape<TNS>;
  using LA = LoadRowK<AQ_BQ, 4, AQ_NT, true, PREC>;
  using LB = LoadRowK<S::NTOK, 4, AQ_NT, false, PREC>;
  constexpr int BUF = S::IA::SIZE + S::IB::SIZE;
  GemmArgs g{};
  g.M = AQ_BQ; g.N = n; g.K = C;
  g.lda = C; g.ldb = C;
  g.a_bytes = (unsigned)(AQ_BQ * C * 4); g.b_bytes = (unsigned)((long long)n * C * 4);
  LA la;
  LB lb;
  la.init(g, A, 0, 0, tid, 0);
  lb.init(g, B, 0, 0, tid, 0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TNS; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = C / BK;
  la.load(g);
  lb.load(g);
  la.store(sm);
  lb.store(sm + S::IA::SIZE);
  if (nt > 1) {
    la.advance();
    lb.advance();
    la.load(g);
    lb.load(g);
  }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const __bf16* Ai = sm + (t & 1) * BUF;
    const __bf16* Bi = Ai + S::IA::SIZE;
    bf16x8 bh[TNS], bl[TNS];
#pragma unroll
    for (int j = 0; j < TNS; ++j) {
      bh[j] = read_frag<S::NTOK, false, 16>(Bi, wn * (S::NTOK / 4) + j * 16, 0, lane);
      if constexpr (PREC != 1) bl[j] = read_frag<S::NTOK, false, 16>(Bi + S::IB::PLANE, wn * (S::NTOK / 4) + j * 16, 0, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16x8 ah = read_frag<AQ_BQ, false, 16>(Ai, wm * 32 + i * 16, 0, lane);
      bf16x8 al{};
      if constexpr (PREC != 1) al = read_frag<AQ_BQ, false, 16>(Ai + S::IA::PLANE, wm * 32 + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < TNS; ++j) mma<PREC>(acc[i][j], ah, al, bh[j], bl[j]);
    }
    if (t + 1 < nt) {  // tile t+1 (in registers) into the other buffer, last read one barrier ago
      __bf16* nb = sm + ((t + 1) & 1) * BUF;
      la.store(nb);
      lb.store(nb + S::IA::SIZE);
      if (t + 2 < nt) {
        la.advance();
        lb.advance();
        la.load(g);
        lb.load(g);
      }
    }
    __syncthreads();
  }
}

// fixed-order row reduction of the block [64 x n] held as acc[i][j][r] (row wm*32 + i*16 + 4*(lane>>4) + r): within the
// wave over its TNS tiles and the 16 lanes of a row (xor tree), then over the 4 column waves through red[4][64]
template <bool MAX, int TNS>
__device__ __forceinline__ void aq_row_reduce(const float (&v)[2][4], float (&out)[2][4], float* red, int lane, int wm,
                                              int wn) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = v[i][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float y = __shfl_xor(x, o, 64);
        x = MAX ? fmaxf(x, y) : x + y;
      }
      if ((lane & 15) == 0) red[wn * AQ_BQ + wm * 32 + i * 16 + 4 * (lane >> 4) + r] = x;
    }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wm * 32 + i * 16 + 4 * (lane >> 4) + r;
      const float a0 = red[row], a1 = red[AQ_BQ + row], a2 = red[2 * AQ_BQ + row], a3 = red[3 * AQ_BQ + row];
      out[i][r] = MAX ? fmaxf(fmaxf(a0, a1), fmaxf(a2, a3)) : (a0 + a1) + (a2 + a3);
    }
}

// the block acc (P or dS, [64 queries x n keys]) -> HBM rows [q0, q0+64) of a [n][n] matrix and the COL images
// [key % 32][query] of K-tile key / 32 (the A operand of the P-products)
template <int PREC, int TNS>
__device__ __forceinline__ void aq_publish(const f32x4 (&acc)[2][TNS], float* dst, int n, __bf16* pimg, int lane, int wm,
                                           int wn) {
  using S = AqShape<TNS>;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TNS; ++j) {
      const int key = wn * (S::NTOK / 4) + j * 16 + (lane & 15);
      const int q = wm * 32 + i * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(long long)(q + r) * n + key] = acc[i][j][r];
      const int kr = key & 31;
      st_split<PREC>(pimg + (key >> 5) * S::IP::SIZE, S::IP::PLANE, kr * S::IP::PITCH + (q ^ col_swz(kr)),
                     float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]});
    }
}

// out_blk[64][C] = (P or dS images)[64][n] . B[n][C] over 128-channel chunks (B = V or K, row-major [token][C])
template <int PREC, int TNS>
__device__ void aq_pmm(const __bf16* pimg, const float* B, float* out, int n, int C, __bf16* vbuf, int tid, int lane,
                       int wm, int wn) {
  using S = AqShape<TNS>;
  using LV = LoadColK<AQ_CB, 4, AQ_NT, false, PREC>;
  GemmArgs h{};
  h.N = C; h.K = n; h.ldb = C; h.b_bytes = (unsigned)((long long)n * C * 4);
  const int nt = n / BK;
  for (int c0 = 0; c0 < C; c0 += AQ_CB) {
    LV lv;
    lv.init(h, B, c0, 0, tid, 0);
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    lv.load(h);
    lv.store(vbuf);
    if (nt > 1) {
      lv.advance();
      lv.load(h);
    }
    __syncthreads();  // (also publishes the P / dS images on the first chunk)
    for (int t = 0; t < nt; ++t) {
      const __bf16* Ai = pimg + t * S::IP::SIZE;
      const __bf16* Bi = vbuf + (t & 1) * S::IV::SIZE;
      bf16x8 ah[2], al[2]{}, bh[2], bl[2]{};
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ah[i] = read_frag<AQ_BQ, true, 16>(Ai, wm * 32 + i * 16, 0, lane);
        if constexpr (PREC != 1) al[i] = read_frag<AQ_BQ, true, 16>(Ai + S::IP::PLANE, wm * 32 + i * 16, 0, lane);
        bh[i] = read_frag<AQ_CB, true, 16>(Bi, wn * 32 + i * 16, 0, lane);
        if constexpr (PREC != 1) bl[i] = read_frag<AQ_CB, true, 16>(Bi + S::IV::PLANE, wn * 32 + i * 16, 0, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) mma<PREC>(acc[i][j], ah[i], al[i], bh[j], bl[j]);
      if (t + 1 < nt) {
        lv.store(vbuf + ((t + 1) & 1) * S::IV::SIZE);
        if (t + 2 < nt) {
          lv.advance();
          lv.load(h);
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = c0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(long long)(wm * 32 + i * 16 + acc_row<16>(r, lane)) * C + col] = acc[i][j][r];
      }
  }
}

template <int PREC, int TNS>
__global__ void __launch_bounds__(AQ_NT) attn_tile_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                              const float* __restrict__ v, float* __restrict__ o,
                                                              float* __restrict__ p, int n, int C, float scale) {
  using S = AqShape<TNS>;
  __shared__ __attribute__((aligned(16))) __bf16 sm[S::BYTES / 2];
  float* red = (float*)(sm + S::ELEMS);
  const int qb = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const long long img = (long long)b * n * C, q0 = (long long)qb * AQ_BQ;
  f32x4 acc[2][TNS];
  aq_scores<PREC, TNS>(q + img + q0 * C, k + img, n, C, sm, acc, tid, lane, wm, wn);
  // row softmax of scale * S (max-subtracted, fixed-order sums)
  float mx[2][4], m[2][4], sum[2][4], l[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = -INFINITY;
#pragma unroll
      for (int j = 0; j < TNS; ++j) x = fmaxf(x, scale * acc[i][j][r]);
      mx[i][r] = x;
    }
  aq_row_reduce<true, TNS>(mx, m, red, lane, wm, wn);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TNS; ++j) {
        const float e = __expf(scale * acc[i][j][r] - m[i][r]);
        acc[i][j][r] = e;
        s += e;
      }
      sum[i][r] = s;
    }
  aq_row_reduce<false, TNS>(sum, l, red + 4 * AQ_BQ, lane, wm, wn);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float inv = 1.f / l[i][r];
#pragma unroll
      for (int j = 0; j < TNS; ++j) acc[i][j][r] *= inv;
    }
  // (the score loop ended on a barrier: its staging buffers are free for the P images)
  __bf16* pimg = sm;
  __bf16* vbuf = sm + (S::NTOK / 32) * S::IP::SIZE;
  aq_publish<PREC, TNS>(acc, p + (long long)b * n * n + q0 * n, n, pimg, lane, wm, wn);
  aq_pmm<PREC, TNS>(pimg, v + img, o + img + q0 * C, n, C, vbuf, tid, lane, wm, wn);
}

template <int PREC, int TNS>
__global__ void __launch_bounds__(AQ_NT) attn_tile_bwd_kernel(const float* __restrict__ k, const float* __restrict__ v,
                                                              const float* __restrict__ dout, const float* __restrict__ p,
                                                              float* __restrict__ dq, float* __restrict__ ds, int n, int C,
                                                              float scale) {
  using S = AqShape<TNS>;
  __shared__ __attribute__((aligned(16))) __bf16 sm[S::BYTES / 2];
  float* red = (float*)(sm + S::ELEMS);
  const int qb = blockIdx.x, b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;
  const long long img = (long long)b * n * C, q0 = (long long)qb * AQ_BQ;
  f32x4 acc[2][TNS];
  aq_scores<PREC, TNS>(dout + img + q0 * C, v + img, n, C, sm, acc, tid, lane, wm, wn);  // dP = dO V^T
  const float* pb = p + (long long)b * n * n + q0 * n;
  float pv[2][TNS][4], dsum[2][4], D[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < TNS; ++j) {
        const int key = wn * (S::NTOK / 4) + j * 16 + (lane & 15);
        pv[i][j][r] = pb[(long long)(wm * 32 + i * 16 + 4 * (lane >> 4) + r) * n + key];
        s += pv[i][j][r] * acc[i][j][r];
      }
      dsum[i][r] = s;
    }
  aq_row_reduce<false, TNS>(dsum, D, red, lane, wm, wn);  // D_i = sum_j P_ij dP_ij
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TNS; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[i][j][r] = scale * pv[i][j][r] * (acc[i][j][r] - D[i][r]);
  __bf16* pimg = sm;
  __bf16* vbuf = sm + (S::NTOK / 32) * S::IP::SIZE;
  aq_publish<PREC, TNS>(acc, ds + (long long)b * n * n + q0 * n, n, pimg, lane, wm, wn);
  aq_pmm<PREC, TNS>(pimg, k + img, dq + img + q0 * C, n, C, vbuf, tid, lane, wm, wn);  // dQ = dS K
}

static bool aq_args_ok(int batch, int n, int c, const void* const* ptrs, int np) {
  if (batch <= 0 || batch > 65535 || n < 64 || n > 256 || n % 64 != 0 || c <= 0 || c % AQ_CB != 0 ||
      (long long)n * c * 4 > MAX_DESC_BYTES) {
    set_error("attention_tile: 64 <= n <= 256 tokens with n %% 64 == 0, C a multiple of 128");
    return false;
  }
  for (int i = 0; i < np; ++i)
    if (ptrs[i] == nullptr || !al16(ptrs[i])) {
      set_error("attention_tile: 16-B aligned device pointers");
      return false;
    }
  return true;
}

template <int TNS, class F>
static void aq_dispatch_prec(F&& launch) {
  const int mm = math_mode();
  if (mm == MATH_BF16) launch(std::integral_constant<int, 1>{});
  else if (mm == MATH_FP32) launch(std::integral_constant<int, 0>{});
  else launch(std::integral_constant<int, 3>{});
}

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_attention_tile_fwd(const float* q, const float* k, const float* v, float* o, float* p, int batch, int n, int c,
                            float scale, void* stream) {
  const void* ptrs[] = {q, k, v, o, p};
  if (!aq_args_ok(batch, n, c, ptrs, 5)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(n / AQ_BQ, batch);
  auto go = [&](auto tns) {
    constexpr int T = decltype(tns)::value;
    aq_dispatch_prec<T>([&](auto pc) {
      constexpr int P = decltype(pc)::value;
      hipLaunchKernelGGL((attn_tile_fwd_kernel<P, T>), grid, dim3(AQ_NT), 0, st, q, k, v, o, p, n, c, scale);
    });
  };
  switch (n / 64) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    default: go(std::integral_constant<int, 4>{}); break;
  }
  return launch_status();
}

int mvae_attention_tile_bwd(const float* k, const float* v, const float* dout, const float* p, float* dq, float* ds,
                            int batch, int n, int c, float scale, void* stream) {
  const void* ptrs[] = {k, v, dout, p, dq, ds};
  if (!aq_args_ok(batch, n, c, ptrs, 6)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid(n / AQ_BQ, batch);
  auto go = [&](auto tns) {
    constexpr int T = decltype(tns)::value;
    aq_dispatch_prec<T>([&](auto pc) {
      constexpr int P = decltype(pc)::value;
      hipLaunchKernelGGL((attn_tile_bwd_kernel<P, T>), grid, dim3(AQ_NT), 0, st, k, v, dout, p, dq, ds, n, c, scale);
    });
  };
  switch (n / 64) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    default: go(std::integral_constant<int, 4>{}); break;
  }
  return launch_status();
}

}  // extern "C"
