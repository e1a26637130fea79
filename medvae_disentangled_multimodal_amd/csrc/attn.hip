// Fused single-tile attention core for n <= 64 tokens: AttnBlock's bmm(q, k) * C^-1/2 -> softmax(dim=2) -> bmm(v, w^T)
// (src/models/encoder_decoder.py:83-107) at the lowest resolutions (the mid blocks at 7x7 = 49 tokens in c1 / c2 / c3
// and 8x8 = 64 tokens in c4 / c5). One workgroup per image, one launch per direction:
//   forward : S = Q K^T (K = C) -> scaled, row softmax in LDS (fp32) -> O = P V, chunked over C; writes O and the row
//             log-sum-exp (64 floats per image) -- the n x n score matrix never goes to HBM
//   backward: recomputes S and P = exp(scale S - lse) from the saved log-sum-exp, dP = dO V^T, dS = scale * P (dP - D)
//             with D_i = sum_j P_ij dP_ij (the softmax backward), then per C-chunk dV = P^T dO, dQ = dS K, dK = dS^T Q
// The products run on the implicit-GEMM core's loaders, LDS images, fragment reads and mma<PREC> (3xBF16, bf16 or
// exact fp32, the process-wide GEMM arithmetic), 4 waves as 2 x 2 over the 64 x 64 block. Row softmax statistics and
// the dS row sums are fixed-order (4 lanes per row + a 2-step xor shuffle): deterministic.
#include "gemm_core.h"

namespace mvae {

constexpr int AT_MAXN = 64;  // tokens per image (the block's rows and the K of the P-products)
constexpr int AT_NT = 256;   // 4 waves, 2 x 2 over the 64 x 64 output block
constexpr int AT_CB = 64;    // channels per output chunk of the P-products
constexpr int AT_PE = 65;    // pitch of the fp32 score scratch

template <int PREC>
struct AtTypes {
  using LRowA = LoadRowK<64, 4, AT_NT, true, PREC>;    // A = [rows][k] row-major (Q, dO)
  using LRowB = LoadRowK<64, 4, AT_NT, false, PREC>;   // B = [n][k] row-major (K, V as the B of Q K^T / dO V^T)
  using LColB = LoadColK<64, 4, AT_NT, false, PREC>;   // B = [k][n] (V, dO, K, Q as the B of the P-products)
  using IR = Img<64, false>;
  using IC = Img<64, true>;
};

// MFMA 16x16x32 operand fragment from a ROW or COL image (read_frag's layout; the COL reads are the compiler's
// ds_read_b64_tr_b16 builtin so its own lgkmcnt waits cover them)
template <bool COL>
__device__ __forceinline__ bf16x8 at_frag(const __bf16* plane, int row0, int lane) {
  return read_frag<64, COL, 16>(plane, row0, 0, lane);
}

// the 64 x 64 block A (M rows) x B (N rows) over g.K, both operands staged from HBM through the LDS images ia / ib
// (register prefetch of the next K-tile during the current one)
template <int PREC, class LA, class LB>
__device__ void at_block_mm(const GemmArgs& g, const float* A, const float* B, __bf16* ia, __bf16* ib,
                            f32x4 (&acc)[2][2], int tid, int lane, int wm, int wn) {
  using IA = Img<64, LA::COL>;
  using IB = Img<64, LB::COL>;
  LA la;
  LB lb;
  la.init(g, A, 0, 0, tid, 0);
  lb.init(g, B, 0, 0, tid, 0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (g.K + BK - 1) / BK;
  if (nt > 0) {
    la.load(g);
    lb.load(g);
  }
  for (int t = 0; t < nt; ++t) {
    __syncthreads();  // every wave's fragment reads of the previous K-tile are done
    la.store(ia);
    lb.store(ib);
    __syncthreads();
    if (t + 1 < nt) {
      la.advance();
      lb.advance();
      la.load(g);
      lb.load(g);
    }
    bf16x8 ah[2], al[2]{}, bh[2], bl[2]{};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ah[i] = at_frag<LA::COL>(ia, wm * 32 + i * 16, lane);
      if constexpr (PREC != 1) al[i] = at_frag<LA::COL>(ia + IA::PLANE, wm * 32 + i * 16, lane);
      bh[i] = at_frag<LB::COL>(ib, wn * 32 + i * 16, lane);
      if constexpr (PREC != 1) bl[i] = at_frag<LB::COL>(ib + IB::PLANE, wn * 32 + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) mma<PREC>(acc[i][j], ah[i], al[i], bh[j], bl[j]);
  }
}

// 64 x CB block of (A from LDS: the P / dS images, one per 32-deep K-tile, ROW or COL) x (B = a [K][N] row-major matrix
// chunk staged from HBM), K = g.K <= 64
template <int PREC, bool ACOL, class LB>
__device__ void at_block_pmm(const GemmArgs& g, const float* B, int n0, const __bf16* ia0, const __bf16* ia1,
                             __bf16* ib, f32x4 (&acc)[2][2], int tid, int lane, int wm, int wn) {
  using IA = Img<64, ACOL>;
  using IB = Img<64, LB::COL>;
  LB lb;
  lb.init(g, B, n0, 0, tid, 0);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (g.K + BK - 1) / BK;
  if (nt > 0) lb.load(g);
  for (int t = 0; t < nt; ++t) {
    __syncthreads();
    lb.store(ib);
    __syncthreads();
    if (t + 1 < nt) {
      lb.advance();
      lb.load(g);
    }
    const __bf16* iat = t == 0 ? ia0 : ia1;
    bf16x8 ah[2], al[2]{}, bh[2], bl[2]{};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ah[i] = at_frag<ACOL>(iat, wm * 32 + i * 16, lane);
      if constexpr (PREC != 1) al[i] = at_frag<ACOL>(iat + IA::PLANE, wm * 32 + i * 16, lane);
      bh[i] = at_frag<LB::COL>(ib, wn * 32 + i * 16, lane);
      if constexpr (PREC != 1) bl[i] = at_frag<LB::COL>(ib + IB::PLANE, wn * 32 + i * 16, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) mma<PREC>(acc[i][j], ah[i], al[i], bh[j], bl[j]);
  }
}

// accumulator block -> fp32 scratch s[64][AT_PE] (times mul)
__device__ __forceinline__ void at_acc_to_lds(const f32x4 (&acc)[2][2], float* s, float mul, int lane, int wm, int wn) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        s[(wm * 32 + i * 16 + acc_row<16>(r, lane)) * AT_PE + wn * 32 + j * 16 + (lane & 15)] = mul * acc[i][j][r];
}

// accumulator block -> rows [0, n) x cols [n0, n0 + 64) of a [n][ldo] fp32 matrix
__device__ __forceinline__ void at_acc_store(const f32x4 (&acc)[2][2], float* o, int ldo, int n, int ncols, int n0,
                                             int lane, int wm, int wn) {
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 32 + i * 16 + acc_row<16>(r, lane);
        if (row < n && col < ncols) o[(long long)row * ldo + col] = acc[i][j][r];
      }
    }
}

// fp32 scratch s[64][AT_PE] (rows = m, cols = k) -> the ROW images (A[m][k], one per 32-deep K-tile) and / or the COL
// images of its transpose (A[m = col][k = row]) in the GEMM's operand format
template <int PREC>
__device__ void at_stage_images(const float* s, __bf16* row_img0, __bf16* row_img1, __bf16* col_img0, __bf16* col_img1,
                                int tid) {
  using IR = Img<64, false>;
  using IC = Img<64, true>;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = tid + q * AT_NT;  // 64 rows x 16 groups of 4 columns
    const int r = idx >> 4, c = (idx & 15) * 4;
    const float4 v{s[r * AT_PE + c], s[r * AT_PE + c + 1], s[r * AT_PE + c + 2], s[r * AT_PE + c + 3]};
    if (row_img0 != nullptr)  // A[m = r][k = c..c+3]
      st_split<PREC>(c < 32 ? row_img0 : row_img1, IR::PLANE, row_off(r, (c & 31) >> 2), v);
    if (col_img0 != nullptr) {  // A^T: m = c..c+3, k = r
      const int kr = r & 31;
      st_split<PREC>(r < 32 ? col_img0 : col_img1, IC::PLANE, kr * IC::PITCH + (c ^ col_swz(kr)), v);
    }
  }
}

template <int PREC>
struct AtFwdSmem {
  using T = AtTypes<PREC>;
  __bf16 ia[T::IR::SIZE], ib[T::IR::SIZE];        // Q K^T staging
  __bf16 pr[2][T::IR::SIZE];                      // P as ROW images (2 K-tiles)
  __bf16 vb[T::IC::SIZE];                         // V chunk (COL)
  float s[AT_MAXN * AT_PE];                       // scores / P (fp32)
};

template <int PREC>
__global__ void __launch_bounds__(AT_NT) attn_small_fwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               const float* __restrict__ v, float* __restrict__ o,
                                                               float* __restrict__ lse, int n, int C, float scale) {
  using T = AtTypes<PREC>;
  __shared__ __attribute__((aligned(16))) AtFwdSmem<PREC> sm;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const long long off = (long long)b * n * C;
  const unsigned bytes = (unsigned)((long long)n * C * 4);
  f32x4 acc[2][2];
  {  // S = Q K^T
    GemmArgs g{};
    g.M = n; g.N = n; g.K = C;
    g.lda = C; g.ldb = C; g.a_bytes = bytes; g.b_bytes = bytes;
    at_block_mm<PREC, typename T::LRowA, typename T::LRowB>(g, q + off, k + off, sm.ia, sm.ib, acc, tid, lane, wm, wn);
  }
  at_acc_to_lds(acc, sm.s, scale, lane, wm, wn);
  __syncthreads();
  {  // row softmax over the n valid keys: 4 lanes per row, 16 columns each
    const int r = tid >> 2, qd = tid & 3;
    float* sr = sm.s + r * AT_PE + qd * 16;
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (qd * 16 + j < n) m = fmaxf(m, sr[j]);
    m = fmaxf(m, __shfl_xor(m, 1, 64));
    m = fmaxf(m, __shfl_xor(m, 2, 64));
    float e[16], l = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      e[j] = (r < n && qd * 16 + j < n) ? __expf(sr[j] - m) : 0.f;
      l += e[j];
    }
    l += __shfl_xor(l, 1, 64);
    l += __shfl_xor(l, 2, 64);
    const float inv = r < n ? 1.f / l : 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) sr[j] = e[j] * inv;
    if (qd == 0 && r < n) lse[(long long)b * AT_MAXN + r] = m + __logf(l);
  }
  __syncthreads();
  at_stage_images<PREC>(sm.s, sm.pr[0], sm.pr[1], nullptr, nullptr, tid);
  GemmArgs g{};  // O = P V: B = V [j][c] (K = n tokens, N = C)
  g.M = n; g.N = C; g.K = n;
  g.ldb = C; g.b_bytes = bytes;
  for (int c0 = 0; c0 < C; c0 += AT_CB) {
    at_block_pmm<PREC, false, typename T::LColB>(g, v + off, c0, sm.pr[0], sm.pr[1], sm.vb, acc, tid, lane, wm, wn);
    at_acc_store(acc, o + off, C, n, C, c0, lane, wm, wn);
  }
}

template <int PREC>
struct AtBwdSmem {
  using T = AtTypes<PREC>;
  __bf16 ia[T::IR::SIZE], ib[T::IR::SIZE];   // Q K^T and dO V^T staging
  __bf16 pc[2][T::IC::SIZE];                 // P^T (COL images): dV = P^T dO
  __bf16 dr[2][T::IR::SIZE];                 // dS (ROW): dQ = dS K
  __bf16 dc[2][T::IC::SIZE];                 // dS^T (COL): dK = dS^T Q
  __bf16 cb[T::IC::SIZE];                    // B chunk (COL)
  float p[AT_MAXN * AT_PE], d[AT_MAXN * AT_PE];
};

template <int PREC>
__global__ void __launch_bounds__(AT_NT) attn_small_bwd_kernel(const float* __restrict__ q, const float* __restrict__ k,
                                                               const float* __restrict__ v, const float* __restrict__ dout,
                                                               const float* __restrict__ lse, float* __restrict__ dq,
                                                               float* __restrict__ dk, float* __restrict__ dv, int n,
                                                               int C, float scale) {
  using T = AtTypes<PREC>;
  __shared__ __attribute__((aligned(16))) AtBwdSmem<PREC> sm;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const long long off = (long long)b * n * C;
  const unsigned bytes = (unsigned)((long long)n * C * 4);
  f32x4 acc[2][2];
  GemmArgs g{};
  g.M = n; g.N = n; g.K = C;
  g.lda = C; g.ldb = C; g.a_bytes = bytes; g.b_bytes = bytes;
  at_block_mm<PREC, typename T::LRowA, typename T::LRowB>(g, q + off, k + off, sm.ia, sm.ib, acc, tid, lane, wm, wn);
  at_acc_to_lds(acc, sm.p, scale, lane, wm, wn);  // scale * S
  at_block_mm<PREC, typename T::LRowA, typename T::LRowB>(g, dout + off, v + off, sm.ia, sm.ib, acc, tid, lane, wm, wn);
  at_acc_to_lds(acc, sm.d, 1.f, lane, wm, wn);  // dP = dO V^T
  __syncthreads();
  {  // P = exp(scale S - lse), D_i = sum_j P_ij dP_ij, dS = scale * P (dP - D)
    const int r = tid >> 2, qd = tid & 3;
    float* pr = sm.p + r * AT_PE + qd * 16;
    float* dr = sm.d + r * AT_PE + qd * 16;
    const float ls = r < n ? lse[(long long)b * AT_MAXN + r] : 0.f;
    float pv[16], dsum = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      pv[j] = (r < n && qd * 16 + j < n) ? __expf(pr[j] - ls) : 0.f;
      dsum += pv[j] * dr[j];
    }
    dsum += __shfl_xor(dsum, 1, 64);
    dsum += __shfl_xor(dsum, 2, 64);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      pr[j] = pv[j];
      dr[j] = scale * pv[j] * (dr[j] - dsum);
    }
  }
  __syncthreads();
  at_stage_images<PREC>(sm.p, nullptr, nullptr, sm.pc[0], sm.pc[1], tid);
  at_stage_images<PREC>(sm.d, sm.dr[0], sm.dr[1], sm.dc[0], sm.dc[1], tid);
  GemmArgs h{};  // the P-products: B = [token][c] chunks, K = n tokens, N = C
  h.M = n; h.N = C; h.K = n;
  h.ldb = C; h.b_bytes = bytes;
  // (three loops over the C-chunks: one loop carrying all three products trips an instruction-selection error in the
  // bf16 instantiation)
  for (int c0 = 0; c0 < C; c0 += AT_CB) {  // dV = P^T dO
    at_block_pmm<PREC, true, typename T::LColB>(h, dout + off, c0, sm.pc[0], sm.pc[1], sm.cb, acc, tid, lane, wm, wn);
    at_acc_store(acc, dv + off, C, n, C, c0, lane, wm, wn);
  }
  for (int c0 = 0; c0 < C; c0 += AT_CB) {  // dQ = dS K
    at_block_pmm<PREC, false, typename T::LColB>(h, k + off, c0, sm.dr[0], sm.dr[1], sm.cb, acc, tid, lane, wm, wn);
    at_acc_store(acc, dq + off, C, n, C, c0, lane, wm, wn);
  }
  for (int c0 = 0; c0 < C; c0 += AT_CB) {  // dK = dS^T Q
    at_block_pmm<PREC, true, typename T::LColB>(h, q + off, c0, sm.dc[0], sm.dc[1], sm.cb, acc, tid, lane, wm, wn);
    at_acc_store(acc, dk + off, C, n, C, c0, lane, wm, wn);
  }
}

static bool at_args_ok(int batch, int n, int c, const void* const* ptrs, int np) {
  if (batch <= 0 || n <= 0 || n > AT_MAXN || c <= 0 || c % AT_CB != 0 || (long long)n * c * 4 > MAX_DESC_BYTES) {
    set_error("attention_small: 1 <= n <= 64 tokens, C a multiple of 64");
    return false;
  }
  for (int i = 0; i < np; ++i)
    if (ptrs[i] == nullptr || !al16(ptrs[i])) {
      set_error("attention_small: 16-B aligned device pointers");
      return false;
    }
  return true;
}

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_attention_small_fwd(const float* q, const float* k, const float* v, float* o, float* lse, int batch, int n,
                             int c, float scale, void* stream) {
  const void* ptrs[] = {q, k, v, o, lse};
  if (!at_args_ok(batch, n, c, ptrs, 5)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int mm = math_mode();
  if (mm == MATH_BF16)
    hipLaunchKernelGGL(attn_small_fwd_kernel<1>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, o, lse, n, c, scale);
  else if (mm == MATH_FP32)
    hipLaunchKernelGGL(attn_small_fwd_kernel<0>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, o, lse, n, c, scale);
  else
    hipLaunchKernelGGL(attn_small_fwd_kernel<3>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, o, lse, n, c, scale);
  return launch_status();
}

int mvae_attention_small_bwd(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                             float* dq, float* dk, float* dv, int batch, int n, int c, float scale, void* stream) {
  const void* ptrs[] = {q, k, v, dout, lse, dq, dk, dv};
  if (!at_args_ok(batch, n, c, ptrs, 8)) return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int mm = math_mode();
  if (mm == MATH_BF16)
    hipLaunchKernelGGL(attn_small_bwd_kernel<1>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, dout, lse, dq, dk, dv, n, c,
                       scale);
  else if (mm == MATH_FP32)
    hipLaunchKernelGGL(attn_small_bwd_kernel<0>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, dout, lse, dq, dk, dv, n, c,
                       scale);
  else
    hipLaunchKernelGGL(attn_small_bwd_kernel<3>, dim3(batch), dim3(AT_NT), 0, st, q, k, v, dout, lse, dq, dk, dv, n, c,
                       scale);
  return launch_status();
}

}  // extern "C"
