// Strided-batched GEMM entry point (attention products, 1x1 convolutions) + the split-K reducer.
#include "gemm_core.h"

namespace mvae {

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
    for (int z = 0; z < a.splits; ++z) s += w[z * mn];  // fixed order: deterministic
    float v = a.alpha * s + (a.bias ? a.bias[col] : 0.f);
    if (a.res) v += a.res[bidx * a.sR + (long long)row * a.ldr + col];
    float* cp = a.C + bidx * a.sC + (long long)row * a.ldc + col;
    if (a.beta != 0.f) v += a.beta * *cp;
    *cp = v;
  }
}

// Same reduction, 4 columns per thread (splitk_reduce4_rows): 2-D grid (column groups x output rows), so the row /
// batch index is block-uniform (no per-element 64-bit division).
__global__ void __launch_bounds__(256) splitk_reduce4_kernel(GemmArgs a) {
  splitk_reduce4_rows(a, blockIdx.x, blockIdx.y, gridDim.y);
}

bool splitk_vec_ok(const GemmArgs& a) {
  return (a.N & 3) == 0 && (a.ldc & 3) == 0 && (a.sC & 3) == 0 && al16(a.C) &&
         (!a.res || ((a.ldr & 3) == 0 && (a.sR & 3) == 0 && al16(a.res))) && (!a.bias || al16(a.bias)) &&
         (long long)a.M * a.batch < (1LL << 31);
}

void splitk_vec_grid(const GemmArgs& a, int& gx, int& gy) {
  gx = cdiv(a.N >> 2, 256);
  gy = (int)std::min<long long>((long long)a.M * a.batch, std::max(1, 8192 / gx));
}

int gemm_finish(GemmArgs& a, hipStream_t st) {
  if (a.splits > 1) {
    if (splitk_vec_ok(a)) {
      int gx, gy;
      splitk_vec_grid(a, gx, gy);
      hipLaunchKernelGGL(splitk_reduce4_kernel, dim3(gx, gy), dim3(256), 0, st, a);
    } else {
      const long long total = (long long)a.M * a.N * a.batch;
      const int blocks = (int)std::min<long long>((total + 255) / 256, 4096);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, a);
    }
  }
  return launch_status();
}

static long long extent(bool trans, long long rows, long long k, long long ld) {
  // bytes spanned by a rows x k operand stored [rows][ld] (trans=0) or [k][ld] (trans=1)
  if (rows <= 0 || k <= 0) return 4;
  return (trans ? (k - 1) * ld + rows : (rows - 1) * ld + k) * 4;
}

}  // namespace mvae

using namespace mvae;

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
  const long long ea = extent(trans_a, m, k, lda), eb = extent(!trans_b, n, k, ldb);
  const long long ec = extent(false, m, n, ldc), er = residual ? extent(false, m, n, ldr) : 4;
  if (std::max(std::max(ea, eb), std::max(ec, er)) > MAX_DESC_BYTES) {
    set_error("gemm: an operand of one batch entry exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  a.a_bytes = (unsigned)ea; a.b_bytes = (unsigned)eb; a.c_bytes = (unsigned)ec; a.r_bytes = (unsigned)er;
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
  return gemm_finish(a, st);
}

size_t mvae_gemm_workspace_bytes(int m, int n, int k, int batch) {
  GemmArgs a{};
  a.M = m; a.N = n; a.K = k; a.batch = batch;
  set_splits(a, choose_splits(a, choose_tile(a, true, true)));
  size_t b1 = splitk_ws_bytes(a);
  set_splits(a, choose_splits(a, choose_tile(a, false, true)));
  return std::max(b1, splitk_ws_bytes(a));
}

}  // extern "C"
