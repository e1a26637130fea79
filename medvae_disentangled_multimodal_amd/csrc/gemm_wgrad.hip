// Weight-gradient entry point of the implicit-GEMM convolution (deterministic split-K over pixels).
#include "gemm_core.h"

namespace mvae {
// dbias[m] = beta*dbias[m] + sum over splits of the per-split row sums: one wave per row, lanes over the
// splits, then the fixed wave tree (deterministic; the splits' loads are all in flight at once)
__device__ __forceinline__ void bias_reduce_rows(const float* __restrict__ part, int splits, int m, float* dbias,
                                                 float beta, int blk) {
  const int i = blk * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= m) return;
  float s = 0.f;
  for (int z = lane; z < splits; z += 64) s += part[(long long)z * m + i];
  s = wave_sum_f(s);
  if (lane == 0) dbias[i] = (beta != 0.f ? beta * dbias[i] : 0.f) + s;
}

__global__ void __launch_bounds__(256) bias_reduce_kernel(const float* __restrict__ part, int splits, int m,
                                                          float* dbias, float beta) {
  bias_reduce_rows(part, splits, m, dbias, beta, blockIdx.x);
}

// The weight-gradient epilogue of a split-K launch in ONE launch: grid rows y < gy reduce the dW partials
// (splitk_reduce4_rows over the reducer's own (gx, gy) grid), the rows after them sum the conv bias gradient from the
// per-split row sums (bias_reduce_rows, block (x, gy + r) -> bias block r * gx + x); the two parts touch disjoint
// memory and no block is idle.
__global__ void __launch_bounds__(256) wgrad_finish4_kernel(GemmArgs a, int gy, float* dbias, float bbeta) {
  if ((int)blockIdx.y < gy) {
    splitk_reduce4_rows(a, blockIdx.x, blockIdx.y, gy);
    return;
  }
  bias_reduce_rows(a.bias_ws, a.splits, a.M, dbias, bbeta, (blockIdx.y - gy) * gridDim.x + blockIdx.x);
}

// Upsample-conv weight gradient from the per-class partials of the sub-pixel form, already summed over the
// split-K slices (class c at part + c*cls_stride, [co][(2a+b)*cin + ci]) ->
// dw[co][r][s][ci] = beta*dw + sum_{(ph,a) in P(r), (pw,b) in P(s)} part[2ph+pw][co][(2a+b)*cin+ci]
// with P(0) = {(0,0),(1,0)}, P(1) = {(0,1),(1,0)}, P(2) = {(0,1),(1,1)} (fixed summation order)
__global__ void __launch_bounds__(256) ups_wgrad_combine_kernel(const float* __restrict__ part, long long cls_stride,
                                                                int cout, int cin, float* __restrict__ dw, float beta) {
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * cin) return;
  const int co = (int)(idx / cin), ci = (int)(idx - (long long)co * cin);
  const long long n4 = 4LL * cin;
  float g[4][4];
#pragma unroll
  for (int cls = 0; cls < 4; ++cls)
#pragma unroll
    for (int t = 0; t < 4; ++t) g[cls][t] = part[cls * cls_stride + (long long)co * n4 + t * cin + ci];
  const int pp[3][2][2] = {{{0, 0}, {1, 0}}, {{0, 1}, {1, 0}}, {{0, 1}, {1, 1}}};  // P(r): (parity, tap)
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      float v = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          v += g[2 * pp[r][u][0] + pp[q][e][0]][2 * pp[r][u][1] + pp[q][e][1]];
      float* o = dw + (((long long)co * 3 + r) * 3 + q) * cin + ci;
      *o = (beta != 0.f ? beta * *o : 0.f) + v;
    }
}
}  // namespace mvae

using namespace mvae;

static void ups_wgrad_shape(GemmArgs& a, int nb, int h, int wd, int cin, int cout) {
  a.M = cout; a.N = 4 * cin; a.K = nb * h * wd; a.batch = 4;
}
static size_t ups_part_bytes(const GemmArgs& a) { return (size_t)a.batch * a.splits * a.M * a.N * sizeof(float); }

static bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }
static bool wgrad_p2_enabled() {  // MVAE_NO_WGRAD_P2=1: the general gather (LoadWgradX / DmaWgradX) everywhere
  static const bool v = getenv("MVAE_NO_WGRAD_P2") == nullptr;
  return v;
}

static void wgrad_shape(GemmArgs& a, int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  a.M = cout; a.N = kh * kw * cin; a.K = nb * ho * wo; a.batch = 1;
}

extern "C" {

// dw[cout][r][s][cin] = beta*dw + sum_pixels dy[pix][cout] * x[src(pix, r, s)][cin]   (modes 0 / 1)
int mvae_conv2d_wgrad_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb, int h,
                           int wd, int cin, int cout, int kh, int kw, int stride, int pad_t,
                           int pad_l, int ho, int wo, int mode, float* workspace,
                           size_t workspace_bytes, void* stream) {
  const bool xsplit = (mode & MVAE_CONV_XSPLIT) != 0;   // x holds split4_bf16 groups
  const bool dysplit = (mode & MVAE_CONV_DYSPLIT) != 0;  // dy holds split4_bf16 groups
  const bool pln = (mode & MVAE_CONV_PLANAR) != 0;      // dy and x planar 3xBF16 (PREC 5)
  const bool bf = (mode & MVAE_CONV_BF16) != 0 || pln;  // dy and x DMA-staged (LDS-DMA main loop)
  mode &= ~(MVAE_CONV_XSPLIT | MVAE_CONV_DYSPLIT | MVAE_CONV_BF16 | MVAE_CONV_PLANAR);
  if (bf && (xsplit || dysplit || mode != 0 || dbias || cin % 8 || cout % 8 || !al16(dy) || !al16(x) ||
             math_mode() != (pln ? MATH_3XBF16 : MATH_BF16))) {
    set_error("wgrad: DMA-staged operands need the matching math mode, mode 0, cin %% 8 == 0, cout %% 8 == 0, "
              "aligned dy / x, no fused bias");
    return MVAE_EINVAL;
  }
  if (dysplit && (cout % 4 != 0 || !al16(dy) || dbias != nullptr)) {
    set_error("wgrad: a pre-split dy needs cout %% 4 == 0, 16-B alignment and no fused bias (sum it from the fp32 dy)");
    return MVAE_EINVAL;
  }
  if (mode != 0 && mode != 1) { set_error("wgrad: mode must be 0 or 1"); return MVAE_EINVAL; }
  if ((xsplit || dysplit) && split_forbidden()) {
    set_error("wgrad: pre-split operands are not allowed in the exact-fp32 math mode");
    return MVAE_EINVAL;
  }
  if (xsplit && (mode != 0 || cin % 4 != 0 || !al16(x))) {
    set_error("wgrad: a pre-split x needs mode 0, cin %% 4 == 0, 16-B alignment");
    return MVAE_EINVAL;
  }
  if (nb <= 0 || cin <= 0 || cout <= 0) { set_error("wgrad: bad sizes"); return MVAE_EINVAL; }
  const long long in_img = (long long)h * wd * cin * 4, out_img = (long long)ho * wo * cout * 4;
  if (std::max(in_img, out_img) > MAX_DESC_BYTES || (long long)cout * kh * kw * cin * 4 > MAX_DESC_BYTES) {
    set_error("wgrad: one image exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  const int chunk = (int)std::min<long long>(nb, MAX_DESC_BYTES / std::max(in_img, out_img));
  hipStream_t st = (hipStream_t)stream;
  const bool va = (cout % 4 == 0) && al16(dy);
  const bool vb = (cin % 4 == 0) && al16(x);
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int n = std::min(chunk, nb - b0);
    GemmArgs a{};
    wgrad_shape(a, n, cin, cout, kh, kw, ho, wo);
    a.A = bf ? (const float*)((const __bf16*)dy + (long long)b0 * (out_img / 4)) : dy + (long long)b0 * (out_img / 4);
    a.lda = cout;
    a.B = bf ? (const float*)((const __bf16*)x + (long long)b0 * (in_img / 4)) : x + (long long)b0 * (in_img / 4);
    a.C = dw; a.ldc = a.N; a.alpha = 1.f; a.beta = b0 == 0 ? beta : 1.f;
    a.a_bytes = (unsigned)(out_img * n / (bf ? 2 : 1)); a.b_bytes = (unsigned)(in_img * n / (bf ? 2 : 1));
    if (pln) {
      a.a_lo = (unsigned)(out_img / 2 * nb);
      a.b_lo = (unsigned)(in_img / 2 * nb);
    }
    a.c_bytes = (unsigned)((long long)a.M * a.N * 4);
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
    set_gather_magic(a);
    a.stride = stride; a.pad_t = pad_t; a.pad_l = pad_l;
    const int cfg = choose_tile(a, va && vb, workspace != nullptr);
    const size_t bias_bytes = dbias ? ((size_t)MAX_SPLITS * a.M * sizeof(float) + 256) : 0;
    if (dbias && workspace_bytes < bias_bytes) { set_error("wgrad: workspace too small"); return MVAE_EWORKSPACE; }
    plan_splits(a, cfg, workspace, workspace_bytes - bias_bytes);
    // bias partials live after the split-K partials
    a.bias_ws = dbias ? (float*)((char*)workspace + ((splitk_ws_bytes(a) + 255) & ~(size_t)255)) : nullptr;
    // stride-1 "same" convs at power-of-two H, W: the shift-and-mask im2col gather (B_WGRAD_P2)
    const bool p2 = wgrad_p2_enabled() && mode == 0 && stride == 1 && ho == h && wo == wd && pow2(h) && pow2(wd);
    if (p2) {
      a.lw = 0;
      while ((1 << a.lw) < wd) ++a.lw;
    }
    if (bf) {
      wgrad_dma(p2 ? B_WGRAD_P2 : B_WGRAD_FWD, a, st, cfg, pln ? 5 : 4);
    } else if (p2 && va && (xsplit || vb)) {
      if (dysplit && xsplit) launch_big<A_COLM_SPLIT, 4, B_WGRAD_P2_SPLIT, 4>(a, st, cfg);
      else if (dysplit) launch_big<A_COLM_SPLIT, 4, B_WGRAD_P2, 4>(a, st, cfg);
      else if (xsplit) launch_big<A_COLM, 4, B_WGRAD_P2_SPLIT, 4>(a, st, cfg);
      else launch_big<A_COLM, 4, B_WGRAD_P2, 4>(a, st, cfg);
    } else if (dysplit) {
      if (xsplit) launch_big<A_COLM_SPLIT, 4, B_WGRAD_FWD_SPLIT, 4>(a, st, cfg);
      else if (mode == 0 && vb) launch_big<A_COLM_SPLIT, 4, B_WGRAD_FWD, 4>(a, st, cfg);
      else if (mode == 0) launch_small<A_COLM_SPLIT, 4, B_WGRAD_FWD, 1>(a, st, cfg);
      else if (vb) launch_big<A_COLM_SPLIT, 4, B_WGRAD_UPS, 4>(a, st, cfg);
      else launch_small<A_COLM_SPLIT, 4, B_WGRAD_UPS, 1>(a, st, cfg);
    } else if (xsplit) {
      if (va) launch_big<A_COLM, 4, B_WGRAD_FWD_SPLIT, 4>(a, st, cfg);
      else launch_small<A_COLM, 1, B_WGRAD_FWD_SPLIT, 4>(a, st, cfg);
    } else if (mode == 0) {
      if (va && vb) launch_big<A_COLM, 4, B_WGRAD_FWD, 4>(a, st, cfg);
      else if (va) launch_small<A_COLM, 4, B_WGRAD_FWD, 1>(a, st, cfg);
      else if (vb) launch_small<A_COLM, 1, B_WGRAD_FWD, 4>(a, st, cfg);
      else launch_small<A_COLM, 1, B_WGRAD_FWD, 1>(a, st, cfg);
    } else {
      if (va && vb) launch_big<A_COLM, 4, B_WGRAD_UPS, 4>(a, st, cfg);
      else if (va) launch_small<A_COLM, 4, B_WGRAD_UPS, 1>(a, st, cfg);
      else if (vb) launch_small<A_COLM, 1, B_WGRAD_UPS, 4>(a, st, cfg);
      else launch_small<A_COLM, 1, B_WGRAD_UPS, 1>(a, st, cfg);
    }
    if (dbias && a.splits > 1 && splitk_vec_ok(a)) {  // dW reduction + bias gradient: one launch
      int gx, gy;
      splitk_vec_grid(a, gx, gy);
      hipLaunchKernelGGL(wgrad_finish4_kernel, dim3(gx, gy + cdiv(cdiv(a.M, 4), gx)), dim3(256), 0, st, a, gy, dbias,
                         b0 == 0 ? beta : 1.f);
      const int rc = launch_status();
      if (rc) return rc;
      continue;
    }
    if (dbias)
      hipLaunchKernelGGL(bias_reduce_kernel, dim3(cdiv(a.M, 4)), dim3(256), 0, st, (const float*)a.bias_ws,
                         a.splits, a.M, dbias, b0 == 0 ? beta : 1.f);
    const int rc = gemm_finish(a, st);
    if (rc) return rc;
  }
  return MVAE_OK;
}

// Weight (+ bias) gradient of Upsample's convolution through its sub-pixel form (see
// mvae_conv2d_upsample_nhwc): per parity class a [cout] x [2*2*cin] GEMM over the class's pixels (A = dY^T
// walking the class, B = 2x2 gather of the low-resolution x), deterministic split-K partials, then a fixed-
// order combine into the 3x3 kernel. 4/9 of the reference's MACs.
int mvae_conv2d_wgrad_upsample_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb,
                                    int h, int wd, int cin, int cout, float* workspace, size_t workspace_bytes,
                                    void* stream) {
  if (nb <= 0 || h <= 0 || wd <= 0 || cin <= 0 || cout <= 0) { set_error("wgrad_upsample: bad sizes"); return MVAE_EINVAL; }
  const long long in_img = (long long)h * wd * cin * 4, out_img = 4LL * h * wd * cout * 4;
  if (std::max(in_img, out_img) > MAX_DESC_BYTES || 16LL * cout * cin * 4 > MAX_DESC_BYTES) {
    set_error("wgrad_upsample: one image exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  if (workspace == nullptr) { set_error("wgrad_upsample: workspace required"); return MVAE_EWORKSPACE; }
  const int chunk = (int)std::min<long long>(nb, MAX_DESC_BYTES / std::max(in_img, out_img));
  hipStream_t st = (hipStream_t)stream;
  const bool va = (cout % 4 == 0) && al16(dy);
  const bool vb = (cin % 4 == 0) && al16(x);
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int n = std::min(chunk, nb - b0);
    GemmArgs a{};
    ups_wgrad_shape(a, n, h, wd, cin, cout);
    a.A = dy + (long long)b0 * (out_img / 4); a.lda = cout; a.sA = 0;
    a.B = x + (long long)b0 * (in_img / 4); a.sB = 0;
    a.alpha = 1.f; a.beta = 0.f;
    a.a_bytes = (unsigned)(out_img * n); a.b_bytes = (unsigned)(in_img * n);
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = h; a.Wo = wd; a.R = 2; a.S = 2;
    set_gather_magic(a);
    a.stride = 1; a.pad_t = 1; a.pad_l = 1;
    a.sub_w2 = 2 * wd; a.sub_par = 0; a.out_remap = 0;
    const int cfg = choose_tile(a, va && vb, true);
    const size_t bias_bytes = dbias ? ((size_t)4 * MAX_SPLITS * a.M * sizeof(float) + 256) : 0;
    if (workspace_bytes < bias_bytes) { set_error("wgrad_upsample: workspace too small"); return MVAE_EWORKSPACE; }
    const size_t avail = workspace_bytes - bias_bytes;
    set_splits(a, choose_splits(a, cfg));
    while (a.splits > 1 && ups_part_bytes(a) > avail) set_splits(a, a.splits / 2);
    if (ups_part_bytes(a) > avail) { set_error("wgrad_upsample: workspace too small"); return MVAE_EWORKSPACE; }
    a.ws = workspace;
    // one split: the kernel writes C = the class partials directly ([cls][1][M][N], same layout)
    a.C = workspace; a.ldc = a.N; a.sC = (long long)a.M * a.N; a.c_bytes = (unsigned)((long long)a.M * a.N * 4);
    a.bias_ws = dbias ? (float*)((char*)workspace + ((ups_part_bytes(a) + 255) & ~(size_t)255)) : nullptr;
    if (va && vb) launch_big<A_COLM_PIX, 4, B_WGRAD_SUBPIX, 4>(a, st, cfg);
    else if (va) launch_small<A_COLM_PIX, 4, B_WGRAD_SUBPIX, 1>(a, st, cfg);
    else if (vb) launch_small<A_COLM_PIX, 1, B_WGRAD_SUBPIX, 4>(a, st, cfg);
    else launch_small<A_COLM_PIX, 1, B_WGRAD_SUBPIX, 1>(a, st, cfg);
    const float bt = b0 == 0 ? beta : 1.f;
    if (dbias)
      hipLaunchKernelGGL(bias_reduce_kernel, dim3(cdiv(a.M, 4)), dim3(256), 0, st, (const float*)a.bias_ws,
                         a.splits * a.batch, a.M, dbias, bt);
    // the split-K slices of every class summed in place into slice 0 (the GEMM's vectorized fixed-order reducer),
    // then the 16 class partials of each 3x3 tap combined
    GemmArgs r = a;
    r.C = workspace; r.ldc = a.N; r.sC = (long long)a.splits * a.M * a.N;
    r.alpha = 1.f; r.beta = 0.f; r.bias = nullptr; r.res = nullptr;
    const int rrc = gemm_finish(r, st);
    if (rrc) return rrc;
    const long long tot = (long long)cout * cin;
    hipLaunchKernelGGL(ups_wgrad_combine_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st,
                       (const float*)workspace, (long long)a.splits * a.M * a.N, cout, cin, dw, bt);
    const int rc = launch_status();
    if (rc) return rc;
  }
  return MVAE_OK;
}

size_t mvae_conv2d_wgrad_upsample_workspace_bytes(int nb, int h, int wd, int cin, int cout) {
  GemmArgs a{};
  ups_wgrad_shape(a, nb, h, wd, cin, cout);
  size_t b = 0;
  for (int big = 0; big < 2; ++big) {
    set_splits(a, choose_splits(a, choose_tile(a, big != 0, true)));
    b = std::max(b, ups_part_bytes(a));
  }
  return ((b + 255) & ~(size_t)255) + (size_t)4 * MAX_SPLITS * a.M * sizeof(float) + 256;
}

size_t mvae_conv2d_wgrad_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  GemmArgs a{};
  wgrad_shape(a, nb, cin, cout, kh, kw, ho, wo);
  set_splits(a, choose_splits(a, choose_tile(a, true, true)));
  size_t b1 = splitk_ws_bytes(a);
  set_splits(a, choose_splits(a, choose_tile(a, false, true)));
  return ((std::max(b1, splitk_ws_bytes(a)) + 255) & ~(size_t)255) + (size_t)MAX_SPLITS * a.M * sizeof(float) + 256;
}

}  // extern "C"
