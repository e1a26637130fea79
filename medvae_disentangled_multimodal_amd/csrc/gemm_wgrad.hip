// Weight-gradient entry point of the implicit-GEMM convolution (deterministic split-K over pixels).
#include "gemm_core.h"

namespace mvae {
// dbias[m] = beta*dbias[m] + sum over splits (fixed order) of the per-split row sums
__global__ void bias_reduce_kernel(const float* __restrict__ part, int splits, int m, float* dbias, float beta) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += part[(long long)z * m + i];
  dbias[i] = (beta != 0.f ? beta * dbias[i] : 0.f) + s;
}
}  // namespace mvae

using namespace mvae;

static void wgrad_shape(GemmArgs& a, int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  a.M = cout; a.N = kh * kw * cin; a.K = nb * ho * wo; a.batch = 1;
}

extern "C" {

// dw[cout][r][s][cin] = beta*dw + sum_pixels dy[pix][cout] * x[src(pix, r, s)][cin]   (modes 0 / 1)
int mvae_conv2d_wgrad_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb, int h,
                           int wd, int cin, int cout, int kh, int kw, int stride, int pad_t,
                           int pad_l, int ho, int wo, int mode, float* workspace,
                           size_t workspace_bytes, void* stream) {
  if (mode != 0 && mode != 1) { set_error("wgrad: mode must be 0 or 1"); return MVAE_EINVAL; }
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
    a.A = dy + (long long)b0 * (out_img / 4); a.lda = cout;
    a.B = x + (long long)b0 * (in_img / 4);
    a.C = dw; a.ldc = a.N; a.alpha = 1.f; a.beta = b0 == 0 ? beta : 1.f;
    a.a_bytes = (unsigned)(out_img * n); a.b_bytes = (unsigned)(in_img * n);
    a.c_bytes = (unsigned)((long long)a.M * a.N * 4);
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
    set_gather_magic(a);
    a.stride = stride; a.pad_t = pad_t; a.pad_l = pad_l;
    const int cfg = choose_tile(a, va && vb, workspace != nullptr);
    const size_t bias_bytes = dbias ? ((size_t)64 * a.M * sizeof(float) + 256) : 0;
    if (dbias && workspace_bytes < bias_bytes) { set_error("wgrad: workspace too small"); return MVAE_EWORKSPACE; }
    plan_splits(a, cfg, workspace, workspace_bytes - bias_bytes);
    // bias partials live after the split-K partials
    a.bias_ws = dbias ? (float*)((char*)workspace + ((splitk_ws_bytes(a) + 255) & ~(size_t)255)) : nullptr;
    if (mode == 0) {
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
    if (dbias)
      hipLaunchKernelGGL(bias_reduce_kernel, dim3(cdiv(a.M, 256)), dim3(256), 0, st, (const float*)a.bias_ws,
                         a.splits, a.M, dbias, b0 == 0 ? beta : 1.f);
    const int rc = gemm_finish(a, st);
    if (rc) return rc;
  }
  return MVAE_OK;
}

size_t mvae_conv2d_wgrad_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  GemmArgs a{};
  wgrad_shape(a, nb, cin, cout, kh, kw, ho, wo);
  set_splits(a, choose_splits(a, choose_tile(a, true, true)));
  size_t b1 = splitk_ws_bytes(a);
  set_splits(a, choose_splits(a, choose_tile(a, false, true)));
  return ((std::max(b1, splitk_ws_bytes(a)) + 255) & ~(size_t)255) + (size_t)64 * a.M * sizeof(float) + 256;
}

}  // extern "C"
