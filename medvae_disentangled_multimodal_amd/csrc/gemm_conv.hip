// Implicit-GEMM convolution entry point (forward, and input-gradient via the transposed gather).
#include "gemm_core.h"

using namespace mvae;

// wc[ci][t][co] = wt[ci][tap[t]][co] for the nt taps of one parity class (wt = [cin][rs][cout])
__global__ void __launch_bounds__(256) tap_select_kernel(const float* __restrict__ wt, float* __restrict__ wc, int cin,
                                                         int rs, int cout, int nt, int4 taps) {
  const long long tot = (long long)cin * nt * cout;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(e % cout);
    const long long r = e / cout;
    const int t = (int)(r % nt), ci = (int)(r / nt);
    const int tap = t == 0 ? taps.x : t == 1 ? taps.y : t == 2 ? taps.z : taps.w;
    wc[e] = wt[((long long)ci * rs + tap) * cout + co];
  }
}
__global__ void __launch_bounds__(256) tap_select_bf16_kernel(const __bf16* __restrict__ wt, __bf16* __restrict__ wc,
                                                              int cin, int rs, int cout, int nt, int4 taps) {
  const long long tot = (long long)cin * nt * cout;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < tot; e += (long long)gridDim.x * blockDim.x) {
    const int co = (int)(e % cout);
    const long long r = e / cout;
    const int t = (int)(r % nt), ci = (int)(r / nt);
    const int tap = t == 0 ? taps.x : t == 1 ? taps.y : t == 2 ? taps.z : taps.w;
    wc[e] = wt[((long long)ci * rs + tap) * cout + co];
  }
}

static bool kperm_enabled() {  // MVAE_NO_KPERM=1: reference K order (A/B experiments)
  static const bool on = getenv("MVAE_NO_KPERM") == nullptr;
  return on;
}

extern "C" {

// Implicit-GEMM convolution over NHWC activations and KRSC ([Cout][R][S][Cin]) weights.
//   mode 0: y = conv(x, stride, pad_t/pad_l; zero padding outside [0,H)x[0,W))
//   mode 1: y = conv(upsample_nearest_x2(x), stride 1, pad_t/pad_l)
//   mode 2: transposed gather: y[oh] += x[(oh + pad - r)/stride] * w[r] (dgrad of a strided conv;
//           stride must be a power of two)
// y[n][ho][wo][cout] = sum + bias[cout] + residual[n][ho][wo][cout]
// GroupNorm backward link of an input-gradient conv (GemmArgs::gnb_part): the conv's input was
// silu?(GroupNorm(x)) with these saved statistics and affine parameters
struct GnBwdLink {
  const float* x;
  const float *mean, *rstd, *gamma, *beta;
  int groups, silu;
  double* part;
};
static int conv2d_impl(const float* x, const float* w, const float* bias, const float* residual, float* y, int nb,
                       int h, int wd, int cin, int cout, int kh, int kw, int stride, int pad_t, int pad_l, int ho,
                       int wo, int mode, double* gn_part, void* stream, const GnBwdLink* gnb = nullptr,
                       float* ws = nullptr, size_t ws_bytes = 0);

int mvae_conv2d_nhwc(const float* x, const float* w, const float* bias, const float* residual,
                     float* y, int nb, int h, int wd, int cin, int cout, int kh, int kw,
                     int stride, int pad_t, int pad_l, int ho, int wo, int mode, void* stream) {
  return conv2d_impl(x, w, bias, residual, y, nb, h, wd, cin, cout, kh, kw, stride, pad_t, pad_l, ho, wo, mode,
                     nullptr, stream);
}

// mvae_conv2d_nhwc with a split-K workspace: a launch whose tiles leave most of the 256 CUs idle for a partial
// round (small spatial sizes at wide channels) may split K over `workspace` (fp32 partials, reduced in a fixed
// order with bias / residual). Size from mvae_conv2d_split_workspace_bytes; a smaller workspace means fewer splits.
int mvae_conv2d_ws_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y, int nb,
                        int h, int wd, int cin, int cout, int kh, int kw, int stride, int pad_t, int pad_l, int ho,
                        int wo, int mode, float* workspace, size_t workspace_bytes, void* stream) {
  return conv2d_impl(x, w, bias, residual, y, nb, h, wd, cin, cout, kh, kw, stride, pad_t, pad_l, ho, wo, mode,
                     nullptr, stream, nullptr, workspace, workspace_bytes);
}

// Workspace bytes mvae_conv2d_ws_nhwc would use for this geometry (0: the launch stays unsplit).
size_t mvae_conv2d_split_workspace_bytes(int nb, int cin, int cout, int kh, int kw, int ho, int wo) {
  if (nb <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || ho <= 0 || wo <= 0 || cin % 4) return 0;
  GemmArgs a{};
  a.M = nb * ho * wo; a.N = cout; a.K = kh * kw * cin; a.batch = 1; a.splits = 1; a.k_split = a.K;
  const int cfg = choose_tile(a, true, false);
  int s = 1;
  const int c2 = conv_split_cfg(a, cfg, (size_t)1 << 40, &s);
  if (c2 < 0) return 0;
  set_splits(a, s);
  return splitk_ws_bytes(a);
}

// mvae_conv2d_nhwc that also emits the GroupNorm statistics of y for the Normalize that follows
// (gn_part: [nb*ho*wo/32][cout/4][2] fp64 {sum, sum of squares}); needs ho*wo % 32 == 0, cout % 4 == 0,
// 16-B aligned y / residual / bias.
int mvae_conv2d_gnstats_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                             int nb, int h, int wd, int cin, int cout, int kh, int kw, int stride, int pad_t,
                             int pad_l, int ho, int wo, int mode, double* gn_part, void* stream) {
  if (gn_part == nullptr || (ho * wo) % 32 != 0 || cout % 4 != 0 || !al16(y) || (residual && !al16(residual)) ||
      (bias && !al16(bias)) || vec_epi_disabled()) {
    set_error("conv2d_gnstats: needs ho*wo %% 32 == 0, cout %% 4 == 0, 16-B aligned outputs");
    return MVAE_EINVAL;
  }
  return conv2d_impl(x, w, bias, residual, y, nb, h, wd, cin, cout, kh, kw, stride, pad_t, pad_l, ho, wo, mode,
                     gn_part, stream);
}

// Input gradient of a stride-1 conv (mode 2 of mvae_conv2d_nhwc: dy [nb][ho][wo][cout] -> dx [nb][h][wd][cin],
// wt = [cin][kh][kw][cout]) whose input was y = silu?(GroupNorm(gn_x)) (ResnetBlock norm1/norm2 -> conv,
// encoder_decoder.py:141-163; norm_out -> conv_out): the epilogue also emits the GroupNorm backward partials
// part = [nb*h*wd/32][cin][2] fp64 {sum dyn, sum dyn*xhat} (dyn = dx * silu'(.)) for
// mvae_group_norm_bwd_part_nhwc. No dropout between the GroupNorm and the conv. Needs h*wd % 32 == 0,
// (cin / groups) % 4 == 0, 16-B aligned dx and gn_x.
int mvae_conv2d_dgrad_gnbwd_nhwc(const float* dy, const float* wt, float* dx, int nb, int ho, int wo, int cout,
                                 int cin, int kh, int kw, int pad_t, int pad_l, int h, int wd, int w_split,
                                 const float* gn_x, const float* mean, const float* rstd, const float* gamma,
                                 const float* beta, int groups, int silu, double* part, void* stream) {
  if (part == nullptr || gn_x == nullptr || mean == nullptr || rstd == nullptr || gamma == nullptr ||
      beta == nullptr || groups <= 0 || cin % groups || (cin / groups) % 4 || (h * wd) % 32 || !al16(dx) ||
      !al16(gn_x) || vec_epi_disabled()) {
    set_error("conv2d_dgrad_gnbwd: needs h*w %% 32 == 0, channels per group %% 4 == 0, 16-B aligned dx / x");
    return MVAE_EINVAL;
  }
  if (cout % 4 || !al16(dy) || !al16(wt)) {
    set_error("conv2d_dgrad_gnbwd: needs the vector (16-B) operand path (cout %% 4 == 0, aligned dy / wt)");
    return MVAE_EINVAL;
  }
  const GnBwdLink link{gn_x, mean, rstd, gamma, beta, groups, silu, part};
  return conv2d_impl(dy, wt, nullptr, nullptr, dx, nb, ho, wo, cout, cin, kh, kw, 1, pad_t, pad_l, h, wd,
                     2 | ((w_split & 1) ? MVAE_CONV_WSPLIT : 0) | ((w_split & 2) ? MVAE_CONV_XSPLIT : 0), nullptr,
                     stream, &link);
}

}  // extern "C"

// Wave-quantization tail: a conv GEMM whose tiles fill k whole rounds of the chip's resident slots (256 CUs x tiles
// per CU) plus a sliver of one more runs that last round on a few CUs for a whole tile time -- c2's 28x28x128 passes
// at B = 256 are 784 tiles of 256x128 = 3.06 rounds, measured 250 us against 190 us at B = 250 (tools/quant_probe.py).
// Such a batch is launched as the images that fit the k rounds, then the remaining images on their own (the cost model
// gives them small tiles spread over the chip). Returns the image count of the first launch (nb: no split).
// MVAE_NO_TAIL_SPLIT=1 turns it off.
static int tail_split_images(int nb, long long hw, int n_cols, int k, bool v) {
  static const bool off = getenv("MVAE_NO_TAIL_SPLIT") != nullptr;
  if (off || nb < 2) return nb;
  GemmArgs t{};
  t.M = (int)std::min<long long>((long long)nb * hw, 1LL << 30); t.N = n_cols; t.K = k; t.batch = 1;
  const int cfg = choose_tile(t, v, false);
  if (cfg < T256x256 || cfg > T64x64) return nb;
  const long long slots = 256LL * resident_of(cfg), tiles = tiles_of(cfg, t);
  const long long full = tiles / slots, rem = tiles - full * slots;
  if (full < 1 || rem == 0 || rem * 2 >= slots) return nb;
  const long long tn = (n_cols + tile_n_of(cfg) - 1) / tile_n_of(cfg);
  const long long nm = (full * slots / tn) * tile_m_of(cfg) / hw;
  return (nm >= 1 && nm < nb) ? (int)nm : nb;
}

static int conv2d_impl(const float* x, const float* w, const float* bias, const float* residual, float* y, int nb,
                       int h, int wd, int cin, int cout, int kh, int kw, int stride, int pad_t, int pad_l, int ho,
                       int wo, int mode, double* gn_part, void* stream, const GnBwdLink* gnb, float* ws,
                       size_t ws_bytes) {
  const bool presplit = (mode & MVAE_CONV_WSPLIT) != 0;
  const bool xsplit = (mode & MVAE_CONV_XSPLIT) != 0;
  const bool pk = (mode & MVAE_CONV_BF16) != 0;      // packed bf16 x (dy) and w: PREC 4
  const bool pln = (mode & MVAE_CONV_PLANAR) != 0;   // planar 3xBF16 x (dy) and w: PREC 5
  const bool bf = pk || pln;                         // LDS-DMA staged operands (bf16 element offsets)
  mode &= ~(MVAE_CONV_WSPLIT | MVAE_CONV_XSPLIT | MVAE_CONV_BF16 | MVAE_CONV_PLANAR);
  if (bf && ((pk && pln) || presplit || xsplit || mode == 1 || cin % 8 || !al16(x) || !al16(w) || kh * kw > 32 ||
             math_mode() != (pln ? MATH_3XBF16 : MATH_BF16) ||
             (pln && (long long)nb * h * wd * cin * 2 >= (1LL << 32)))) {
    set_error("conv2d: DMA-staged operands need the matching math mode (packed bf16: bf16, planar: 3xBF16), mode 0 "
              "or 2, cin %% 8 == 0, <= 32 taps, 16-B aligned x, w, a hi plane < 4 GiB");
    return MVAE_EINVAL;
  }
  if (xsplit && mode == 1) { set_error("conv2d: a pre-split input needs mode 0 or 2"); return MVAE_EINVAL; }
  if ((xsplit || presplit) && split_forbidden()) {
    set_error("conv2d: pre-split operands are not allowed in the exact-fp32 math mode");
    return MVAE_EINVAL;
  }
  if (nb <= 0 || h <= 0 || wd <= 0 || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || ho <= 0 || wo <= 0 ||
      stride <= 0 || mode < 0 || mode > 2 || (mode == 2 && (stride & (stride - 1)))) {
    set_error("conv2d: bad geometry");
    return MVAE_EINVAL;
  }
  const long long in_img = (long long)h * wd * cin * 4, out_img = (long long)ho * wo * cout * 4;
  const long long wbytes = (long long)cout * kh * kw * cin * 4;
  if (std::max(in_img, out_img) > MAX_DESC_BYTES || wbytes > MAX_DESC_BYTES) {
    set_error("conv2d: one image exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  // samples per launch so that every operand fits one buffer descriptor
  const int chunk = (int)std::min<long long>(nb, MAX_DESC_BYTES / std::max(in_img, out_img));
  hipStream_t st = (hipStream_t)stream;
  // the vector gather keeps one bit per filter tap (LoadConvA): kernels of more than 32 taps take the scalar path
  const bool v = (cin % 4 == 0) && al16(x) && al16(w) && kh * kw <= 32;
  if ((presplit || xsplit) && !v) {
    set_error("conv2d: pre-split operands need cin %% 4 == 0 and 16-B aligned x, w");
    return MVAE_EINVAL;
  }
  int shift = 0;
  while ((1 << shift) < stride) ++shift;
  const int n_main = (!bf && nb <= chunk) ? tail_split_images(nb, (long long)ho * wo, cout, kh * kw * cin, v) : nb;
  for (int b0 = 0, n_ = 0; b0 < nb; b0 += n_) {
    n_ = (b0 == 0 && n_main < nb) ? n_main : std::min(chunk, nb - b0);
    const int n = n_;
    GemmArgs a{};
    a.M = n * ho * wo; a.N = cout; a.K = kh * kw * cin; a.batch = 1; a.splits = 1; a.k_split = a.K;
    a.A = bf ? (const float*)((const __bf16*)x + (long long)b0 * (in_img / 4)) : x + (long long)b0 * (in_img / 4);
    a.B = w; a.ldb = a.K;
    a.C = y + (long long)b0 * (out_img / 4); a.ldc = cout; a.bias = bias;
    a.res = residual ? residual + (long long)b0 * (out_img / 4) : nullptr; a.ldr = cout;
    a.alpha = 1.f; a.beta = 0.f;
    a.a_bytes = (unsigned)(in_img * n / (bf ? 2 : 1)); a.b_bytes = (unsigned)(wbytes / (bf ? 2 : 1));
    if (pln) {  // lo planes: one whole hi plane after the hi plane
      a.a_lo = (unsigned)(in_img / 2 * nb);
      a.b_lo = (unsigned)(wbytes / 2);
    }
    a.c_bytes = (unsigned)(out_img * n); a.r_bytes = a.c_bytes;
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
    a.perm_rs = (v && cin % (bf ? DBK : BK) == 0 && kh * kw > 1 && kperm_enabled()) ? kh * kw : 1;
    set_gather_magic(a);
    a.stride = stride; a.stride_shift = shift; a.pad_t = pad_t; a.pad_l = pad_l;
    a.gn_part = gn_part ? gn_part + (long long)b0 * (ho * wo / 32) * (cout / 4) * 2 : nullptr;
    if (gnb) {
      const int hw = ho * wo;
      a.gnb_part = gnb->part + (long long)b0 * (hw / 32) * cout * 2;
      a.gnb_x = gnb->x + (long long)b0 * (out_img / 4);
      a.gnb_mean = gnb->mean + (long long)b0 * gnb->groups;
      a.gnb_rstd = gnb->rstd + (long long)b0 * gnb->groups;
      a.gnb_gamma = gnb->gamma; a.gnb_beta = gnb->beta;
      a.gnb_hw = hw; a.gnb_G = gnb->groups; a.gnb_cpg = cout / gnb->groups; a.gnb_silu = gnb->silu;
    }
    int cfg = choose_tile(a, v, false);
    if (ws != nullptr && gn_part == nullptr && gnb == nullptr && v) {  // under-filled launch: split K (conv_split_cfg)
      int s = 1;
      const int c2 = conv_split_cfg(a, cfg, ws_bytes, &s);
      if (c2 >= 0) {
        cfg = c2;
        set_splits(a, s);
        a.ws = ws;
      }
    }
    if ((gn_part || gnb) && !v) {
      set_error("conv2d_gnstats: needs the vector (16-B) operand path");
      return MVAE_EINVAL;
    }
    if (bf) {  // DMA-staged x (dy) and weights: LDS-DMA main loop
      conv_dma(mode == 0 ? A_CONV_FWD : A_CONV_DGRAD, a, st, cfg, pln ? 5 : 4);
    } else if (xsplit && mode == 2) {  // dy (the gathered operand of the input gradient) holds split4_bf16 groups
      if (presplit) launch_big<A_CONV_DGRAD_SPLIT, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else launch_big<A_CONV_DGRAD_SPLIT, 4, B_ROWK, 4>(a, st, cfg);
    } else if (xsplit) {  // x (and w) hold split4_bf16 groups: no staging split at all
      if (presplit) launch_big<A_CONV_FWD_SPLIT, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else launch_big<A_CONV_FWD_SPLIT, 4, B_ROWK, 4>(a, st, cfg);
    } else if (presplit) {  // w holds split4_bf16 groups (MVAE_CONV_WSPLIT): no staging split for B
      if (mode == 0) launch_big<A_CONV_FWD, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else if (mode == 1) launch_big<A_CONV_UPS, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else launch_big<A_CONV_DGRAD, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
    } else if (mode == 0) {
      if (v) launch_big<A_CONV_FWD, 4, B_ROWK, 4>(a, st, cfg);
      else launch_small<A_CONV_FWD, 1, B_ROWK, 1>(a, st, cfg);
    } else if (mode == 1) {
      if (v) launch_big<A_CONV_UPS, 4, B_ROWK, 4>(a, st, cfg);
      else launch_small<A_CONV_UPS, 1, B_ROWK, 1>(a, st, cfg);
    } else {
      if (v) launch_big<A_CONV_DGRAD, 4, B_ROWK, 4>(a, st, cfg);
      else launch_small<A_CONV_DGRAD, 1, B_ROWK, 1>(a, st, cfg);
    }
    const int rc = gemm_finish(a, st);
    if (rc) return rc;
  }
  return MVAE_OK;
}

extern "C" {

// Input gradient of a stride-2 convolution (Downsample, encoder_decoder.py:184-188) by parity class:
// dx pixel (2m+p, 2j+q) only receives the taps r with r = p + pad_t (mod 2) (and likewise s), so each
// of the 4 classes is a dense stride-1 conv of dY with its own <= 2x2 taps (9 taps over the 4 classes)
// instead of the 9-tap transposed gather at every dx pixel, 3/4 of whose taps fall in stride holes.
// wt = [cin][kh][kw][cout] (mvae_conv_weight_transpose); needs even h, w; workspace >= 4*kh*kw*cin*cout B.
int mvae_conv2d_dgrad_stride2_nhwc(const float* dy, const float* wt, float* dx, int nb, int h, int wd, int cin,
                                   int cout, int kh, int kw, int pad_t, int pad_l, int ho, int wo, int w_split,
                                   float* workspace, size_t workspace_bytes, void* stream) {
  if (nb <= 0 || h <= 0 || wd <= 0 || (h & 1) || (wd & 1) || cin <= 0 || cout <= 0 || kh <= 0 || kw <= 0 ||
      kh > 4 || kw > 4 || ho <= 0 || wo <= 0) {
    set_error("dgrad_stride2: bad geometry (needs even h, w and kernel <= 4)");
    return MVAE_EINVAL;
  }
  if (workspace == nullptr || workspace_bytes < (size_t)kh * kw * cin * cout * 4) {
    set_error("dgrad_stride2: workspace too small");
    return MVAE_EWORKSPACE;
  }
  const long long in_img = (long long)ho * wo * cout * 4, out_img = (long long)h * wd * cin * 4;
  if (std::max(in_img, out_img) > MAX_DESC_BYTES || (long long)kh * kw * cin * cout * 4 > MAX_DESC_BYTES) {
    set_error("dgrad_stride2: one image exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  const int chunk = (int)std::min<long long>(nb, MAX_DESC_BYTES / std::max(in_img, out_img));
  hipStream_t st = (hipStream_t)stream;
  const int hc = h / 2, wc = wd / 2;
  // w_split 4: dy and wt are packed bf16 (bf16-mixed mode); 8: planar 3xBF16 (LDS-DMA main loop)
  const bool pln = w_split == 8;
  const bool bf = w_split == 4 || pln;
  if (bf && (cout % 8 || !al16(dy) || !al16(wt) || math_mode() != (pln ? MATH_3XBF16 : MATH_BF16))) {
    set_error("dgrad_stride2: DMA-staged operands need the matching math mode, cout %% 8 == 0, aligned dy / wt");
    return MVAE_EINVAL;
  }
  if (bf && workspace_bytes < (size_t)kh * kw * cin * cout * (pln ? 4 : 2)) {
    set_error("dgrad_stride2: workspace too small");
    return MVAE_EWORKSPACE;
  }
  const long long wt_plane = (long long)cin * kh * kw * cout;  // planar wt: lo plane this many elements later
  float* wcls = workspace;
  bool empty_class = false;  // a kernel too small to reach every parity: those dx pixels are 0
  for (int p = 0; p < 2; ++p) {
    bool hr = false, hs = false;
    for (int r = 0; r < kh; ++r) hr |= ((p + pad_t - r) & 1) == 0;
    for (int s_ = 0; s_ < kw; ++s_) hs |= ((p + pad_l - s_) & 1) == 0;
    empty_class |= !hr || !hs;
  }
  if (empty_class && hipMemsetAsync(dx, 0, (size_t)nb * out_img, st) != hipSuccess) return launch_status();
  for (int cls = 0; cls < 4; ++cls) {
    const int p = cls >> 1, q = cls & 1;
    // taps of this class in increasing dY row: r with (p + pad_t - r) even, descending r
    int rl[4], sl[4], nr = 0, ns = 0;
    for (int r = kh - 1; r >= 0; --r)
      if (((p + pad_t - r) & 1) == 0) rl[nr++] = r;
    for (int s_ = kw - 1; s_ >= 0; --s_)
      if (((q + pad_l - s_) & 1) == 0) sl[ns++] = s_;
    const int nt = nr * ns;
    if (nt == 0) continue;  // zero-filled above
    int tp[4] = {0, 0, 0, 0};
    for (int a = 0; a < nr; ++a)
      for (int b = 0; b < ns; ++b) tp[a * ns + b] = rl[a] * kw + sl[b];
    if (nt > 4) { set_error("dgrad_stride2: class with more than 4 taps"); return MVAE_EINVAL; }
    const long long tot = (long long)cin * nt * cout;
    if (bf) {
      for (int pl = 0; pl < (pln ? 2 : 1); ++pl)  // planar: the class's hi block, then its lo block
        hipLaunchKernelGGL(tap_select_bf16_kernel, dim3((unsigned)std::min<long long>((tot + 255) / 256, 8192)),
                           dim3(256), 0, st, (const __bf16*)wt + pl * wt_plane, (__bf16*)wcls + pl * tot, cin, kh * kw,
                           cout, nt, make_int4(tp[0], tp[1], tp[2], tp[3]));
    }
    else
      hipLaunchKernelGGL(tap_select_kernel, dim3((unsigned)std::min<long long>((tot + 255) / 256, 8192)), dim3(256), 0,
                         st, wt, wcls, cin, kh * kw, cout, nt, make_int4(tp[0], tp[1], tp[2], tp[3]));
    // dY row of class row m for tap a: m - pt + a with pt = (r_max - p - pad_t) / 2
    const int pt = (rl[0] - p - pad_t) / 2, pl = (sl[0] - q - pad_l) / 2;
    const bool v = (cout % 4 == 0) && al16(dy) && al16(wcls);
    if (w_split && !v) { set_error("dgrad_stride2: pre-split operands need cout %% 4 == 0"); return MVAE_EINVAL; }
    if (w_split && split_forbidden()) { set_error("dgrad_stride2: pre-split operands in exact-fp32 mode"); return MVAE_EINVAL; }
    for (int b0 = 0; b0 < nb; b0 += chunk) {
      const int n = std::min(chunk, nb - b0);
      GemmArgs a{};
      a.M = n * hc * wc; a.N = cin; a.K = nt * cout; a.batch = 1; a.splits = 1; a.k_split = a.K;
      a.A = bf ? (const float*)((const __bf16*)dy + (long long)b0 * (in_img / 4)) : dy + (long long)b0 * (in_img / 4);
      a.B = wcls; a.ldb = a.K;
      a.C = dx + (long long)b0 * (out_img / 4); a.ldc = cin;
      a.alpha = 1.f; a.beta = 0.f;
      a.a_bytes = (unsigned)(in_img * n / (bf ? 2 : 1)); a.b_bytes = (unsigned)(tot * (bf ? 2 : 4));
      if (pln) {
        a.a_lo = (unsigned)(in_img / 2 * nb);
        a.b_lo = (unsigned)(tot * 2);
      }
      a.c_bytes = (unsigned)(out_img * n); a.r_bytes = 0;
      a.H = ho; a.W = wo; a.Cx = cout; a.Ho = hc; a.Wo = wc; a.R = nr; a.S = ns;
      a.perm_rs = (v && cout % (bf ? DBK : BK) == 0 && nt > 1 && kperm_enabled()) ? nt : 1;
      set_gather_magic(a);
      a.stride = 1; a.stride_shift = 0; a.pad_t = pt; a.pad_l = pl;
      a.sub_w2 = wd; a.sub_par = cls; a.out_remap = 1;
      const int cfg = choose_tile(a, v, false);
      if (bf) conv_dma(A_CONV_FWD, a, st, cfg, pln ? 5 : 4);
      else if ((w_split & 3) == 3) launch_big<A_CONV_FWD_SPLIT, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else if (w_split & 2) launch_big<A_CONV_FWD_SPLIT, 4, B_ROWK, 4>(a, st, cfg);
      else if (w_split) launch_big<A_CONV_FWD, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
      else if (v) launch_big<A_CONV_FWD, 4, B_ROWK, 4>(a, st, cfg);
      else launch_small<A_CONV_FWD, 1, B_ROWK, 1>(a, st, cfg);
      const int rc = gemm_finish(a, st);
      if (rc) return rc;
    }
    wcls = bf ? (float*)((__bf16*)wcls + (pln ? 2 : 1) * tot) : wcls + tot;
  }
  return MVAE_OK;
}

// Sub-pixel form of Upsample's convolution (nearest x2 then 3x3, stride 1, pad 1;
// encoder_decoder.py:194-209): output parity class (ph, pw) -- pixels (2i+ph, 2j+pw) -- is a 2x2 conv of
// the LOW-resolution input x with the tap-summed weights w4[2*ph+pw] ([cout][2][2][cin], from
// mvae_conv_weight_upsample_fwd) and padding (1-ph, 1-pw): 4 taps per output pixel instead of 9 and no
// upsampled intermediate. The 4 classes are one batched launch whose epilogue writes interleaved rows.
// y [nb][2h][2wd][cout] = conv3x3(upsample2(x)) + bias + residual
int mvae_conv2d_upsample_nhwc(const float* x, const float* w4, const float* bias, const float* residual, float* y,
                              int nb, int h, int wd, int cin, int cout, int w_split, void* stream) {
  if (nb <= 0 || h <= 0 || wd <= 0 || cin <= 0 || cout <= 0) {
    set_error("conv2d_upsample: bad geometry");
    return MVAE_EINVAL;
  }
  const long long in_img = (long long)h * wd * cin * 4, out_img = 4LL * h * wd * cout * 4;
  const long long wbytes = 4LL * cout * 4 * cin * 4;
  if (std::max(in_img, out_img) > MAX_DESC_BYTES || wbytes > MAX_DESC_BYTES) {
    set_error("conv2d_upsample: one image exceeds 4 GiB");
    return MVAE_EINVAL;
  }
  const int chunk = (int)std::min<long long>(nb, MAX_DESC_BYTES / std::max(in_img, out_img));
  hipStream_t st = (hipStream_t)stream;
  const bool v = (cin % 4 == 0) && al16(x) && al16(w4);
  // w_split 2: x and w4 are packed bf16 (bf16-mixed mode); 3: planar 3xBF16 (LDS-DMA main loop)
  const bool pln = w_split == 3;
  const bool bf = w_split == 2 || pln;
  if (bf && (cin % 8 || !v || math_mode() != (pln ? MATH_3XBF16 : MATH_BF16))) {
    set_error("conv2d_upsample: DMA-staged operands need the matching math mode, cin %% 8 == 0, aligned x / w4");
    return MVAE_EINVAL;
  }
  if (w_split && !v) { set_error("conv2d_upsample: pre-split weights need cin %% 4 == 0"); return MVAE_EINVAL; }
  if (w_split && split_forbidden()) { set_error("conv2d_upsample: pre-split weights in exact-fp32 mode"); return MVAE_EINVAL; }
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int n = std::min(chunk, nb - b0);
    GemmArgs a{};
    a.M = n * h * wd; a.N = cout; a.K = 4 * cin; a.batch = 4; a.splits = 1; a.k_split = a.K;
    a.A = bf ? (const float*)((const __bf16*)x + (long long)b0 * (in_img / 4)) : x + (long long)b0 * (in_img / 4);
    a.sA = 0;
    a.B = w4; a.ldb = a.K; a.sB = (long long)cout * a.K;
    a.C = y + (long long)b0 * (out_img / 4); a.ldc = cout; a.sC = 0; a.bias = bias;
    a.res = residual ? residual + (long long)b0 * (out_img / 4) : nullptr; a.ldr = cout; a.sR = 0;
    a.alpha = 1.f; a.beta = 0.f;
    a.a_bytes = (unsigned)(in_img * n / (bf ? 2 : 1)); a.b_bytes = (unsigned)(wbytes / 4 / (bf ? 2 : 1));
    if (pln) {
      a.a_lo = (unsigned)(in_img / 2 * nb);
      a.b_lo = (unsigned)(wbytes / 2);
    }
    a.c_bytes = (unsigned)(out_img * n); a.r_bytes = a.c_bytes;
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = h; a.Wo = wd; a.R = 2; a.S = 2;
    a.perm_rs = (v && cin % (bf ? DBK : BK) == 0 && kperm_enabled()) ? 4 : 1;
    set_gather_magic(a);
    a.stride = 1; a.stride_shift = 0; a.pad_t = 1; a.pad_l = 1;
    a.sub_w2 = 2 * wd; a.sub_par = 0; a.out_remap = 1;
    const int cfg = choose_tile(a, v, false);
    if (bf) conv_dma(A_CONV_SUBPIX, a, st, cfg, pln ? 5 : 4);
    else if (w_split) launch_big<A_CONV_SUBPIX, 4, B_ROWK_SPLIT, 4>(a, st, cfg);
    else if (v) launch_big<A_CONV_SUBPIX, 4, B_ROWK, 4>(a, st, cfg);
    else launch_small<A_CONV_SUBPIX, 1, B_ROWK, 1>(a, st, cfg);
    const int rc = gemm_finish(a, st);
    if (rc) return rc;
  }
  return MVAE_OK;
}

}  // extern "C"
