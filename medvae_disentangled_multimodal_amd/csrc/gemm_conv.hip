// Implicit-GEMM convolution entry point (forward, and input-gradient via the transposed gather).
#include "gemm_core.h"

using namespace mvae;

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
int mvae_conv2d_nhwc(const float* x, const float* w, const float* bias, const float* residual,
                     float* y, int nb, int h, int wd, int cin, int cout, int kh, int kw,
                     int stride, int pad_t, int pad_l, int ho, int wo, int mode, void* stream) {
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
  const bool v = (cin % 4 == 0) && al16(x) && al16(w);
  int shift = 0;
  while ((1 << shift) < stride) ++shift;
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int n = std::min(chunk, nb - b0);
    GemmArgs a{};
    a.M = n * ho * wo; a.N = cout; a.K = kh * kw * cin; a.batch = 1; a.splits = 1; a.k_split = a.K;
    a.A = x + (long long)b0 * (in_img / 4);
    a.B = w; a.ldb = a.K;
    a.C = y + (long long)b0 * (out_img / 4); a.ldc = cout; a.bias = bias;
    a.res = residual ? residual + (long long)b0 * (out_img / 4) : nullptr; a.ldr = cout;
    a.alpha = 1.f; a.beta = 0.f;
    a.a_bytes = (unsigned)(in_img * n); a.b_bytes = (unsigned)wbytes;
    a.c_bytes = (unsigned)(out_img * n); a.r_bytes = a.c_bytes;
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = ho; a.Wo = wo; a.R = kh; a.S = kw;
    a.perm_rs = (v && cin % BK == 0 && kh * kw > 1 && kperm_enabled()) ? kh * kw : 1;
    set_gather_magic(a);
    a.stride = stride; a.stride_shift = shift; a.pad_t = pad_t; a.pad_l = pad_l;
    const int cfg = choose_tile(a, v, false);
    if (mode == 0) {
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

// Sub-pixel form of Upsample's convolution (nearest x2 then 3x3, stride 1, pad 1;
// encoder_decoder.py:194-209): output parity class (ph, pw) -- pixels (2i+ph, 2j+pw) -- is a 2x2 conv of
// the LOW-resolution input x with the tap-summed weights w4[2*ph+pw] ([cout][2][2][cin], from
// mvae_conv_weight_upsample_fwd) and padding (1-ph, 1-pw): 4 taps per output pixel instead of 9 and no
// upsampled intermediate. The 4 classes are one batched launch whose epilogue writes interleaved rows.
// y [nb][2h][2wd][cout] = conv3x3(upsample2(x)) + bias + residual
int mvae_conv2d_upsample_nhwc(const float* x, const float* w4, const float* bias, const float* residual, float* y,
                              int nb, int h, int wd, int cin, int cout, void* stream) {
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
  for (int b0 = 0; b0 < nb; b0 += chunk) {
    const int n = std::min(chunk, nb - b0);
    GemmArgs a{};
    a.M = n * h * wd; a.N = cout; a.K = 4 * cin; a.batch = 4; a.splits = 1; a.k_split = a.K;
    a.A = x + (long long)b0 * (in_img / 4); a.sA = 0;
    a.B = w4; a.ldb = a.K; a.sB = (long long)cout * a.K;
    a.C = y + (long long)b0 * (out_img / 4); a.ldc = cout; a.sC = 0; a.bias = bias;
    a.res = residual ? residual + (long long)b0 * (out_img / 4) : nullptr; a.ldr = cout; a.sR = 0;
    a.alpha = 1.f; a.beta = 0.f;
    a.a_bytes = (unsigned)(in_img * n); a.b_bytes = (unsigned)(wbytes / 4);
    a.c_bytes = (unsigned)(out_img * n); a.r_bytes = a.c_bytes;
    a.H = h; a.W = wd; a.Cx = cin; a.Ho = h; a.Wo = wd; a.R = 2; a.S = 2;
    a.perm_rs = (v && cin % BK == 0 && kperm_enabled()) ? 4 : 1;
    set_gather_magic(a);
    a.stride = 1; a.stride_shift = 0; a.pad_t = 1; a.pad_l = 1;
    a.sub_w2 = 2 * wd; a.sub_par = 0; a.out_remap = 1;
    const int cfg = choose_tile(a, v, false);
    if (v) launch_big<A_CONV_SUBPIX, 4, B_ROWK, 4>(a, st, cfg);
    else launch_small<A_CONV_SUBPIX, 1, B_ROWK, 1>(a, st, cfg);
    const int rc = gemm_finish(a, st);
    if (rc) return rc;
  }
  return MVAE_OK;
}

}  // extern "C"
