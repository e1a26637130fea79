// Direct 3x3 / stride-1 / pad-1 convolution at 32 input and 32 output channels: the 28x28 level of the c3 disentangled
// model (hidden 32: ResnetBlock conv1 / conv2, encoder_decoder.py:123-146), forward and input gradient.
//
// As an implicit GEMM this is M = pixels (401k at bs 512), N = 32, K = 288: 64x64 tiles leave half the MFMA columns
// empty and each tile walks 9 short K-tiles with a barrier and a global-load latency per K-tile (76 us per launch,
// ~100 TF/s). Here a workgroup owns a band of R output rows of one image: the band's input rows plus the 1-pixel halo
// are staged ONCE into LDS as a ROW image in "padded pixel" order (row pitch W + 2, k = the 32 channels), so filter tap
// (r, s) is the constant pixel offset r*(W+2) + s and the 9 per-tap products y[p][:] += x[p + off_t][:] W_t are
// 16x16x32 MFMA tiles (K = 32 = one k-step per tap) read straight from that image; the 9 weight taps are staged once
// per workgroup (persistent grid) as [co][ci] ROW images. The next band's input is prefetched into registers while the
// current one is multiplied. Arithmetic = the GEMM's (mma<PREC>: 3xBF16, bf16 or exact fp32).
// Input gradient (DGRAD): dx = the same stencil over dy with the flipped, transposed kernel W'_t[ci][co] =
// W_{8-t}[co][ci] (the transposed conv of a stride-1, pad-1 3x3 conv).
#include "gemm_core.h"

namespace mvae {

constexpr int CD_C = 32;     // channels in and out
constexpr int CD_PITCH = 40; // ROW image pitch (bf16 elements per pixel row: 32 + 8 pad), as the GEMM's images
// (NT, MAXPIX): threads per workgroup, staged padded pixels per band (R*(W+2) + 2*(W+2) + 2 + one M-tile of overhang)
//   (512, 384): 8 waves, 107.5 KB of LDS, one workgroup per CU
//   (256, 208): 4 waves, 79.4 KB, two workgroups per CU (one stages while the other multiplies)

struct CdArgs {
  const float* x;      // [n][h][w][32] fp32, or split4_bf16 groups (XSPLIT)
  const float* w;      // [32][3][3][32] fp32 (KRSC), or split4_bf16 groups along ci (WSPLIT, forward only)
  const float* bias;   // [32] or null
  const float* res;    // [n][h][w][32] or null (added to the output)
  float* y;            // [n][h][w][32]
  int n, h, wd, R, PW, bands, units, mtiles;
  int xsplit, wsplit, dgrad;
};

// staged input of one band: float4 slots (padded pixel p, channel quad q), p in [0, NPIX), zero outside the image
template <int NT, int NS>
__device__ __forceinline__ void cd_load(const CdArgs& a, int u, int tid, int npix, float4 (&v)[NS]) {
  const int img = u / a.bands, y0 = (u - img * a.bands) * a.R;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * NT;
    const int p = i >> 3, q = i & 7;
    const int py = p / a.PW, px = p - py * a.PW;
    const int yy = y0 - 1 + py, xx = px - 1;
    const bool ok = (u < a.units) & (p < npix) & ((unsigned)yy < (unsigned)a.h) & ((unsigned)xx < (unsigned)a.wd);
    v[j] = ok ? *(const float4*)(a.x + (((long long)img * a.h + yy) * a.wd + xx) * CD_C + q * 4)
              : float4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int PREC, int NT, int MAXPIX, int NS>
__device__ __forceinline__ void cd_store(const CdArgs& a, __bf16* img, int tid, int npix, const float4 (&v)[NS]) {
  constexpr int PL = MAXPIX * CD_PITCH;
#pragma unroll
  for (int j = 0; j < NS; ++j) {
    const int i = tid + j * NT;
    const int p = i >> 3, q = i & 7;
    if (p < npix) {
      if (a.xsplit) st_presplit<PREC>(img, PL, row_off(p, q), v[j]);
      else st_split<PREC>(img, PL, row_off(p, q), v[j]);
    }
  }
}

template <int PREC, int NT, int MAXPIX>
__global__ void __launch_bounds__(NT) conv_direct32_kernel(CdArgs a) {
  constexpr int PL = MAXPIX * CD_PITCH;         // x image plane (elements)
  constexpr int WPL = 9 * CD_C * CD_PITCH;      // weight image plane
  constexpr int NS = (MAXPIX * 8 + NT - 1) / NT;  // float4 slots per thread per band
  __shared__ __attribute__((aligned(16))) __bf16 xs[2 * PL];
  __shared__ __attribute__((aligned(16))) __bf16 ws[2 * WPL];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int npix = (a.R + 2) * a.PW + 2;  // rows y0-1 .. y0+R plus the tap overhang of the last M-tile's junk columns
  // weights: tap t image [n][k] with n = output channel of this pass, k = input channel
  for (int i = tid; i < 9 * CD_C * 8; i += NT) {
    const int t = i / (CD_C * 8), rem = i - t * (CD_C * 8), nn = rem >> 3, q = rem & 7;
    float4 v;
    if (!a.dgrad) {
      const float* src = a.w + ((long long)nn * 9 + t) * CD_C + q * 4;  // w[co = nn][t][ci = 4q..]
      v = *(const float4*)src;
      if (a.wsplit) {
        st_presplit<PREC>(ws, WPL, t * CD_C * CD_PITCH + row_off(nn, q), v);
        continue;
      }
    } else {  // W'_t[ci = nn][co = 4q..] = w[co][8 - t][ci]
      const float* src = a.w + (long long)(q * 4) * 9 * CD_C + (8 - t) * CD_C + nn;
      v = float4{src[0], src[9 * CD_C], src[2 * 9 * CD_C], src[3 * 9 * CD_C]};
    }
    st_split<PREC>(ws, WPL, t * CD_C * CD_PITCH + row_off(nn, q), v);
  }
  float4 v[NS];
  int u = blockIdx.x;
  cd_load<NT, NS>(a, u, tid, npix, v);
  float bsv[2] = {0.f, 0.f};
  if (a.bias != nullptr) {
    bsv[0] = a.bias[lane & 15];
    bsv[1] = a.bias[16 + (lane & 15)];
  }
  for (; u < a.units; u += gridDim.x) {
    __syncthreads();  // the previous band's fragment reads are done (and, first time, the weight image is complete)
    cd_store<PREC, NT, MAXPIX, NS>(a, xs, tid, npix, v);
    __syncthreads();
    cd_load<NT, NS>(a, u + gridDim.x, tid, npix, v);  // next band: in flight during this band's products
    const int img = u / a.bands, y0 = (u - img * a.bands) * a.R;
    for (int mt = wid; mt < a.mtiles; mt += NT / 64) {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int off = (t / 3) * a.PW + (t % 3);  // output padded pixel p reads input padded pixel p + off
        const bf16x8 ah = read_frag<MAXPIX, false, 16>(xs, mt * 16 + off, 0, lane);
        bf16x8 al{};
        if constexpr (PREC != 1) al = read_frag<MAXPIX, false, 16>(xs + PL, mt * 16 + off, 0, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const bf16x8 bh = read_frag<CD_C, false, 16>(ws + t * CD_C * CD_PITCH, j * 16, 0, lane);
          bf16x8 bl{};
          if constexpr (PREC != 1) bl = read_frag<CD_C, false, 16>(ws + WPL + t * CD_C * CD_PITCH, j * 16, 0, lane);
          mma<PREC>(acc[j], ah, al, bh, bl);
        }
      }
      // output padded pixel p = mt*16 + row -> image row y0 + p / PW, column p % PW (columns >= W are junk)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = mt * 16 + acc_row<16>(r, lane);
        const int py = p / a.PW, px = p - py * a.PW;
        const int yy = y0 + py;
        if (py < a.R && yy < a.h && px < a.wd) {
          const long long o = (((long long)img * a.h + yy) * a.wd + px) * CD_C + (lane & 15);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            float val = acc[j][r] + bsv[j];
            if (a.res != nullptr) val += a.res[o + j * 16];
            a.y[o + j * 16] = val;
          }
        }
      }
    }
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

// y = conv3x3(x, w) [+ bias][+ residual] (mode & MVAE_CONV_DGRAD_DIRECT == 0), or the input gradient dx = the
// transposed conv of dy (x := dy, w = the forward conv's weights, no bias / residual). 32 channels in and out, NHWC.
// mode: MVAE_CONV_XSPLIT (x holds split4_bf16 groups), MVAE_CONV_WSPLIT (w holds split4_bf16 groups; forward only).
int mvae_conv2d_direct32_nhwc(const float* x, const float* w, const float* bias, const float* residual, float* y,
                              int n, int h, int wd, int mode, void* stream) {
  const bool dgrad = (mode & MVAE_CONV_DGRAD_DIRECT) != 0;
  const bool xsplit = (mode & MVAE_CONV_XSPLIT) != 0, wsplit = (mode & MVAE_CONV_WSPLIT) != 0;
  if (n <= 0 || h <= 0 || wd <= 0 || wd + 2 > 64 || x == nullptr || w == nullptr || y == nullptr || !al16(x) ||
      !al16(w) || (dgrad && (bias || residual || wsplit)) || ((xsplit || wsplit) && split_forbidden())) {
    set_error("conv2d_direct32: 32 -> 32 channels, W <= 62, aligned x / w; dgrad: no bias / residual / split weights");
    return MVAE_EINVAL;
  }
  static const bool big_env = getenv("MVAE_CD_BIG") != nullptr;  // experiment knob: 8-wave workgroups, one per CU
  const bool big = big_env || 3 * (wd + 2) + 2 + 16 > 208;      // (a band of one row does not fit the small image)
  const int maxpix = big ? 384 : 208;
  CdArgs a{};
  a.x = x; a.w = w; a.bias = bias; a.res = residual; a.y = y;
  a.n = n; a.h = h; a.wd = wd; a.PW = wd + 2;
  // rows per band: the largest R with (R + 2) * PW + 2 padded pixels staged and R * PW rounded to whole M-tiles
  int R = 0;
  for (int r = 1; r <= h; ++r)
    if ((r + 2) * a.PW + 2 + 16 <= maxpix) R = r;
  if (R == 0) {
    set_error("conv2d_direct32: image too wide for one band row");
    return MVAE_EINVAL;
  }
  a.R = R;
  a.bands = (h + R - 1) / R;
  a.units = n * a.bands;
  a.mtiles = (R * a.PW + 15) / 16;
  a.xsplit = xsplit; a.wsplit = wsplit; a.dgrad = dgrad;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::max(1, std::min(a.units, std::max(1, cus) * (big ? 1 : 2)));
  hipStream_t st = (hipStream_t)stream;
  const int mm = math_mode();
#define CD_LAUNCH(P, NT_, MP)                                                                            \
  hipLaunchKernelGGL((conv_direct32_kernel<P, NT_, MP>), dim3(grid), dim3(NT_), 0, st, a)
  if (big) {
    if (mm == MATH_BF16) CD_LAUNCH(1, 512, 384);
    else if (mm == MATH_FP32) CD_LAUNCH(0, 512, 384);
    else CD_LAUNCH(3, 512, 384);
  } else {
    if (mm == MATH_BF16) CD_LAUNCH(1, 256, 208);
    else if (mm == MATH_FP32) CD_LAUNCH(0, 256, 208);
    else CD_LAUNCH(3, 256, 208);
  }
#undef CD_LAUNCH
  return launch_status();
}

}  // extern "C"
