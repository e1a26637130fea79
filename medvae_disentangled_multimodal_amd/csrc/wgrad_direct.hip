// Weight (+ bias) gradient of a 3x3 / stride-1 / pad-1 convolution with few channels (cin, cout in {32, 64}:
// the 28x28 / 14x14 levels of the c3 disentangled model, hidden 32 -- encoder_decoder.py:123-146 convs inside
// ResnetBlock, Encoder.conv_in / Decoder levels).
//
// As an implicit GEMM (M = cout, N = 9*cin, K = pixels) these are 32..64 x 288..576 outputs over 25k-400k
// pixels: 64x64 tiles leave half the MFMA rows empty for cout 32, the 5-9 N-tiles re-read dY, and split-K
// turns each K loop into short latency-bound runs (128 us for the 28x28x32 layer at bs 512, 58 TF/s).
// Here a workgroup owns a band of R (<= 8) output rows of one image: dY of the band ([pixel][cout]) and x of the
// band plus its 1-pixel halo ([pixel][cin]) are staged once into LDS as 3xBF16 hi/lo planes in "padded pixel"
// order (row pitch W + 2), so filter tap (r, s) is a constant row offset r*(W+2) + s of the x image: the 9
// per-tap products dW_t[co][ci] += sum_p dY[p][co] x[p + off_t][ci] are 32x32x16 MFMA tiles whose operand
// fragments come from the same two images (ds_read_b64_tr_b16 transposed reads). Every workgroup accumulates
// its dW partial in registers over all its bands (persistent grid), the waves of a workgroup are combined in
// LDS in a fixed order, and a fixed-order reducer sums the workgroup partials (deterministic, no atomics).
// The bias gradient (sum of dY) is accumulated while staging dY.
#include "gemm_core.h"

namespace mvae {

constexpr int WD_NT = 768;  // 12 waves: (co-block, ci-block) pair x kernel row x k-slice per wave
// staged float4 per thread per band (register budget at 3 waves/SIMD): 4 for a 32-channel operand, 6 for 64
template <int C> constexpr int wd_slots() { return C == 32 ? 4 : 6; }

// LDS image [k-row][NCOL] of bf16 (hi plane, then lo plane). 64-column images swizzle 32-column halves by
// k-row bit 1 so the 4 k-rows of a transposed read land in disjoint 16-bank windows (32-column images:
// the 64-B pitch already does).
template <int NCOL>
__device__ __forceinline__ int wd_off(int kr, int col) {
  return kr * NCOL + (NCOL == 64 ? (col ^ (((kr >> 1) & 1) << 5)) : col);
}

// 32x32x16 MFMA operand fragment of a [k][col] image: lane l holds element (col0 + (l & 31), k0 + 8*(l>>5) + j)
template <int NCOL>
__device__ __forceinline__ bf16x8 wd_frag(const __bf16* plane, int col0, int k0, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int kr = k0 + (g >> 1) * 8 + (li >> 2);
  const int col = col0 + (g & 1) * 16 + 4 * (li & 3);
  const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(plane + wd_off<NCOL>(kr, col)));
  const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(plane + wd_off<NCOL>(kr + 4, col)));
  return __builtin_shufflevector(v0, v1, 0, 1, 2, 3, 4, 5, 6, 7);
}

// band geometry: R output rows per band, padded-pixel row pitch PW = W + 2
struct WdGeom {
  int H, W, R, PW, KA, KX, bands, units;
  __host__ __device__ WdGeom(int nb, int h, int w, int r) {
    H = h; W = w; R = r; PW = w + 2;
    KA = ((R * PW + 15) / 16) * 16;
    KX = KA + 2 * PW + 2;
    bands = (h + R - 1) / R;
    units = nb * bands;
  }
};

template <int CO, int CI>
__host__ __device__ constexpr size_t wd_stage_bytes(int KA, int KX) {
  return (size_t)2 * KA * CO * 2 + (size_t)2 * KX * CI * 2;  // hi + lo planes of both images
}
template <int CO, int CI>
size_t wd_lds_bytes(const WdGeom& g) {
  constexpr int P = (CO / 32) * (CI / 32);
  const size_t stage2 = 2 * wd_stage_bytes<CO, CI>(g.KA, g.KX);  // double-buffered
  const size_t red = (size_t)P * 9 * 1024 * 4;
  return std::max(std::max(stage2, red), (size_t)WD_NT * 4 * 4);
}

// Per-thread staging registers of one band: the A (dY) and X (x + halo) float4 slots this thread loads
template <int CO, int CI>
struct WdStage {
  static constexpr int MA = wd_slots<CO>(), MX = wd_slots<CI>();
  float4 va[MA], vx[MX];
  __device__ void load(const float* __restrict__ dy, const float* __restrict__ x, const WdGeom& g, int u, int tid,
                       float (&bsum)[4]) {
    const int n = u / g.bands, y0 = (u - n * g.bands) * g.R;
    const float4 zero{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < MA; ++j) {  // dY rows y0 .. y0+R-1, padded-pixel order; padding is zero
      const int i = tid + j * WD_NT;
      const int kr = i / (CO / 4), q = i - kr * (CO / 4);
      const int yy = kr / g.PW, xx = kr - yy * g.PW, y = y0 + yy;
      const bool ok = kr < g.KA && yy < g.R && xx < g.W && y < g.H;
      va[j] = ok ? *(const float4*)(dy + (((long long)n * g.H + y) * g.W + xx) * CO + q * 4) : zero;
    }
#pragma unroll
    for (int j = 0; j < MX; ++j) {  // x rows y0-1 .. y0+R, columns -1 .. W (+ padding rows)
      const int i = tid + j * WD_NT;
      const int r = i / (CI / 4), q = i - r * (CI / 4);
      const int yy = r / g.PW, xx = r - yy * g.PW, y = y0 - 1 + yy, xw = xx - 1;
      const bool ok = r < g.KX && y >= 0 && y < g.H && xw >= 0 && xw < g.W;
      vx[j] = ok ? *(const float4*)(x + (((long long)n * g.H + y) * g.W + xw) * CI + q * 4) : zero;
    }
#pragma unroll
    for (int j = 0; j < MA; ++j) {  // bias: dY column sums (a thread's channel quad is tid % (CO/4))
      bsum[0] += va[j].x; bsum[1] += va[j].y; bsum[2] += va[j].z; bsum[3] += va[j].w;
    }
  }
  template <int PREC, bool XSPLIT>
  __device__ void store(__bf16* A, __bf16* X, const WdGeom& g, int tid) const {
#pragma unroll
    for (int j = 0; j < MA; ++j) {
      const int i = tid + j * WD_NT;
      const int kr = i / (CO / 4), q = i - kr * (CO / 4);
      if (kr < g.KA) st_split<PREC>(A, g.KA * CO, wd_off<CO>(kr, q * 4), va[j]);
    }
#pragma unroll
    for (int j = 0; j < MX; ++j) {
      const int i = tid + j * WD_NT;
      const int r = i / (CI / 4), q = i - r * (CI / 4);
      if (r < g.KX) {
        if constexpr (XSPLIT)
          st_presplit<PREC>(X, g.KX * CI, wd_off<CI>(r, q * 4), vx[j]);
        else
          st_split<PREC>(X, g.KX * CI, wd_off<CI>(r, q * 4), vx[j]);
      }
    }
  }
};

template <int CO, int CI, int PREC, bool XSPLIT>
__global__ void __launch_bounds__(WD_NT) wgrad_direct_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                             float* __restrict__ part, float* __restrict__ bpart,
                                                             int nb, int H, int W, int R) {
  extern __shared__ __bf16 wd_sm[];
  const WdGeom gm(nb, H, W, R);
  const int SB = (int)(wd_stage_bytes<CO, CI>(gm.KA, gm.KX) / 2);  // one stage buffer, in bf16 elements
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int P = (CO / 32) * (CI / 32), NSL = 4 / P;
  // wave -> (pair, kernel row dr, k-slice): 12 = P x 3 x NSL
  const int pair = wv % P, dr = (wv / P) % 3, sl = wv / (3 * P);
  const int cob = pair / (CI / 32), cib = pair % (CI / 32);
  f32x16 acc[3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  WdStage<CO, CI> stg;
  int u = blockIdx.x, cur = 0;
  if (u < gm.units) {
    stg.load(dy, x, gm, u, tid, bsum);
    stg.template store<PREC, XSPLIT>(wd_sm, wd_sm + 2 * gm.KA * CO, gm, tid);
  }
  __syncthreads();
  const int nch = gm.KA / 16;
  for (; u < gm.units; u += gridDim.x) {
    const int un = u + gridDim.x;
    if (un < gm.units) stg.load(dy, x, gm, un, tid, bsum);  // next band: loads fly during this band's MFMAs
    const __bf16* A = wd_sm + cur * SB;
    const __bf16* X = A + 2 * gm.KA * CO;
    for (int c = sl; c < nch; c += NSL) {
      const int k0 = c * 16;
      const bf16x8 ah = wd_frag<CO>(A, cob * 32, k0, lane);
      const bf16x8 al = PREC == 3 ? wd_frag<CO>(A + gm.KA * CO, cob * 32, k0, lane) : ah;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int off = dr * gm.PW + s;  // tap (dr, s) = row offset of the x image
        const bf16x8 bh = wd_frag<CI>(X, cib * 32, k0 + off, lane);
        const bf16x8 bl = PREC == 3 ? wd_frag<CI>(X + gm.KX * CI, cib * 32, k0 + off, lane) : bh;
        mma<PREC>(acc[s], ah, al, bh, bl);
      }
    }
    if (un < gm.units) {
      __bf16* An = wd_sm + (cur ^ 1) * SB;  // last read two barriers ago
      stg.template store<PREC, XSPLIT>(An, An + 2 * gm.KA * CO, gm, tid);
    }
    __syncthreads();
    cur ^= 1;
  }
  // ---- combine the k-slices of each (pair, dr) in a fixed order, then the workgroup partial [co][tap][ci] ----
  float* red = (float*)wd_sm;  // [P][9][32][32]
  float* out = part + (size_t)blockIdx.x * (CO * 9 * CI);
  for (int s2 = 0; s2 < NSL; ++s2) {
    if (sl == s2) {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = acc_row<32>(r, lane), nn = lane & 31;
          float* p = red + ((pair * 9 + dr * 3 + t) * 32 + m) * 32 + nn;
          *p = s2 == 0 ? acc[t][r] : *p + acc[t][r];
        }
    }
    __syncthreads();
  }
  for (int i = tid; i < P * 9 * 1024; i += WD_NT) {
    const int pr = i / (9 * 1024), rem = i - pr * 9 * 1024, t = rem >> 10, m = (rem >> 5) & 31, nn = rem & 31;
    const int co = (pr / (CI / 32)) * 32 + m, ci = (pr % (CI / 32)) * 32 + nn;
    out[(co * 9 + t) * CI + ci] = red[i];
  }
  __syncthreads();
  // bias: threads with the same channel quad, fixed order
#pragma unroll
  for (int e = 0; e < 4; ++e) red[tid * 4 + e] = bsum[e];
  __syncthreads();
  if (tid < CO) {
    const int q = tid >> 2, e = tid & 3;
    float s = 0.f;
    for (int j = q; j < WD_NT; j += CO / 4) s += red[j * 4 + e];
    bpart[(size_t)blockIdx.x * CO + tid] = s;
  }
}

// dw[i] = beta*dw[i] + sum_g part[g][i] (i < nw), dbias[c] likewise from bpart: 64 outputs x 4 partial lanes per
// block, each lane a fixed stride over the workgroup partials, lanes combined in order
__global__ void __launch_bounds__(256) wgrad_direct_final_kernel(const float* __restrict__ part,
                                                                 const float* __restrict__ bpart, int G, int nw, int co,
                                                                 float* dw, float* dbias, float beta) {
  __shared__ float sh[4][64];
  const int o = blockIdx.x * 64 + (threadIdx.x & 63), gl = threadIdx.x >> 6;
  const bool isw = o < nw, isb = !isw && dbias != nullptr && o < nw + co;
  float s = 0.f;
  if (isw)
    for (int g = gl; g < G; g += 4) s += part[(size_t)g * nw + o];
  else if (isb)
    for (int g = gl; g < G; g += 4) s += bpart[(size_t)g * co + (o - nw)];
  sh[gl][threadIdx.x & 63] = s;
  __syncthreads();
  if (gl == 0 && (isw || isb)) {
    const int l = threadIdx.x & 63;
    const float v = ((sh[0][l] + sh[1][l]) + sh[2][l]) + sh[3][l];
    float* dst = isw ? dw + o : dbias + (o - nw);
    *dst = (beta != 0.f ? beta * *dst : 0.f) + v;
  }
}

constexpr int WD_MAX_G = 512;  // persistent grid cap (workspace sizing): 2 workgroups per CU on 256 CUs

// persistent grid: the workgroups resident at once (occupancy query with the launch's dynamic LDS)
static int wd_grid(const void* kernel, size_t lds, int units) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || cus <= 0)
    cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, WD_NT, lds) != hipSuccess || per_cu <= 0)
    per_cu = 1;
  return std::max(1, std::min(units, std::min(WD_MAX_G, cus * per_cu)));
}

template <int CO, int CI, int PREC, bool XS>
static int wd_launch(const float* dy, const float* x, float* part, float* bpart, int nb, int h, int w, int r,
                     size_t lds, hipStream_t st) {
  const void* k = (const void*)wgrad_direct_kernel<CO, CI, PREC, XS>;
  static bool attr = false;  // dynamic LDS above 64 KB must be allowed per kernel
  if (!attr) {
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int G = wd_grid(k, lds, WdGeom(nb, h, w, r).units);
  hipLaunchKernelGGL((wgrad_direct_kernel<CO, CI, PREC, XS>), dim3(G), dim3(WD_NT), lds, st, dy, x, part, bpart, nb,
                     h, w, r);
  return G;
}

// band height: the largest R in {8, 4, 2, 1} whose double-buffered images fit 152 KB of LDS and whose per-thread
// staging fits the per-thread slots of each operand
template <int CO, int CI>
static int wd_rows(int nb, int h, int w) {
  for (int r = 8; r >= 1; r >>= 1) {
    const WdGeom g(nb, h, w, r);
    if (wd_lds_bytes<CO, CI>(g) > 152 * 1024) continue;
    if ((long long)g.KA * (CO / 4) > (long long)wd_slots<CO>() * WD_NT ||
        (long long)g.KX * (CI / 4) > (long long)wd_slots<CI>() * WD_NT)
      continue;
    return r;
  }
  return 0;
}

// returns the grid size (the number of workgroup partials), or a negative error
template <int CO, int CI>
static int wd_dispatch(const float* dy, const float* x, float* part, float* bpart, int nb, int h, int w, int prec,
                       bool xs, hipStream_t st) {
  const int r = wd_rows<CO, CI>(nb, h, w);
  if (r == 0) {
    set_error("wgrad_direct: image row too wide for LDS (w = %d)", w);
    return MVAE_EINVAL;
  }
  const size_t lds = wd_lds_bytes<CO, CI>(WdGeom(nb, h, w, r));
  if (prec == 3) return xs ? wd_launch<CO, CI, 3, true>(dy, x, part, bpart, nb, h, w, r, lds, st)
                           : wd_launch<CO, CI, 3, false>(dy, x, part, bpart, nb, h, w, r, lds, st);
  return xs ? wd_launch<CO, CI, 1, true>(dy, x, part, bpart, nb, h, w, r, lds, st)
            : wd_launch<CO, CI, 1, false>(dy, x, part, bpart, nb, h, w, r, lds, st);
}

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_conv2d_wgrad_direct_workspace_bytes(int nb, int h, int w, int cin, int cout) {
  (void)nb; (void)h; (void)w;
  return (size_t)WD_MAX_G * ((size_t)cout * 9 * cin + cout) * sizeof(float) + 512;
}

// dw[cout][3][3][cin] = beta*dw + sum over pixels (3x3, stride 1, pad 1); dbias (optional) likewise.
// cin, cout in {32, 64}; x_split: x holds split4_bf16 groups (bf16 mode reads their hi halves). 3xBF16 (math
// mode 0) or bf16 (mode 1).
int mvae_conv2d_wgrad_direct_nhwc(const float* dy, const float* x, float* dw, float* dbias, float beta, int nb, int h,
                                  int w, int cin, int cout, int x_split, void* workspace, size_t workspace_bytes,
                                  void* stream) {
  if (nb <= 0 || h <= 0 || w <= 0 || (cin != 32 && cin != 64) || (cout != 32 && cout != 64) || !dy || !x || !dw) {
    set_error("wgrad_direct: needs cin, cout in {32, 64}");
    return MVAE_EINVAL;
  }
  if ((((uintptr_t)dy | (uintptr_t)x) & 15) != 0) {
    set_error("wgrad_direct: dy and x must be 16-B aligned");
    return MVAE_EINVAL;
  }
  const int mm = math_mode();
  if (mm == MATH_FP32) {
    set_error("wgrad_direct: not available in the exact-fp32 math mode (use mvae_conv2d_wgrad_nhwc)");
    return MVAE_EINVAL;
  }
  if (workspace == nullptr || workspace_bytes < mvae_conv2d_wgrad_direct_workspace_bytes(nb, h, w, cin, cout)) {
    set_error("wgrad_direct: workspace too small");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)workspace;
  float* bpart = (float*)(((uintptr_t)(part + (size_t)WD_MAX_G * cout * 9 * cin) + 255) & ~(uintptr_t)255);
  const int prec = mm == MATH_BF16 ? 1 : 3;
  const bool xs = x_split != 0;
  int G;
  if (cout == 32 && cin == 32) G = wd_dispatch<32, 32>(dy, x, part, bpart, nb, h, w, prec, xs, st);
  else if (cout == 32) G = wd_dispatch<32, 64>(dy, x, part, bpart, nb, h, w, prec, xs, st);
  else if (cin == 32) G = wd_dispatch<64, 32>(dy, x, part, bpart, nb, h, w, prec, xs, st);
  else G = wd_dispatch<64, 64>(dy, x, part, bpart, nb, h, w, prec, xs, st);
  if (G < 0) return G;
  const int nw = cout * 9 * cin;
  hipLaunchKernelGGL(wgrad_direct_final_kernel, dim3(cdiv(nw + cout, 64)), dim3(256), 0, st, (const float*)part,
                     (const float*)bpart, G, nw, cout, dw, dbias, beta);
  return launch_status();
}

}  // extern "C"
