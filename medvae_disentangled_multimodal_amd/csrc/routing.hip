// Modality routing of the DisentangledConditionalVAE (src/models/disentangled_conditional_vae.py) on gfx950.
//
// The reference routes every sample through a Python loop: `.item()` per sample, then the sample's own
// input projector (:137-169) and, after the shared decoder, the sample's own modality head
// conv3x3 -> ReLU -> conv3x3 (+ output projector 1x1, :255-301), each as a batch-of-1 ATen conv launch.
// Here ONE launch routes the whole batch: a workgroup per sample reads the sample's modality id on the
// device (clamped to the last modality like :142-146 / :260-265), picks that modality's parameters from a
// pointer table and runs only that modality's layers -- no host sync, no work on the other modalities'
// heads. The image, the hidden activation and the gradients live in LDS (zero-bordered, so the 3x3
// stencils need no bounds checks). Weight gradients are per-sample partials reduced per modality in
// sample order by a second kernel: deterministic, no float atomics.
//
// HBM-bound: per image the head pass reads the decoder output once and writes the routed output once
// (forward), and reads the output gradient once and writes the input gradient once (backward).
#include "common.h"

namespace mvae {

constexpr int RT_MAXM = 8;  // modalities per pointer table
constexpr int RT_NT = 256;

struct HeadTable {  // per modality; NULL entries: the modality has no such module
  const float* w1[RT_MAXM];  // modality_decoders.m.0.weight  [C][3][3][C] (KRSC)
  const float* b1[RT_MAXM];
  const float* w2[RT_MAXM];  // modality_decoders.m.2.weight
  const float* b2[RT_MAXM];
  const float* pw[RT_MAXM];  // modality_output_projectors.m.weight [cm][C] (1x1), NULL: colour modality
  const float* pb[RT_MAXM];
  int cm[RT_MAXM];           // output channels of the projector (its cout)
};
struct HeadGrad {  // flat gradient slots (accumulated, beta = 1)
  float* w1[RT_MAXM];
  float* b1[RT_MAXM];
  float* w2[RT_MAXM];
  float* b2[RT_MAXM];
  float* pw[RT_MAXM];
  float* pb[RT_MAXM];
};
struct ProjTable {  // modality_input_projectors.m: 1x1 conv 1 -> C (NULL: the modality keeps its channels)
  const float* w[RT_MAXM];
  const float* b[RT_MAXM];
};
struct ProjGrad {
  float* w[RT_MAXM];
  float* b[RT_MAXM];
};

// ids past the last modality use the last one (:142-146, :260-265); negative ids (a KeyError in the
// reference) are clamped to 0 so a bad id can never index outside the parameter table
__device__ __forceinline__ int clamp_mod(long long v, int nm) { return v >= nm ? nm - 1 : (v < 0 ? 0 : (int)v); }
__device__ __forceinline__ float nz(float v) { return v != v ? 0.f : v; }  // NaN -> 0 (:132-134, :160-167)

// per-sample parameter-gradient partial layout: [w1 C*9*C][b1 C][w2 C*9*C][b2 C][pw CM*C][pb CM]
template <int C, int CM>
struct HeadLayout {
  static constexpr int W = C * 9 * C;
  static constexpr int W1 = 0, B1 = W, W2 = W + C, B2 = 2 * W + C, PW = 2 * W + 2 * C, PB = PW + CM * C;
  static constexpr int P = PB + CM;
};

// zero-bordered LDS plane [(H+2)][(W+2)][C]
struct Pad {
  int h, w;
  __device__ __forceinline__ int at(int y, int x) const { return ((y + 1) * (w + 2) + (x + 1)); }
  __device__ __forceinline__ int size() const { return (h + 2) * (w + 2); }
};

// conv3x3 (pad 1) of a zero-bordered plane: out[c] at pixel (y, x) with KRSC weights W [co][kh][kw][ci]
template <int C>
__device__ __forceinline__ void conv3(const float* src, const Pad& pd, int y, int x, const float* W, const float* b,
                                      float* out) {
#pragma unroll
  for (int co = 0; co < C; ++co) out[co] = b ? b[co] : 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const float* s = src + pd.at(y + kh - 1, x + kw - 1) * C;
#pragma unroll
      for (int ci = 0; ci < C; ++ci) {
        const float v = s[ci];
#pragma unroll
        for (int co = 0; co < C; ++co) out[co] = fmaf(W[((co * 3 + kh) * 3 + kw) * C + ci], v, out[co]);
      }
    }
}
// transposed conv3x3 (input gradient of a pad-1 conv): g = sum over taps of d[p - (kh-1, kw-1)][co] W[co][kh][kw][ci]
template <int C>
__device__ __forceinline__ void conv3t(const float* d, const Pad& pd, int y, int x, const float* W, float* out) {
#pragma unroll
  for (int ci = 0; ci < C; ++ci) out[ci] = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const float* s = d + pd.at(y - (kh - 1), x - (kw - 1)) * C;
#pragma unroll
      for (int co = 0; co < C; ++co) {
        const float v = s[co];
#pragma unroll
        for (int ci = 0; ci < C; ++ci) out[ci] = fmaf(W[((co * 3 + kh) * 3 + kw) * C + ci], v, out[ci]);
      }
    }
}

// ---- forward: out = route(head_m(rec)) ---------------------------------------------------------------------
template <int C>
__global__ void __launch_bounds__(RT_NT) heads_fwd_kernel(const float* __restrict__ rec, const long long* __restrict__ idx,
                                                           int h, int w, int nm, HeadTable tab, int out_c,
                                                           float* __restrict__ out) {
  extern __shared__ float sm[];
  const Pad pd{h, w};
  float* in = sm;                  // decoder output, zero border
  float* r = sm + pd.size() * C;   // relu(conv1), zero border
  const int b = blockIdx.x, hw = h * w;
  const int m = clamp_mod(idx[b], nm);
  const float* W1 = tab.w1[m];
  const float* B1 = tab.b1[m];
  const float* W2 = tab.w2[m];
  const float* B2 = tab.b2[m];
  const float* PW = tab.pw[m];
  const float* PB = tab.pb[m];
  const int cm = tab.cm[m];
  for (int i = threadIdx.x; i < 2 * pd.size() * C; i += RT_NT) sm[i] = 0.f;
  __syncthreads();
  const float* src = rec + (long long)b * hw * C;
  for (int i = threadIdx.x; i < hw * C; i += RT_NT) {
    const int p = i / C, c = i - p * C, y = p / w, x = p - y * w;
    in[pd.at(y, x) * C + c] = src[i];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float o[C];
    conv3<C>(in, pd, y, x, W1, B1, o);
#pragma unroll
    for (int c = 0; c < C; ++c) r[pd.at(y, x) * C + c] = fmaxf(o[c], 0.f);
  }
  __syncthreads();
  float* dst = out + (long long)b * hw * out_c;
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float o[C];
    conv3<C>(r, pd, y, x, W2, B2, o);
    if (PW != nullptr) {  // output projector (1x1, C -> cm), zero-padded to out_c (:272-297)
      for (int j = 0; j < out_c; ++j) {
        float v = 0.f;
        if (j < cm) {
          v = PB ? PB[j] : 0.f;
#pragma unroll
          for (int c = 0; c < C; ++c) v = fmaf(PW[j * C + c], o[c], v);
        }
        dst[p * out_c + j] = v;
      }
    } else {
      for (int j = 0; j < out_c; ++j) {
        float v = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) v = (c == j) ? o[c] : v;
        dst[p * out_c + j] = v;
      }
    }
  }
}

// ---- backward: per-sample input gradient + parameter-gradient partials --------------------------------------
template <int C, int CM>
__global__ void __launch_bounds__(RT_NT) heads_bwd_kernel(const float* __restrict__ rec, const long long* __restrict__ idx,
                                                           int h, int w, int nm, HeadTable tab, int out_c,
                                                           const float* __restrict__ dout, float* __restrict__ drec,
                                                           float* __restrict__ part) {
  using LY = HeadLayout<C, CM>;
  extern __shared__ float sm[];
  const Pad pd{h, w};
  const int S = pd.size() * C;
  float* in = sm;            // decoder output (zero border)
  float* r = sm + S;         // relu(conv1) (zero border)
  float* dh2 = sm + 2 * S;   // gradient at the head output (zero border)
  float* dh1 = sm + 3 * S;   // gradient at conv1's output (zero border)
  float* h2 = sm + 4 * S;    // head output (interior only, [hw][C]) -- projector weight gradient
  const int b = blockIdx.x, hw = h * w;
  const int m = clamp_mod(idx[b], nm);
  const float* W1 = tab.w1[m];
  const float* B1 = tab.b1[m];
  const float* W2 = tab.w2[m];
  const float* B2 = tab.b2[m];
  const float* PW = tab.pw[m];
  const int cm = PW != nullptr ? tab.cm[m] : 0;
  for (int i = threadIdx.x; i < 4 * S; i += RT_NT) sm[i] = 0.f;
  __syncthreads();
  const float* src = rec + (long long)b * hw * C;
  const float* go = dout + (long long)b * hw * out_c;
  for (int i = threadIdx.x; i < hw * C; i += RT_NT) {
    const int p = i / C, c = i - p * C, y = p / w, x = p - y * w;
    in[pd.at(y, x) * C + c] = src[i];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float o[C];
    conv3<C>(in, pd, y, x, W1, B1, o);
#pragma unroll
    for (int c = 0; c < C; ++c) r[pd.at(y, x) * C + c] = fmaxf(o[c], 0.f);
  }
  __syncthreads();
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float o[C], d[C];
    conv3<C>(r, pd, y, x, W2, B2, o);
#pragma unroll
    for (int c = 0; c < C; ++c) {
      h2[p * C + c] = o[c];
      d[c] = 0.f;
    }
    if (PW != nullptr) {
      for (int j = 0; j < cm && j < out_c; ++j) {
        const float g = go[p * out_c + j];
#pragma unroll
        for (int c = 0; c < C; ++c) d[c] = fmaf(PW[j * C + c], g, d[c]);
      }
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) d[c] = c < out_c ? go[p * out_c + c] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < C; ++c) dh2[pd.at(y, x) * C + c] = d[c];
  }
  __syncthreads();
  // dh1 = conv2^T(dh2) * relu'(conv1)
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float g[C];
    conv3t<C>(dh2, pd, y, x, W2, g);
#pragma unroll
    for (int c = 0; c < C; ++c) dh1[pd.at(y, x) * C + c] = r[pd.at(y, x) * C + c] > 0.f ? g[c] : 0.f;
  }
  __syncthreads();
  // input gradient drec = conv1^T(dh1) (each (pixel, channel) written once)
  float* dst = drec + (long long)b * hw * C;
  for (int p = threadIdx.x; p < hw; p += RT_NT) {
    const int y = p / w, x = p - y * w;
    float g[C];
    conv3t<C>(dh1, pd, y, x, W1, g);
#pragma unroll
    for (int c = 0; c < C; ++c) dst[p * C + c] = g[c];
  }
  // parameter-gradient partials of this sample: one parameter per thread, a fixed walk over the rows with
  // pointer increments (no per-pixel index division) and two interleaved accumulators
  float* pp = part + (long long)b * LY::P;
  const int rs = (w + 2) * C;  // padded row stride of the LDS planes
  for (int q = threadIdx.x; q < LY::P; q += RT_NT) {
    float s0 = 0.f, s1 = 0.f;
    if (q < LY::B1 || (q >= LY::W2 && q < LY::B2)) {  // conv weights [co][kh][kw][ci]
      const bool second = q >= LY::W2;
      const int e = second ? q - LY::W2 : q;
      const int ci = e % C, kw = (e / C) % 3, kh = (e / (3 * C)) % 3, co = e / (9 * C);
      const float* d = (second ? dh2 : dh1) + pd.at(0, 0) * C + co;
      const float* a = (second ? r : in) + pd.at(kh - 1, kw - 1) * C + ci;
      for (int y = 0; y < h; ++y, d += rs, a += rs) {
        int x = 0;
        for (; x + 1 < w; x += 2) {
          s0 = fmaf(d[x * C], a[x * C], s0);
          s1 = fmaf(d[(x + 1) * C], a[(x + 1) * C], s1);
        }
        if (x < w) s0 = fmaf(d[x * C], a[x * C], s0);
      }
    } else if (q < LY::W2 || q < LY::PW) {  // conv biases
      const bool second = q >= LY::B2;
      const int co = second ? q - LY::B2 : q - LY::B1;
      const float* d = (second ? dh2 : dh1) + pd.at(0, 0) * C + co;
      for (int y = 0; y < h; ++y, d += rs) {
        int x = 0;
        for (; x + 1 < w; x += 2) {
          s0 += d[x * C];
          s1 += d[(x + 1) * C];
        }
        if (x < w) s0 += d[x * C];
      }
    } else if (q < LY::PB) {  // projector weight [j][c]
      const int e = q - LY::PW, j = e / C, c = e - j * C;
      if (j < cm && j < out_c) {
        int p = 0;
        for (; p + 1 < hw; p += 2) {
          s0 = fmaf(go[p * out_c + j], h2[p * C + c], s0);
          s1 = fmaf(go[(p + 1) * out_c + j], h2[(p + 1) * C + c], s1);
        }
        if (p < hw) s0 = fmaf(go[p * out_c + j], h2[p * C + c], s0);
      }
    } else {  // projector bias
      const int j = q - LY::PB;
      if (j < cm && j < out_c) {
        int p = 0;
        for (; p + 1 < hw; p += 2) {
          s0 += go[p * out_c + j];
          s1 += go[(p + 1) * out_c + j];
        }
        if (p < hw) s0 += go[p * out_c + j];
      }
    }
    pp[q] = s0 + s1;
  }
}

// per-modality reduction of the per-sample partials into the flat gradient slots: one wave per (modality,
// parameter), lanes over the samples, then the fixed wave tree (deterministic)
template <int C, int CM>
__global__ void __launch_bounds__(256) heads_grad_reduce_kernel(const float* __restrict__ part,
                                                                const long long* __restrict__ idx, int nb, int nm,
                                                                HeadGrad g) {
  using LY = HeadLayout<C, CM>;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (t >= nm * LY::P) return;
  const int m = t / LY::P, q = t - m * LY::P;
  float s = 0.f;
  for (int b = lane; b < nb; b += 64)
    if (clamp_mod(idx[b], nm) == m) s += part[(long long)b * LY::P + q];
  s = wave_sum_f(s);
  if (lane != 0) return;
  float* dst;
  int off;
  if (q < LY::B1) { dst = g.w1[m]; off = q; }
  else if (q < LY::W2) { dst = g.b1[m]; off = q - LY::B1; }
  else if (q < LY::B2) { dst = g.w2[m]; off = q - LY::W2; }
  else if (q < LY::PW) { dst = g.b2[m]; off = q - LY::B2; }
  else if (q < LY::PB) { dst = g.pw[m]; off = q - LY::PW; }
  else { dst = g.pb[m]; off = q - LY::PB; }
  if (dst != nullptr) dst[off] += s;
}

// ---- input routing: routed = projector_m(x[:, :1]) or x[:, :C] -------------------------------------------
template <int C>
__global__ void route_in_fwd_kernel(const float* __restrict__ x, int cx, const long long* __restrict__ idx, int hw, int nm,
                                    ProjTable tab, float* __restrict__ routed) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= hw) return;
  const int m = clamp_mod(idx[b], nm);
  const float* xp = x + ((long long)b * hw + p) * cx;
  float* o = routed + ((long long)b * hw + p) * C;
  const float* W = tab.w[m];
  if (W != nullptr) {
    const float g = nz(xp[0]);
    const float* B = tab.b[m];
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = nz(fmaf(W[c], g, B ? B[c] : 0.f));
  } else {
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = c < cx ? nz(xp[c]) : 0.f;
  }
}

// per-sample partials {dW[c], db[c]} of the input projector (zero for samples without one)
template <int C>
__global__ void __launch_bounds__(RT_NT) route_in_bwd_kernel(const float* __restrict__ x, int cx,
                                                              const long long* __restrict__ idx, int hw, int nm,
                                                              ProjTable tab, const float* __restrict__ drouted,
                                                              float* __restrict__ part) {
  __shared__ float red[RT_NT / 64][2 * C];
  const int b = blockIdx.x;
  const int m = clamp_mod(idx[b], nm);
  const float* W = tab.w[m];
  const float* B = tab.b[m];
  float sw[C], sb[C];
#pragma unroll
  for (int c = 0; c < C; ++c) sw[c] = sb[c] = 0.f;
  if (W != nullptr) {
    for (int p = threadIdx.x; p < hw; p += RT_NT) {
      const float g = nz(x[((long long)b * hw + p) * cx]);
      const float* d = drouted + ((long long)b * hw + p) * C;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float v = fmaf(W[c], g, B ? B[c] : 0.f);
        const float dd = v != v ? 0.f : d[c];  // the NaN scrub passes no gradient where it fired
        sw[c] = fmaf(dd, g, sw[c]);
        sb[c] += dd;
      }
    }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    sw[c] = wave_sum_f(sw[c]);
    sb[c] = wave_sum_f(sb[c]);
    if (lane == 0) {
      red[wv][c] = sw[c];
      red[wv][C + c] = sb[c];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * C) {
    float s = 0.f;
    for (int q = 0; q < RT_NT / 64; ++q) s += red[q][threadIdx.x];
    part[(long long)b * 2 * C + threadIdx.x] = s;
  }
}

template <int C>
__global__ void __launch_bounds__(256) route_in_grad_reduce_kernel(const float* __restrict__ part,
                                                                   const long long* __restrict__ idx, int nb, int nm,
                                                                   ProjGrad g) {
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;  // one wave per (modality, param)
  if (t >= nm * 2 * C) return;
  const int m = t / (2 * C), q = t - m * 2 * C;
  float s = 0.f;
  for (int b = lane; b < nb; b += 64)
    if (clamp_mod(idx[b], nm) == m) s += part[(long long)b * 2 * C + q];
  s = wave_sum_f(s);
  float* dst = q < C ? g.w[m] : g.b[m];
  if (lane == 0 && dst != nullptr) dst[q < C ? q : q - C] += s;
}

static size_t heads_lds_bytes(int h, int w, int c, bool bwd) {
  const size_t S = (size_t)(h + 2) * (w + 2) * c;
  return (bwd ? 4 * S + (size_t)h * w * c : 2 * S) * sizeof(float);
}
constexpr size_t RT_LDS_MAX = 160 * 1024;

static int head_params(int c) { return 2 * (c * 9 * c + c) + 1 * c + 1; }  // CM = 1

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_modality_heads_workspace_bytes(int nb, int c) { return (size_t)nb * head_params(c) * sizeof(float); }

static bool table_ok(int nm, int c) { return nm >= 1 && nm <= RT_MAXM && c == 3; }

int mvae_modality_heads_fwd(const float* rec, const long long* idx, int nb, int h, int w, int c, int nm,
                            const void* const* table, int out_c, float* out, void* stream) {
  if (!table_ok(nm, c) || nb < 0 || h < 1 || w < 1 || out_c < 1 || out_c > 8 || !rec || !idx || !out || !table ||
      heads_lds_bytes(h, w, c, false) > RT_LDS_MAX) {
    set_error("modality_heads_fwd: bad arguments (c must be 3, nm <= %d, image must fit LDS)", RT_MAXM);
    return MVAE_EINVAL;
  }
  if (nb == 0) return MVAE_OK;
  HeadTable t{};
  for (int m = 0; m < nm; ++m) {
    t.w1[m] = (const float*)table[6 * m + 0];
    t.b1[m] = (const float*)table[6 * m + 1];
    t.w2[m] = (const float*)table[6 * m + 2];
    t.b2[m] = (const float*)table[6 * m + 3];
    t.pw[m] = (const float*)table[6 * m + 4];
    t.pb[m] = (const float*)table[6 * m + 5];
    t.cm[m] = 1;
    if (!t.w1[m] || !t.w2[m]) {
      set_error("modality_heads_fwd: modality %d has no head weights", m);
      return MVAE_EINVAL;
    }
  }
  const size_t lds = heads_lds_bytes(h, w, c, false);
  hipLaunchKernelGGL(heads_fwd_kernel<3>, dim3(nb), dim3(RT_NT), lds, (hipStream_t)stream, rec, idx, h, w, nm, t, out_c,
                     out);
  return launch_status();
}

int mvae_modality_heads_bwd(const float* rec, const long long* idx, int nb, int h, int w, int c, int nm,
                            const void* const* table, int out_c, const float* dout, float* drec,
                            void* const* grad_table, void* workspace, size_t ws_bytes, void* stream) {
  if (!table_ok(nm, c) || nb < 0 || h < 1 || w < 1 || out_c < 1 || out_c > 8 || !rec || !idx || !dout || !drec ||
      !table || !grad_table || heads_lds_bytes(h, w, c, true) > RT_LDS_MAX) {
    set_error("modality_heads_bwd: bad arguments");
    return MVAE_EINVAL;
  }
  if (nb == 0) return MVAE_OK;
  if (ws_bytes < mvae_modality_heads_workspace_bytes(nb, c) || !workspace) {
    set_error("modality_heads_bwd: workspace too small");
    return MVAE_EWORKSPACE;
  }
  HeadTable t{};
  HeadGrad g{};
  for (int m = 0; m < nm; ++m) {
    t.w1[m] = (const float*)table[6 * m + 0];
    t.b1[m] = (const float*)table[6 * m + 1];
    t.w2[m] = (const float*)table[6 * m + 2];
    t.b2[m] = (const float*)table[6 * m + 3];
    t.pw[m] = (const float*)table[6 * m + 4];
    t.pb[m] = (const float*)table[6 * m + 5];
    t.cm[m] = 1;
    g.w1[m] = (float*)grad_table[6 * m + 0];
    g.b1[m] = (float*)grad_table[6 * m + 1];
    g.w2[m] = (float*)grad_table[6 * m + 2];
    g.b2[m] = (float*)grad_table[6 * m + 3];
    g.pw[m] = (float*)grad_table[6 * m + 4];
    g.pb[m] = (float*)grad_table[6 * m + 5];
    if (!t.w1[m] || !t.w2[m]) {
      set_error("modality_heads_bwd: modality %d has no head weights", m);
      return MVAE_EINVAL;
    }
  }
  float* part = (float*)workspace;
  const size_t lds = heads_lds_bytes(h, w, c, true);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL((heads_bwd_kernel<3, 1>), dim3(nb), dim3(RT_NT), lds, st, rec, idx, h, w, nm, t, out_c, dout, drec,
                     part);
  const int tot = nm * HeadLayout<3, 1>::P;
  hipLaunchKernelGGL((heads_grad_reduce_kernel<3, 1>), dim3((tot + 3) / 4), dim3(256), 0, st, part, idx, nb, nm, g);
  return launch_status();
}

size_t mvae_modality_route_in_workspace_bytes(int nb, int c) { return (size_t)nb * 2 * c * sizeof(float); }

int mvae_modality_route_in_fwd(const float* x, int cx, const long long* idx, int nb, int hw, int c, int nm,
                               const void* const* table, float* routed, void* stream) {
  if (!table_ok(nm, c) || nb < 0 || hw < 1 || cx < 1 || !x || !idx || !routed || !table) {
    set_error("modality_route_in_fwd: bad arguments");
    return MVAE_EINVAL;
  }
  if (nb == 0) return MVAE_OK;
  ProjTable t{};
  for (int m = 0; m < nm; ++m) {
    t.w[m] = (const float*)table[2 * m];
    t.b[m] = (const float*)table[2 * m + 1];
  }
  hipLaunchKernelGGL(route_in_fwd_kernel<3>, dim3((hw + 255) / 256, nb), dim3(256), 0, (hipStream_t)stream, x, cx, idx, hw,
                     nm, t, routed);
  return launch_status();
}

int mvae_modality_route_in_bwd(const float* x, int cx, const long long* idx, int nb, int hw, int c, int nm,
                               const void* const* table, const float* drouted, void* const* grad_table, void* workspace,
                               size_t ws_bytes, void* stream) {
  if (!table_ok(nm, c) || nb < 0 || hw < 1 || cx < 1 || !x || !idx || !drouted || !table || !grad_table) {
    set_error("modality_route_in_bwd: bad arguments");
    return MVAE_EINVAL;
  }
  if (nb == 0) return MVAE_OK;
  if (ws_bytes < mvae_modality_route_in_workspace_bytes(nb, c) || !workspace) {
    set_error("modality_route_in_bwd: workspace too small");
    return MVAE_EWORKSPACE;
  }
  ProjTable t{};
  ProjGrad g{};
  for (int m = 0; m < nm; ++m) {
    t.w[m] = (const float*)table[2 * m];
    t.b[m] = (const float*)table[2 * m + 1];
    g.w[m] = (float*)grad_table[2 * m];
    g.b[m] = (float*)grad_table[2 * m + 1];
  }
  float* part = (float*)workspace;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(route_in_bwd_kernel<3>, dim3(nb), dim3(RT_NT), 0, st, x, cx, idx, hw, nm, t, drouted, part);
  hipLaunchKernelGGL(route_in_grad_reduce_kernel<3>, dim3(cdiv(nm * 2 * 3, 4)), dim3(256), 0, st, part, idx, nb, nm, g);
  return launch_status();
}

}  // extern "C"
