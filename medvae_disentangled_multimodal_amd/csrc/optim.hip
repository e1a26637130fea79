// Fused optimizer step over ONE flat fp32 parameter/gradient/moment buffer (multi-tensor):
//   on_before_optimizer_step: a tensor with any non-finite gradient has its whole grad zeroed
//       (lightning_module.py:468-477, per tensor, no host sync: flags stay on the device)
//   configure_gradient_clipping: global L2 norm clip, coef = min(max_norm/(norm+1e-6), 1)
//       (lightning_module.py:452-466 -> torch.nn.utils.clip_grad_norm_)
//   configure_optimizers: Adam (L2 weight decay) / AdamW (decoupled) with per-tensor step counts
//       (lightning_module.py:390-408 -> torch.optim single-tensor arithmetic)
// Tensors whose gradient is absent this step (`used[t] == 0`, e.g. heads of modalities that are
// not in the batch) are skipped exactly like torch skips params with grad None.
#include "common.h"

namespace mvae {

struct MtArgs {
  float* p; float* g; float* m; float* v;
  const int* chunk_tensor; const long long* chunk_start; const int* chunk_len;
  const int* tensor_chunk_begin;  // [T+1]
  const int* used; int* step; int* bad;
  double* chunk_sumsq; int* chunk_bad;
  float* scalars;  // [0] total norm, [1] clip coef
  int T, nchunks;
  float gscale;
};

__global__ void __launch_bounds__(256) mt_chunk_stats_kernel(MtArgs a) {
  __shared__ double sh[4];
  __shared__ int shb[4];
  const int ch = blockIdx.x;
  const long long s = a.chunk_start[ch];
  const int len = a.chunk_len[ch];
  double acc = 0;
  int badf = 0;
  const int body = (s & 3) == 0 ? (len & ~3) : 0;
  for (int i = threadIdx.x * 4; i < body; i += blockDim.x * 4) {
    const float4 g4 = *(const float4*)(a.g + s + i);
    const float xs[4] = {g4.x * a.gscale, g4.y * a.gscale, g4.z * a.gscale, g4.w * a.gscale};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!isfinite(xs[e])) badf = 1;
      acc += (double)xs[e] * xs[e];
    }
  }
  for (int i = body + threadIdx.x; i < len; i += blockDim.x) {
    const float x = a.g[s + i] * a.gscale;
    if (!isfinite(x)) badf = 1;
    acc += (double)x * x;
  }
  acc = wave_sum_d(acc);
  badf = __any(badf) ? 1 : 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { sh[w] = acc; shb[w] = badf; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    int b = 0;
    for (int i = 0; i < 4; ++i) { t += sh[i]; b |= shb[i]; }
    a.chunk_sumsq[ch] = t;
    a.chunk_bad[ch] = b;
  }
}

__global__ void __launch_bounds__(256) mt_finalize_kernel(MtArgs a, float max_norm, int do_clip) {
  __shared__ double sh[4];
  double acc = 0;
  for (int t = threadIdx.x; t < a.T; t += blockDim.x) {
    double s = 0;
    int b = 0;
    for (int c = a.tensor_chunk_begin[t]; c < a.tensor_chunk_begin[t + 1]; ++c) {
      s += a.chunk_sumsq[c];
      b |= a.chunk_bad[c];
    }
    a.bad[t] = b;
    if (a.used[t]) {
      a.step[t] += 1;
      if (!b) acc += s;
    }
  }
  acc = wave_sum_d(acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double tot = sqrt(sh[0] + sh[1] + sh[2] + sh[3]);
    float coef = 1.f;
    if (do_clip) {
      coef = (float)((double)max_norm / (tot + 1e-6));
      if (coef > 1.f) coef = 1.f;
    }
    a.scalars[0] = (float)tot;
    a.scalars[1] = coef;
  }
}

__global__ void __launch_bounds__(256) mt_adam_kernel(MtArgs a, float lr, float b1, float b2, float eps, float wd,
                                                      int decoupled) {
  const int ch = blockIdx.x;
  const int t = a.chunk_tensor[ch];
  if (!a.used[t]) return;
  const long long s = a.chunk_start[ch];
  const int len = a.chunk_len[ch];
  const bool zero = a.bad[t] != 0;
  const float coef = a.scalars[1];
  const int step = a.step[t];
  const double bc1 = 1.0 - pow((double)b1, (double)step);
  const double bc2 = 1.0 - pow((double)b2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float decay = (float)(1.0 - (double)lr * (double)wd);
  const float w = 1.f - b1;
  // one element of the update (torch.optim.Adam/AdamW single-tensor arithmetic, in its operation order)
  auto upd = [&](float g, float& p, float& m, float& v) -> float {
    g = zero ? 0.f : g * a.gscale;
    g = g * coef;
    const float gout = g;
    if (decoupled) p = p * decay;
    else if (wd != 0.f) g = g + wd * p;
    m = (w < 0.5f) ? m + w * (g - m) : g - (g - m) * (1.f - w);
    v = v * b2 + (1.f - b2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + (-step_size) * (m / denom);
    return gout;
  };
  // 16-B body (flat-buffer tensors are 16-B aligned), scalar tail
  const int body = (s & 3) == 0 ? (len & ~3) : 0;
  for (int i = threadIdx.x * 4; i < body; i += blockDim.x * 4) {
    const long long e = s + i;
    float4 g4 = *(const float4*)(a.g + e), p4 = *(const float4*)(a.p + e);
    float4 m4 = *(const float4*)(a.m + e), v4 = *(const float4*)(a.v + e);
    g4.x = upd(g4.x, p4.x, m4.x, v4.x);
    g4.y = upd(g4.y, p4.y, m4.y, v4.y);
    g4.z = upd(g4.z, p4.z, m4.z, v4.z);
    g4.w = upd(g4.w, p4.w, m4.w, v4.w);
    *(float4*)(a.g + e) = g4;
    *(float4*)(a.p + e) = p4;
    *(float4*)(a.m + e) = m4;
    *(float4*)(a.v + e) = v4;
  }
  for (int i = body + threadIdx.x; i < len; i += blockDim.x) {
    const long long e = s + i;
    float g = zero ? 0.f : a.g[e] * a.gscale;
    g = g * coef;
    a.g[e] = g;
    float p = a.p[e];
    if (decoupled) p = p * decay;
    else if (wd != 0.f) g = g + wd * p;
    float m = a.m[e];
    m = (w < 0.5f) ? m + w * (g - m) : g - (g - m) * (1.f - w);
    float v = a.v[e] * b2 + (1.f - b2) * g * g;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p = p + (-step_size) * (m / denom);
    a.m[e] = m;
    a.v[e] = v;
    a.p[e] = p;
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

// One optimizer step over flat buffers. chunk tables / tensor_chunk_begin describe how the flat
// buffer splits into tensors (host-built once). Workspace: chunk_sumsq (double[nchunks]),
// chunk_bad (int[nchunks]), bad (int[T]); scalars: float[2] out (total norm, clip coef).
int mvae_multi_tensor_adam(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const int* chunk_tensor,
                           const long long* chunk_start, const int* chunk_len, int nchunks,
                           const int* tensor_chunk_begin, int ntensors, const int* used, int* step, float grad_scale,
                           float max_norm, int do_clip, float lr, float beta1, float beta2, float eps,
                           float weight_decay, int decoupled, void* workspace, size_t workspace_bytes, float* scalars,
                           void* stream) {
  const size_t need = (size_t)nchunks * (sizeof(double) + sizeof(int)) + (size_t)ntensors * sizeof(int) + 64;
  if (nchunks <= 0 || ntensors <= 0) { set_error("adam: empty"); return MVAE_EINVAL; }
  if (workspace_bytes < need) { set_error("adam: workspace too small"); return MVAE_EWORKSPACE; }
  MtArgs a{};
  a.p = params; a.g = grads; a.m = exp_avg; a.v = exp_avg_sq;
  a.chunk_tensor = chunk_tensor; a.chunk_start = chunk_start; a.chunk_len = chunk_len;
  a.tensor_chunk_begin = tensor_chunk_begin; a.used = used; a.step = step;
  a.chunk_sumsq = (double*)workspace;
  a.chunk_bad = (int*)((char*)workspace + (size_t)nchunks * sizeof(double));
  a.bad = a.chunk_bad + nchunks;
  a.scalars = scalars; a.T = ntensors; a.nchunks = nchunks; a.gscale = grad_scale;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(mt_chunk_stats_kernel, dim3(nchunks), dim3(256), 0, st, a);
  hipLaunchKernelGGL(mt_finalize_kernel, dim3(1), dim3(256), 0, st, a, max_norm, do_clip);
  hipLaunchKernelGGL(mt_adam_kernel, dim3(nchunks), dim3(256), 0, st, a, lr, beta1, beta2, eps, weight_decay,
                     decoupled);
  return launch_status();
}

size_t mvae_multi_tensor_adam_workspace_bytes(int nchunks, int ntensors) {
  return (size_t)nchunks * (sizeof(double) + sizeof(int)) + (size_t)ntensors * sizeof(int) + 64;
}

}  // extern "C"
