// Reparameterization, KL and reconstruction (MSE) terms of the VAE objective.
//   reparameterize  z = mu + eps * exp(0.5*logvar)                 base_vae.py:83-87
//   KL(N(mu, e^{lv/2}) || N(0,1)) = 0.5*(s^2 + mu^2 - 1 - log s^2)  torch.distributions (vae_losses.py:58)
//   MSE mean                                                       vae_losses.py:41-42
// mu / logvar are channel slices of the encoder's [pixels][2z] output (row stride `ld`), so no
// chunk copy is needed. Reductions are deterministic: fp64 block partials, then one fixed-order pass.
#include "common.h"
#include <algorithm>

namespace mvae {

constexpr int RED_BLOCKS = 1024;

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double t = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  return t;  // valid in thread 0
}

__global__ void __launch_bounds__(256) reparam_fwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                                          long long ld, const float* __restrict__ eps,
                                                          float* __restrict__ z, long long npix, int zc) {
  const long long n = npix * zc;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / zc;
    const int c = (int)(e - p * zc);
    const float m = mu[p * ld + c], l = lv[p * ld + c];
    z[e] = m + eps[e] * expf(0.5f * l);
  }
}

// dlogvar = dz * eps * 0.5 * exp(0.5*logvar)   (dmu = dz is passed through by the host)
__global__ void __launch_bounds__(256) reparam_bwd_kernel(const float* __restrict__ dz, const float* __restrict__ eps,
                                                          const float* __restrict__ lv, long long ld,
                                                          float* __restrict__ dlv, long long npix, int zc) {
  const long long n = npix * zc;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / zc;
    const int c = (int)(e - p * zc);
    dlv[e] = dz[e] * eps[e] * 0.5f * expf(0.5f * lv[p * ld + c]);
  }
}

// kind 0: KL elementwise sum (torch.distributions form) ; kind 1: squared error sum ;
// kind 2: absolute error sum ; kind 3: "-0.5*(1 + lv - mu^2 - exp(lv))" sum (DisentangledVAELoss);
// kinds 4-6 (discriminator hinge / generator terms, vae_losses.py:297-352): relu(1-a), relu(1+a), a
__global__ void __launch_bounds__(256) reduce_partial_kernel(int kind, const float* __restrict__ a,
                                                             const float* __restrict__ b, long long ld, long long npix,
                                                             int zc, double* __restrict__ part) {
  __shared__ double sh[4];
  const long long n = npix * zc;
  double acc = 0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    if (kind == 0 || kind == 3) {
      const long long p = e / zc;
      const int c = (int)(e - p * zc);
      const float m = a[p * ld + c], l = b[p * ld + c];
      if (kind == 0) {
        const float s = expf(0.5f * l);
        const float r = s * s;
        acc += 0.5f * (r + m * m - 1.f - logf(r));
      } else {
        acc += 1.f + l - m * m - expf(l);
      }
    } else if (kind >= 4) {  // adversarial terms on logits a: relu(1 - a), relu(1 + a), a
      const float v = a[e];
      acc += kind == 4 ? (double)fmaxf(1.f - v, 0.f) : kind == 5 ? (double)fmaxf(1.f + v, 0.f) : (double)v;
    } else {
      const float d = a[e] - b[e];
      acc += kind == 1 ? (double)d * d : (double)fabsf(d);
    }
  }
  const double t = block_sum_d(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ void reduce_final_kernel(const double* __restrict__ part, int nparts, double scale, float* out) {
  __shared__ double sh[4];
  double acc = 0;
  // fixed assignment of partials to threads + fixed-order combine => deterministic
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  const double t = block_sum_d(acc, sh);
  if (threadIdx.x == 0) out[0] = (float)(t * scale);
}

// dmu = g*mu ; dlv = g*0.5*(exp(lv) - 1), g = gscale[0] * mult (device scalar, no host sync)
// kind 0: torch KL form, kind 3: Disentangled closed form (same derivative)
__global__ void __launch_bounds__(256) kl_bwd_kernel(const float* __restrict__ mu, const float* __restrict__ lv,
                                                     long long ld, const float* __restrict__ gscale, double mult,
                                                     float* __restrict__ dmu, float* __restrict__ dlv, long long npix,
                                                     int zc) {
  const float g = (float)(gscale[0] * mult);
  const long long n = npix * zc;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / zc;
    const int c = (int)(e - p * zc);
    const float m = mu[p * ld + c], l = lv[p * ld + c];
    const float s = expf(0.5f * l);
    dmu[e] = g * m;
    dlv[e] = g * 0.5f * (s * s - 1.f);
  }
}

// d/da of the adversarial terms (kinds 4-6) times gscale[0] * mult
__global__ void __launch_bounds__(256) adv_bwd_kernel(int kind, const float* __restrict__ a,
                                                      const float* __restrict__ gscale, double mult,
                                                      float* __restrict__ da, long long n) {
  const float g = (float)(gscale[0] * mult);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float v = a[e];
    da[e] = kind == 4 ? (1.f - v > 0.f ? -g : 0.f) : kind == 5 ? (1.f + v > 0.f ? g : 0.f) : g;
  }
}

// d/da of mean((a-b)^2) or mean|a-b| times upstream gradient gscale[0]
__global__ void __launch_bounds__(256) recon_bwd_kernel(int kind, const float* __restrict__ a,
                                                        const float* __restrict__ b, const float* __restrict__ gscale,
                                                        double mult, float* __restrict__ da, long long n) {
  const float g = (float)(gscale[0] * mult);
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float d = a[e] - b[e];
    da[e] = kind == 1 ? g * 2.f * d : g * (float)((d > 0.f) - (d < 0.f));
  }
}

// Latent preparation of the disentangled model, one pass (disentangled_conditional_vae.py:388-398 on the
// encode output of :255-301, base_vae.py:83-87): with the NaN scrub of encode,
//   mu = clamp(nan0(h_mu), -10, 10), lv = clamp(nan0(h_lv), -10, 10), s = exp(0.5 lv),
//   z = mu + eps * s, std = clamp(s, 1e-6, 10)
// replacing the isnan / where / clamp / exp / mul / clamp chain and the reparameterization launch.
__global__ void __launch_bounds__(256) latent_prep_fwd_kernel(const float* __restrict__ hm, const float* __restrict__ hl,
                                                              long long ld, const float* __restrict__ eps,
                                                              float* __restrict__ mu, float* __restrict__ lv,
                                                              float* __restrict__ sd, float* __restrict__ z,
                                                              long long npix, int zc) {
  const long long n = npix * zc;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / zc;
    const int c = (int)(e - p * zc);
    float m = hm[p * ld + c], l = hl[p * ld + c];
    m = fminf(fmaxf(m != m ? 0.f : m, -10.f), 10.f);
    l = fminf(fmaxf(l != l ? 0.f : l, -10.f), 10.f);
    const float s = expf(0.5f * l);
    mu[e] = m;
    lv[e] = l;
    sd[e] = fminf(fmaxf(s, 1e-6f), 10.f);
    z[e] = m + eps[e] * s;
  }
}

// Backward of latent_prep_fwd as torch's autograd composes it: the incoming gradients of mu / lv / std / z (null = 0)
// give d(h_mu) = [h_mu not NaN, -10 <= h_mu <= 10] (g_mu + g_z) and d(h_lv) = [same for h_lv] (g_lv + g_z eps s/2 +
// [1e-6 <= s <= 10] g_std s/2), written at row stride ldo (straight into the gradient of the encoder's [pixels][2 zc]
// output: no chunk / cat / accumulation launches).
__global__ void __launch_bounds__(256) latent_prep_bwd_kernel(const float* __restrict__ hm, const float* __restrict__ hl,
                                                              long long ld, const float* __restrict__ eps,
                                                              const float* __restrict__ gmu,
                                                              const float* __restrict__ glv,
                                                              const float* __restrict__ gsd,
                                                              const float* __restrict__ gz, float* __restrict__ dm,
                                                              float* __restrict__ dl, long long ldo, long long npix,
                                                              int zc) {
  const long long n = npix * zc;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const long long p = e / zc;
    const int c = (int)(e - p * zc);
    const float m = hm[p * ld + c], l = hl[p * ld + c];
    const float lc = fminf(fmaxf(l != l ? 0.f : l, -10.f), 10.f);
    const float s = expf(0.5f * lc);
    const float g_z = gz ? gz[e] : 0.f;
    const float g_m = (gmu ? gmu[e] : 0.f) + g_z;
    float g_l = glv ? glv[e] : 0.f;
    g_l += g_z * eps[e] * 0.5f * s;
    if (gsd && s >= 1e-6f && s <= 10.f) g_l += gsd[e] * s * 0.5f;
    dm[p * ldo + c] = (m >= -10.f && m <= 10.f) ? g_m : 0.f;  // NaN compares false: scrubbed values get 0
    dl[p * ldo + c] = (l >= -10.f && l <= 10.f) ? g_l : 0.f;
  }
}

// The weighted total of up to 4 scalar loss terms with DisentangledVAELoss's non-finite handling
// (disentangled_conditional_vae.py:528-565): out[1 + i] = v_i if finite else 0, out[0] = sum_i w_i out[1 + i] in
// order (fp32, no contraction: torch's 0-d arithmetic), replaced by `nonfinite_total` when it is not finite.
// flags[i] = v_i finite, flags[nt] = total finite (read by the backward). One thread, one launch.
// a product rounded to fp32 before any following add (hipcc's default -ffp-contract=fast ignores the contract
// pragma; the empty asm keeps the multiply and the add separate, as torch's 0-d arithmetic rounds them)
__device__ __forceinline__ float mul_rounded(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}

struct CombineArgs {
  const float* v[4];
  float w[4];
  float* o[5];  // forward: total, then the finite-or-zero terms (separate 0-d tensors)
};

__global__ void __launch_bounds__(64) loss_combine_fwd_entry(CombineArgs a, int nt, float nonfinite_total,
                                                             float* __restrict__ flags) {
  if (threadIdx.x != 0) return;
  float tot = 0.f;
  for (int i = 0; i < nt; ++i) {
    const float x = *a.v[i];
    const bool ok = isfinite(x);
    const float f = ok ? x : 0.f;
    *a.o[1 + i] = f;
    flags[i] = ok ? 1.f : 0.f;
    tot = i == 0 ? mul_rounded(a.w[i], f) : tot + mul_rounded(a.w[i], f);
  }
  const bool okt = isfinite(tot);
  *a.o[0] = okt ? tot : nonfinite_total;
  flags[nt] = okt ? 1.f : 0.f;
}

__global__ void __launch_bounds__(64) loss_combine_bwd_entry(CombineArgs a, int nt, const float* __restrict__ flags,
                                                             const float* __restrict__ gtot, float* __restrict__ g) {
  if (threadIdx.x != 0) return;
  const float gt = (gtot && flags[nt] != 0.f) ? *gtot : 0.f;
  for (int i = 0; i < nt; ++i) {
    const float go = a.v[i] ? *a.v[i] : 0.f;  // a.v holds the incoming gradients of the per-term outputs here
    g[i] = flags[i] != 0.f ? go + mul_rounded(a.w[i], gt) : 0.f;  // [v_i finite](g_out_i + w_i g_total)
  }
}

static int egrid(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_reduce_workspace_bytes(void) { return RED_BLOCKS * sizeof(double); }

int mvae_reparam_fwd(const float* mu, const float* logvar, long long ld, const float* eps, float* z, long long npix,
                     int zc, void* stream) {
  if (npix <= 0 || zc <= 0 || ld < zc) { set_error("reparam: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(reparam_fwd_kernel, dim3(egrid(npix * zc)), dim3(256), 0, (hipStream_t)stream, mu, logvar, ld,
                     eps, z, npix, zc);
  return launch_status();
}

int mvae_reparam_bwd(const float* dz, const float* eps, const float* logvar, long long ld, float* dlogvar,
                     long long npix, int zc, void* stream) {
  if (npix <= 0 || zc <= 0 || ld < zc) { set_error("reparam_bwd: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(reparam_bwd_kernel, dim3(egrid(npix * zc)), dim3(256), 0, (hipStream_t)stream, dz, eps,
                     logvar, ld, dlogvar, npix, zc);
  return launch_status();
}

// out[0] = scale * sum_e term(e); kind as in reduce_partial_kernel. For kinds 1/2, a and b are
// dense [n] (npix = n, zc = 1, ld unused).
int mvae_loss_reduce(int kind, const float* a, const float* b, long long ld, long long npix, int zc, double scale,
                     float* out, void* workspace, size_t workspace_bytes, void* stream) {
  if (kind < 0 || kind > 6 || npix <= 0 || zc <= 0) { set_error("loss_reduce: bad args"); return MVAE_EINVAL; }
  if (workspace_bytes < RED_BLOCKS * sizeof(double)) { set_error("loss_reduce: workspace"); return MVAE_EWORKSPACE; }
  hipStream_t st = (hipStream_t)stream;
  const long long n = npix * zc;
  const int blocks = (int)std::min<long long>(RED_BLOCKS, (n + 255) / 256);
  hipLaunchKernelGGL(reduce_partial_kernel, dim3(blocks), dim3(256), 0, st, kind, a, b, ld, npix, zc,
                     (double*)workspace);
  hipLaunchKernelGGL(reduce_final_kernel, dim3(1), dim3(256), 0, st, (const double*)workspace, blocks, scale, out);
  return launch_status();
}

int mvae_kl_bwd(const float* mu, const float* logvar, long long ld, const float* gscale, double mult, float* dmu,
                float* dlogvar, long long npix, int zc, void* stream) {
  if (npix <= 0 || zc <= 0) { set_error("kl_bwd: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(kl_bwd_kernel, dim3(egrid(npix * zc)), dim3(256), 0, (hipStream_t)stream, mu, logvar, ld, gscale,
                     mult, dmu, dlogvar, npix, zc);
  return launch_status();
}

int mvae_recon_bwd(int kind, const float* a, const float* b, const float* gscale, double mult, float* da, long long n,
                   void* stream) {
  if ((kind != 1 && kind != 2) || n <= 0) { set_error("recon_bwd: bad args"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(recon_bwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, kind, a, b, gscale, mult, da,
                     n);
  return launch_status();
}

int mvae_latent_prep_fwd(const float* h_mu, const float* h_logvar, long long ld, const float* eps, float* mu,
                         float* logvar, float* std_out, float* z, long long npix, int zc, void* stream) {
  if (npix <= 0 || zc <= 0 || ld < zc || !h_mu || !h_logvar || !eps || !mu || !logvar || !std_out || !z) {
    set_error("latent_prep_fwd: bad args");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(latent_prep_fwd_kernel, dim3(egrid(npix * zc)), dim3(256), 0, (hipStream_t)stream, h_mu, h_logvar,
                     ld, eps, mu, logvar, std_out, z, npix, zc);
  return launch_status();
}

int mvae_latent_prep_bwd(const float* h_mu, const float* h_logvar, long long ld, const float* eps, const float* g_mu,
                         const float* g_logvar, const float* g_std, const float* g_z, float* d_mu, float* d_logvar,
                         long long ld_out, long long npix, int zc, void* stream) {
  if (npix <= 0 || zc <= 0 || ld < zc || ld_out < zc || !h_mu || !h_logvar || !eps || !d_mu || !d_logvar) {
    set_error("latent_prep_bwd: bad args");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(latent_prep_bwd_kernel, dim3(egrid(npix * zc)), dim3(256), 0, (hipStream_t)stream, h_mu, h_logvar,
                     ld, eps, g_mu, g_logvar, g_std, g_z, d_mu, d_logvar, ld_out, npix, zc);
  return launch_status();
}

int mvae_loss_combine4_fwd(const float* v0, const float* v1, const float* v2, const float* v3, float w0, float w1,
                           float w2, float w3, int nt, float nonfinite_total, float* total, float* o0, float* o1,
                           float* o2, float* o3, float* flags, void* stream) {
  CombineArgs a{{v0, v1, v2, v3}, {w0, w1, w2, w3}, {total, o0, o1, o2, o3}};
  if (nt < 1 || nt > 4 || !total || !flags) { set_error("loss_combine4_fwd: bad args"); return MVAE_EINVAL; }
  for (int i = 0; i < nt; ++i)
    if (!a.v[i] || !a.o[1 + i]) { set_error("loss_combine4_fwd: null term"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(loss_combine_fwd_entry, dim3(1), dim3(64), 0, (hipStream_t)stream, a, nt, nonfinite_total, flags);
  return launch_status();
}

int mvae_loss_combine4_bwd(const float* flags, float w0, float w1, float w2, float w3, int nt, const float* g_total,
                           const float* g0, const float* g1, const float* g2, const float* g3, float* g_terms,
                           void* stream) {
  CombineArgs a{{g0, g1, g2, g3}, {w0, w1, w2, w3}, {}};
  if (nt < 1 || nt > 4 || !flags || !g_terms) { set_error("loss_combine4_bwd: bad args"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(loss_combine_bwd_entry, dim3(1), dim3(64), 0, (hipStream_t)stream, a, nt, flags, g_total,
                     g_terms);
  return launch_status();
}

int mvae_adv_bwd(int kind, const float* a, const float* gscale, double mult, float* da, long long n, void* stream) {
  if (kind < 4 || kind > 6 || n <= 0) { set_error("adv_bwd: bad args"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(adv_bwd_kernel, dim3(egrid(n)), dim3(256), 0, (hipStream_t)stream, kind, a, gscale, mult, da, n);
  return launch_status();
}

}  // extern "C"
