// Batch-coupled latent losses of DisentangledConditionalVAE, fused (src/models/disentangled_conditional_vae.py):
//   partition_latent (:195-206)            zm[b][j] = z.view(B, -1)[b][off + j]   (NCHW flatten order)
//   modality_separation_loss (:305-349)    -mean pdist of the centroids of every distinct id (torch.unique order)
//   contrastive_loss (:351-386)            masked InfoNCE over zn = normalize(zm), temperature T
// The torch formulation issues ~90 small launches per step (sort, scatter, [B,B] masks and exps, reductions, their
// autograd) and materialises [B,B,D] centroid differences. Here: four launches per step, no [B,B] tensor.
//   fwd_rows  (B/16 blocks): per row i of the contrastive term, e_ij = exp(zn_i . zn_j / T) over all j:
//             ps_i = sum_{j != i, id_j == id_i} e_ij, tot_i = sum_j e_ij - e_ii, l_i = -log(ps_i / tot_i + 1e-8)
//   fwd_final (1 block):   separation (distinct ids, centroids in index order, pairwise distances) and the mean of
//             l_i over rows with ps_i > 0 -> out[0] = separation, out[1] = contrastive
//   bwd_prep  (1 block):   separation gradient per sample (pdist / mean / centroid adjoints) and the per-row InfoNCE
//             coefficients; a non-finite forward value drops its term's gradient (DisentangledVAELoss replaces such
//             a term by 0, :540-550)
//   bwd_rows  (B/16 blocks): dzn_i = (1/T) sum_j (G_ij + G_ji) zn_j, the normalize adjoint, plus the separation part,
//             scattered into dz at the partition's NCHW positions (dz's other elements are zero)
// All sums run in a fixed order (deterministic); fp64 accumulation for the batch means.
#include "common.h"

namespace mvae {

constexpr int LAT_MAXD = 16;     // latent partition width
constexpr int LAT_MAXB = 1024;   // batch (one workgroup handles the O(B K) separation pass)
constexpr int LAT_ROWS = 16;     // contrastive rows per block (16 lanes per row)
constexpr int LAT_THREADS = 256;
constexpr int LAT_ROWW = 5;      // per-row workspace: ps, tot, l, has, neg

struct LatentArgs {
  const float* z;             // [B][C][HW] logical, stored NHWC (cl=1) or NCHW (cl=0)
  const long long* idx;       // [B]
  int B, D, C, HW, cl, off;   // partition = flat elements [off, off + D)
  float inv_t;                // 1 / temperature
  float* ws;                  // per row: ps, tot, l, has, neg; then dzsep [B][D], A[B], Bc[B]
  float* out;                 // [2]: separation, contrastive (+ [2] = valid-row count)
};

__device__ __forceinline__ long long lat_pos(const LatentArgs& a, int b, int j) {
  const int f = a.off + j;
  const int c = f / a.HW, p = f - (f / a.HW) * a.HW;
  return (long long)b * a.C * a.HW + (a.cl ? (long long)p * a.C + c : (long long)c * a.HW + p);
}

// zn of every row into LDS (fp32 norm in index order, F.normalize eps 1e-12)
__device__ void lat_load_zn(const LatentArgs& a, float* zn, float* nrm) {
  __shared__ int offs[LAT_MAXD];
  if (threadIdx.x < a.D) {
    const int f = a.off + threadIdx.x;
    const int c = f / a.HW, p = f - c * a.HW;
    offs[threadIdx.x] = a.cl ? p * a.C + c : c * a.HW + p;
  }
  __syncthreads();
  const long long per = (long long)a.C * a.HW;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    float v[LAT_MAXD];
    float ss = 0.f;
    for (int j = 0; j < a.D; ++j) {
      v[j] = a.z[b * per + offs[j]];
      ss += v[j] * v[j];
    }
    const float n = fmaxf(sqrtf(ss), 1e-12f);
    if (nrm) nrm[b] = sqrtf(ss);
    for (int j = 0; j < a.D; ++j) zn[b * a.D + j] = v[j] / n;
  }
}

__device__ __forceinline__ float lat_dot(const float* x, const float* y, int D) {
  float s = 0.f;
  for (int j = 0; j < D; ++j) s += x[j] * y[j];
  return s;
}

__global__ void __launch_bounds__(LAT_THREADS) latent_fwd_rows_kernel(LatentArgs a) {
  __shared__ float zn[LAT_MAXB * LAT_MAXD];
  __shared__ long long ids[LAT_MAXB];
  lat_load_zn(a, zn, nullptr);
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) ids[b] = a.idx[b];
  __syncthreads();
  const int r = threadIdx.x >> 4, l = threadIdx.x & 15;
  const int i = blockIdx.x * LAT_ROWS + r;
  float ps = 0.f, all = 0.f, eii = 0.f, neg = 0.f;
  if (i < a.B) {
    const float* zi = zn + i * a.D;
    for (int j = l; j < a.B; j += 16) {  // lane l takes columns l, l+16, ... ; fixed-order tree below
      const float e = __expf(lat_dot(zi, zn + j * a.D, a.D) * a.inv_t);
      all += e;
      if (j == i) eii = e;
      else if (ids[j] == ids[i]) ps += e;
      else neg += e;
    }
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    ps += __shfl_xor(ps, o, 16);
    all += __shfl_xor(all, o, 16);
    eii += __shfl_xor(eii, o, 16);
    neg += __shfl_xor(neg, o, 16);
  }
  if (i < a.B && l == 0) {
    const float tot = all - eii;
    float* w = a.ws + (long long)LAT_ROWW * i;
    w[0] = ps;
    w[1] = tot;
    w[2] = -logf(ps / tot + 1e-8f);
    w[3] = ps > 0.f ? 1.f : 0.f;
    w[4] = neg;
  }
}

// distinct ids in ascending order (torch.unique): fst[b] = no earlier sample has id_b (early exit: with few distinct
// ids almost every sample finds its match within a few entries); the K first samples take their rank among the
// distinct ids (O(B) each), every sample its segment by a scan of the K-entry sorted list, and each segment its
// multiplicity. seg[b] = #distinct ids < id_b; cnt[s], rep[s] = multiplicity and first sample of segment s.
__device__ void lat_segments(const LatentArgs& a, const long long* ids, int* fst, int* seg, int* cnt, int* rep,
                             int& K) {
  __shared__ long long dist[LAT_MAXB];
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const long long v = ids[b];
    int first = 1;
    for (int j = 0; j < b; ++j)
      if (ids[j] == v) {
        first = 0;
        break;
      }
    fst[b] = first;
  }
  __syncthreads();
  K = 0;
  for (int j = 0; j < a.B; ++j) K += fst[j];
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    if (!fst[b]) continue;
    int rnk = 0;
    for (int j = 0; j < a.B; ++j) rnk += fst[j] & (ids[j] < ids[b]);
    dist[rnk] = ids[b];
    rep[rnk] = b;
  }
  __syncthreads();
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    int lo = 0, hi = K - 1;  // binary search of id_b in the sorted distinct ids
    const long long v = ids[b];
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (dist[mid] < v) lo = mid + 1;
      else hi = mid;
    }
    seg[b] = lo;
  }
  __syncthreads();
  for (int s_ = threadIdx.x; s_ < K; s_ += blockDim.x) {
    int c = 0;
    for (int b = 0; b < a.B; ++b) c += seg[b] == s_;
    cnt[s_] = c;
  }
  __syncthreads();
}

// zm[b][j] of every sample into LDS (coalesced over the B*D elements; the NCHW offsets of the D partition elements
// computed once)
__device__ void lat_load_zm(const LatentArgs& a, float* zm) {
  __shared__ int offs[LAT_MAXD];
  if (threadIdx.x < a.D) {
    const int f = a.off + threadIdx.x;
    const int c = f / a.HW, p = f - c * a.HW;
    offs[threadIdx.x] = a.cl ? p * a.C + c : c * a.HW + p;
  }
  __syncthreads();
  const long long per = (long long)a.C * a.HW;
  for (int e = threadIdx.x; e < a.B * a.D; e += blockDim.x) {
    const int b = e / a.D, j = e - (e / a.D) * a.D;
    zm[e] = a.z[b * per + offs[j]];
  }
  __syncthreads();
}

// centroid of segment s (its samples in index order), fp32 like torch's mean: one thread per (segment, dim)
__device__ void lat_centroids(const LatentArgs& a, const long long* ids, const float* zm, const int* cnt,
                              const int* rep, int K, float* cen) {
  for (int e = threadIdx.x; e < K * a.D; e += blockDim.x) {
    const int s = e / a.D, q = e - (e / a.D) * a.D;
    const long long id = ids[rep[s]];
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b)
      if (ids[b] == id) acc += zm[b * a.D + q];
    cen[e] = acc / (float)cnt[s];
  }
  __syncthreads();
}

__device__ double lat_block_sum(double v, double* sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += sh[w];
  return t;
}

__global__ void __launch_bounds__(1024) latent_fwd_final_kernel(LatentArgs a) {
  __shared__ long long ids[LAT_MAXB];
  __shared__ int fst[LAT_MAXB], seg[LAT_MAXB], cnt[LAT_MAXB], rep[LAT_MAXB];
  __shared__ float cen[LAT_MAXB * LAT_MAXD];
  __shared__ float zm[LAT_MAXB * LAT_MAXD / 2];
  __shared__ double sh[16];
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) ids[b] = a.idx[b];
  lat_load_zm(a, zm);
  int K = 0;
  lat_segments(a, ids, fst, seg, cnt, rep, K);
  lat_centroids(a, ids, zm, cnt, rep, K, cen);
  // pairwise distances (i < j), summed in fp64
  double dsum = 0.0;
  const long long npair = (long long)K * (K - 1) / 2;
  for (int i = 0; i < K; ++i)
    for (int j = i + 1 + threadIdx.x; j < K; j += blockDim.x) {
      float d2 = 0.f;
      for (int q = 0; q < a.D; ++q) {
        const float d = cen[i * a.D + q] - cen[j * a.D + q];
        d2 += d * d;
      }
      dsum += (double)sqrtf(d2);
    }
  const double tot = lat_block_sum(dsum, sh);
  // contrastive mean over rows with positives
  double ls = 0.0, nv = 0.0;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const float* w = a.ws + (long long)LAT_ROWW * b;
    if (w[3] > 0.f) {
      ls += (double)w[2];
      nv += 1.0;
    }
  }
  const double lsum = lat_block_sum(ls, sh);
  const double nvalid = lat_block_sum(nv, sh);
  if (threadIdx.x == 0) {
    a.out[0] = npair > 0 ? (float)(-tot / (double)npair) : 0.f;
    a.out[1] = nvalid > 0 ? (float)(lsum / nvalid) : 0.f;
    a.out[2] = (float)nvalid;
  }
}

// gsep / gcon: upstream gradients (device scalars). Writes dzsep [B][D] and the row coefficients
// A_i = w_i * dl_i/dps_i, Bc_i = w_i * dl_i/dtot_i (w_i = gcon / n for rows with positives)
__global__ void __launch_bounds__(1024) latent_bwd_prep_kernel(LatentArgs a, const float* gsep, const float* gcon) {
  __shared__ long long ids[LAT_MAXB];
  __shared__ int fst[LAT_MAXB], seg[LAT_MAXB], cnt[LAT_MAXB], rep[LAT_MAXB];
  __shared__ float cen[LAT_MAXB * LAT_MAXD];
  __shared__ float zm[LAT_MAXB * LAT_MAXD / 2];
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) ids[b] = a.idx[b];
  lat_load_zm(a, zm);
  int K = 0;
  lat_segments(a, ids, fst, seg, cnt, rep, K);
  lat_centroids(a, ids, zm, cnt, rep, K, cen);
  float* dzsep = a.ws + (long long)LAT_ROWW * a.B;
  float* A = dzsep + (long long)a.B * a.D;
  float* Bc = A + a.B;
  const float sepv = a.out[0], conv_ = a.out[1], nvalid = a.out[2];
  const float gs = (K >= 2 && isfinite(sepv)) ? gsep[0] : 0.f;
  const float gc = (nvalid > 0.f && isfinite(conv_)) ? gcon[0] : 0.f;
  const float npair = (float)((long long)K * (K - 1) / 2);
  if (threadIdx.x == 0) Bc[a.B] = gc != 0.f ? 1.f : 0.f;  // contrastive gradient live (read by the rows pass)
  // d(-mean dist)/dc_s = -(1/npair) sum_{t != s} (c_s - c_t) / |c_s - c_t|, then / cnt_s to every member
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    const int s = seg[b];
    float g[LAT_MAXD];
    for (int q = 0; q < a.D; ++q) g[q] = 0.f;
    if (gs != 0.f) {
      for (int t = 0; t < K; ++t) {
        if (t == s) continue;
        float d2 = 0.f;
        for (int q = 0; q < a.D; ++q) {
          const float d = cen[s * a.D + q] - cen[t * a.D + q];
          d2 += d * d;
        }
        const float dist = sqrtf(d2);
        if (dist > 0.f)
          for (int q = 0; q < a.D; ++q) g[q] += (cen[s * a.D + q] - cen[t * a.D + q]) / dist;
      }
    }
    const float sc = gs != 0.f ? -gs / (npair * (float)cnt[s]) : 0.f;
    for (int q = 0; q < a.D; ++q) dzsep[b * a.D + q] = g[q] * sc;
    const float* w = a.ws + (long long)LAT_ROWW * b;
    const float ps = w[0], tot = w[1], neg = w[4];
    const float wi = (w[3] > 0.f && gc != 0.f) ? gc / nvalid : 0.f;
    const float inv = 1.f / (ps / tot + 1e-8f);
    // a positive e_ij enters ps and tot: dl/dps + dl/dtot = -inv (tot - ps) / tot^2 = -inv * neg / tot^2, taken
    // from the negatives' sum directly (no cancellation: exactly 0 when every other row is positive); a negative
    // e_ij enters tot only: dl/dtot = inv * ps / tot^2
    A[b] = wi * (-inv * neg / (tot * tot));
    Bc[b] = wi * (inv * ps / (tot * tot));
  }
}

__global__ void __launch_bounds__(LAT_THREADS) latent_bwd_rows_kernel(LatentArgs a, float* dz) {
  __shared__ float zn[LAT_MAXB * LAT_MAXD];
  __shared__ float nrm[LAT_MAXB], Ash[LAT_MAXB], Bsh[LAT_MAXB];
  __shared__ long long ids[LAT_MAXB];
  lat_load_zn(a, zn, nrm);
  const float* dzsep = a.ws + (long long)LAT_ROWW * a.B;
  const float* A = dzsep + (long long)a.B * a.D;
  const float* Bc = A + a.B;
  for (int b = threadIdx.x; b < a.B; b += blockDim.x) {
    ids[b] = a.idx[b];
    Ash[b] = A[b];
    Bsh[b] = Bc[b];
  }
  __syncthreads();
  const int r = threadIdx.x >> 4, l = threadIdx.x & 15;
  const int i = blockIdx.x * LAT_ROWS + r;
  const bool live = Bc[a.B] != 0.f;  // a gated (non-finite) contrastive term contributes nothing, NaN latents included
  float g[LAT_MAXD];
  for (int q = 0; q < LAT_MAXD; ++q) g[q] = 0.f;
  if (i < a.B && live) {
    const float* zi = zn + i * a.D;
    for (int j = l; j < a.B; j += 16) {
      if (j == i) continue;  // d tot / d e_ii = 0 (tot = sum - e_ii), and e_ii is never positive
      const float e = __expf(lat_dot(zi, zn + j * a.D, a.D) * a.inv_t);
      const bool pos = ids[j] == ids[i];
      // G_ij + G_ji (e symmetric): row i's and row j's coefficients (positives: A, negatives: Bc)
      const float c = e * (pos ? Ash[i] + Ash[j] : Bsh[i] + Bsh[j]) * a.inv_t;
      for (int q = 0; q < a.D; ++q) g[q] += c * zn[j * a.D + q];
    }
  }
  for (int q = 0; q < a.D; ++q) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) g[q] += __shfl_xor(g[q], o, 16);
  }
  if (i < a.B && l == 0) {
    // F.normalize adjoint: zn = x / max(|x|, eps)
    const float n = nrm[i];
    const float* zi = zn + i * a.D;
    float dot = 0.f;
    for (int q = 0; q < a.D; ++q) dot += zi[q] * g[q];
    for (int q = 0; q < a.D; ++q) {
      const float dx = !live ? 0.f : n > 1e-12f ? (g[q] - zi[q] * dot) / n : g[q] / 1e-12f;
      dz[lat_pos(a, i, q)] = dx + dzsep[i * a.D + q];
    }
  }
}

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_latent_aux_workspace_bytes(int nb, int d) { return ((size_t)nb * (LAT_ROWW + d + 2) + 1) * sizeof(float); }

static bool lat_args(LatentArgs& a, const float* z, const long long* idx, int nb, int c, int hw, int cl, int off,
                     int d, float temperature, float* out, float* ws, size_t ws_bytes, const char* who) {
  if (!z || !idx || !out || !ws || nb <= 0 || nb > LAT_MAXB || d <= 0 || d > LAT_MAXD || nb * d > LAT_MAXB * LAT_MAXD / 2 ||
      c <= 0 || hw <= 0 ||
      off < 0 || off + d > c * hw || !(temperature > 0.f)) {
    set_error("%s: bad arguments (nb=%d d=%d; needs nb <= %d, d <= %d)", who, nb, d, LAT_MAXB, LAT_MAXD);
    return false;
  }
  if (ws_bytes < mvae_latent_aux_workspace_bytes(nb, d)) {
    set_error("%s: workspace too small", who);
    return false;
  }
  a = LatentArgs{z, idx, nb, d, c, hw, cl, off, 1.f / temperature, ws, out};
  return true;
}

// out[0] = separation loss, out[1] = contrastive loss, out[2] = rows with positives (kept for the backward)
int mvae_latent_aux_fwd(const float* z, const long long* idx, int nb, int c, int hw, int cl, int off, int d,
                        float temperature, float* out, float* ws, size_t ws_bytes, void* stream) {
  LatentArgs a;
  if (!lat_args(a, z, idx, nb, c, hw, cl, off, d, temperature, out, ws, ws_bytes, "mvae_latent_aux_fwd"))
    return ws_bytes < mvae_latent_aux_workspace_bytes(nb > 0 ? nb : 1, d > 0 ? d : 1) ? MVAE_EWORKSPACE : MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(latent_fwd_rows_kernel, dim3(cdiv(nb, LAT_ROWS)), dim3(LAT_THREADS), 0, st, a);
  hipLaunchKernelGGL(latent_fwd_final_kernel, dim3(1), dim3(1024), 0, st, a);
  return launch_status();
}

// dz: [B][C][HW] (same layout as z), zero outside the partition (the caller zero-fills it); gsep / gcon: device
// scalars (upstream gradients); out / ws: from the forward
int mvae_latent_aux_bwd(const float* z, const long long* idx, int nb, int c, int hw, int cl, int off, int d,
                        float temperature, const float* out, const float* gsep, const float* gcon, float* dz, float* ws,
                        size_t ws_bytes, void* stream) {
  LatentArgs a;
  if (!dz || !gsep || !gcon ||
      !lat_args(a, z, idx, nb, c, hw, cl, off, d, temperature, const_cast<float*>(out), ws, ws_bytes,
                "mvae_latent_aux_bwd"))
    return MVAE_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(latent_bwd_prep_kernel, dim3(1), dim3(1024), 0, st, a, gsep, gcon);
  hipLaunchKernelGGL(latent_bwd_rows_kernel, dim3(cdiv(nb, LAT_ROWS)), dim3(LAT_THREADS), 0, st, a, dz);
  return launch_status();
}

}  // extern "C"
