// Small helpers of the convolution backward pass.
//   * weight re-layout for dgrad: KRSC [Cout][R][S][Cin] -> [Cin][R][S][Cout]
//   * dgrad weights of Upsample's conv (nearest x2 then 3x3, encoder_decoder.py:205-209): the
//     gradient w.r.t. the LOW-resolution input is a stride-2, pad-1 4x4 convolution of dY with the
//     tap-summed kernel Weff[t] = sum{ W[r] : 2-r == t or 3-r == t } per spatial axis, which skips
//     the 4x-upsampled intermediate gradient entirely (16 taps on H*W instead of 9 on 4*H*W).
//   * bias gradient: fixed-order column sums of dY [pixels][Cout].
#include "common.h"
#include <algorithm>

namespace mvae {

// per tap t: [cout][cin] (row stride rs*cin) -> [cin][cout] (row stride rs*cout), 64x64 tiles through
// LDS so both the reads (along cin) and the writes (along cout) are coalesced
// write phase of a transposed 64x64 tile: tile[o_local][c_local] -> wt rows c (row stride rs*cout, tap t)
// along o; split 1: groups of 4 consecutive o as split4_bf16 (needs cout % 4 == 0); split 2: packed bf16 (RNE; the
// bf16-mixed mode's GEMM operand, 2 B per element at the same element offsets)
__device__ __forceinline__ void write_transposed(const float (*tile)[65], float* __restrict__ wt, int c0, int o0, int t,
                                                 int rs, int cin, int cout, int split) {
  if (split == 3) {  // planar 3xBF16: hi plane [cin*rs*cout] bf16, then the lo plane
    const int g = threadIdx.x & 31, cr = threadIdx.x >> 5;
    __bf16* wb = (__bf16*)wt;
    const long long plane = (long long)cin * rs * cout;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = cr + 8 * i, c = c0 + cl, o = o0 + 2 * g;
      if (c < cin && o < cout) {  // cout % 4 == 0: o + 1 < cout
        const long long e = ((long long)c * rs + t) * cout + o;
        const float v0 = tile[2 * g][cl], v1 = tile[2 * g + 1][cl];
        const unsigned h = pk_bf16x2(v0, v1);
        *(unsigned*)(wb + e) = h;
        *(unsigned*)(wb + plane + e) = pk_bf16x2(v0 - __uint_as_float(h << 16), v1 - __uint_as_float(h & 0xFFFF0000u));
      }
    }
  } else if (split == 2) {
    const int g = threadIdx.x & 31, cr = threadIdx.x >> 5;
    __bf16* wb = (__bf16*)wt;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int cl = cr + 8 * i, c = c0 + cl, o = o0 + 2 * g;
      if (c < cin && o < cout) {
        const long long e = ((long long)c * rs + t) * cout + o;
        if (o + 1 < cout && (e & 1) == 0) *(unsigned*)(wb + e) = pk_bf16x2(tile[2 * g][cl], tile[2 * g + 1][cl]);
        else {
          wb[e] = (__bf16)tile[2 * g][cl];
          if (o + 1 < cout) wb[e + 1] = (__bf16)tile[2 * g + 1][cl];
        }
      }
    }
  } else if (!split) {
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = c0 + ty + 4 * i, o = o0 + tx;
      if (o < cout && c < cin) wt[((long long)c * rs + t) * cout + o] = tile[tx][ty + 4 * i];
    }
  } else {
    const int g = threadIdx.x & 15, cr = threadIdx.x >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cl = cr + 16 * i, c = c0 + cl, o = o0 + 4 * g;
      if (o < cout && c < cin) {
        const float4 v{tile[4 * g][cl], tile[4 * g + 1][cl], tile[4 * g + 2][cl], tile[4 * g + 3][cl]};
        *(uint4*)(wt + ((long long)c * rs + t) * cout + o) = split4_bf16(v);
      }
    }
  }
}

__global__ void __launch_bounds__(256) w_transpose_kernel(const float* __restrict__ w, float* __restrict__ wt,
                                                          int cout, int rs, int cin, int split) {
  __shared__ float tile[64][65];
  const int t = blockIdx.z;
  const int c0 = blockIdx.x * 64, o0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int o = o0 + ty + 4 * i, c = c0 + tx;
    tile[ty + 4 * i][tx] = (o < cout && c < cin) ? w[((long long)o * rs + t) * cin + c] : 0.f;
  }
  __syncthreads();
  write_transposed(tile, wt, c0, o0, t, rs, cin, cout, split);
}

// Every dgrad weight re-layout of a training step in one launch (mvae_conv_weight_transpose_batched): a 1-D grid over
// the concatenated (cin/64, cout/64, tap) tiles of all descriptors; each workgroup finds its descriptor by binary
// search over the block offsets (wave-uniform loads) and runs w_transpose_kernel's body.
__global__ void __launch_bounds__(256) w_transpose_batched_kernel(const mvae_wt_desc* __restrict__ d, int nd) {
  __shared__ float tile[64][65];
  const int blk = blockIdx.x;
  int lo = 0, hi = nd - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].block0 <= blk) lo = mid; else hi = mid - 1;
  }
  const float* __restrict__ w = d[lo].w;
  float* __restrict__ wt = d[lo].wt;
  const int cout = d[lo].cout, rs = d[lo].rs, cin = d[lo].cin, split = d[lo].split;
  const int bx = (cin + 63) / 64, by = (cout + 63) / 64;
  int b = blk - d[lo].block0;
  const int cx = b % bx;
  b /= bx;
  const int c0 = cx * 64, o0 = (b % by) * 64, t = b / by;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int o = o0 + ty + 4 * i, c = c0 + tx;
    tile[ty + 4 * i][tx] = (o < cout && c < cin) ? w[((long long)o * rs + t) * cin + c] : 0.f;
  }
  __syncthreads();
  write_transposed(tile, wt, c0, o0, t, rs, cin, cout, split);
}

__device__ __forceinline__ int tap_mask(int t) {
  // bit r set when source tap r contributes to effective tap t
  return t == 0 ? 0b100 : t == 1 ? 0b110 : t == 2 ? 0b011 : 0b001;
}

// grid (cin/64, cout/64, 16 effective taps): sum the <= 4 contributing source taps of a 64x64
// [cout][cin] tile (coalesced along cin), transpose through LDS, write along cout
__global__ void __launch_bounds__(256) w_ups_dgrad_kernel(const float* __restrict__ w, float* __restrict__ wt,
                                                          int cout, int cin, int split) {
  __shared__ float tile[64][65];
  const int tu = blockIdx.z;
  const int mt = tap_mask(tu >> 2), mu = tap_mask(tu & 3);
  const int c0 = blockIdx.x * 64, o0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int o = o0 + ty + 4 * i, c = c0 + tx;
    float s = 0.f;
    if (o < cout && c < cin) {
      for (int r = 0; r < 3; ++r) {
        if (!((mt >> r) & 1)) continue;
        for (int u = 0; u < 3; ++u)
          if ((mu >> u) & 1) s += w[(((long long)o * 3 + r) * 3 + u) * cin + c];
      }
    }
    tile[ty + 4 * i][tx] = s;
  }
  __syncthreads();
  write_transposed(tile, wt, c0, o0, tu, 16, cin, cout, split);
}

// forward weights of the sub-pixel Upsample conv: w4[2*ph+pw][co][a][b][ci] = sum of w[co][r][s][ci] over
// r in T(ph, a), s in T(pw, b): T(0,0) = {0}, T(0,1) = {1,2}, T(1,0) = {0,1}, T(1,1) = {2}
__device__ __forceinline__ int sub_mask(int p, int a) { return p == 0 ? (a == 0 ? 0b001 : 0b110) : (a == 0 ? 0b011 : 0b100); }

__global__ void __launch_bounds__(256) w_ups_fwd_kernel(const float* __restrict__ w, float* __restrict__ w4, int cout,
                                                        int cin, int split) {
  // one thread per (co, group of 4 ci) (split 1: split4_bf16, split 2: packed bf16; cin % 4 == 0) or per (co, ci)
  const int gw = split ? 4 : 1, ng = cin / gw;
  const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long long)cout * ng) return;
  const int co = (int)(idx / ng), ci = (int)(idx - (long long)co * ng) * gw;
  float t[3][3][4];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[r][s][e] = e < gw ? w[(((long long)co * 3 + r) * 3 + s) * cin + ci + e] : 0.f;
#pragma unroll
  for (int cls = 0; cls < 4; ++cls)
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int mr = sub_mask(cls >> 1, a), ms = sub_mask(cls & 1, b);
        float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int s = 0; s < 3; ++s)
            if (((mr >> r) & 1) && ((ms >> s) & 1))
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += t[r][s][e];
        float* o = w4 + ((((long long)cls * cout + co) * 2 + a) * 2 + b) * cin + ci;
        if (split >= 2) {  // packed bf16 (2) or planar 3xBF16 (3: lo plane 16*cout*cin elements later)
          __bf16* ob = (__bf16*)w4 + (o - w4);
          const unsigned h01 = pk_bf16x2(v[0], v[1]), h23 = pk_bf16x2(v[2], v[3]);
          *(uint2*)ob = uint2{h01, h23};
          if (split == 3)
            *(uint2*)(ob + 16LL * cout * cin) =
                uint2{pk_bf16x2(v[0] - __uint_as_float(h01 << 16), v[1] - __uint_as_float(h01 & 0xFFFF0000u)),
                      pk_bf16x2(v[2] - __uint_as_float(h23 << 16), v[3] - __uint_as_float(h23 & 0xFFFF0000u))};
        } else if (split) {
          *(uint4*)o = split4_bf16(float4{v[0], v[1], v[2], v[3]});
        } else {
          *o = v[0];
        }
      }
}

__global__ void __launch_bounds__(256) split_bf16_kernel(const float4* __restrict__ x, uint4* __restrict__ y, long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x)
    y[i] = split4_bf16(x[i]);
}

// packed bf16 (RNE) of 8 fp32 values per thread step
__global__ void __launch_bounds__(256) pack_bf16_kernel(const float4* __restrict__ x, uint4* __restrict__ y, long long n8) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
    const float4 a = x[2 * i], b = x[2 * i + 1];
    y[i] = uint4{pk_bf16x2(a.x, a.y), pk_bf16x2(a.z, a.w), pk_bf16x2(b.x, b.y), pk_bf16x2(b.z, b.w)};
  }
}

// planar 3xBF16 of 4 fp32 values: hi (returned in .x) and lo (.y) bf16 pairs x 2
__device__ __forceinline__ void planar4(float4 v, uint2& hi, uint2& lo) {
  const unsigned h01 = pk_bf16x2(v.x, v.y), h23 = pk_bf16x2(v.z, v.w);
  hi = uint2{h01, h23};
  lo = uint2{pk_bf16x2(v.x - __uint_as_float(h01 << 16), v.y - __uint_as_float(h01 & 0xFFFF0000u)),
             pk_bf16x2(v.z - __uint_as_float(h23 << 16), v.w - __uint_as_float(h23 & 0xFFFF0000u))};
}
// planar 3xBF16 of n values: y[0, n) hi plane, y[n, 2n) lo plane (bf16)
__global__ void __launch_bounds__(256) split_planar_kernel(const float4* __restrict__ x, uint2* __restrict__ y, long long n4) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    uint2 h, l;
    planar4(x[i], h, l);
    y[i] = h;
    y[n4 + i] = l;
  }
}

// packed bf16 of x [rows][n] (n % 4 == 0, row stride n) plus the fp64 column sums of the fp32 values per chunk of
// rows: part[chunk][n] (the conv bias gradient of a dy that the bf16-mixed GEMMs read packed: one pass over dy for
// both). 256 threads = 64 column groups of 4 x 4 row phases; fixed summation order.
template <bool PLANAR>
__global__ void __launch_bounds__(256) pack_colsum_kernel(const float* __restrict__ x, uint2* __restrict__ y,
                                                          long long rows, int n, int rows_per_chunk,
                                                          double* __restrict__ part) {
  __shared__ double sh[4][64][4];
  const int cg = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int c = cg * 4;
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = std::min<long long>(rows, r0 + rows_per_chunk);
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (c < n) {
    // PU rows in flight per thread (the loads of a batch issue together; one 16-B load per iteration left the kernel
    // latency-bound at ~1 TB/s), summed in row order: the same fp64 sums as a row-at-a-time walk (masked rows add 0)
    constexpr int PU = 8;
    for (long long r = r0 + rg; r < r1; r += 4 * PU) {
      float4 v[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const long long rr = r + 4 * u;
        v[u] = rr < r1 ? *(const float4*)(x + rr * n + c) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < PU; ++u) {
        const long long rr = r + 4 * u;
        if (rr >= r1) break;
        if constexpr (PLANAR) {  // hi plane, then the lo plane rows * n elements later
          uint2 h, l;
          planar4(v[u], h, l);
          y[(rr * n + c) >> 2] = h;
          y[((rows * n) >> 2) + ((rr * n + c) >> 2)] = l;
        } else {
          y[(rr * n + c) >> 2] = uint2{pk_bf16x2(v[u].x, v[u].y), pk_bf16x2(v[u].z, v[u].w)};
        }
        a0 += v[u].x; a1 += v[u].y; a2 += v[u].z; a3 += v[u].w;
      }
    }
  }
  sh[rg][threadIdx.x & 63][0] = a0;
  sh[rg][threadIdx.x & 63][1] = a1;
  sh[rg][threadIdx.x & 63][2] = a2;
  sh[rg][threadIdx.x & 63][3] = a3;
  __syncthreads();
  if (rg == 0 && c < n) {
    double* o = part + (long long)blockIdx.y * n + c;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      o[e] = sh[0][threadIdx.x][e] + sh[1][threadIdx.x][e] + sh[2][threadIdx.x][e] + sh[3][threadIdx.x][e];
  }
}

// column sums: part[chunk][n] = sum over rows in chunk ; then out[n] += sum_chunks (fixed order)
__global__ void __launch_bounds__(256) colsum_partial_kernel(const float* __restrict__ x, long long rows, int n,
                                                             long long ld, int rows_per_chunk,
                                                             double* __restrict__ part) {
  __shared__ double sh[256];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const long long r0 = (long long)blockIdx.y * rows_per_chunk;
  const long long r1 = std::min<long long>(rows, r0 + rows_per_chunk);
  double acc = 0;
  if (col < n) {
    constexpr int PU = 8;  // rows in flight per thread, summed in row order
    for (long long r = r0 + rg; r < r1; r += 4 * PU) {
      float v[PU];
#pragma unroll
      for (int u = 0; u < PU; ++u) v[u] = r + 4 * u < r1 ? x[(r + 4 * u) * ld + col] : 0.f;
#pragma unroll
      for (int u = 0; u < PU; ++u) acc += v[u];
    }
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  if (rg == 0 && col < n) part[(long long)blockIdx.y * n + col] = sh[threadIdx.x] + sh[threadIdx.x + 64] +
                                                                 sh[threadIdx.x + 128] + sh[threadIdx.x + 192];
}

__global__ void colsum_final_kernel(const double* __restrict__ part, int chunks, int n, float* out, float beta) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= n) return;
  double s = 0;
  int c = 0;
  for (; c + 16 <= chunks; c += 16) {  // 16 partial loads in flight, summed in chunk order
    double v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = part[(long long)(c + j) * n + col];
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
  }
  for (; c < chunks; ++c) s += part[(long long)c * n + col];
  out[col] = (beta != 0.f ? beta * out[col] : 0.f) + (float)s;
}

static int colsum_chunks(long long rows, int n) {
  const int colblocks = (n + 63) / 64;
  long long chunks = std::max<long long>(1, 1024 / colblocks);
  chunks = std::min<long long>(chunks, std::max<long long>(1, rows / 64));
  return (int)chunks;
}

static int egrid(long long n) { return (int)std::max<long long>(1, std::min<long long>((n + 255) / 256, 8192)); }

}  // namespace mvae

using namespace mvae;

extern "C" {

int mvae_conv_weight_transpose(const float* w, float* wt, int cout, int kh, int kw, int cin, int split, void* stream) {
  if (cout <= 0 || kh <= 0 || kw <= 0 || cin <= 0 || split < 0 || split > 3 || (split && (cout & 3))) {
    set_error("w_transpose: bad sizes");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(w_transpose_kernel, dim3((cin + 63) / 64, (cout + 63) / 64, kh * kw), dim3(256), 0,
                     (hipStream_t)stream, w, wt, cout, kh * kw, cin, split);
  return launch_status();
}

int mvae_conv_weight_transpose_batched(const mvae_wt_desc* table, int n, int total_blocks, void* stream) {
  if (n <= 0 || !table || total_blocks <= 0) { set_error("w_transpose_batched: bad args"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(w_transpose_batched_kernel, dim3(total_blocks), dim3(256), 0, (hipStream_t)stream, table, n);
  return launch_status();
}

// wt [cin][4][4][cout] for the dgrad of "nearest-x2 upsample then 3x3 conv"
int mvae_conv_weight_upsample_dgrad(const float* w, float* wt, int cout, int cin, int split, void* stream) {
  if (cout <= 0 || cin <= 0 || split < 0 || split > 3 || (split && (cout & 3))) { set_error("w_ups: bad sizes"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(w_ups_dgrad_kernel, dim3((cin + 63) / 64, (cout + 63) / 64, 16), dim3(256), 0,
                     (hipStream_t)stream, w, wt, cout, cin, split);
  return launch_status();
}

// w4 [4][cout][2][2][cin] for the sub-pixel forward of "nearest-x2 upsample then 3x3 conv"
int mvae_conv_weight_upsample_fwd(const float* w, float* w4, int cout, int cin, int split, void* stream) {
  if (cout <= 0 || cin <= 0 || split < 0 || split > 3 || (split && (cin & 3))) { set_error("w_ups_fwd: bad sizes"); return MVAE_EINVAL; }
  const long long tot = (long long)cout * (split ? cin / 4 : cin);
  hipLaunchKernelGGL(w_ups_fwd_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, w, w4,
                     cout, cin, split);
  return launch_status();
}

int mvae_split_bf16(const float* x, void* y, long long n, void* stream) {
  if (n <= 0 || (n & 3)) { set_error("split_bf16: n must be a positive multiple of 4"); return MVAE_EINVAL; }
  hipLaunchKernelGGL(split_bf16_kernel, dim3(egrid(n / 4)), dim3(256), 0, (hipStream_t)stream, (const float4*)x, (uint4*)y,
                     n / 4);
  return launch_status();
}

// y (bf16, n elements) = x (fp32) rounded to nearest even: the bf16-mixed mode's packed GEMM operands
int mvae_pack_bf16(const float* x, void* y, long long n, void* stream) {
  if (n <= 0 || (n & 7) || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) {
    set_error("pack_bf16: n must be a positive multiple of 8, x / y 16-B aligned");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(pack_bf16_kernel, dim3(egrid(n / 8)), dim3(256), 0, (hipStream_t)stream, (const float4*)x, (uint4*)y,
                     n / 8);
  return launch_status();
}

// y = packed bf16 of x [rows][n] (fp32, row stride n) and out[n] = beta*out[n] + sum_rows x (the conv bias gradient,
// fp64 partials in a fixed order): the bf16-mixed mode's output-gradient pack (MVAE_CONV_BF16) and bias gradient in
// one pass over dy. Workspace: mvae_bias_grad_workspace_bytes(rows, n).
static int pack_colsum(bool planar, const float* x, void* y, long long rows, int n, float* out, float beta,
                       void* workspace, size_t workspace_bytes, void* stream);
int mvae_pack_bf16_colsum(const float* x, void* y, long long rows, int n, float* out, float beta, void* workspace,
                          size_t workspace_bytes, void* stream) {
  return pack_colsum(false, x, y, rows, n, out, beta, workspace, workspace_bytes, stream);
}
// the same pass writing dy as planar 3xBF16 (hi plane, then lo plane rows * n elements later; MVAE_CONV_PLANAR)
int mvae_split_planar_colsum(const float* x, void* y, long long rows, int n, float* out, float beta, void* workspace,
                             size_t workspace_bytes, void* stream) {
  return pack_colsum(true, x, y, rows, n, out, beta, workspace, workspace_bytes, stream);
}
// planar 3xBF16 of n fp32 values (n % 4 == 0): y = [hi plane n bf16][lo plane n bf16]
int mvae_split_planar(const float* x, void* y, long long n, void* stream) {
  if (n <= 0 || (n & 3) || ((uintptr_t)x & 15) || ((uintptr_t)y & 7)) {
    set_error("split_planar: n must be a positive multiple of 4, x 16-B / y 8-B aligned");
    return MVAE_EINVAL;
  }
  hipLaunchKernelGGL(split_planar_kernel, dim3(egrid(n / 4)), dim3(256), 0, (hipStream_t)stream, (const float4*)x,
                     (uint2*)y, n / 4);
  return launch_status();
}
static int pack_colsum(bool planar, const float* x, void* y, long long rows, int n, float* out, float beta,
                       void* workspace, size_t workspace_bytes, void* stream) {
  if (rows <= 0 || n <= 0 || (n & 3) || ((uintptr_t)x & 15) || ((uintptr_t)y & 7)) {
    set_error("pack_bf16_colsum: n %% 4 == 0, 16-B aligned x, 8-B aligned y");
    return MVAE_EINVAL;
  }
  const int chunks = colsum_chunks(rows, n);
  if (workspace_bytes < (size_t)chunks * n * sizeof(double)) { set_error("pack_bf16_colsum: workspace"); return MVAE_EWORKSPACE; }
  const int rpc = (int)((rows + chunks - 1) / chunks);
  hipStream_t st = (hipStream_t)stream;
  if (planar)
    hipLaunchKernelGGL(pack_colsum_kernel<true>, dim3((n / 4 + 63) / 64, chunks), dim3(256), 0, st, x, (uint2*)y, rows, n,
                       rpc, (double*)workspace);
  else
    hipLaunchKernelGGL(pack_colsum_kernel<false>, dim3((n / 4 + 63) / 64, chunks), dim3(256), 0, st, x, (uint2*)y, rows,
                       n, rpc, (double*)workspace);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const double*)workspace, chunks, n,
                     out, beta);
  return launch_status();
}

size_t mvae_bias_grad_workspace_bytes(long long rows, int n) {
  return (size_t)colsum_chunks(rows, n) * n * sizeof(double);
}

// out[n] = beta*out[n] + sum_rows x[row*ld + n]
int mvae_bias_grad(const float* x, long long rows, int n, long long ld, float* out, float beta, void* workspace,
                   size_t workspace_bytes, void* stream) {
  if (rows <= 0 || n <= 0) { set_error("bias_grad: bad sizes"); return MVAE_EINVAL; }
  const int chunks = colsum_chunks(rows, n);
  if (workspace_bytes < (size_t)chunks * n * sizeof(double)) { set_error("bias_grad: workspace"); return MVAE_EWORKSPACE; }
  const int rpc = (int)((rows + chunks - 1) / chunks);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((n + 63) / 64, chunks), dim3(256), 0, st, x, rows, n, ld, rpc,
                     (double*)workspace);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((n + 255) / 256), dim3(256), 0, st, (const double*)workspace, chunks, n,
                     out, beta);
  return launch_status();
}

}  // extern "C"
