// Microbenchmark: the 3xBF16 main-loop structure with a 128x128 output block per wave, 4 waves per workgroup
// (1 per SIMD, 256 accumulator registers per lane), against mfma_shape.hip's 128x64 per wave on 8 waves. Same
// LDS image layout (pitch 40, hi / lo planes), fragments re-read from LDS every K-step, random operands, 16x16x32
// MFMA, one barrier per K-tile (BAR 1) or none. Per K-tile a wave reads (128 + 128) x 32 x 2 planes from LDS for
// 192 MFMAs (the 8-wave form: (128 + 64) x 32 x 2 for 96), so the LDS bytes per MFMA drop by a third.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float rnd(unsigned i) {
  i ^= i >> 16; i *= 0x7feb352dU; i ^= i >> 15; i *= 0x846ca68bU; i ^= i >> 16;
  return (float)(i & 0xFFFFFF) / 8388608.0f - 1.0f;
}

constexpr int LDS_ELEMS = 64 * 1024;  // 128 KB

template <int BAR>
__global__ void __launch_bounds__(256) loop4(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[LDS_ELEMS];
  for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) lds[i] = (__bf16)rnd(i + 7919u * blockIdx.x);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x4 acc[8][8] = {};
  for (int it = 0; it < iters; ++it) {
    const int base = (it & 3) * 4096;
    bf16x8 bh[8], bl[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int off = base + 20480 + ((wid >> 1) * 128 + j * 16 + (lane & 15)) * 40 + (lane >> 4) * 8;
      bh[j] = *(const bf16x8*)(lds + off);
      bl[j] = *(const bf16x8*)(lds + off + 10240 + 8);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int off = base + ((wid & 1) * 128 + i * 16 + (lane & 15)) * 40 + (lane >> 4) * 8;
      const bf16x8 ah = *(const bf16x8*)(lds + off);
      const bf16x8 al = *(const bf16x8*)(lds + off + 10240 + 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
      }
    }
    if (BAR) __syncthreads();
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 8; ++j)
      for (int r = 0; r < 4; ++r) s += acc[i][j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int B>
double run(float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((loop4<B>), dim3(256), dim3(256), 0, 0, out, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((loop4<B>), dim3(256), dim3(256), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per iteration per wave: 128x128 block x K=32 x 3 products
  const double flop = 10.0 * 256 * 4 * (double)iters * 2.0 * 128 * 128 * 32 * 3;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 256 * sizeof(float));
  const int iters = 10000;
  for (int rep = 0; rep < 3; ++rep)
    printf("rep %d: 4 waves x 128x128, 16x16x32: %.1f  +barrier %.1f  TFLOP/s bf16\n", rep, run<0>(out, iters),
           run<1>(out, iters));
  return 0;
}
