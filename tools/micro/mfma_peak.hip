// Microbenchmark: sustained v_mfma_f32_32x32x16_bf16 rate on the whole chip (register operands,
// no memory traffic) and with ds_read_b128 fragment loads from LDS in the loop, at 2 waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int WITH_LDS>
__global__ void __launch_bounds__(512) mfma_loop(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[64 * 1024];
  const int lane = threadIdx.x & 63;
  bf16x8 a[4], b[2];
  for (int i = 0; i < 4; ++i)
    for (int e = 0; e < 8; ++e) a[i][e] = (__bf16)(0.001f * (lane + i + e));
  for (int j = 0; j < 2; ++j)
    for (int e = 0; e < 8; ++e) b[j][e] = (__bf16)(0.002f * (lane - j + e));
  if (WITH_LDS) {
    for (int i = threadIdx.x; i < 64 * 1024; i += blockDim.x) lds[i] = (__bf16)(i * 1e-5f);
    __syncthreads();
  }
  f32x16 acc[4][2] = {};
  for (int it = 0; it < iters; ++it) {
    if (WITH_LDS) {
      const int wid = threadIdx.x >> 6;
      for (int i = 0; i < 4; ++i)
        a[i] = *(const bf16x8*)(lds + ((wid * 4 + i) * 32 + (lane & 31)) * 40 + (lane >> 5) * 8 + (it & 1) * 16);
      for (int j = 0; j < 2; ++j)
        b[j] = *(const bf16x8*)(lds + 32768 + ((j * 8 + wid) * 32 + (lane & 31)) * 40 + (lane >> 5) * 8);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    if (WITH_LDS == 2) __syncthreads();
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 2; ++j)
      for (int r = 0; r < 16; ++r) s += acc[i][j][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int W>
void run(const char* name, float* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(mfma_loop<W>, dim3(blocks), dim3(512), 0, 0, out, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(mfma_loop<W>, dim3(blocks), dim3(512), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop = 5.0 * blocks * 8.0 * iters * 24 * 32768.0;  // 8 waves, 24 MFMA/iter
  printf("%-28s %8.1f TFLOP/s bf16 (%.3f ms/launch)\n", name, flop / (ms * 1e-3) / 1e12, ms / 5);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 512 * sizeof(float));
  run<0>("regs only", out, 256 * 4, 4000);
  run<1>("ds_read frags", out, 256 * 4, 4000);
  run<2>("ds_read frags + barrier", out, 256 * 4, 4000);
  run<0>("regs only, 1 wg/CU", out, 256, 4000);
  return 0;
}
