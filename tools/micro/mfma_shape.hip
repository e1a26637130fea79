// Microbenchmark: 32x32x16 vs 16x16x32 bf16 MFMA inside the 3xBF16 GEMM's per-wave structure
// (128x64 output block per wave, 8 waves = 2 per SIMD, 1 workgroup per CU, fragments re-read from LDS
// every K-step, random operands so the clock sees realistic toggling). Same FLOPs per iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float rnd(unsigned i) {
  i ^= i >> 16; i *= 0x7feb352dU; i ^= i >> 15; i *= 0x846ca68bU; i ^= i >> 16;
  return (float)(i & 0xFFFFFF) / 8388608.0f - 1.0f;
}

constexpr int LDS_ELEMS = 64 * 1024;  // 128 KB

template <int SHAPE, int BAR>  // SHAPE 32: 32x32x16, 16: 16x16x32
__global__ void __launch_bounds__(512) loop(float* out, int iters) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[LDS_ELEMS];
  for (int i = threadIdx.x; i < LDS_ELEMS; i += blockDim.x) lds[i] = (__bf16)rnd(i + 7919u * blockIdx.x);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if constexpr (SHAPE == 32) {
    f32x16 acc[4][2] = {};
    for (int it = 0; it < iters; ++it) {
      const int base = (it & 7) * 4096;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 ah[4], al[4], bh[2], bl[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int off = base + ((wid & 1) * 128 + i * 32 + (lane & 31)) * 40 + ks * 16 + (lane >> 5) * 8;
          ah[i] = *(const bf16x8*)(lds + off);
          al[i] = *(const bf16x8*)(lds + off + 10240 + 8);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int off = base + 20480 + ((wid >> 1) * 64 + j * 32 + (lane & 31)) * 40 + ks * 16 + (lane >> 5) * 8;
          bh[j] = *(const bf16x8*)(lds + off);
          bl[j] = *(const bf16x8*)(lds + off + 10240 + 8);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          }
      }
      if (BAR) __syncthreads();
    }
    float s = 0.f;
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else {
    f32x4 acc[8][4] = {};
    for (int it = 0; it < iters; ++it) {
      const int base = (it & 7) * 4096;
      bf16x8 bh[4], bl[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int off = base + 20480 + ((wid >> 1) * 64 + j * 16 + (lane & 15)) * 40 + (lane >> 4) * 8;
        bh[j] = *(const bf16x8*)(lds + off);
        bl[j] = *(const bf16x8*)(lds + off + 10240 + 8);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int off = base + ((wid & 1) * 128 + i * 16 + (lane & 15)) * 40 + (lane >> 4) * 8;
        const bf16x8 ah = *(const bf16x8*)(lds + off);
        const bf16x8 al = *(const bf16x8*)(lds + off + 10240 + 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
        }
      }
      if (BAR) __syncthreads();
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 4; ++r) s += acc[i][j][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

template <int S, int B>
double run(float* out, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((loop<S, B>), dim3(256), dim3(512), 0, 0, out, iters);
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL((loop<S, B>), dim3(256), dim3(512), 0, 0, out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  // per iteration per wave: 128x64 block x K=32 x 3 products
  const double flop = 10.0 * 256 * 8 * (double)iters * 2.0 * 128 * 64 * 32 * 3;
  return flop / (ms * 1e-3) / 1e12;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 512 * sizeof(float));
  const int iters = 20000;
  for (int rep = 0; rep < 3; ++rep) {
    printf("rep %d: 32x32x16 %.1f  16x16x32 %.1f  | +barrier: 32x32x16 %.1f  16x16x32 %.1f  TFLOP/s bf16\n", rep,
           run<32, 0>(out, iters), run<16, 0>(out, iters), run<32, 1>(out, iters), run<16, 1>(out, iters));
  }
  return 0;
}
