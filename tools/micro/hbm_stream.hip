// Microbenchmark: achievable HBM bandwidth on the whole chip -- float4 copy (read + write) and float4 read-only
// sum over 4 GiB buffers, grid-stride, 4 x 256-thread workgroups per CU.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void __launch_bounds__(256) copy4(const float4* __restrict__ a, float4* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) b[i] = a[i];
}
__global__ void __launch_bounds__(256) read4(const float4* __restrict__ a, float* __restrict__ out, long long n) {
  float s = 0.f;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1234.5f) out[0] = s;  // keeps the loads live
}

int main() {
  const long long bytes = 4LL << 30, n = bytes / 16;
  float4 *a, *b;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
  (void)hipMemset(a, 0, bytes);
  (void)hipMemset(b, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int g : {1024, 2048, 4096}) {
    hipLaunchKernelGGL(copy4, dim3(g), dim3(256), 0, 0, a, b, n);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(copy4, dim3(g), dim3(256), 0, 0, a, b, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double cp = 5.0 * 2.0 * bytes / (ms * 1e-3) / 1e9;
    hipLaunchKernelGGL(read4, dim3(g), dim3(256), 0, 0, a, (float*)b, n);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(read4, dim3(g), dim3(256), 0, 0, a, (float*)b, n);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double rd = 5.0 * bytes / (ms * 1e-3) / 1e9;
    printf("grid %5d: copy (read+write) %7.1f GB/s   read-only %7.1f GB/s\n", g, cp, rd);
  }
  return 0;
}
