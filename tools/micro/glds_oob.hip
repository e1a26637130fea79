// LDS-DMA (buffer_load_dwordx4 ... lds) behaviour check: out-of-range offsets through a buffer descriptor must
// land as zeros in the LDS image (the conv gathers rely on it for padding / tails).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((address_space(3))) void lds_void;
__global__ void k(const float* p, float* out, int nbytes) {
  __shared__ __attribute__((aligned(16))) float lds[64 * 4 * 2];
  for (int i = threadIdx.x; i < 512; i += 64) lds[i] = -7.f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, nbytes, 0x00020000);
  // lanes with odd id read past the range
  unsigned off = (threadIdx.x & 1) ? 0xFFFFFFF0u : threadIdx.x * 16;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds, 16, off, 0, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)(lds + 256), 16, threadIdx.x * 16 + 4096 * 4, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}
int main() {
  std::vector<float> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = 1.f + i;
  float *d, *o;
  hipMalloc(&d, 4096 * 4 + 4096);
  hipMalloc(&o, 512 * 4);
  hipMemcpy(d, h.data(), 4096, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, 1024 * 4);
  std::vector<float> r(512);
  hipMemcpy(r.data(), o, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int e = 0; e < 4; ++e) {
      float want = (l & 1) ? 0.f : h[l * 4 + e];
      if (r[l * 4 + e] != want) ++bad;
      if (r[256 + l * 4 + e] != 0.f) ++bad;  // whole second load out of range
    }
  printf("glds_oob: %s (%d mismatches) sample %g %g %g %g | %g\n", bad ? "FAIL" : "ok", bad, r[0], r[4], r[8], r[12], r[256]);
  return bad != 0;
}
