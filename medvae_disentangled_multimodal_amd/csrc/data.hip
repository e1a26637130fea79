// On-device MedMNIST batch assembly (row (f)1): the per-sample path of MedMNISTDataset.__getitem__
// (src/data/medmnist_data.py:186-251) + the modality transforms (:319-375) + mixed_modality_collate_fn
// (:16-72), for a batch of sample indices into a resident uint8 image store:
//   ToTensor (/255) -> channel conversion to the modality's target channels (gray = 0.299 R + 0.587 G
//   + 0.114 B; gray -> RGB by repeat) -> [train] RandomHorizontalFlip, RandomRotation (nearest,
//   zero fill; torchvision's affine grid + grid_sample(align_corners=False)), ColorJitter(brightness,
//   contrast) in the sampled order -> Normalize(0.5, 0.5) -> zero-pad to the batch's channel count.
// Random parameters are drawn by the host per sample and passed in `aug` (see data.py); with
// aug == nullptr the transform is the evaluation one (no augmentation).
// Output x is NHWC fp32 [nb][h][w][cout]; onehot [nb][n_mod], idx [nb], labels [nb].
// Float arithmetic is spelled with explicit round-to-nearest helpers (no FMA contraction) in the
// operation order of the torch/torchvision code it restates, so the evaluation transform is
// bit-exact and the augmented one differs only where a rotated coordinate sits on a rounding tie.
#include "common.h"
#include <algorithm>

// Every multiply and add rounds separately, as in the torch CPU kernels: FMA contraction is off for
// this file's code (the HIP headers' __f*_rn helpers are plain operators compiled with contraction
// on, so local helpers are used instead).
#pragma clang fp contract(off)
__device__ __forceinline__ float mul_rn(float a, float b) { return a * b; }
__device__ __forceinline__ float add_rn(float a, float b) { return a + b; }
__device__ __forceinline__ float sub_rn(float a, float b) { return a - b; }
__device__ __forceinline__ float div_rn(float a, float b) { return a / b; }  // IEEE division (default)

namespace mvae {

struct SampleAug {     // per-sample augmentation parameters (host-drawn, see data.py)
  float flip;          // 1: horizontal flip
  float r0, r1;        // inverse-rotation row 0 divided by w/2: (cos, sin(-a)) / (0.5 w)
  float r3, r4;        // row 1 divided by h/2: (-sin(-a), cos) / (0.5 h)
  float bright, one_minus_bright;      // brightness factor f and (1 - f) (rounded from double)
  float contrast, one_minus_contrast;  // contrast factor
  float order;         // 0: brightness before contrast, 1: contrast first
  float pad0, pad1;
};

// pre-contrast value of target channel ch at output pixel (i, j) of sample s, in [0, 1]
__device__ __forceinline__ float fetch(const unsigned char* __restrict__ img, int h, int w, int nat, int tgt,
                                       int ch, int si, int sj) {
  if ((unsigned)si >= (unsigned)h || (unsigned)sj >= (unsigned)w) return 0.f;  // rotation zero fill
  const unsigned char* p = img + ((long long)si * w + sj) * nat;
  if (tgt == 1 && nat == 3) {  // 0.299 * image[0] + 0.587 * image[1] + 0.114 * image[2] (fp32)
    const float r = div_rn((float)p[0], 255.f), g = div_rn((float)p[1], 255.f), b = div_rn((float)p[2], 255.f);
    return add_rn(add_rn(mul_rn(0.299f, r), mul_rn(0.587f, g)), mul_rn(0.114f, b));
  }
  return div_rn((float)p[nat == 1 ? 0 : ch], 255.f);  // ToTensor: .div(255), correctly rounded
}

// source pixel of output (i, j) after flip then rotation (torchvision: hflip, then rotate with the
// inverse affine matrix [cos, sin, 0; -sin, cos, 0] of angle a, base grid at pixel centres,
// normalised by (w/2, h/2), grid_sample nearest with align_corners=False: ix = ((gx+1)w - 1)/2)
__device__ __forceinline__ void src_pixel(const SampleAug* aug, int h, int w, int i, int j, int& si, int& sj) {
  if (aug == nullptr) {
    si = i;
    sj = j;
    return;
  }
  // base grid (exact half-integers) x rescaled theta (bmm order), then grid_sample's unnormalize
  const float x = -0.5f * w + 0.5f + (float)j, y = -0.5f * h + 0.5f + (float)i;
  const float gx = add_rn(mul_rn(x, aug->r0), mul_rn(y, aug->r1));
  const float gy = add_rn(mul_rn(x, aug->r3), mul_rn(y, aug->r4));
  const float ix = mul_rn(sub_rn(mul_rn(add_rn(gx, 1.f), (float)w), 1.f), 0.5f);
  const float iy = mul_rn(sub_rn(mul_rn(add_rn(gy, 1.f), (float)h), 1.f), 0.5f);
  si = (int)rintf(iy);
  sj = (int)rintf(ix);
  if (aug->flip != 0.f) sj = w - 1 - sj;  // the rotation reads the flipped image
}

// torchvision _blend: (ratio * img1 + (1 - ratio) * img2).clamp(0, 1)
__device__ __forceinline__ float blend(float v, float other, float f, float omf) {
  return fminf(fmaxf(add_rn(mul_rn(f, v), mul_rn(omf, other)), 0.f), 1.f);
}

// pass 1: one workgroup per (sample, row block): write the pre-contrast image (or the final
// normalised one when no contrast stage follows) and per-block grayscale partial sums
__global__ void __launch_bounds__(256) decode_kernel(const unsigned char* __restrict__ store,
                                                     const long long* __restrict__ s_off,
                                                     const int* __restrict__ s_nat, const int* __restrict__ s_tgt,
                                                     const long long* __restrict__ index, const SampleAug* aug_all,
                                                     int h, int w, int cout, float* __restrict__ x,
                                                     double* __restrict__ part, int rows_per_block, int final_pass) {
  __shared__ double red[256];
  const int b = blockIdx.x, rb = blockIdx.y;
  const long long s = index[b];
  const unsigned char* img = store + s_off[s];
  const int nat = s_nat[s], tgt = s_tgt[s];
  const SampleAug* aug = aug_all ? aug_all + b : nullptr;
  const int i0 = rb * rows_per_block, i1 = min(h, i0 + rows_per_block);
  const bool bright_first = aug && aug->order == 0.f;
  double gsum = 0.0;
  for (int e = threadIdx.x; e < (i1 - i0) * w; e += blockDim.x) {
    const int i = i0 + e / w, j = e % w;
    int si, sj;
    src_pixel(aug, h, w, i, j, si, sj);
    float v[3] = {0.f, 0.f, 0.f};
    for (int ch = 0; ch < tgt; ++ch) {
      v[ch] = fetch(img, h, w, nat, tgt, ch, si, sj);
      if (bright_first) v[ch] = blend(v[ch], 0.f, aug->bright, aug->one_minus_bright);
    }
    // torchvision rgb_to_grayscale weights for the contrast mean
    gsum += tgt == 3 ? (double)add_rn(add_rn(mul_rn(0.2989f, v[0]), mul_rn(0.587f, v[1])),
                                         mul_rn(0.114f, v[2]))
                     : (double)v[0];
    float* out = x + (((long long)b * h + i) * w + j) * cout;
    for (int ch = 0; ch < cout; ++ch) {
      float o = ch < tgt ? v[ch] : 0.f;
      if (final_pass && ch < tgt) o = div_rn(sub_rn(o, 0.5f), 0.5f);
      out[ch] = o;
    }
  }
  red[threadIdx.x] = gsum;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && part) part[(long long)b * gridDim.y + rb] = red[0];
}

// pass 2 (train): contrast against the image's grayscale mean, then brightness if it comes
// second, then Normalize(0.5, 0.5); padded channels stay 0
__global__ void jitter_normalize_kernel(float* __restrict__ x, const long long* __restrict__ index,
                                        const int* __restrict__ s_tgt, const SampleAug* __restrict__ aug_all,
                                        const double* __restrict__ part, int nparts, int h, int w, int cout, int nb) {
  const long long n = (long long)nb * h * w * cout;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int ch = (int)(e % cout);
    const int b = (int)(e / ((long long)h * w * cout));
    const int tgt = s_tgt[index[b]];
    if (ch >= tgt) continue;
    const SampleAug& a = aug_all[b];
    double sum = 0.0;
    for (int q = 0; q < nparts; ++q) sum += part[(long long)b * nparts + q];  // fixed order
    const float mean = (float)(sum / ((double)h * w));
    float v = x[e];
    v = blend(v, mean, a.contrast, a.one_minus_contrast);
    if (a.order != 0.f) v = blend(v, 0.f, a.bright, a.one_minus_bright);
    x[e] = div_rn(sub_rn(v, 0.5f), 0.5f);
  }
}

__global__ void batch_meta_kernel(const long long* __restrict__ index, const int* __restrict__ s_mod,
                                  const long long* __restrict__ s_label, int nb, int n_mod, float* __restrict__ onehot,
                                  long long* __restrict__ idx_out, long long* __restrict__ labels) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const long long s = index[b];
  const int m = s_mod[s];
  for (int k = 0; k < n_mod; ++k) onehot[(long long)b * n_mod + k] = k == m ? 1.f : 0.f;
  idx_out[b] = m;
  labels[b] = s_label[s];
}

}  // namespace mvae

using namespace mvae;

extern "C" {

size_t mvae_decode_batch_workspace_bytes(int nb, int h) {
  const int rows = 8;
  return (size_t)nb * ((h + rows - 1) / rows) * sizeof(double);
}

int mvae_decode_batch(const unsigned char* store, const long long* sample_offset, const int* sample_channels,
                      const int* sample_target_channels, const int* sample_modality, const long long* sample_label,
                      const long long* index, const float* aug, int nb, int h, int w, int cout, int n_modalities,
                      float* x, float* onehot, long long* modality_idx, long long* labels, void* workspace,
                      size_t workspace_bytes, void* stream) {
  if (nb <= 0 || h <= 0 || w <= 0 || cout < 1 || cout > 3 || n_modalities <= 0) {
    set_error("decode_batch: bad sizes");
    return MVAE_EINVAL;
  }
  const int rows = 8, nparts = (h + rows - 1) / rows;
  if (aug && workspace_bytes < (size_t)nb * nparts * sizeof(double)) {
    set_error("decode_batch: workspace");
    return MVAE_EWORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  const SampleAug* a = (const SampleAug*)aug;
  double* part = aug ? (double*)workspace : nullptr;
  hipLaunchKernelGGL(decode_kernel, dim3(nb, nparts), dim3(256), 0, st, store, sample_offset, sample_channels,
                     sample_target_channels, index, a, h, w, cout, x, part, rows, aug ? 0 : 1);
  if (aug) {
    const long long n = (long long)nb * h * w * cout;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(jitter_normalize_kernel, dim3(blocks), dim3(256), 0, st, x, index, sample_target_channels, a,
                       part, nparts, h, w, cout, nb);
  }
  hipLaunchKernelGGL(batch_meta_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, index, sample_modality, sample_label,
                     nb, n_modalities, onehot, modality_idx, labels);
  return launch_status();
}

}  // extern "C"
