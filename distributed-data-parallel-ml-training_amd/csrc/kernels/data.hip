// On-device synthetic datasets and the fused augmentation kernel (gfx950).
//
// Reference parity: torchvision CIFAR10 + RandomCrop(32, padding=4) -> RandomHorizontalFlip ->
// ToTensor -> Normalize(mean=[125.3,123.0,113.9]/255, std=[63.0,62.1,66.7]/255)
// (part1/main.py:19-50). There is no network on the GPU box and
// no torchvision, so images are generated deterministically from a seed: each class has a
// fixed random template and every image mixes its class template with per-image noise, so
// the task is learnable. The identical integer formula lives in data/synthetic.py (CPU path).
//
// augment: one thread per (sample, output pixel); writes an NHWC bf16 pixel of Cp channels
// (3 real + zero padding to 8, so the first conv runs with C % 8 == 0 on MFMA).
// The sample cursor lives in device memory so the kernel can sit inside a replayed hipGraph.
#include "common.h"
#include "api.h"

namespace ddp_amd {

__host__ __device__ __forceinline__ unsigned char synth_pixel(uint32_t seed, uint32_t idx,
                                                              uint32_t label, uint32_t p) {
  const uint32_t t = hash3(seed, 0x1000u + label, p) & 255u;
  const uint32_t u = hash3(seed ^ 0x5bd1e995u, idx, p) & 255u;
  return (unsigned char)((t * 5u + u * 3u) >> 3);
}

__host__ __device__ __forceinline__ uint32_t synth_label(uint32_t seed, uint32_t idx,
                                                         uint32_t classes) {
  return hash3(seed, idx, 0xabcdefu) % classes;
}

__global__ __launch_bounds__(256) void synth_generate_kernel(unsigned char* images, int* labels,
                                                             int n, int pix_per_img,
                                                             uint32_t seed, int classes) {
  const size_t total = (size_t)n * pix_per_img;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint32_t idx = (uint32_t)(i / pix_per_img);
    const uint32_t p = (uint32_t)(i % pix_per_img);
    const uint32_t label = synth_label(seed, idx, classes);
    images[i] = synth_pixel(seed, idx, label, p);
    if (p == 0) labels[idx] = (int)label;
  }
}

__global__ __launch_bounds__(256) void augment_kernel(AugArgs a) {
  const int cur = a.cursor ? *a.cursor : 0;
  const size_t total = (size_t)a.B * a.H * a.W;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += stride) {
    const int b = (int)(t / ((size_t)a.H * a.W));
    const int pix = (int)(t % ((size_t)a.H * a.W));
    const int oy = pix / a.W, ox = pix % a.W;
    const int pos = (int)(((long long)cur * a.B + b) % a.L);
    const int idx = a.indices[pos];
    int cy = 0, cx = 0, fl = 0;
    if (a.pad > 0 || a.flip) {
      const uint32_t h = hash3(a.seed ^ 0x68e31da4u, a.epoch, (uint32_t)idx);
      const int span = 2 * a.pad + 1;
      cy = (int)(h % span);
      cx = (int)((h / span) % span);
      fl = a.flip ? (int)((h >> 20) & 1u) : 0;
    }
    const int sx = fl ? (a.W - 1 - ox) : ox;            // flip after crop
    const int iy = oy + cy - a.pad, ix = sx + cx - a.pad;  // zero padding outside the image
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    const bool in = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
    const unsigned char* src = a.images + (((size_t)idx * a.H + (in ? iy : 0)) * a.W + (in ? ix : 0)) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float raw = in ? (float)src[c] : 0.f;
      v[c] = f2bf((raw * (1.f / 255.f) - a.mean[c]) * a.inv_std[c]);
    }
    unsigned short* dst = a.x + (size_t)t * a.Cp;
    if (a.Cp == 8) {
      st8(dst, v);
    } else {
      for (int c = 0; c < a.Cp; ++c) dst[c] = c < 8 ? v[c] : 0;
    }
    if (pix == 0) a.y[b] = a.labels[idx];
  }
  // side job: clear the next forward's BN-statistics scratch (saves a fill launch per step)
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < a.zero_n; i += stride)
    a.zero[i] = 0.f;
}

// NCHW fp32 -> NHWC bf16 with channel zero-padding (generic model input).
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, int N,
                                                           int C, int H, int W, int Cp,
                                                           unsigned short* __restrict__ out) {
  const size_t total = (size_t)N * H * W * Cp;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c = (int)(i % Cp);
    const size_t pix = i / Cp;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const int n = (int)(pix / ((size_t)W * H));
    out[i] = c < C ? f2bf(x[(((size_t)n * C + c) * H + h) * W + w]) : 0;
  }
}

}  // namespace ddp_amd

using namespace ddp_amd;

extern "C" int ddp_synth_generate(unsigned char* images, int* labels, int n, int pix_per_img,
                                  unsigned int seed, int classes, hipStream_t st) {
  hipLaunchKernelGGL(synth_generate_kernel, dim3(4096), dim3(256), 0, st, images, labels, n,
                     pix_per_img, seed, classes);
  return (int)hipGetLastError();
}

extern "C" int ddp_augment(const AugArgs* args, hipStream_t st) {
  AugArgs a = *args;
  size_t blocks = ((size_t)a.B * a.H * a.W + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(augment_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

extern "C" int ddp_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cp, void* out,
                                hipStream_t st) {
  size_t blocks = ((size_t)N * H * W * Cp + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, N, C, H, W,
                     Cp, (unsigned short*)out);
  return (int)hipGetLastError();
}
