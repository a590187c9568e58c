// Pooling kernels for gfx950 (NHWC bf16, 8 channels = one 16-byte vector per thread).
//
// ResNet-50 (driver config, SURVEY.md §2.D "Extra ops for the driver's ResNet-50 config"):
//   * MaxPool2d(3, stride 2, padding 1) after the stem: forward stores the window argmax as one
//     byte per element; backward is a GATHER (each input pixel sums the output windows whose
//     argmax points at it) — no atomics, deterministic.
//   * AdaptiveAvgPool2d(1): global average over H*W, backward broadcasts dy / (H*W).
// (VGG's 2x2/s2 max-pool is fused into the BatchNorm/ReLU kernels, bn_act.hip.)
#include "common.h"
#include "api.h"
#include <algorithm>

namespace ddp_amd {

__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const unsigned short* __restrict__ x,
                                                          int N, int H, int W, int C, int KH,
                                                          int KW, int stride, int pad, int Ho,
                                                          int Wo, unsigned short* __restrict__ y,
                                                          unsigned char* __restrict__ idx) {
  // 32-bit index math (the launcher guarantees N*Ho*Wo*C/8 < 2^31): 64-bit divisions by
  // runtime values were most of this kernel's instruction stream
  const unsigned G = C / 8;
  const unsigned total = (unsigned)N * Ho * Wo * G;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned pix = t / G;
    const int cg = (int)(t - pix * G);
    const unsigned prow = pix / (unsigned)Wo;
    const int wo = (int)(pix - prow * Wo);
    const int n = (int)(prow / (unsigned)Ho);
    const int ho = (int)(prow - (unsigned)n * Ho);
    float best[8];
    unsigned char arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
    for (int kh = 0; kh < KH; ++kh) {
      const int h = ho * stride - pad + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int w = wo * stride - pad + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        const u16x8 v = ld8(x + (((size_t)n * H + h) * W + w) * C + cg * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf2f(v[e]);
          if (f > best[e] || f != f) { best[e] = f; arg[e] = (unsigned char)(kh * KW + kw); }
        }
      }
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    const size_t off = (size_t)pix * C + cg * 8;
    st8(y + off, o);
    uint2 packed;
    packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((unsigned)arg[3] << 24);
    packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((unsigned)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + off) = packed;
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const unsigned short* __restrict__ dy,
                                                          const unsigned char* __restrict__ idx,
                                                          int N, int H, int W, int C, int KH,
                                                          int KW, int stride, int pad, int Ho,
                                                          int Wo, unsigned short* __restrict__ dx) {
  const unsigned G = C / 8;
  const unsigned total = (unsigned)N * H * W * G;  // < 2^31 (launcher)
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned pix = t / G;
    const int cg = (int)(t - pix * G);
    const unsigned prow = pix / (unsigned)W;
    const int w = (int)(pix - prow * W);
    const int n = (int)(prow / (unsigned)H);
    const int h = (int)(prow - (unsigned)n * H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // output windows covering (h, w): ho*stride - pad <= h <= ho*stride - pad + KH - 1
    const int ho_lo = max(0, (h + pad - KH + stride) / stride);
    const int ho_hi = min(Ho - 1, (h + pad) / stride);
    const int wo_lo = max(0, (w + pad - KW + stride) / stride);
    const int wo_hi = min(Wo - 1, (w + pad) / stride);
    for (int ho = ho_lo; ho <= ho_hi; ++ho) {
      const int kh = h - (ho * stride - pad);
      if (kh < 0 || kh >= KH) continue;
      for (int wo = wo_lo; wo <= wo_hi; ++wo) {
        const int kw = w - (wo * stride - pad);
        if (kw < 0 || kw >= KW) continue;
        const size_t off = (((size_t)n * Ho + ho) * Wo + wo) * C + cg * 8;
        const uint2 packed = *reinterpret_cast<const uint2*>(idx + off);
        const u16x8 g = ld8(dy + off);
        const unsigned char me = (unsigned char)(kh * KW + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned word = e < 4 ? packed.x : packed.y;
          const unsigned char a = (unsigned char)((word >> (8 * (e & 3))) & 0xff);
          if (a == me) acc[e] += bf2f(g[e]);
        }
      }
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(acc[e]);
    st8(dx + (size_t)pix * C + cg * 8, o);
  }
}

// Global average pool: a block = 64 (n, 8-channel) items x 4 waves, wave w summing pixels
// w, w + 4, ... (4 loads in flight per thread), the 4 partial sums meet in LDS. (One thread per
// item walking all 49 pixels serially ran ResNet-50's 51 MB input in 26 us on 256 blocks.)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const unsigned short* __restrict__ x,
                                                          int N, int HW, int C,
                                                          unsigned short* __restrict__ y) {
  __shared__ float red[3][64][9];
  const int G = C / 8;
  const int it = blockIdx.x * 64 + (threadIdx.x & 63);
  const int wv = threadIdx.x >> 6;
  const bool ok = it < N * G;
  const int n = ok ? it / G : 0, cg = ok ? it % G : 0;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned short* base = x + (size_t)n * HW * C + cg * 8;
  int p = wv;
  for (; p + 12 < HW; p += 16) {
    u16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld8(base + (size_t)(p + 4 * u) * C);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[u][e]);
  }
  for (; p < HW; p += 4) {
    const u16x8 v = ld8(base + (size_t)p * C);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
  }
  if (wv) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wv - 1][threadIdx.x & 63][e] = acc[e];
  }
  __syncthreads();
  if (wv || !ok) return;
  u16x8 o;
  const float inv = 1.f / (float)HW;
#pragma unroll
  for (int e = 0; e < 8; ++e)
    o[e] = f2bf((acc[e] + red[0][threadIdx.x][e] + red[1][threadIdx.x][e] +
                 red[2][threadIdx.x][e]) * inv);
  st8(y + (size_t)n * C + cg * 8, o);
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const unsigned short* __restrict__ dy,
                                                          int N, int HW, int C,
                                                          unsigned short* __restrict__ dx) {
  const int G = C / 8;
  const size_t total = (size_t)N * HW * G;
  const float inv = 1.f / (float)HW;
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int cg = (int)(t % G);
    const size_t pix = t / G;
    const int n = (int)(pix / HW);
    const u16x8 g = ld8(dy + (size_t)n * C + cg * 8);
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(bf2f(g[e]) * inv);
    st8(dx + (size_t)pix * C + cg * 8, o);
  }
}

// db[j] += sum_b dl[b][j]  (bias gradient of a GEMM-based Linear; bf16 dlogits). A block = 16
// columns x 16 row groups (row group r sums rows r, r + 16, ..., 4 loads in flight), partials
// meet in LDS. (One thread per column walking all B rows serially took 62 us for ResNet-50's
// 256 x 1000 logits on 4 blocks.)
__global__ __launch_bounds__(256) void colsum_kernel(const unsigned short* __restrict__ dl, int B,
                                                     int J, float* __restrict__ db) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int j = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (j < J) {
    int b = rg;
    for (; b + 48 < B; b += 64) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = bf2f(dl[(size_t)(b + 16 * u) * J + j]);
      s += (v[0] + v[1]) + (v[2] + v[3]);
    }
    for (; b < B; b += 16) s += bf2f(dl[(size_t)b * J + j]);
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg || j >= J) return;
  float t = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) t += red[r][cl];
  db[j] += t;
}

}  // namespace ddp_amd

using namespace ddp_amd;

static unsigned grid_items(size_t items) {
  size_t b = (items + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int ddp_maxpool_fwd(const void* x, int N, int H, int W, int C, int KH, int KW,
                               int stride, int pad, int Ho, int Wo, void* y, void* idx,
                               hipStream_t st) {
  if (C % 8 || (size_t)N * std::max(H * W, Ho * Wo) * (C / 8) >= (1u << 31)) return -1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_items((size_t)N * Ho * Wo * (C / 8))), dim3(256),
                     0, st, (const unsigned short*)x, N, H, W, C, KH, KW, stride, pad, Ho, Wo,
                     (unsigned short*)y, (unsigned char*)idx);
  return (int)hipGetLastError();
}

extern "C" int ddp_maxpool_bwd(const void* dy, const void* idx, int N, int H, int W, int C, int KH,
                               int KW, int stride, int pad, int Ho, int Wo, void* dx,
                               hipStream_t st) {
  if (C % 8 || (size_t)N * std::max(H * W, Ho * Wo) * (C / 8) >= (1u << 31)) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_items((size_t)N * H * W * (C / 8))), dim3(256),
                     0, st, (const unsigned short*)dy, (const unsigned char*)idx, N, H, W, C, KH,
                     KW, stride, pad, Ho, Wo, (unsigned short*)dx);
  return (int)hipGetLastError();
}

extern "C" int ddp_avgpool_fwd(const void* x, int N, int HW, int C, void* y, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * (C / 8) + 63) / 64), dim3(256), 0, st,
                     (const unsigned short*)x, N, HW, C, (unsigned short*)y);
  return (int)hipGetLastError();
}

extern "C" int ddp_avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, hipStream_t st) {
  if (C % 8) return -1;
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_items((size_t)N * HW * (C / 8))), dim3(256), 0,
                     st, (const unsigned short*)dy, N, HW, C, (unsigned short*)dx);
  return (int)hipGetLastError();
}

extern "C" int ddp_colsum(const void* dl, int B, int J, float* db, hipStream_t st) {
  hipLaunchKernelGGL(colsum_kernel, dim3((J + 15) / 16), dim3(256), 0, st,
                     (const unsigned short*)dl, B, J, db);
  return (int)hipGetLastError();
}
