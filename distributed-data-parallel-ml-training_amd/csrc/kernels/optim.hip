// Optimizer and weight-layout kernels for gfx950.
//
// Reference parity: optim.SGD(lr=0.1, momentum=0.9, weight_decay=1e-4) over the 34 VGG-11
// parameter tensors (part1/main.py:124-125, step at :77) — SURVEY.md §2.B N2g. Here ONE
// launch updates the whole flat fp32 parameter arena (all tensors are views into it):
//     d = g * grad_scale + wd * p ; buf = momentum * buf + d ; d = nesterov ? d + momentum*buf : buf
//     p -= lr * d
// A zero-initialised momentum buffer reproduces torch's "buf = clone(d) on the first step"
// exactly (momentum * 0 + d == d), so the kernel needs no first-step flag (graph friendly).
//
// pack_conv_weights re-lays the fp32 master weights (PyTorch [K][C][R][S]) into the two bf16
// MFMA operand layouts used by conv_igemm.hip: Wc [K][R][S][Cpad] (fwd) and Wt [C][R][S][K]
// (dgrad); all conv tensors of the model in one launch (blockIdx.y = tensor).
#include "common.h"
#include "api.h"

namespace ddp_amd {

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ buf, size_t n, float lr,
                                                  float momentum, float wd, float grad_scale,
                                                  int nesterov) {
  const size_t n4 = n / 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 bv = reinterpret_cast<float4*>(buf)[i];
    float* pp = &pv.x;
    const float* gg = &gv.x;
    float* bb = &bv.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = gg[e] * grad_scale + wd * pp[e];
      if (momentum != 0.f) {
        bb[e] = momentum * bb[e] + d;
        d = nesterov ? d + momentum * bb[e] : bb[e];
      }
      pp[e] -= lr * d;
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // scalar tail
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float d = g[i] * grad_scale + wd * p[i];
    if (momentum != 0.f) {
      buf[i] = momentum * buf[i] + d;
      d = nesterov ? d + momentum * buf[i] : buf[i];
    }
    p[i] -= lr * d;
  }
}

constexpr int kMaxPack = 64;
struct PackTable {
  PackDesc d[kMaxPack];
  int n;
};

__global__ __launch_bounds__(256) void pack_conv_weights_kernel(PackTable t) {
  const PackDesc d = t.d[blockIdx.y];
  const int rs = d.R * d.S;
  const size_t total = (size_t)d.K * rs * d.C;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    if (d.wc) {  // i indexes Wc [k][r][s][c]
      const int c = (int)(i % d.C);
      const size_t t1 = i / d.C;
      const int s = (int)(t1 % d.S);
      const size_t t2 = t1 / d.S;
      const int r = (int)(t2 % d.R);
      const int k = (int)(t2 / d.R);
      const float v = c < d.Cr ? d.p[(((size_t)k * d.Cr + c) * d.R + r) * d.S + s] : 0.f;
      d.wc[i] = f2bf(v);
    }
    if (d.wt) {  // i indexes Wt [c][r][s][k]
      const int k = (int)(i % d.K);
      const size_t t1 = i / d.K;
      const int s = (int)(t1 % d.S);
      const size_t t2 = t1 / d.S;
      const int r = (int)(t2 % d.R);
      const int c = (int)(t2 / d.R);
      const float v = c < d.Cr ? d.p[(((size_t)k * d.Cr + c) * d.R + r) * d.S + s] : 0.f;
      d.wt[i] = f2bf(v);
    }
  }
}

__global__ void counter_add_kernel(int* c, int delta) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *c += delta;
}

}  // namespace ddp_amd

using namespace ddp_amd;

extern "C" int ddp_sgd(float* p, const float* g, float* buf, size_t n, float lr, float momentum,
                       float wd, float grad_scale, int nesterov, hipStream_t st) {
  size_t blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sgd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, buf, n, lr,
                     momentum, wd, grad_scale, nesterov);
  return (int)hipGetLastError();
}

extern "C" int ddp_pack_conv_weights(const PackDesc* descs, int n, hipStream_t st) {
  for (int base = 0; base < n; base += kMaxPack) {
    PackTable t{};
    t.n = n - base < kMaxPack ? n - base : kMaxPack;
    size_t maxel = 0;
    for (int i = 0; i < t.n; ++i) {
      t.d[i] = descs[base + i];
      const size_t el = (size_t)t.d[i].K * t.d[i].R * t.d[i].S * t.d[i].C;
      if (el > maxel) maxel = el;
    }
    size_t bx = (maxel + 255) / 256;
    if (bx > 512) bx = 512;
    hipLaunchKernelGGL(pack_conv_weights_kernel, dim3((unsigned)bx, t.n), dim3(256), 0, st, t);
  }
  return (int)hipGetLastError();
}

extern "C" int ddp_counter_add(int* c, int delta, hipStream_t st) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, st, c, delta);
  return (int)hipGetLastError();
}
