// Classifier head for gfx950: small-output Linear fused with softmax cross-entropy.
//
// Reference parity: fc1 = Linear(512, 10) (part1/model.py:40,45) + CrossEntropyLoss (mean)
// (part1/main.py:75,119) and the eval metrics argmax/eq/sum (part1/main.py:105-106);
// SURVEY.md §2.B N2d/N2f/N2i.
//
// fwd  : one wave per row; each lane owns F/64 features, 10 dot products reduced across the
//        wave, softmax in registers, loss/accuracy accumulated with one atomic per row.
//        dlogits = (softmax - onehot) / B is written for the backward (mean reduction).
// bwd  : dx[b][:] = g * dlogits[b] @ W     (one wave per row, bf16 out)
//        dW[j][f] += g * sum_b dlogits[b][j] x[b][f]; db[j] += g * sum_b dlogits[b][j]
//        (both in one launch; g is read from device memory: autograd's incoming gradient)
// The Linear weight is read straight from the fp32 master copy (20 KB).
// A separate generic softmax-CE (any J, logits from the MFMA GEMM) serves ResNet-50's 1000-way head.
#include "common.h"
#include "api.h"
#include "linear_blocks.h"

namespace ddp_amd {


// BN = true: the head input x is the last Conv->BN->ReLU->2x2-pool block's output over 2x2
// images, computed here from its conv output z (HeadBnIn) instead of by a separate BatchNorm
// pass: the block's coefficients are folded from its statistics replicas in every block (block
// 0 writes the [6][F] table its backward reads), each lane applies BN + ReLU to its 8 channels
// of the four window pixels, max-pools them (bn_act.hip's rule) and stores the bf16 feature,
// which then feeds the dot products exactly as a loaded x would.
constexpr int kMaxHeadF = 1024;
template <bool BN>
__global__ __launch_bounds__(256) void linear_ce_fwd_kernel(
    const unsigned short* __restrict__ x, const float* __restrict__ W, const float* __restrict__ b,
    const long long* __restrict__ labels, int B, int F, int J, float inv_b, float* logits_out,
    float* dlogits, float* loss_sum, int* correct, float* loss_acc, HeadBnIn bn) {
  __shared__ float cf[BN ? 2 * kMaxHeadF : 1];
  if constexpr (BN) {
    const float M = 4.f * B;
    for (int c = threadIdx.x; c < F; c += 256) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < kStatRep; ++r) {
        s1 += bn.stats[r * 2 * F + c];
        s2 += bn.stats[r * 2 * F + F + c];
      }
      const float mu = s1 / M;
      const float var = fmaxf(s2 / M - mu * mu, 0.f);
      const float is = rsqrtf(var + bn.eps);
      const float sc = bn.gamma[c] * is, sh = bn.beta[c] - mu * sc;
      cf[c] = sc;
      cf[F + c] = sh;
      if (blockIdx.x == 0) {
        bn.coef[0 * F + c] = sc;
        bn.coef[1 * F + c] = sh;
        bn.coef[2 * F + c] = mu;
        bn.coef[3 * F + c] = is;
      }
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int row_raw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool live = row_raw < B;
  const int row = live ? row_raw : B - 1;  // dead waves recompute the last row, store nothing
  float acc[kMaxJ];
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) acc[j] = 0.f;
  for (int f0 = lane * 8; f0 < F; f0 += 64 * 8) {
    u16x8 xv;
    if constexpr (BN) {
      const unsigned short* zp = bn.z + (size_t)row * 4 * F + f0;  // pixels (0,0) (0,1) (1,0) (1,1)
      u16x8 q[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) q[d] = ld8(zp + d * F);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float best = 0.f;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          float y = bf2f(q[d][e]) * cf[f0 + e] + cf[F + f0 + e];  // (bn_act.hip apply expression)
          if (bn.relu) y = fmaxf(y, 0.f);
          if (d == 0 || y > best || y != y) best = y;  // bn_act.hip's pool rule
        }
        xv[e] = f2bf(best);
      }
      if (live) st8(bn.y + (size_t)row * F + f0, xv);
    } else {
      xv = ld8(x + (size_t)row * F + f0);
    }
    float xf[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) xf[e] = bf2f(xv[e]);
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j) {
      if (j < J) {
        const float4 w0 = *reinterpret_cast<const float4*>(W + (size_t)j * F + f0);
        const float4 w1 = *reinterpret_cast<const float4*>(W + (size_t)j * F + f0 + 4);
        acc[j] += xf[0] * w0.x + xf[1] * w0.y + xf[2] * w0.z + xf[3] * w0.w + xf[4] * w1.x +
                  xf[5] * w1.y + xf[6] * w1.z + xf[7] * w1.w;
      }
    }
  }
  float mx = -INFINITY;
  int arg = 0;
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) {
    if (j < J) {
      acc[j] = wave_sum(acc[j]) + (b ? b[j] : 0.f);
      if (acc[j] > mx) { mx = acc[j]; arg = j; }
    }
  }
  float se = 0.f;
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j)
    if (j < J) se += __expf(acc[j] - mx);
  const float lse = mx + __logf(se);
  const int y = labels ? (int)labels[row] : -1;
  if (live && lane < J) {
    float lj = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j)
      if (j == lane) lj = acc[j];
    if (logits_out) logits_out[(size_t)row * J + lane] = lj;
    if (dlogits && labels) {
      const float p = __expf(lj - lse);
      dlogits[(size_t)row * J + lane] = (p - (lane == y ? 1.f : 0.f)) * inv_b;
    }
  }
  // per-block reduction of the 4 rows' loss / hit terms, then one atomic per accumulator
  __shared__ float lrow[4];
  __shared__ int hrow[4];
  if (lane == 0) {
    float ly = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j)
      if (j == y) ly = acc[j];
    lrow[threadIdx.x >> 6] = (live && labels) ? (lse - ly) * inv_b : 0.f;
    hrow[threadIdx.x >> 6] = (live && labels && arg == y) ? 1 : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0 && labels) {
    float l = 0.f;
    int h = 0;
    for (int r = 0; r < 4; ++r) { l += lrow[r]; h += hrow[r]; }
    if (loss_sum) atomicAdd(loss_sum, l);
    if (loss_acc) atomicAdd(loss_acc, l);  // running sum across steps
    if (correct) atomicAdd(correct, h);
  }
}

// dx: one wave per row (block bx covers rows 4 bx .. 4 bx + 3).
__device__ __forceinline__ void linear_dx_block(const float* __restrict__ dlogits,
                                                const float* __restrict__ W, int B, int F, int J,
                                                const float* gscale, unsigned short* dx, int bx) {
  const int lane = threadIdx.x & 63;
  const int row = bx * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const float g = gscale ? *gscale : 1.f;
  float dl[kMaxJ];
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) dl[j] = (j < J) ? dlogits[(size_t)row * J + j] * g : 0.f;
  for (int f0 = lane * 8; f0 < F; f0 += 64 * 8) {
    float o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j) {
      if (j < J) {
        const float4 w0 = *reinterpret_cast<const float4*>(W + (size_t)j * F + f0);
        const float4 w1 = *reinterpret_cast<const float4*>(W + (size_t)j * F + f0 + 4);
        o[0] += dl[j] * w0.x; o[1] += dl[j] * w0.y; o[2] += dl[j] * w0.z; o[3] += dl[j] * w0.w;
        o[4] += dl[j] * w1.x; o[5] += dl[j] * w1.y; o[6] += dl[j] * w1.z; o[7] += dl[j] * w1.w;
      }
    }
    u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = f2bf(o[e]);
    st8(dx + (size_t)row * F + f0, v);
  }
}

// dx and dW/db in ONE launch: blocks [0, ndx) compute dx rows, the rest dW chunks.
__global__ __launch_bounds__(256) void linear_bwd_kernel(const float* __restrict__ dlogits,
                                                         const unsigned short* __restrict__ x,
                                                         const float* __restrict__ W, int B,
                                                         int F, int J, const float* gscale,
                                                         unsigned short* dx, float* dW, float* db,
                                                         int ndx, int nfx) {
  const int b = blockIdx.x;
  if (b < ndx) {
    linear_dx_block(dlogits, W, B, F, J, gscale, dx, b);
  } else {
    const int t = b - ndx;
    linear_dw_block(dlogits, x, B, F, J, gscale, dW, db, t % nfx, t / nfx);
  }
}

// Generic softmax cross-entropy on [B][J] logits (bf16 or fp32), one block per row.
// Writes dlogits (bf16, scaled by 1/B * g) for the MFMA GEMM backward.
__global__ __launch_bounds__(256) void softmax_ce_kernel(const void* logits, int logits_bf16,
                                                         const long long* labels, int B, int J,
                                                         float inv_b, float* loss_sum,
                                                         int* correct, void* dlogits,
                                                         int dlogits_bf16) {
  __shared__ float red[2][4];
  __shared__ int redi[4];
  const int row = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  auto get = [&](int j) -> float {
    return logits_bf16 ? bf2f(((const unsigned short*)logits)[(size_t)row * J + j])
                       : ((const float*)logits)[(size_t)row * J + j];
  };
  float mx = -INFINITY;
  int arg = 0x7fffffff;
  for (int j = tid; j < J; j += 256) {
    const float v = get(j);
    if (v > mx) { mx = v; arg = j; }
  }
  // argmax with lowest-index tie-break
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(mx, o, kWave);
    const int oa = __shfl_xor(arg, o, kWave);
    if (om > mx || (om == mx && oa < arg)) { mx = om; arg = oa; }
  }
  if (lane == 0) { red[0][wid] = mx; redi[wid] = arg; }
  __syncthreads();
  mx = red[0][0]; arg = redi[0];
  for (int w = 1; w < 4; ++w)
    if (red[0][w] > mx || (red[0][w] == mx && redi[w] < arg)) { mx = red[0][w]; arg = redi[w]; }
  float se = 0.f;
  for (int j = tid; j < J; j += 256) se += __expf(get(j) - mx);
  se = wave_sum(se);
  __syncthreads();
  if (lane == 0) red[1][wid] = se;
  __syncthreads();
  se = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  const float lse = mx + __logf(se);
  const int y = (int)labels[row];
  if (dlogits)
    for (int j = tid; j < J; j += 256) {
      const float p = __expf(get(j) - lse);
      const float d = (p - (j == y ? 1.f : 0.f)) * inv_b;
      if (dlogits_bf16) ((unsigned short*)dlogits)[(size_t)row * J + j] = f2bf(d);
      else ((float*)dlogits)[(size_t)row * J + j] = d;
    }
  if (tid == 0) {
    if (loss_sum) atomicAdd(loss_sum, (lse - get(y)) * inv_b);
    if (correct && arg == y) atomicAdd(correct, 1);
  }
}

}  // namespace ddp_amd

using namespace ddp_amd;

extern "C" int ddp_linear_ce_fwd(const void* x, const float* W, const float* b,
                                 const long long* labels, int B, int F, int J, float* logits,
                                 float* dlogits, float* loss_sum, int* correct, float* loss_acc,
                                 hipStream_t st) {
  if (J > kMaxJ || F % 8) return -1;
  hipLaunchKernelGGL(linear_ce_fwd_kernel<false>, dim3((B + 3) / 4), dim3(256), 0, st,
                     (const unsigned short*)x, W, b, labels, B, F, J, 1.f / (float)B, logits,
                     dlogits, loss_sum, correct, loss_acc, HeadBnIn{});
  return (int)hipGetLastError();
}

// the head with the last block's BatchNorm + ReLU + 2x2 pool folded in (x = bn->y is written)
extern "C" int ddp_bn_pool_linear_ce_fwd(const HeadBnIn* bn, const float* W, const float* b,
                                         const long long* labels, int B, int F, int J,
                                         float* dlogits, float* loss_sum, int* correct,
                                         float* loss_acc, hipStream_t st) {
  if (J > kMaxJ || F % 8 || F > kMaxHeadF || !bn || !bn->z || !bn->stats || !bn->gamma ||
      !bn->beta || !bn->coef || !bn->y)
    return -1;
  hipLaunchKernelGGL(linear_ce_fwd_kernel<true>, dim3((B + 3) / 4), dim3(256), 0, st,
                     (const unsigned short*)bn->y, W, b, labels, B, F, J, 1.f / (float)B,
                     nullptr, dlogits, loss_sum, correct, loss_acc, *bn);
  return (int)hipGetLastError();
}

extern "C" int ddp_linear_bwd(const float* dlogits, const void* x, const float* W, int B, int F,
                              int J, const float* gscale, void* dx, float* dW, float* db,
                              hipStream_t st) {
  if (J > kMaxJ || F % 8) return -1;
  const int ndx = dx ? (B + 3) / 4 : 0;
  const int nfx = (F + 63) / 64, nry = (B + kDwRows - 1) / kDwRows;
  hipLaunchKernelGGL(linear_bwd_kernel, dim3(ndx + nfx * nry), dim3(256), 0, st, dlogits,
                     (const unsigned short*)x, W, B, F, J, gscale, (unsigned short*)dx, dW, db,
                     ndx, nfx);
  return (int)hipGetLastError();
}

extern "C" int ddp_softmax_ce(const void* logits, int logits_bf16, const long long* labels, int B,
                              int J, float* loss_sum, int* correct, void* dlogits,
                              int dlogits_bf16, hipStream_t st) {
  hipLaunchKernelGGL(softmax_ce_kernel, dim3(B), dim3(256), 0, st, logits, logits_bf16, labels, B,
                     J, 1.f / (float)B, loss_sum, correct, dlogits, dlogits_bf16);
  return (int)hipGetLastError();
}
