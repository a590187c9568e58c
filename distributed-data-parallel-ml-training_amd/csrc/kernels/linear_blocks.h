// Classifier-head weight-gradient block shared by linear_ce.hip (linear_bwd_kernel) and
// conv_igemm.hip (linear_head_bwd_kernel: the head's dW / db in the same launch as its dx fused
// with the last block's BatchNorm backward).
#pragma once
#include "common.h"

namespace ddp_amd {

constexpr int kMaxJ = 16;

// dW / db: block = 64 feature columns x one 64-row batch chunk (4 row groups of 16 rows);
// partial sums reduced through LDS, one atomic per (j, f) per block.
// many small row chunks (latency-bound otherwise), combined with float atomics; the
// deterministic build takes every row in one chunk (one add per address onto zero)
constexpr int kDwRows = kDeterministic ? (1 << 24) : 8;
__device__ __forceinline__ void linear_dw_block(const float* __restrict__ dlogits,
                                                const unsigned short* __restrict__ x, int B, int F,
                                                int J, const float* gscale, float* dW, float* db,
                                                int bx, int by) {
  __shared__ float red[4][kMaxJ][64];
  const int fl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int f = bx * 64 + fl;
  const int r0 = by * kDwRows;
  const int r1 = min(B, r0 + kDwRows);
  const float g = gscale ? *gscale : 1.f;
  float acc[kMaxJ];
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) acc[j] = 0.f;
  if (f < F)
    for (int r = r0 + rg; r < r1; r += 4) {
      const float xv = bf2f(x[(size_t)r * F + f]);
#pragma unroll
      for (int j = 0; j < kMaxJ; ++j)
        if (j < J) acc[j] += dlogits[(size_t)r * J + j] * xv;
    }
#pragma unroll
  for (int j = 0; j < kMaxJ; ++j) red[rg][j][fl] = acc[j];
  __syncthreads();
  if (rg == 0 && f < F) {
#pragma unroll
    for (int j = 0; j < kMaxJ; ++j)
      if (j < J)
        atomicAdd(dW + (size_t)j * F + f,
                  (red[0][j][fl] + red[1][j][fl] + red[2][j][fl] + red[3][j][fl]) * g);
  }
  if (bx == 0 && threadIdx.x < J && db) {
    float s = 0.f;
    for (int r = r0; r < r1; ++r) s += dlogits[(size_t)r * J + threadIdx.x];
    atomicAdd(db + threadIdx.x, s * g);
  }
}


}  // namespace ddp_amd
