// Direct MFMA convolution for input layers with few channels (C = 8 after zero-padding the 3
// image channels): VGG-11 layer 0 (3x3 s1, K = 64, reduction 72) and the ResNet-50 stem
// (7x7 s2, K = 64, reduction 392). Reference parity: part1/model.py:18-23 layer 0 conv (+ bias),
// SURVEY.md §2.D row 0 ("pad K to 32; memory-bound; dedicated kernel").
//
// The implicit GEMM is a poor fit here: a 64-wide k-step holds 8 taps of 8 channels, the
// reduction is 1-2 k-steps, and every tile pays an LDS round trip plus a barrier for almost no
// MFMA work. Instead each WAVE owns 16 output pixels x 64 output channels at a time and feeds
// the MFMA straight from global memory:
//   * v_mfma_f32_16x16x32_bf16 wants, per lane, 8 consecutive k-values of one row — exactly
//     one 16-byte load of the 8 (padded) channels of one input pixel at one tap. A k-step of 32
//     covers 4 taps: lane l loads tap 4t + (l >> 4) of pixel (l & 15). No LDS, no barrier.
//   * the weight fragments (Wc [K][R][S][8], 16 B per lane per tap as well) are loaded once per
//     wave into registers when the reduction is short (VGG: 3 k-steps = 48 VGPRs), otherwise
//     re-read per k-step from L1 (stem: 13 k-steps; 50 KB of weights, cache-resident);
//   * operands are swapped (D^T = W x^T) so a lane owns one output pixel and 4 consecutive
//     channels per 16-channel tile: 8-byte bf16 stores;
//   * the BatchNorm statistics of the bf16-rounded output accumulate in registers across all the
//     pixel tiles a wave processes and are reduced once per wave at the end (16 replicas).
// Waves stride over pixel tiles; the A loads of the next tile are issued before the MFMAs of
// the current one.
#include "common.h"
#include "api.h"

#include <algorithm>
#include <cstdlib>

namespace ddp_amd {

namespace {

typedef short v8i16 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8 as_bf16x8(const uint4& v) { return __builtin_bit_cast(bf16x8, v); }

struct SmallKArgs {
  const unsigned short* x;  // [N][H][W][8]
  const unsigned short* wc; // [K][R][S][8]
  const float* bias;        // [K] or null
  unsigned short* y;        // [N][P][Q][K]
  float* stats;             // [kStatRep][2][K] or null
  int N, H, W, K, R, S, stride, pad, P, Q;
  int tiles;                // ceil(N*P*Q / 16)
};

// NT = K / 16 column tiles (<= 4), NKS = ceil(R*S / 4) k-steps; BREG: weights in registers
template <int NT, int NKS, bool BREG>
__global__ __launch_bounds__(256) void conv_smallk_fwd_kernel(SmallKArgs a) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, rl = lane & 15;
  const int RS = a.R * a.S;
  const int M = a.N * a.P * a.Q;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;

  // weight fragments: lane holds Wc[j*16 + rl][tap 4t + g][0..7]
  uint4 wreg[BREG ? NKS : 1][NT];
  auto load_w = [&](int t, int j) -> uint4 {
    const int tap = 4 * t + g;
    if (tap >= RS) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(a.wc + ((size_t)(j * 16 + rl) * RS + tap) * 8);
  };
  if (BREG) {
#pragma unroll
    for (int t = 0; t < NKS; ++t)
#pragma unroll
      for (int j = 0; j < NT; ++j) wreg[t][j] = load_w(t, j);
  }
  float bias[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) bias[j][v] = a.bias ? a.bias[j * 16 + 4 * g + v] : 0.f;

  // activation fragments of one 16-pixel tile
  auto load_x = [&](int tile, uint4 (&xf)[NKS]) {
    const int row = tile * 16 + rl;
    const bool rok = row < M;
    const int rr = rok ? row : 0;
    const int pq = a.P * a.Q;
    const int n = rr / pq, rem = rr - n * pq;
    const int p = rem / a.Q, q = rem - p * a.Q;
    const int h0 = p * a.stride - a.pad, w0 = q * a.stride - a.pad;
#pragma unroll
    for (int t = 0; t < NKS; ++t) {
      const int tap = 4 * t + g;
      const int r = tap / a.S, s = tap - r * a.S;
      const int h = h0 + r, w = w0 + s;
      if (rok && tap < RS && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        xf[t] = *reinterpret_cast<const uint4*>(a.x + (((size_t)n * a.H + h) * a.W + w) * 8);
      else
        xf[t] = make_uint4(0, 0, 0, 0);
    }
  };

  float s1[NT][4], s2[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) { s1[j][v] = 0.f; s2[j][v] = 0.f; }

  // short reductions double-buffer the activation fragments in registers (the next tile's
  // loads fly during this tile's MFMAs); long ones (stem) stream tap by tap and rely on wave
  // parallelism (small register footprint -> high occupancy)
  constexpr bool PREF = NKS <= 4;
  uint4 xf[PREF ? NKS : 1], xn[PREF ? NKS : 1];
  int tile = wave;
  if (PREF && tile < a.tiles) load_x(tile, *reinterpret_cast<uint4(*)[NKS]>(xf));
  for (; tile < a.tiles; tile += nwaves) {
    const int next = tile + nwaves;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (PREF) {
      if (next < a.tiles) load_x(next, *reinterpret_cast<uint4(*)[NKS]>(xn));
#pragma unroll
      for (int t = 0; t < (PREF ? NKS : 1); ++t) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const uint4 wv = BREG ? wreg[BREG ? t : 0][j] : load_w(t, j);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wv), as_bf16x8(xf[t]), acc[j], 0, 0, 0);
        }
      }
    } else {
      const int row = tile * 16 + rl;
      const bool rok = row < M;
      const int rr = rok ? row : 0;
      const int pq = a.P * a.Q;
      const int n = rr / pq, rem = rr - n * pq;
      const int p = rem / a.Q, q = rem - p * a.Q;
      const int h0 = p * a.stride - a.pad, w0 = q * a.stride - a.pad;
      const unsigned short* xb = a.x + (size_t)n * a.H * a.W * 8;
#pragma clang loop unroll(disable)
      for (int t = 0; t < NKS; ++t) {
        // keep the (L1-resident) weight loads inside the loop: hoisting all 4 x NKS fragments
        // out of the tile loop would cost ~200 VGPRs
        asm volatile("" ::: "memory");
        const int tap = 4 * t + g;
        const int r = tap / a.S, s = tap - r * a.S;
        const int h = h0 + r, w = w0 + s;
        uint4 xv = make_uint4(0, 0, 0, 0);
        if (rok && tap < RS && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
          xv = *reinterpret_cast<const uint4*>(xb + ((size_t)h * a.W + w) * 8);
#pragma unroll
        for (int j = 0; j < NT; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(load_w(t, j)), as_bf16x8(xv), acc[j], 0, 0, 0);
      }
    }
    // lane: pixel row tile*16 + rl, channels j*16 + 4g + v
    const int row = tile * 16 + rl;
    if (row < M) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        unsigned short hv[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          hv[v] = f2bf(acc[j][v] + bias[j][v]);
          const float r = bf2f(hv[v]);
          s1[j][v] += r;
          s2[j][v] += r * r;
        }
        uint2 pk;
        pk.x = (unsigned)hv[0] | ((unsigned)hv[1] << 16);
        pk.y = (unsigned)hv[2] | ((unsigned)hv[3] << 16);
        *reinterpret_cast<uint2*>(a.y + (size_t)row * a.K + j * 16 + 4 * g) = pk;
      }
    }
    if (PREF) {
#pragma unroll
      for (int t = 0; t < (PREF ? NKS : 1); ++t) xf[t] = xn[t];
    }
  }
  if (!a.stats) return;
  // reduce over the 16 pixel lanes of each group, then over the block's 4 waves through LDS:
  // ONE atomic per channel per block (memory-side float atomics serialise per address; per-wave
  // atomics cost this kernel more than its MFMA work: 38.6 vs 17.4 us with / without stats)
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        s1[j][v] += __shfl_xor(s1[j][v], m, kWave);
        s2[j][v] += __shfl_xor(s2[j][v], m, kWave);
      }
  __shared__ float red[4][2][64];
  const int wib = threadIdx.x >> 6;
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        red[wib][0][j * 16 + 4 * g + v] = s1[j][v];
        red[wib][1][j * 16 + 4 * g + v] = s2[j][v];
      }
  }
  __syncthreads();
  if (threadIdx.x < 2 * a.K) {
    const int k = threadIdx.x / a.K, c = threadIdx.x - k * a.K;
    const float t = red[0][k][c] + red[1][k][c] + red[2][k][c] + red[3][k][c];
    atomicAdd(a.stats + stat_rep(blockIdx.x) * 2 * a.K + k * a.K + c, stat_val(t, blockIdx.x));
  }
}

// Long reductions (ResNet-50 stem: 7x7 s2, 13 k-steps of 4 taps): the weights (64 x 49 x 8 bf16 =
// 50 KB) do not fit the 32 KB vector L1, so re-reading a weight fragment per MFMA from global
// memory streams ~10 GB through L2 per step at batch 256. Here the block stages all weights in
// LDS once, and every wave works on PT pixel tiles at a time: each LDS weight fragment feeds PT
// MFMAs (register blocking), activation fragments of the next k-step are prefetched.
constexpr int kStemMaxTaps = 52;  // 13 k-steps x 4 taps (7x7 = 49 padded)

template <int NT, int NKS, int PT>
__global__ __launch_bounds__(256) void conv_smallk_lds_kernel(SmallKArgs a) {
  // LDS weight image [NT*16 rows][NKS*4 taps + 1 pad][8 ch] (the pad tap spreads the rows over
  // the LDS banks for the 16-row ds_read_b128 groups)
  constexpr int TAPS = NKS * 4;
  constexpr int ROW = TAPS + 1;
  __shared__ __attribute__((aligned(16))) uint4 wl[NT * 16 * ROW];
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, rl = lane & 15;
  const int RS = a.R * a.S;
  const int M = a.N * a.P * a.Q;
  for (int i = threadIdx.x; i < NT * 16 * TAPS; i += 256) {
    const int k = i / TAPS, tap = i - k * TAPS;
    wl[k * ROW + tap] = tap < RS ? *reinterpret_cast<const uint4*>(a.wc + ((size_t)k * RS + tap) * 8)
                                 : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  float bias[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) bias[j][v] = a.bias ? a.bias[j * 16 + 4 * g + v] : 0.f;
  float s1[NT][4], s2[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v) { s1[j][v] = 0.f; s2[j][v] = 0.f; }

  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int groups = (a.tiles + PT - 1) / PT;  // PT consecutive 16-pixel tiles per group
  const int pq = a.P * a.Q;
  for (int grp = wave; grp < groups; grp += nwaves) {
    int base[PT], h0[PT], w0[PT];
    bool rok[PT];
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int row = (grp * PT + u) * 16 + rl;
      rok[u] = row < M;
      const int rr = rok[u] ? row : 0;
      const int n = rr / pq, rem = rr - n * pq;
      const int p = rem / a.Q, q = rem - p * a.Q;
      base[u] = n * a.H * a.W * 8;
      h0[u] = p * a.stride - a.pad;
      w0[u] = q * a.stride - a.pad;
    }
    auto load_act = [&](int t, uint4 (&xf)[PT]) {
      const int tap = 4 * t + g;
      const int r = tap / a.S, sx = tap - r * a.S;
#pragma unroll
      for (int u = 0; u < PT; ++u) {
        const int h = h0[u] + r, w = w0[u] + sx;
        xf[u] = (rok[u] && tap < RS && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
                    ? *reinterpret_cast<const uint4*>(a.x + base[u] + ((size_t)h * a.W + w) * 8)
                    : make_uint4(0, 0, 0, 0);
      }
    };
    f32x4 acc[PT][NT];
#pragma unroll
    for (int u = 0; u < PT; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[u][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    uint4 xa[PT], xb[PT];
    load_act(0, xa);
#pragma unroll 1
    for (int t = 0; t < NKS; ++t) {
      if (t + 1 < NKS) load_act(t + 1, xb);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint4 wv = wl[(j * 16 + rl) * ROW + 4 * t + g];
#pragma unroll
        for (int u = 0; u < PT; ++u)
          acc[u][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(wv), as_bf16x8(xa[u]), acc[u][j], 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < PT; ++u) xa[u] = xb[u];
    }
#pragma unroll
    for (int u = 0; u < PT; ++u) {
      const int row = (grp * PT + u) * 16 + rl;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        unsigned short hv[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          hv[v] = f2bf(acc[u][j][v] + bias[j][v]);
          const float r = bf2f(hv[v]);
          s1[j][v] += r;
          s2[j][v] += r * r;
        }
        uint2 pk;
        pk.x = (unsigned)hv[0] | ((unsigned)hv[1] << 16);
        pk.y = (unsigned)hv[2] | ((unsigned)hv[3] << 16);
        *reinterpret_cast<uint2*>(a.y + (size_t)row * a.K + j * 16 + 4 * g) = pk;
      }
    }
  }
  if (!a.stats) return;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        s1[j][v] += __shfl_xor(s1[j][v], m, kWave);
        s2[j][v] += __shfl_xor(s2[j][v], m, kWave);
      }
  // block reduction through LDS (the weight image is no longer needed), one atomic per channel
  __syncthreads();
  float* red = reinterpret_cast<float*>(wl);  // [4 waves][2][64]
  const int wib = threadIdx.x >> 6;
  if (rl == 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        red[(wib * 2 + 0) * 64 + j * 16 + 4 * g + v] = s1[j][v];
        red[(wib * 2 + 1) * 64 + j * 16 + 4 * g + v] = s2[j][v];
      }
  }
  __syncthreads();
  if (threadIdx.x < 2 * a.K) {
    const int k = threadIdx.x / a.K, c = threadIdx.x - k * a.K;
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) t += red[(w * 2 + k) * 64 + c];
    atomicAdd(a.stats + stat_rep(blockIdx.x) * 2 * a.K + k * a.K + c, stat_val(t, blockIdx.x));
  }
}

int kSmallkTilesPerWave = 8;

template <int NT, int NKS>
void launch_smallk(const SmallKArgs& a, hipStream_t st) {
  if constexpr (NKS > 4) {
    // weights staged in LDS once per block: few, long-lived blocks (~2 per CU), each wave
    // walking groups of kStemPT pixel tiles
    constexpr int PT = 4;
    const int groups = (a.tiles + PT - 1) / PT;
    const int waves = std::max(1, std::min(groups, 2048));
    hipLaunchKernelGGL((conv_smallk_lds_kernel<NT, NKS, PT>), dim3((waves + 3) / 4), dim3(256), 0, st, a);
    return;
  }
  // ~TPW tiles per wave: enough waves to fill the chip, weight-register loads and the per-block
  // statistics atomics amortised
  const int waves = (a.tiles + kSmallkTilesPerWave - 1) / kSmallkTilesPerWave;
  const int blocks = (waves + 3) / 4;
  hipLaunchKernelGGL((conv_smallk_fwd_kernel<NT, NKS, (NKS <= 4)>), dim3(blocks), dim3(256), 0, st, a);
}

}  // namespace
}  // namespace ddp_amd

using namespace ddp_amd;

// Returns -1 when the shape is not served (caller falls back to the implicit GEMM).
extern "C" int ddp_conv_fwd_smallk(const ConvGeom* g, const void* x, const void* wc,
                                   const float* bias, void* y, float* stats, hipStream_t st) {
  if (g->C != 8 || g->K % 16 || g->K > 64) return -1;
  const int taps = g->R * g->S;
  const int nks = (taps + 3) / 4;
  SmallKArgs a;
  a.x = (const unsigned short*)x;
  a.wc = (const unsigned short*)wc;
  a.bias = bias;
  a.y = (unsigned short*)y;
  a.stats = stats;
  a.N = g->N; a.H = g->H; a.W = g->W; a.K = g->K; a.R = g->R; a.S = g->S;
  a.stride = g->stride; a.pad = g->pad; a.P = g->P; a.Q = g->Q;
  a.tiles = (g->N * g->P * g->Q + 15) / 16;
  const int nt = g->K / 16;
#define DDP_SMALLK(NT_, NKS_) \
  if (nt == NT_ && nks == NKS_) { launch_smallk<NT_, NKS_>(a, st); return (int)hipGetLastError(); }
  DDP_SMALLK(4, 3)   // 3x3, K = 64 (VGG layer 0)
  DDP_SMALLK(4, 13)  // 7x7, K = 64 (ResNet stem)
  DDP_SMALLK(2, 3)
  DDP_SMALLK(1, 3)
#undef DDP_SMALLK
  return -1;
}
