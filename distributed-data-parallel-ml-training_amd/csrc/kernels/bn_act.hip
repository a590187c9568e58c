// Fused training-mode BatchNorm + (residual add) + ReLU + (2x2/s2 max-pool) for gfx950.
//
// Reference parity: BatchNorm2d(track_running_stats=False) -> ReLU(inplace) -> MaxPool2d(2,2)
// from part1/model.py:16,24-25. Batch statistics are used in
// both train and eval mode (no running buffers), exactly like the reference.
//
// Forward statistics (per-channel sum / sum of squares of the bf16 conv output) are produced
// by the conv epilogue (conv_igemm.hip), so the forward here is a single streaming pass:
//     a = pool( relu( gamma * (z - mean) * invstd + beta (+ res) ) )
// Backward is two streaming passes that RECOMPUTE the pre-activation from z (no saved masks
// or pool indices):
//     reduce : dy_bn = route_pool(dout) * [y > 0];  S1 += dy_bn, S2 += dy_bn * xhat
//     apply  : dz = gamma*invstd*(dy_bn - S1/M - xhat*S2/M); dgamma += S2, dbeta += S1,
//              dbias(conv) += sum(dz), d_res = dy_bn (residual branch)
// Every thread owns 8 contiguous channels (one 16-byte vector) of one output pixel.
#include "common.h"
#include "api.h"

namespace ddp_amd {

__device__ __forceinline__ void bn_coeffs(const BnArgs& a, int c0, float* scale, float* shift,
                                          float* mean, float* invstd) {
  if (a.use_running) {  // eval mode of track_running_stats=True BatchNorm
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = c0 + e;
      const float mu = a.running_mean[c];
      const float is = rsqrtf(a.running_var[c] + a.eps);
      const float sc = a.gamma[c] * is;
      scale[e] = sc;
      shift[e] = a.beta[c] - mu * sc;
      mean[e] = mu;
      invstd[e] = is;
    }
    return;
  }
  const float inv_m = 1.f / (float)(a.N * a.H * a.W);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  for (int r = 0; r < kStatRep; ++r) {  // sum the contention-spreading replicas
    const float4* p1 = reinterpret_cast<const float4*>(a.stats + r * 2 * a.C + c0);
    const float4* p2 = reinterpret_cast<const float4*>(a.stats + r * 2 * a.C + a.C + c0);
    const float4 x0 = p1[0], x1 = p1[1], y0 = p2[0], y1 = p2[1];
    s1[0] += x0.x; s1[1] += x0.y; s1[2] += x0.z; s1[3] += x0.w;
    s1[4] += x1.x; s1[5] += x1.y; s1[6] += x1.z; s1[7] += x1.w;
    s2[0] += y0.x; s2[1] += y0.y; s2[2] += y0.z; s2[3] += y0.w;
    s2[4] += y1.x; s2[5] += y1.y; s2[6] += y1.z; s2[7] += y1.w;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const float mu = s1[e] * inv_m;
    const float var = fmaxf(s2[e] * inv_m - mu * mu, 0.f);
    const float is = rsqrtf(var + a.eps);
    const float sc = a.gamma[c] * is;
    scale[e] = sc;
    shift[e] = a.beta[c] - mu * sc;
    mean[e] = mu;
    invstd[e] = is;
  }
}

// Block-cooperative per-channel coefficients for channels [c_begin, c_begin + n): the 16
// statistics replicas are summed ONCE per channel per block (not once per thread) into LDS.
__device__ __forceinline__ void block_coeffs(const BnArgs& a, int c_begin, int n, float* l_sc,
                                             float* l_sh, float* l_mu, float* l_is) {
  const float inv_m = 1.f / (float)(a.N * a.H * a.W);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int c = c_begin + i;
    float mu, is;
    if (a.use_running) {
      mu = a.running_mean[c];
      is = rsqrtf(a.running_var[c] + a.eps);
    } else {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < kStatRep; ++r) {
        s1 += a.stats[r * 2 * a.C + c];
        s2 += a.stats[r * 2 * a.C + a.C + c];
      }
      mu = s1 * inv_m;
      is = rsqrtf(fmaxf(s2 * inv_m - mu * mu, 0.f) + a.eps);
    }
    const float sc = a.gamma[c] * is;
    l_sc[i] = sc;
    l_sh[i] = a.beta[c] - mu * sc;
    if (l_mu) l_mu[i] = mu;
    if (l_is) l_is[i] = is;
  }
  __syncthreads();
}

// ------------------------------- forward -------------------------------
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(BnArgs a) {
  const int G = a.C / 8;
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t total = (size_t)a.N * Ho * Wo * G;
  // running statistics (track_running_stats=True, training): block 0 updates every channel
  if (a.running_mean && !a.use_running && blockIdx.x == 0) {
    const float M = (float)(a.N * a.H * a.W);
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      float s1 = 0.f, s2 = 0.f;
      for (int r = 0; r < kStatRep; ++r) {
        s1 += a.stats[r * 2 * a.C + c];
        s2 += a.stats[r * 2 * a.C + a.C + c];
      }
      const float mu = s1 / M;
      const float var = fmaxf(s2 / M - mu * mu, 0.f);
      const float unbiased = M > 1.f ? var * M / (M - 1.f) : var;
      a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mu;
      a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unbiased;
    }
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  block_coeffs(a, 0, a.C, lds, lds + a.C, nullptr, nullptr);
  float sc[8], sh[8];
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
       t += (size_t)gridDim.x * blockDim.x) {
    const int cg = (int)(t % G);
    const size_t pix = t / G;
    const int wo = (int)(pix % Wo);
    const int ho = (int)((pix / Wo) % Ho);
    const int n = (int)(pix / ((size_t)Wo * Ho));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = lds[cg * 8 + e];
      sh[e] = lds[a.C + cg * 8 + e];
    }
    u16x8 o;
    if (!a.pool) {
      const size_t off = (((size_t)n * a.H + ho) * a.W + wo) * a.C + cg * 8;
      const u16x8 zv = ld8(a.z + off);
      u16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (a.res) rv = ld8(a.res + off);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = bf2f(zv[e]) * sc[e] + sh[e];
        if (a.res) y += bf2f(rv[e]);
        if (a.relu) y = fmaxf(y, 0.f);
        o[e] = f2bf(y);
      }
    } else {
      float best[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) best[e] = -INFINITY;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int h = 2 * ho + (d >> 1), w = 2 * wo + (d & 1);
        const size_t off = (((size_t)n * a.H + h) * a.W + w) * a.C + cg * 8;
        const u16x8 zv = ld8(a.z + off);
        u16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
        if (a.res) rv = ld8(a.res + off);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float y = bf2f(zv[e]) * sc[e] + sh[e];
          if (a.res) y += bf2f(rv[e]);
          if (a.relu) y = fmaxf(y, 0.f);
          if (y > best[e] || y != y) best[e] = y;
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    }
    st8(a.out + (((size_t)n * Ho + ho) * Wo + wo) * a.C + cg * 8, o);
  }
}

// ------------------------------- backward -------------------------------
// Computes dy_bn for the (up to 4) pre-pool pixels owned by thread item t.
// POOL: 4 pixels per item, else 1; fills offsets, xhat and dy_bn.
template <bool POOL>
__device__ __forceinline__ void bwd_item(const BnArgs& a, size_t t, int G, int Ho, int Wo,
                                        const float* sc, const float* sh, const float* mu,
                                        const float* is, size_t* offs, float (*xh)[8],
                                        float (*dyb)[8], int* cg_out) {
  const int cg = (int)(t % G);
  *cg_out = cg;
  const size_t pix = t / G;
  const int wo = (int)(pix % Wo);
  const int ho = (int)((pix / Wo) % Ho);
  const int n = (int)(pix / ((size_t)Wo * Ho));
  const u16x8 dv = ld8(a.dout + (((size_t)n * Ho + ho) * Wo + wo) * a.C + cg * 8);
  if (!POOL) {
    const size_t off = (((size_t)n * a.H + ho) * a.W + wo) * a.C + cg * 8;
    offs[0] = off;
    const u16x8 zv = ld8(a.z + off);
    u16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (a.res) rv = ld8(a.res + off);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zf = bf2f(zv[e]);
      float y = zf * sc[e] + sh[e];
      if (a.res) y += bf2f(rv[e]);
      xh[0][e] = (zf - mu[e]) * is[e];
      const float g = bf2f(dv[e]);
      dyb[0][e] = (a.relu && !(y > 0.f)) ? 0.f : g;
    }
    return;
  }
  float best[8], yv[4][8];
  int arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const int h = 2 * ho + (d >> 1), w = 2 * wo + (d & 1);
    const size_t off = (((size_t)n * a.H + h) * a.W + w) * a.C + cg * 8;
    offs[d] = off;
    const u16x8 zv = ld8(a.z + off);
    u16x8 rv = {0, 0, 0, 0, 0, 0, 0, 0};
    if (a.res) rv = ld8(a.res + off);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zf = bf2f(zv[e]);
      float y = zf * sc[e] + sh[e];
      if (a.res) y += bf2f(rv[e]);
      xh[d][e] = (zf - mu[e]) * is[e];
      yv[d][e] = y;
      const float yr = a.relu ? fmaxf(y, 0.f) : y;
      if (yr > best[e] || yr != yr) { best[e] = yr; arg[e] = d; }
    }
  }
#pragma unroll
  for (int d = 0; d < 4; ++d)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = (arg[e] == d) ? bf2f(dv[e]) : 0.f;
      dyb[d][e] = (a.relu && !(yv[d][e] > 0.f)) ? 0.f : g;
    }
}

// Block-wide reduction of 8-channel partial sums for threads that share a channel group.
// Threads are laid out cg_local = tid % Gb; 256/Gb threads share each group.
template <int NV>
__device__ __forceinline__ void block_reduce_atomic(float (&v)[NV][8], int Gb, int cg_base,
                                                    float* const* dst, float* red) {
  const int tid = threadIdx.x;
  const int rows = 256 / Gb;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[e * 256 + tid] = v[k][e];
    __syncthreads();
    for (int idx = tid; idx < Gb * 8; idx += 256) {
      const int cgl = idx / 8, e = idx % 8;
      float s = 0.f;
      for (int r = 0; r < rows; ++r) s += red[e * 256 + r * Gb + cgl];
      if (dst[k]) atomicAdd(dst[k] + (cg_base + cgl) * 8 + e, s);
    }
  }
}

// Grid: x = blocks over pixels, y = channel chunks of (at most) 256 groups.
// Per-thread copy of the block's LDS coefficient tables for its 8 channels.
__device__ __forceinline__ void load_coeffs(const float* lds, int nch, int cl0, float* sc,
                                            float* sh, float* mu, float* is) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = lds[cl0 + e];
    sh[e] = lds[nch + cl0 + e];
    mu[e] = lds[2 * nch + cl0 + e];
    is[e] = lds[3 * nch + cl0 + e];
  }
}

template <bool POOL>
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(BnArgs a) {
  __shared__ float red[8 * 256];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int G = a.C / 8;
  const int Gb = G < 256 ? G : 256;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const int cg_base = blockIdx.y * Gb;
  const int cgl = threadIdx.x % Gb;
  const int prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int nch = Gb * 8;
  block_coeffs(a, cg_base * 8, nch, lds, lds + nch, lds + 2 * nch, lds + 3 * nch);
  float sc[8], sh[8], mu[8], is[8];
  load_coeffs(lds, nch, cgl * 8, sc, sh, mu, is);
  float acc[2][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { acc[0][e] = 0.f; acc[1][e] = 0.f; }
  for (size_t p = blockIdx.x * (size_t)prows + prow; p < npix; p += (size_t)gridDim.x * prows) {
    constexpr int NP = POOL ? 4 : 1;
    size_t offs[NP];
    float xh[NP][8], dyb[NP][8];
    int cg;
    bwd_item<POOL>(a, p * G + cg_base + cgl, G, Ho, Wo, sc, sh, mu, is, offs, xh, dyb, &cg);
#pragma unroll
    for (int d = 0; d < NP; ++d)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        acc[0][e] += dyb[d][e];
        acc[1][e] += dyb[d][e] * xh[d][e];
      }
  }
  float* dst[2] = {a.sums, a.sums + a.C};
  block_reduce_atomic<2>(acc, Gb, cg_base, dst, red);
}

template <bool POOL>
__global__ __launch_bounds__(256) void bn_act_bwd_apply_kernel(BnArgs a) {
  __shared__ float red[8 * 256];
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int G = a.C / 8;
  const int Gb = G < 256 ? G : 256;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const int cg_base = blockIdx.y * Gb;
  const int cgl = threadIdx.x % Gb;
  const int prow = threadIdx.x / Gb, prows = 256 / Gb;
  const float inv_m = 1.f / (float)(a.N * a.H * a.W);
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8], gi[8];
  const int c0 = (cg_base + cgl) * 8;
  const int nch = Gb * 8;
  block_coeffs(a, cg_base * 8, nch, lds, lds + nch, lds + 2 * nch, lds + 3 * nch);
  load_coeffs(lds, nch, cgl * 8, sc, sh, mu, is);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    k1[e] = a.sums[c0 + e] * inv_m;
    k2[e] = a.sums[a.C + c0 + e] * inv_m;
    gi[e] = a.gamma[c0 + e] * is[e];
  }
  // dgamma / dbeta: one contribution per channel from the first block row
  if (blockIdx.x == 0 && prow == 0) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (a.dgamma) atomicAdd(a.dgamma + c0 + e, a.sums[a.C + c0 + e]);
      if (a.dbeta) atomicAdd(a.dbeta + c0 + e, a.sums[c0 + e]);
    }
  }
  float acc[1][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[0][e] = 0.f;
  for (size_t p = blockIdx.x * (size_t)prows + prow; p < npix; p += (size_t)gridDim.x * prows) {
    constexpr int NP = POOL ? 4 : 1;
    size_t offs[NP];
    float xh[NP][8], dyb[NP][8];
    int cg;
    bwd_item<POOL>(a, p * G + cg_base + cgl, G, Ho, Wo, sc, sh, mu, is, offs, xh, dyb, &cg);
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      u16x8 o, r;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dz = gi[e] * (dyb[d][e] - k1[e] - xh[d][e] * k2[e]);
        o[e] = f2bf(dz);
        acc[0][e] += bf2f(o[e]);
        r[e] = f2bf(dyb[d][e]);
      }
      st8(a.dz + offs[d], o);
      if (a.dres) st8(a.dres + offs[d], r);
    }
  }
  if (a.dbias) {
    float* dst[1] = {a.dbias};
    block_reduce_atomic<1>(acc, Gb, cg_base, dst, red);
  }
}

}  // namespace ddp_amd

using namespace ddp_amd;

static int grid_for(size_t items, int cap) {
  size_t b = (items + 255) / 256;
  if (b > (size_t)cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

extern "C" int ddp_bn_act_fwd(const BnArgs* args, hipStream_t st) {
  BnArgs a = *args;
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t items = (size_t)a.N * Ho * Wo * (a.C / 8);
  if (a.C % 8) return -1;
  // each block builds the [scale|shift] table of all C channels in LDS, then streams items
  hipLaunchKernelGGL(bn_act_fwd_kernel, dim3(grid_for(items / 4, 1024)), dim3(256),
                     2 * a.C * sizeof(float), st, a);
  return (int)hipGetLastError();
}

extern "C" int ddp_bn_act_bwd(const BnArgs* args, hipStream_t st) {
  BnArgs a = *args;
  if (a.C % 8) return -1;
  const int G = a.C / 8;
  const int Gb = G < 256 ? G : 256;
  if ((Gb < 256 && 256 % Gb) || (G > 256 && G % 256)) return -1;  // channel groups must tile 256 threads
  const int chunks = (G + Gb - 1) / Gb;
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const size_t rows_per_block = 256 / Gb;
  // enough blocks to fill the chip, but each thread still loops over several pixels
  size_t bx = (npix + rows_per_block * 4 - 1) / (rows_per_block * 4);
  const size_t cap = (size_t)(1024 / chunks > 0 ? 1024 / chunks : 1);
  const size_t lds = 4 * (size_t)Gb * 8 * sizeof(float);
  if (bx > cap) bx = cap;
  if (bx < 1) bx = 1;
  // a.sums must be zero on entry (the caller's per-step scratch is zeroed once per forward)
  if (a.pool) {
    hipLaunchKernelGGL(bn_act_bwd_reduce_kernel<true>, dim3((unsigned)bx, chunks), dim3(256), lds, st, a);
    hipLaunchKernelGGL(bn_act_bwd_apply_kernel<true>, dim3((unsigned)bx, chunks), dim3(256), lds, st, a);
  } else {
    hipLaunchKernelGGL(bn_act_bwd_reduce_kernel<false>, dim3((unsigned)bx, chunks), dim3(256), lds, st, a);
    hipLaunchKernelGGL(bn_act_bwd_apply_kernel<false>, dim3((unsigned)bx, chunks), dim3(256), lds, st, a);
  }
  return (int)hipGetLastError();
}
