// Fused training-mode BatchNorm + (residual add) + ReLU + (2x2/s2 max-pool) for gfx950.
//
// Reference parity: BatchNorm2d(track_running_stats=False) -> ReLU(inplace) -> MaxPool2d(2,2)
// from part1/model.py:16,24-25. Batch statistics are used in
// both train and eval mode (no running buffers), exactly like the reference; the ResNet-50
// path (track_running_stats=True) also updates / uses running statistics.
//
// Forward statistics (per-channel sum / sum of squares of the bf16 conv output, in kStatRep
// contention-spreading replicas) are produced by the conv epilogue (conv_igemm.hip).
//   fwd : finalize  — one thread per channel: replicas -> mean, invstd, scale, shift (coef
//                     table, [6][C]); running-statistics update
//         apply     — a = pool( relu( scale * z + shift (+ res) ) ), one streaming pass
//   bwd : reduce    — RECOMPUTES the pre-activation from z (no saved masks / pool indices):
//                     dy_bn = route_pool(dout) * [y > 0];  S1 += dy_bn, S2 += dy_bn * xhat
//                     (replicated partial sums, fp32 atomics)
//         finalize  — one thread per channel: k1 = S1/M, k2 = S2/M; dgamma += S2, dbeta += S1
//         apply     — dz = scale * (dy_bn - k1 - xhat * k2);  d_res = dy_bn (residual branch)
// The coefficient table is built ONCE per layer (a table rebuilt by every block would re-read
// 16 replicas x C channels per block: ~800 MB per ResNet-50 BN layer). For small forward layers
// (blocks x channels x replicas below kFoldBytes) the finalize step is FOLDED into the apply
// kernel instead: every block reduces the replicas it needs into LDS, saving a launch (each
// dispatch costs ~4-5 us of the captured step).
// Every apply/reduce thread owns 8 contiguous channels (one 16-byte vector) of an output pixel
// and reads its coefficients straight from the (L2-resident) table: no LDS, no barrier before
// the streaming loads.
//
// The conv-bias gradient is NOT accumulated: for train-mode BN the gradient w.r.t. its input
// sums to exactly zero over (N, H, W) per channel (BN is invariant to a per-channel constant
// shift), so d(bias) of the producing convolution is identically 0 — PyTorch's value is
// rounding noise around 0 (part1/model.py:18-24: conv with bias followed by BatchNorm2d).
#include "common.h"
#include "api.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace ddp_amd {

enum { kSc = 0, kSh = 1, kMu = 2, kIs = 3, kK1 = 4, kK2 = 5 };  // coef table rows

__device__ __forceinline__ void ld8f(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ------------------------------- finalize kernels -------------------------------
__device__ __forceinline__ void finalize_fwd_ch(const BnArgs& a, int c) {
  float mu, is;
  if (a.use_running) {  // eval mode of track_running_stats=True BatchNorm
    mu = a.running_mean[c];
    is = rsqrtf(a.running_var[c] + a.eps);
  } else {
    const float M = (float)a.N * a.H * a.W;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int r = 0; r < kStatRep; ++r) {
      s1 += a.stats[r * 2 * a.C + c];
      s2 += a.stats[r * 2 * a.C + a.C + c];
    }
    mu = s1 / M;
    const float var = fmaxf(s2 / M - mu * mu, 0.f);
    is = rsqrtf(var + a.eps);
    if (a.running_mean) {  // training with track_running_stats=True (unbiased variance)
      const float unbiased = M > 1.f ? var * M / (M - 1.f) : var;
      a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mu;
      a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unbiased;
    }
  }
  const float sc = a.gamma[c] * is;
  a.coef[kSc * a.C + c] = sc;
  a.coef[kSh * a.C + c] = a.beta[c] - mu * sc;
  a.coef[kMu * a.C + c] = mu;
  a.coef[kIs * a.C + c] = is;
}

__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(BnArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < a.C) finalize_fwd_ch(a, c);
}

// residual block + projection shortcut: both tables in one launch (y = 0: the block's own BN,
// y = 1: the shortcut's)
__global__ __launch_bounds__(256) void bn_finalize_fwd2_kernel(BnArgs a, BnArgs r) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < a.C) finalize_fwd_ch(blockIdx.y ? r : a, c);
}

__global__ __launch_bounds__(256) void bn_finalize_bwd_kernel(BnArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  const float inv_m = 1.f / ((float)a.N * a.H * a.W);
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int r = 0; r < kStatRep; ++r) {
    s1 += a.sums[r * 2 * a.C + c];
    s2 += a.sums[r * 2 * a.C + a.C + c];
  }
  a.coef[kK1 * a.C + c] = s1 * inv_m;
  a.coef[kK2 * a.C + c] = s2 * inv_m;
  if (a.dgamma) a.dgamma[c] += s2;  // one writer per channel: plain accumulate into the arena
  if (a.dbeta) a.dbeta[c] += s1;
}

// ... with the projection shortcut's BN: both BatchNorms see the same gradient dy_bn (the block
// output's gradient through the ReLU mask), so they share S1; the shortcut's S2 (sum dy_bn *
// its xhat) is the third sum of the reduce, in its own replicas' S2 row
__global__ __launch_bounds__(256) void bn_finalize_bwd_res_kernel(BnArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.C) return;
  const float inv_m = 1.f / ((float)a.N * a.H * a.W);
  float s1 = 0.f, s2 = 0.f, s3 = 0.f;
#pragma unroll
  for (int r = 0; r < kStatRep; ++r) {
    s1 += a.sums[r * 2 * a.C + c];
    s2 += a.sums[r * 2 * a.C + a.C + c];
    s3 += a.rsums[r * 2 * a.C + a.C + c];
  }
  a.coef[kK1 * a.C + c] = s1 * inv_m;
  a.coef[kK2 * a.C + c] = s2 * inv_m;
  a.rcoef[kK1 * a.C + c] = s1 * inv_m;
  a.rcoef[kK2 * a.C + c] = s3 * inv_m;
  if (a.dgamma) a.dgamma[c] += s2;
  if (a.dbeta) a.dbeta[c] += s1;
  if (a.rdgamma) a.rdgamma[c] += s3;
  if (a.rdbeta) a.rdbeta[c] += s1;
}

// Replica reduction + coefficients of ALL channels into LDS (sc | sh), done by every block of a
// FOLDed launch (small C x blocks: cheaper than a separate finalize launch); block 0 also writes
// the coef table for the backward and updates the running statistics.
__device__ __forceinline__ void fold_fwd_coeffs(const BnArgs& a, float* l_sc, float* l_sh) {
  const float M = (float)a.N * a.H * a.W;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
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
      mu = s1 / M;
      const float var = fmaxf(s2 / M - mu * mu, 0.f);
      is = rsqrtf(var + a.eps);
      if (a.running_mean && blockIdx.x == 0) {
        const float unbiased = M > 1.f ? var * M / (M - 1.f) : var;
        a.running_mean[c] = (1.f - a.momentum) * a.running_mean[c] + a.momentum * mu;
        a.running_var[c] = (1.f - a.momentum) * a.running_var[c] + a.momentum * unbiased;
      }
    }
    const float sc = a.gamma[c] * is, sh = a.beta[c] - mu * sc;
    l_sc[c] = sc;
    l_sh[c] = sh;
    if (blockIdx.x == 0) {
      a.coef[kSc * a.C + c] = sc;
      a.coef[kSh * a.C + c] = sh;
      a.coef[kMu * a.C + c] = mu;
      a.coef[kIs * a.C + c] = is;
    }
  }
  __syncthreads();
}

// ------------------------------- forward apply -------------------------------
// One thread = IPT items (output pixels) x 8 channels; every load is issued up front. A grid
// smaller than the item blocks walks them with a grid stride (the capped FOLD launch: the
// replica reduction of fold_fwd_coeffs is paid once per block, not once per 256 x IPT items).
// GS: grid-stride launch (a capped FOLD grid); MASK: also store the ReLU mask bits (residual
// blocks, BnArgs::mask). Both are template switches so the common launches keep their code.
// RBN: res is the projection shortcut's pre-BN output, normalised here with BnArgs::rcoef (the
// host guarantees 256 % (C / 8) == 0, so a thread's items share one channel group)
template <bool POOL, int IPT, bool FOLD, bool GS = false, bool MASK = false, bool RBN = false>
__global__ __launch_bounds__(256) void bn_act_fwd_kernel(BnArgs a) {
  constexpr int NP = POOL ? 4 : 1;
  const int G = a.C / 8;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t total = (size_t)a.N * Ho * Wo * G;
  const size_t nbt = GS ? (total + 256 * IPT - 1) / (256 * IPT) : (size_t)blockIdx.x + 1;
  bool folded = false;
  for (size_t blk = blockIdx.x; blk < nbt; blk += gridDim.x) {
  u16x8 zv[IPT][NP], rv[IPT][POOL ? 1 : NP];
  float sc[IPT][8], sh[IPT][8];
  const size_t t0 = blk * 256 * IPT + threadIdx.x;
  float rsc[8], rsh[8];
  if (RBN) {
    const int cg = (int)((t0 < total ? t0 : 0) % G);
    ld8f(a.rcoef + kSc * a.C + cg * 8, rsc);
    ld8f(a.rcoef + kSh * a.C + cg * 8, rsh);
  }
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const size_t t = t0 + it * 256;
    const size_t tt = t < total ? t : 0;
    const int cg = (int)(tt % G);
    const size_t pix = tt / G;
    const int wo = (int)(pix % Wo);
    const int ho = (int)((pix / Wo) % Ho);
    const int n = (int)(pix / ((size_t)Wo * Ho));
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      const int h = POOL ? 2 * ho + (d >> 1) : ho, w = POOL ? 2 * wo + (d & 1) : wo;
      const size_t off = (((size_t)n * a.H + h) * a.W + w) * a.C + cg * 8;
      zv[it][d] = ld8(a.z + off);
      if (!POOL && a.res) rv[it][POOL ? 0 : d] = ld8(a.res + off);
    }
    if (!FOLD) {
      ld8f(a.coef + kSc * a.C + cg * 8, sc[it]);
      ld8f(a.coef + kSh * a.C + cg * 8, sh[it]);
    }
  }
  if (FOLD) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    if (!GS || !folded) {  // (uniform: the first walked item block of every block)
      fold_fwd_coeffs(a, lds, lds + a.C);
      folded = true;
    }
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      const size_t t = t0 + it * 256;
      const int cg = (int)((t < total ? t : 0) % G);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[it][e] = lds[cg * 8 + e];
        sh[it][e] = lds[a.C + cg * 8 + e];
      }
    }
  }
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const size_t t = t0 + it * 256;
    if (t >= total) break;
    const int cg = (int)(t % G);
    const size_t pix = t / G;
    float best[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) best[e] = -INFINITY;
    unsigned mb = 0;
#pragma unroll
    for (int d = 0; d < NP; ++d) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = bf2f(zv[it][d][e]) * sc[it][e] + sh[it][e];
        if (RBN) y += bf2f(rv[it][POOL ? 0 : d][e]) * rsc[e] + rsh[e];
        else if (!POOL && a.res) y += bf2f(rv[it][POOL ? 0 : d][e]);
        if (MASK) mb |= (y > 0.f ? 1u : 0u) << e;  // the backward's ReLU rule (NaN -> 0)
        if (a.relu) y = fmaxf(y, 0.f);
        if (!POOL || y > best[e] || y != y) best[e] = y;
      }
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    st8(a.out + pix * a.C + cg * 8, o);
    if (MASK) a.mask[t] = (unsigned char)mb;  // t = pixel * G + cg
  }
  if (!GS) break;  // (one item block per block)
  }
}

// ------------------------------- backward -------------------------------
// One thread = IPT items x 8 channels. Each item is one (post-pool) output pixel; with POOL its
// 4 pre-pool pixels are recomputed to route the gradient to the window's argmax.
template <bool POOL, int IPT>
struct BwdItems {
  static constexpr int NP = POOL ? 4 : 1;
  u16x8 dv[IPT];
  u16x8 zv[IPT][NP];
  u16x8 rv[IPT][POOL ? 1 : NP];  // residual: only without pooling (host rejects pool + res)
  unsigned mb[IPT];              // ReLU mask byte (BnArgs::mask) in place of the residual
  size_t off[IPT][NP];
  bool ok[IPT];
};

template <bool POOL, int IPT, bool MASK = false, bool RBN = false>
__device__ __forceinline__ void bwd_load(const BnArgs& a, BwdItems<POOL, IPT>& L, size_t p0,
                                         size_t pstride, size_t npix, int cg, int Ho, int Wo) {
  constexpr int NP = POOL ? 4 : 1;
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    const size_t p = p0 + it * pstride;
    L.ok[it] = p < npix;
    const size_t pp = L.ok[it] ? p : 0;
    L.mb[it] = 0;
    const int wo = (int)(pp % Wo);
    const int ho = (int)((pp / Wo) % Ho);
    const int n = (int)(pp / ((size_t)Wo * Ho));
    L.dv[it] = ld8(a.dout + pp * a.C + cg * 8);
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      const int h = POOL ? 2 * ho + (d >> 1) : ho, w = POOL ? 2 * wo + (d & 1) : wo;
      const size_t off = (((size_t)n * a.H + h) * a.W + w) * a.C + cg * 8;
      L.off[it][d] = off;
      L.zv[it][d] = ld8(a.z + off);
      if (MASK) L.mb[it] = a.mask[off / 8];
      // (RBN: the shortcut's pre-BN z, for its xhat)
      if (RBN || (!MASK && !POOL && a.res)) L.rv[it][POOL ? 0 : d] = ld8(a.res + off);
    }
  }
}

// dy_bn (gradient at the BN output, after ReLU mask and pool routing) and xhat for one item
template <bool POOL, bool MASK = false>
__device__ __forceinline__ void bwd_compute(const BnArgs& a, const u16x8& dv, const u16x8* zv,
                                            const u16x8* rv, unsigned mb, const float* sc,
                                            const float* sh, const float* mu, const float* is,
                                            float (*xh)[8], float (*dyb)[8]) {
  constexpr int NP = POOL ? 4 : 1;
  float best[8], yv[NP][8];
  int arg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
  for (int d = 0; d < NP; ++d) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float zf = bf2f(zv[d][e]);
      float y = zf * sc[e] + sh[e];
      if (!POOL && !MASK && a.res) y += bf2f(rv[POOL ? 0 : d][e]);
      xh[d][e] = (zf - mu[e]) * is[e];
      yv[d][e] = y;
      if (POOL) {
        const float yr = a.relu ? fmaxf(y, 0.f) : y;
        if (yr > best[e] || yr != yr) { best[e] = yr; arg[e] = d; }
      }
    }
  }
#pragma unroll
  for (int d = 0; d < NP; ++d)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = (!POOL || arg[e] == d) ? bf2f(dv[e]) : 0.f;
      // with the forward's mask byte: the same verdict (bit e = y > 0), residual never read
      const bool pos = MASK ? ((mb >> e) & 1u) != 0 : yv[d][e] > 0.f;
      dyb[d][e] = (a.relu && !pos) ? 0.f : g;
    }
}

// Grid: x = blocks of (256/Gb) x IPT items, y = channel chunks of (at most) 256 groups.
// Partial sums go to kStatRep replicas of [2][C] (replica = blockIdx.x % kStatRep): the number
// of atomic adders per address drops 16x (memory-side atomics serialise per address).
// STRIDE: the capped grid walks the item blocks (launch_bwd); else one item block per block.
// RBN (projection shortcut folded in): a third sum, S2 of the shortcut's BN (sum dy_bn * its
// xhat), into BnArgs::rsums' S2 row (S1 is shared: both BNs see the same dy_bn)
template <bool POOL, int IPT, bool MASK = false, bool STRIDE = false, bool RBN = false>
__global__ __launch_bounds__(256) void bn_act_bwd_reduce_kernel(BnArgs a) {
  constexpr int NS = RBN ? 3 : 2;
  constexpr int NP = POOL ? 4 : 1;
  __shared__ float red[8 * 256];
  DDP_DEVICE_CHECK(a.C % 8 == 0 && (!POOL || (a.H % 2 == 0 && a.W % 2 == 0)));
  const int G = a.C / 8;
  const int Gb = a.red_gb ? a.red_gb : (G < 256 ? G : 256);  // (reduce_split)
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const int cg_base = blockIdx.y * Gb;
  const int cgl = threadIdx.x % Gb;
  const int prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int c0 = (cg_base + cgl) * 8;
  // grid-stride over the item blocks (nbx of them): a capped grid adds its partial sums once
  // per block instead of once per 256 x IPT items (launch_bwd's reduce grid). The items of the
  // first block are loaded before the coefficients (the one-block-per-item launch's order).
  const size_t per_blk = (size_t)prows * IPT;
  const size_t nbx = STRIDE ? (npix + per_blk - 1) / per_blk : (size_t)blockIdx.x + 1;
  BwdItems<POOL, IPT> L;
  bwd_load<POOL, IPT, MASK, RBN>(a, L, (size_t)blockIdx.x * per_blk + prow, prows, npix,
                                 cg_base + cgl, Ho, Wo);
  float sc[8], sh[8], mu[8], is[8], rmu[8], ris[8];
  ld8f(a.coef + kSc * a.C + c0, sc);
  ld8f(a.coef + kSh * a.C + c0, sh);
  ld8f(a.coef + kMu * a.C + c0, mu);
  ld8f(a.coef + kIs * a.C + c0, is);
  if (RBN) {
    ld8f(a.rcoef + kMu * a.C + c0, rmu);
    ld8f(a.rcoef + kIs * a.C + c0, ris);
  }
  float acc[NS][8];
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  for (size_t bb = blockIdx.x;;) {
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      if (!L.ok[it]) continue;
      float xh[NP][8], dyb[NP][8];
      bwd_compute<POOL, MASK>(a, L.dv[it], L.zv[it], L.rv[it], L.mb[it], sc, sh, mu, is, xh, dyb);
#pragma unroll
      for (int d = 0; d < NP; ++d) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          acc[0][e] += dyb[d][e];
          acc[1][e] += dyb[d][e] * xh[d][e];
          if (RBN) acc[NS - 1][e] += dyb[d][e] * ((bf2f(L.rv[it][0][e]) - rmu[e]) * ris[e]);
        }
      }
    }
    bb += gridDim.x;
    if (!STRIDE || bb >= nbx) break;
    bwd_load<POOL, IPT, MASK, RBN>(a, L, bb * per_blk + prow, prows, npix, cg_base + cgl, Ho, Wo);
  }
  // block reduction over the 256/Gb threads sharing each channel group, then one atomic per
  // channel per block into this block's replica
  float* rep = a.sums + stat_rep(blockIdx.x) * 2 * a.C;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    if (k) __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) red[e * 256 + tid] = acc[k][e];
    __syncthreads();
    // (k == 2: the shortcut's S2 row)
    float* dst = k < 2 ? rep + k * a.C : a.rsums + stat_rep(blockIdx.x) * 2 * a.C + a.C;
    for (int idx = tid; idx < Gb * 8; idx += 256) {
      const int g = idx / 8, e = idx % 8;
      float s = 0.f;
      for (int r = 0; r < prows; ++r) s += red[e * 256 + r * Gb + g];
      atomicAdd(dst + (cg_base + g) * 8 + e, stat_val(s, blockIdx.x));
    }
  }
}

// FOLD: the backward finalize folded into the apply (no bn_finalize_bwd launch): the block's
// 256 threads load the 16 replicas of its channel chunk's S1 / S2 with coalesced 16-B loads (16
// per thread at 256 channels), reduce them in registers in replica order — the finalize's own
// order, so k1 / k2 are bit-identical to the separate launch — and hand k1 / k2 over in LDS;
// blocks x == 0 also add dgamma / dbeta and write the table's k1 / k2 rows. The launcher folds
// only while the grid's replica re-reads stay small (kFoldBwdBytes).
// RBN: also the projection shortcut's dz (BnArgs::rdz) from the same dy_bn and its own table.
template <bool POOL, int IPT, bool FOLD = false, bool MASK = false, bool STRIDE = false,
          bool RBN = false>
__global__ __launch_bounds__(256) void bn_act_bwd_apply_kernel(BnArgs a) {
  constexpr int NP = POOL ? 4 : 1;
  const int G = a.C / 8;
  const int Gb = G < 256 ? G : 256;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const int cg_base = blockIdx.y * Gb;
  const int cgl = threadIdx.x % Gb;
  const int prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int c0 = (cg_base + cgl) * 8;
  // a capped FOLD grid walks the item blocks with a grid stride (one replica fold per block)
  const size_t per_blk = (size_t)prows * IPT;
  const size_t nbx = (npix + per_blk - 1) / per_blk;
  BwdItems<POOL, IPT> L;
  bwd_load<POOL, IPT, MASK, RBN>(a, L, (size_t)blockIdx.x * per_blk + prow, prows, npix,
                                 cg_base + cgl, Ho, Wo);
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8], rsc[8], rmu[8], ris[8], rk2[8];
  if (RBN) {
    ld8f(a.rcoef + kSc * a.C + c0, rsc);
    ld8f(a.rcoef + kMu * a.C + c0, rmu);
    ld8f(a.rcoef + kIs * a.C + c0, ris);
    ld8f(a.rcoef + kK2 * a.C + c0, rk2);
  }
  ld8f(a.coef + kSc * a.C + c0, sc);
  ld8f(a.coef + kSh * a.C + c0, sh);
  ld8f(a.coef + kMu * a.C + c0, mu);
  ld8f(a.coef + kIs * a.C + c0, is);
  if (FOLD) {
    __shared__ __attribute__((aligned(16))) float kk[2][2048];  // k1 | k2 of the chunk
    const int nch = Gb * 8;                 // channels of this block's chunk (<= 2048)
    const float inv_m = 1.f / ((float)a.N * a.H * a.W);
    // 4 consecutive values (one float4) per thread and pass: [which][channel] of the chunk
    for (int q = threadIdx.x * 4; q < 2 * nch; q += 1024) {
      const int which = q / nch, cl = q - which * nch;
      const float* src = a.sums + which * a.C + cg_base * 8 + cl;
      float4 t = *reinterpret_cast<const float4*>(src);
#pragma unroll
      for (int r = 1; r < kStatRep; ++r) {
        const float4 v = *reinterpret_cast<const float4*>(src + (size_t)r * 2 * a.C);
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        kk[which][cl + e] = tv[e] * inv_m;
        if (blockIdx.x == 0) {
          const int c = cg_base * 8 + cl + e;
          a.coef[(which ? kK2 : kK1) * a.C + c] = tv[e] * inv_m;
          float* dst = which ? a.dgamma : a.dbeta;  // S2 -> dgamma, S1 -> dbeta
          if (dst) dst[c] += tv[e];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      k1[e] = kk[0][cgl * 8 + e];
      k2[e] = kk[1][cgl * 8 + e];
    }
  } else {
    ld8f(a.coef + kK1 * a.C + c0, k1);
    ld8f(a.coef + kK2 * a.C + c0, k2);
  }
  for (size_t bb = blockIdx.x;;) {
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
      if (!L.ok[it]) continue;
      float xh[NP][8], dyb[NP][8];
      bwd_compute<POOL, MASK>(a, L.dv[it], L.zv[it], L.rv[it], L.mb[it], sc, sh, mu, is, xh, dyb);
#pragma unroll
      for (int d = 0; d < NP; ++d) {
        u16x8 o, r;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = f2bf(sc[e] * (dyb[d][e] - k1[e] - xh[d][e] * k2[e]));  // sc = gamma * invstd
          if (RBN) {  // the shortcut's BN backward: same dy_bn and k1, its xhat / k2 / scale
            const float xr = (bf2f(L.rv[it][0][e]) - rmu[e]) * ris[e];
            r[e] = f2bf(rsc[e] * (dyb[d][e] - k1[e] - xr * rk2[e]));
          } else {
            r[e] = f2bf(dyb[d][e]);
          }
        }
        st8(a.dz + L.off[it][d], o);
        if (RBN) st8(a.rdz + L.off[it][d], r);
        else if (a.dres) st8(a.dres + L.off[it][d], r);
      }
    }
    bb += gridDim.x;
    if (!STRIDE || bb >= nbx) break;
    bwd_load<POOL, IPT, MASK, RBN>(a, L, bb * per_blk + prow, prows, npix, cg_base + cgl, Ho, Wo);
  }
}

// ------------------------------- backward, one block per channel group -------------------------------
// Small layers (the strong-scaling batches): ONE block owns 8 channels over EVERY (post-pool)
// pixel. Its threads keep their items (dy, z [, res]) in registers, the block reduces S1 / S2
// itself (wave shuffles + LDS: no atomics, no replicas), writes dgamma / dbeta / k1 / k2, and
// applies from the same registers: the whole BatchNorm backward is ONE launch instead of three
// dependent ones (reduce, finalize, apply ~ 4.5 us each in the captured b32 step), and dy / z are
// read once instead of twice.
template <bool POOL, int IPT, int NT, bool MASK = false>
__global__ __launch_bounds__(NT) void bn_act_bwd_local_kernel(BnArgs a) {
  constexpr int NP = POOL ? 4 : 1;
  constexpr int NW = NT / kWave;
  __shared__ float red[NW][16];
  __shared__ float fin[16];
  const int cg = blockIdx.x;
  const int c0 = cg * 8;
  const int Ho = POOL ? a.H / 2 : a.H, Wo = POOL ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  BwdItems<POOL, IPT> L;
  bwd_load<POOL, IPT, MASK>(a, L, threadIdx.x, NT, npix, cg, Ho, Wo);
  float sc[8], sh[8], mu[8], is[8];
  ld8f(a.coef + kSc * a.C + c0, sc);
  ld8f(a.coef + kSh * a.C + c0, sh);
  ld8f(a.coef + kMu * a.C + c0, mu);
  ld8f(a.coef + kIs * a.C + c0, is);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    if (!L.ok[it]) continue;
    float xh[NP][8], dyb[NP][8];
    bwd_compute<POOL, MASK>(a, L.dv[it], L.zv[it], L.rv[it], L.mb[it], sc, sh, mu, is, xh, dyb);
#pragma unroll
    for (int d = 0; d < NP; ++d)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += dyb[d][e];
        s2[e] += dyb[d][e] * xh[d][e];
      }
  }
  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t1 = wave_sum(s1[e]), t2 = wave_sum(s2[e]);
    if (lane == 0) { red[wave][e] = t1; red[wave][8 + e] = t2; }
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += red[w][threadIdx.x];
    fin[threadIdx.x] = t;
    const int e = threadIdx.x & 7;
    const float inv_m = 1.f / ((float)a.N * a.H * a.W);
    if (threadIdx.x < 8) {
      a.coef[kK1 * a.C + c0 + e] = t * inv_m;
      if (a.dbeta) a.dbeta[c0 + e] += t;  // one block per channel: plain accumulate
    } else {
      a.coef[kK2 * a.C + c0 + e] = t * inv_m;
      if (a.dgamma) a.dgamma[c0 + e] += t;
    }
  }
  __syncthreads();
  const float inv_m = 1.f / ((float)a.N * a.H * a.W);
  float k1[8], k2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { k1[e] = fin[e] * inv_m; k2[e] = fin[8 + e] * inv_m; }
#pragma unroll
  for (int it = 0; it < IPT; ++it) {
    if (!L.ok[it]) continue;
    float xh[NP][8], dyb[NP][8];
    bwd_compute<POOL, MASK>(a, L.dv[it], L.zv[it], L.rv[it], L.mb[it], sc, sh, mu, is, xh, dyb);
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      u16x8 o, r;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        o[e] = f2bf(sc[e] * (dyb[d][e] - k1[e] - xh[d][e] * k2[e]));
        r[e] = f2bf(dyb[d][e]);
      }
      st8(a.dz + L.off[it][d], o);
      if (a.dres) st8(a.dres + L.off[it][d], r);
    }
  }
}

// ------------------------------- ResNet stem: BN + ReLU + 3x3/s2/p1 max-pool -------------------------------
// The stem's 112x112 BatchNorm output only exists to be max-pooled (torchvision ResNet conv1 ->
// bn1 -> relu -> maxpool): forward computes relu(scale*z + shift) for the nine taps of each
// pooled output and stores only the pooled value and the window argmax (one byte); backward
// routes the pooled gradient by a GATHER (each input pixel sums the <= 2x2 windows whose argmax
// is its tap) straight into the BN-backward reduce and apply, so neither the 411 MB pre-pool
// activation (batch 256) nor its gradient is ever written. Argmax tie-break / NaN rule: first
// tap in row-major window order, NaN wins (pool.hip maxpool_fwd_kernel).
constexpr int kP3 = 3, kP3S = 2, kP3P = 1;

__global__ __launch_bounds__(256) void bn_pool3_fwd_kernel(BnArgs a, int Ho, int Wo,
                                                           unsigned char* __restrict__ idx) {
  const unsigned G = a.C / 8;
  const unsigned total = (unsigned)a.N * Ho * Wo * G;  // < 2^31 (host)
  for (unsigned t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const unsigned pix = t / G;
    const int cg = (int)(t - pix * G);
    const unsigned prow = pix / (unsigned)Wo;
    const int wo = (int)(pix - prow * Wo);
    const int n = (int)(prow / (unsigned)Ho);
    const int ho = (int)(prow - (unsigned)n * Ho);
    float sc[8], sh[8], best[8];
    unsigned char arg[8];
    ld8f(a.coef + kSc * a.C + cg * 8, sc);
    ld8f(a.coef + kSh * a.C + cg * 8, sh);
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
    for (int kh = 0; kh < kP3; ++kh) {
      const int h = ho * kP3S - kP3P + kh;
      if ((unsigned)h >= (unsigned)a.H) continue;
#pragma unroll
      for (int kw = 0; kw < kP3; ++kw) {
        const int w = wo * kP3S - kP3P + kw;
        if ((unsigned)w >= (unsigned)a.W) continue;
        const u16x8 v = ld8(a.z + (((size_t)n * a.H + h) * a.W + w) * a.C + cg * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float y = bf2f(v[e]) * sc[e] + sh[e];
          if (a.relu) y = fmaxf(y, 0.f);
          if (y > best[e] || y != y) { best[e] = y; arg[e] = (unsigned char)(kh * kP3 + kw); }
        }
      }
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    const size_t off = (size_t)pix * a.C + cg * 8;
    st8(a.out + off, o);
    uint2 packed;
    packed.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((unsigned)arg[3] << 24);
    packed.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((unsigned)arg[7] << 24);
    *reinterpret_cast<uint2*>(idx + off) = packed;
  }
}

// Backward item = the 2x2 pre-pool pixels (2i+a, 2j+b) of pooled position (i, j), 8 channels.
// With k3 / s2 / p1 a pre-pool row 2i is covered only by window row i (tap row 1), row 2i+1 by
// window rows i (tap 2) and i+1 (tap 0) — same for columns — so the four windows (i..i+1,
// j..j+1) serve all four pixels: 4 argmax + 4 gradient loads instead of 9 of each, and 4
// independent z loads per thread.
struct Pool3Quad {
  u16x8 z[4];      // pixel (a, b) -> z[2a + b]
  float dyb[4][8]; // gradient at the BN output (window-routed, ReLU-masked)
  bool ok[4];
  size_t off[4];
};

__device__ __forceinline__ void pool3_quad(const BnArgs& a, const unsigned char* __restrict__ idx,
                                           int Ho, int Wo, int n, int i, int j, int cg,
                                           const float* sc, const float* sh, Pool3Quad& q) {
  u16x8 d[4];
  uint2 am[4];
  bool wok[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {  // window (i + (t >> 1), j + (t & 1))
    const int ho = i + (t >> 1), wo = j + (t & 1);
    wok[t] = ho < Ho && wo < Wo;
    const size_t off = (((size_t)n * Ho + (wok[t] ? ho : i)) * Wo + (wok[t] ? wo : j)) * a.C + cg * 8;
    am[t] = *reinterpret_cast<const uint2*>(idx + off);
    d[t] = ld8(a.dout + off);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // pre-pool pixel (2i + (p >> 1), 2j + (p & 1))
    const int h = 2 * i + (p >> 1), w = 2 * j + (p & 1);
    q.ok[p] = h < a.H && w < a.W;
    q.off[p] = ((((size_t)n * a.H + (q.ok[p] ? h : 2 * i)) * a.W) + (q.ok[p] ? w : 2 * j)) * a.C + cg * 8;
    q.z[p] = ld8(a.z + q.off[p]);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int pa = p >> 1, pb = p & 1;
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int da = t >> 1, db = t & 1;
      if (pa == 0 && da == 1) continue;  // row 2i: only window row i
      if (pb == 0 && db == 1) continue;
      const int kh = pa == 0 ? 1 : (da == 0 ? 2 : 0), kw = pb == 0 ? 1 : (db == 0 ? 2 : 0);
      const unsigned me = (unsigned)(kh * kP3 + kw);
      if (!wok[t]) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned word = e < 4 ? am[t].x : am[t].y;
        if (((word >> (8 * (e & 3))) & 0xffu) == me) g[e] += bf2f(d[t][e]);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float y = bf2f(q.z[p][e]) * sc[e] + sh[e];
      q.dyb[p][e] = (a.relu && !(y > 0.f)) ? 0.f : g[e];
    }
  }
}

// APPLY = false: S1 / S2 (grid-stride over the 2x2 quads, one channel group per thread, block
// reduction, one atomic per channel per block into a replica); APPLY = true: dz.
template <bool APPLY>
__global__ __launch_bounds__(256) void bn_pool3_bwd_kernel(BnArgs a, int Ho, int Wo,
                                                           const unsigned char* __restrict__ idx) {
  const int G = a.C / 8;            // host: 64 % G == 0
  const int cg = threadIdx.x % G;
  const int per = 256 / G;          // quads per block iteration
  const unsigned nq = (unsigned)a.N * Ho * Wo;
  float sc[8], sh[8], mu[8], is[8], k1[8], k2[8];
  ld8f(a.coef + kSc * a.C + cg * 8, sc);
  ld8f(a.coef + kSh * a.C + cg * 8, sh);
  ld8f(a.coef + kMu * a.C + cg * 8, mu);
  ld8f(a.coef + kIs * a.C + cg * 8, is);
  if (APPLY) {
    ld8f(a.coef + kK1 * a.C + cg * 8, k1);
    ld8f(a.coef + kK2 * a.C + cg * 8, k2);
  }
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  for (unsigned qi = blockIdx.x * per + threadIdx.x / G; qi < nq; qi += gridDim.x * per) {
    const unsigned prow = qi / (unsigned)Wo;
    const int j = (int)(qi - prow * Wo);
    const int n = (int)(prow / (unsigned)Ho);
    const int i = (int)(prow - (unsigned)n * Ho);
    Pool3Quad q;
    pool3_quad(a, idx, Ho, Wo, n, i, j, cg, sc, sh, q);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (!q.ok[p]) continue;
      if (APPLY) {
        u16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (bf2f(q.z[p][e]) - mu[e]) * is[e];
          o[e] = f2bf(sc[e] * (q.dyb[p][e] - k1[e] - xh * k2[e]));
        }
        st8(a.dz + q.off[p], o);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += q.dyb[p][e];
          s2[e] += q.dyb[p][e] * ((bf2f(q.z[p][e]) - mu[e]) * is[e]);
        }
      }
    }
  }
  if (APPLY) return;
  // lanes l, l + G, ... of a wave share the channel group: butterfly, then the 4 waves via LDS
  for (int m = G; m < 64; m *= 2)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s1[e] += __shfl_xor(s1[e], m);
      s2[e] += __shfl_xor(s2[e], m);
    }
  __shared__ float red[4][2][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane < G) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[wv][0][lane * 8 + e] = s1[e];
      red[wv][1][lane * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  float* rep = a.sums + stat_rep(blockIdx.x) * 2 * a.C;
  for (int k = threadIdx.x; k < 2 * a.C; k += 256) {
    const int which = k / a.C, c = k - which * a.C;
    atomicAdd(rep + which * a.C + c,
              stat_val(red[0][which][c] + red[1][which][c] + red[2][which][c] + red[3][which][c],
                       blockIdx.x));
  }
}

}  // namespace ddp_amd

using namespace ddp_amd;

static unsigned blocks_for(size_t items, size_t per_block) {
  size_t b = (items + per_block - 1) / per_block;
  return (unsigned)(b < 1 ? 1 : b);
}

// Folding the finalize into the apply kernel costs every block a replica reduction of its
// channels; worth it (one launch fewer) while that re-read traffic stays small.
constexpr size_t kFoldBytes = 24u << 20;
// Big layers: the FOLD kernels on a capped grid (fold_fwd_grid() blocks walking the
// item blocks, forward and backward apply) while that grid's replica re-reads stay within
// kFoldGridBytes. Off by default: at 2048 blocks ResNet-50 b256 ran 26.26 vs 25.68 ms with the
// separate finalize launches (profiles/r5v_bn_fold.md) — the 25088-block streaming applies
// lose more to the capped grid than the finalize launch costs.
constexpr size_t kFoldGridBytes = 64u << 20;
static unsigned g_fold_grid = 0;  // ddp_bn_fold_grid (A/B studies)
static unsigned fold_fwd_grid() { return g_fold_grid; }
extern "C" void ddp_bn_fold_grid(int blocks) { g_fold_grid = blocks > 0 ? (unsigned)blocks : 0u; }

template <bool POOL, int IPT, bool MASK>
static void launch_fwd_m(const BnArgs& a, size_t items, hipStream_t st) {
  const unsigned nb = blocks_for(items, 256 * IPT);
  const size_t per_block = (size_t)a.C * 2 * kStatRep * sizeof(float);
  const unsigned cap = std::min(nb, fold_fwd_grid());
  if ((size_t)nb * per_block <= kFoldBytes) {
    hipLaunchKernelGGL((bn_act_fwd_kernel<POOL, IPT, true, false, MASK>), dim3(nb), dim3(256),
                       2 * a.C * sizeof(float), st, a);
  } else if (!kDeterministic && cap >= 1024 && (size_t)cap * per_block <= kFoldGridBytes) {
    hipLaunchKernelGGL((bn_act_fwd_kernel<POOL, IPT, true, true, MASK>), dim3(cap), dim3(256),
                       2 * a.C * sizeof(float), st, a);
  } else {
    hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(blocks_for(a.C, 256)), dim3(256), 0, st, a);
    hipLaunchKernelGGL((bn_act_fwd_kernel<POOL, IPT, false, false, MASK>), dim3(nb), dim3(256), 0,
                       st, a);
  }
}

template <bool POOL, int IPT>
static void launch_fwd(const BnArgs& a, size_t items, hipStream_t st) {
  if constexpr (!POOL) {
    if (a.mask) return launch_fwd_m<POOL, IPT, true>(a, items, st);
  }
  launch_fwd_m<POOL, IPT, false>(a, items, st);
}

// residual block + projection shortcut BN (ddp_bn_act_fwd_res): both finalizes in one launch,
// then the apply normalising both inputs (never folded: a shortcut block's layers are big)
template <int IPT>
static void launch_fwd_res(const BnArgs& a, const BnArgs& r, size_t items, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_fwd2_kernel, dim3(blocks_for(a.C, 256), 2), dim3(256), 0, st, a, r);
  const unsigned nb = blocks_for(items, 256 * IPT);
  if (a.mask)
    hipLaunchKernelGGL((bn_act_fwd_kernel<false, IPT, false, false, true, true>), dim3(nb),
                       dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((bn_act_fwd_kernel<false, IPT, false, false, false, true>), dim3(nb),
                       dim3(256), 0, st, a);
}

// the shortcut's table goes to a.rcoef; r carries its stats / gamma / beta / running buffers
static bool res_shape_ok(const BnArgs& a) {
  return a.C % 8 == 0 && 256 % (a.C / 8) == 0 && !a.pool && a.relu && a.res && a.rcoef &&
         a.coef;
}

extern "C" int ddp_bn_act_fwd_res(const BnArgs* args, const BnArgs* rargs, hipStream_t st) {
  BnArgs a = *args;
  BnArgs r = *rargs;
  if (!res_shape_ok(a) || r.coef != a.rcoef || r.C != a.C || r.stats == nullptr) return -1;
  r.N = a.N; r.H = a.H; r.W = a.W; r.use_running = a.use_running;
  const size_t items = (size_t)a.N * a.H * a.W * (a.C / 8);
  if (items >= 256 * 4096) launch_fwd_res<4>(a, r, items, st);
  else launch_fwd_res<1>(a, r, items, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_bn_act_fwd(const BnArgs* args, hipStream_t st) {
  BnArgs a = *args;
  a.rcoef = nullptr;  // (the shortcut-BN variant is ddp_bn_act_fwd_res)
  if (a.C % 8 || a.coef == nullptr) return -1;
  if (a.pool && (a.res || a.mask)) return -1;  // residual add / mask only without pooling
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t items = (size_t)a.N * Ho * Wo * (a.C / 8);
  // 1 item per thread for small layers; 2 (pooled) / 4 (plain) when there are enough to keep
  // every CU busy with several resident blocks
  if (a.pool) {
    if (items >= 256 * 2048) launch_fwd<true, 2>(a, items, st);
    else launch_fwd<true, 1>(a, items, st);
  } else {
    if (items >= 256 * 4096) launch_fwd<false, 4>(a, items, st);
    else launch_fwd<false, 1>(a, items, st);
  }
  return (int)hipGetLastError();
}

// Target reduce-grid size (measured).
static size_t kBwdBlocks = 1024;

// Largest grid-wide replica re-read of a folded backward apply (default
// 32 MB; 0 = always the separate finalize launch; ddp_bn_fold_bwd_mb for A/B studies)
static size_t g_fold_bwd_mb = 32;
static size_t fold_bwd_bytes() { return g_fold_bwd_mb << 20; }
extern "C" void ddp_bn_fold_bwd_mb(int mb) { g_fold_bwd_mb = (size_t)(mb < 0 ? 0 : mb); }

// Reduce-grid cap (kReduceGrid, 0 = uncapped): the reduce walks its item blocks
// with a grid stride, so every block adds ONE partial sum per channel. Uncapped, ResNet-50's
// 56x56x256 layers ran 25088 blocks = 51 MB of memory-side float atomics per layer (~40 us at
// the ~1.3 TB/s atomic rate, MI355X_MICROARCH.md "Global float atomics").
static unsigned kReduceGrid = 2048;

// Channel groups per reduce block (kReduceGb, 32 = 256 channels): every
// block adds one partial sum per channel of its chunk, so a block spanning all of a wide
// layer's channels (the apply's layout: 2048 channels x 1 pixel row) made the capped grid
// issue 2048 x 2 x C memory-side atomics — 33 MB at C = 2048, more time than the layer's
// loads (ResNet-50 layer4: reduce 51 us vs apply 27 us over the same tensors). Narrower chunks
// reduce 256 / Gb pixel rows in LDS first.
static int kReduceGb = 32;
static void reduce_split(const BnArgs& a, int Gb, int chunks, int* rGb, int* rchunks) {
  const int G = a.C / 8;
  *rGb = Gb;
  *rchunks = chunks;
  if (kReduceGb > 0 && Gb > kReduceGb && 256 % kReduceGb == 0 && G % kReduceGb == 0) {
    *rGb = kReduceGb;
    *rchunks = G / kReduceGb;
  }
}

// reduce blocks along x for bx item blocks x chunks channel chunks
static unsigned reduce_grid_x(unsigned bx, int chunks) {
  // (the deterministic build keeps one replica per block: block ids stay below kStatRep)
  unsigned rx = kReduceGrid ? std::min(bx, std::max(1u, kReduceGrid / (unsigned)chunks)) : bx;
  if (kDeterministic) rx = std::min(rx, std::max(1u, (unsigned)kStatRep / (unsigned)chunks));
  return rx;
}

// residual block + projection shortcut BN: reduce (3 sums), dual finalize, apply (dz and rdz)
template <int IPT>
static void launch_bwd_res(const BnArgs& a, size_t npix, int Gb, int chunks, hipStream_t st) {
  const unsigned bx = blocks_for(npix, (size_t)(256 / Gb) * IPT);
  BnArgs ra = a;
  int rGb, rch;
  reduce_split(a, Gb, chunks, &rGb, &rch);
  ra.red_gb = rGb;
  const unsigned rbx = blocks_for(npix, (size_t)(256 / rGb) * IPT);
  const unsigned rx = reduce_grid_x(rbx, rch);
  if (rx < rbx)
    hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<false, IPT, true, true, true>), dim3(rx, rch),
                       dim3(256), 0, st, ra);
  else
    hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<false, IPT, true, false, true>), dim3(rbx, rch),
                       dim3(256), 0, st, ra);
  hipLaunchKernelGGL(bn_finalize_bwd_res_kernel, dim3(blocks_for(a.C, 256)), dim3(256), 0, st, a);
  hipLaunchKernelGGL((bn_act_bwd_apply_kernel<false, IPT, false, true, false, true>),
                     dim3(bx, chunks), dim3(256), 0, st, a);
}

template <bool POOL, int IPT, bool MASK>
static void launch_bwd_m(const BnArgs& a, size_t npix, int Gb, int chunks, hipStream_t st) {
  const unsigned bx = blocks_for(npix, (size_t)(256 / Gb) * IPT);
  if (!a.sums_ready) {  // (else: accumulated by the next layer's dgrad epilogue, BnBwdFuse)
    BnArgs ra = a;
    int rGb, rch;
    reduce_split(a, Gb, chunks, &rGb, &rch);
    ra.red_gb = rGb;
    const unsigned rbx = blocks_for(npix, (size_t)(256 / rGb) * IPT);
    const unsigned rx = reduce_grid_x(rbx, rch);
    if (rx < rbx)
      hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<POOL, IPT, MASK, true>), dim3(rx, rch),
                         dim3(256), 0, st, ra);
    else
      hipLaunchKernelGGL((bn_act_bwd_reduce_kernel<POOL, IPT, MASK, false>), dim3(rbx, rch),
                         dim3(256), 0, st, ra);
  }
  // The finalize stays its own launch: folding it into the apply (every block re-reducing the 16
  // replicas the reduce just wrote with memory-side atomics) measured 3-4x slower applies at
  // batch 256 and +50 us per b32 step; the reduce's last-arriving block doing it measured slower
  // than the launch boundary too (profiles/r2_launch_reduction_ab.md, r3_bn_bwd_one_launch.md).
  // finalize folded into the apply while the grid's replica re-reads stay small (every block
  // reads 16 x 2 x its chunk's channels; L2-served after the first XCD miss)
  // — or, for bigger grids, on a capped grid that walks the item blocks (kFoldGrid blocks in all)
  const size_t per_block = (size_t)kStatRep * 2 * (size_t)Gb * 8 * sizeof(float);
  const size_t fold_bytes = (size_t)bx * chunks * per_block;
  if (!kDeterministic && fold_bwd_bytes() > 0 && fold_bytes <= fold_bwd_bytes()) {
    hipLaunchKernelGGL((bn_act_bwd_apply_kernel<POOL, IPT, true, MASK, false>), dim3(bx, chunks),
                       dim3(256), 0, st, a);
    return;
  }
  const unsigned cx = std::min(bx, fold_fwd_grid() / (unsigned)chunks);
  if (!kDeterministic && fold_bwd_bytes() > 0 && cx * chunks >= 1024 &&
      (size_t)cx * chunks * per_block <= kFoldGridBytes) {
    hipLaunchKernelGGL((bn_act_bwd_apply_kernel<POOL, IPT, true, MASK, true>), dim3(cx, chunks),
                       dim3(256), 0, st, a);
    return;
  }
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3(blocks_for(a.C, 256)), dim3(256), 0, st, a);
  hipLaunchKernelGGL((bn_act_bwd_apply_kernel<POOL, IPT, false, MASK, false>), dim3(bx, chunks),
                     dim3(256), 0, st, a);
}

template <bool POOL, int IPT>
static void launch_bwd(const BnArgs& a, size_t npix, int Gb, int chunks, hipStream_t st) {
  if constexpr (!POOL) {
    if (a.rcoef) return launch_bwd_res<IPT>(a, npix, Gb, chunks, st);
    if (a.mask) return launch_bwd_m<POOL, IPT, true>(a, npix, Gb, chunks, st);
  }
  launch_bwd_m<POOL, IPT, false>(a, npix, Gb, chunks, st);
}

// One-block-per-channel-group backward (bn_act_bwd_local_kernel): items per thread for npix
// (post-pool) pixels; false when the layer is too big for it. A block streams its 8-channel
// column alone — every 16-byte load is its own cache line — so its time grows with the loads
// per thread (measured, b64 step: 2 loads 5.1 us, 5 loads 9.6, 8 loads 9.5, 16-20 loads 22 us,
// against 12-19 us for reduce + finalize + apply): served while ipt x (dy + z [+ res] vectors)
// <= kLocalMaxLoads (0 = never; bn_bwd_local_set). Step A/B of the limit (0/5/8/10):
// 8 is best at b32..b128 (b32 0.416 -> 0.405 ms, b64 -1.2 %, b128 -0.9 %), neutral at b256.
// (1024-thread blocks for the next-bigger layers and a clustered grid-synchronised variant were
// measured slower and removed in round 4: profiles/r3_conv_occupancy.md, r3_bn_bwd_one_launch.md)
static int kLocalMaxLoads = 8;
constexpr int kLocalThreads = 256;
static bool local_cfg(const BnArgs& a, int* ipt) {
  if (a.C % 8 || (a.pool && a.res)) return false;
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  const int per_item = 1 + (a.pool ? 4 : 1) + (a.res ? 1 : 0);
  for (int i = 1; i <= 8; i *= 2) {
    if ((size_t)kLocalThreads * i < npix) continue;
    if (a.pool && i > 4) return false;  // register budget: 4 pre-pool vectors per item
    if (i * per_item > kLocalMaxLoads) return false;
    *ipt = i;
    return true;
  }
  return false;
}

template <bool POOL, bool MASK>
static void launch_local_m(const BnArgs& a, int ipt, hipStream_t st) {
  const dim3 grid(a.C / 8), block(kLocalThreads);
  if (ipt == 1) hipLaunchKernelGGL((bn_act_bwd_local_kernel<POOL, 1, kLocalThreads, MASK>), grid, block, 0, st, a);
  else if (ipt == 2) hipLaunchKernelGGL((bn_act_bwd_local_kernel<POOL, 2, kLocalThreads, MASK>), grid, block, 0, st, a);
  else if (ipt == 4) hipLaunchKernelGGL((bn_act_bwd_local_kernel<POOL, 4, kLocalThreads, MASK>), grid, block, 0, st, a);
  else if constexpr (!POOL) hipLaunchKernelGGL((bn_act_bwd_local_kernel<POOL, 8, kLocalThreads, MASK>), grid, block, 0, st, a);
}

template <bool POOL>
static void launch_local(const BnArgs& a, int ipt, hipStream_t st) {
  if constexpr (!POOL) {
    if (a.mask) return launch_local_m<POOL, true>(a, ipt, st);
  }
  launch_local_m<POOL, false>(a, ipt, st);
}

// tests / sweeps: the loads-per-thread limit of the one-launch backward (0 = off)
extern "C" void ddp_bn_bwd_local_set(long long max_loads) {
  BnArgs a{};
  int ipt;
  (void)local_cfg(a, &ipt);  // run the env init first so it cannot override this later
  kLocalMaxLoads = (int)std::max(0LL, max_loads);
}

extern "C" int ddp_bn_bwd_local_ok(int N, int H, int W, int C, int pool) {
  BnArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.pool = pool;
  int ipt;
  return local_cfg(a, &ipt) ? 1 : 0;
}

// reduce + finalize + apply
static int launch_reduce_chain(const BnArgs& a, hipStream_t st) {
  const int G = a.C / 8;
  const int Gb = G < 256 ? G : 256;
  if ((Gb < 256 && 256 % Gb) || (G > 256 && G % 256)) return -1;  // channel groups must tile 256 threads
  const int chunks = (G + Gb - 1) / Gb;
  const int Ho = a.pool ? a.H / 2 : a.H, Wo = a.pool ? a.W / 2 : a.W;
  const size_t npix = (size_t)a.N * Ho * Wo;
  // Items per thread: enough to keep the reduce grid near kBwdBlocks blocks. Every reduce block
  // adds one partial sum per channel into one of kStatRep replicas, and memory-side float atomics
  // serialise per address: 2048 one-item blocks (VGG layer 0) put 128 adders on every address.
  const size_t per1 = (size_t)(256 / Gb);  // items per block at one item per thread
  const size_t blocks1 = (npix + per1 - 1) / per1 * chunks;
  // Measured: VGG-11's layers (<= 2048 one-item blocks) are fastest at one item per thread;
  // ResNet-50's 56x56 layers (6272 blocks) gain 0.7 ms/step from 4 items per thread.
  int ipt = 1;
  if (blocks1 > 2 * kBwdBlocks)
    while (ipt < 4 && blocks1 / ipt > kBwdBlocks) ipt *= 2;
  if (a.pool) {
    if (ipt >= 4) launch_bwd<true, 4>(a, npix, Gb, chunks, st);
    else if (ipt == 2) launch_bwd<true, 2>(a, npix, Gb, chunks, st);
    else launch_bwd<true, 1>(a, npix, Gb, chunks, st);
  } else {
    if (ipt >= 4) launch_bwd<false, 4>(a, npix, Gb, chunks, st);
    else if (ipt == 2) launch_bwd<false, 2>(a, npix, Gb, chunks, st);
    else launch_bwd<false, 1>(a, npix, Gb, chunks, st);
  }
  return (int)hipGetLastError();
}

// a.coef must hold the table written by the matching forward; a.sums ([kStatRep][2][C]) must be
// zero on entry (per-step scratch, zeroed once per forward).
extern "C" int ddp_bn_act_bwd_res(const BnArgs* args, hipStream_t st) {
  const BnArgs a = *args;
  if (!res_shape_ok(a) || a.mask == nullptr || a.sums == nullptr || a.rsums == nullptr ||
      a.dz == nullptr || a.rdz == nullptr || a.sums_ready)
    return -1;
  return launch_reduce_chain(a, st);  // (never the one-block local kernel)
}

extern "C" int ddp_bn_act_bwd(const BnArgs* args, hipStream_t st) {
  BnArgs a = *args;
  if (a.C % 8 || a.coef == nullptr || a.sums == nullptr) return -1;
  if (a.pool && (a.res || a.mask)) return -1;
  a.rcoef = nullptr;  // (the shortcut-BN variant is ddp_bn_act_bwd_res)
  int ipt;
  if (local_cfg(a, &ipt)) {
    // small layer: the whole backward in one launch (any sums the next layer's dgrad
    // accumulated are simply not needed)
    if (a.pool) launch_local<true>(a, ipt, st);
    else launch_local<false>(a, ipt, st);
    return (int)hipGetLastError();
  }
  return launch_reduce_chain(a, st);
}

// ResNet stem BN + ReLU + MaxPool2d(3, 2, 1) (bn_pool3_*): a.H x a.W = conv output, a.out /
// a.dout = pooled [N][Ho][Wo][C], idx = the forward's window argmax bytes (pooled shape).
static bool pool3_shape_ok(const BnArgs& a, int* Ho, int* Wo) {
  if (a.C % 8 || 64 % (a.C / 8) || a.coef == nullptr || a.res || a.pool) return false;
  *Ho = (a.H + 2 * kP3P - kP3) / kP3S + 1;
  *Wo = (a.W + 2 * kP3P - kP3) / kP3S + 1;
  return (size_t)a.N * a.H * a.W * a.C < (1ull << 31);
}

// grid caps of the stem passes (fwd, reduce, apply). Kernel-trace sweep on
// ResNet-50 b256 (profiles/r5az_pool3_grids.md): 16384 / 2048 / 4096 take 498 us for the three
// passes against 524 us at the previous 8192 / 4096 / 16384
static void pool3_grids(unsigned* g) {
  static const unsigned v[3] = {16384, 2048, 4096};
  g[0] = std::max(1u, v[0]); g[1] = std::max(1u, v[1]); g[2] = std::max(1u, v[2]);
}

extern "C" int ddp_bn_pool3_fwd(const BnArgs* args, unsigned char* idx, hipStream_t st) {
  const BnArgs a = *args;
  int Ho, Wo;
  if (!pool3_shape_ok(a, &Ho, &Wo) || idx == nullptr) return -1;
  unsigned caps[3];
  pool3_grids(caps);
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(blocks_for(a.C, 256)), dim3(256), 0, st, a);
  const size_t items = (size_t)a.N * Ho * Wo * (a.C / 8);
  const unsigned nb = (unsigned)std::min<size_t>(blocks_for(items, 256), caps[0]);
  hipLaunchKernelGGL(bn_pool3_fwd_kernel, dim3(nb), dim3(256), 0, st, a, Ho, Wo, idx);
  return (int)hipGetLastError();
}

// a.sums must be zero on entry (per-step scratch); dgamma / dbeta are accumulated
extern "C" int ddp_bn_pool3_bwd(const BnArgs* args, const unsigned char* idx, hipStream_t st) {
  const BnArgs a = *args;
  int Ho, Wo;
  if (!pool3_shape_ok(a, &Ho, &Wo) || idx == nullptr || a.sums == nullptr || a.dz == nullptr)
    return -1;
  const size_t nq = (size_t)a.N * Ho * Wo;  // 2x2 pre-pool quads
  const size_t per = 256 / (a.C / 8);
  unsigned caps[3];
  pool3_grids(caps);
  // reduce: ~4 quad iterations per thread (fewer replica atomics); apply: one pass
  const unsigned nr = (unsigned)std::max<size_t>(1, std::min<size_t>(blocks_for(nq, per * 4), caps[1]));
  const unsigned na = (unsigned)std::min<size_t>(blocks_for(nq, per), caps[2]);
  hipLaunchKernelGGL((bn_pool3_bwd_kernel<false>), dim3(nr), dim3(256), 0, st, a, Ho, Wo, idx);
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3(blocks_for(a.C, 256)), dim3(256), 0, st, a);
  hipLaunchKernelGGL((bn_pool3_bwd_kernel<true>), dim3(na), dim3(256), 0, st, a, Ho, Wo, idx);
  return (int)hipGetLastError();
}
