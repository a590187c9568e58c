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
      pp[e] = sgd_update1(pp[e], gg[e], bb[e], lr, momentum, wd, grad_scale, nesterov);
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(buf)[i] = bv;
  }
  // scalar tail
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    p[i] = sgd_update1(p[i], g[i], buf[i], lr, momentum, wd, grad_scale, nesterov);
  }
}

constexpr int kMaxPack = 64;
struct PackTable {
  PackDesc d[kMaxPack];
  int n;
};

__device__ __forceinline__ size_t master_index(const PackDesc& d, int k, int c, int r, int s) {
  return d.krsc ? (((size_t)k * d.R + r) * d.S + s) * d.Cr + c
                : (((size_t)k * d.Cr + c) * d.R + r) * d.S + s;
}

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
      const float v = c < d.Cr ? d.p[master_index(d, k, c, r, s)] : 0.f;
      d.wc[i] = f2bf(v);
    }
    if (d.wt) {  // i indexes Wt [c][r][s][k]
      const int k = (int)(i % d.K);
      const size_t t1 = i / d.K;
      const int s = (int)(t1 % d.S);
      const size_t t2 = t1 / d.S;
      const int r = (int)(t2 % d.R);
      const int c = (int)(t2 / d.R);
      const float v = c < d.Cr ? d.p[master_index(d, k, c, r, s)] : 0.f;
      d.wt[i] = f2bf(v);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused SGD + weight re-pack: ONE launch updates the whole arena and writes the bf16 MFMA
// operand copies of every conv weight from the freshly updated values (no second pass over the
// fp32 weights). Work items (int4): {0, offset, count, -} = plain elementwise chunk;
// {2, rel_offset, count, desc} = elementwise chunk of a conv weight stored [K][R][S][C] (the GPU
// arena layout): its bf16 copy Wc has the same index order, so it is written in the same pass;
// {1, desc, k0, c0} = one TK x TC x (R*S) tile of a conv weight that needs a layout change
// (channel-padded input layer, or a [K][C][R][S] master), staged through LDS so that the Wc
// ([k][r][s][c], c fastest) and optional Wt ([c][r][s][k], k fastest) writes are coalesced.
// Conv descriptor (int64 x 12): {p_offset, K, Cr, C, R, S, wc_ptr, wt_ptr, krsc, -, -, -};
// krsc selects the fp32 master layout ([K][R][S][Cr] vs [K][Cr][R][S]).
constexpr int kTileElems = 9216;  // fp32 LDS tile (36 KB)

__device__ __forceinline__ void tile_dims(int RS, int* TK, int* TC) {
  if (RS == 1) { *TK = 64; *TC = 64; }
  else if (RS <= 9) { *TK = 32; *TC = 32; }
  else { *TK = 8; *TC = 16; }
}

struct SgdHyper {
  float lr, momentum, wd, grad_scale;
  int nesterov;
  int zero_grad;  // write 0 to every gradient after use (replaces the next step's zero_grad fill)
  int* counter;   // optional step counter (data cursor): += delta by one thread
  int delta;
  // optional error word (engine/step.py SegmentedDDPStep): non-zero when a device-side wait for
  // a gradient bucket timed out — the update is then skipped instead of applying gradients
  // that were never averaged (the host raises on the error at its next check)
  const unsigned* skip;
  // sharded update with a bf16 operand all-gather (parallel/zero.py ShardedBf16Update): item 3
  // also stores bf16(new p) into ``shadow`` (the bf16 operand image of the arena, same element
  // index) and, for the small fp32-wire tensors, the new p into ``slot`` (the all-gather send slot)
  unsigned short* shadow;
  float* slot;
  // optional completion signal (engine/step.py SegmentedDDPStep, last bucket): the last block
  // to finish (``done`` ticket, reset by it) release-increments ``signal`` — the step's
  // "every parameter updated" flag without a separate signal launch
  unsigned* done;
  unsigned* signal;
};

// Last-block-done hand-off: every block's writes are fenced, the block that takes the last
// ticket resets the ticket and release-increments the flag (acquired by flag_wait_kernel).
// The step's error word (SegmentedDDPStep: a device-side wait timed out), read ONCE per block:
// every thread of the block takes the same branch, so no thread can leave while others still
// wait at a barrier of a tile item or of last_block_done (the word may flip during the launch).
__device__ __forceinline__ bool block_skip(const unsigned* skip) {
  if (!skip) return false;  // (a kernel argument: uniform)
  __shared__ unsigned s_skip;
  if (threadIdx.x == 0) s_skip = __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return s_skip != 0u;
}

__device__ __forceinline__ bool last_block_done(unsigned* done) {
  __syncthreads();
  __shared__ unsigned last;
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned t = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == gridDim.x - 1) ? 1u : 0u;
  }
  __syncthreads();
  return last != 0u;
}

__device__ __forceinline__ void signal_flag(unsigned* done, unsigned* signal) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(signal, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ float sgd1(float p, float g, float& b, const SgdHyper& h) {
  return sgd_update1(p, g, b, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
}

__device__ void sgd_pack_body(const int4* __restrict__ items, const long long* __restrict__ descs,
                              float* __restrict__ p, float* __restrict__ g,
                              float* __restrict__ buf, const SgdHyper& h, float* tile);

__global__ __launch_bounds__(256) void sgd_pack_kernel(const int4* __restrict__ items,
                                                       const long long* __restrict__ descs,
                                                       float* __restrict__ p,
                                                       float* __restrict__ g,
                                                       float* __restrict__ buf, SgdHyper h) {
  __shared__ float tile[kTileElems];
  sgd_pack_body(items, descs, p, g, buf, h, tile);
  if (h.signal && last_block_done(h.done)) signal_flag(h.done, h.signal);
}

__device__ void sgd_pack_body(const int4* __restrict__ items, const long long* __restrict__ descs,
                              float* __restrict__ p, float* __restrict__ g,
                              float* __restrict__ buf, const SgdHyper& h, float* tile) {
  const int4 it = items[blockIdx.x];
  const int tid = threadIdx.x;
  if (h.counter && blockIdx.x == 0 && tid == 0) atomicAdd(h.counter, h.delta);
  if (block_skip(h.skip)) return;
  if (it.x == 0) {
    const size_t off = (size_t)(unsigned)it.y;
    const int cnt = it.z;
    for (int i = tid * 4; i < cnt; i += 256 * 4) {
      if (i + 4 <= cnt && ((off + i) & 3) == 0) {
        float4 pv = *reinterpret_cast<float4*>(p + off + i);
        const float4 gv = *reinterpret_cast<const float4*>(g + off + i);
        float4 bv = *reinterpret_cast<float4*>(buf + off + i);
        pv.x = sgd1(pv.x, gv.x, bv.x, h);
        pv.y = sgd1(pv.y, gv.y, bv.y, h);
        pv.z = sgd1(pv.z, gv.z, bv.z, h);
        pv.w = sgd1(pv.w, gv.w, bv.w, h);
        *reinterpret_cast<float4*>(p + off + i) = pv;
        *reinterpret_cast<float4*>(buf + off + i) = bv;
        if (h.zero_grad) *reinterpret_cast<float4*>(g + off + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      } else {
        for (int e = i; e < min(cnt, i + 4); ++e) {
          float b = buf[off + e];
          p[off + e] = sgd1(p[off + e], g[off + e], b, h);
          buf[off + e] = b;
          if (h.zero_grad) g[off + e] = 0.f;
        }
      }
    }
    return;
  }
  if (it.x == 3) {
    // {3, offset, count, slot_offset | -1}: this rank's shard of a sharded bucket — SGD on the
    // fp32 master + momentum, bf16 operand image of the new values, fp32 send slot of the
    // small tensors (offset, count and slot_offset multiples of 4: 64-aligned tensors, shards
    // of n/w with n % 64 == 0 and w | 8)
    const size_t off = (size_t)(unsigned)it.y;
    const int cnt = it.z;
    float* slot = it.w >= 0 && h.slot ? h.slot + it.w : nullptr;
    for (int i = tid * 4; i < cnt; i += 256 * 4) {
      float4 pv = *reinterpret_cast<float4*>(p + off + i);
      const float4 gv = *reinterpret_cast<const float4*>(g + off + i);
      float4 bv = *reinterpret_cast<float4*>(buf + off + i);
      pv.x = sgd1(pv.x, gv.x, bv.x, h);
      pv.y = sgd1(pv.y, gv.y, bv.y, h);
      pv.z = sgd1(pv.z, gv.z, bv.z, h);
      pv.w = sgd1(pv.w, gv.w, bv.w, h);
      *reinterpret_cast<float4*>(p + off + i) = pv;
      *reinterpret_cast<float4*>(buf + off + i) = bv;
      if (h.zero_grad) *reinterpret_cast<float4*>(g + off + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      if (h.shadow) {
        uint2 pk;
        pk.x = (unsigned)f2bf(pv.x) | ((unsigned)f2bf(pv.y) << 16);
        pk.y = (unsigned)f2bf(pv.z) | ((unsigned)f2bf(pv.w) << 16);
        *reinterpret_cast<uint2*>(h.shadow + off + i) = pk;
      }
      if (slot) *reinterpret_cast<float4*>(slot + i) = pv;
    }
    return;
  }
  if (it.x == 4) {
    // {4, offset, count, -}: clear gradients outside this rank's shard (count multiple of 4)
    const size_t off = (size_t)(unsigned)it.y;
    for (int i = tid * 4; i < it.z; i += 256 * 4)
      *reinterpret_cast<float4*>(g + off + i) = make_float4(0.f, 0.f, 0.f, 0.f);
    return;
  }
  if (it.x == 5) {
    // {5, offset in the tensor, count, desc}: operand re-pack only — the fp32 master was already
    // updated by the backward (conv_igemm.hip ConvArgs::sgd); bf16(p) into the operand copy
    // (same index order as item 2; count multiple of 4)
    const long long* d = descs + 12 * it.w;
    const size_t base = (size_t)d[0] + (unsigned)it.y;
    unsigned short* wc = reinterpret_cast<unsigned short*>(d[6]) + (unsigned)it.y;
    for (int i = tid * 4; i < it.z; i += 256 * 4) {
      const float4 pv = *reinterpret_cast<const float4*>(p + base + i);
      uint2 pk;
      pk.x = (unsigned)f2bf(pv.x) | ((unsigned)f2bf(pv.y) << 16);
      pk.y = (unsigned)f2bf(pv.z) | ((unsigned)f2bf(pv.w) << 16);
      *reinterpret_cast<uint2*>(wc + i) = pk;
    }
    return;
  }
  if (it.x == 2) {
    // conv weight whose bf16 operand copy has the master's own index order ([K][R][S][C] with
    // C == Cr, or 1x1): elementwise update + bf16 store, no LDS staging
    const long long* d = descs + 12 * it.w;
    const size_t base = (size_t)d[0] + (unsigned)it.y;
    unsigned short* wc = reinterpret_cast<unsigned short*>(d[6]) + (unsigned)it.y;
    const int cnt = it.z;  // multiple of 4, base 4-aligned (arena tensors are 64-aligned)
    for (int i = tid * 4; i < cnt; i += 256 * 4) {
      float4 pv = *reinterpret_cast<float4*>(p + base + i);
      const float4 gv = *reinterpret_cast<const float4*>(g + base + i);
      float4 bv = *reinterpret_cast<float4*>(buf + base + i);
      pv.x = sgd1(pv.x, gv.x, bv.x, h);
      pv.y = sgd1(pv.y, gv.y, bv.y, h);
      pv.z = sgd1(pv.z, gv.z, bv.z, h);
      pv.w = sgd1(pv.w, gv.w, bv.w, h);
      *reinterpret_cast<float4*>(p + base + i) = pv;
      *reinterpret_cast<float4*>(buf + base + i) = bv;
      if (h.zero_grad) *reinterpret_cast<float4*>(g + base + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      uint2 pk;
      pk.x = (unsigned)f2bf(pv.x) | ((unsigned)f2bf(pv.y) << 16);
      pk.y = (unsigned)f2bf(pv.z) | ((unsigned)f2bf(pv.w) << 16);
      *reinterpret_cast<uint2*>(wc + i) = pk;
    }
    return;
  }
  const long long* d = descs + 12 * it.y;
  const size_t poff = (size_t)d[0];
  const int K = (int)d[1], Cr = (int)d[2], C = (int)d[3], R = (int)d[4], S = (int)d[5];
  unsigned short* wc = reinterpret_cast<unsigned short*>(d[6]);
  unsigned short* wt = reinterpret_cast<unsigned short*>(d[7]);
  const int RS = R * S;
  int TK, TC;
  tile_dims(RS, &TK, &TC);
  const int k0 = it.z, c0 = it.w;
  const int tk = min(TK, K - k0);
  const int tcr = max(0, min(TC, Cr - c0));  // real channels in this tile
  const int tcp = min(TC, C - c0);           // padded channels in this tile (Wc width)
  const bool krsc = d[8] != 0;
  if (!krsc) {
    // 1) SGD on p[k][c][r][s] for the tile's real channels; runs of tcr*RS contiguous floats
    const int run = tcr * RS;
    for (int idx = tid; idx < tk * run; idx += 256) {
      const int kl = idx / run, e = idx - kl * run;
      const size_t gi = poff + (size_t)(k0 + kl) * Cr * RS + (size_t)c0 * RS + e;
      float b = buf[gi];
      const float np = sgd1(p[gi], g[gi], b, h);
      p[gi] = np;
      buf[gi] = b;
      if (h.zero_grad) g[gi] = 0.f;
      tile[kl * TC * RS + e] = np;  // tile layout [kl][cl][rs]
    }
  } else {
    // 1) SGD on p[k][r][s][c]: runs of tcr contiguous channels per (k, r, s)
    for (int idx = tid; idx < tk * RS * tcr; idx += 256) {
      const int cl = idx % tcr, t = idx / tcr;
      const int rs = t % RS, kl = t / RS;
      const size_t gi = poff + ((size_t)(k0 + kl) * RS + rs) * Cr + c0 + cl;
      float b = buf[gi];
      const float np = sgd1(p[gi], g[gi], b, h);
      p[gi] = np;
      buf[gi] = b;
      if (h.zero_grad) g[gi] = 0.f;
      tile[kl * TC * RS + cl * RS + rs] = np;
    }
  }
  __syncthreads();
  // 2) Wc[k][r][s][c] (c fastest, zero for padded channels)
  if (wc) {
    for (int idx = tid; idx < tk * RS * tcp; idx += 256) {
      const int cl = idx % tcp, t = idx / tcp;
      const int rs = t % RS, kl = t / RS;
      const float v = cl < tcr ? tile[(kl * TC + cl) * RS + rs] : 0.f;
      wc[((size_t)(k0 + kl) * RS + rs) * C + c0 + cl] = f2bf(v);
    }
  }
  // 3) Wt[c][r][s][k] (k fastest)
  if (wt) {
    for (int idx = tid; idx < tcr * RS * tk; idx += 256) {
      const int kl = idx % tk, t = idx / tk;
      const int rs = t % RS, cl = t / RS;
      wt[((size_t)(c0 + cl) * RS + rs) * K + k0 + kl] = f2bf(tile[(kl * TC + cl) * RS + rs]);
    }
  }
}

// Tail of a pipelined step with sharded buckets (parallel/zero.py ShardedBf16Update.tail): one
// block per segment copies gathered small-tensor values (fp32 send slots of every rank) into
// the fp32 parameter arena; the last block to finish re-packs the bf16 operand copies of the
// channel-padded conv weights among them (their masters are complete only now) and signals
// the step's "every parameter updated" flag. Segment entries: int4 {src, dst, count, -}.
constexpr int kMaxTailPack = 4;
struct TailArgs {
  const int4* segs;
  int n_segs;
  const float* src;
  float* dst;
  PackDesc pack[kMaxTailPack];
  int n_pack;
  unsigned* done;
  unsigned* signal;
  const unsigned* skip;
};

__global__ __launch_bounds__(256) void shard_tail_kernel(TailArgs a) {
  const bool skipped = block_skip(a.skip);
  if (!skipped && (int)blockIdx.x < a.n_segs) {
    const int4 e = a.segs[blockIdx.x];
    const float* s = a.src + (size_t)(unsigned)e.x;
    float* d = a.dst + (size_t)(unsigned)e.y;
    for (int i = threadIdx.x; i < e.z; i += 256) d[i] = s[i];
  }
  if (!last_block_done(a.done)) return;
  __threadfence();  // acquire side: the other blocks' copies are visible to this block
  if (!skipped) {
    for (int q = 0; q < a.n_pack; ++q) {
      const PackDesc& d = a.pack[q];
      const int rs = d.R * d.S;
      const int total = d.K * rs * d.C;
      for (int i = threadIdx.x; i < total; i += 256) {  // Wc [k][r][s][c], zero padded c
        const int c = i % d.C, t1 = i / d.C;
        const int sx = t1 % d.S, t2 = t1 / d.S;
        const int r = t2 % d.R, k = t2 / d.R;
        const float v = c < d.Cr ? d.p[master_index(d, k, c, r, sx)] : 0.f;
        d.wc[i] = f2bf(v);
      }
    }
    __syncthreads();
    __threadfence();
  }
  if (a.signal) signal_flag(a.done, a.signal);
  else if (threadIdx.x == 0) __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

extern "C" int ddp_sgd_pack(const void* items, int n_items, const long long* descs, float* p,
                            float* g, float* buf, float lr, float momentum, float wd,
                            float grad_scale, int nesterov, int zero_grad, int* counter,
                            int delta, const unsigned* skip, unsigned short* shadow, float* slot,
                            unsigned* done, unsigned* signal, hipStream_t st) {
  SgdHyper h{lr, momentum, wd, grad_scale, nesterov, zero_grad, counter, delta, skip, shadow, slot,
             done, signal};
  if (n_items <= 0) return 0;
  hipLaunchKernelGGL(sgd_pack_kernel, dim3(n_items), dim3(256), 0, st, (const int4*)items, descs,
                     p, g, buf, h);
  return (int)hipGetLastError();
}

extern "C" int ddp_shard_tail(const void* segs, int n_segs, const float* src, float* dst,
                              const PackDesc* pack, int n_pack, unsigned* done, unsigned* signal,
                              const unsigned* skip, hipStream_t st) {
  if (n_pack > kMaxTailPack || !done) return -1;
  TailArgs a{};
  a.segs = (const int4*)segs; a.n_segs = n_segs; a.src = src; a.dst = dst;
  for (int i = 0; i < n_pack; ++i) a.pack[i] = pack[i];
  a.n_pack = n_pack; a.done = done; a.signal = signal; a.skip = skip;
  hipLaunchKernelGGL(shard_tail_kernel, dim3(n_segs > 0 ? n_segs : 1), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// Host-side tile shape (must match tile_dims above) so Python can build the item table.
extern "C" void ddp_sgd_tile_dims(int RS, int* TK, int* TC) {
  if (RS == 1) { *TK = 64; *TC = 64; }
  else if (RS <= 9) { *TK = 32; *TC = 32; }
  else { *TK = 8; *TC = 16; }
}

extern "C" int ddp_counter_add(int* c, int delta, hipStream_t st) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, st, c, delta);
  return (int)hipGetLastError();
}
