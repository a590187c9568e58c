// Tap-reuse 3x3 convolution forward for gfx950: the input tile stays resident in LDS for all
// nine taps (bf16 MFMA v_mfma_f32_16x16x32_bf16, fp32 accumulation).
//
// Reference parity: the Conv2d(3x3, stride 1, pad 1, bias) of every VGG block after the first
// (part1/model.py:18-23; SURVEY.md §2.D shapes 64->128 ... 512->512 at 16x16 .. 2x2).
//
// Why a second forward kernel: the implicit-GEMM kernel (conv_igemm.hip) gathers the A operand
// per k-step = (tap, 64 channels), so every input pixel crosses L2 -> LDS nine times per output
// column tile (VGG-11 b256 256->256 8x8: 302 MB of A traffic for an 8.4 MB input) and each
// k-step pays its own A DMA instructions. Here a block owns BM output pixels that are whole image
// rows (or whole images), loads the input patch they need — the rows plus a one-pixel halo — ONCE
// per 64-channel block into LDS, and runs the nine taps as nine shifted reads of that patch: A
// traffic drops to ~1.3-4x the input (halo overhead) and only the weights stream per tap.
//
// LDS patch image (one per 64-channel block, double-buffered): 8 chunk planes (8 channels =
// 16 B each) of `plane` pixels; plane c starts at pixel c * plane + 4 * (c >> 1). A fragment read
// (ds_read_b128; lane l reads output row l & 15 at chunk plane l >> 4, so the four hardware lane
// groups each mix two adjacent planes) then hits 16 distinct bank quads whenever the 16 rows are
// 16 consecutive patch pixels — true for W >= 4 (rows of 16, 8 or 4 pixels are contiguous in the
// patch); for W = 2 the per-image pitch `imgp` is chosen by the host so that four 2x2 images
// land on distinct quads. The halo COLUMNS are not stored: for the s = 0 / 2 tap an edge lane
// reads its own centre pixel (an address a neighbour lane reads anyway: no extra bank traffic)
// and zeroes the fragment; halo ROWS are loaded (zeros at the image border).
// The patch is loaded through registers (buffer_load_dwordx4, eight lanes per pixel = one
// coalesced 128-B pixel row; out-of-range offsets read zero) and written to the planes by
// ds_write_b128 (2-way bank conflicts); the weights stream by LDS-DMA (buffer_load ... lds).
//
// Loop: k-step j = (channel block cb, tap t), cb-major. B (weights [K][3][3][C], [col][k] tiles,
// XOR-swizzled as in conv_igemm.hip) streams through an NST-deep ring; the patch of cb+1 is
// loaded into registers at k-step (cb, 0) and written to the other patch buffer after k-step
// (cb, 8), so its latency hides behind the current patch's nine taps. Split-K over channel blocks
// writes fp32 slabs [split][M][K] reduced by conv_igemm.hip's finish kernels (including the
// BatchNorm-fused finish of the small strong-scaling layers).
// Epilogue: bias, bf16 z, per-channel BatchNorm statistics of the rounded output (as
// conv_igemm.hip).
#include "common.h"
#include "api.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <tuple>

namespace ddp_amd {
namespace tr {

typedef __attribute__((address_space(3))) void lds_void;

constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

// buffer_load_dwordx4 ... lds: LDS destination = wave-uniform base (M0) + lane * 16
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t rs, unsigned byte_off, unsigned short* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds, 16, (int)byte_off, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// wait for k-step j's B stage given how many B stages (NB = bafter) and whether the next patch's
// loads (NLn instructions) were issued after it; NB is a runtime value in [0, NBMAX]
template <int NBMAX, int CBn, int NLn>
__device__ __forceinline__ void wait_stage(int bafter, bool anext) {
  if constexpr (NBMAX > 0) {
    if (bafter >= NBMAX) {
      if (anext) wait_dma_barrier<NBMAX * CBn + NLn>();
      else wait_dma_barrier<NBMAX * CBn>();
      return;
    }
    wait_stage<NBMAX - 1, CBn, NLn>(bafter, anext);
  } else {
    wait_dma_barrier<0>();
  }
}

// [col][k] weight tile, 64 bf16 per row, 16-B chunk XOR (row >> 1) & 7 (conv_igemm.hip rk_off)
__device__ __forceinline__ int rk_off(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3);
}

__host__ __device__ __forceinline__ int plane_base(int c, int plane) { return c * plane + 4 * (c >> 1); }

struct Args {
  int N, H, W, C, K;
  const unsigned short* x;   // [N][H][W][C]
  const unsigned short* wc;  // [K][3][3][C]
  const float* bias;
  unsigned short* z;         // [N][H][W][K]
  float* stats;              // [kStatRep][2][K] (may be null)
  float* ws;                 // split-K slabs [splits][M][K]
  int splits, cbps;          // split-K factor, channel blocks per split
  int imgs, rows, bands;     // images per tile, output rows per image in a tile, tiles per image
  int imgp, plane, zslot;    // patch pitch per image, pixels per chunk plane, zero pixel
  int x_bytes, w_bytes;
  int tiles_m, tiles_n;
  int abuf_elems;            // bf16 elements of one patch buffer (16-B multiple)
  // fused input (template IN = 1: BN + ReLU, IN = 2: BN + ReLU + 2x2/s2 max-pool): the conv
  // input x = [pool](relu(scale * zin + shift)) is computed while the patch is loaded; zin is
  // the preceding block's conv output [N][Hz][Wz][C] (Hz = 2H when pooled), its BatchNorm
  // coefficients are folded here from the statistics replicas, block 0 writes the coefficient
  // table the preceding block's backward reads, and the first column tile's blocks materialise
  // x into y_out (the wgrad's operand)
  const unsigned short* zin;
  const float* in_stats;     // [kStatRep][2][C]
  const float* in_gamma;
  const float* in_beta;
  float in_eps;
  int in_relu;
  float* in_coef;            // [6][C]: scale, shift, mean, invstd (written by block 0)
  unsigned short* y_out;     // [N][H][W][C]
  int z_bytes;
};

template <int BM, int BN, int NST, int NL, int IN>
#ifndef DDP_TR_WAVES_PER_EU
#define DDP_TR_WAVES_PER_EU 1  // (A/B knob: -DDDP_TR_WAVES_PER_EU=3 asks for 3 waves per SIMD)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DDP_TR_WAVES_PER_EU)))
void conv_tr_fwd_kernel(Args a) {
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  constexpr int CB = BN * 64 / 8 / 256;  // B DMA instructions per thread per k-step
  constexpr int BTILE = BN * 64;         // bf16 elements per B stage
  static_assert(CB >= 1 && TM >= 1 && TN >= 1, "tile");
  static_assert(NST >= 3 && NST <= 9, "the next patch is issued at tap 0: at most one in the window");
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  const int aelems = a.abuf_elems;                      // one patch buffer (bf16 elements)
  unsigned short* abuf = smem;                          // 2 patch buffers
  unsigned short* bring = smem + 2 * aelems;            // NST x BTILE
  float* cf = reinterpret_cast<float*>(bring + NST * BTILE);  // IN: [2][C] scale | shift
  constexpr int NP = IN == 2 ? 4 : 1;                   // source loads per patch item
  constexpr bool BNIN = IN == 1 || IN == 2;             // BN + ReLU (+ pool) input

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int W = a.W, H = a.H, C = a.C, K = a.K;
  const int M = a.N * H * W;
  const int ncb = C / 64;

  const int tiles = a.tiles_m * a.tiles_n;
  const int item = blockIdx.x;
  const int sp = item / tiles;
  const int tile = xcd_remap(item - sp * tiles, tiles);
  const int tm = tile / a.tiles_n;  // column tiles fastest (as conv_igemm.hip)
  const int tn = tile - tm * a.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int cb0 = sp * a.cbps, cb1 = min(ncb, cb0 + a.cbps);
  const int nsteps = (cb1 - cb0) * 9;
  // tile -> images / band
  const int n0 = (tm / a.bands) * a.imgs;
  const int h0 = (tm % a.bands) * a.rows;  // first output row of the band

  const __amdgpu_buffer_rsrc_t rsA = IN ? make_rsrc(a.zin, a.z_bytes) : make_rsrc(a.x, a.x_bytes);
  if (BNIN) {
    // BatchNorm finalize of the input channels (batch statistics of zin over N*Hz*Wz), as
    // bn_act.hip fold_fwd_coeffs: every block reduces the replicas into LDS; block 0 also
    // writes the coefficient table for the backward
    const int Hz = IN == 2 ? 2 * H : H, Wz = IN == 2 ? 2 * W : W;
    const float Mz = (float)a.N * Hz * Wz;
    for (int c = tid; c < C; c += 256) {
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int r = 0; r < kStatRep; ++r) {
        s1 += a.in_stats[r * 2 * C + c];
        s2 += a.in_stats[r * 2 * C + C + c];
      }
      const float mu = s1 / Mz;
      const float var = fmaxf(s2 / Mz - mu * mu, 0.f);
      const float is = rsqrtf(var + a.in_eps);
      const float sc = a.in_gamma[c] * is, sh = a.in_beta[c] - mu * sc;
      cf[c] = sc;
      cf[C + c] = sh;
      if (blockIdx.x == 0) {
        a.in_coef[0 * C + c] = sc;
        a.in_coef[1 * C + c] = sh;
        a.in_coef[2 * C + c] = mu;
        a.in_coef[3 * C + c] = is;
      }
    }
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(a.wc, a.w_bytes);

  // ---- A patch loads: item u*256 + tid = (stored pixel, chunk) with the chunk fastest (eight
  // lanes read one pixel's 128 B); destination = plane `chunk` at the pixel's patch index
  unsigned asrc[NL];
  int adst[NL];  // byte offset in a patch buffer, -1 = no item
  int ydst[NL];  // IN: element offset of the item in y_out (channel block 0), -1 = not written
  const bool write_y = BNIN && tn == 0;
  {
    const int pw = (a.rows + 2) * W;  // stored pixels per image
    const int npix = a.imgs * pw;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int it = u * 256 + tid;
      const int px = it >> 3, c = it & 7;
      unsigned off = kOOB;
      int dst = -1, yd = -1;
      if (px < npix) {
        const int img = px / pw, loc = px - img * pw;
        const int hr = loc / W, wc = loc - hr * W;
        const int h = h0 + hr - 1;
        if (h >= 0 && h < H) {
          const int n = n0 + img;
          if (IN == 2)  // top-left pixel of the 2x2 window in zin [N][2H][2W][C]
            off = (unsigned)(2 * (((n * 2 * H + 2 * h) * 2 * W + 2 * wc) * C + c * 8));
          else
            off = (unsigned)(2 * (((n * H + h) * W + wc) * C + c * 8));
          // the band's own rows (not its halo) are materialised by the first column tile
          if (write_y && hr >= 1 && hr <= a.rows) yd = ((n * H + h) * W + wc) * C + c * 8;
        }
        dst = (plane_base(c, a.plane) + img * a.imgp + loc) * 16;
      }
      asrc[u] = off;
      adst[u] = dst;
      ydst[u] = yd;
    }
  }
  typedef int v4i __attribute__((ext_vector_type(4)));
  v4i areg[NL][NP];
  // (IN == 2) byte offsets of the window's other three pixels: (0, 1), (1, 0), (1, 1)
  const unsigned pofs[4] = {0u, (unsigned)(2 * C), (unsigned)(2 * 2 * W * C),
                            (unsigned)(2 * (2 * W * C + C))};
  auto load_a = [&](int cb) {
    const unsigned coff = (unsigned)(cb * 128);
#pragma unroll
    for (int u = 0; u < NL; ++u)
#pragma unroll
      for (int d = 0; d < NP; ++d)
        areg[u][d] = __builtin_amdgcn_raw_buffer_load_b128(rsA, (int)(asrc[u] + coff + pofs[d]), 0, 0);
  };
  auto store_a = [&](int buf, int cb) {
    char* dst = reinterpret_cast<char*>(abuf + buf * aelems);
    float sc[8], sh[8];
    if (BNIN) {  // this thread's eight channels (its chunk is the same for every item)
      const int c0 = cb * 64 + (tid & 7) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sc[e] = cf[c0 + e];
        sh[e] = cf[C + c0 + e];
      }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      if (adst[u] < 0) continue;
      v4i v = areg[u][0];
      if (BNIN) {
        if (asrc[u] == kOOB) {
          v = (v4i){0, 0, 0, 0};  // conv zero padding of the post-BN activation
        } else {
          float best[8];
#pragma unroll
          for (int d = 0; d < NP; ++d) {
            const v4i q = areg[u][d];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const unsigned w32 = (unsigned)q[e >> 1];
              const float zf = __uint_as_float((e & 1) ? (w32 & 0xffff0000u) : (w32 << 16));
              float y = zf * sc[e] + sh[e];
              if (a.in_relu) y = fmaxf(y, 0.f);
              if (d == 0 || y > best[e] || y != y) best[e] = y;  // bn_act.hip's pool rule
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[e] = (int)((unsigned)f2bf(best[2 * e]) | ((unsigned)f2bf(best[2 * e + 1]) << 16));
          if (ydst[u] >= 0)
            *reinterpret_cast<v4i*>(a.y_out + ydst[u] + cb * 64) = v;
        }
      }
      *reinterpret_cast<v4i*>(dst + adst[u]) = v;
    }
  };
  // ---- B (weights) DMA: row (tid >> 3) + 32 i of the [col][k] tile, logical chunk lcB
  const int lcB = (tid & 7) ^ ((tid >> 4) & 7);
  unsigned boff[CB];
#pragma unroll
  for (int i = 0; i < CB; ++i) {
    const int col = col0 + (tid >> 3) + 32 * i;
    boff[i] = col < K ? (unsigned)(2 * (col * 9 * C + lcB * 8)) : kOOB;
  }

  auto issue_b = [&](int j, int slot) {
    const int cb = cb0 + j / 9, t = j - (j / 9) * 9;
    const unsigned k0 = (unsigned)(2 * (t * C + cb * 64));
    unsigned short* dst = bring + slot * BTILE;
#pragma unroll
    for (int i = 0; i < CB; ++i) dma(rsB, boff[i] + k0, dst + (wid * 64 + 256 * i) * 8);
  };

  // ---- fragment addresses (bytes within a patch buffer / B stage)
  int fa_base[TM];       // patch pixel of tap (r, s) = (0, 1) at chunk plane (lane >> 4), bytes
  unsigned col_ok[TM];   // bit 0: tap s = 0 valid, bit 1: s = 2 valid
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = wm * WTM + i * 16 + (lane & 15);  // tile-local output row
    const int per_img = a.rows * W;
    const int img = m / per_img, rem = m - img * per_img;
    const int rr = rem / W, cc = rem - rr * W;
    const int pix = img * a.imgp + rr * W + cc;  // patch pixel at tap row 0, column cc
    fa_base[i] = (plane_base(lane >> 4, a.plane) + pix) * 16;
    col_ok[i] = (cc >= 1 ? 1u : 0u) | (cc <= W - 2 ? 2u : 0u);
  }
  const int kk_a = (plane_base(4, a.plane) - plane_base(0, a.plane)) * 16;  // chunk planes +4
  int fb_off[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) fb_off[j] = rk_off(wn * WTN + j * 16 + (lane & 15), lane >> 4);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int t, int abuf_i, int slot) {
    const char* Ab = reinterpret_cast<const char*>(abuf + abuf_i * aelems);
    const unsigned short* Bs = bring + slot * BTILE;
    const int r = t / 3, s = t - r * 3;
    const int trow = r * W * 16, tcol = (s - 1) * 16;
#pragma unroll
    for (int kk = 0; kk < 64; kk += 32) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        // an edge column's s = 0 / 2 tap is padding: the lane reads its own (centre) pixel —
        // the address its neighbour lane reads for that tap, so no extra bank traffic — and
        // zeroes the fragment
        const bool ok = s == 1 || (col_ok[i] & (s == 0 ? 1u : 2u));
        const int off = fa_base[i] + trow + (ok ? tcol : 0) + (kk ? kk_a : 0);
        fa[i] = *reinterpret_cast<const bf16x8*>(Ab + off);
        if (s != 1 && !ok) fa[i] = (bf16x8){};
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(Bs + (fb_off[j] ^ (kk ? 32 : 0)));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  // ---- prologue: patch of cb0 (through registers), B k-steps 0 .. NST-2
  load_a(cb0);
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nsteps) issue_b(s, s);
  store_a(0, cb0);  // (waits for the patch loads, not for the B DMAs issued after them)

  // ---- main loop: channel blocks x the nine taps (unrolled: tap offsets, the zero-column
  // selects and the wait counts are compile-time). Wait count at k-step j = vector-memory
  // instructions issued after B(j): the B stages j+1 .. j+NST-2 still in flight, plus the next
  // patch's loads when they were issued inside that window (at t == 0 of this channel block,
  // i.e. t in [1, NST-2]). The patch's LDS writes are drained before the first barrier of the
  // channel block that reads them.
  const int ncbl = cb1 - cb0;
  int slot = 0;
  for (int cbl = 0; cbl < ncbl; ++cbl) {
    const bool more = cbl + 1 < ncbl;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int j = cbl * 9 + t;
      const int bafter = min(NST - 2, nsteps - 1 - j);
      const bool anext = (t >= 1 && t <= NST - 2) && more;
      if (t == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_stage<NST - 2, CB, NL * NP>(bafter, anext);
      // every wave finished k-step j-1: ring slot (j-1) % NST is free
      if (t == 0 && more) load_a(cb0 + cbl + 1);
      if (j + NST - 1 < nsteps) issue_b(j + NST - 1, slot == 0 ? NST - 1 : slot - 1);
      compute(t, cbl & 1, slot);
      // after the last tap: the next patch goes to the other buffer (its readers, channel
      // block cb-1, all passed this block's first barrier)
      if (t == 8 && more) store_a((cbl + 1) & 1, cb0 + cbl + 1);
      slot = slot + 1 == NST ? 0 : slot + 1;
    }
  }

  // ---- epilogue: acc[i][j][v] = D[row0 + wm*WTM + i*16 + (lane&15)][col0 + wn*WTN + j*16 + 4*(lane>>4) + v]
  const int rl = lane & 15, cq = 4 * (lane >> 4);
  const int cbase = col0 + wn * WTN + cq;
  if (a.splits > 1) {
    float* slab = a.ws + (size_t)sp * M * K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = row0 + wm * WTM + i * 16 + rl;
      if (row >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = cbase + j * 16;
        if (col >= K) continue;
        const f32x4 v = acc[i][j];
        *reinterpret_cast<float4*>(slab + (size_t)row * K + col) = (float4){v[0], v[1], v[2], v[3]};
      }
    }
    return;
  }
  const bool red = a.stats != nullptr;
  float* sl = reinterpret_cast<float*>(smem);
  if (red) __syncthreads();  // the LDS operand space takes the statistics hand-off
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = cbase + j * 16;
    float4 bj = {0.f, 0.f, 0.f, 0.f};
    if (a.bias != nullptr && col < K) bj = *reinterpret_cast<const float4*>(a.bias + col);
    float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = row0 + wm * WTM + i * 16 + rl;
      if (row >= M || col >= K) continue;
      const f32x4 v = acc[i][j];
      uint2 pk;
      pk.x = (unsigned)f2bf(v[0] + bj.x) | ((unsigned)f2bf(v[1] + bj.y) << 16);
      pk.y = (unsigned)f2bf(v[2] + bj.z) | ((unsigned)f2bf(v[3] + bj.w) << 16);
      *reinterpret_cast<uint2*>(a.z + (size_t)row * K + col) = pk;
      if (red) {  // statistics of the stored (bf16-rounded) values
        const float r0 = __uint_as_float(pk.x << 16), r1 = __uint_as_float(pk.x & 0xffff0000u);
        const float r2 = __uint_as_float(pk.y << 16), r3 = __uint_as_float(pk.y & 0xffff0000u);
        s[0] += r0; s[1] += r1; s[2] += r2; s[3] += r3;
        ss[0] += r0 * r0; ss[1] += r1 * r1; ss[2] += r2 * r2; ss[3] += r3 * r3;
      }
    }
    if (red) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        s[q] = dpp_sum16(s[q]);
        ss[q] = dpp_sum16(ss[q]);
      }
      float* st = sl + ((((wm * 2 + wn) * TN + j) * 4 + (lane >> 4)) * 8);
      if (rl == 0) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          st[q] = s[q];
          st[4 + q] = ss[q];
        }
      }
    }
  }
  if (!red) return;
  __syncthreads();
  if (wm == 0 && rl == 0) {
    float* st = a.stats + stat_rep(blockIdx.x) * 2 * K;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = cbase + j * 16;
      if (col >= K) continue;
      const float* s0 = sl + (((wn * TN + j) * 4 + (lane >> 4)) * 8);
      const float* s1 = sl + ((((2 + wn) * TN + j) * 4 + (lane >> 4)) * 8);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        atomicAdd(st + col + q, stat_val(s0[q] + s1[q], blockIdx.x));
        atomicAdd(st + K + col + q, stat_val(s0[4 + q] + s1[4 + q], blockIdx.x));
      }
    }
  }
}

// ------------------------------------------------------------------ host side
// Tile geometry of a problem: (BM, W, H) -> images / rows per tile, patch pitch, plane size.
struct Geo {
  int imgs, rows, bands, imgp, plane, zslot, nl, abuf;
  bool ok;
};

// ds_read_b128 lane groups (MI355X_MICROARCH.md §LDS): one LDS cycle each
static const int kGroups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

// every fragment read of every tap hits 16 distinct bank quads (reads of the zero slot — edge
// columns of the s = 0 / 2 taps — are ignored: at most two such lanes per group)
static bool conflict_free(int BM, int W, int rows, int imgp, int plane) {
  const int per_img = rows * W;
  for (int m0 = 0; m0 < BM; m0 += 16)
    for (int t = 0; t < 9; ++t) {
      const int r = t / 3, s = t % 3;
      for (int kk = 0; kk < 2; ++kk)
        for (int g = 0; g < 4; ++g) {
          bool used[16] = {false};
          for (int e = 0; e < 16; ++e) {
            const int l = kGroups[g][e];
            const int m = m0 + (l & 15), cp = (l >> 4) + 4 * kk;
            const int img = m / per_img, rem = m % per_img, rr = rem / W, cc = rem % W;
            const bool ok = (s == 1) || (s == 0 && cc >= 1) || (s == 2 && cc <= W - 2);
            if (!ok) continue;
            const int pix = img * imgp + (rr + r) * W + cc + s - 1;
            const int q = (plane_base(cp, plane) + pix) & 15;
            if (used[q]) return false;
            used[q] = true;
          }
        }
    }
  return true;
}

static Geo geometry_uncached(int BM, int N, int H, int W) {
  Geo g{};
  g.ok = false;
  const int hw = H * W;
  if (W < 2 || BM % 16) return g;
  if (hw <= BM) {
    if (BM % hw || N % (BM / hw)) return g;
    g.imgs = BM / hw;
    g.rows = H;
    g.bands = 1;
  } else {
    if (BM % W) return g;
    g.rows = BM / W;
    if (H % g.rows) return g;
    g.imgs = 1;
    g.bands = H / g.rows;
  }
  const int pw = (g.rows + 2) * W;
  for (int imgp = pw; imgp < pw + 32; ++imgp) {
    const int npix = g.imgs * imgp;
    const int plane = (npix + 1 + 15) / 16 * 16;
    if (conflict_free(BM, W, g.rows, imgp, plane)) {
      g.imgp = imgp;
      g.plane = plane;
      g.zslot = npix;
      g.nl = (g.imgs * pw * 8 + 255) / 256;
      g.abuf = (plane_base(7, plane) + plane) * 8;  // bf16 elements
      g.ok = true;
      return g;
    }
    if (g.imgs == 1) break;  // a single image's pitch never matters: rows are contiguous
  }
  return g;
}

// the conflict search runs once per (BM, N, H, W) — it is host work on every launch otherwise
static Geo geometry(int BM, int N, int H, int W) {
  static std::map<std::tuple<int, int, int, int>, Geo> cache;
  const auto key = std::make_tuple(BM, N, H, W);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const Geo g = geometry_uncached(BM, N, H, W);
  cache[key] = g;
  return g;
}

// in: 0 plain, 1 / 2 BN + ReLU (+ pool) input ([2][C] table)
static size_t lds_bytes(const Args& a, int nst, int bn, int in) {
  const size_t table = in ? 2 * (size_t)a.C * 4 : 0;
  return 2 * (size_t)a.abuf_elems * 2 + (size_t)nst * bn * 64 * 2 + table;
}

template <int BM, int BN, int NST, int NL, int IN>
static void launch_t(const Args& a, int items, hipStream_t st) {
  const size_t lds = lds_bytes(a, NST, BN, IN);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(conv_tr_fwd_kernel<BM, BN, NST, NL, IN>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((conv_tr_fwd_kernel<BM, BN, NST, NL, IN>), dim3(items), dim3(256), lds, st, a);
}

template <int BM, int BN, int NST, int IN>
static bool launch_nl(const Args& a, int nl, int items, hipStream_t st) {
  if (lds_bytes(a, NST, BN, IN) > 160 * 1024) return false;
  switch (nl) {
    case 1: launch_t<BM, BN, NST, 1, IN>(a, items, st); return true;
    case 2: launch_t<BM, BN, NST, 2, IN>(a, items, st); return true;
    case 3: launch_t<BM, BN, NST, 3, IN>(a, items, st); return true;
    case 4: launch_t<BM, BN, NST, 4, IN>(a, items, st); return true;
    case 5: launch_t<BM, BN, NST, 5, IN>(a, items, st); return true;
    case 6: launch_t<BM, BN, NST, 6, IN>(a, items, st); return true;
    default: return false;
  }
}

template <int BM, int BN>
static bool launch_bmbn(int nst, int in, const Args& a, int nl, int items, hipStream_t st) {
  if (in == 1) return nst == 3 && launch_nl<BM, BN, 3, 1>(a, nl, items, st);
  if (in == 2) return nst == 3 && launch_nl<BM, BN, 3, 2>(a, nl, items, st);
  switch (nst) {
    case 3: return launch_nl<BM, BN, 3, 0>(a, nl, items, st);
    case 5: return launch_nl<BM, BN, 5, 0>(a, nl, items, st);
    case 8: return launch_nl<BM, BN, 8, 0>(a, nl, items, st);
    default: return false;
  }
}

// configuration table (tools/conv_tune.py --tr writes ops/conv_tuning.json "tr" entries):
// (M, K, C, H) -> (BM, BN, splits); absent -> heuristic
struct Cfg {
  int bm, bn, splits, stages;  // stages: B ring depth (3, 5 or 8; 0 = policy)
};

// B ring depth: the table's (3 was fastest for every VGG layer: deeper rings cost occupancy,
// profiles/r3_conv_tr_sweep.jsonl); the fused-input modes are built with 3 only
static bool launch_stages(const Cfg& c, int in, const Args& a, int nl, int items, hipStream_t st) {
  const int n = in ? 3 : (c.stages ? c.stages : 3);
  if (c.bm == 128 && c.bn == 128) return launch_bmbn<128, 128>(n, in, a, nl, items, st);
  if (c.bm == 128 && c.bn == 64) return launch_bmbn<128, 64>(n, in, a, nl, items, st);
  if (c.bm == 64 && c.bn == 128) return launch_bmbn<64, 128>(n, in, a, nl, items, st);
  if (c.bm == 64 && c.bn == 64) return launch_bmbn<64, 64>(n, in, a, nl, items, st);
  return false;
}
static std::map<std::tuple<int, int, int, int>, Cfg> g_tr_tuned;  // (M, K, C, H)
static int g_tr_mode = 1;  // 0 off, 1 table entries only, 2 also the heuristic (ddp_conv_tr_mode)
static Cfg g_tr_force{0, 0, 0, 0};

static Cfg heuristic(int N, int H, int W, int C, int K) {
  const int M = N * H * W;
  const int ncb = C / 64;
  Cfg c{128, K % 128 == 0 && K >= 256 ? 128 : 64, 1, 0};
  if (M / 128 * (K / c.bn) < 256) c.bm = 64;
  if (!geometry(c.bm, N, H, W).ok) c.bm = c.bm == 128 ? 64 : 128;
  const int tiles = (M / c.bm) * (K / c.bn);
  int s = 1;
  while (tiles * s < 256 && s * 2 <= ncb) s *= 2;
  c.splits = s;
  return c;
}

}  // namespace tr
}  // namespace ddp_amd

using namespace ddp_amd;

extern "C" int ddp_conv_fwd_finish(const ConvGeom* g, float* ws, int splits, const float* bias,
                                   void* z, float* stats, const BnFwdFuse* bn, int* bn_done,
                                   hipStream_t st);

extern "C" void ddp_conv_tr_set(int mode, int M, int K, int C, int H, int bm, int bn, int splits,
                                int stages) {
  // mode: -1 clear table, 0/1 enable, 2 add table entry, 3 force (bm, bn, splits) for sweeps
  if (mode == -1) { tr::g_tr_tuned.clear(); return; }
  if (mode == 0 || mode == 1 || mode == 4) { tr::g_tr_mode = mode == 4 ? 2 : mode; return; }
  if (mode == 2) { tr::g_tr_tuned[std::make_tuple(M, K, C, H)] = tr::Cfg{bm, bn, splits, stages}; return; }
  if (mode == 3) tr::g_tr_force = tr::Cfg{bm, bn, splits, stages};
}

namespace ddp_amd {
namespace tr {
struct Plan {
  Cfg c;
  Geo geo;
  int splits, cbps;
};

// the launch decision shared by ddp_conv_fwd_tr and ddp_conv_tr_would_serve
static bool plan(const ConvGeom* g, float* ws, size_t ws_elems, int in_mode, Plan* p) {
  if (!g_tr_mode) return false;
  if (g->R != 3 || g->S != 3 || g->stride != 1 || g->pad != 1 || g->P != g->H || g->Q != g->W)
    return false;
  if (g->C % 64 || g->K % 64 || g->Creal != g->C) return false;
  // 2x2 images go to the dense GEMM form (conv_igemm.hip: 4 of 9 taps per pixel are real),
  // unless a sweep / test forces this kernel
  if (!g_tr_force.bm && ddp_conv_dense2x2_ok(g)) return false;
  const int N = g->N, H = g->H, W = g->W, C = g->C, K = g->K;
  const size_t M = (size_t)N * H * W;
  const size_t xe = M * C * (in_mode == 2 ? 4 : 1), we = (size_t)K * 9 * C;
  if (2 * xe >= kOOB || 2 * we >= kOOB || M * K >= kOOB) return false;
  Cfg c;
  auto it = g_tr_tuned.find(std::make_tuple((int)M, K, C, H));
  if (g_tr_force.bm) c = g_tr_force;
  else if (it != g_tr_tuned.end()) c = it->second;
  else if (g_tr_mode == 2) c = heuristic(N, H, W, C, K);
  else return false;  // default: only the layers the measured table assigns to this kernel
  if (c.bm == 0) return false;  // table entry "use the implicit-GEMM kernel"
  if (K % c.bn || M % c.bm) return false;
  const Geo geo = geometry(c.bm, N, H, W);
  if (!geo.ok || geo.nl < 1 || geo.nl > 6) return false;
  const int nst = in_mode ? 3 : (c.stages ? c.stages : 3);
  const size_t lds = 2 * (size_t)geo.abuf * 2 + (size_t)nst * c.bn * 64 * 2 +
                     (in_mode ? 2 * (size_t)C * 4 : 0);
  if (lds > 160 * 1024) return false;
  const int ncb = C / 64;
  int splits = std::max(1, std::min(c.splits, ncb));
  int cbps = (ncb + splits - 1) / splits;
  splits = (ncb + cbps - 1) / cbps;
  if (splits > 1 && (ws == nullptr || (size_t)splits * M * K > ws_elems)) {
    splits = 1;
    cbps = ncb;
  }
  p->c = c;
  p->geo = geo;
  p->splits = splits;
  p->cbps = cbps;
  return true;
}
}  // namespace tr
}  // namespace ddp_amd

// 3x3 / stride 1 / pad 1 forward through the tap-reuse kernel. ``in`` (optional): the input is
// computed from the preceding block's conv output while the patch is loaded (TrFwdIn). Returns
// 1 when served (z and the statistics written; with ``bn`` and a split-K launch whose finish
// fused this block's BatchNorm forward *bn_done = 1), 0 when not served (caller falls back to
// ddp_conv_fwd[_bn], after materialising a fused input itself), < 0 invalid arguments, >= 2 HIP
// error (rc - 2).
extern "C" int ddp_conv_fwd_tr(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                               void* z, float* stats, float* ws, size_t ws_elems,
                               const BnFwdFuse* bn, int* bn_done, const TrFwdIn* in,
                               hipStream_t st) {
  using namespace ddp_amd::tr;
  if (bn_done) *bn_done = 0;
  const int in_mode = in ? (in->pool ? 2 : 1) : 0;
  if (in && (!in->z || !in->stats || !in->gamma || !in->beta || !in->coef || !in->y)) return -1;
  Plan pl;
  if (!plan(g, ws, ws_elems, in_mode, &pl)) return 0;
  const Cfg& c = pl.c;
  const Geo& geo = pl.geo;
  const int N = g->N, H = g->H, W = g->W, C = g->C, K = g->K;
  const size_t M = (size_t)N * H * W;
  Args a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.K = K;
  a.x = (const unsigned short*)x;
  a.wc = (const unsigned short*)wc;
  a.bias = bias;
  a.z = (unsigned short*)z;
  a.stats = stats;
  a.ws = ws;
  a.splits = pl.splits;
  a.cbps = pl.cbps;
  a.imgs = geo.imgs; a.rows = geo.rows; a.bands = geo.bands;
  a.imgp = geo.imgp; a.plane = geo.plane; a.zslot = geo.zslot;
  a.x_bytes = (int)(2 * M * C);
  a.w_bytes = (int)(2 * (size_t)K * 9 * C);
  a.abuf_elems = geo.abuf;
  a.tiles_m = (int)(M / c.bm);
  a.tiles_n = K / c.bn;
  if (in) {
    a.zin = (const unsigned short*)in->z;
    a.in_stats = in->stats;
    a.in_gamma = in->gamma;
    a.in_beta = in->beta;
    a.in_eps = in->eps;
    a.in_relu = in->relu;
    a.in_coef = in->coef;
    a.y_out = (unsigned short*)in->y;
    a.z_bytes = (int)(2 * M * C * (in->pool ? 4 : 1));
  }
  const int items = a.tiles_m * a.tiles_n * pl.splits;
  if (!launch_stages(c, in_mode, a, geo.nl, items, st)) return 0;
  int e = (int)hipGetLastError();
  if (e) return 2 + e;
  if (pl.splits > 1) {
    e = ddp_conv_fwd_finish(g, ws, pl.splits, bias, z, stats, bn, bn_done, st);
    if (e) return 2 + e;
  }
  return 1;
}

// would ddp_conv_fwd_tr serve this problem (with a fused input of mode in_mode: 0 none,
// 1 BN+ReLU, 2 BN+ReLU+pool)? No launch.
extern "C" int ddp_conv_tr_would_serve(const ConvGeom* g, size_t ws_elems, int in_mode) {
  ddp_amd::tr::Plan pl;
  float dummy;
  if (in_mode < 0) return 0;
  return ddp_amd::tr::plan(g, ws_elems ? &dummy : nullptr, ws_elems, in_mode, &pl) ? 1 : 0;
}

// host-side geometry probe for tests: (ok, imgs, rows, bands, imgp, plane, na)
extern "C" int ddp_conv_tr_geometry(int BM, int N, int H, int W, int* out7) {
  const ddp_amd::tr::Geo g = ddp_amd::tr::geometry(BM, N, H, W);
  out7[0] = g.ok; out7[1] = g.imgs; out7[2] = g.rows; out7[3] = g.bands;
  out7[4] = g.imgp; out7[5] = g.plane; out7[6] = g.nl;
  return g.ok ? 1 : 0;
}
