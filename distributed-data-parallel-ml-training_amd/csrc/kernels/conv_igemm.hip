// Implicit-GEMM convolution for gfx950: forward, backward-data and backward-weight on bf16
// MFMA (v_mfma_f32_16x16x32_bf16) with fp32 accumulation.
//
// Reference parity: replaces the ATen/oneDNN Conv2d fwd/bwd the reference triggers from
// part1/model.py:18-23 (3x3 s1 p1 + bias) — SURVEY.md §2.B N1, shapes in §2.D. Also serves
// ResNet-50's 1x1 / 3x3 / 7x7, stride 1/2 convolutions and the 2048->1000 classifier (1x1 conv).
//
// Layouts (NHWC, channels innermost, C % 8 == 0 — layer 0 is zero-padded 3 -> 8):
//   x  [N][H][W][C]      bf16  activations
//   y  [N][P][Q][K]      bf16  conv output (pre-BN)
//   Wc [K][R][S][C]      bf16  forward weight copy   (GEMM B operand, k-contiguous)
//   Wt [C][R][S][K]      bf16  dgrad weight copy     (GEMM B operand, k-contiguous)
//   dW [K][Creal][R][S]  fp32  PyTorch-layout weight gradient (accumulated)
//
// GEMM views (rows x cols, reduction):
//   FWD   : M=N*P*Q, N=K,      red=R*S*C   A=im2col(x)          B=Wc
//   DGRAD : M=N*H*W, N=C,      red=R*S*K   A=col2im-gather(dy)  B=Wt
//   WGRAD : M=K,     N=R*S*C,  red=N*P*Q   A=dy^T               B=im2col(x)^T
//
// Kernel structure (256 threads = 4 waves in 2x2, BK = 64):
//   * operands are gathered global->registers (implicit im2col with zero fill), written to a
//     double-buffered LDS tile AFTER the MFMA phase that overlaps their flight, one barrier per
//     k-step (cdna_hip_programming.md §5.5 T14 / Guideline 15);
//   * FWD/DGRAD tiles are [row][k] with the 16-B chunk index XOR-swizzled by (row>>1)&7, read
//     by ds_read_b128 conflict-free (T2);
//   * WGRAD tiles keep the global order [m][channel] (m = the reduction index) and the MFMA
//     fragments are read with ds_read_b64_tr_b16 (gfx950 transposing LDS read, T10), chunk
//     XOR-swizzled by m so both 16-lane groups of a half-wave hit disjoint banks;
//   * XCD-aware bijective tile order (T1); split-K writes plain fp32 slabs [split][M][N] that a
//     finish kernel reduces in a fixed order (no float atomics on the GEMM output);
//   * FWD epilogue adds the bias, rounds to bf16 and accumulates the per-channel BatchNorm
//     statistics of the rounded output (sum, sum of squares) — BN needs no separate stats pass.
#include "common.h"
#include "api.h"
#include <algorithm>

namespace ddp_amd {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

struct ConvArgs {
  ConvGeom g;
  const unsigned short* a;   // FWD: x, DGRAD: dy, WGRAD: dy
  const unsigned short* b;   // FWD: Wc, DGRAD: Wt, WGRAD: x
  unsigned short* out;       // FWD: y, DGRAD: dx (bf16)
  float* dw;                 // WGRAD output (PyTorch layout, accumulated)
  float* ws;                 // split-K slabs [splits][Mg][Ng]
  const float* bias;         // FWD only (may be null)
  float* stats;              // FWD only: [2*Ng] sum / sum-of-squares of the bf16 output
  int Mg, Ng, Kg;            // GEMM dims
  int splits;
  int ksteps_per_split;
  int wg_atomic;             // WGRAD split-K: fp32 atomics into dw instead of slabs + finish
};

// ------------------------------------------------------------------ operand gathers
// Index math is hoisted: the pixel decomposition of a GEMM row is computed once per kernel
// (RowInfo), the (r, s, c) decomposition of the reduction index once per k-step, and runtime
// divisions inside the k-loop use a float-reciprocal divmod (exact for x < 2^23).
__device__ __forceinline__ int fdiv(int x, int d, float inv) {
  int q = (int)((float)x * inv);
  const int r = x - q * d;
  q += (r < 0) ? -1 : (r >= d ? 1 : 0);
  return q;
}

struct RowInfo {
  int base;    // element offset of the row's image (FWD: n*H*W*C, DGRAD: n*P*Q*K)
  int h0, w0;  // FWD: p*stride-pad, q*stride-pad ; DGRAD: h+pad, w+pad ; invalid row: h0 < -2^20
};

template <int MODE>
__device__ __forceinline__ RowInfo row_info(const ConvArgs& A, int row) {
  const ConvGeom& g = A.g;
  RowInfo ri{0, -(1 << 24), 0};
  if (row >= A.Mg) return ri;
  if (MODE == MODE_FWD) {
    const int pq = g.P * g.Q;
    const int n = row / pq, rem = row - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    ri.base = n * g.H * g.W * g.C;
    ri.h0 = p * g.stride - g.pad;
    ri.w0 = q * g.stride - g.pad;
  } else {
    const int hw = g.H * g.W;
    const int n = row / hw, rem = row - n * hw;
    const int h = rem / g.W, w = rem - h * g.W;
    ri.base = n * g.P * g.Q * g.K;
    ri.h0 = h + g.pad;
    ri.w0 = w + g.pad;
  }
  return ri;
}

struct KInfo {
  int r, s, c;  // kernel tap and channel of the chunk's first reduction element
  bool ok;
};

template <int MODE>
__device__ __forceinline__ KInfo k_info(const ConvArgs& A, int kk, float invC, float invS) {
  const ConvGeom& g = A.g;
  KInfo k;
  k.ok = kk < A.Kg;
  const int cdim = MODE == MODE_FWD ? g.C : g.K;
  const int rs = fdiv(kk, cdim, invC);
  k.c = kk - rs * cdim;
  k.r = fdiv(rs, g.S, invS);
  k.s = rs - k.r * g.S;
  return k;
}

template <int MODE>
__device__ __forceinline__ u16x8 gather_a(const ConvArgs& A, const RowInfo& ri, const KInfo& k) {
  const ConvGeom& g = A.g;
  u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!k.ok) return z;
  if (MODE == MODE_FWD) {
    const int h = ri.h0 + k.r, w = ri.w0 + k.s;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return z;
    return ld8(A.a + ri.base + (h * g.W + w) * g.C + k.c);
  } else {
    int ph = ri.h0 - k.r, pw = ri.w0 - k.s;
    if (ph < 0 || pw < 0) return z;
    if (g.stride != 1) {
      if ((ph % g.stride) | (pw % g.stride)) return z;
      ph /= g.stride;
      pw /= g.stride;
    }
    if (ph >= g.P || pw >= g.Q) return z;
    return ld8(A.a + ri.base + (ph * g.Q + pw) * g.K + k.c);
  }
}

// WGRAD B' chunk: x at pixel-index m for the 8 consecutive (r,s,c) columns described by k.
__device__ __forceinline__ u16x8 gather_x_wgrad(const ConvArgs& A, const KInfo& k, int m,
                                                float invPQ, float invQ) {
  const ConvGeom& g = A.g;
  u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!k.ok || m >= A.Kg) return z;
  const int pq = g.P * g.Q;
  const int n = fdiv(m, pq, invPQ), rem = m - n * pq;
  const int p = fdiv(rem, g.Q, invQ), q = rem - p * g.Q;
  const int h = p * g.stride - g.pad + k.r, w = q * g.stride - g.pad + k.s;
  if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return z;
  return ld8(A.b + ((n * g.H + h) * g.W + w) * g.C + k.c);
}

// ------------------------------------------------------------------ LDS addressing
// [row][k] tile, 64 bf16 per row = 8 chunks of 16 B; chunk XOR (row>>1)&7 (ds_read_b128 reads
// of 16 consecutive rows at one logical chunk hit 16 distinct slots).
__device__ __forceinline__ int rk_off(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3);
}
// [m][col] tile with NCOL bf16 per row (WGRAD), read with ds_read_b64_tr_b16. A half-wave reads
// rows {m0..m0+3} and {m0+8..m0+11} at the same two 16-B chunks; the XOR makes those 16
// (row, chunk) pairs land on 16 distinct bank slots (conflict-free).
template <int NCOL>
__device__ __forceinline__ int mc_swz(int m) {
  if (NCOL >= 128) return (((m & 3) | (((m >> 3) & 1) << 2)) << 1) & (NCOL / 8 - 1);
  return ((((m >> 1) & 1) | (((m >> 3) & 1) << 1)) << 1);  // 8 chunks: row parity splits banks
}
template <int NCOL>
__device__ __forceinline__ int mc_off(int m, int col) {
  return m * NCOL + (((col >> 3) ^ mc_swz<NCOL>(m)) << 3) + (col & 7);
}

// 16 zero bytes: the source of every LDS-DMA lane whose im2col element lies in the padding.
__device__ __attribute__((aligned(64))) unsigned short g_zero16[32];

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(const void* src, unsigned short* lds_wave_base) {
  // global_load_lds_dwordx4: LDS destination = wave-uniform base + lane * 16 (no VGPR staging)
  __builtin_amdgcn_global_load_lds(src, (lds_void*)lds_wave_base, 16, 0, 0);
}

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs args) {
  constexpr int BK = 64;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = BM * BK / 8 / 256;  // 16-B chunks per thread per tile
  constexpr int CB = BN * BK / 8 / 256;
  constexpr int TILE_A = BM * BK, TILE_B = BN * BK;
  static_assert(CA >= 1 && CB >= 1, "tile too small for 256 threads");
  __shared__ __attribute__((aligned(16))) unsigned short smem[2 * (TILE_A + TILE_B)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_n = (args.Ng + BN - 1) / BN;
  const int tiles_m = (args.Mg + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;

  const int ksteps = (args.Kg + BK - 1) / BK;
  const int ks_begin = blockIdx.z * args.ksteps_per_split;
  const int ks_end = min(ksteps, ks_begin + args.ksteps_per_split);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const ConvGeom& gg = args.g;
  const unsigned short* zero = g_zero16;

  // ---------------- per-thread gather state (index math hoisted out of the k-loop) ----------------
  // FWD/DGRAD: DMA chunk c = tid + 256 i lands at LDS byte 16 c = row (tid>>3)+32i, physical
  // chunk tid&7; it must carry LOGICAL chunk lc = (tid&7) ^ ((row>>1)&7) = constant per thread.
  // WGRAD: row = m (reduction), physical chunk tid % (BX/8), logical = phys ^ swz(m) (constant).
  constexpr int NA = (MODE != MODE_WGRAD) ? CA : 1;
  int a_rowoff[NA];      // FWD: n*H*W*C + (h0*W + w0)*C ; DGRAD: n*P*Q*K + (h0*Q + w0)*K
  int a_h0[NA], a_w0[NA];
  int b_col_ok = 0;      // bit i: B row i valid
  int lcA, lcB;
  int kr = 0, ks_ = 0, kc = 0;  // (r, s, c) of this thread's reduction chunk for the current k-step
  KInfo xk;              // WGRAD: (r,s,c) of this thread's B' column group
  const float invPQ = 1.f / (float)(gg.P * gg.Q), invQ = 1.f / (float)gg.Q;
  if (MODE != MODE_WGRAD) {
    lcA = lcB = (tid & 7) ^ ((tid >> 4) & 7);
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const RowInfo ri = row_info<MODE>(args, row0 + (tid >> 3) + 32 * i);
      a_h0[i] = ri.h0;
      a_w0[i] = ri.w0;
      a_rowoff[i] = (MODE == MODE_FWD) ? ri.base + (ri.h0 * gg.W + ri.w0) * gg.C
                                       : ri.base + (ri.h0 * gg.Q + ri.w0) * gg.K;
    }
#pragma unroll
    for (int i = 0; i < CB; ++i)
      if (col0 + (tid >> 3) + 32 * i < args.Ng) b_col_ok |= 1 << i;
    // decomposition of the first reduction index this thread loads
    const int cdim = MODE == MODE_FWD ? gg.C : gg.K;
    const int kk = ks_begin * BK + lcA * 8;
    const int rs = kk / cdim;
    kc = kk - rs * cdim;
    kr = rs / gg.S;
    ks_ = rs - kr * gg.S;
  } else {
    constexpr int NCA = BM / 8, NCB = BN / 8;
    lcA = (tid % NCA) ^ mc_swz<BM>(tid / NCA);
    lcB = (tid % NCB) ^ mc_swz<BN>(tid / NCB);
    const int j = col0 + lcB * 8;
    const int rs = j / gg.C;
    xk.c = j - rs * gg.C;
    xk.r = rs / gg.S;
    xk.s = rs - xk.r * gg.S;
    xk.ok = j < args.Ng;
  }

  // issue the LDS-DMA of k-step ks into buffer buf (and advance the incremental k state)
  auto issue = [&](int ks, int buf) {
    unsigned short* As = smem + buf * (TILE_A + TILE_B);
    unsigned short* Bs = As + TILE_A;
    const int k0 = ks * BK;
    if (MODE != MODE_WGRAD) {
      const int kk = k0 + lcA * 8;
      const bool kok = kk < args.Kg;
      const int W_ = MODE == MODE_FWD ? gg.W : gg.Q;
      const int cdim = MODE == MODE_FWD ? gg.C : gg.K;
      const int tap = MODE == MODE_FWD ? (kr * W_ + ks_) * cdim + kc : kc - (kr * W_ + ks_) * cdim;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const void* src = zero;
        if (MODE == MODE_FWD) {
          const int h = a_h0[i] + kr, w = a_w0[i] + ks_;
          if (kok && (unsigned)h < (unsigned)gg.H && (unsigned)w < (unsigned)gg.W)
            src = args.a + a_rowoff[i] + tap;
        } else {
          int ph = a_h0[i] - kr, pw = a_w0[i] - ks_;
          bool ok = kok && ph >= 0 && pw >= 0;
          if (gg.stride == 1) {
            ok = ok && ph < gg.P && pw < gg.Q;
            if (ok) src = args.a + a_rowoff[i] + tap;
          } else {  // strided conv: only taps that hit an output pixel contribute
            ok = ok && (ph % gg.stride) == 0 && (pw % gg.stride) == 0;
            ph /= gg.stride;
            pw /= gg.stride;
            ok = ok && ph < gg.P && pw < gg.Q;
            if (ok) {
              const int base = a_rowoff[i] - (a_h0[i] * gg.Q + a_w0[i]) * gg.K;
              src = args.a + base + (ph * gg.Q + pw) * gg.K + kc;
            }
          }
        }
        dma16(src, As + (wid * 64 + 256 * i) * 8);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int col = col0 + (tid >> 3) + 32 * i;
        const void* src = (kok && ((b_col_ok >> i) & 1)) ? (const void*)(args.b + (size_t)col * args.Kg + kk) : zero;
        dma16(src, Bs + (wid * 64 + 256 * i) * 8);
      }
      // advance (r, s, c) by BK reduction elements
      kc += BK;
      while (kc >= cdim) {
        kc -= cdim;
        if (++ks_ == gg.S) { ks_ = 0; ++kr; }
      }
    } else {
      constexpr int NCA = BM / 8, NCB = BN / 8;
      const int kout = row0 + lcA * 8;
#pragma unroll
      for (int i = 0; i < CA; ++i) {  // dy[m][kout]
        const int m = k0 + (tid + i * 256) / NCA;
        const void* src = (m < args.Kg && kout < args.Mg) ? (const void*)(args.a + (size_t)m * gg.K + kout) : zero;
        dma16(src, As + (wid * 64 + 256 * i) * 8);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {  // x gather at pixel m for columns (r, s, c..c+7)
        const int m = k0 + (tid + i * 256) / NCB;
        const void* src = zero;
        if (xk.ok && m < args.Kg) {
          const int pq = gg.P * gg.Q;
          const int n = fdiv(m, pq, invPQ), rem = m - n * pq;
          const int p = fdiv(rem, gg.Q, invQ), q = rem - p * gg.Q;
          const int h = p * gg.stride - gg.pad + xk.r, w = q * gg.stride - gg.pad + xk.s;
          if ((unsigned)h < (unsigned)gg.H && (unsigned)w < (unsigned)gg.W)
            src = args.b + ((n * gg.H + h) * gg.W + w) * gg.C + xk.c;
        }
        dma16(src, Bs + (wid * 64 + 256 * i) * 8);
      }
    }
  };

  // fragment LDS offsets (elements), loop-invariant
  int fa_off[TM], fb_off[TN];
  if (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < TM; ++i) fa_off[i] = rk_off(wm * WTM + i * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb_off[j] = rk_off(wn * WTN + j * 16 + (lane & 15), lane >> 4);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int m0 = 8 * g + q;
#pragma unroll
    for (int i = 0; i < TM; ++i) fa_off[i] = mc_off<BM>(m0, wm * WTM + i * 16 + 4 * p);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb_off[j] = mc_off<BN>(m0, wn * WTN + j * 16 + 4 * p);
  }

  auto compute = [&](int buf) {
    const unsigned short* As = smem + buf * (TILE_A + TILE_B);
    const unsigned short* Bs = As + TILE_A;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 fa[TM], fb[TN];
      if (MODE != MODE_WGRAD) {
        // logical chunk kk/8 + (lane>>4): the XOR swizzle is linear in the chunk index, so the
        // kk = 32 read is the kk = 0 address with chunk bit 2 flipped
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[i] = *reinterpret_cast<const bf16x8*>(As + (fa_off[i] ^ (kk ? 32 : 0)));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = *reinterpret_cast<const bf16x8*>(Bs + (fb_off[j] ^ (kk ? 32 : 0)));
      } else {
        // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group supplies row q, columns 4p..4p+3;
        // lane i receives column i of the 4 rows. Two reads give the 8 k-values of a fragment.
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const unsigned short* base = As + fa_off[i] + kk * BM;
          v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
          v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * BM));
          const short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          fa[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const unsigned short* base = Bs + fb_off[j] + kk * BN;
          v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
          v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * BN));
          const short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
          fb[j] = __builtin_bit_cast(bf16x8, v);
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          // operands swapped (D^T = B^T A^T): each lane ends up owning ONE output row and FOUR
          // consecutive output columns, so the epilogue stores 8 B (bf16) / 16 B (fp32) per lane
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  if (ks_begin < ks_end) {
    issue(ks_begin, 0);
    __syncthreads();  // waits for the DMA (vmcnt(0)) and publishes buffer 0
    int buf = 0;
    for (int ks = ks_begin; ks < ks_end; ++ks) {
      if (ks + 1 < ks_end) issue(ks + 1, buf ^ 1);  // lands during this step's MFMAs
      compute(buf);
      __syncthreads();  // next buffer landed + everyone done reading this one
      buf ^= 1;
    }
  }

  // ---------------- epilogue ----------------
  // acc[i][j][v] = D[row0 + wm*WTM + i*16 + (lane&15)][col0 + wn*WTN + j*16 + 4*(lane>>4) + v]
  // Ng % 8 == 0 for every mode (C, K multiples of 8), so a lane's 4 columns are all valid or not.
  const ConvGeom& g = args.g;
  const bool split = args.splits > 1;
  float* slab = split ? args.ws + (size_t)blockIdx.z * args.Mg * args.Ng : nullptr;
  const int rl = lane & 15, cq = 4 * (lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + wn * WTN + j * 16 + cq;
    const bool cok = col < args.Ng;
    float4 bias = {0.f, 0.f, 0.f, 0.f};
    if (MODE == MODE_FWD && !split && args.bias && cok)
      bias = (float4){args.bias[col], args.bias[col + 1], args.bias[col + 2], args.bias[col + 3]};
    float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
    int wrs = 0, wc = 0;
    if (MODE == MODE_WGRAD) {  // GEMM column -> (r*S + s, c); c..c+3 share the tap
      wrs = col / g.C;
      wc = col - wrs * g.C;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = row0 + wm * WTM + i * 16 + rl;
      if (!cok || row >= args.Mg) continue;
      const f32x4 v = acc[i][j];
      if (MODE == MODE_WGRAD && (!split || args.wg_atomic)) {
        if (g.wkrsc && g.Creal == g.C) {
          float* d = args.dw + ((size_t)row * g.R * g.S + wrs) * g.C + wc;
          if (split) {
#pragma unroll
            for (int t = 0; t < 4; ++t) unsafeAtomicAdd(d + t, v[t]);
          } else {
            float4 o = *reinterpret_cast<float4*>(d);
            o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
            *reinterpret_cast<float4*>(d) = o;
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (wc + t >= g.Creal) break;
            const size_t di = g.wkrsc ? ((size_t)row * g.R * g.S + wrs) * g.Creal + wc + t
                                      : ((size_t)row * g.Creal + wc + t) * g.R * g.S + wrs;
            if (split) unsafeAtomicAdd(args.dw + di, v[t]);
            else args.dw[di] += v[t];
          }
        }
      } else if (split) {
        *reinterpret_cast<float4*>(slab + (size_t)row * args.Ng + col) = (float4){v[0], v[1], v[2], v[3]};
      } else {
        const unsigned short h0 = f2bf(v[0] + bias.x), h1 = f2bf(v[1] + bias.y);
        const unsigned short h2 = f2bf(v[2] + bias.z), h3 = f2bf(v[3] + bias.w);
        uint2 pk;
        pk.x = (unsigned)h0 | ((unsigned)h1 << 16);
        pk.y = (unsigned)h2 | ((unsigned)h3 << 16);
        *reinterpret_cast<uint2*>(args.out + (size_t)row * args.Ng + col) = pk;
        if (MODE == MODE_FWD) {
          const float r0 = bf2f(h0), r1 = bf2f(h1), r2 = bf2f(h2), r3 = bf2f(h3);
          s[0] += r0; s[1] += r1; s[2] += r2; s[3] += r3;
          ss[0] += r0 * r0; ss[1] += r1 * r1; ss[2] += r2 * r2; ss[3] += r3 * r3;
        }
      }
    }
    if (MODE == MODE_FWD && !split && args.stats) {
      // reduce over the 16 rows held by lanes (lane & 15) of each 16-lane group
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) {
          s[t] += __shfl_xor(s[t], m, kWave);
          ss[t] += __shfl_xor(ss[t], m, kWave);
        }
      }
      if (rl == 0 && cok) {
        float* st = args.stats + (blockIdx.x % kStatRep) * 2 * args.Ng;  // spread contention
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          atomicAdd(st + col + t, s[t]);
          atomicAdd(st + args.Ng + col + t, ss[t]);
        }
      }
    }
  }
}

// Split-K finish for FWD/DGRAD: sum the slabs in split order -> (+bias) bf16 output
// (+ per-channel stats of the rounded output for FWD).
// Thread layout: cg_local = tid % Gb (8 channels each), rows strided; stats reduced in
// registers, then through LDS, then ONE atomic per channel per block.
__global__ __launch_bounds__(256) void splitk_finish_kernel(const float* ws, int splits,
                                                            unsigned short* out,
                                                            const float* bias, float* stats,
                                                            int Mg, int Ng) {
  __shared__ float red[2][8][256];
  const int G = Ng / 8;
  const int Gb = G < 256 ? G : 256;
  const int cgl = threadIdx.x % Gb, prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int cg = blockIdx.y * Gb + cgl;
  const bool active = prow < prows && cg < G;  // Gb need not divide 256 (e.g. 1000 classes)
  const size_t slab = (size_t)Mg * Ng;
  float s[8], ss[8], bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = 0.f;
    ss[e] = 0.f;
    bv[e] = (bias && cg < G) ? bias[cg * 8 + e] : 0.f;
  }
  for (int row = blockIdx.x * prows + prow; active && row < Mg; row += gridDim.x * prows) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bv[e];
    for (int z = 0; z < splits; ++z) {
      const float4* src = reinterpret_cast<const float4*>(ws + z * slab + (size_t)row * Ng + cg * 8);
      const float4 a = src[0], b = src[1];
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(v[e]);
      const float r = bf2f(o[e]);
      s[e] += r;
      ss[e] += r * r;
    }
    st8(out + (size_t)row * Ng + cg * 8, o);
  }
  if (!stats) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][e][threadIdx.x] = s[e];
    red[1][e][threadIdx.x] = ss[e];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < Gb * 16; idx += 256) {
    const int k = idx / (Gb * 8), rem = idx % (Gb * 8);
    const int c = rem / 8, e = rem % 8;
    if (blockIdx.y * Gb + c >= G) continue;
    float t = 0.f;
    for (int r = 0; r < prows; ++r) t += red[k][e][r * Gb + c];
    float* st = stats + ((blockIdx.x + blockIdx.y) % kStatRep) * 2 * Ng;
    atomicAdd(st + k * Ng + (blockIdx.y * Gb + c) * 8 + e, t);
  }
}

// Split-K finish for WGRAD: dW[k][c][r][s] += sum_z slab[z][k][(r,s,c)].
// Block (k, split-group): sums its group of slabs for GEMM row k with coalesced reads
// (reduction order fixed inside a group), transposes (r,s,c) -> (c,r,s) through LDS, and adds
// into the PyTorch-layout gradient with coalesced stores (one atomic add per group when the
// splits are divided into several groups).
constexpr int kWgFinishGroup = 32;
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* ws, int splits, int K,
                                                           int R, int S, int C, int Creal,
                                                           float* dw) {
  extern __shared__ __attribute__((aligned(16))) float row[];
  const int k = blockIdx.x;
  const int RS = R * S, RSC = RS * C;
  const size_t slab = (size_t)K * RSC;
  const int z0 = blockIdx.y * kWgFinishGroup, z1 = min(splits, z0 + kWgFinishGroup);
  for (int j = threadIdx.x; j < RSC; j += blockDim.x) {
    float v = 0.f;
    for (int z = z0; z < z1; ++z) v += ws[z * slab + (size_t)k * RSC + j];
    row[j] = v;
  }
  __syncthreads();
  float* out = dw + (size_t)k * Creal * RS;
  const bool single = gridDim.y == 1;
  // consecutive threads take consecutive channels: conflict-free LDS reads; each thread's
  // RS outputs are contiguous in dW (the lines are completed by neighbouring lanes in L2)
  for (int c = threadIdx.x; c < Creal; c += blockDim.x) {
    for (int rs = 0; rs < RS; ++rs) {
      const float v = row[rs * C + c];
      if (single) out[c * RS + rs] += v;
      else atomicAdd(out + c * RS + rs, v);
    }
  }
}

// Split-K finish for WGRAD into a [K][R][S][Cr] gradient: the GEMM row IS the gradient row, so
// this is a vectorised sum of the slabs — no transpose. blockIdx.y = group of kWgFinishGroupKrsc
// slabs (fixed order inside a group); several groups combine with atomics.
constexpr int kWgFinishGroupKrsc = 16;
__global__ __launch_bounds__(256) void wgrad_finish_krsc_kernel(const float* __restrict__ ws,
                                                                int splits, int K, int RS, int C,
                                                                int Creal, float* __restrict__ dw) {
  const size_t slab = (size_t)K * RS * C;
  const size_t n4 = slab / 4;
  const int z0 = blockIdx.y * kWgFinishGroupKrsc, z1 = min(splits, z0 + kWgFinishGroupKrsc);
  const bool single = gridDim.y == 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(ws + z0 * slab)[i];
    for (int z = z0 + 1; z < z1; ++z) {
      const float4 a = reinterpret_cast<const float4*>(ws + z * slab)[i];
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
    if (Creal == C) {
      if (single) {
        float4* o = reinterpret_cast<float4*>(dw) + i;
        float4 d = *o;
        d.x += v.x; d.y += v.y; d.z += v.z; d.w += v.w;
        *o = d;
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) unsafeAtomicAdd(dw + i * 4 + t, vv[t]);
      }
    } else {  // channel-padded input layer: drop the pad channels
      const size_t e = i * 4;
      const int c = (int)(e % C);
      const size_t krs = e / C;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (c + t >= Creal) continue;
        if (single) dw[krs * Creal + c + t] += vv[t];
        else unsafeAtomicAdd(dw + krs * Creal + c + t, vv[t]);
      }
    }
  }
}

}  // namespace ddp_amd

// ------------------------------- host launcher -------------------------------
using namespace ddp_amd;

constexpr int kMaxAtomicSplits = 32;

// Split-K factor for a tile config: aim for >= 2 workgroups per CU, keep >= 4 k-steps per
// split, fit the slab workspace.
static int pick_splits(int tiles, int ksteps, size_t slab, const ConvArgs& a, size_t ws_elems) {
  if (a.splits > 0) return std::max(1, std::min(a.splits, ksteps));

  if (a.ws == nullptr) return 1;
  int s = (512 + tiles - 1) / tiles;
  s = std::max(1, std::min(s, ksteps / 4));
  s = (int)std::min<size_t>((size_t)s, std::max<size_t>(1, ws_elems / slab));
  return s;
}

// Rough cost model (arbitrary units): MFMA work / (tile efficiency x chip fill) + split slab
// traffic. Tile efficiency reflects LDS-bytes-per-MFMA of the 2x2-wave tile; fill = fraction of
// the 256 CUs x resident blocks that the grid occupies.
static double tile_cost(int BM, int BN, const ConvArgs& a, size_t ws_elems, int* splits_out) {
  const int tiles = ((a.Mg + BM - 1) / BM) * ((a.Ng + BN - 1) / BN);
  const int ksteps = (a.Kg + 63) / 64;
  const size_t slab = (size_t)a.Mg * a.Ng;
  const int splits = pick_splits(tiles, ksteps, slab, a, ws_elems);
  *splits_out = splits;
  const double eff = (BM == 128 && BN == 128) ? 1.0 : ((BM == 64 && BN == 64) ? 0.55 : 0.8);
  const int resident = (BM == 128 && BN == 128) ? 2 : ((BM == 64 && BN == 64) ? 4 : 3);
  const double blocks = (double)tiles * splits;
  const double fill = std::min(1.0, blocks / (256.0 * resident));
  // padded work actually issued
  const double work = (double)tiles * BM * BN * ksteps * 64.0;
  const double t_mfma = work / (eff * fill) / 1.0e15 * 2.0;
  // slab write + read at ~4 TB/s plus the finish launch (~3 us); atomics: one RMW per element
  // per split, no finish pass
  double t_split = 0.0;
  if (splits > 1)
    t_split = (a.wg_atomic && splits <= kMaxAtomicSplits) ? 4.0 * splits * (double)slab / 1.3e12
                          : 8.0 * splits * (double)slab / 4.0e12 + 3.0e-6;
  return t_mfma + t_split;
}

template <int MODE, int BM, int BN>
static void launch_cfg(ConvArgs& a, int splits, hipStream_t st) {
  constexpr int BK = 64;
  const int tiles = ((a.Mg + BM - 1) / BM) * ((a.Ng + BN - 1) / BN);
  const int ksteps = (a.Kg + BK - 1) / BK;
  const int per = (ksteps + splits - 1) / splits;
  splits = (ksteps + per - 1) / per;
  a.splits = splits;
  a.ksteps_per_split = per;
  // same-address fp32 atomics serialise: beyond kMaxAtomicSplits partial sums per element the
  // slab + grouped-finish reduction is cheaper
  if (a.wg_atomic && splits > kMaxAtomicSplits) a.wg_atomic = 0;
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((conv_igemm_kernel<MODE, BM, BN>), grid, dim3(256), 0, st, a);
  if (splits == 1) return;
  if (MODE == MODE_WGRAD && a.wg_atomic) return;
  if (MODE == MODE_WGRAD && a.g.wkrsc) {
    const size_t n4 = (size_t)a.Mg * a.Ng / 4;
    const int groups = (splits + kWgFinishGroupKrsc - 1) / kWgFinishGroupKrsc;
    const int bx = (int)std::min<size_t>((n4 + 255) / 256, std::max(1, 2048 / groups));
    hipLaunchKernelGGL(wgrad_finish_krsc_kernel, dim3(bx, groups), dim3(256), 0, st, a.ws, splits,
                       a.g.K, a.g.R * a.g.S, a.g.C, a.g.Creal, a.dw);
  } else if (MODE == MODE_WGRAD) {
    const int groups = (splits + kWgFinishGroup - 1) / kWgFinishGroup;
    const size_t lds = sizeof(float) * a.g.R * a.g.S * a.g.C;
    hipLaunchKernelGGL(wgrad_finish_kernel, dim3(a.g.K, groups), dim3(256), lds, st, a.ws, splits,
                       a.g.K, a.g.R, a.g.S, a.g.C, a.g.Creal, a.dw);
  } else {
    const int G = a.Ng / 8;
    const int Gb = G < 256 ? G : 256;
    const int chunks = (G + Gb - 1) / Gb;
    const int rows_per_block = std::max(1, 256 / Gb);
    // ~2 rows per thread: enough workgroups in flight for a bandwidth-bound pass
    int bx = (a.Mg + rows_per_block * 2 - 1) / (rows_per_block * 2);
    bx = std::max(1, std::min(bx, 2048 / chunks + 1));
    hipLaunchKernelGGL(splitk_finish_kernel, dim3(bx, chunks), dim3(256), 0, st, a.ws, splits,
                       a.out, MODE == MODE_FWD ? a.bias : nullptr,
                       MODE == MODE_FWD ? a.stats : nullptr, a.Mg, a.Ng);
  }
}

template <int MODE>
static void launch_mode(ConvArgs& a, size_t ws_elems, hipStream_t st) {
  int sp[4];
  const double c[4] = {tile_cost(128, 128, a, ws_elems, &sp[0]), tile_cost(128, 64, a, ws_elems, &sp[1]),
                       tile_cost(64, 128, a, ws_elems, &sp[2]), tile_cost(64, 64, a, ws_elems, &sp[3])};
  int best = 0;
  for (int i = 1; i < 4; ++i)
    if (c[i] < c[best]) best = i;
  switch (best) {
    case 0: launch_cfg<MODE, 128, 128>(a, sp[0], st); break;
    case 1: launch_cfg<MODE, 128, 64>(a, sp[1], st); break;
    case 2: launch_cfg<MODE, 64, 128>(a, sp[2], st); break;
    default: launch_cfg<MODE, 64, 64>(a, sp[3], st); break;
  }
}

static int g_wgrad_atomic = 0;
extern "C" void ddp_conv_options(int wgrad_atomic) { g_wgrad_atomic = wgrad_atomic; }

extern "C" int ddp_conv_fwd(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                            void* y, float* stats, float* ws, size_t ws_elems, int splits,
                            hipStream_t st) {
  if (g->C % 8 || g->K % 8) return -1;
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)x;
  a.b = (const unsigned short*)wc;
  a.out = (unsigned short*)y;
  a.ws = ws;
  a.bias = bias;
  a.stats = stats;
  a.Mg = g->N * g->P * g->Q;
  a.Ng = g->K;
  a.Kg = g->R * g->S * g->C;
  a.splits = splits;
  launch_mode<MODE_FWD>(a, ws_elems, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_dgrad(const ConvGeom* g, const void* dy, const void* wt, void* dx,
                              float* ws, size_t ws_elems, int splits, hipStream_t st) {
  if (g->C % 8 || g->K % 8) return -1;
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)dy;
  a.b = (const unsigned short*)wt;
  a.out = (unsigned short*)dx;
  a.ws = ws;
  a.Mg = g->N * g->H * g->W;
  a.Ng = g->C;
  a.Kg = g->R * g->S * g->K;
  a.splits = splits;
  launch_mode<MODE_DGRAD>(a, ws_elems, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_wgrad(const ConvGeom* g, const void* dy, const void* x, float* dw,
                              float* ws, size_t ws_elems, int splits, hipStream_t st) {
  if (g->C % 8 || g->K % 8) return -1;
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)dy;
  a.b = (const unsigned short*)x;
  a.dw = dw;
  a.ws = ws;
  a.wg_atomic = g_wgrad_atomic;
  a.Mg = g->K;
  a.Ng = g->R * g->S * g->C;
  a.Kg = g->N * g->P * g->Q;
  a.splits = splits;
  launch_mode<MODE_WGRAD>(a, ws_elems, st);
  return (int)hipGetLastError();
}
