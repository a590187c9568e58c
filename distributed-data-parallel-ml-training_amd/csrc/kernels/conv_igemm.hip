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
//   dW [K][R][S][Creal]  fp32  weight gradient in the GPU arena layout (optim/arena.py), or
//      [K][Creal][R][S]        the standard layout (ConvGeom::wkrsc selects), accumulated
//
// GEMM views (rows x cols, reduction):
//   FWD   : M=N*P*Q, N=K,      red=R*S*C   A=im2col(x)          B=Wc
//   DGRAD : M=N*H*W, N=C,      red=R*S*K   A=col2im-gather(dy)  B=Wc read k-major
//           (strided convs: one stride-1 GEMM per output phase, see ConvArgs::phase)
//   WGRAD : M=K,     N=R*S*C,  red=N*P*Q   A=dy^T               B=im2col(x)^T
//
// Kernel structure (256 threads = 4 waves in 2x2, BK = 64):
//   * operands go global -> LDS by buffer_load_dwordx4 ... lds (no VGPR staging); padding and
//     tails are out-of-range buffer offsets that read as zero; the k-step's tap is uniform
//     over the block whenever the channel dimension is a multiple of 64, so the per-chunk cost
//     is one bounds test (cdna_hip_programming.md T14 / Guideline 15);
//   * double-buffered LDS: the DMA of k-step s+1 is in flight during the MFMAs of step s;
//   * FWD/DGRAD tiles are [row][k] with the 16-B chunk index XOR-swizzled by (row>>1)&7, read
//     by ds_read_b128 conflict-free (T2);
//   * WGRAD tiles keep the global order [m][channel] (m = the reduction index) and the MFMA
//     fragments are read with ds_read_b64_tr_b16 (gfx950 transposing LDS read, T10), chunk
//     XOR-swizzled by m so both 16-lane groups of a half-wave hit disjoint banks;
//   * MFMA operands are swapped (D^T = B^T A^T) so each lane owns one output row and four
//     consecutive columns: 8-B bf16 / 16-B fp32 stores in the epilogue;
//   * XCD-aware bijective tile order (T1); split-K writes plain fp32 slabs [split][M][N] that a
//     finish kernel reduces in a fixed order (deterministic; fp32-atomic variants — a "ticket
//     fixup" and WGRAD atomics into dW — measured 3-5x slower on MI355X and were removed in
//     round 4: profiles/r2_launch_reduction_ab.md);
//   * FWD epilogue adds the bias, rounds to bf16 and accumulates the per-channel BatchNorm
//     statistics of the rounded output (sum, sum of squares) — BN needs no separate stats pass.
#include "common.h"
#include "api.h"
#include "linear_blocks.h"
#include <algorithm>
#include <map>
#include <set>
#include <cstdlib>

namespace ddp_amd {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

// x / d for 0 <= x < 2^31 with a precomputed multiplier (d >= 1):  q = (mulhi(x, mul) + x) >> sh
struct FastDiv {
  unsigned mul;
  int sh;
};
__device__ __forceinline__ int fast_div(int x, FastDiv d) {
  return (int)((__umulhi((unsigned)x, d.mul) + (unsigned)x) >> d.sh);
}
// zero n16 16-byte chunks (the strided dgrad's untouched phases; see conv_dgrad_impl)
__global__ __launch_bounds__(256) void zero16_kernel(uint4* __restrict__ p, size_t n16) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256)
    p[i] = (uint4){0u, 0u, 0u, 0u};
}

__device__ __forceinline__ void ld8f_conv(const float* p, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

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
  // DGRAD of a strided conv, one output phase (pa, pb): GEMM rows are the input pixels
  // h = pa + stride*i, w = pb + stride*j (i < Hp, j < Wp); the only taps that reach them are
  // r = r0 + stride*t (t < Rt), s = s0 + stride*u (u < St), read from dy at (i + qa - t,
  // j + qb - u): a stride-1 problem with 1/stride^2 of the rows and taps (sub-pixel split).
  int phase;
  int pa, pb, Hp, Wp, r0, s0, Rt, St, qa, qb;
  int accumulate;            // DGRAD: dx = bf16(dx + result) (merges a second gradient branch)
  int a_bytes, b_bytes;      // operand sizes: buffer-resource bounds (reads past them give 0)
  FastDiv dPQ, dQ;           // row -> pixel: FWD / WGRAD P*Q, Q; DGRAD H*W, W (phase: Hp*Wp, Wp)
  int has_bnf;               // DGRAD (stride 1, no accumulate): accumulate the preceding
  BnBwdFuse bnf;             //   block's BatchNorm-backward sums in the epilogue (api.h)
  // FWD (host-side only, never read by a kernel): BatchNorm forward to fuse into the split-K
  // finish (splitk_finish_bnfwd_kernel) and where to report that it was fused
  const BnFwdFuse* bnfwd;
  int* bnfwd_done;
  // DGRAD with has_bnf (host-side only): the preceding block's BN backward to complete in the
  // split-K finish (splitk_finish_bnbwd_kernel) and where to report that it was
  const BnBwdApply* bnapply;
  int* bnapply_done;
  // FWD / DGRAD bf16 output through the LDS-staged epilogue (conv_igemm_body): full 16-B
  // stores of whole tile rows instead of 8-B fragments of 16 rows per instruction
  int epi_stage;
  // Dense 2x2 form of a 3x3 / s1 / p1 conv over 2x2 images (FWD, DGRAD; host: dense2x2_args):
  // every output pixel (p, q) sees every input pixel (h, w) through tap (h - p + 1, w - q + 1),
  // so the conv is ONE GEMM over whole images — FWD: [N] x [(h, w, c) = 4C] x [(p, q, k) = 4K],
  // DGRAD the transpose — with a block-structured weight W2[(p,q,k)][(h,w,c)] = Wc[k][tap][c]
  // that is never materialised: the B offsets pick the tap per (column tile, k-step). It skips
  // the 5 of 9 taps per pixel that hit padding (2.25x fewer MFMAs than the implicit GEMM), and
  // its NHWC output bytes are the standard ones (the split-K finish runs on the 3x3 view).
  int d2x2;                  // 1: g is the dense 1x1 view (N, 1, 1, 4C -> 4K), B = Wc [K][9][C]
  int d2C, d2K;              // the 3x3 conv's C and K
  int no_finish;             // host: launch the GEMM only (the caller runs the finish)
  // accumulate with a DEFERRED first branch (ResNet identity blocks): the branch's gradient
  // was never stored; it is acc_dy (the block output's gradient) through acc_mask (the
  // residual BatchNorm's ReLU bits, bn_act.hip BnArgs::mask; bit e of byte i = channel 8i + e
  // of the flat [rows][Ng] tensor) — dx = bf16(result + (bit ? acc_dy : 0)), dx never read
  const unsigned short* acc_dy;
  const unsigned char* acc_mask;
  // WGRAD without split-K (its epilogue owns complete gradient elements) inside the backward
  // pair launch, SGD in the backward (TrainStep, one GPU): the epilogue applies the update to
  // the fp32 master + momentum instead of storing the gradient (sgd.p != nullptr). The bf16
  // operand copy is NOT written here — the pair's DGRAD half is still reading it — but by the
  // step's SGD launch (pack-only items, optim.hip item 5).
  SgdFuse sgd;
  // WGRAD, pixel-major reduction (host: wgrad_pixmajor_ok): the reduction rows m are walked as
  // (pixel pq, 64 images) k-steps instead of 64 consecutive pixels. A column tile covers one tap
  // (C % BN == 0), so whether the tap reaches inside the image is uniform over a k-step, and the
  // k-steps whose pixel it pushes into the zero padding are skipped: 31 % of them on a 4x4
  // layer, 56 % on 2x2, 16 % on 8x8 (VGG-11). Every surviving row is in range, so the gathers need
  // no border test and take the k-step's position as a scalar offset (soffset) — no per-chunk
  // vector work at all. Needs N % 64 == 0; a tap's valid pixels form a rectangle, walked
  // row-major (ddp_conv_wgrad_pm_set: 1 = images of <= 64 pixels, 2 = any size).
  // FWD / DGRAD (host: rows_pixmajor_ok): the GEMM rows are ordered (pixel, image) and a row
  // tile holds one pixel of BM images, so the taps that reach into the padding are uniform over
  // the tile and their k-steps are skipped (31 % of them on a 4x4 layer, 16 % on 8x8); the A
  // gather is a scalar offset per k-step. The epilogues (and split-K slabs) store to the NHWC
  // rows, so every finish kernel is unchanged. Needs N % BM == 0 and R*S <= 32 (the valid taps
  // are a 32-bit mask); ddp_conv_rows_pm_set picks the images (<= 64 pixels or any, all convs
  // or R*S > 1 only).
  int pixmajor;
};

// the accumulating DGRAD's first-branch value of 4 / 8 consecutive channels starting at flat
// element e (stored dx, or the deferred masked gradient): bf16 values as stored
__device__ __forceinline__ uint2 acc_old4(const unsigned short* dx, const unsigned short* acc_dy,
                                          const unsigned char* acc_mask, size_t e) {
  if (!acc_mask) return *reinterpret_cast<const uint2*>(dx + e);
  uint2 v = *reinterpret_cast<const uint2*>(acc_dy + e);
  const unsigned mb = (unsigned)acc_mask[e >> 3] >> (e & 4);
  v.x &= ((mb & 1u) ? 0xFFFFu : 0u) | ((mb & 2u) ? 0xFFFF0000u : 0u);
  v.y &= ((mb & 4u) ? 0xFFFFu : 0u) | ((mb & 8u) ? 0xFFFF0000u : 0u);
  return v;
}
__device__ __forceinline__ u16x8 acc_old8(const unsigned short* dx, const unsigned short* acc_dy,
                                          const unsigned char* acc_mask, size_t e) {
  if (!acc_mask) return ld8(dx + e);
  u16x8 v = ld8(acc_dy + e);
  const unsigned mb = acc_mask[e >> 3];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = ((mb >> i) & 1u) ? v[i] : (unsigned short)0;
  return v;
}

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
  // A.dPQ / A.dQ divide by the row image size / width of the mode (prepare_cfg)
  if (MODE == MODE_FWD) {
    const int pq = g.P * g.Q;
    const int n = fast_div(row, A.dPQ), rem = row - n * pq;
    const int p = fast_div(rem, A.dQ), q = rem - p * g.Q;
    ri.base = n * g.H * g.W * g.C;
    ri.h0 = p * g.stride - g.pad;
    ri.w0 = q * g.stride - g.pad;
  } else if (A.phase) {
    const int hw = A.Hp * A.Wp;
    const int n = fast_div(row, A.dPQ), rem = row - n * hw;
    const int i = fast_div(rem, A.dQ), j = rem - i * A.Wp;
    ri.base = n * g.P * g.Q * g.K;
    ri.h0 = i + A.qa;
    ri.w0 = j + A.qb;
  } else {
    const int hw = g.H * g.W;
    const int n = fast_div(row, A.dPQ), rem = row - n * hw;
    const int h = fast_div(rem, A.dQ), w = rem - h * g.W;
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
// Logical-chunk correction of DMA chunk i relative to chunk 0 of the same thread in an [m][NCOL]
// tile: chunk i sits 2048 / NCOL rows further down. For NCOL <= 128 that step (>= 16 rows) keeps
// every bit mc_swz reads; at NCOL = 256 it is 8 rows, which flips bit 3 of m on odd i -> the
// swizzle flips chunk bit 3. (The WGRAD B' gather keeps one tap decomposition per thread and so
// still requires NCOL <= 128: WGRAD BN = 256 tiles are refused by the launcher.)
template <int NCOL>
__device__ __forceinline__ int swz_row_step(int i) {
  return NCOL >= 256 ? ((i & 1) << 3) : 0;
}
template <int NCOL>
__device__ __forceinline__ int mc_off(int m, int col) {
  return m * NCOL + (((col >> 3) ^ mc_swz<NCOL>(m)) << 3) + (col & 7);
}

// Buffer resource over a tensor (raw, stride 0): offsets >= num_records read as zero.
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma_buf(__amdgpu_buffer_rsrc_t rs, int byte_off,
                                        unsigned short* lds_wave_base) {
  // buffer_load_dwordx4 ... lds: LDS destination = wave-uniform base (M0) + lane * 16
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_wave_base, 16, byte_off, 0, 0, 0);
}
// ... with a wave-uniform part of the offset in soffset (an SGPR: no vector add per chunk)
__device__ __forceinline__ void dma_buf_s(__amdgpu_buffer_rsrc_t rs, int byte_off, int soff,
                                          unsigned short* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_wave_base, 16, byte_off,
                                           __builtin_amdgcn_readfirstlane(soff), 0, 0);
}

// LDS-DMA completion + workgroup barrier without the vmcnt(0) that __syncthreads implies:
// waits until at most N of this wave's vector-memory ops are outstanding (the DMAs of the
// stages issued after the one about to be read), then s_barrier. The "memory" clobber keeps the
// compiler from moving LDS accesses across it.
template <int N>
__device__ __forceinline__ void wait_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// BNF (DGRAD only): the epilogue also accumulates the preceding block's BatchNorm-backward sums
// (ConvArgs::bnf) — a separate instantiation so the plain kernels keep their register budget
// LDS bytes of one (BM, BN, NST) tile ring (the kernels' single __shared__ array)
template <int BM, int BN, int NST>
struct ConvSmem {
  static constexpr int elems = NST * (BM + BN) * 64;
};

// The GEMM body. ``bid`` / ``nblk`` stand for blockIdx.x / gridDim.x, so a grouped launch
// (conv_bwd_pair_kernel: the DGRAD and WGRAD GEMMs of one layer in ONE launch) can hand each
// problem its own block range. ``smem`` = the launching kernel's single LDS array.
// SGDM (WGRAD, backward pair only): the unsplit epilogue applies SGD to the master
// (ConvArgs::sgd) — a template switch so the other WGRAD launches keep their code
template <int MODE, int BM, int BN, int NST, int BNF = 0, bool XSTAT = false, bool SGDM = false>
__device__ __forceinline__ void conv_igemm_body(const ConvArgs& args, unsigned short* smem,
                                                const int bid, const int nblk) {
  constexpr int BK = 64;
  constexpr int WTM = BM / 2, WTN = BN / 2;
  // BNF: 0 none, 1 = the preceding block is pooled (generic epilogue, window-argmax routing),
  // 2 = no pool (lean epilogue, same row offsets as the output). The generic epilogue also
  // serves BNF 2 on 64x64 tiles, which never take the lean path.
  constexpr bool kOldBnf = BNF == 1 || (BNF == 2 && BM == 64 && BN == 64);
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = BM * BK / 8 / 256;  // 16-B chunks per thread per tile
  constexpr int CB = BN * BK / 8 / 256;
  constexpr int TILE_A = BM * BK, TILE_B = BN * BK;
  constexpr int STAGE = TILE_A + TILE_B;
  static_assert(CA >= 1 && CB >= 1, "tile too small for 256 threads");
  static_assert(NST >= 2 && NST <= 4, "2..4 LDS stages");

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  DDP_DEVICE_CHECK(blockDim.x == 256 && args.g.C % 8 == 0 && args.g.K % 8 == 0);
  DDP_DEVICE_CHECK(args.splits >= 1 && args.ksteps_per_split >= 1);

  // Persistent work loop: item = (split z, tile); a block walks items bid, +nblk, ...
  // and prefetches the first k-step of its NEXT item while it finishes (last MFMAs + epilogue)
  // the current one, so short-K tiles do not pay the DMA latency once per tile.
  const int tiles_n = (args.Ng + BN - 1) / BN;
  const int tiles_m = (args.Mg + BM - 1) / BM;
  const int tiles = tiles_m * tiles_n;
  const int nitems = tiles * args.splits;
  const int ksteps = (args.Kg + BK - 1) / BK;

  f32x4 acc[TM][TN];
  const ConvGeom& gg = args.g;

  // ---------------- per-thread gather state (index math hoisted out of the k-loop) ----------------
  // Operands are fetched with buffer_load_dwordx4 ... lds (LDS-DMA through a buffer resource):
  // an out-of-range byte offset returns zeros, so padding / tails cost one v_cndmask to the
  // kOOB sentinel instead of a pointer select, and all offsets are 32-bit.
  // FWD/DGRAD: DMA chunk c = tid + 256 i lands at LDS byte 16 c = row (tid>>3)+32i, physical
  // chunk tid&7; it must carry LOGICAL chunk lc = (tid&7) ^ ((row>>1)&7) = constant per thread.
  // WGRAD: row = m (reduction), physical chunk tid % (BX/8), logical = phys ^ swz(m) (constant).
  constexpr int NA = (MODE != MODE_WGRAD) ? CA : 1;
  int a_off[CA];         // FWD/DGRAD: byte offset of the row's (tap 0) pixel + lcA*8 channels
                         // WGRAD: byte offset of (m-row within the k-step, kout) or kOOB
  int a_h0[NA], a_w0[NA];
  int b_off[CB];         // FWD/DGRAD: byte offset of B row + lcB*8 (kOOB past Ng)
  int kr = 0, ks_ = 0, kc = 0;  // slow path: (r, s, c) of this thread's chunk; fast path: uniform
  KInfo xk;              // WGRAD: (r,s,c) of this thread's B' column group
  int xk_same = 0;       // WGRAD "same" conv: byte offset of tap (r,s) channel c relative to m
  // WGRAD "same" conv (stride 1, P == H, Q == W): the B' gather walks the reduction rows m of
  // each chunk 64 at a time, so its pixel (p, q) = ((m mod PQ) / Q, m mod Q) is carried from
  // k-step to k-step with adds and one conditional wrap each (no per-k-step divides or
  // multiplies: those made this gather VALU-bound, ~30 integer ops incl. 4-5 quarter-rate
  // multiplies per 16-B chunk). b_off[i] = byte offset of the chunk's (m, tap, c) in x.
  int wp[CB], wq[CB];
  int w_rr = 0, w_ss = 0, w_lim = 0;  // tap offsets r - pad, s - pad; b_off bound (m < Kg)
  const bool wsame = MODE == MODE_WGRAD && gg.stride == 1 && gg.P == gg.H && gg.Q == gg.W;
  const int w_dq = wsame ? BK % gg.Q : 0;                 // q advance per k-step
  const int w_dp = wsame ? (BK / gg.Q) % gg.P : 0;        // p advance per k-step (mod P)
  const int w_dm = wsame ? 2 * BK * gg.C : 0;             // byte advance per k-step
  // pixel-major WGRAD (ConvArgs::pixmajor): the k-step's (image block n0, pixel pq) and the
  // tile's tap (pm_r, pm_s), all uniform; the pixels the tap keeps inside the image are the
  // rectangle [p_lo, p_hi) x [pm_qlo, pm_qhi), walked row-major from (pm_p, pm_q)
  const bool pm = MODE == MODE_WGRAD && args.pixmajor;
  // pixel-major FWD / DGRAD rows: the item's pixel, first image and first row; the pixel's
  // valid taps and the k-step's tap
  const bool pmr = MODE != MODE_WGRAD && args.pixmajor;
  int pmr_pq = 0, pmr_n0 = 0, pmr_row0 = 0, pmr_t = 0;
  unsigned pmr_mask = 0;
  int pm_p = 0, pm_q = 0, pm_qlo = 0, pm_qhi = 0, pm_n0 = 0, pm_r = 0, pm_s = 0;
  int row0 = 0, col0 = 0, zsplit = 0, ks_begin = 0, ks_end = 0, cur_tile = 0;
  int d2pos = 0;         // dense 2x2: the column tile's output pixel (FWD) / input pixel (DGRAD)
  const bool phase = MODE == MODE_DGRAD && args.phase;
  const int Sdec = phase ? args.St : gg.S;  // taps per kernel row in the reduction index
  const int cdim = MODE == MODE_FWD ? gg.C : gg.K;
  // k-step = one tap x 64 channels (uniform over the block) when the channel dim is a multiple
  // of 64; otherwise (C = 8 input layers, K = 32 tests) every chunk decodes its own tap
  const bool fast = MODE != MODE_WGRAD && (cdim % BK) == 0;
  const int lcA = (MODE != MODE_WGRAD) ? ((tid & 7) ^ ((tid >> 4) & 7))
                                       : ((tid % (BM / 8)) ^ mc_swz<BM>(tid / (BM / 8)));
  // B operand: FWD reads Wc [K][RSC] k-contiguous into a [col][k] tile; DGRAD and WGRAD fill a
  // k-major [k][col] tile (DGRAD straight from Wc: 8 consecutive input channels of one output
  // channel and tap per chunk — no transposed weight copy) read with ds_read_b64_tr_b16
  constexpr bool BKM = MODE != MODE_FWD;
  const int lcB = !BKM ? lcA : ((tid % (BN / 8)) ^ mc_swz<BN>(tid / (BN / 8)));
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(args.a, args.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(args.b, args.b_bytes);

  auto setup = [&](int item) {
    zsplit = item / tiles;
    const int tile = xcd_remap(item - zsplit * tiles, tiles);
    cur_tile = tile;
    // column tiles fastest: the run of consecutive tiles xcd_remap gives one XCD shares an
    // A-row slice in its L2 (row-tiles-fastest measured slower: VGG-11 b256 0.854 vs 0.835 ms,
    // ResNet-50 26.84 vs 26.41 ms, same box; tools/gpu/r4m.sh)
    const int tm = tile / tiles_n;
    const int tn = tile - tm * tiles_n;
    row0 = tm * BM;
    col0 = tn * BN;
    ks_begin = zsplit * args.ksteps_per_split;
    ks_end = min(ksteps, ks_begin + args.ksteps_per_split);
    if (MODE != MODE_WGRAD) {
      if (pmr) {
        // row (pq, n): the tile's pixel and images; per chunk only the row's image stride
        pmr_pq = row0 / gg.N;
        pmr_n0 = row0 - pmr_pq * gg.N;
        pmr_row0 = row0;
        const int img = MODE == MODE_FWD ? gg.H * gg.W * gg.C : gg.P * gg.Q * gg.K;
#pragma unroll
        for (int i = 0; i < CA; ++i) a_off[i] = 2 * (((tid >> 3) + 32 * i) * img + lcA * 8);
      } else {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
          const RowInfo ri = row_info<MODE>(args, row0 + (tid >> 3) + 32 * i);
          a_h0[i] = ri.h0;
          a_w0[i] = ri.w0;
          const int e = (MODE == MODE_FWD) ? ri.base + (ri.h0 * gg.W + ri.w0) * gg.C
                                           : ri.base + (ri.h0 * gg.Q + ri.w0) * gg.K;
          a_off[i] = 2 * (e + (fast ? lcA * 8 : 0));
        }
      }
      if (MODE == MODE_FWD && args.d2x2) {
        // dense 2x2: column (p, q, k) reads Wc row k; the tap follows (p, q) and the k-step
        d2pos = col0 / args.d2K;
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const int col = col0 + (tid >> 3) + 32 * i;
          b_off[i] = col < args.Ng ? 2 * ((col - d2pos * args.d2K) * 9 * args.d2C + lcB * 8)
                                   : (int)kOOB;
        }
      } else if (MODE == MODE_FWD) {
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const int col = col0 + (tid >> 3) + 32 * i;
          b_off[i] = col < args.Ng ? 2 * (col * args.Kg + lcB * 8) : (int)kOOB;
        }
      } else if (args.d2x2) {
        // dense 2x2 DGRAD: column (h, w, c) = channel c of Wc rows k (the k-step's reduction
        // rows (p, q, k)), tap from (h, w) and the k-step's (p, q)
        d2pos = col0 / args.d2C;
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const int col = col0 + (lcB ^ swz_row_step<BN>(i)) * 8;
          b_off[i] = col < args.Ng ? 2 * (((tid + i * 256) / (BN / 8)) * 9 * args.d2C + col -
                                          d2pos * args.d2C)
                                   : (int)kOOB;
        }
      } else {  // DGRAD: row m of the k-step = output channel kc + m, columns = input channels
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          // chunk i lands on row m + (256 / (BN/8)) i; at BN = 256 that is m + 8 i, whose swizzle
          // differs from row m's in bit 3 (mc_swz): the logical chunk follows the row
          const int col = col0 + (lcB ^ swz_row_step<BN>(i)) * 8;
          b_off[i] = col < args.Ng ? 2 * (((tid + i * 256) / (BN / 8)) * gg.R * gg.S * gg.C + col)
                                   : (int)kOOB;
        }
      }
      if (pmr) {
        // the taps that keep the tile's pixel inside the image; this split's share of their
        // k-steps; the first one's tap and channel block
        const int pp = pmr_pq / gg.Q, qq = pmr_pq - pp * gg.Q, kb = cdim / BK;
        unsigned m = 0;
        for (int r = 0; r < gg.R; ++r)
          for (int s2 = 0; s2 < gg.S; ++s2) {
            const bool ok = MODE == MODE_FWD
                ? (unsigned)(pp + r - gg.pad) < (unsigned)gg.H && (unsigned)(qq + s2 - gg.pad) < (unsigned)gg.W
                : (unsigned)(pp - r + gg.pad) < (unsigned)gg.P && (unsigned)(qq - s2 + gg.pad) < (unsigned)gg.Q;
            if (ok) m |= 1u << (r * gg.S + s2);
          }
        pmr_mask = m;
        const int V = __builtin_popcount(m) * kb;
        const int per = (V + args.splits - 1) / args.splits;
        ks_begin = min(V, zsplit * per);
        ks_end = min(V, ks_begin + per);
        int jv = ks_begin / kb;
        unsigned mm = m;
        for (; jv > 0 && mm; --jv) mm &= mm - 1;
        pmr_t = mm ? __builtin_ctz(mm) : 0;
        kc = (ks_begin - (ks_begin / kb) * kb) * BK;
        kr = pmr_t / gg.S;
        ks_ = pmr_t - kr * gg.S;
      } else {
        // decomposition of the first reduction index (fast: of the k-step; slow: of the chunk)
        const int kk = ks_begin * BK + (fast ? 0 : lcA * 8);
        const int rs = kk / cdim;
        kc = kk - rs * cdim;
        kr = rs / Sdec;
        ks_ = rs - kr * Sdec;
      }
    } else {
      constexpr int NCA = BM / 8;
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int kout = row0 + (lcA ^ swz_row_step<BM>(i)) * 8;  // (BM = 256: see DGRAD's B)
        a_off[i] = kout < args.Mg ? 2 * (((tid + i * 256) / NCA) * gg.K + kout) : (int)kOOB;
      }
      const int j = col0 + lcB * 8;
      const int rs = j / gg.C;
      xk.c = j - rs * gg.C;
      xk.r = rs / gg.S;
      xk.s = rs - xk.r * gg.S;
      xk.ok = j < args.Ng;
      if (pm) {
        // one tap per column tile: its valid pixels, this split's share of the valid k-steps
        const int t = col0 / gg.C;
        pm_r = t / gg.S;
        pm_s = t - pm_r * gg.S;
        // the pixels (p, q) with (p + r - pad, q + s - pad) inside the image: a rectangle
        const int PQ = gg.P * gg.Q, nb = gg.N / BK;
        const int p_lo = max(0, gg.pad - pm_r), p_hi = min(gg.P, gg.H + gg.pad - pm_r);
        pm_qlo = max(0, gg.pad - pm_s);
        pm_qhi = min(gg.Q, gg.W + gg.pad - pm_s);
        const int nq = max(0, pm_qhi - pm_qlo);
        const int V = max(0, p_hi - p_lo) * nq * nb;
        const int per = (V + args.splits - 1) / args.splits;
        ks_begin = min(V, zsplit * per);
        ks_end = min(V, ks_begin + per);
        // the first k-step's pixel: the (ks_begin / nb)-th of the rectangle, row-major
        const int jv = ks_begin / nb;
        pm_p = p_lo + (nq ? jv / nq : 0);
        pm_q = pm_qlo + (nq ? jv - (jv / nq) * nq : 0);
        pm_n0 = (ks_begin - jv * nb) * BK;
        constexpr int NCA = BM / 8;
        constexpr int NCB = BN / 8;
#pragma unroll
        for (int i = 0; i < CA; ++i) {  // dy[(n0 + row) * PQ + pq][kout]
          const int kout = row0 + (lcA ^ swz_row_step<BM>(i)) * 8;
          a_off[i] = kout < args.Mg ? 2 * (((tid + i * 256) / NCA) * PQ * gg.K + kout) : (int)kOOB;
        }
#pragma unroll
        for (int i = 0; i < CB; ++i)    // x[n0 + row][p + r - pad][q + s - pad][c]
          b_off[i] = 2 * (((tid + i * 256) / NCB) * gg.H * gg.W * gg.C + (j - t * gg.C));
      }
      if (!xk.ok) xk.r = -(1 << 20);  // every border test fails -> zeros
      xk_same = xk.ok ? 2 * (((xk.r - gg.pad) * gg.W + (xk.s - gg.pad)) * gg.C + xk.c) : 0;
      if (wsame && !pm) {
        constexpr int NCB = BN / 8;
        const int pq = gg.P * gg.Q;
        w_rr = xk.r - gg.pad;
        w_ss = xk.s - gg.pad;
        w_lim = args.Kg * (2 * gg.C) + xk_same;
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const int m = ks_begin * BK + (tid + i * 256) / NCB;
          const int rem = m % pq;
          wp[i] = rem / gg.Q;
          wq[i] = rem - wp[i] * gg.Q;
          b_off[i] = m * (2 * gg.C) + xk_same;
        }
      }
    }
  };

  // issue the LDS-DMA of k-step ks into buffer buf (and advance the incremental k state)
  auto issue = [&](int ks, int buf) {
    unsigned short* As = smem + buf * STAGE;
    unsigned short* Bs = As + TILE_A;
    const int k0 = ks * BK;
    if (MODE != MODE_WGRAD && pmr) {
      const int pp = pmr_pq / gg.Q, qq = pmr_pq - pp * gg.Q;
      const int hh = MODE == MODE_FWD ? pp + kr - gg.pad : pp - kr + gg.pad;
      const int ww = MODE == MODE_FWD ? qq + ks_ - gg.pad : qq - ks_ + gg.pad;
      const int sa = MODE == MODE_FWD ? 2 * (((pmr_n0 * gg.H + hh) * gg.W + ww) * cdim + kc)
                                      : 2 * (((pmr_n0 * gg.P + hh) * gg.Q + ww) * cdim + kc);
#pragma unroll
      for (int i = 0; i < CA; ++i) dma_buf_s(rsA, a_off[i], sa, As + (wid * 64 + 256 * i) * 8);
      const int boff = MODE == MODE_FWD ? 2 * (pmr_t * cdim + kc)
                                        : 2 * ((kc * gg.R * gg.S + kr * gg.S + ks_) * gg.C);
#pragma unroll
      for (int i = 0; i < CB; ++i) dma_buf(rsB, b_off[i] + boff, Bs + (wid * 64 + 256 * i) * 8);
      kc += BK;
      if (kc == cdim) {  // next valid tap
        kc = 0;
        const unsigned rest = pmr_mask & ~((2u << pmr_t) - 1u);
        pmr_t = rest ? __builtin_ctz(rest) : pmr_t;
        kr = pmr_t / gg.S;
        ks_ = pmr_t - kr * gg.S;
      }
    } else if (MODE != MODE_WGRAD) {
      const int W_ = MODE == MODE_FWD ? gg.W : gg.Q;
      if (fast) {
        // uniform tap (kr, ks_) and channel block kc: the per-chunk work is one bounds test
        const int tap = 2 * (MODE == MODE_FWD ? (kr * W_ + ks_) * cdim + kc : kc - (kr * W_ + ks_) * cdim);
#pragma unroll
        for (int i = 0; i < CA; ++i) {
          bool ok;
          if (MODE == MODE_FWD)
            ok = (unsigned)(a_h0[i] + kr) < (unsigned)gg.H && (unsigned)(a_w0[i] + ks_) < (unsigned)gg.W;
          else
            ok = (unsigned)(a_h0[i] - kr) < (unsigned)gg.P && (unsigned)(a_w0[i] - ks_) < (unsigned)gg.Q;
          dma_buf(rsA, ok ? a_off[i] + tap : (int)kOOB, As + (wid * 64 + 256 * i) * 8);
        }
        int boff;
        if (args.d2x2) {
          // FWD: k-step = input pixel hw, channels c0..; DGRAD: k-step = output pixel pq,
          // channels k0..; the column tile fixed the other pixel (d2pos)
          const int pix = MODE == MODE_FWD ? kc / args.d2C : kc / args.d2K;
          const int ch = kc - pix * (MODE == MODE_FWD ? args.d2C : args.d2K);
          const int pq = MODE == MODE_FWD ? d2pos : pix, hw = MODE == MODE_FWD ? pix : d2pos;
          const int tap = ((hw >> 1) - (pq >> 1) + 1) * 3 + ((hw & 1) - (pq & 1) + 1);
          boff = MODE == MODE_FWD ? 2 * (tap * args.d2C + ch) : 2 * ((ch * 9 + tap) * args.d2C);
        } else if (MODE == MODE_FWD) {
          boff = 2 * k0;
        } else {  // Wc[kc + m][r][s][c]
          const int rr = phase ? args.r0 + gg.stride * kr : kr, ss = phase ? args.s0 + gg.stride * ks_ : ks_;
          boff = 2 * ((kc * gg.R * gg.S + rr * gg.S + ss) * gg.C);
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) dma_buf(rsB, b_off[i] + boff, Bs + (wid * 64 + 256 * i) * 8);
        kc += BK;
        if (kc == cdim) {
          kc = 0;
          if (++ks_ == Sdec) { ks_ = 0; ++kr; }
        }
      } else {
        const int kk = k0 + lcA * 8;
        const bool kok = kk < args.Kg;
        const int tap = 2 * (MODE == MODE_FWD ? (kr * W_ + ks_) * cdim + kc : kc - (kr * W_ + ks_) * cdim);
#pragma unroll
        for (int i = 0; i < CA; ++i) {
          bool ok;
          if (MODE == MODE_FWD)
            ok = (unsigned)(a_h0[i] + kr) < (unsigned)gg.H && (unsigned)(a_w0[i] + ks_) < (unsigned)gg.W;
          else
            ok = (unsigned)(a_h0[i] - kr) < (unsigned)gg.P && (unsigned)(a_w0[i] - ks_) < (unsigned)gg.Q;
          dma_buf(rsA, (kok && ok) ? a_off[i] + tap : (int)kOOB, As + (wid * 64 + 256 * i) * 8);
        }
        if (MODE == MODE_FWD) {
#pragma unroll
          for (int i = 0; i < CB; ++i)
            dma_buf(rsB, kok ? b_off[i] + 2 * k0 : (int)kOOB, Bs + (wid * 64 + 256 * i) * 8);
        } else {
          // DGRAD, K % 64 != 0: the k-step spans taps; decode every row's reduction index
          const int RSC = gg.R * gg.S * gg.C;
#pragma unroll
          for (int i = 0; i < CB; ++i) {
            const int m = (tid + i * 256) / (BN / 8);
            const int kkr = k0 + m;
            const int tap = kkr / gg.K, kout = kkr - tap * gg.K;
            const int tr = tap / Sdec, ts = tap - tr * Sdec;
            const int rr = phase ? args.r0 + gg.stride * tr : tr, ss = phase ? args.s0 + gg.stride * ts : ts;
            const int off = b_off[i] - 2 * m * RSC + 2 * ((kout * gg.R * gg.S + rr * gg.S + ss) * gg.C);
            dma_buf(rsB, (kkr < args.Kg && b_off[i] != (int)kOOB) ? off : (int)kOOB,
                    Bs + (wid * 64 + 256 * i) * 8);
          }
        }
        kc += BK;
        while (kc >= cdim) {
          kc -= cdim;
          if (++ks_ == Sdec) { ks_ = 0; ++kr; }
        }
      }
    } else {
      constexpr int NCB = BN / 8;
      if (pm) {  // (k-steps are issued in order: advance (n0, pq) after each)
        const int PQ = gg.P * gg.Q;
        const int sa = 2 * ((pm_n0 * PQ + pm_p * gg.Q + pm_q) * gg.K);
        const int sb = 2 * ((pm_n0 * gg.H + pm_p + pm_r - gg.pad) * gg.W + pm_q + pm_s - gg.pad) * gg.C;
#pragma unroll
        for (int i = 0; i < CA; ++i) dma_buf_s(rsA, a_off[i], sa, As + (wid * 64 + 256 * i) * 8);
#pragma unroll
        for (int i = 0; i < CB; ++i) dma_buf_s(rsB, b_off[i], sb, Bs + (wid * 64 + 256 * i) * 8);
        pm_n0 += BK;
        if (pm_n0 == gg.N) {
          pm_n0 = 0;
          if (++pm_q == pm_qhi) {
            pm_q = pm_qlo;
            ++pm_p;
          }
        }
        return;
      }
      const int ka = 2 * k0 * gg.K;
#pragma unroll
      for (int i = 0; i < CA; ++i)  // dy[m][kout]; m >= Kg lands past the buffer -> zeros
        dma_buf(rsA, a_off[i] + ka, As + (wid * 64 + 256 * i) * 8);
      // "same" convolution (stride 1, P == H, Q == W): the input pixel of output pixel m at tap
      // (r, s) is m + (r - pad) * W + (s - pad), so the offset is linear in m; only the border
      // test needs (p, q), carried from the previous k-step (wp / wq, set up per item)
      if (wsame) {
#pragma unroll
        for (int i = 0; i < CB; ++i) {  // x gather at pixel m for columns (r, s, c..c+7)
          const bool ok = b_off[i] < w_lim && (unsigned)(wp[i] + w_rr) < (unsigned)gg.H &&
                          (unsigned)(wq[i] + w_ss) < (unsigned)gg.W;
          dma_buf(rsB, ok ? b_off[i] : (int)kOOB, Bs + (wid * 64 + 256 * i) * 8);
          // m += 64 for the next k-step (k-steps are issued in order)
          b_off[i] += w_dm;
          int q = wq[i] + w_dq;
          const int cq = q >= gg.Q ? 1 : 0;
          q -= cq ? gg.Q : 0;
          int pp = wp[i] + w_dp + cq;
          pp -= pp >= gg.P ? gg.P : 0;
          wq[i] = q;
          wp[i] = pp;
        }
      } else {
#pragma unroll
        for (int i = 0; i < CB; ++i) {
          const int m = k0 + (tid + i * 256) / NCB;
          const int n = fast_div(m, args.dPQ);
          const int rem = m - n * (gg.P * gg.Q);
          const int p = fast_div(rem, args.dQ);
          const int q = rem - p * gg.Q;
          const int h = p * gg.stride - gg.pad + xk.r, w = q * gg.stride - gg.pad + xk.s;
          const bool ok = m < args.Kg && (unsigned)h < (unsigned)gg.H && (unsigned)w < (unsigned)gg.W;
          dma_buf(rsB, ok ? 2 * (((n * gg.H + h) * gg.W + w) * gg.C + xk.c) : (int)kOOB,
                  Bs + (wid * 64 + 256 * i) * 8);
        }
      }
    }
  };

  // fragment LDS offsets (elements), loop-invariant
  int fa_off[TM], fb_off[TN];
  {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int m0 = 8 * g + q;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa_off[i] = MODE != MODE_WGRAD ? rk_off(wm * WTM + i * 16 + (lane & 15), lane >> 4)
                                     : mc_off<BM>(m0, wm * WTM + i * 16 + 4 * p);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb_off[j] = !BKM ? rk_off(wn * WTN + j * 16 + (lane & 15), lane >> 4)
                       : mc_off<BN>(m0, wn * WTN + j * 16 + 4 * p);
  }

  // fragments of one 32-deep half of a k-step (kk = 0 / 32) from LDS buffer ``buf``
  auto load_frags = [&](int buf, int kk, bf16x8 (&fa)[TM], bf16x8 (&fb)[TN]) {
    const unsigned short* As = smem + buf * STAGE;
    const unsigned short* Bs = As + TILE_A;
    // [row][k] tiles: logical chunk kk/8 + (lane>>4); the XOR swizzle is linear in the chunk
    // index, so the kk = 32 read is the kk = 0 address with chunk bit 2 flipped.
    // [k][col] tiles: ds_read_b64_tr_b16 — lane 4q+p of each 16-lane group supplies row q,
    // columns 4p..4p+3; lane i receives column i of the 4 rows; two reads = 8 k-values.
    if (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(As + (fa_off[i] ^ (kk ? 32 : 0)));
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const unsigned short* base = As + fa_off[i] + kk * BM;
        v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
        v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * BM));
        const short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        fa[i] = __builtin_bit_cast(bf16x8, v);
      }
    }
    if (!BKM) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        fb[j] = *reinterpret_cast<const bf16x8*>(Bs + (fb_off[j] ^ (kk ? 32 : 0)));
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const unsigned short* base = Bs + fb_off[j] + kk * BN;
        v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
        v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * BN));
        const short8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        fb[j] = __builtin_bit_cast(bf16x8, v);
      }
    }
  };
  auto mma = [&](const bf16x8 (&fa)[TM], const bf16x8 (&fb)[TN]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        // operands swapped (D^T = B^T A^T): each lane ends up owning ONE output row and FOUR
        // consecutive output columns, so the epilogue stores 8 B (bf16) / 16 B (fp32) per lane
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
  };

  // ---------------- epilogue ----------------
  // FWD statistics of the LDS-staged epilogue, accumulated ACROSS the work items of one column
  // tile (a thread keeps its 8 channels for every item with the same col0) and added to the
  // replicas once per run of such items: with a capped grid (launch_gemm_t, kFwdStatGrid) a
  // block adds one partial sum per channel instead of one per tile — ResNet-50's 64->256 56x56
  // convs otherwise add 12544 x 2 KB = 26 MB of memory-side float atomics each.
  // (XSTAT only: the kernel instantiation of the capped-grid launches, launch_gemm_t — the
  // one-item-per-block launches keep per-item sums and no live running registers)
  constexpr int SCPR = BN / 8;  // the staged epilogue's 16-B chunks per tile row
  float run_s[XSTAT ? 8 : 1], run_ss[XSTAT ? 8 : 1];
#pragma unroll
  for (int e = 0; e < (XSTAT ? 8 : 1); ++e) { run_s[e] = 0.f; run_ss[e] = 0.f; }
  int run_col = -1;  // column tile the running sums belong to (uniform), -1: none
  auto flush_stats = [&](const int c0, float (&fs)[8], float (&fss)[8]) {
    // lanes l, l + CPR, ... of a wave share the chunk column: butterfly over them, then the four
    // waves meet in LDS (after every wave is done with the operand ring / the staged tile)
#pragma unroll
    for (int m = SCPR; m < 64; m *= 2)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        fs[e] += __shfl_xor(fs[e], m);
        fss[e] += __shfl_xor(fss[e], m);
      }
    __syncthreads();
    float* sl = reinterpret_cast<float*>(smem);  // [wave][2][BN]
    if (lane < SCPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sl[(wid * 2 + 0) * BN + lane * 8 + e] = fs[e];
        sl[(wid * 2 + 1) * BN + lane * 8 + e] = fss[e];
      }
    }
    __syncthreads();
    float* st = args.stats + stat_rep(bid) * 2 * args.Ng;  // spread contention
    for (int k = tid; k < 2 * BN; k += 256) {
      const int which = k / BN, cl = k - which * BN;
      if (c0 + cl >= args.Ng) continue;
      const float t = sl[(0 * 2 + which) * BN + cl] + sl[(1 * 2 + which) * BN + cl] +
                      sl[(2 * 2 + which) * BN + cl] + sl[(3 * 2 + which) * BN + cl];
      atomicAdd(st + which * args.Ng + c0 + cl, stat_val(t, bid));
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { fs[e] = 0.f; fss[e] = 0.f; }
  };

  // acc[i][j][v] = D[row0 + wm*WTM + i*16 + (lane&15)][col0 + wn*WTN + j*16 + 4*(lane>>4) + v]
  // Ng % 8 == 0 for every mode (C, K multiples of 8), so a lane's 4 columns are all valid or not.
  auto epilogue = [&](const int row0, const int col0, const int zs, const bool split) {
  const ConvGeom& g = args.g;
  float* slab = split ? args.ws + (size_t)zs * args.Mg * args.Ng : nullptr;
  const int rl = lane & 15, cq = 4 * (lane >> 4);
  float stat_s[TN][4], stat_ss[TN][4];
  // per-channel sums reduced in the epilogue: FWD = BatchNorm statistics of the output, DGRAD with
  // a BnBwdFuse = the preceding block's BatchNorm-backward sums
  const bool red = (MODE == MODE_FWD && !split && args.stats != nullptr) ||
                   (MODE == MODE_DGRAD && BNF && !split);
  // LDS-staged output (FWD, DGRAD incl. the accumulating second branch; no BN-backward
  // fusion): the MFMA layout gives each lane one row and 4 columns, so a direct store writes
  // 16 rows x 32 B per instruction — partial lines that run the big-output 1x1 convs at about
  // half the HBM write rate (tools/probes/epilogue_probe.py). Instead each wave row parks its
  // fp32 accumulators in the idle operand ring ([BM/2][BN] fp32, 16-B chunks XOR-swizzled by
  // row; two halves, so the ring needs BM*BN*2 bytes), then every thread stores whole 16-B bf16
  // chunks of 8 consecutive channels (a wave writes 64 x 16 B of 2-8 full rows), adding the
  // bias / the old dx and rounding exactly like the direct path (bit-identical output), and
  // accumulates the BatchNorm statistics of its fixed 8 channels on the way out.
  if (MODE != MODE_WGRAD && BNF == 0 && !(BM == 64 && BN == 64) && !split && args.epi_stage) {
    constexpr int HM = BM / 2;             // rows per half (= one wave row's WTM)
    constexpr int C4 = BN / 4;             // fp32 16-B chunks per staged row
    constexpr int CPR = BN / 8;            // bf16 16-B output chunks per tile row
    constexpr int RPP = 256 / CPR;         // tile rows per pass of the block
    constexpr int PASSES = HM / RPP;
    static_assert(HM % RPP == 0 && HM == WTM, "half tiles must cover whole passes");
    float* cf = reinterpret_cast<float*>(smem);  // launch_gemm_t sizes the ring >= BM*BN*2 B
    const int rl = lane & 15, cq = 4 * (lane >> 4);
    const int cc = tid % CPR;              // this thread's output chunk (8 channels)
    const int col = col0 + cc * 8;
    const bool cok = col < args.Ng;
    float bv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (MODE == MODE_FWD && args.bias && cok) ld8f_conv(args.bias + col, bv);
    float s[8], ss[8];  // this item's sums (XSTAT: the running sums instead)
#pragma unroll
    for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
    if constexpr (XSTAT) {
      if (MODE == MODE_FWD && red && run_col != col0) {  // a new column tile: settle the last one
        if (run_col >= 0) flush_stats(run_col, *reinterpret_cast<float(*)[8]>(run_s),
                                      *reinterpret_cast<float(*)[8]>(run_ss));
        run_col = col0;
      }
    }
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      __syncthreads();                     // ring idle (last MFMA reads / previous half stored)
      if (wm == h) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int c = wn * WTN + j * 16 + cq;
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int r = i * 16 + rl;
            *reinterpret_cast<f32x4*>(cf + r * BN + (((c >> 2) ^ (r & (C4 - 1))) << 2)) = acc[i][j];
          }
        }
      }
      __syncthreads();
#pragma unroll
      for (int p = 0; p < PASSES; ++p) {
        const int r = tid / CPR + p * RPP;
        const int row = row0 + h * HM + r;
        const f32x4 lo = *reinterpret_cast<const f32x4*>(cf + r * BN + (((2 * cc) ^ (r & (C4 - 1))) << 2));
        const f32x4 hi = *reinterpret_cast<const f32x4*>(cf + r * BN + (((2 * cc + 1) ^ (r & (C4 - 1))) << 2));
        if (!cok || row >= args.Mg) continue;
        const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        size_t orow = row;
        if (phase) {  // phase-local row -> input pixel
          const int hw = args.Hp * args.Wp;
          const int n = fast_div(row, args.dPQ), rem = row - n * hw;
          const int pi = fast_div(rem, args.dQ), pj = rem - pi * args.Wp;
          orow = ((size_t)n * g.H + args.pa + g.stride * pi) * g.W + args.pb + g.stride * pj;
        } else if (pmr) {  // (pixel, image) row -> NHWC row
          orow = (size_t)(pmr_n0 + row - pmr_row0) * (g.P * g.Q) + pmr_pq;
        }
        unsigned short* dst = args.out + orow * args.Ng + col;
        u16x8 o;
        if (MODE == MODE_DGRAD && args.accumulate) {  // dx += (second gradient branch)
          const u16x8 old = acc_old8(args.out, args.acc_dy, args.acc_mask, orow * args.Ng + col);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e] + bf2f(old[e]));
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = f2bf(v[e] + bv[e]);
        }
        st8(dst, o);
        if (MODE == MODE_FWD && red) {  // statistics of the stored (bf16-rounded) values
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float rv = bf2f(o[e]);
            if constexpr (XSTAT) {
              run_s[e] += rv;
              run_ss[e] += rv * rv;
            } else {
              s[e] += rv;
              ss[e] += rv * rv;
            }
          }
        }
      }
    }
    // (XSTAT: the running sums are added by the next column tile or after the last item)
    if (!XSTAT && MODE == MODE_FWD && red) flush_stats(col0, s, ss);
    return;
  }
  // the LDS operand ring is reused for the statistics hand-off: every wave must be done with it
  if (red) __syncthreads();
  // (not for 64x64 tiles: measured slower there — the VGG-11 forward convs, whose long
  // reductions hide the epilogue anyway — the generic path below keeps their codegen)
  // With a BnBwdFuse the preceding block's BatchNorm-backward sums ride along when that block
  // has no pool (its z has this output's shape: the same row offsets); pooled (VGG) fusions keep
  // the generic path, which routes through the window argmax.
  // (BNF 0 takes the LDS-staged path above, or the generic one below when it is switched off:
  // keeping this lean path out of those instantiations keeps them at 2 waves per SIMD)
  if (MODE != MODE_WGRAD && !(BM == 64 && BN == 64) && !split &&
      !(MODE == MODE_DGRAD && args.accumulate) && BNF == 2) {
    // Plain bf16 output (FWD, DGRAD overwriting dx). Short-reduction GEMMs (1x1 convs over
    // 64-128 channels: 1-2 k-steps) spend most of their VALU issue in the epilogue and the
    // gather setup, so: one row offset per (lane, i) computed up front (column groups are
    // immediate offsets), DPP row sums, and the statistics hand-off through LDS for both wave
    // rows, so no per-column sums stay live across the tile.
    const int cbase = col0 + wn * WTN + cq;
    const bool has_bias = MODE == MODE_FWD && args.bias != nullptr;
    int ro[TM];  // element offset of the lane's output row + cbase, -1 past Mg
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = row0 + wm * WTM + i * 16 + rl;
      int orow = row;
      if (phase) {  // phase-local row -> input pixel
        const int hw = args.Hp * args.Wp;  // dPQ / dQ = Hp*Wp / Wp for a phase GEMM
        const int n = fast_div(row, args.dPQ), rem = row - n * hw;
        const int pi = fast_div(rem, args.dQ), pj = rem - pi * args.Wp;
        orow = (n * g.H + args.pa + g.stride * pi) * g.W + args.pb + g.stride * pj;
      } else if (pmr) {  // (pixel, image) row -> NHWC row
        orow = (pmr_n0 + row - pmr_row0) * (g.P * g.Q) + pmr_pq;
      }
      ro[i] = row < args.Mg ? orow * args.Ng + cbase : -1;
    }
    float* sl = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (cbase + j * 16 >= args.Ng) continue;  // uniform over each 16-lane DPP row
      float4 bj = {0.f, 0.f, 0.f, 0.f};
      if (has_bias) bj = *reinterpret_cast<const float4*>(args.bias + cbase + j * 16);
      float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
      float4 bsc = {0.f, 0.f, 0.f, 0.f}, bsh = bsc, bmu = bsc, bis = bsc;
      if (MODE == MODE_DGRAD && BNF == 2 && red) {  // coefficients of the 4 channels ([6][C])
        const float* cf = args.bnf.coef + cbase + j * 16;
        bsc = *reinterpret_cast<const float4*>(cf + 0 * args.Ng);
        bsh = *reinterpret_cast<const float4*>(cf + 1 * args.Ng);
        bmu = *reinterpret_cast<const float4*>(cf + 2 * args.Ng);
        bis = *reinterpret_cast<const float4*>(cf + 3 * args.Ng);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if (ro[i] < 0) continue;
        const f32x4 v = acc[i][j];
        uint2 pk;
        pk.x = (unsigned)f2bf(v[0] + bj.x) | ((unsigned)f2bf(v[1] + bj.y) << 16);
        pk.y = (unsigned)f2bf(v[2] + bj.z) | ((unsigned)f2bf(v[3] + bj.w) << 16);
        *reinterpret_cast<uint2*>(args.out + ro[i] + j * 16) = pk;
        if (MODE == MODE_FWD && red) {  // statistics of the stored (bf16-rounded) values
          const float r0 = __uint_as_float(pk.x << 16), r1 = __uint_as_float(pk.x & 0xffff0000u);
          const float r2 = __uint_as_float(pk.y << 16), r3 = __uint_as_float(pk.y & 0xffff0000u);
          s[0] += r0; s[1] += r1; s[2] += r2; s[3] += r3;
          ss[0] += r0 * r0; ss[1] += r1 * r1; ss[2] += r2 * r2; ss[3] += r3 * r3;
        }
        if (MODE == MODE_DGRAD && BNF == 2 && red) {
          // this row's stored gradient flows through the preceding block's ReLU mask:
          // dy_bn; S1 += dy_bn, S2 += dy_bn * xhat (bn_act.hip bwd_compute, no pool)
          const uint2 zz = *reinterpret_cast<const uint2*>(args.bnf.z + ro[i] + j * 16);
          const float gv[4] = {__uint_as_float(pk.x << 16), __uint_as_float(pk.x & 0xffff0000u),
                               __uint_as_float(pk.y << 16), __uint_as_float(pk.y & 0xffff0000u)};
          const float zf[4] = {__uint_as_float(zz.x << 16), __uint_as_float(zz.x & 0xffff0000u),
                               __uint_as_float(zz.y << 16), __uint_as_float(zz.y & 0xffff0000u)};
          const float fsc[4] = {bsc.x, bsc.y, bsc.z, bsc.w}, fsh[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
          const float fmu[4] = {bmu.x, bmu.y, bmu.z, bmu.w}, fis[4] = {bis.x, bis.y, bis.z, bis.w};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const float y = zf[t] * fsc[t] + fsh[t];
            const float dyb = (args.bnf.relu && !(y > 0.f)) ? 0.f : gv[t];
            s[t] += dyb;
            ss[t] += dyb * ((zf[t] - fmu[t]) * fis[t]);
          }
        }
      }
      if (red) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s[t] = dpp_sum16(s[t]);
          ss[t] = dpp_sum16(ss[t]);
        }
        // LDS slot [wm][wn][j][lane>>4][8]
        float* slot = sl + ((((wm * 2 + wn) * TN + j) * 4 + (lane >> 4)) * 8);
        if (rl == 0) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            slot[t] = s[t];
            slot[4 + t] = ss[t];
          }
        }
      }
    }
    if (red) {
      __syncthreads();
      if (wm == 0 && rl == 0) {
        float* st = (MODE == MODE_FWD ? args.stats : args.bnf.sums) +
                    stat_rep(bid) * 2 * args.Ng;  // spread contention
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = cbase + j * 16;
          if (col >= args.Ng) continue;
          const float* s0 = sl + (((wn * TN + j) * 4 + (lane >> 4)) * 8);
          const float* s1 = sl + ((((2 + wn) * TN + j) * 4 + (lane >> 4)) * 8);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            atomicAdd(st + col + t, stat_val(s0[t] + s1[t], bid));
            atomicAdd(st + args.Ng + col + t, stat_val(s0[4 + t] + s1[4 + t], bid));
          }
        }
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + wn * WTN + j * 16 + cq;
    const bool cok = col < args.Ng;
    float4 bias = {0.f, 0.f, 0.f, 0.f};
    if (MODE == MODE_FWD && !split && args.bias && cok)
      bias = (float4){args.bias[col], args.bias[col + 1], args.bias[col + 2], args.bias[col + 3]};
    float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f};
    float4 bsc = {0.f, 0.f, 0.f, 0.f}, bsh = bsc, bmu = bsc, bis = bsc;
    if (MODE == MODE_DGRAD && kOldBnf && red && cok) {  // coefficients of the 4 channels ([6][C])
      const float* cf = args.bnf.coef;
      bsc = *reinterpret_cast<const float4*>(cf + 0 * args.Ng + col);
      bsh = *reinterpret_cast<const float4*>(cf + 1 * args.Ng + col);
      bmu = *reinterpret_cast<const float4*>(cf + 2 * args.Ng + col);
      bis = *reinterpret_cast<const float4*>(cf + 3 * args.Ng + col);
    }
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
      if (MODE == MODE_WGRAD && !split) {
        if (SGDM && g.wkrsc && g.Creal == g.C && args.sgd.p) {  // master-only SGD (ConvArgs::sgd)
          const size_t e = ((size_t)row * g.R * g.S + wrs) * g.C + wc;
          float4 pv = *reinterpret_cast<const float4*>(args.sgd.p + e);
          float4 bv = *reinterpret_cast<const float4*>(args.sgd.buf + e);
          const SgdFuse& h = args.sgd;
          pv.x = sgd_update1(pv.x, v[0], bv.x, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
          pv.y = sgd_update1(pv.y, v[1], bv.y, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
          pv.z = sgd_update1(pv.z, v[2], bv.z, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
          pv.w = sgd_update1(pv.w, v[3], bv.w, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
          *reinterpret_cast<float4*>(args.sgd.p + e) = pv;
          *reinterpret_cast<float4*>(args.sgd.buf + e) = bv;
        } else if (g.wkrsc && g.Creal == g.C) {
          float* d = args.dw + ((size_t)row * g.R * g.S + wrs) * g.C + wc;
          float4 o = *reinterpret_cast<float4*>(d);
          o.x += v[0]; o.y += v[1]; o.z += v[2]; o.w += v[3];
          *reinterpret_cast<float4*>(d) = o;
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (wc + t >= g.Creal) break;
            const size_t di = g.wkrsc ? ((size_t)row * g.R * g.S + wrs) * g.Creal + wc + t
                                      : ((size_t)row * g.Creal + wc + t) * g.R * g.S + wrs;
            args.dw[di] += v[t];
          }
        }
      } else if (split) {
        // (pixel-major rows: the slab takes the NHWC row, so every finish kernel is unchanged)
        const size_t srow = pmr ? (size_t)(pmr_n0 + row - pmr_row0) * (g.P * g.Q) + pmr_pq : (size_t)row;
        *reinterpret_cast<float4*>(slab + srow * args.Ng + col) = (float4){v[0], v[1], v[2], v[3]};
      } else {
        const unsigned short h0 = f2bf(v[0] + bias.x), h1 = f2bf(v[1] + bias.y);
        const unsigned short h2 = f2bf(v[2] + bias.z), h3 = f2bf(v[3] + bias.w);
        uint2 pk;
        pk.x = (unsigned)h0 | ((unsigned)h1 << 16);
        pk.y = (unsigned)h2 | ((unsigned)h3 << 16);
        size_t orow = row;
        if (phase) {  // phase-local row -> input pixel
          const int hw = args.Hp * args.Wp;
          const int n = fast_div(row, args.dPQ), rem = row - n * hw;
          const int i = fast_div(rem, args.dQ), j = rem - i * args.Wp;
          orow = ((size_t)n * gg.H + args.pa + gg.stride * i) * gg.W + args.pb + gg.stride * j;
        } else if (pmr) {  // (pixel, image) row -> NHWC row
          orow = (size_t)(pmr_n0 + row - pmr_row0) * (gg.P * gg.Q) + pmr_pq;
        }
        if (MODE == MODE_DGRAD && args.accumulate) {  // dx += (second gradient branch)
          uint2* dst = reinterpret_cast<uint2*>(args.out + orow * args.Ng + col);
          const uint2 old = acc_old4(args.out, args.acc_dy, args.acc_mask, orow * args.Ng + col);
          pk.x = (unsigned)f2bf(v[0] + bf2f((unsigned short)(old.x & 0xffff))) |
                 ((unsigned)f2bf(v[1] + bf2f((unsigned short)(old.x >> 16))) << 16);
          pk.y = (unsigned)f2bf(v[2] + bf2f((unsigned short)(old.y & 0xffff))) |
                 ((unsigned)f2bf(v[3] + bf2f((unsigned short)(old.y >> 16))) << 16);
          *dst = pk;
        } else {
          *reinterpret_cast<uint2*>(args.out + orow * args.Ng + col) = pk;
        }
        if (MODE == MODE_FWD) {
          const float r0 = bf2f(h0), r1 = bf2f(h1), r2 = bf2f(h2), r3 = bf2f(h3);
          s[0] += r0; s[1] += r1; s[2] += r2; s[3] += r3;
          ss[0] += r0 * r0; ss[1] += r1 * r1; ss[2] += r2 * r2; ss[3] += r3 * r3;
        }
        if (MODE == MODE_DGRAD && kOldBnf && red) {
          // this row is pixel (n, h, w) of the preceding block's output; its gradient (as
          // stored, bf16-rounded) flows to the window argmax of relu(bn(z)) (pool) and through
          // the ReLU mask: dy_bn; S1 += dy_bn, S2 += dy_bn * xhat — bn_act.hip bwd_compute
          const float gv[4] = {bf2f(h0), bf2f(h1), bf2f(h2), bf2f(h3)};
          const float fsc[4] = {bsc.x, bsc.y, bsc.z, bsc.w}, fsh[4] = {bsh.x, bsh.y, bsh.z, bsh.w};
          const float fmu[4] = {bmu.x, bmu.y, bmu.z, bmu.w}, fis[4] = {bis.x, bis.y, bis.z, bis.w};
          const BnBwdFuse& f = args.bnf;
          const int hw = g.H * g.W;
          const int n = fast_div((int)orow, args.dPQ), rem = (int)orow - n * hw;  // H*W, W
          const int h = fast_div(rem, args.dQ), w = rem - h * g.W;
          const int np = f.pool ? 4 : 1;
          float zf[4][4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            if (d >= np) break;
            const int zh = f.pool ? 2 * h + (d >> 1) : h, zw = f.pool ? 2 * w + (d & 1) : w;
            const uint2 zz = *reinterpret_cast<const uint2*>(
                f.z + (((size_t)n * f.Hz + zh) * f.Wz + zw) * args.Ng + col);
            zf[d][0] = bf2f((unsigned short)(zz.x & 0xffff));
            zf[d][1] = bf2f((unsigned short)(zz.x >> 16));
            zf[d][2] = bf2f((unsigned short)(zz.y & 0xffff));
            zf[d][3] = bf2f((unsigned short)(zz.y >> 16));
          }
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            float best = -INFINITY, yarg = 0.f, zarg = 0.f;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
              if (d >= np) break;
              const float y = zf[d][t] * fsc[t] + fsh[t];
              const float yr = f.relu ? fmaxf(y, 0.f) : y;
              if (d == 0 || yr > best || yr != yr) { best = yr; yarg = y; zarg = zf[d][t]; }
            }
            const float dyb = (f.relu && !(yarg > 0.f)) ? 0.f : gv[t];
            s[t] += dyb;
            ss[t] += dyb * ((zarg - fmu[t]) * fis[t]);
          }
        }
      }
    }
    if (red) {
      // reduce over the 16 rows held by lanes (lane & 15) of each 16-lane group
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        s[t] = dpp_sum16(s[t]);
        ss[t] = dpp_sum16(ss[t]);
      }
      // wave row 1 parks its column sums in LDS slot [wn][j][lane>>4][8]; row 0 adds them
      float* slot = reinterpret_cast<float*>(smem) + (((wn * TN + j) * 4 + (lane >> 4)) * 8);
      if (wm == 1 && rl == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          slot[t] = s[t];
          slot[4 + t] = ss[t];
        }
      }
      stat_s[j][0] = s[0]; stat_s[j][1] = s[1]; stat_s[j][2] = s[2]; stat_s[j][3] = s[3];
      stat_ss[j][0] = ss[0]; stat_ss[j][1] = ss[1]; stat_ss[j][2] = ss[2]; stat_ss[j][3] = ss[3];
    }
  }
  if (red) {
    __syncthreads();
    if (wm == 0 && rl == 0) {
      float* st = (MODE == MODE_FWD ? args.stats : args.bnf.sums) +
                  stat_rep(bid) * 2 * args.Ng;  // spread contention
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = col0 + wn * WTN + j * 16 + cq;
        if (col >= args.Ng) continue;
        const float* slot = reinterpret_cast<const float*>(smem) + (((wn * TN + j) * 4 + (lane >> 4)) * 8);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          atomicAdd(st + col + t, stat_val(stat_s[j][t] + slot[t], bid));
          atomicAdd(st + args.Ng + col + t, stat_val(stat_ss[j][t] + slot[4 + t], bid));
        }
      }
    }
  }
  };

  // NST-stage LDS ring: the DMAs of up to NST-1 k-steps are in flight while one is computed.
  constexpr int DMA = CA + CB;  // vector-memory instructions per thread per stage
  for (int item = bid; item < nitems; item += nblk) {
    setup(item);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    const int kb = ks_begin, ke = ks_end;  // host guarantees kb < ke for every item
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (kb + s < ke) issue(kb + s, s);
    int stage = 0;
    for (int ks = kb; ks < ke; ++ks) {
      // stages issued after ks and still allowed in flight: min(NST-2, ke-1-ks)
      const int ahead = ke - 1 - ks;
      if (NST >= 4 && ahead >= 2) wait_dma_barrier<(NST >= 4 ? 2 : 0) * DMA>();
      else if (NST >= 3 && ahead >= 1) wait_dma_barrier<(NST >= 3 ? 1 : 0) * DMA>();
      else wait_dma_barrier<0>();
      // the first half's fragment reads go out before the next DMA is issued, so their LDS
      // latency hides behind the gather's address math instead of stalling the MFMAs after it
      bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
      load_frags(stage, 0, fa0, fb0);
      // every wave finished computing ks-1: its buffer takes k-step ks+NST-1
      if (ks + NST - 1 < ke) issue(ks + NST - 1, stage == 0 ? NST - 1 : stage - 1);
      load_frags(stage, 32, fa1, fb1);
      mma(fa0, fb0);
      mma(fa1, fb1);
      stage = stage + 1 == NST ? 0 : stage + 1;
    }
    epilogue(row0, col0, zsplit, args.splits > 1);
    // all reads of the ring done before the next item's prologue DMA. Not after the last item:
    // vmcnt also counts the epilogue's stores, and waiting for their acknowledgement would hold
    // the workgroup slot (and its registers) for a full memory round trip after the last MFMA
    if (item + nblk < nitems) wait_dma_barrier<0>();
  }
  if constexpr (XSTAT) {
    if (MODE == MODE_FWD && run_col >= 0)  // (uniform: run_col is)
      flush_stats(run_col, *reinterpret_cast<float(*)[8]>(run_s),
                  *reinterpret_cast<float(*)[8]>(run_ss));
  }
}

// 2 waves per SIMD (<= 256 VGPR + AGPR per lane): left to itself the compiler gives the big
// tiles 256 VGPRs + ~100 AGPRs (1 wave per SIMD), and these GEMMs are latency-bound
// (-DDDP_CONV_WAVES_PER_EU=1 builds the unconstrained variant for A/B runs)
#ifndef DDP_CONV_WAVES_PER_EU
#define DDP_CONV_WAVES_PER_EU 2
#endif
template <int MODE, int BM, int BN, int NST, int BNF = 0, bool XSTAT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DDP_CONV_WAVES_PER_EU)))
void conv_igemm_kernel(ConvArgs args) {
  // dynamic: the launcher sizes the ring to the stages a work item can use (launch_gemm_t)
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  conv_igemm_body<MODE, BM, BN, NST, BNF, XSTAT>(args, smem, blockIdx.x, gridDim.x);
}

// BNF 2 (no-pool BN-backward sums in the lean epilogue): the extra per-column coefficients push
// the big tiles past 256 registers (1 wave per SIMD); ask the register allocator for 2 waves.
template <int MODE, int BM, int BN, int NST>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void conv_igemm_bnf2_kernel(ConvArgs args) {
  extern __shared__ __attribute__((aligned(16))) unsigned short smem[];
  conv_igemm_body<MODE, BM, BN, NST, 2>(args, smem, blockIdx.x, gridDim.x);
}

// One layer's backward GEMMs in ONE launch: blocks [0, n_dg) run the DGRAD problem, the rest
// the WGRAD problem (independent outputs, both read dy). At the strong-scaling batches each of
// them alone leaves most of the 256 CUs idle and pays its own latency floor; side by side they
// fill each other's idle slots and cost one dispatch. Same tile config for both (one LDS array).
template <int BM, int BN, int NST, int BNF, bool SGDM = false>
__global__ __launch_bounds__(256) void conv_bwd_pair_kernel(ConvArgs dg, ConvArgs wg, int n_dg) {
  __shared__ __attribute__((aligned(16))) unsigned short smem[ConvSmem<BM, BN, NST>::elems];
  if ((int)blockIdx.x < n_dg)
    conv_igemm_body<MODE_DGRAD, BM, BN, NST, BNF>(dg, smem, blockIdx.x, n_dg);
  else
    conv_igemm_body<MODE_WGRAD, BM, BN, NST, 0, false, SGDM>(wg, smem, blockIdx.x - n_dg,
                                                           gridDim.x - n_dg);
}
// Split-K finish for FWD/DGRAD: sum the slabs in split order -> (+bias) bf16 output
// (+ per-channel stats of the rounded output for FWD).
// Thread layout: cg_local = tid % Gb (8 channels each), rows strided; stats reduced in
// registers, then through LDS, then ONE atomic per channel per block.
struct RowMap {  // phase-local GEMM row -> output pixel (strided DGRAD); stride 0 = identity
  int stride, Hp, Wp, H, W, pa, pb;
};

__device__ __forceinline__ size_t map_row(const RowMap& m, int row) {
  if (m.stride == 0) return row;
  const int hw = m.Hp * m.Wp;
  const int n = row / hw, rem = row - n * hw;
  const int i = rem / m.Wp, j = rem - i * m.Wp;
  return ((size_t)n * m.H + m.pa + m.stride * i) * m.W + m.pb + m.stride * j;
}

// v[0..8) += p[z * slab + 0..8) for z = z0 .. z1-1, summed in z order (bit-identical to the
// plain loop) but with the loads of up to kSlabBatch slabs issued before the first add: the
// finish passes are latency-bound at the small batches (a plain loop waits one L2/HBM round
// trip per split; 16-row grids at 32 images/GPU spent 6-8 us that way).
constexpr int kSlabBatch = 8;
__device__ __forceinline__ void sum_slabs8(const float* p, size_t slab, int z0, int z1, float* v) {
  for (int zb = z0; zb < z1; zb += kSlabBatch) {
    float4 a[kSlabBatch], b[kSlabBatch];
#pragma unroll
    for (int u = 0; u < kSlabBatch; ++u) {
      if (zb + u < z1) {
        const float4* src = reinterpret_cast<const float4*>(p + (size_t)(zb + u) * slab);
        a[u] = src[0];
        b[u] = src[1];
      }
    }
#pragma unroll
    for (int u = 0; u < kSlabBatch; ++u) {
      if (zb + u < z1) {
        v[0] += a[u].x; v[1] += a[u].y; v[2] += a[u].z; v[3] += a[u].w;
        v[4] += b[u].x; v[5] += b[u].y; v[6] += b[u].z; v[7] += b[u].w;
      }
    }
  }
}

struct FinishArgs {  // split-K finish of a FWD / DGRAD GEMM (one launch or one pair half)
  const float* ws;
  int splits;
  unsigned short* out;
  const float* bias;
  float* stats;
  int Mg, Ng;
  RowMap rmap;
  int accumulate;
  BnBwdFuse bnf;
  int H, W;
  const unsigned short* acc_dy;  // ConvArgs::acc_dy / acc_mask (deferred first branch)
  const unsigned char* acc_mask;
};

// body of splitk_finish_kernel: (bx, by) / gx stand for blockIdx.(x, y) / gridDim.x;
// red = 2 x 8 x 256 floats of LDS
template <bool BNF>
__device__ __forceinline__ void splitk_finish_body(const FinishArgs& fa, float* red_, int bx,
                                                   int by, int gx) {
  const float* ws = fa.ws;
  const int splits = fa.splits, Mg = fa.Mg, Ng = fa.Ng, accumulate = fa.accumulate;
  const int H = fa.H, W = fa.W;
  unsigned short* out = fa.out;
  const float* bias = fa.bias;
  float* stats = fa.stats;
  const RowMap rmap = fa.rmap;
  const BnBwdFuse& bnf = fa.bnf;
  float (*red)[8][256] = reinterpret_cast<float (*)[8][256]>(red_);
  constexpr bool has_bnf = BNF;
  const int G = Ng / 8;
  const int Gb = G < 256 ? G : 256;
  const int cgl = threadIdx.x % Gb, prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int cg = by * Gb + cgl;
  const bool active = prow < prows && cg < G;  // Gb need not divide 256 (e.g. 1000 classes)
  const size_t slab = (size_t)Mg * Ng;
  float s[8], ss[8], bv[8];
  float fsc[8], fsh[8], fmu[8], fis[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = 0.f;
    ss[e] = 0.f;
    bv[e] = (bias && cg < G) ? bias[cg * 8 + e] : 0.f;
    fsc[e] = fsh[e] = fmu[e] = fis[e] = 0.f;
  }
  if (has_bnf && cg < G) {  // DGRAD with the preceding block's BN-backward sums (BnBwdFuse)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fsc[e] = bnf.coef[0 * Ng + cg * 8 + e];
      fsh[e] = bnf.coef[1 * Ng + cg * 8 + e];
      fmu[e] = bnf.coef[2 * Ng + cg * 8 + e];
      fis[e] = bnf.coef[3 * Ng + cg * 8 + e];
    }
    stats = bnf.sums;
  }
  for (int row = bx * prows + prow; active && row < Mg; row += gx * prows) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bv[e];
    sum_slabs8(ws + (size_t)row * Ng + cg * 8, slab, 0, splits, v);
    unsigned short* dst = out + map_row(rmap, row) * Ng + cg * 8;
    if (accumulate) {
      const u16x8 old = acc_old8(out, fa.acc_dy, fa.acc_mask, map_row(rmap, row) * Ng + cg * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bf2f(old[e]);
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(v[e]);
      const float r = bf2f(o[e]);
      if (!has_bnf) {
        s[e] += r;
        ss[e] += r * r;
      }
    }
    st8(dst, o);
    if (has_bnf && bnf.code) {
      // VGG input block: row = its pooled window; the gradient goes to the position the forward
      // recorded (code < 4: conv_l0.hip, 4 = ReLU cut, 0xFF = NaN window) and that pixel's z is
      // the recorded zw — l0_sums_kernel's sums S1 = sum dy, S2 = sum dy * xhat, here
      // Code bytes of channel c: window * 64 + ((c % 16) / 4) * 16 + (c / 16) * 4 + c % 4
      const int c0 = cg * 8;
      const unsigned* cw = bnf.code + (size_t)row * 16 + ((c0 & 15) >> 2) * 4 + (c0 >> 4);
      const unsigned w0 = cw[0], w1 = cw[4];  // channels c0..c0+3 | c0+4..c0+7
      const u16x8 zz = ld8(bnf.z + (size_t)row * Ng + c0);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const unsigned code = ((e < 4 ? w0 : w1) >> (8 * (e & 3))) & 0xFFu;
        const float d = code < 4u ? bf2f(o[e]) : 0.f;
        s[e] += d;
        ss[e] += d * ((bf2f(zz[e]) - fmu[e]) * fis[e]);
      }
    } else if (has_bnf) {  // same recomputation as the GEMM epilogue / bn_act.hip bwd_compute
      const int hw = H * W;
      const int n = row / hw, rem = row - n * hw;
      const int h = rem / W, w = rem - h * W;
      const int np = bnf.pool ? 4 : 1;
      float best[8], yarg[8], zarg[8];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (d >= np) break;
        const int zh = bnf.pool ? 2 * h + (d >> 1) : h, zw = bnf.pool ? 2 * w + (d & 1) : w;
        const u16x8 zz = ld8(bnf.z + (((size_t)n * bnf.Hz + zh) * bnf.Wz + zw) * Ng + cg * 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float zf = bf2f(zz[e]);
          const float y = zf * fsc[e] + fsh[e];
          const float yr = bnf.relu ? fmaxf(y, 0.f) : y;
          if (d == 0 || yr > best[e] || yr != yr) { best[e] = yr; yarg[e] = y; zarg[e] = zf; }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float dyb = (bnf.relu && !(yarg[e] > 0.f)) ? 0.f : bf2f(o[e]);
        s[e] += dyb;
        ss[e] += dyb * ((zarg[e] - fmu[e]) * fis[e]);
      }
    }
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
    if (by * Gb + c >= G) continue;
    float t = 0.f;
    for (int r = 0; r < prows; ++r) t += red[k][e][r * Gb + c];
    const int lb = by * gx + bx;  // linear block id (the deterministic build needs it unique)
    float* st = stats + stat_rep(lb) * 2 * Ng;
    atomicAdd(st + k * Ng + (by * Gb + c) * 8 + e, stat_val(t, lb));
  }
}

template <bool BNF>
__global__ __launch_bounds__(256) void splitk_finish_kernel(FinishArgs fa) {
  __shared__ float red[2 * 8 * 256];
  splitk_finish_body<BNF>(fa, red, blockIdx.x, blockIdx.y, gridDim.x);
}

// Slab sums of the BN-fused finishes: rows lane, lane + 128, ... of channels [c0, c0 + 8);
// 8 / RPT splits of every row in flight per batch (the small layers take 4-12 splits; a plain
// loop paid one L2 round trip per split), split order kept per element.
template <int RPT>
__device__ __forceinline__ void fused_finish_slabs(const float* ws, size_t slab, int Ng, int Mg,
                                                   int splits, int lane, int c0, float (*v)[8]) {
  constexpr int ZB = RPT >= 8 ? 1 : 8 / RPT;
  for (int zb = 0; zb < splits; zb += ZB) {
    float4 a[ZB][RPT], b[ZB][RPT];
#pragma unroll
    for (int u = 0; u < ZB; ++u)
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const int row = lane + r * 128;
        if (zb + u < splits && row < Mg) {
          const float4* src =
              reinterpret_cast<const float4*>(ws + (size_t)(zb + u) * slab + (size_t)row * Ng + c0);
          a[u][r] = src[0];
          b[u][r] = src[1];
        }
      }
#pragma unroll
    for (int u = 0; u < ZB; ++u)
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        if (zb + u < splits && lane + r * 128 < Mg) {
          v[r][0] += a[u][r].x; v[r][1] += a[u][r].y; v[r][2] += a[u][r].z; v[r][3] += a[u][r].w;
          v[r][4] += b[u][r].x; v[r][5] += b[u][r].y; v[r][6] += b[u][r].z; v[r][7] += b[u][r].w;
        }
      }
  }
}

// Split-K finish + training-mode BatchNorm + ReLU (+ 2x2/s2 max-pool) of a SMALL forward GEMM
// (Mg <= 128 * RPT rows): block b owns channels [16b, 16b + 16) over EVERY row — waves 0-1 the
// first 8 channels, waves 2-3 the next 8, lane l of a half the rows l, l + 128, ... — so the
// batch statistics of its channels are complete in the block: slab sums (+bias) -> bf16 z
// (stored: the backward reads it) -> sum / sum of squares of the rounded values (DPP wave sums,
// 4 partials through LDS) -> mean, invstd, scale, shift (coefficient table for the backward) ->
// y = relu(z * scale + shift), max-pooled through LDS. Replaces finish + BN-apply launches, the
// statistic replicas and their atomics (the strong-scaling batches: 16-512-row GEMMs, where
// every launch is a ~5 us latency step). Same formulas as bn_act.hip's finalize + apply.
constexpr int kBnFwdFuseMaxRows = 1024;
template <int RPT>
__global__ __launch_bounds__(256) void splitk_finish_bnfwd_kernel(FinishArgs fa, BnFwdFuse bf) {
  extern __shared__ __attribute__((aligned(16))) float act[];  // [Mg][16] (pooled layers)
  __shared__ float wred[4][2][8];
  __shared__ float cf[2][16];
  const int Mg = fa.Mg, Ng = fa.Ng, splits = fa.splits;
  const int half = threadIdx.x >> 7, lane = threadIdx.x & 127;
  const int c0 = blockIdx.x * 16 + half * 8;
  const size_t slab = (size_t)Mg * Ng;
  float v[RPT][8];
#pragma unroll
  for (int r = 0; r < RPT; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) v[r][e] = fa.bias ? fa.bias[c0 + e] : 0.f;
  // every row's loads of a split in flight together (split order kept per element)
  fused_finish_slabs<RPT>(fa.ws, slab, Ng, Mg, splits, lane, c0, v);
  float s[8], ss[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s[e] = 0.f; ss[e] = 0.f; }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = lane + r * 128;
    if (row >= Mg) continue;
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(v[r][e]);
      v[r][e] = bf2f(o[e]);  // statistics and the BN input are the ROUNDED conv output
      s[e] += v[r][e];
      ss[e] += v[r][e] * v[r][e];
    }
    st8(fa.out + (size_t)row * Ng + c0, o);
  }
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t1 = wave_sum(s[e]), t2 = wave_sum(ss[e]);
    if ((threadIdx.x & 63) == 0) {
      wred[wave][0][e] = t1;
      wred[wave][1][e] = t2;
    }
  }
  __syncthreads();
  if (threadIdx.x < 16) {
    const int h = threadIdx.x >> 3, e = threadIdx.x & 7;
    const float M = (float)Mg;
    const float s1 = wred[2 * h][0][e] + wred[2 * h + 1][0][e];
    const float s2 = wred[2 * h][1][e] + wred[2 * h + 1][1][e];
    const float mu = s1 / M;
    const float var = fmaxf(s2 / M - mu * mu, 0.f);
    const float is = rsqrtf(var + bf.eps);
    const int c = blockIdx.x * 16 + threadIdx.x;
    const float sc = bf.gamma[c] * is;
    const float sh = bf.beta[c] - mu * sc;
    bf.coef[0 * Ng + c] = sc;  // rows of bn_act.hip's coefficient table
    bf.coef[1 * Ng + c] = sh;
    bf.coef[2 * Ng + c] = mu;
    bf.coef[3 * Ng + c] = is;
    cf[0][threadIdx.x] = sc;
    cf[1][threadIdx.x] = sh;
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = cf[0][half * 8 + e];
    sh[e] = cf[1][half * 8 + e];
  }
  if (!bf.pool) {
#pragma unroll
    for (int r = 0; r < RPT; ++r) {
      const int row = lane + r * 128;
      if (row >= Mg) continue;
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float y = v[r][e] * sc[e] + sh[e];
        if (bf.relu) y = fmaxf(y, 0.f);
        o[e] = f2bf(y);
      }
      st8(bf.y + (size_t)row * Ng + c0, o);
    }
    return;
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = lane + r * 128;
    if (row >= Mg) continue;
    float y[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      y[e] = v[r][e] * sc[e] + sh[e];
      if (bf.relu) y[e] = fmaxf(y[e], 0.f);
    }
    float4* dst = reinterpret_cast<float4*>(act + row * 16 + half * 8);
    dst[0] = make_float4(y[0], y[1], y[2], y[3]);
    dst[1] = make_float4(y[4], y[5], y[6], y[7]);
  }
  __syncthreads();
  const int P = bf.P, Q = bf.Q, Po = P / 2, Qo = Q / 2;
  const int Mo = Mg / 4;
  for (int orow = lane; orow < Mo; orow += 128) {
    const int n = orow / (Po * Qo), rem = orow - n * (Po * Qo);
    const int i = rem / Qo, j = rem - i * Qo;
    const int r00 = (n * P + 2 * i) * Q + 2 * j;
    float best[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) best[e] = -INFINITY;
#pragma unroll
    for (int d = 0; d < 4; ++d) {  // window order of bn_act_fwd_kernel
      const int rr = r00 + (d >> 1) * Q + (d & 1);
      const float4* src = reinterpret_cast<const float4*>(act + rr * 16 + half * 8);
      const float4 p0 = src[0], p1 = src[1];
      const float yv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (yv[e] > best[e] || yv[e] != yv[e]) best[e] = yv[e];
    }
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf(best[e]);
    st8(bf.y + (size_t)orow * Ng + c0, o);
  }
}

// Split-K finish of a SMALL stride-1 DGRAD fused with the COMPLETE BatchNorm backward of the
// preceding Conv->BN->ReLU(->2x2 pool) block (the BnBwdFuse chain, api.h BnBwdApply): block bx
// owns channels [16 bx, 16 bx + 16) over every dgrad row (lane l of each 128-thread half: rows
// l, l + 128, ...), so the block has the whole batch of its channels —
//   dgrad slabs -> bf16-rounded dx (never stored: its only consumer is this BN backward)
//   -> recompute the ReLU mask / pool routing from the block's conv output z (bn_act.hip
//      bwd_compute) -> S1 = sum dy_bn, S2 = sum dy_bn * xhat (DPP wave sums + LDS)
//   -> k1 = S1 / M, k2 = S2 / M; dgamma += S2, dbeta += S1 (one writer per channel)
//   -> dz = scale * (dy_bn - k1 - xhat * k2) for all 4 pre-pool pixels.
// Replaces the finish with memory-side sum atomics, the finalize launch and the apply launch of
// the strong-scaling batches' 4x4 / 2x2 layers by one pass.
template <int RPT, bool POOL>
__device__ __forceinline__ void bnbwd_from_dx(const BnBwdFuse& bn, const BnBwdApply& ba, int Mg,
                                              int Ng, int H, int W, float (*v)[8],
                                              float (*wred)[2][8], int half, int lane, int c0);

template <int RPT, bool POOL>
__device__ __forceinline__ void finish_bnbwd_body(const FinishArgs& fa, const BnBwdApply& ba,
                                                  float (*wred)[2][8], int bx) {
  const BnBwdFuse& bn = fa.bnf;
  const int Mg = fa.Mg, Ng = fa.Ng, splits = fa.splits;
  const int half = threadIdx.x >> 7, lane = threadIdx.x & 127;
  const int c0 = bx * 16 + half * 8;
  const size_t slab = (size_t)Mg * Ng;
  float v[RPT][8];
#pragma unroll
  for (int r = 0; r < RPT; ++r)
#pragma unroll
    for (int e = 0; e < 8; ++e) v[r][e] = 0.f;
  fused_finish_slabs<RPT>(fa.ws, slab, Ng, Mg, splits, lane, c0, v);
  bnbwd_from_dx<RPT, POOL>(bn, ba, Mg, Ng, fa.H, fa.W, v, wred, half, lane, c0);
}

// The BN-backward part of finish_bnbwd_body for dx rows held in v (fp32, rounded to bf16 here
// like a stored dgrad output): used by the classifier-head kernel (linear_head_bwd_kernel).
template <int RPT, bool POOL>
__device__ __forceinline__ void bnbwd_from_dx(const BnBwdFuse& bn, const BnBwdApply& ba, int Mg,
                                              int Ng, int H, int W, float (*v)[8],
                                              float (*wred)[2][8], int half, int lane, int c0) {
  constexpr int NP = POOL ? 4 : 1;
  float sc[8], sh[8], mu[8], is[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = bn.coef[0 * Ng + c0 + e];
    sh[e] = bn.coef[1 * Ng + c0 + e];
    mu[e] = bn.coef[2 * Ng + c0 + e];
    is[e] = bn.coef[3 * Ng + c0 + e];
  }
  // the block's z pixels (kept for the apply), dx rounded like the stored dgrad output
  u16x8 zz[RPT][NP];
  unsigned zoff[RPT][NP];  // (host: z has < 2^31 elements)
  const int hw = H * W;
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = lane + r * 128;
    const int rr = row < Mg ? row : 0;
    const int n = rr / hw, rem = rr - n * hw;
    const int h = rem / W, w = rem - h * W;
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      const int zh = POOL ? 2 * h + (d >> 1) : h, zw = POOL ? 2 * w + (d & 1) : w;
      zoff[r][d] = (unsigned)((((size_t)n * bn.Hz + zh) * bn.Wz + zw) * Ng + c0);
      zz[r][d] = ld8(bn.z + zoff[r][d]);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[r][e] = round_bf(v[r][e]);
  }
  // routing, once per (row, channel): the window's argmax (bn_act.hip bwd_compute order and NaN
  // rule) and the gradient it receives, already masked by the ReLU; every other pixel gets 0
  int arg[RPT][8];
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const bool ok = lane + r * 128 < Mg;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float best = -INFINITY, yarg = 0.f, zarg = 0.f;
      int a = 0;
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const float zf = bf2f(zz[r][q][e]);
        const float y = zf * sc[e] + sh[e];
        const float yr = bn.relu ? fmaxf(y, 0.f) : y;
        if (q == 0 || yr > best || yr != yr) { best = yr; a = q; yarg = y; zarg = zf; }
      }
      arg[r][e] = a;
      v[r][e] = (!ok || (bn.relu && !(yarg > 0.f))) ? 0.f : v[r][e];  // now dy_bn at the argmax
      s1[e] += v[r][e];
      s2[e] += v[r][e] * ((zarg - mu[e]) * is[e]);
    }
  }
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float t1 = wave_sum(s1[e]), t2 = wave_sum(s2[e]);
    if ((threadIdx.x & 63) == 0) {
      wred[wave][0][e] = t1;
      wred[wave][1][e] = t2;
    }
  }
  __syncthreads();
  // every thread needs k1 / k2 of its 8 channels: both waves of its half add the same 2 partials
  const float inv_m = 1.f / ((float)Mg * NP);
  float k1[8], k2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float S1 = wred[2 * half][0][e] + wred[2 * half + 1][0][e];
    const float S2 = wred[2 * half][1][e] + wred[2 * half + 1][1][e];
    k1[e] = S1 * inv_m;
    k2[e] = S2 * inv_m;
    if (lane == 0) {
      if (ba.dgamma) ba.dgamma[c0 + e] += S2;
      if (ba.dbeta) ba.dbeta[c0 + e] += S1;
    }
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    if (lane + r * 128 >= Mg) continue;
#pragma unroll
    for (int d = 0; d < NP; ++d) {
      u16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (bf2f(zz[r][d][e]) - mu[e]) * is[e];
        const float dy = (!POOL || arg[r][e] == d) ? v[r][e] : 0.f;
        o[e] = f2bf(sc[e] * (dy - k1[e] - xh * k2[e]));
      }
      st8(ba.dz + zoff[r][d], o);
    }
  }
}

constexpr int kBnBwdFuseMaxRows = 512;  // (template limit: RPT <= 4)
template <int RPT, bool POOL>
__global__ __launch_bounds__(256) void splitk_finish_bnbwd_kernel(FinishArgs fa, BnBwdApply ba) {
  __shared__ float wred[4][2][8];
  finish_bnbwd_body<RPT, POOL>(fa, ba, wred, blockIdx.x);
}

// Classifier head (Linear(F, J), J <= 16) input gradient fused with the whole BatchNorm
// backward of the block before it (VGG: the last Conv->BN->ReLU->2x2 pool, 2x2 -> 1x1): dx =
// (g * dlogits) . W in the order of linear_ce.hip linear_dx_block, never stored, then the same
// per-block BN backward as the small dgrad finishes. Replaces the head's dx pass and that
// block's reduce + finalize + apply launches (linear_bwd then only computes dW / db).
template <int RPT>
__device__ __forceinline__ void linear_dx_bnbwd_body(const float* __restrict__ dl,
                                                     const float* __restrict__ Wt, int B, int F,
                                                     int J, const float* gscale, BnBwdFuse bn,
                                                     BnBwdApply ba, int bx) {
  __shared__ float wred[4][2][8];
  const int half = threadIdx.x >> 7, lane = threadIdx.x & 127;
  const int c0 = bx * 16 + half * 8;
  const float g = gscale ? *gscale : 1.f;
  float w[16][8];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
    if (j < J) {
      w0 = *reinterpret_cast<const float4*>(Wt + (size_t)j * F + c0);
      w1 = *reinterpret_cast<const float4*>(Wt + (size_t)j * F + c0 + 4);
    }
    w[j][0] = w0.x; w[j][1] = w0.y; w[j][2] = w0.z; w[j][3] = w0.w;
    w[j][4] = w1.x; w[j][5] = w1.y; w[j][6] = w1.z; w[j][7] = w1.w;
  }
  float v[RPT][8];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int row = lane + r * 128;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[r][e] = 0.f;
    if (row >= B) continue;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < J) {
        const float d = dl[(size_t)row * J + j] * g;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[r][e] += d * w[j][e];
      }
    }
  }
  bnbwd_from_dx<RPT, true>(bn, ba, B, F, 1, 1, v, wred, half, lane, c0);
}

// The whole head backward in ONE launch: blocks [0, F/16) run the fused dx + BatchNorm backward
// above, the rest the weight / bias gradient (linear_blocks.h linear_dw_block) — one dispatch
// instead of two on the strong-scaling step's critical chain.
template <int RPT>
__global__ __launch_bounds__(256) void linear_head_bwd_kernel(const float* __restrict__ dl,
                                                              const float* __restrict__ Wt,
                                                              const unsigned short* __restrict__ x,
                                                              int B, int F, int J,
                                                              const float* gscale, BnBwdFuse bn,
                                                              BnBwdApply ba, float* dW, float* db,
                                                              int ndx, int nfx) {
  if ((int)blockIdx.x < ndx) {
    linear_dx_bnbwd_body<RPT>(dl, Wt, B, F, J, gscale, bn, ba, blockIdx.x);
  } else {
    const int t = blockIdx.x - ndx;
    linear_dw_block(dl, x, B, F, J, gscale, dW, db, t % nfx, t / nfx);
  }
}

// Split-K finish for WGRAD: dW[k][c][r][s] += sum_z slab[z][k][(r,s,c)].
// Block (k, split-group): sums its group of slabs for GEMM row k with coalesced reads
// (reduction order fixed inside a group), transposes (r,s,c) -> (c,r,s) through LDS, and adds
// into the PyTorch-layout gradient with coalesced stores (one atomic add per group when the
// splits are divided into several groups).
// slabs per finish block row; several rows combine with float atomics (one row in the
// deterministic build: a fixed summation order)
constexpr int kWgFinishGroup = kDeterministic ? (1 << 30) : 32;
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
__device__ __forceinline__ float sgd_step1(float p, float g, float& b, const SgdFuse& h) {
  return sgd_update1(p, g, b, h.lr, h.momentum, h.wd, h.grad_scale, h.nesterov);
}

// With ``sg.p`` (SGD in the backward, api.h SgdFuse; single group only: the sum is the final
// gradient) the finish applies the optimizer step to the layer's weights instead of storing the
// gradient: p -= lr * (momentum buffer update of g + wd * p), plus the bf16 forward operand copy
// — the gradient never reaches memory and the step's separate SGD pass skips this tensor.
constexpr int kWgFinishGroupKrsc = kDeterministic ? (1 << 30) : 16;
__device__ __forceinline__ void wgrad_finish_krsc_body(const float* __restrict__ ws, int splits,
                                                       int K, int RS, int C, int Creal,
                                                       float* __restrict__ dw, int bx, int by,
                                                       int gx, int gy, const SgdFuse& sg) {
  const size_t slab = (size_t)K * RS * C;
  const size_t n4 = slab / 4;
  const int z0 = by * kWgFinishGroupKrsc, z1 = min(splits, z0 + kWgFinishGroupKrsc);
  const bool single = gy == 1;
  const bool opt = single && sg.p != nullptr;
  for (size_t i = bx * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gx * blockDim.x) {
    float4 v = reinterpret_cast<const float4*>(ws + z0 * slab)[i];
    // loads of up to kSlabBatch slabs in flight before the (in-order) adds
    for (int zb = z0 + 1; zb < z1; zb += kSlabBatch) {
      float4 a[kSlabBatch];
#pragma unroll
      for (int u = 0; u < kSlabBatch; ++u)
        if (zb + u < z1) a[u] = reinterpret_cast<const float4*>(ws + (size_t)(zb + u) * slab)[i];
#pragma unroll
      for (int u = 0; u < kSlabBatch; ++u)
        if (zb + u < z1) { v.x += a[u].x; v.y += a[u].y; v.z += a[u].z; v.w += a[u].w; }
    }
    const float vv[4] = {v.x, v.y, v.z, v.w};
    if (opt) {
      if (Creal == C) {
        float4 pv = reinterpret_cast<float4*>(sg.p)[i];
        float4 bv = reinterpret_cast<float4*>(sg.buf)[i];
        pv.x = sgd_step1(pv.x, v.x, bv.x, sg);
        pv.y = sgd_step1(pv.y, v.y, bv.y, sg);
        pv.z = sgd_step1(pv.z, v.z, bv.z, sg);
        pv.w = sgd_step1(pv.w, v.w, bv.w, sg);
        reinterpret_cast<float4*>(sg.p)[i] = pv;
        reinterpret_cast<float4*>(sg.buf)[i] = bv;
        uint2 pk;
        pk.x = (unsigned)f2bf(pv.x) | ((unsigned)f2bf(pv.y) << 16);
        pk.y = (unsigned)f2bf(pv.z) | ((unsigned)f2bf(pv.w) << 16);
        *reinterpret_cast<uint2*>(sg.wc + i * 4) = pk;
      } else {  // channel-padded input layer: master [K][R][S][Creal], copy [K][R][S][C]
        const size_t e = i * 4;
        const int c = (int)(e % C);
        const size_t krs = e / C;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (c + t >= Creal) continue;
          const size_t mi = krs * Creal + c + t;
          float b = sg.buf[mi];
          const float np = sgd_step1(sg.p[mi], vv[t], b, sg);
          sg.p[mi] = np;
          sg.buf[mi] = b;
          sg.wc[e + t] = f2bf(np);
        }
      }
      continue;
    }
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

__global__ __launch_bounds__(256) void wgrad_finish_krsc_kernel(const float* __restrict__ ws,
                                                                int splits, int K, int RS, int C,
                                                                int Creal, float* __restrict__ dw,
                                                                SgdFuse sg) {
  wgrad_finish_krsc_body(ws, splits, K, RS, C, Creal, dw, blockIdx.x, blockIdx.y, gridDim.x,
                         gridDim.y, sg);
}

struct WgFinishArgs {
  const float* ws;
  int splits, K, RS, C, Creal;
  float* dw;
  int gx, gy;  // its own grid (0 x 0 = no WGRAD finish in this launch)
  SgdFuse sgd;  // SGD in the backward (sgd.p == nullptr: store the gradient)
};

// The split-K finishes of one layer's backward pair in ONE launch: blocks [0, dgx*dgy) reduce
// the DGRAD slabs (dgy channel chunks), the rest the WGRAD slabs ([K][R][S][C] gradient)
template <bool BNF>
__global__ __launch_bounds__(256) void bwd_pair_finish_kernel(FinishArgs fa, int dgx, int dgy,
                                                              WgFinishArgs wa) {
  __shared__ float red[2 * 8 * 256];
  const int b = blockIdx.x;
  if (b < dgx * dgy) {
    splitk_finish_body<BNF>(fa, red, b % dgx, b / dgx, dgx);
  } else {
    const int w = b - dgx * dgy;
    wgrad_finish_krsc_body(wa.ws, wa.splits, wa.K, wa.RS, wa.C, wa.Creal, wa.dw, w % wa.gx,
                           w / wa.gx, wa.gx, wa.gy, wa.sgd);
  }
}

}  // namespace ddp_amd

// ------------------------------- host launcher -------------------------------
using namespace ddp_amd;

static FastDiv make_fastdiv(int d) {
  FastDiv f;
  int sh = 0;
  while ((1ll << sh) < d) ++sh;
  f.sh = sh;
  f.mul = (unsigned)((((1ull << sh) - (unsigned long long)d) << 32) / (unsigned long long)d + 1);
  return f;
}

static bool fits_buffer(size_t elems) { return elems * 2 < (size_t)kOOB; }

static int g_stages = 2;        // LDS ring depth policy (see stages_for)
constexpr int kNumCUs = 256;
// LDS-staged FWD / DGRAD epilogue (conv_igemm_body); ddp_conv_epi_stage_set(0) restores the direct
// fragment stores
static int g_epi_stage = 1;  // ddp_conv_epi_stage_set (tests: the direct-store oracle)
static bool epi_stage_enabled() { return g_epi_stage != 0; }
extern "C" void ddp_conv_epi_stage_set(int on) { g_epi_stage = on ? 1 : 0; }

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
  // slab write + read at ~4 TB/s plus the finish launch (~3 us)
  double t_split = 0.0;
  if (splits > 1) t_split = 8.0 * splits * (double)slab / 4.0e12 + 3.0e-6;
  return t_mfma + t_split;
}

// LDS ring depth per tile shape (ddp_conv_options selects the policy; 2 = double buffer).
// Bytes per stage: (BM + BN) x 64 x 2 — 32 KB at 128x128, 24 KB at 128x64, 16 KB at 64x64.
static int stages_for(int BM, int BN) {
  if (g_stages <= 2) return 2;
  if (BM == 128 && BN == 128) return g_stages >= 4 ? 4 : 2;  // 3 would not fit 2 blocks either
  if (BM == 64 && BN == 64) return g_stages >= 4 ? 4 : 3;
  return 3;
}

// grid cap of the statistics-reducing FWD GEMMs (measured: profiles/r5u_fwd_stat_grid.md)
static int fwd_stat_grid() {
  constexpr int g = 2048;
  return (kDeterministic ? std::min(g, kStatRep) : g) / 8 * 8;
}

template <int MODE, int BM, int BN, int NST, int BNF>
static void launch_gemm_t(const ConvArgs& a, int items, hipStream_t st) {
  constexpr int kStageBytes = (BM + BN) * 64 * 2;
  // A work item of k k-steps touches min(NST, k) ring stages (the prologue issues k-steps
  // 0..NST-2, the loop refills the stage freed by the previous k-step only while k-steps
  // remain). Short reductions — the 1x1 convs over 64/128 channels, 1-2 k-steps — thus need a
  // fraction of the ring, and the smaller LDS footprint doubles the resident workgroups per CU
  // (their tiles are latency-bound: DMA in, a few MFMAs, stores out).
  // the LDS-staged epilogue needs the whole bf16 tile (more than one stage only for the
  // 256x128 / 128x256 tiles)
  constexpr int kTileBytes = BM * BN * 2;
  const int stages = std::max(1, std::min(NST, a.ksteps_per_split));
  size_t lds = (size_t)stages * kStageBytes;
  if (a.epi_stage && lds < (size_t)kTileBytes) lds = kTileBytes;
  // FWD GEMMs with statistics over many items: a capped grid whose blocks walk the items and
  // keep running statistics (the XSTAT instantiation, conv_igemm_body)
  int grid = items;
  if (MODE == MODE_FWD && a.stats && a.splits <= 1 && a.epi_stage && !(BM == 64 && BN == 64) &&
      fwd_stat_grid() > 0 && items > fwd_stat_grid())
    grid = fwd_stat_grid();
  void (*kern)(ConvArgs);
  if constexpr (BNF == 2 && MODE == MODE_DGRAD) kern = conv_igemm_bnf2_kernel<MODE, BM, BN, NST>;
  else if constexpr (MODE == MODE_FWD && BNF == 0 && !(BM == 64 && BN == 64))
    kern = grid < items ? conv_igemm_kernel<MODE, BM, BN, NST, 0, true>
                        : conv_igemm_kernel<MODE, BM, BN, NST, 0, false>;
  else kern = conv_igemm_kernel<MODE, BM, BN, NST, BNF>;
  static bool attr[2] = {false, false};
  if (!attr[grid < items]) {
    // an error here surfaces through the caller's hipGetLastError
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              std::max(NST * kStageBytes, kTileBytes));
    attr[grid < items] = true;
  }
  // one work item (tile x split) per workgroup (a persistent grid sized to the resident slots
  // was measured no faster and removed in round 5) — except FWD GEMMs whose LDS-staged
  // epilogue reduces the BatchNorm statistics: a grid of kFwdStatGrid blocks (a multiple of 8,
  // so item % 8 keeps naming the block's XCD for xcd_remap) walks the items and adds each
  // column tile's partial sums once per block (the running sums of conv_igemm_body)
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, a);
}

template <int MODE, int BM, int BN, int NST>
static void launch_gemm(const ConvArgs& a, int items, hipStream_t st) {
  if constexpr (MODE == MODE_DGRAD) {
    // the BN-backward sums are reduced in the non-split epilogue: a single split only (split
    // GEMMs reduce them in the finish kernel)
    if (a.has_bnf && a.splits <= 1)
      return a.bnf.pool ? launch_gemm_t<MODE, BM, BN, NST, 1>(a, items, st)
                        : launch_gemm_t<MODE, BM, BN, NST, 2>(a, items, st);
  }
  launch_gemm_t<MODE, BM, BN, NST, 0>(a, items, st);
}

// pixel-major WGRAD (ConvArgs::pixmajor) for this tile: stride-1 "same" conv, 64-image blocks,
// at most 64 output pixels per image, one tap per column tile. ddp_conv_wgrad_pm_set(0) keeps
// the pixel-order reduction (tests compare the two).
static int g_wgrad_pm = 1, g_rows_pm = 1;
// WGRAD: 0 off, 1 the <= 64-pixel images, 2 any image size
extern "C" void ddp_conv_wgrad_pm_set(int mode) { g_wgrad_pm = std::max(0, std::min(2, mode)); }
// rows: 0 off, 1 the <= 64-pixel images, 2 any image size, 3 / 4 = 1 / 2 for R*S > 1 only
extern "C" void ddp_conv_rows_pm_set(int mode) { g_rows_pm = std::max(0, std::min(4, mode)); }
// pixel-major FWD / DGRAD rows (ConvArgs::pixmajor) for a BM-row tile
template <int MODE>
static bool rows_pixmajor_ok(const ConvArgs& a, int BM) {
  const ConvGeom& g = a.g;
  const int cdim = MODE == MODE_FWD ? g.C : g.K;
  const bool any_pq = g_rows_pm == 2 || g_rows_pm == 4;
  if (g_rows_pm >= 3 && g.R * g.S == 1) return false;
  return g_rows_pm && !a.d2x2 && !a.phase && !a.accumulate && g.stride == 1 && g.P == g.H &&
         g.Q == g.W && cdim % 64 == 0 && g.N % BM == 0 && (any_pq || g.P * g.Q <= 64) &&
         g.R * g.S <= 32 && g.Creal == g.C && a.Mg == g.N * g.P * g.Q;
}
static bool wgrad_pixmajor_ok(const ConvArgs& a, int BN) {
  const ConvGeom& g = a.g;
  return g_wgrad_pm && g.stride == 1 && g.P == g.H && g.Q == g.W && g.N % 64 == 0 &&
         (g_wgrad_pm == 2 || g.P * g.Q <= 64) && g.C % BN == 0 && g.Creal == g.C && a.Ng == g.R * g.S * g.C &&
         a.Kg == g.N * g.P * g.Q;
}

// Normalise the split count (no empty split); returns the number of work items (tiles x splits).
template <int MODE, int BM, int BN>
static int prepare_cfg(ConvArgs& a, int splits) {
  constexpr int BK = 64;
  const int tiles = ((a.Mg + BM - 1) / BM) * ((a.Ng + BN - 1) / BN);
  const int ksteps = (a.Kg + BK - 1) / BK;
  const int per = (ksteps + splits - 1) / splits;
  splits = (ksteps + per - 1) / per;
  a.splits = splits;
  a.ksteps_per_split = per;
  a.epi_stage = MODE != MODE_WGRAD && epi_stage_enabled();
  a.pixmajor = MODE == MODE_WGRAD ? wgrad_pixmajor_ok(a, BN) : rows_pixmajor_ok<MODE>(a, BM);
  if (MODE == MODE_DGRAD) {
    const int hh = a.phase ? a.Hp : a.g.H, ww = a.phase ? a.Wp : a.g.W;
    a.dPQ = make_fastdiv(std::max(1, hh * ww));
    a.dQ = make_fastdiv(std::max(1, ww));
  } else {
    a.dPQ = make_fastdiv(std::max(1, a.g.P * a.g.Q));
    a.dQ = make_fastdiv(std::max(1, a.g.Q));
  }
  return tiles * splits;
}

// split-K finish geometry / arguments of a prepared problem
static bool needs_finish(int mode, const ConvArgs& a) {
  (void)mode;
  return a.splits > 1;
}

// Rows per thread of the FWD / DGRAD split-K finish: 1 for small grids (<= 128 blocks at one
// row per thread: the latency-bound finishes of the strong-scaling batches), else 2 (enough
// workgroups in flight for a bandwidth-bound pass). Measured, same session (gpurun_out/finish,
// profiles/r2_finish_batched.md): VGG-11 b32 0.4849 -> 0.4705 (2 rows) -> 0.4596 ms (1 row);
// b256 0.9018 -> 0.8984 (2 rows) vs 0.908 ms (1 row everywhere).
static int finish_rows_per_thread(int Mg, int rows_per_block) {
  return (Mg + rows_per_block - 1) / rows_per_block <= 128 ? 1 : 2;
}

static void dg_finish_grid(const ConvArgs& a, int* bx_out, int* chunks_out) {
  const int G = a.Ng / 8;
  const int Gb = G < 256 ? G : 256;
  const int chunks = (G + Gb - 1) / Gb;
  const int rows_per_block = std::max(1, 256 / Gb);
  const int rpt = finish_rows_per_thread(a.Mg, rows_per_block);
  int bx = (a.Mg + rows_per_block * rpt - 1) / (rows_per_block * rpt);
  *bx_out = std::max(1, std::min(bx, 2048 / chunks + 1));
  *chunks_out = chunks;
}

static FinishArgs finish_args(int mode, const ConvArgs& a) {
  RowMap rm{0, 0, 0, 0, 0, 0, 0};
  if (a.phase) rm = RowMap{a.g.stride, a.Hp, a.Wp, a.g.H, a.g.W, a.pa, a.pb};
  const bool fwd = mode == MODE_FWD;
  return FinishArgs{a.ws, a.splits, a.out, fwd ? a.bias : nullptr, fwd ? a.stats : nullptr,
                    a.Mg, a.Ng, rm, a.accumulate, a.bnf, a.g.H, a.g.W, a.acc_dy, a.acc_mask};
}

// ---- SGD in the backward (world 1, engine/step.py TrainStep): registered weights whose WGRAD
// finish reduces every slab in one group take the optimizer step in that finish (SgdFuse);
// ddp_sgd_fuse_taken reports which did, and the step's SGD launch skips exactly those.
// Only where nothing reads the layer's weights after its WGRAD finish within the backward: the
// grouped pair launch (its DGRAD half ran before the finish), a separate DGRAD issued first, or
// a layer without a DGRAD (g_sgd_allow is raised around exactly those finishes).
static std::map<const float*, SgdFuse> g_sgd_reg;  // gradient view -> its fused update
static std::set<const float*> g_sgd_taken;
static std::set<const float*> g_sgd_master;  // master updated in a pair's WGRAD epilogue: the
                                             // step's SGD launch re-packs the operand only
// the pair launch's unsplit WGRAD half (ConvArgs::sgd): any registered weight qualifies, the
// fp32 master is read by nothing else in the backward
static SgdFuse sgd_fuse_master(const float* dw) {
  if (g_sgd_reg.empty()) return SgdFuse{};
  auto it = g_sgd_reg.find(dw);
  if (it == g_sgd_reg.end()) return SgdFuse{};
  g_sgd_master.insert(dw);
  return it->second;
}
static bool g_sgd_allow = false;
static SgdFuse sgd_fuse_for(const float* dw, int groups) {
  if (!g_sgd_allow || groups != 1 || g_sgd_reg.empty()) return SgdFuse{};
  auto it = g_sgd_reg.find(dw);
  if (it == g_sgd_reg.end()) return SgdFuse{};
  g_sgd_taken.insert(dw);
  return it->second;
}

static WgFinishArgs wg_finish_args(const ConvArgs& a) {
  const size_t n4 = (size_t)a.Mg * a.Ng / 4;
  const int groups = (a.splits + kWgFinishGroupKrsc - 1) / kWgFinishGroupKrsc;
  const int bx = (int)std::min<size_t>((n4 + 255) / 256, std::max(1, 2048 / groups));
  return WgFinishArgs{a.ws, a.splits, a.g.K, a.g.R * a.g.S, a.g.C, a.g.Creal, a.dw, bx, groups,
                      sgd_fuse_for(a.dw, groups)};
}

// DGRAD split-K finish with the preceding block's complete BatchNorm backward (small stride-1
// problems). With ``wa`` (a WGRAD finish of the same backward pair) both run in ONE launch.
// false = not applicable (plain finish with the BnBwdFuse sums).
// Row limit of both fused finishes (ddp_conv_bn_fuse_rows): one block owns 16 channels of
// every row, so a bigger GEMM gives each thread several rows of serial, poorly coalesced slab
// reads on only Ng/16 blocks. Measured on the VGG-11 b32 step (profiles/r2_bn_fused_finish.md):
// at 128 rows (2x2 layers) the fused forward finish takes 6.4 us vs 5.1 + 4.4-5.3 us for finish
// + BN apply, the fused backward 11.8 us vs 17 us for finish + finalize + apply; at 512 rows
// (4x4 layers) 10-13 us (forward, no gain) and 29 us (backward, vs 16 us).
static int g_bn_fuse_rows = 128;  // ddp_conv_bn_fuse_rows (tests)
static int bn_fuse_max_rows() { return g_bn_fuse_rows; }
// the backward variant's limit: the common one
static int bn_bwd_fuse_max_rows() { return bn_fuse_max_rows(); }

static bool bnbwd_fusable(const ConvArgs& a) {
  return a.has_bnf && a.bnapply && a.splits > 1 && !a.phase && !a.accumulate &&
         a.Mg <= bn_bwd_fuse_max_rows() && a.Mg <= kBnBwdFuseMaxRows && a.Ng % 16 == 0 &&
         a.g.stride == 1 &&
         (!a.bnf.pool || (a.bnf.Hz == 2 * a.g.H && a.bnf.Wz == 2 * a.g.W)) &&
         (a.bnf.pool || (a.bnf.Hz == a.g.H && a.bnf.Wz == a.g.W));
}

template <int RPT, bool POOL>
__global__ __launch_bounds__(256) void bwd_pair_finish_bnbwd_kernel(FinishArgs fa, BnBwdApply ba,
                                                                    int dgx, WgFinishArgs wa) {
  __shared__ float wred[4][2][8];
  const int b = blockIdx.x;
  if (b < dgx) {
    finish_bnbwd_body<RPT, POOL>(fa, ba, wred, b);
  } else {
    const int w = b - dgx;
    wgrad_finish_krsc_body(wa.ws, wa.splits, wa.K, wa.RS, wa.C, wa.Creal, wa.dw, w % wa.gx,
                           w / wa.gx, wa.gx, wa.gy, wa.sgd);
  }
}

template <int RPT, bool POOL>
static void launch_bnbwd_t(const FinishArgs& fa, const BnBwdApply& ba, int dgx,
                           const WgFinishArgs* wa, hipStream_t st) {
  if (wa)
    hipLaunchKernelGGL((bwd_pair_finish_bnbwd_kernel<RPT, POOL>), dim3(dgx + wa->gx * wa->gy),
                       dim3(256), 0, st, fa, ba, dgx, *wa);
  else
    hipLaunchKernelGGL((splitk_finish_bnbwd_kernel<RPT, POOL>), dim3(dgx), dim3(256), 0, st, fa, ba);
}

static bool launch_finish_bnbwd(const ConvArgs& a, hipStream_t st, const WgFinishArgs* wa) {
  if (!bnbwd_fusable(a)) return false;
  const FinishArgs fa = finish_args(MODE_DGRAD, a);
  const BnBwdApply& ba = *a.bnapply;
  const int dgx = a.Ng / 16, rpt = (a.Mg + 127) / 128;
  if (a.bnf.pool) {
    if (rpt <= 1) launch_bnbwd_t<1, true>(fa, ba, dgx, wa, st);
    else if (rpt <= 2) launch_bnbwd_t<2, true>(fa, ba, dgx, wa, st);
    else launch_bnbwd_t<4, true>(fa, ba, dgx, wa, st);
  } else {
    if (rpt <= 1) launch_bnbwd_t<1, false>(fa, ba, dgx, wa, st);
    else if (rpt <= 2) launch_bnbwd_t<2, false>(fa, ba, dgx, wa, st);
    else launch_bnbwd_t<4, false>(fa, ba, dgx, wa, st);
  }
  if (a.bnapply_done) *a.bnapply_done = 1;
  return true;
}

// FWD split-K finish with the fused BatchNorm forward when the GEMM is small enough for one
// block per 16 channels over all rows; false = not applicable (plain finish + stats).
static bool launch_finish_bnfwd(const ConvArgs& a, hipStream_t st) {
  const BnFwdFuse& bf = *a.bnfwd;
  if (a.Mg > kBnFwdFuseMaxRows || a.Mg > bn_fuse_max_rows() || a.Ng % 16 || a.accumulate ||
      a.phase)
    return false;
  if (bf.P * bf.Q <= 0 || a.Mg % (bf.P * bf.Q)) return false;
  if (bf.pool && (bf.P % 2 || bf.Q % 2)) return false;
  const FinishArgs fa = finish_args(MODE_FWD, a);
  const dim3 grid(a.Ng / 16);
  const size_t lds = bf.pool ? (size_t)a.Mg * 16 * sizeof(float) : 0;
  static const bool attr = [] {  // the <8> instance needs 64 KB of dynamic + its static LDS
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(splitk_finish_bnfwd_kernel<8>),
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              kBnFwdFuseMaxRows * 16 * sizeof(float));
    return true;
  }();
  (void)attr;
  const int rpt = (a.Mg + 127) / 128;
  if (rpt <= 1) hipLaunchKernelGGL(splitk_finish_bnfwd_kernel<1>, grid, dim3(256), lds, st, fa, bf);
  else if (rpt <= 2) hipLaunchKernelGGL(splitk_finish_bnfwd_kernel<2>, grid, dim3(256), lds, st, fa, bf);
  else if (rpt <= 4) hipLaunchKernelGGL(splitk_finish_bnfwd_kernel<4>, grid, dim3(256), lds, st, fa, bf);
  else hipLaunchKernelGGL(splitk_finish_bnfwd_kernel<8>, grid, dim3(256), lds, st, fa, bf);
  if (a.bnfwd_done) *a.bnfwd_done = 1;
  return true;
}

template <int MODE>
static void launch_finish(const ConvArgs& a, hipStream_t st) {
  if (!needs_finish(MODE, a)) return;
  if (MODE == MODE_WGRAD && a.g.wkrsc) {
    const WgFinishArgs w = wg_finish_args(a);
    hipLaunchKernelGGL(wgrad_finish_krsc_kernel, dim3(w.gx, w.gy), dim3(256), 0, st, a.ws,
                       a.splits, a.g.K, a.g.R * a.g.S, a.g.C, a.g.Creal, a.dw, w.sgd);
  } else if (MODE == MODE_WGRAD) {
    const int groups = (a.splits + kWgFinishGroup - 1) / kWgFinishGroup;
    const size_t lds = sizeof(float) * a.g.R * a.g.S * a.g.C;
    hipLaunchKernelGGL(wgrad_finish_kernel, dim3(a.g.K, groups), dim3(256), lds, st, a.ws,
                       a.splits, a.g.K, a.g.R, a.g.S, a.g.C, a.g.Creal, a.dw);
  } else {
    if (MODE == MODE_FWD && a.bnfwd && launch_finish_bnfwd(a, st)) return;
    if (MODE == MODE_DGRAD && a.has_bnf && a.bnapply && launch_finish_bnbwd(a, st, nullptr)) return;
    int bx, chunks;
    dg_finish_grid(a, &bx, &chunks);
    const FinishArgs fa = finish_args(MODE, a);
    if (MODE == MODE_DGRAD && a.has_bnf)
      hipLaunchKernelGGL(splitk_finish_kernel<true>, dim3(bx, chunks), dim3(256), 0, st, fa);
    else
      hipLaunchKernelGGL(splitk_finish_kernel<false>, dim3(bx, chunks), dim3(256), 0, st, fa);
  }
}

template <int MODE, int BM, int BN>
static void launch_cfg(ConvArgs& a, int splits, hipStream_t st, int nst_req = 0) {
  const int items = prepare_cfg<MODE, BM, BN>(a, splits);
  // deepest ring that fits the 160 KiB LDS for this tile ((BM + BN) x 64 bf16 per stage)
  constexpr int kStageBytes = (BM + BN) * 64 * 2;
  constexpr int kMaxStages = kStageBytes * 4 <= 163840 ? 4 : (kStageBytes * 3 <= 163840 ? 3 : 2);
  int nst = nst_req >= 2 && nst_req <= 4 ? nst_req : stages_for(BM, BN);
  nst = std::min(nst, kMaxStages);
  if constexpr (kMaxStages >= 4) {
    if (nst == 4) { launch_gemm<MODE, BM, BN, 4>(a, items, st); goto launched; }
  }
  if constexpr (kMaxStages >= 3) {
    if (nst == 3) { launch_gemm<MODE, BM, BN, 3>(a, items, st); goto launched; }
  }
  launch_gemm<MODE, BM, BN, 2>(a, items, st);
launched:
  if (!a.no_finish) launch_finish<MODE>(a, st);
}

// Measured tile / split-K choices per GEMM problem (tools/conv_tune.py sweeps every candidate
// on the GPU and writes ops/conv_tuning.json, loaded into this table at import). Problems not
// in the table fall back to the cost model. g_force_tile (sweeps only) overrides both.
struct TuneKey {
  int mode, M, N, K;
  int hw = 0;  // pair entries: the layer's H*W (different convs share GEMM dims: VGG-11's
               // b256 2x2 and b64 4x4 512->512 DGRADs are both 1024 x 512 x 4608); 0 = any
  bool operator<(const TuneKey& o) const {
    if (mode != o.mode) return mode < o.mode;
    if (M != o.M) return M < o.M;
    if (N != o.N) return N < o.N;
    if (K != o.K) return K < o.K;
    return hw < o.hw;
  }
};
struct TuneVal {
  int tile, splits, stages;
};
static std::map<TuneKey, TuneVal> g_tuned;  // -> (tile index, splits, LDS stages)
// Backward-pair entries (table mode 3), keyed by the layer's DGRAD problem: tile = 1 pair with
// splits (DGRAD) / stages (= WGRAD splits), tile = 0 the separate launches measured faster
static std::map<TuneKey, TuneVal> g_pair_tuned;
static int g_pair_force_dg = 0, g_pair_force_wg = 0;  // sweeps: forced pair splits (0 = off)
static int g_force_tile = 0;                // 1..4 = tile index + 1
static int g_force_stages = 0;              // 2..4 (sweeps), 0 = policy

// tile index: 0 = 128x128, 1 = 128x64, 2 = 64x128, 3 = 64x64 (cost model + table), and the
// big tiles 4 = 256x64, 5 = 64x256, 6 = 256x128, 7 = 128x256 (measured table entries only: less
// L2 -> LDS traffic per MFMA, fewer tiles)
constexpr int kNumTiles = 8;

// Tiles a mode may run. WGRAD keeps one tap decomposition of its B' (x) gather per thread, which
// needs BN <= 128 (swz_row_step): 64x256 / 128x256 are never launched for WGRAD. (Before round 4
// the 256-wide k-major tiles put odd DMA chunks in the wrong swizzled LDS slot — DGRAD 64x256 /
// 128x256 computed a wrong dx, WGRAD 256x64 / 256x128 a wrong dW; tests/test_gpu_kernels.py
// ::test_conv_every_tile now checks every tile in every mode.)
template <int MODE>
static bool tile_ok(int tile) {
  if (MODE == MODE_WGRAD && (tile == 5 || tile == 7)) return false;
  return tile >= 0 && tile < kNumTiles;
}

// tile / split-K / LDS-stage choice for a problem: the measured table, else the cost model
// (a forced or tabulated tile the mode may not run falls back to the cost model's choice)
template <int MODE>
static void plan_mode(ConvArgs& a, size_t ws_elems, int* best_out, int* sp, int* nst_out) {
  const double c[4] = {tile_cost(128, 128, a, ws_elems, &sp[0]), tile_cost(128, 64, a, ws_elems, &sp[1]),
                       tile_cost(64, 128, a, ws_elems, &sp[2]), tile_cost(64, 64, a, ws_elems, &sp[3])};
  int best = 0, nst = g_force_stages;
  for (int i = 1; i < 4; ++i)
    if (c[i] < c[best]) best = i;
  if (g_force_tile >= 1 && g_force_tile <= kNumTiles && tile_ok<MODE>(g_force_tile - 1)) {
    best = g_force_tile - 1;
    if (best >= 4) {
      static const int bmn[4][2] = {{256, 64}, {64, 256}, {256, 128}, {128, 256}};
      tile_cost(bmn[best - 4][0], bmn[best - 4][1], a, ws_elems, &sp[best]);
    }
  } else if (a.splits <= 0) {
    auto it = g_tuned.find(TuneKey{MODE, a.Mg, a.Ng, a.Kg});
    if (it != g_tuned.end() && tile_ok<MODE>(it->second.tile)) {
      const size_t slab = (size_t)a.Mg * a.Ng;
      const int ksteps = (a.Kg + 63) / 64;
      int spl = std::max(1, std::min(it->second.splits, ksteps));
      if (spl > 1 && (size_t)spl * slab > ws_elems) spl = std::max<int>(1, (int)(ws_elems / slab));
      if (ws_elems == 0) spl = 1;
      best = it->second.tile;
      sp[best] = spl;
      nst = it->second.stages;
    }
  }
  *best_out = best;
  *nst_out = nst;
}

template <int MODE>
static void launch_mode(ConvArgs& a, size_t ws_elems, hipStream_t st) {
  int sp[kNumTiles], best, nst;
  plan_mode<MODE>(a, ws_elems, &best, sp, &nst);
  switch (best) {
    case 0: launch_cfg<MODE, 128, 128>(a, sp[0], st, nst); break;
    case 1: launch_cfg<MODE, 128, 64>(a, sp[1], st, nst); break;
    case 2: launch_cfg<MODE, 64, 128>(a, sp[2], st, nst); break;
    case 3: launch_cfg<MODE, 64, 64>(a, sp[3], st, nst); break;
    case 4: launch_cfg<MODE, 256, 64>(a, sp[4], st, nst); break;
    case 6: launch_cfg<MODE, 256, 128>(a, sp[6], st, nst); break;
    default:
      if constexpr (MODE != MODE_WGRAD) {  // BN = 256 (tile_ok keeps WGRAD off them)
        if (best == 5) launch_cfg<MODE, 64, 256>(a, sp[5], st, nst);
        else launch_cfg<MODE, 128, 256>(a, sp[7], st, nst);
      }
      break;
  }
}

extern "C" void ddp_conv_options(int stages) { g_stages = stages; }

// tile: index into the launch_mode table (0..kNumTiles-1)
extern "C" void ddp_conv_tune_set(int mode, int M, int N, int K, int tile, int splits, int stages) {
  if (mode == 3) {  // backward pair: tile = 0 separate / pair tile 1..4 (kPairTiles), splits /
                    // stages = DGRAD / WGRAD splits
    g_pair_tuned[TuneKey{MODE_DGRAD, M, N, K}] = {tile >= 0 && tile < 6 ? tile : 1,
                                                  std::max(1, splits), std::max(1, stages)};
    return;
  }
  if (tile < 0 || tile >= kNumTiles) return;
  g_tuned[TuneKey{mode, M, N, K}] = {tile, std::max(1, splits), stages};
}
// backward-pair entry for the layer with H*W = hw (tile 0 = separate launches, 1..5 pair tiles)
extern "C" void ddp_conv_pair_tune_set(int M, int N, int K, int hw, int tile, int sd, int sw) {
  g_pair_tuned[TuneKey{MODE_DGRAD, M, N, K, hw}] = {tile >= 0 && tile < 6 ? tile : 1,
                                                    std::max(1, sd), std::max(1, sw)};
}
extern "C" void ddp_conv_tune_clear() {
  g_tuned.clear();
  g_pair_tuned.clear();
}
static int g_pair_force_tile_req = 0;  // sweeps: 1..4 forces the pair tile
extern "C" void ddp_conv_pair_force(int splits_dg, int splits_wg, int tile) {
  g_pair_force_dg = splits_dg;
  g_pair_force_wg = splits_wg;
  g_pair_force_tile_req = tile;
}
extern "C" void ddp_conv_force_tile(int tile_plus_one, int stages) {
  g_force_tile = tile_plus_one;
  g_force_stages = stages;
}

// ---- dense 2x2 form of the 3x3 convs over 2x2 images (ConvArgs::d2x2; VGG-11's last two
// layers): ddp_conv_dense2x2_set(0) restores the implicit GEMM
static int g_dense2x2 = 1;  // ddp_conv_dense2x2_set (tests: the implicit-GEMM oracle)
static bool dense2x2_on() { return g_dense2x2 != 0; }
extern "C" void ddp_conv_dense2x2_set(int on) { g_dense2x2 = on ? 1 : 0; }
extern "C" int ddp_conv_dense2x2_ok(const ConvGeom* g) {
  return dense2x2_on() && g->R == 3 && g->S == 3 && g->stride == 1 && g->pad == 1 &&
         g->H == 2 && g->W == 2 && g->P == 2 && g->Q == 2 && g->C % 64 == 0 && g->K % 64 == 0 &&
         g->Creal == g->C && fits_buffer((size_t)g->K * 9 * g->C) &&
         fits_buffer((size_t)g->N * 4 * std::max(g->C, g->K));
}
// the dense GEMM's operands: A = the NHWC activation of whole 2x2 images (x for FWD, dy for
// DGRAD) read as [N][4 * channels], B = Wc [K][9][C] through ConvArgs::d2x2 addressing
static void dense2x2_args(ConvArgs& a, const ConvGeom* g, int mode) {
  a.g = *g;
  a.g.H = a.g.W = a.g.P = a.g.Q = 1;
  a.g.R = a.g.S = 1;
  a.g.pad = 0;
  a.g.C = a.g.Creal = 4 * g->C;
  a.g.K = 4 * g->K;
  a.Mg = g->N;
  a.Ng = mode == MODE_FWD ? 4 * g->K : 4 * g->C;
  a.Kg = mode == MODE_FWD ? 4 * g->C : 4 * g->K;
  a.d2x2 = 1;
  a.d2C = g->C;
  a.d2K = g->K;
  a.a_bytes = (int)(2 * (size_t)g->N * a.Kg);
  a.b_bytes = (int)(2 * (size_t)g->K * 9 * g->C);
}
// split-K factor of a dense problem that must end in a finish (>= 2; 0 = does not fit ws)
static int dense2x2_splits(const ConvArgs& a, size_t ws_elems) {
  const int tiles = ((a.Mg + 63) / 64) * ((a.Ng + 63) / 64), ksteps = a.Kg / 64;
  int sp = std::max(2, std::min((512 + tiles - 1) / tiles, ksteps / 4));
  const size_t slab = (size_t)a.Mg * a.Ng;
  if ((size_t)sp * slab > ws_elems) sp = (int)(ws_elems / slab);
  return sp >= 2 ? sp : 0;
}
// the 3x3 view of a dense problem for its split-K finish: the slab bytes [split][N][4 x ch]
// are [split][N * 4][ch] (NHWC), so the standard finishes (bias, statistics, BatchNorm) apply
static ConvArgs finish_view(const ConvArgs& a, const ConvGeom* g, int mode) {
  if (!a.d2x2) return a;
  ConvArgs f = a;
  f.g = *g;
  f.d2x2 = 0;
  f.Mg = g->N * g->P * g->Q;
  f.Ng = mode == MODE_FWD ? g->K : g->C;
  f.Kg = 9 * (mode == MODE_FWD ? g->C : g->K);
  return f;
}

// FWD through the dense 2x2 GEMM + the standard finish; -1 = not served
static int conv_fwd_dense(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                          void* y, float* stats, float* ws, size_t ws_elems, const BnFwdFuse* bn,
                          int* bn_done, hipStream_t st) {
  if (!ddp_conv_dense2x2_ok(g) || ws == nullptr) return -1;
  ConvArgs a{};
  dense2x2_args(a, g, MODE_FWD);
  a.a = (const unsigned short*)x;
  a.b = (const unsigned short*)wc;
  a.out = (unsigned short*)y;
  a.ws = ws;
  a.splits = dense2x2_splits(a, ws_elems);
  if (a.splits < 2) return -1;
  a.no_finish = 1;
  launch_mode<MODE_FWD>(a, ws_elems, st);
  ConvArgs f = finish_view(a, g, MODE_FWD);
  f.no_finish = 0;
  f.bias = bias;
  f.stats = stats;
  if (bn && f.Mg <= kBnFwdFuseMaxRows) {
    f.bnfwd = bn;
    f.bnfwd_done = bn_done;
  }
  launch_finish<MODE_FWD>(f, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_fwd(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                            void* y, float* stats, float* ws, size_t ws_elems, int splits,
                            hipStream_t st) {
  if (g->C % 8 || g->K % 8) return -1;
  {
    const int r = conv_fwd_dense(g, x, wc, bias, y, stats, ws, ws_elems, nullptr, nullptr, st);
    if (r >= 0) return r;
  }
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
  const size_t xa = (size_t)g->N * g->H * g->W * g->C, wb = (size_t)a.Ng * a.Kg;
  // (the output too: the epilogue addresses it with 32-bit element offsets)
  if (!fits_buffer(xa) || !fits_buffer(wb) || !fits_buffer((size_t)a.Mg * a.Ng)) return -2;
  a.a_bytes = (int)(2 * xa);
  a.b_bytes = (int)(2 * wb);
  launch_mode<MODE_FWD>(a, ws_elems, st);
  return (int)hipGetLastError();
}

// dx fused with the BatchNorm backward AND dW / db in one launch. 1: launched (dx NOT written;
// dz / dgamma / dbeta of the block before the head written), 0: shape not served (nothing
// launched; caller runs linear_bwd with dx + that block's BN backward), < 0 invalid,
// >= 2: HIP error (rc - 2)
extern "C" int ddp_linear_head_bwd_bn(const float* dl, const float* W, const void* x, int B,
                                      int F, int J, const float* gscale, const BnBwdFuse* bn,
                                      const BnBwdApply* ba, float* dW, float* db, hipStream_t st) {
  if (!bn || !ba || !dl || !W || !x || !dW) return -1;
  if (J < 1 || J > 16 || F % 16 || B < 1 || B > 512 || !bn->pool || bn->Hz != 2 || bn->Wz != 2)
    return 0;
  const int ndx = F / 16, nfx = (F + 63) / 64, nry = (B + kDwRows - 1) / kDwRows;
  const dim3 grid(ndx + nfx * nry);
  const unsigned short* xb = (const unsigned short*)x;
  if (B <= 128) hipLaunchKernelGGL(linear_head_bwd_kernel<1>, grid, dim3(256), 0, st, dl, W, xb, B, F, J, gscale, *bn, *ba, dW, db, ndx, nfx);
  else if (B <= 256) hipLaunchKernelGGL(linear_head_bwd_kernel<2>, grid, dim3(256), 0, st, dl, W, xb, B, F, J, gscale, *bn, *ba, dW, db, ndx, nfx);
  else hipLaunchKernelGGL(linear_head_bwd_kernel<4>, grid, dim3(256), 0, st, dl, W, xb, B, F, J, gscale, *bn, *ba, dW, db, ndx, nfx);
  const int e = (int)hipGetLastError();
  return e ? 2 + e : 1;
}

extern "C" void ddp_conv_bn_fuse_rows(int rows) { g_bn_fuse_rows = std::max(0, rows); }

extern "C" int ddp_conv_fwd_bn(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                               void* z, float* stats, float* ws, size_t ws_elems,
                               const BnFwdFuse* bn, hipStream_t st) {
  constexpr bool enabled = true;  // (ops/layers.py BN_FWD_FUSE switches the caller)
  if (g->C % 8 || g->K % 8) return -1;
  int done = 0;
  {
    const int r = conv_fwd_dense(g, x, wc, bias, z, stats, ws, ws_elems, enabled ? bn : nullptr,
                                 &done, st);
    if (r > 0) return 2 + r;
    if (r == 0) return done;
  }
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)x;
  a.b = (const unsigned short*)wc;
  a.out = (unsigned short*)z;
  a.ws = ws;
  a.bias = bias;
  a.stats = stats;
  a.Mg = g->N * g->P * g->Q;
  a.Ng = g->K;
  a.Kg = g->R * g->S * g->C;
  const size_t xa = (size_t)g->N * g->H * g->W * g->C, wb = (size_t)a.Ng * a.Kg;
  if (!fits_buffer(xa) || !fits_buffer(wb) || !fits_buffer((size_t)a.Mg * a.Ng)) return -2;
  a.a_bytes = (int)(2 * xa);
  a.b_bytes = (int)(2 * wb);
  if (enabled && bn && a.Mg <= kBnFwdFuseMaxRows) {
    a.bnfwd = bn;
    a.bnfwd_done = &done;
  }
  launch_mode<MODE_FWD>(a, ws_elems, st);
  const int e = (int)hipGetLastError();
  return e ? 2 + e : done;
}

// Split-K finish of a FWD GEMM computed elsewhere (conv_tr.hip's tap-reuse kernel): slabs
// [splits][N*P*Q][K] -> bias + bf16 z + statistics, or with ``bn`` (small problems) the
// BatchNorm-fused finish (*bn_done = 1). Returns the HIP error code.
extern "C" int ddp_conv_fwd_finish(const ConvGeom* g, float* ws, int splits, const float* bias,
                                   void* z, float* stats, const BnFwdFuse* bn, int* bn_done,
                                   hipStream_t st) {
  ConvArgs a{};
  a.g = *g;
  a.out = (unsigned short*)z;
  a.ws = ws;
  a.bias = bias;
  a.stats = stats;
  a.Mg = g->N * g->P * g->Q;
  a.Ng = g->K;
  a.Kg = g->R * g->S * g->C;
  a.splits = splits;
  if (bn && a.Mg <= kBnFwdFuseMaxRows) {
    a.bnfwd = bn;
    a.bnfwd_done = bn_done;
  }
  launch_finish<MODE_FWD>(a, st);
  return (int)hipGetLastError();
}

static int conv_dgrad_impl(const ConvGeom* g, const void* dy, const void* wc, void* dx,
                           float* ws, size_t ws_elems, int splits, int accumulate,
                           const BnBwdFuse* bn, const BnBwdApply* ba, int* bn_done,
                           hipStream_t st, const void* acc_dy = nullptr,
                           const unsigned char* acc_mask = nullptr) {
  if (bn_done) *bn_done = 0;
  if (g->C % 8 || g->K % 8) return -1;
  if (bn && bn->code) return -3;  // the input block's sums: the pair launch's finish only
  if (bn && (accumulate || g->stride != 1)) return -3;  // fused BN sums: plain stride-1 dgrad only
  // deferred first branch: every dx element must be written by this call (stride 1)
  if (acc_mask && (!accumulate || !acc_dy || g->stride != 1)) return -3;
  if (!accumulate && ddp_conv_dense2x2_ok(g) && ws != nullptr) {
    // dense 2x2 GEMM; the preceding block's BatchNorm-backward sums (bn) and the split-K
    // reduction run in the standard finish of the 3x3 view
    ConvArgs d{};
    dense2x2_args(d, g, MODE_DGRAD);
    d.a = (const unsigned short*)dy;
    d.b = (const unsigned short*)wc;
    d.out = (unsigned short*)dx;
    d.ws = ws;
    d.splits = bn ? dense2x2_splits(d, ws_elems) : splits;
    if (!bn || d.splits >= 2) {
      d.no_finish = 1;
      launch_mode<MODE_DGRAD>(d, ws_elems, st);
      if (d.splits > 1) {
        ConvArgs f = finish_view(d, g, MODE_DGRAD);
        f.no_finish = 0;
        if (bn) {
          f.has_bnf = 1;
          f.bnf = *bn;
          f.bnapply = ba;
          f.bnapply_done = bn_done;
        }
        launch_finish<MODE_DGRAD>(f, st);
      }
      return (int)hipGetLastError();
    }
  }
  ConvArgs a{};
  a.accumulate = accumulate;
  a.acc_dy = (const unsigned short*)acc_dy;
  a.acc_mask = acc_mask;
  if (bn) {
    a.has_bnf = 1;
    a.bnf = *bn;
    a.bnapply = ba;
    a.bnapply_done = bn_done;
  }
  a.g = *g;
  a.a = (const unsigned short*)dy;
  a.b = (const unsigned short*)wc;
  a.out = (unsigned short*)dx;
  a.ws = ws;
  a.Ng = g->C;
  a.splits = splits;
  // B = the forward weight copy Wc [K][R][S][C] (read k-major, see BKM in the kernel)
  const size_t dya = (size_t)g->N * g->P * g->Q * g->K, wb = (size_t)g->K * g->R * g->S * g->C;
  if (!fits_buffer(dya) || !fits_buffer(wb) || !fits_buffer((size_t)g->N * g->H * g->W * g->C))
    return -2;
  a.a_bytes = (int)(2 * dya);
  a.b_bytes = (int)(2 * wb);
  if (g->stride == 1) {
    a.Mg = g->N * g->H * g->W;
    a.Kg = g->R * g->S * g->K;
    launch_mode<MODE_DGRAD>(a, ws_elems, st);
    return (int)hipGetLastError();
  }
  // strided conv: one stride-1 GEMM per output phase; phases no tap reaches get zeros
  const int sd = g->stride;
  bool zero_fill = false;
  for (int pa = 0; pa < sd && !zero_fill; ++pa)
    for (int pb = 0; pb < sd; ++pb) {
      const int r0 = (pa + g->pad) % sd, s0 = (pb + g->pad) % sd;
      if ((r0 >= g->R || s0 >= g->S) && pa < g->H && pb < g->W) zero_fill = true;
    }
  if (zero_fill && !accumulate) {  // (accumulating: untouched phases keep their values)
    // a kernel, not hipMemsetAsync: captured into a hipGraph, the memset node was measured to
    // leave dx unwritten before the phase GEMM / the second branch's accumulating dgrad read it
    // (sporadic NaN gradients in replayed ResNet-50 steps, never in eager ones;
    // tools/probes/resnet_graph_probe.py)
    const size_t n16 = (size_t)g->N * g->H * g->W * g->C / 8;  // C % 8 == 0: 16-B chunks
    const unsigned nb = (unsigned)std::min<size_t>((n16 + 255) / 256, 8192);
    hipLaunchKernelGGL(zero16_kernel, dim3(std::max(1u, nb)), dim3(256), 0, st,
                       reinterpret_cast<uint4*>(dx), n16);
  }
  for (int pa = 0; pa < sd; ++pa) {
    for (int pb = 0; pb < sd; ++pb) {
      ConvArgs p = a;
      p.phase = 1;
      p.pa = pa;
      p.pb = pb;
      p.r0 = (pa + g->pad) % sd;
      p.s0 = (pb + g->pad) % sd;
      p.Rt = p.r0 < g->R ? (g->R - p.r0 + sd - 1) / sd : 0;
      p.St = p.s0 < g->S ? (g->S - p.s0 + sd - 1) / sd : 0;
      p.Hp = pa < g->H ? (g->H - pa + sd - 1) / sd : 0;
      p.Wp = pb < g->W ? (g->W - pb + sd - 1) / sd : 0;
      if (p.Rt * p.St == 0 || p.Hp * p.Wp == 0) continue;
      p.qa = (pa + g->pad - p.r0) / sd;
      p.qb = (pb + g->pad - p.s0) / sd;
      p.Mg = g->N * p.Hp * p.Wp;
      p.Kg = p.Rt * p.St * g->K;
      launch_mode<MODE_DGRAD>(p, ws_elems, st);
    }
  }
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_dgrad(const ConvGeom* g, const void* dy, const void* wc, void* dx,
                              float* ws, size_t ws_elems, int splits, int accumulate,
                              hipStream_t st) {
  return conv_dgrad_impl(g, dy, wc, dx, ws, ws_elems, splits, accumulate, nullptr, nullptr,
                         nullptr, st);
}

extern "C" int ddp_conv_dgrad_acc(const ConvGeom* g, const void* dy, const void* wc, void* dx,
                                  float* ws, size_t ws_elems, int splits, const void* acc_dy,
                                  const unsigned char* acc_mask, hipStream_t st) {
  return conv_dgrad_impl(g, dy, wc, dx, ws, ws_elems, splits, 1, nullptr, nullptr, nullptr, st,
                         acc_dy, acc_mask);
}

extern "C" int ddp_conv_dgrad_bn(const ConvGeom* g, const void* dy, const void* wc, void* dx,
                                 float* ws, size_t ws_elems, int splits, const BnBwdFuse* bn,
                                 const BnBwdApply* ba, int* bn_done, hipStream_t st) {
  return conv_dgrad_impl(g, dy, wc, dx, ws, ws_elems, splits, 0, bn, ba, bn_done, st);
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
  if (g->R * g->S == 1) a.g.wkrsc = 1;  // 1x1: [K][C][1][1] == [K][1][1][C]
  a.Mg = g->K;
  a.Ng = g->R * g->S * g->C;
  a.Kg = g->N * g->P * g->Q;
  a.splits = splits;
  const size_t dya = (size_t)g->N * g->P * g->Q * g->K, xb = (size_t)g->N * g->H * g->W * g->C;
  if (!fits_buffer(dya) || !fits_buffer(xb)) return -2;
  a.a_bytes = (int)(2 * dya);
  a.b_bytes = (int)(2 * xb);
  a.dPQ = make_fastdiv(g->P * g->Q);
  a.dQ = make_fastdiv(g->Q);
  launch_mode<MODE_WGRAD>(a, ws_elems, st);
  return (int)hipGetLastError();
}

// ------------------------------- backward pair -------------------------------
// DGRAD + WGRAD of one stride-1 layer in ONE launch (conv_bwd_pair_kernel) and their split-K
// finishes in one more (bwd_pair_finish_kernel): two dispatches instead of up to four, and the
// two latency-bound GEMMs of a small batch share the chip instead of running back to back.
// Policy (ddp_conv_pair_mode, ops/common.py BWD_PAIR_MODE): 0 never; 1 when the measured / modelled
// choice is the 64x64 tile for both problems; 2 always (both forced to 64x64); 3 (default) when
// both pick 64x64, or when the paired 64x64 launch has at most g_pair_items work items (about
// one wave of 4 blocks per CU: the small problems of the strong-scaling batches, where pairing
// beat the separately tuned launches — VGG-11 b64 0.544 vs 0.608 ms, b128 0.666 vs 0.702 —
// while forcing it on the big b256 layers lost 5%).
static int g_pair_mode = 3;
static int g_pair_items = 1024;
extern "C" void ddp_conv_pair_mode(int m, int items) {
  g_pair_mode = m;
  if (items > 0) g_pair_items = items;
}

// Tile of a pair launch (both halves share it: one LDS array). Measured pair-table entries
// (tools/conv_tune.py --pairs) carry it in their ``tile`` field: 0 = separate launches,
// 1 = 64x64 (3 LDS stages, 3 blocks per CU), 2 = 128x128 (2 stages, 2 per CU), 3 = 64x128 and
// 4 = 128x64 (3 stages, 2 per CU). The big tiles halve the L2 -> LDS bytes per MFMA of the
// 64x64 tile, which at b256 needs ~2x the L2 read rate its MFMAs could consume.
// 5 = 128x128 with 3 stages (96 KB: one block per CU, two k-steps of prefetch)
constexpr int kPairTiles = 6;
template <int BM, int BN, int NST, bool BNF1, bool SGDM>
static void pair_kernel_launch(const ConvArgs& d, const ConvArgs& w, int itd, int itw,
                               hipStream_t st) {
  hipLaunchKernelGGL((conv_bwd_pair_kernel<BM, BN, NST, BNF1 ? 1 : 0, SGDM>), dim3(itd + itw),
                     dim3(256), 0, st, d, w, itd);
}
template <int BM, int BN, int NST>
static void pair_launch_t(ConvArgs& d, ConvArgs& w, int sd, int sw, float* ws, size_t ws_elems,
                          int* itd_out, int* itw_out, bool* ok_out, const float* dw,
                          bool launch, hipStream_t st) {
  // the slab workspace is split between the two problems
  const int itd = prepare_cfg<MODE_DGRAD, BM, BN>(d, std::max(1, sd));
  size_t dneed = needs_finish(MODE_DGRAD, d) ? (size_t)d.splits * d.Mg * d.Ng : 0;
  dneed = (dneed + 63) / 64 * 64;
  w.ws = ws + dneed;
  const int itw = prepare_cfg<MODE_WGRAD, BM, BN>(w, std::max(1, sw));
  const size_t wneed = needs_finish(MODE_WGRAD, w) ? (size_t)w.splits * w.Mg * w.Ng : 0;
  *itd_out = itd;
  *itw_out = itw;
  *ok_out = dneed + wneed <= ws_elems;
  if (!launch || !*ok_out) return;
  // unsplit WGRAD half: SGD on the master in its epilogue (no finish would take it)
  if (!needs_finish(MODE_WGRAD, w) && w.g.wkrsc && w.g.Creal == w.g.C) w.sgd = sgd_fuse_master(dw);
  const bool bnf1 = d.has_bnf && d.splits <= 1;
  const bool sgdm = w.sgd.p != nullptr;
  if (bnf1 && sgdm) pair_kernel_launch<BM, BN, NST, true, true>(d, w, itd, itw, st);
  else if (bnf1) pair_kernel_launch<BM, BN, NST, true, false>(d, w, itd, itw, st);
  else if (sgdm) pair_kernel_launch<BM, BN, NST, false, true>(d, w, itd, itw, st);
  else pair_kernel_launch<BM, BN, NST, false, false>(d, w, itd, itw, st);
}

extern "C" int ddp_conv_bwd_pair(const ConvGeom* g, const void* dy, const void* wc, void* dx,
                                 const void* x, float* dw, float* ws, size_t ws_elems,
                                 const BnBwdFuse* bn, const BnBwdApply* ba, int* bn_done,
                                 hipStream_t st) {
  if (bn_done) *bn_done = 0;
  if (!bn) ba = nullptr;
  auto separate = [&]() -> int {
    // DGRAD first: the WGRAD finish may then apply the layer's SGD step (g_sgd_allow)
    // (the input block's sums, bn->code, are taken in the pair's finish only)
    const BnBwdFuse* bsep = bn && bn->code ? nullptr : bn;
    const int r = conv_dgrad_impl(g, dy, wc, dx, ws, ws_elems, 0, 0, bsep, bsep ? ba : nullptr,
                                  bn_done, st);
    if (r) return r;
    g_sgd_allow = true;
    const int rw = ddp_conv_wgrad(g, dy, x, dw, ws, ws_elems, 0, st);
    g_sgd_allow = false;
    return rw;
  };
  if (g_pair_mode == 0 || g->stride != 1 || g->C % 8 || g->K % 8 || g->Creal != g->C)
    return separate();
  const size_t dya = (size_t)g->N * g->P * g->Q * g->K, wb = (size_t)g->K * g->R * g->S * g->C;
  const size_t xb = (size_t)g->N * g->H * g->W * g->C;
  if (!fits_buffer(dya) || !fits_buffer(wb) || !fits_buffer(xb)) return separate();
  ConvArgs d{};  // as conv_dgrad_impl (stride 1, no accumulate)
  d.g = *g;
  if (bn) {
    d.has_bnf = 1;
    d.bnf = *bn;
    d.bnapply = ba;
    d.bnapply_done = bn_done;
  }
  d.a = (const unsigned short*)dy;
  d.b = (const unsigned short*)wc;
  d.out = (unsigned short*)dx;
  d.ws = ws;
  d.Mg = g->N * g->H * g->W;
  d.Ng = g->C;
  d.Kg = g->R * g->S * g->K;
  d.a_bytes = (int)(2 * dya);
  d.b_bytes = (int)(2 * wb);
  ConvArgs w{};  // as ddp_conv_wgrad
  w.g = *g;
  if (g->R * g->S == 1) w.g.wkrsc = 1;
  w.a = (const unsigned short*)dy;
  w.b = (const unsigned short*)x;
  w.dw = dw;
  w.ws = ws;
  w.Mg = g->K;
  w.Ng = g->R * g->S * g->C;
  w.Kg = g->N * g->P * g->Q;
  w.a_bytes = (int)(2 * dya);
  w.b_bytes = (int)(2 * xb);
  w.dPQ = make_fastdiv(g->P * g->Q);
  w.dQ = make_fastdiv(g->Q);
  // measured pair entry (tools/conv_tune.py --pairs) or forced splits (its sweep) first
  bool tuned = false;
  int sd = 1, sw = 1, pt = 1;
  if (g_pair_force_dg > 0 && g_pair_force_wg > 0) {
    tuned = true;
    sd = g_pair_force_dg;
    sw = g_pair_force_wg;
  } else if (g_force_tile == 0 && g_pair_mode == 3) {
    auto it = g_pair_tuned.find(TuneKey{MODE_DGRAD, d.Mg, d.Ng, d.Kg, g->H * g->W});
    if (it == g_pair_tuned.end()) it = g_pair_tuned.find(TuneKey{MODE_DGRAD, d.Mg, d.Ng, d.Kg, 0});
    if (it != g_pair_tuned.end()) {
      if (!it->second.tile) return separate();
      tuned = true;
      pt = it->second.tile < kPairTiles ? it->second.tile : 1;
      sd = it->second.splits;
      sw = it->second.stages;
    }
  }
  // dense 2x2 DGRAD (the WGRAD half stays 3x3 and keeps the measured entry's split, so its
  // finish still takes the layer's SGD step): the DGRAD split from the cost model
  if (ddp_conv_dense2x2_ok(g)) {
    dense2x2_args(d, g, MODE_DGRAD);
    if (tuned) tile_cost(64, 64, d, ws_elems, &sd);
  }
  bool both64 = tuned;
  if (!tuned) {
    int spd[kNumTiles], bd, nd, spw[kNumTiles], bw, nw;
    plan_mode<MODE_DGRAD>(d, ws_elems, &bd, spd, &nd);
    plan_mode<MODE_WGRAD>(w, ws_elems, &bw, spw, &nw);
    both64 = bd == 3 && bw == 3;
    if (g_pair_mode == 1 && !both64) return separate();
    sd = spd[3];
    sw = spw[3];
    if (bd != 3) tile_cost(64, 64, d, ws_elems, &sd);
    if (bw != 3) tile_cost(64, 64, w, ws_elems, &sw);
    if (bd == 3 && bw == 3 && g_force_tile == 0) {  // measured splits (plan_mode filled sp[3])
      sd = spd[3];
      sw = spw[3];
    }
  }
  // a dense DGRAD reduces the BatchNorm-backward sums in the finish of its 3x3 view; the input
  // block's sums (bn->code) are taken only in a split-K finish: a split DGRAD costs the pair
  // ~0.5 us where the standalone l0_sums launch it replaces costs 3-6 us (the pair table is
  // measured on the GEMMs alone, tools/conv_tune.py --pairs)
  if (d.d2x2 && d.has_bnf) sd = std::max(sd, 2);
  if (bn && bn->code && !ba && !d.d2x2) sd = std::max(sd, 2);
  // the pair's tile: the measured entry's, a forced one (sweeps), else 64x64; the dense 2x2
  // DGRAD keeps 64x64 (its column tiles pick the weight tap per input pixel)
  if (g_pair_force_tile_req >= 1 && g_pair_force_tile_req < kPairTiles) pt = g_pair_force_tile_req;
  if (d.d2x2) pt = 1;
  // the input block's sums (bn->code) exist only in the split-K finish: without one, or if the
  // pair would fuse the BN backward into that finish, drop them (the caller runs l0_sums).
  // (decided on the prepared DGRAD: a dry run of the tile's prepare step)
  int itd = 0, itw = 0;
  bool fits = false;
  auto prep = [&](bool launch) {
    switch (pt) {
      case 2: pair_launch_t<128, 128, 2>(d, w, sd, sw, ws, ws_elems, &itd, &itw, &fits, dw, launch, st); break;
      case 5: pair_launch_t<128, 128, 3>(d, w, sd, sw, ws, ws_elems, &itd, &itw, &fits, dw, launch, st); break;
      case 3: pair_launch_t<64, 128, 3>(d, w, sd, sw, ws, ws_elems, &itd, &itw, &fits, dw, launch, st); break;
      case 4: pair_launch_t<128, 64, 3>(d, w, sd, sw, ws, ws_elems, &itd, &itw, &fits, dw, launch, st); break;
      default: pair_launch_t<64, 64, 3>(d, w, sd, sw, ws, ws_elems, &itd, &itw, &fits, dw, launch, st); break;
    }
  };
  prep(false);
  if (!fits) return separate();
  if (g_pair_mode == 3 && !both64 && itd + itw > g_pair_items) return separate();
  if (d.d2x2 && d.has_bnf && d.splits < 2) return separate();
  if (bn && bn->code && (!needs_finish(MODE_DGRAD, d) || ba || d.d2x2)) {
    d.has_bnf = 0;
    bn = nullptr;
  }
  const bool l0_sums = d.has_bnf && d.bnf.code != nullptr;  // (a finish exists: checked above)
  prep(true);
  const bool fd = needs_finish(MODE_DGRAD, d), fw = needs_finish(MODE_WGRAD, w);
  struct Allow {  // the finishes below run after both GEMMs of the pair
    Allow() { g_sgd_allow = true; }
    ~Allow() { g_sgd_allow = false; }
  } allow;
  const ConvArgs dv = finish_view(d, g, MODE_DGRAD);  // (d itself unless dense)
  if (fd && fw && w.g.wkrsc && bnbwd_fusable(dv)) {
    const WgFinishArgs wa = wg_finish_args(w);
    launch_finish_bnbwd(dv, st, &wa);
  } else if (fd && fw && w.g.wkrsc) {
    int bx, ch;
    dg_finish_grid(dv, &bx, &ch);
    const FinishArgs fa = finish_args(MODE_DGRAD, dv);
    const WgFinishArgs wa = wg_finish_args(w);
    const dim3 grid(bx * ch + wa.gx * wa.gy);
    if (dv.has_bnf)
      hipLaunchKernelGGL(bwd_pair_finish_kernel<true>, grid, dim3(256), 0, st, fa, bx, ch, wa);
    else
      hipLaunchKernelGGL(bwd_pair_finish_kernel<false>, grid, dim3(256), 0, st, fa, bx, ch, wa);
  } else {
    launch_finish<MODE_DGRAD>(dv, st);
    launch_finish<MODE_WGRAD>(w, st);
  }
  if (l0_sums && bn_done) *bn_done = 2;
  return (int)hipGetLastError();
}

// SGD in the backward: register (dw -> update) pairs (clear = 1 drops the registry first),
// reset / read the set of gradients whose finish took the update since the last begin.
extern "C" void ddp_sgd_fuse_register(float* dw, const SgdFuse* f, int clear) {
  if (clear) g_sgd_reg.clear();
  if (dw && f) g_sgd_reg[dw] = *f;
}
extern "C" void ddp_sgd_fuse_begin() {
  g_sgd_taken.clear();
  g_sgd_master.clear();
}
extern "C" int ddp_sgd_fuse_taken_master(uintptr_t* out, int cap) {
  int n = 0;
  for (const float* p : g_sgd_master) {
    if (n < cap) out[n] = reinterpret_cast<uintptr_t>(p);
    ++n;
  }
  return n;
}
// a WGRAD whose layer runs no DGRAD (the input layer): its finish may apply the SGD step
extern "C" int ddp_conv_wgrad_final(const ConvGeom* g, const void* dy, const void* x, float* dw,
                                    float* ws, size_t ws_elems, int splits, hipStream_t st) {
  g_sgd_allow = true;
  const int r = ddp_conv_wgrad(g, dy, x, dw, ws, ws_elems, splits, st);
  g_sgd_allow = false;
  return r;
}
extern "C" int ddp_sgd_fuse_taken(uintptr_t* out, int cap) {
  int n = 0;
  for (const float* p : g_sgd_taken) {
    if (n < cap) out[n] = reinterpret_cast<uintptr_t>(p);
    ++n;
  }
  return n;
}
