// Implicit-GEMM convolution for gfx950: forward, backward-data and backward-weight on bf16
// MFMA (v_mfma_f32_16x16x32_bf16) with fp32 accumulation, LDS-tiled, register-staged
// prefetch, optional split-K, XCD-aware tile order.
//
// Reference parity: replaces the ATen/oneDNN Conv2d fwd/bwd the reference triggers from
// part1/model.py:18-23 (3x3 s1 p1 + bias) — see SURVEY.md §2.B N1 and §2.D for shapes.
// Also serves ResNet-50's 1x1 / 3x3 / 7x7, stride 1/2 convolutions.
//
// Layouts (all NHWC, channels innermost, C % 8 == 0 — layer 0 is zero-padded 3 -> 8):
//   x  [N][H][W][C]      bf16  activations
//   y  [N][P][Q][K]      bf16  conv output (pre-BN)
//   Wc [K][R][S][C]      bf16  forward weight copy   (GEMM B operand, k-contiguous)
//   Wt [C][R][S][K]      bf16  dgrad weight copy     (GEMM B operand, k-contiguous)
//   dW [K][Creal][R][S]  fp32  PyTorch-layout weight gradient (accumulated, atomics)
//
// GEMM views (rows x cols, reduction):
//   FWD   : M=N*P*Q, N=K,      red=R*S*C   A=im2col(x)  B=Wc
//   DGRAD : M=N*H*W, N=C,      red=R*S*K   A=col2im-gather(dy) B=Wt
//   WGRAD : M=K,     N=R*S*C,  red=N*P*Q   A=dy^T       B=im2col(x)^T  (transposed in LDS)
#include "common.h"
#include "api.h"
#include <algorithm>

namespace ddp_amd {

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct ConvArgs {
  ConvGeom g;
  const unsigned short* a;   // FWD: x, DGRAD: dy, WGRAD: dy
  const unsigned short* b;   // FWD: Wc, DGRAD: Wt, WGRAD: x
  unsigned short* out;       // FWD: y, DGRAD: dx (bf16), unused for WGRAD
  float* out_f32;            // split-K workspace (FWD/DGRAD) or dW (WGRAD)
  const float* bias;         // FWD only (may be null)
  float* stats;              // FWD only: [2*K] sum / sum-of-squares of the bf16 output (may be null)
  int Mg, Ng, Kg;            // GEMM dims
  int splits;                // split-K factor (gridDim.z)
  int ksteps_per_split;
};

template <int MODE, int BM, int BN, int BK>
struct TileLoader {
  // chunks of 8 bf16 (16 B) per thread per operand tile
  static constexpr int CA = BM * BK / 8 / 256;
  static constexpr int CB = BN * BK / 8 / 256;
  static_assert(CA >= 1 && CB >= 1, "tile too small for 256 threads");
};

// Gather one 16-byte chunk of the A operand.
//   FWD/DGRAD: row = GEMM row (pixel), kk = reduction index (multiple of 8)
//   WGRAD    : row = output channel group start (multiple of 8), kk = pixel index m
template <int MODE>
__device__ __forceinline__ u16x8 load_a(const ConvArgs& A, int row, int kk) {
  const ConvGeom& g = A.g;
  u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  if (MODE == MODE_FWD) {
    if (row >= A.Mg || kk >= A.Kg) return z;
    const int pq = g.P * g.Q;
    const int n = row / pq, rem = row - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    const int rs = kk / g.C, c = kk - rs * g.C;
    const int r = rs / g.S, s = rs - r * g.S;
    const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return z;
    return ld8(A.a + ((size_t)(n * g.H + h) * g.W + w) * g.C + c);
  } else if (MODE == MODE_DGRAD) {
    if (row >= A.Mg || kk >= A.Kg) return z;
    const int hw = g.H * g.W;
    const int n = row / hw, rem = row - n * hw;
    const int h = rem / g.W, w = rem - h * g.W;
    const int rs = kk / g.K, ko = kk - rs * g.K;
    const int r = rs / g.S, s = rs - r * g.S;
    int ph = h + g.pad - r, pw = w + g.pad - s;
    if (ph < 0 || pw < 0) return z;
    if (g.stride != 1) {
      if ((ph % g.stride) | (pw % g.stride)) return z;
      ph /= g.stride; pw /= g.stride;
    }
    if (ph >= g.P || pw >= g.Q) return z;
    return ld8(A.a + ((size_t)(n * g.P + ph) * g.Q + pw) * g.K + ko);
  } else {  // WGRAD: A'[kout][m] = dy[m][kout]  (row = kout group start, kk = m)
    if (row >= A.Mg || kk >= A.Kg) return z;
    return ld8(A.a + (size_t)kk * g.K + row);
  }
}

template <int MODE>
__device__ __forceinline__ u16x8 load_b(const ConvArgs& A, int col, int kk) {
  const ConvGeom& g = A.g;
  u16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  if (MODE == MODE_FWD || MODE == MODE_DGRAD) {
    if (col >= A.Ng || kk >= A.Kg) return z;
    return ld8(A.b + (size_t)col * A.Kg + kk);
  } else {  // WGRAD: B'[j=(r,s,c)][m] = x[n][p*st-pad+r][q*st-pad+s][c]  (col = j group start, kk = m)
    if (col >= A.Ng || kk >= A.Kg) return z;
    const int pq = g.P * g.Q;
    const int n = kk / pq, rem = kk - n * pq;
    const int p = rem / g.Q, q = rem - p * g.Q;
    const int rs = col / g.C, c = col - rs * g.C;
    const int r = rs / g.S, s = rs - r * g.S;
    const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
    if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) return z;
    return ld8(A.b + ((size_t)(n * g.H + h) * g.W + w) * g.C + c);
  }
}

template <int MODE, int BM, int BN, int BK>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs args) {
  constexpr int LDK = BK + 8;            // padded LDS row (bf16 elements), 16-B aligned rows
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int CA = TileLoader<MODE, BM, BN, BK>::CA;
  constexpr int CB = TileLoader<MODE, BM, BN, BK>::CB;
  __shared__ __attribute__((aligned(16))) unsigned short smem[(BM + BN) * LDK];
  unsigned short* As = smem;
  unsigned short* Bs = smem + BM * LDK;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_n = (args.Ng + BN - 1) / BN;
  const int tiles_m = (args.Mg + BM - 1) / BM;
  const int tile = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;

  const int ksteps = (args.Kg + BK - 1) / BK;
  const int ks_begin = blockIdx.z * args.ksteps_per_split;
  const int ks_end = min(ksteps, ks_begin + args.ksteps_per_split);
  if (ks_begin >= ks_end) return;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u16x8 ra[CA], rb[CB];

  auto gload = [&](int ks) {
    const int k0 = ks * BK;
    if (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + i * 256;
        const int r = c / (BK / 8), kc = c - r * (BK / 8);
        ra[i] = load_a<MODE>(args, row0 + r, k0 + kc * 8);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + i * 256;
        const int r = c / (BK / 8), kc = c - r * (BK / 8);
        rb[i] = load_b<MODE>(args, col0 + r, k0 + kc * 8);
      }
    } else {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + i * 256;
        const int m = c / (BM / 8), grp = c - m * (BM / 8);
        ra[i] = load_a<MODE>(args, row0 + grp * 8, k0 + m);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + i * 256;
        const int m = c / (BN / 8), grp = c - m * (BN / 8);
        rb[i] = load_b<MODE>(args, col0 + grp * 8, k0 + m);
      }
    }
  };

  auto lstore = [&]() {
    if (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + i * 256;
        const int r = c / (BK / 8), kc = c - r * (BK / 8);
        st8(As + r * LDK + kc * 8, ra[i]);
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + i * 256;
        const int r = c / (BK / 8), kc = c - r * (BK / 8);
        st8(Bs + r * LDK + kc * 8, rb[i]);
      }
    } else {  // transpose into [row][k] while writing LDS
#pragma unroll
      for (int i = 0; i < CA; ++i) {
        const int c = tid + i * 256;
        const int m = c / (BM / 8), grp = c - m * (BM / 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) As[(grp * 8 + e) * LDK + m] = ra[i][e];
      }
#pragma unroll
      for (int i = 0; i < CB; ++i) {
        const int c = tid + i * 256;
        const int m = c / (BN / 8), grp = c - m * (BN / 8);
#pragma unroll
        for (int e = 0; e < 8; ++e) Bs[(grp * 8 + e) * LDK + m] = rb[i][e];
      }
    }
  };

  gload(ks_begin);
  for (int ks = ks_begin; ks < ks_end; ++ks) {
    __syncthreads();
    lstore();
    __syncthreads();
    if (ks + 1 < ks_end) gload(ks + 1);
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const unsigned short* p = As + (wm * WTM + i * 16 + (lane & 15)) * LDK + kk + 8 * (lane >> 4);
        fa[i] = *reinterpret_cast<const bf16x8*>(p);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const unsigned short* p = Bs + (wn * WTN + j * 16 + (lane & 15)) * LDK + kk + 8 * (lane >> 4);
        fb[j] = *reinterpret_cast<const bf16x8*>(p);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
  }

  // ---------------- epilogue ----------------
  const ConvGeom& g = args.g;
  const bool split = args.splits > 1;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = col0 + wn * WTN + j * 16 + (lane & 15);
    const bool cok = col < args.Ng;
    float bias = 0.f;
    if (MODE == MODE_FWD && !split && args.bias && cok) bias = args.bias[col];
    float s = 0.f, ss = 0.f;
    // WGRAD output decomposition of col = (r, s, c)
    int wr = 0, wsx = 0, wc = 0;
    if (MODE == MODE_WGRAD) {
      const int rs = col / g.C;
      wc = col - rs * g.C;
      wr = rs / g.S;
      wsx = rs - wr * g.S;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = row0 + wm * WTM + i * 16 + 4 * (lane >> 4) + v;
        if (!cok || row >= args.Mg) continue;
        const float val = acc[i][j][v];
        if (MODE == MODE_WGRAD) {
          if (wc < g.Creal)
            atomicAdd(args.out_f32 + (((size_t)row * g.Creal + wc) * g.R + wr) * g.S + wsx, val);
        } else if (split) {
          atomicAdd(args.out_f32 + (size_t)row * args.Ng + col, val);
        } else {
          const unsigned short h = f2bf(val + bias);
          args.out[(size_t)row * args.Ng + col] = h;
          if (MODE == MODE_FWD) {
            const float r = bf2f(h);
            s += r;
            ss += r * r;
          }
        }
      }
    }
    if (MODE == MODE_FWD && !split && args.stats) {
      s += __shfl_xor(s, 16, kWave);
      s += __shfl_xor(s, 32, kWave);
      ss += __shfl_xor(ss, 16, kWave);
      ss += __shfl_xor(ss, 32, kWave);
      if ((lane >> 4) == 0 && cok) {
        atomicAdd(args.stats + col, s);
        atomicAdd(args.stats + args.Ng + col, ss);
      }
    }
  }
}

// Split-K finish: fp32 workspace -> (+bias) bf16 output (+ per-channel stats for FWD).
// Thread layout: cg_local = tid % Gb (8 channels each), rows strided; the per-channel sums are
// reduced in registers, then across the block through LDS, then ONE atomic per channel per block.
// Grid: x = row blocks, y = channel chunks of Gb groups.
__global__ __launch_bounds__(256) void splitk_finish_kernel(const float* ws, unsigned short* out,
                                                            const float* bias, float* stats,
                                                            int Mg, int Ng) {
  __shared__ float red[2][8][256];
  const int G = Ng / 8;
  const int Gb = G < 256 ? G : 256;
  const int cgl = threadIdx.x % Gb, prow = threadIdx.x / Gb, prows = 256 / Gb;
  const int cg = blockIdx.y * Gb + cgl;
  float s[8], ss[8], bv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    s[e] = 0.f;
    ss[e] = 0.f;
    bv[e] = (bias && cg < G) ? bias[cg * 8 + e] : 0.f;
  }
  const bool active = prow < prows && cg < G;  // Gb need not divide 256 (e.g. 1000 classes)
  for (int row = blockIdx.x * prows + prow; active && row < Mg; row += gridDim.x * prows) {
    const float4* src = reinterpret_cast<const float4*>(ws + (size_t)row * Ng + cg * 8);
    const float4 a = src[0], b = src[1];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = f2bf(v[e] + bv[e]);
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
    atomicAdd(stats + k * Ng + (blockIdx.y * Gb + c) * 8 + e, t);
  }
}

}  // namespace ddp_amd

// ------------------------------- host launcher -------------------------------
using namespace ddp_amd;

template <int MODE, int BM, int BN, int BK>
static void launch_cfg(ConvArgs& a, int target_blocks, hipStream_t st) {
  const int tiles = ((a.Mg + BM - 1) / BM) * ((a.Ng + BN - 1) / BN);
  const int ksteps = (a.Kg + BK - 1) / BK;
  int splits = 1;
  if (a.splits <= 0) {  // auto split-K: fill the chip, keep >= 4 k-steps per split
    splits = (target_blocks + tiles - 1) / tiles;
    splits = max(1, min(splits, ksteps / 4));
  } else {
    splits = min(a.splits, ksteps);
  }
  if (MODE != MODE_WGRAD && splits > 1 && a.out_f32 == nullptr) splits = 1;  // no workspace
  const int per = (ksteps + splits - 1) / splits;
  splits = (ksteps + per - 1) / per;
  a.splits = splits;
  a.ksteps_per_split = per;
  if (MODE != MODE_WGRAD && splits > 1)
    (void)hipMemsetAsync(a.out_f32, 0, sizeof(float) * (size_t)a.Mg * a.Ng, st);
  dim3 grid(tiles, 1, splits);
  hipLaunchKernelGGL((conv_igemm_kernel<MODE, BM, BN, BK>), grid, dim3(256), 0, st, a);
  if (MODE != MODE_WGRAD && splits > 1) {
    const int G = a.Ng / 8;
    const int Gb = G < 256 ? G : 256;
    const int chunks = (G + Gb - 1) / Gb;
    const int rows_per_block = 256 / Gb;
    // ~8 rows per thread keeps the per-block atomics cheap while filling the chip
    int bx = (a.Mg + rows_per_block * 8 - 1) / (rows_per_block * 8);
    bx = std::max(1, std::min(bx, 1024 / chunks + 1));
    hipLaunchKernelGGL(splitk_finish_kernel, dim3(bx, chunks), dim3(256), 0, st, a.out_f32, a.out,
                       MODE == MODE_FWD ? a.bias : nullptr, MODE == MODE_FWD ? a.stats : nullptr,
                       a.Mg, a.Ng);
  }
}

template <int MODE>
static void launch_mode(ConvArgs& a, hipStream_t st) {
  const long long area = (long long)a.Mg * a.Ng;
  const int target = 1024;  // >= 4 workgroups per CU on 256 CUs
  if (area >= (long long)128 * 128 * 512)
    launch_cfg<MODE, 128, 128, 32>(a, target, st);
  else
    launch_cfg<MODE, 64, 64, 32>(a, target, st);
}

extern "C" int ddp_conv_fwd(const ConvGeom* g, const void* x, const void* wc, const float* bias,
                            void* y, float* stats, float* ws, int splits, hipStream_t st) {
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)x;
  a.b = (const unsigned short*)wc;
  a.out = (unsigned short*)y;
  a.out_f32 = ws;
  a.bias = bias;
  a.stats = stats;
  a.Mg = g->N * g->P * g->Q;
  a.Ng = g->K;
  a.Kg = g->R * g->S * g->C;
  a.splits = splits;
  launch_mode<MODE_FWD>(a, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_dgrad(const ConvGeom* g, const void* dy, const void* wt, void* dx,
                              float* ws, int splits, hipStream_t st) {
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)dy;
  a.b = (const unsigned short*)wt;
  a.out = (unsigned short*)dx;
  a.out_f32 = ws;
  a.Mg = g->N * g->H * g->W;
  a.Ng = g->C;
  a.Kg = g->R * g->S * g->K;
  a.splits = splits;
  launch_mode<MODE_DGRAD>(a, st);
  return (int)hipGetLastError();
}

extern "C" int ddp_conv_wgrad(const ConvGeom* g, const void* dy, const void* x, float* dw,
                              int splits, hipStream_t st) {
  ConvArgs a{};
  a.g = *g;
  a.a = (const unsigned short*)dy;
  a.b = (const unsigned short*)x;
  a.out_f32 = dw;
  a.Mg = g->K;
  a.Ng = g->R * g->S * g->C;
  a.Kg = g->N * g->P * g->Q;
  a.splits = splits;
  launch_mode<MODE_WGRAD>(a, st);
  return (int)hipGetLastError();
}
