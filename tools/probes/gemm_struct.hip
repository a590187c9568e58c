// Main-loop structure study for the conv GEMM shapes (standalone; no torch, no library code).
//
// C[M][N] = A[M][K] . B[N][K]^T (bf16 operands, fp32 accumulation; bf16 C, or fp32 split-K
// slabs [split][M][N]). Both operands k-contiguous — the conv FWD / DGRAD operand layout with
// the gather removed — staged by LDS-DMA (buffer_load ... lds) into XOR-swizzled [row][64] tiles
// exactly as conv_igemm.hip stages them, v_mfma_f32_16x16x32_bf16, counted vmcnt + s_barrier
// per stage. What varies (template): block tile BM x BN, wave grid WM x WN (4 or 8 waves), LDS
// ring depth NST, and KPB = 64-deep k-sub-tiles per stage (k-steps per barrier).
//
// The question it answers: on VGG-11's GEMM shapes (b256 and b32), which structure gets how
// close to the same-shape hipBLASLt time (tools/probes/roofline.py) — before porting one into
// the gather kernels.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probes/gemm_struct.hip -o /tmp/gemm_struct
//   /tmp/gemm_struct [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned short u16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__device__ __forceinline__ int rk_off(int row, int chunk) {
  return row * 64 + ((chunk ^ ((row >> 1) & 7)) << 3);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t rs, int off, u16* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)lds_wave_base, 16, off, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  if (nwg < 8) return orig;
  const int q = nwg / 8, r = nwg % 8, x = orig % 8, idx = orig / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + idx;
}
__device__ __forceinline__ u16 f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7fff + ((u >> 16) & 1);
  return (u16)(u >> 16);
}

template <int BM, int BN, int WM, int WN, int NST, int KPB>
__global__ __launch_bounds__(64 * WM * WN) void gemm_kernel(const u16* __restrict__ A,
                                                            const u16* __restrict__ B,
                                                            u16* __restrict__ C,
                                                            float* __restrict__ ws, int M, int N,
                                                            int K, int splits) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TA = BM * 64, TB = BN * 64;          // one 64-deep sub-tile
  constexpr int STAGE = KPB * (TA + TB);
  constexpr int CA = BM * 64 / 8 / NT, CB = BN * 64 / 8 / NT;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int DMA = KPB * (CA + CB);
  static_assert(CA >= 1 && CB >= 1 && TM >= 1 && TN >= 1, "tile");
  static_assert(NST >= 2 && NST <= 4, "ring");
  extern __shared__ __attribute__((aligned(16))) u16 smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
  const int item = blockIdx.x;
  const int sp = item / tiles;
  const int tile = xcd_remap(item - sp * tiles, tiles);
  const int row0 = (tile / tiles_n) * BM, col0 = (tile % tiles_n) * BN;
  const int kper = K / splits;                     // multiple of 64 * KPB (host checks)
  const int kbeg = sp * kper;
  const int nk = kper / (64 * KPB);
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, M * K * 2), rsB = make_rsrc(B, N * K * 2);
  const int lc = (tid & 7) ^ ((tid >> 4) & 7);
  int a_off[CA], b_off[CB];
#pragma unroll
  for (int i = 0; i < CA; ++i) a_off[i] = 2 * ((row0 + (tid >> 3) + (NT / 8) * i) * K + lc * 8);
#pragma unroll
  for (int i = 0; i < CB; ++i) b_off[i] = 2 * ((col0 + (tid >> 3) + (NT / 8) * i) * K + lc * 8);

  auto issue = [&](int ks, int slot) {
    u16* st = smem + slot * STAGE;
#pragma unroll
    for (int u = 0; u < KPB; ++u) {
      const int k0 = 2 * (kbeg + (ks * KPB + u) * 64);
      u16* As = st + u * (TA + TB);
      u16* Bs = As + TA;
#pragma unroll
      for (int i = 0; i < CA; ++i) dma(rsA, a_off[i] + k0, As + (wid * 64 + NT * i) * 8);
#pragma unroll
      for (int i = 0; i < CB; ++i) dma(rsB, b_off[i] + k0, Bs + (wid * 64 + NT * i) * 8);
    }
  };
  int fa_off[TM], fb_off[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) fa_off[i] = rk_off(wm * WTM + i * 16 + (lane & 15), lane >> 4);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb_off[j] = rk_off(wn * WTN + j * 16 + (lane & 15), lane >> 4);
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int slot) {
    const u16* st = smem + slot * STAGE;
#pragma unroll
    for (int u = 0; u < KPB; ++u) {
      const u16* As = st + u * (TA + TB);
      const u16* Bs = As + TA;
#pragma unroll
      for (int kk = 0; kk < 64; kk += 32) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(As + (fa_off[i] ^ (kk ? 32 : 0)));
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(Bs + (fb_off[j] ^ (kk ? 32 : 0)));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    }
  };
#pragma unroll
  for (int s = 0; s < NST - 1; ++s)
    if (s < nk) issue(s, s);
  int slot = 0;
  for (int ks = 0; ks < nk; ++ks) {
    const int ahead = nk - 1 - ks;
    if (NST >= 4 && ahead >= 2) wait_barrier<(NST >= 4 ? 2 : 0) * DMA>();
    else if (NST >= 3 && ahead >= 1) wait_barrier<(NST >= 3 ? 1 : 0) * DMA>();
    else wait_barrier<0>();
    if (ks + NST - 1 < nk) issue(ks + NST - 1, slot == 0 ? NST - 1 : slot - 1);
    compute(slot);
    slot = slot + 1 == NST ? 0 : slot + 1;
  }
  const int rl = lane & 15, cq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int row = row0 + wm * WTM + i * 16 + rl;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = col0 + wn * WTN + j * 16 + cq;
      const f32x4 v = acc[i][j];
      if (splits > 1) {
        *reinterpret_cast<float4*>(ws + ((size_t)sp * M + row) * N + col) = (float4){v[0], v[1], v[2], v[3]};
      } else {
        uint2 pk;
        pk.x = (unsigned)f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        pk.y = (unsigned)f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(C + (size_t)row * N + col) = pk;
      }
    }
  }
}

static float bf2f_h(u16 h) {
  unsigned u = (unsigned)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
static u16 f2bf_h(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (u16)(u >> 16);
}

struct Shape {
  const char* name;
  int M, N, K, splits;
};

template <int BM, int BN, int WM, int WN, int NST, int KPB>
static void run(const Shape& s, const u16* dA, const u16* dB, u16* dC, float* dws,
                const std::vector<u16>& hA, const std::vector<u16>& hB, int reps) {
  constexpr int NT = 64 * WM * WN;
  if (s.M % BM || s.N % BN || s.K % (s.splits * 64 * KPB)) return;
  const size_t lds = (size_t)NST * KPB * (BM + BN) * 64 * 2;
  if (lds > 160 * 1024) return;
  auto kern = gemm_kernel<BM, BN, WM, WN, NST, KPB>;
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const int items = (s.M / BM) * (s.N / BN) * s.splits;
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL(kern, dim3(items), dim3(NT), lds, 0, dA, dB, dC, dws, s.M, s.N, s.K, s.splits);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL(kern, dim3(items), dim3(NT), lds, 0, dA, dB, dC, dws, s.M, s.N, s.K, s.splits);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = 1000.0 * ms / reps;
  // spot check 64 outputs against a host fp32 reference (sum of the split slabs when split)
  double maxrel = 0.0;
  std::vector<u16> hC;
  std::vector<float> hws;
  if (s.splits > 1) {
    hws.resize((size_t)s.splits * s.M * s.N);
    CK(hipMemcpy(hws.data(), dws, hws.size() * 4, hipMemcpyDeviceToHost));
  } else {
    hC.resize((size_t)s.M * s.N);
    CK(hipMemcpy(hC.data(), dC, hC.size() * 2, hipMemcpyDeviceToHost));
  }
  for (int t = 0; t < 64; ++t) {
    const int m = (int)((1103515245u * (t + 1) + 12345u) % (unsigned)s.M);
    const int n = (int)((2654435761u * (t + 7)) % (unsigned)s.N);
    double ref = 0.0, mag = 0.0;
    for (int k = 0; k < s.K; ++k) {
      const double p = (double)bf2f_h(hA[(size_t)m * s.K + k]) * bf2f_h(hB[(size_t)n * s.K + k]);
      ref += p;
      mag += std::fabs(p);
    }
    double got = 0.0;
    if (s.splits > 1)
      for (int z = 0; z < s.splits; ++z) got += hws[((size_t)z * s.M + m) * s.N + n];
    else
      got = bf2f_h(hC[(size_t)m * s.N + n]);
    maxrel = std::fmax(maxrel, std::fabs(got - ref) / (mag + 1e-30));
  }
  const double tf = 2.0 * s.M * s.N * s.K / (us * 1e-6) / 1e12;
  std::printf("{\"shape\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"splits\": %d, \"tile\": \"%dx%d\", "
              "\"waves\": \"%dx%d\", \"nst\": %d, \"kpb\": %d, \"lds_kb\": %zu, \"blocks\": %d, "
              "\"us\": %.2f, \"tflops\": %.1f, \"max_rel_err\": %.2e}\n",
              s.name, s.M, s.N, s.K, s.splits, BM, BN, WM, WN, NST, KPB, lds / 1024, items, us, tf,
              maxrel);
  std::fflush(stdout);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 50;
  const Shape shapes[] = {
      {"L3fwd_b256", 16384, 256, 2304, 1}, {"L2fwd_b256", 16384, 256, 1152, 1},
      {"L5fwd_b256", 4096, 512, 4608, 1},  {"L4fwd_b256", 4096, 512, 2304, 1},
      {"L1fwd_b256", 65536, 128, 576, 1},  {"L6fwd_b256", 1024, 512, 4608, 4},
      {"L3wg_b256", 256, 2304, 16384, 8},  {"L5wg_b256", 512, 4608, 4096, 4},
      {"L3fwd_b32", 2048, 256, 2304, 2},   {"L5fwd_b32", 512, 512, 4608, 8},
  };
  size_t maxA = 0, maxB = 0, maxC = 0, maxW = 0;
  for (const Shape& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxB = std::max(maxB, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxW = std::max(maxW, (size_t)s.splits * s.M * s.N);
  }
  std::vector<u16> hA(maxA), hB(maxB);
  unsigned x = 12345u;
  for (auto& v : hA) { x = x * 1664525u + 1013904223u; v = f2bf_h(((x >> 8) & 0xffff) / 32768.f - 1.f); }
  for (auto& v : hB) { x = x * 1664525u + 1013904223u; v = f2bf_h(((x >> 8) & 0xffff) / 32768.f - 1.f); }
  u16 *dA, *dB, *dC;
  float* dws;
  CK(hipMalloc(&dA, maxA * 2));
  CK(hipMalloc(&dB, maxB * 2));
  CK(hipMalloc(&dC, maxC * 2));
  CK(hipMalloc(&dws, maxW * 4));
  CK(hipMemcpy(dA, hA.data(), maxA * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, hB.data(), maxB * 2, hipMemcpyHostToDevice));
  for (const Shape& s : shapes) {
    // (the host reference reads hA / hB with the shape's own M, N, K strides: same buffers)
    run<64, 64, 2, 2, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<64, 128, 2, 2, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 64, 2, 2, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 128, 2, 2, 2, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 128, 2, 2, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 128, 2, 4, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<256, 128, 2, 4, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 256, 2, 4, 3, 1>(s, dA, dB, dC, dws, hA, hB, reps);
    run<64, 64, 2, 2, 3, 2>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 64, 2, 2, 3, 2>(s, dA, dB, dC, dws, hA, hB, reps);
    run<128, 128, 2, 2, 2, 2>(s, dA, dB, dC, dws, hA, hB, reps);
  }
  CK(hipFree(dA));
  CK(hipFree(dB));
  CK(hipFree(dC));
  CK(hipFree(dws));
  return 0;
}
