// Shared device helpers for the gfx950 (CDNA4) kernel library.
// Activations are NHWC bf16; master weights / gradients / optimizer state are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "api.h"

namespace ddp_amd {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

// Debug builds (DDP_AMD_DEBUG_BUILD=1 -> -DDDP_AMD_DEBUG, see _build.py): device-side bounds /
// shape checks that print the failing condition and stop the offending thread's work. No-ops
// in release builds. (GPU sanitizers are not available on this pool; this plus
// HIP_LAUNCH_BLOCKING=1 localises a faulting kernel)
#ifdef DDP_AMD_DEBUG
#define DDP_DEVICE_CHECK(cond)                                                              \
  do {                                                                                      \
    if (!(cond)) {                                                                          \
      printf("[ddp_amd debug] %s:%d check failed: %s (block %d thread %d)\n", __FILE__,     \
             __LINE__, #cond, (int)blockIdx.x, (int)threadIdx.x);                           \
      return;                                                                               \
    }                                                                                       \
  } while (0)
#else
#define DDP_DEVICE_CHECK(cond) \
  do {                        \
  } while (0)
#endif

// Replica of a block's BatchNorm-statistics partial sums (api.h kStatRep) and the value it adds:
// release builds spread blocks over the replicas; the deterministic build gives each block its
// own replica and poisons replica 0 with NaN when a grid outgrows kStatRep.
__device__ __forceinline__ int stat_rep(int b) {
#ifdef DDP_AMD_DETERMINISTIC
  return b < kStatRep ? b : 0;
#else
  return b % kStatRep;
#endif
}
__device__ __forceinline__ float stat_val(float v, int b) {
#ifdef DDP_AMD_DETERMINISTIC
  return b < kStatRep ? v : __builtin_nanf("");
#else
  (void)b;
  return v;
#endif
}

// One SGD element update (torch.optim.SGD: d = g + wd p; b = m b + d; d = nesterov ? d + m b : b;
// p -= lr d), with every multiply-add an explicit fma in one fixed order: the optimizer launch
// (optim.hip) and the SGD in the WGRAD finish (conv_igemm.hip) are separate translation units,
// and left to -ffp-contract they round differently (1 ulp; tests/test_gpu_deterministic.py).
__device__ __forceinline__ float sgd_update1(float p, float g, float& b, float lr, float momentum,
                                             float wd, float grad_scale, int nesterov) {
  float d = __builtin_fmaf(wd, p, g * grad_scale);
  if (momentum != 0.f) {
    b = __builtin_fmaf(momentum, b, d);
    d = nesterov ? __builtin_fmaf(momentum, b, d) : b;
  }
  return __builtin_fmaf(-lr, d, p);
}

// bf16 <-> fp32 bit conversions. round-to-nearest-even; NaN kept NaN.
__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float(((unsigned int)h) << 16);
}
// A plain cast lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950 -O3.
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// 16-byte vector load/store of 8 bf16 values as raw u16 lanes.
__device__ __forceinline__ u16x8 ld8(const unsigned short* p) {
  return *reinterpret_cast<const u16x8*>(p);
}
__device__ __forceinline__ void st8(unsigned short* p, u16x8 v) {
  *reinterpret_cast<u16x8*>(p) = v;
}

// DPP lane exchange within each 16-lane row (ctrl: quad_perm / row_half_mirror / row_mirror)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Sum over the 16 lanes of a DPP row, result in every lane of the row: quad_perm [1,0,3,2] and
// [2,3,0,1], row_half_mirror, row_mirror — four DPP adds instead of four ds_bpermute round
// trips through the LDS unit (__shfl_xor).
__device__ __forceinline__ float dpp_sum16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// Full-wave reductions, result in every lane; all 64 lanes must be active (uniform control
// flow): DPP within the rows, then the four row results through v_readlane.
__device__ __forceinline__ float wave_sum(float v) {
  v = dpp_sum16(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD (shared L2) instead of round-robin.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int nx = 8;
  if (nwg < nx) return orig;
  const int q = nwg / nx, r = nwg % nx;
  const int xcd = orig % nx, idx = orig / nx;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Counter-based RNG (splitmix-style 32-bit hash); identical formula in data/synthetic.py.
__host__ __device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du;
  x ^= x >> 15; x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  return hash_u32(a ^ hash_u32(b ^ hash_u32(c + 0x9e3779b9u)));
}

}  // namespace ddp_amd
