// Small kernels used by the gradient-synchronisation strategies (gfx950).
//
// mean_ws : 2A rank-0 averaging — out[i] = (sum_k in[k][i]) / ws over the gathered
//           [ws][n] buffer (reference: torch.mean(torch.stack(list), dim=0),
//           part2/part2a/main.py:108).
// scale   : x *= s (2B's `param.grad /= world_size`, part2/part2b/main.py:103, when the
//           backend has no native average).
// comm_standin : world-1 stand-in for a collective (overlap studies on one GPU): a few blocks
//           (like RCCL's channels) make one read+write pass over the bucket and hold their
//           CUs until the modelled transfer time has elapsed since the kernel started
//           (s_sleep on the constant clock).
// flag_signal / flag_wait : device-side stream edge between the step graph and the comm stream
//           (engine/step.py SegmentedDDPStep): signal = one agent-scope release increment of a
//           counter; wait = one wave spins (s_sleep) until the counter reaches the next expected
//           value (its own monotonic counter), acquire. Bounded: after `timeout` it records an
//           error code and returns instead of hanging the GPU.
// pack / unpack bf16 : fp32 gradient bucket <-> bf16 communication buffer (DDP with
//           grad_comm_dtype="bf16": half the bytes on the xGMI links; like PyTorch's
//           bf16_compress_hook). Round-to-nearest-even on the way in, exact widening back.
#include "common.h"
#include "api.h"

namespace ddp_amd {

__global__ __launch_bounds__(256) void mean_ws_kernel(const float* __restrict__ in, size_t n,
                                                      int ws, float* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const float inv = 1.f / (float)ws;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float s = 0.f;
    for (int k = 0; k < ws; ++k) s += in[(size_t)k * n + i];
    out[i] = s * inv;
  }
}

__global__ __launch_bounds__(256) void scale_kernel(float* x, size_t n, float s) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= s;
}

__global__ __launch_bounds__(256) void comm_standin_kernel(float* x, size_t n, long long ticks,
                                                           float scale, int passes) {
  // one read + write pass over the bucket, then hold the CU until the modelled time has
  // elapsed since the kernel started: the modelled collective time INCLUDES its own memory
  // traffic, as an RCCL kernel's does (until round 4 the pass ran after the full wait, adding
  // ~20-30 us per 19 MB bucket on top of the model).
  // scale != 1 (tests): the scaling pass is the LAST thing the kernel does, after the whole
  // modelled time — a consumer that does not wait for the collective reads the old values.
  // passes > 1 ("busy" stand-in): that many paced read + write passes spread over the modelled
  // time instead of one pass and a sleep — the memory traffic of a live collective (a ring
  // all-reduce reads and writes its bucket ~2 (w-1)/w times each way) beside the backward
  const long long t0 = wall_clock64();
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (int p = 0; p < passes; ++p) {
    const float sc = p == passes - 1 ? scale : 1.f;
    const long long until = t0 + ticks * (p + 1) / passes;
    const bool late = sc != 1.f;  // write late: wait first
    if (late)
      while (wall_clock64() - until < 0) __builtin_amdgcn_s_sleep(4);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n / 4; i += stride) {
      float4 v = reinterpret_cast<float4*>(x)[i];
      v.x *= sc; v.y *= sc; v.z *= sc; v.w *= sc;
      asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w));  // keep the store at scale 1
      reinterpret_cast<float4*>(x)[i] = v;
    }
    if (blockIdx.x == 0)
      for (size_t i = (n / 4) * 4 + threadIdx.x; i < n; i += blockDim.x) x[i] *= sc;
    if (!late)
      while (wall_clock64() - until < 0) __builtin_amdgcn_s_sleep(4);
  }
}

__global__ __launch_bounds__(64) void flag_signal_kernel(unsigned* flag) {
  if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void flag_wait_kernel(const unsigned* flag, unsigned* expected,
                                                       unsigned* err, long long timeout_ticks) {
  if (threadIdx.x != 0) return;
  // vector load/store of the private counter (never a scalar-cache read of a value this kernel
  // itself rewrites every launch)
  const unsigned target = __hip_atomic_load(expected, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  __hip_atomic_store(expected, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const long long t0 = wall_clock64();
  while ((int)(__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
    if (wall_clock64() - t0 > timeout_ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// copy / fill used by the communicator instead of hipMemcpyAsync / hipMemsetAsync: inside a
// captured step those become memcpy / memset graph nodes, and a captured memset node was seen
// not to order before its readers on ROCm 7 (profiles/r3_conv_occupancy.md section 6) — a
// kernel node is ordered like every other kernel of the stream
__global__ __launch_bounds__(256) void copy_bytes_kernel(unsigned char* __restrict__ dst,
                                                         const unsigned char* __restrict__ src,
                                                         size_t n, int vec) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t head = 0;
  if (vec) {
    const size_t n16 = n / 16;
    for (size_t i = i0; i < n16; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    head = n16 * 16;
  }
  for (size_t i = head + i0; i < n; i += stride) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void fill_bytes_kernel(unsigned char* __restrict__ dst,
                                                         unsigned v, size_t n, int vec) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t i0 = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t head = 0;
  if (vec) {
    const unsigned w = v * 0x01010101u;
    const size_t n16 = n / 16;
    for (size_t i = i0; i < n16; i += stride)
      reinterpret_cast<uint4*>(dst)[i] = (uint4){w, w, w, w};
    head = n16 * 16;
  }
  for (size_t i = head + i0; i < n; i += stride) dst[i] = (unsigned char)v;
}

__global__ __launch_bounds__(256) void pack_bf16_kernel(const float* __restrict__ x, size_t n,
                                                        unsigned short* __restrict__ y) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    uint2 o;
    o.x = (unsigned)f2bf(v.x) | ((unsigned)f2bf(v.y) << 16);
    o.y = (unsigned)f2bf(v.z) | ((unsigned)f2bf(v.w) << 16);
    reinterpret_cast<uint2*>(y)[i] = o;
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = f2bf(x[i]);
}

__global__ __launch_bounds__(256) void unpack_bf16_kernel(const unsigned short* __restrict__ y,
                                                          size_t n, float* __restrict__ x) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const uint2 v = reinterpret_cast<const uint2*>(y)[i];
    reinterpret_cast<float4*>(x)[i] = (float4){bf2f((unsigned short)(v.x & 0xffff)),
                                               bf2f((unsigned short)(v.x >> 16)),
                                               bf2f((unsigned short)(v.y & 0xffff)),
                                               bf2f((unsigned short)(v.y >> 16))};
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += stride)
    x[i] = bf2f(y[i]);
}

// fp32 segment copy: one block per {src_index, dst_index, count} entry (the sharded update's
// unpack of the gathered small-tensor slots into the parameter arena)
__global__ __launch_bounds__(256) void seg_copy_f32_kernel(const int4* __restrict__ table,
                                                           const float* __restrict__ src,
                                                           float* __restrict__ dst) {
  const int4 e = table[blockIdx.x];
  const float* s = src + (size_t)(unsigned)e.x;
  float* d = dst + (size_t)(unsigned)e.y;
  for (int i = threadIdx.x; i < e.z; i += 256) d[i] = s[i];
}

}  // namespace ddp_amd

using namespace ddp_amd;

extern "C" int ddp_seg_copy_f32(const void* table, int n, const float* src, float* dst,
                                hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(seg_copy_f32_kernel, dim3(n), dim3(256), 0, st, (const int4*)table, src, dst);
  return (int)hipGetLastError();
}

static unsigned blocks_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

static int wall_khz() {
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
      khz = 100000;
  }
  return khz;
}

extern "C" int ddp_mean_ws(const float* in, size_t n, int ws, float* out, hipStream_t st) {
  hipLaunchKernelGGL(mean_ws_kernel, dim3(blocks_for(n)), dim3(256), 0, st, in, n, ws, out);
  return (int)hipGetLastError();
}

extern "C" int ddp_copy_bytes(void* dst, const void* src, size_t n, hipStream_t st) {
  if (n == 0 || dst == src) return 0;
  const int vec = ((uintptr_t)dst % 16 == 0 && (uintptr_t)src % 16 == 0) ? 1 : 0;
  hipLaunchKernelGGL(copy_bytes_kernel, dim3(blocks_for(vec ? n / 16 + 1 : n)), dim3(256), 0, st,
                     (unsigned char*)dst, (const unsigned char*)src, n, vec);
  return (int)hipGetLastError();
}

extern "C" int ddp_fill_bytes(void* dst, int value, size_t n, hipStream_t st) {
  if (n == 0) return 0;
  const int vec = (uintptr_t)dst % 16 == 0 ? 1 : 0;
  hipLaunchKernelGGL(fill_bytes_kernel, dim3(blocks_for(vec ? n / 16 + 1 : n)), dim3(256), 0, st,
                     (unsigned char*)dst, (unsigned)(value & 0xff), n, vec);
  return (int)hipGetLastError();
}

extern "C" int ddp_scale(float* x, size_t n, float s, hipStream_t st) {
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n)), dim3(256), 0, st, x, n, s);
  return (int)hipGetLastError();
}

extern "C" int ddp_comm_standin(float* x, size_t n, int blocks, float usec, float scale,
                                int passes, hipStream_t st) {
  const int khz = wall_khz();
  if ((uintptr_t)x % 16) return -1;
  const long long ticks = (long long)((double)usec * khz / 1000.0);
  hipLaunchKernelGGL(comm_standin_kernel, dim3(blocks < 1 ? 1 : blocks), dim3(256), 0, st, x, n, ticks,
                     scale, passes < 1 ? 1 : passes);
  return (int)hipGetLastError();
}

extern "C" int ddp_flag_signal(unsigned* flag, hipStream_t st) {
  hipLaunchKernelGGL(flag_signal_kernel, dim3(1), dim3(64), 0, st, flag);
  return (int)hipGetLastError();
}

extern "C" int ddp_flag_wait(const unsigned* flag, unsigned* expected, unsigned* err,
                             float timeout_s, hipStream_t st) {
  const long long ticks = (long long)((double)timeout_s * wall_khz() * 1000.0);
  hipLaunchKernelGGL(flag_wait_kernel, dim3(1), dim3(64), 0, st, flag, expected, err, ticks);
  return (int)hipGetLastError();
}

// x / y must be 16- / 8-byte aligned (arena tensors start on 64-element boundaries, so every
// bucket does); a count that is not a multiple of 4 is finished by the scalar tail loop
extern "C" int ddp_pack_bf16(const float* x, size_t n, unsigned short* y, hipStream_t st) {
  if ((uintptr_t)x % 16 || (uintptr_t)y % 8) return -1;
  hipLaunchKernelGGL(pack_bf16_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, st, x, n, y);
  return (int)hipGetLastError();
}

extern "C" int ddp_unpack_bf16(const unsigned short* y, size_t n, float* x, hipStream_t st) {
  if ((uintptr_t)x % 16 || (uintptr_t)y % 8) return -1;
  hipLaunchKernelGGL(unpack_bf16_kernel, dim3(blocks_for(n / 4 + 1)), dim3(256), 0, st, y, n, x);
  return (int)hipGetLastError();
}
