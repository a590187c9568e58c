// Kernel-boundary cost on MI355X: a hipGraph chain of dependent kernels, each reading the
// previous kernel's output and writing a new buffer (ping-pong), like the BN-apply / split-K
// finish chain of a small-batch training step. Per-kernel time vs bytes moved, store flavour
// (plain vs nontemporal) and grid size; an empty-kernel chain gives the dispatch floor.
//   hipcc --offload-arch=gfx950 -O3 boundary_probe.hip -o boundary_probe && ./boundary_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

__global__ void empty_kernel(int) {}

template <int NT>
__global__ __launch_bounds__(256) void chain_kernel(const float4* __restrict__ in,
                                                    float4* __restrict__ out, int n) {
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    float4 v = in[i];
    v.x = v.x * 1.0001f + 1.f; v.y += 1.f; v.z -= 1.f; v.w *= 0.9999f;
    if (NT) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      f4v w = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(w, reinterpret_cast<f4v*>(out) + i);
    } else {
      out[i] = v;
    }
  }
}

// "statistics" producer: every block reduces its values and adds 2 x 256 per-channel partial
// sums into one of 16 replicas with float atomics (ATOM = 1), or stores them as a per-block
// partial row (ATOM = 0); then a one-block "finalize" sums the replicas / rows per channel.
template <int ATOM>
__global__ __launch_bounds__(256) void stats_kernel(const float* __restrict__ in, float* acc, int nblk) {
  const int c = threadIdx.x;
  float s = in[blockIdx.x * 256 + c], q = s * s;
  if (ATOM) {
    float* rep = acc + (blockIdx.x % 16) * 512;
    atomicAdd(rep + c, s);
    atomicAdd(rep + 256 + c, q);
  } else {
    acc[blockIdx.x * 512 + c] = s;
    acc[blockIdx.x * 512 + 256 + c] = q;
  }
}
template <int ATOM>
__global__ __launch_bounds__(256) void finalize_kernel(float* acc, float* coef, int nblk) {
  const int c = threadIdx.x;
  float s = 0.f, q = 0.f;
  const int rows = ATOM ? 16 : nblk;
  for (int r = 0; r < rows; ++r) { s += acc[r * 512 + c]; q += acc[r * 512 + 256 + c]; }
  coef[c] = s;
  coef[256 + c] = q;
  if (ATOM) for (int r = 0; r < 16; ++r) { acc[r * 512 + c] = 0.f; acc[r * 512 + 256 + c] = 0.f; }
}

int main() {
  const int kChain = 200, kReps = 10;
  const size_t maxn = (16u << 20) / 16;  // 16 MB of float4
  float4 *a, *b;
  CK(hipMalloc(&a, maxn * 16));
  CK(hipMalloc(&b, maxn * 16));
  CK(hipMemset(a, 0, maxn * 16));
  CK(hipMemset(b, 0, maxn * 16));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](int kind, size_t bytes, int grid, float* us) -> int {
    const int n = (int)(bytes / 16);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int k = 0; k < kChain; ++k) {
      const float4* src = (k & 1) ? b : a;
      float4* dst = (k & 1) ? a : b;
      if (kind == 0) hipLaunchKernelGGL(empty_kernel, dim3(grid), dim3(256), 0, s, k);
      else if (kind == 1) hipLaunchKernelGGL(chain_kernel<0>, dim3(grid), dim3(256), 0, s, src, dst, n);
      else hipLaunchKernelGGL(chain_kernel<1>, dim3(grid), dim3(256), 0, s, src, dst, n);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < kReps; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s));
    CK(hipStreamSynchronize(s));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    *us = ms * 1000.f / (kReps * kChain);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
  };
  const char* names[3] = {"empty", "plain", "nontemporal"};
  printf("%-12s %10s %6s %10s\n", "kind", "bytes", "grid", "us/kernel");
  for (int grid : {8, 64, 512}) {
    float us;
    if (run(0, 0, grid, &us)) return 1;
    printf("%-12s %10d %6d %10.2f\n", names[0], 0, grid, us);
    for (size_t bytes : {size_t(16) << 10, size_t(256) << 10, size_t(2) << 20, size_t(8) << 20}) {
      for (int kind : {1, 2}) {
        if (run(kind, bytes, grid, &us)) return 1;
        printf("%-12s %10zu %6d %10.2f\n", names[kind], bytes, grid, us);
      }
    }
  }
  // stats -> finalize pairs (kChain / 2 of each)
  float *in, *acc, *coef;
  CK(hipMalloc(&in, 1024 * 256 * 4));
  CK(hipMalloc(&acc, 1024 * 512 * 4));
  CK(hipMalloc(&coef, 512 * 4));
  CK(hipMemset(in, 0, 1024 * 256 * 4));
  CK(hipMemset(acc, 0, 1024 * 512 * 4));
  for (int atom : {1, 0}) {
    for (int nblk : {16, 64, 256, 1024}) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
      for (int k = 0; k < kChain / 2; ++k) {
        if (atom) {
          hipLaunchKernelGGL(stats_kernel<1>, dim3(nblk), dim3(256), 0, s, in, acc, nblk);
          hipLaunchKernelGGL(finalize_kernel<1>, dim3(1), dim3(256), 0, s, acc, coef, nblk);
        } else {
          hipLaunchKernelGGL(stats_kernel<0>, dim3(nblk), dim3(256), 0, s, in, acc, nblk);
          hipLaunchKernelGGL(finalize_kernel<0>, dim3(1), dim3(256), 0, s, acc, coef, nblk);
        }
      }
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < kReps; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipStreamSynchronize(s));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("stats+finalize %s nblk %5d: %6.2f us per pair\n", atom ? "atomics " : "partials",
             nblk, ms * 1000.f / (kReps * kChain / 2));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
    }
  }
  return 0;
}
