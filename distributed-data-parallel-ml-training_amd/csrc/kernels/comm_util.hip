// Small kernels used by the gradient-synchronisation strategies (gfx950).
//
// mean_ws : 2A rank-0 averaging — out[i] = (sum_k in[k][i]) / ws over the gathered
//           [ws][n] buffer (reference: torch.mean(torch.stack(list), dim=0),
//           part2/part2a/main.py:108).
// scale   : x *= s (2B's `param.grad /= world_size`, part2/part2b/main.py:103, when the
//           backend has no native average).
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

}  // namespace ddp_amd

using namespace ddp_amd;

static unsigned blocks_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int ddp_mean_ws(const float* in, size_t n, int ws, float* out, hipStream_t st) {
  hipLaunchKernelGGL(mean_ws_kernel, dim3(blocks_for(n)), dim3(256), 0, st, in, n, ws, out);
  return (int)hipGetLastError();
}

extern "C" int ddp_scale(float* x, size_t n, float s, hipStream_t st) {
  hipLaunchKernelGGL(scale_kernel, dim3(blocks_for(n)), dim3(256), 0, st, x, n, s);
  return (int)hipGetLastError();
}
