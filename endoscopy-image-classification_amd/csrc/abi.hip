// Library identity + standalone elementwise fallbacks of the C-ABI (gfx950).
#include "common.h"

namespace {
__global__ void gelu_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (bf16)gelu_f((float)x[i]);
}
__global__ void gelu_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dx[i] = (bf16)((float)dy[i] * gelu_grad_f((float)x[i]));
}
}  // namespace

extern "C" {

#define ES_ABI_VERSION 1
int es_abi_version(void) { return ES_ABI_VERSION; }

int es_gelu_fwd(const void* x, void* y, long n, hipStream_t stream) {
  if (n <= 0) return ES_BAD_SHAPE;
  long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(gelu_fwd_kernel, (int)grid, 256, 0, stream, (const bf16*)x, (bf16*)y, n);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_gelu_bwd(const void* x, const void* dy, void* dx, long n, hipStream_t stream) {
  if (n <= 0) return ES_BAD_SHAPE;
  long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(gelu_bwd_kernel, (int)grid, 256, 0, stream, (const bf16*)x, (const bf16*)dy, (bf16*)dx, n);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
