// MFMA issue-rate calibration on MI355X: 256 workgroups x WAVES waves, each wave runs ITER x 72
// v_mfma_f32_16x16x32_bf16 on register operands with CH independent accumulator chains.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <int CH, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k(float* out, int iters, float seed) {
  bf16x8 a[12], b;
  for (int i = 0; i < 8; ++i) b[i] = (__bf16)(seed * (threadIdx.x + i));
  for (int j = 0; j < 12; ++j)
    for (int i = 0; i < 8; ++i) a[j][i] = (__bf16)(seed * (j + i + threadIdx.x));
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int t = 0; t < 72 / CH; ++t)
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(t + c) % 12], b, acc[c], 0, 0, 0);
    asm volatile("" : "+v"(b));
  }
  float s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][3];
  if (s == 1.2345f) out[threadIdx.x] = s;
}
template <int CH, int WAVES>
void run(float* out) {
  const int iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k<CH, WAVES>), 256, WAVES * 64, 0, 0, out, iters, 0.01f);
  hipEventRecord(e0);
  hipLaunchKernelGGL((k<CH, WAVES>), 256, WAVES * 64, 0, 0, out, iters, 0.01f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double flop = 256.0 * WAVES * iters * 72 * 16384.0;
  printf("chains %2d waves/CU %d: %.3f ms  %.0f TF/s  (%.2f of 2516.6)\n", CH, WAVES, ms, flop / ms / 1e9, flop / ms / 1e9 / 2516.6);
}
int main() {
  float* out; hipMalloc(&out, 4096);
  run<3, 8>(out); run<6, 8>(out); run<12, 8>(out); run<3, 4>(out); run<6, 4>(out); run<12, 4>(out);
  run<3, 16>(out); run<6, 16>(out);
  return 0;
}
