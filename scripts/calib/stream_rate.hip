// Streaming calibration (all accesses coalesced: lane i touches element r*n+i of stream r) on MI355X (round 6): what HBM rate a kernel with no arithmetic reaches for the read : write
// byte mixes of the ViT step's GEMMs / LayerNorms / attention, and for the weight-stationary GEMM's store pattern.
//   mix R:W   read R x 16 B and write W x 16 B per lane-iteration, grid-stride over a buffer far larger than the
//             256-MiB Infinity Cache, plain loads / stores (nt: non-temporal stores)
//   seg32     the K = 384 GEMM's bytes with C stored as 16 rows x 32 B per store instruction (8 B / lane) and A
//             read once per 384-column group (the weight-stationary kernel's memory pattern, no MFMA)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int R, int W, bool NT>
__global__ __launch_bounds__(256) void mix(const u32x4* __restrict__ A, u32x4* __restrict__ C, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    u32x4 s = u32x4{1u, 2u, 3u, 4u};
#pragma unroll
    for (int r = 0; r < R; ++r) s += A[r * n + i];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      if constexpr (NT) __builtin_nontemporal_store(s + (unsigned)w, C + w * n + i);
      else C[w * n + i] = s + (unsigned)w;
    }
    if constexpr (W == 0) if (s[0] == 0x12345u) C[i] = s;  // keeps the loads of the read-only case
  }
}
__global__ void seg32(const u32x4* __restrict__ A, char* __restrict__ C, int M) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int tiles = M / 32;
  for (int t = blockIdx.x; t < tiles * 3; t += gridDim.x) {
    const int rt = t / 3, cgp = t % 3;
    const u32x4 s = A[((long)rt * 32 * 48) + threadIdx.x] + A[((long)rt * 32 * 48) + 512 + threadIdx.x] +
                    A[((long)rt * 32 * 48) + 1024 + threadIdx.x];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const long row = (long)rt * 32 + rb * 16 + r;
        const int col = cgp * 384 + w * 48 + 16 * j + 4 * g;
        *(u32x2*)(C + (row * 1152 + col) * 2) = u32x2{s[0] + j, s[1] + rb};
      }
  }
}
// row768: the same bytes with the C tile stored row-contiguous (32 rows x 768 B, 16 B / lane), as an LDS-staged
// epilogue of the weight-stationary kernel would store it
__global__ void row768(const u32x4* __restrict__ A, char* __restrict__ C, int M) {
  const int tiles = M / 32;
  for (int t = blockIdx.x; t < tiles * 3; t += gridDim.x) {
    const int rt = t / 3, cgp = t % 3;
    const u32x4 s = A[((long)rt * 32 * 48) + threadIdx.x] + A[((long)rt * 32 * 48) + 512 + threadIdx.x] +
                    A[((long)rt * 32 * 48) + 1024 + threadIdx.x];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const int e = p * 512 + threadIdx.x;  // 16-B piece of the 32 x 768 B tile
      const long row = (long)rt * 32 + e / 48;
      *(u32x4*)(C + row * 2304 + cgp * 768 + (e % 48) * 16) = s + (unsigned)p;
    }
  }
}
int main() {
  const long bytes = 1L << 30;  // 1 GiB per buffer
  u32x4 *A, *C;
  if (hipMalloc(&A, bytes) != hipSuccess || hipMalloc(&C, bytes) != hipSuccess) return 1;
  (void)hipMemset(A, 1, bytes);
  (void)hipMemset(C, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  auto tm = [&](const char* name, auto launch, double nbytes) {
    launch(); (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0); for (int i = 0; i < 10; ++i) launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 10;
    printf("%-14s %8.1f us  %5.2f TB/s\n", name, ms * 1e3, nbytes / ms / 1e9);
  };
  const int grid = 8192;
#define MIX(R, W, NT, NAME)                                                                                  \
  {                                                                                                          \
    const long n = bytes / 16 / (R > W ? R : W);                                                             \
    tm(NAME, [&] { hipLaunchKernelGGL((mix<R, W, NT>), grid, 256, 0, 0, A, C, n); }, (double)n * 16 * (R + W)); \
  }
  MIX(1, 0, false, "read 1:0")
  MIX(0, 1, false, "write 0:1")
  MIX(0, 1, true, "write nt 0:1")
  MIX(1, 1, false, "mix 1:1")
  MIX(1, 1, true, "mix nt 1:1")
  MIX(2, 1, false, "mix 2:1")
  MIX(1, 2, false, "mix 1:2")
  MIX(1, 3, false, "mix 1:3")
  MIX(1, 3, true, "mix nt 1:3")
  MIX(1, 4, false, "mix 1:4")
  MIX(1, 8, false, "mix 1:8")
  MIX(1, 8, true, "mix nt 1:8")
  MIX(3, 1, false, "mix 3:1")
  const long M = 100864;
  tm("seg32 (qkv)", [&] { hipLaunchKernelGGL(seg32, 512, 512, 0, 0, A, (char*)C, (int)M); },
     (double)M * 384 * 2 * 3 + (double)M * 1152 * 2);
  tm("row768 (qkv)", [&] { hipLaunchKernelGGL(row768, 512, 512, 0, 0, A, (char*)C, (int)M); },
     (double)M * 384 * 2 * 3 + (double)M * 1152 * 2);
  tm("row768 g1024", [&] { hipLaunchKernelGGL(row768, 1024, 512, 0, 0, A, (char*)C, (int)M); },
     (double)M * 384 * 2 * 3 + (double)M * 1152 * 2);
  return 0;
}
