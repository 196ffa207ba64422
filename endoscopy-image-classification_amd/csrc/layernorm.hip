// LayerNorm(eps=1e-6) forward / backward over the fp32 residual stream (gfx950).
//
// Replaces Block.norm1 / norm2 (code/models/conformer.py:58,60,65,70-71; nn.LayerNorm(dim, 1e-6)).
// One wave per token row (two rows in flight), D/128 float2 per lane (coalesced), statistics in
// fp32 with a two-pass variance.  Forward writes the bf16 GEMM operand and the per-row (mean, rstd) the backward needs.
// Backward fuses the residual-gradient add (dx = dres + LN'(dy)), writes fp32 and bf16 copies of
// dx, and per-workgroup partial sums of dgamma / dbeta that es_splitk_reduce folds into the grads.
#include "common.h"

namespace {

// Two rows per wave (R = 2): 3 KiB of loads in flight per wave at D = 384 -- with one row per wave
// the ~48 KiB in flight per CU did not cover HBM latency (MI355X_MICROARCH.md §HBM).
template <int V>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int ldx,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     bf16* __restrict__ y, int ldy, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int M, float eps) {
  constexpr int D = V * 128, R = 2;
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  float2 v[R][V];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int row = min(row0 + q, M - 1);
    const float* xr = x + (size_t)row * ldx;
#pragma unroll
    for (int j = 0; j < V; ++j) v[q][j] = *(const float2*)(xr + (j * 64 + lane) * 2);
  }
  float2 gm[V], bt[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = (j * 64 + lane) * 2;
    gm[j] = *(const float2*)(gamma + c);
    bt[j] = *(const float2*)(beta + c);
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int row = row0 + q;
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) s += v[q][j].x + v[q][j].y;
    const float mean = warp_sum(s) * (1.0f / D);
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const float a = v[q][j].x - mean, b = v[q][j].y - mean;
      ss += a * a + b * b;
    }
    const float rstd = 1.0f / sqrtf(warp_sum(ss) * (1.0f / D) + eps);
    if (row < M) {
      bf16* yr = y + (size_t)row * ldy;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = (j * 64 + lane) * 2;
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        bf16x2 o = {(bf16)((v[q][j].x - mean) * rstd * gm[j].x + bt[j].x),
                    (bf16)((v[q][j].y - mean) * rstd * gm[j].y + bt[j].y)};
        *(bf16x2*)(yr + c) = o;
      }
      if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
      }
    }
  }
}

// The same rows, numerics and stores as ln_fwd_kernel, but each wave walks row pairs grid-stride and issues
// the next pair's loads before it normalises the current one (two pairs in flight per wave).
template <int V>
__global__ __launch_bounds__(256) void ln_fwd_loop_kernel(const float* __restrict__ x, int ldx,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, bf16* __restrict__ y,
                                                          int ldy, float* __restrict__ mean_out,
                                                          float* __restrict__ rstd_out, int M, float eps) {
  constexpr int D = V * 128, R = 2;
  const int lane = threadIdx.x & 63;
  const int stride = gridDim.x * 4 * R;
  int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= M) return;
  auto load = [&](float2 (&v)[R][V], int r0) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const float* xr = x + (size_t)min(r0 + q, M - 1) * ldx;
#pragma unroll
      for (int j = 0; j < V; ++j) v[q][j] = *(const float2*)(xr + (j * 64 + lane) * 2);
    }
  };
  float2 v[R][V];
  load(v, row0);
  float2 gm[V], bt[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = (j * 64 + lane) * 2;
    gm[j] = *(const float2*)(gamma + c);
    bt[j] = *(const float2*)(beta + c);
  }
  for (;;) {
    const int nx = row0 + stride;
    float2 nv[R][V];
    if (nx < M) load(nv, nx);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q;
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) s += v[q][j].x + v[q][j].y;
      const float mean = warp_sum(s) * (1.0f / D);
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float a = v[q][j].x - mean, b = v[q][j].y - mean;
        ss += a * a + b * b;
      }
      const float rstd = 1.0f / sqrtf(warp_sum(ss) * (1.0f / D) + eps);
      if (row < M) {
        bf16* yr = y + (size_t)row * ldy;
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const int c = (j * 64 + lane) * 2;
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
          bf16x2 o = {(bf16)((v[q][j].x - mean) * rstd * gm[j].x + bt[j].x),
                      (bf16)((v[q][j].y - mean) * rstd * gm[j].y + bt[j].y)};
          *(bf16x2*)(yr + c) = o;
        }
        if (lane == 0) {
          mean_out[row] = mean;
          rstd_out[row] = rstd;
        }
      }
    }
    if (nx >= M) break;
#pragma unroll
    for (int q = 0; q < R; ++q)
#pragma unroll
      for (int j = 0; j < V; ++j) v[q][j] = nv[q][j];
    row0 = nx;
  }
}

// two consecutive dy values as float2 (fp32 or bf16 storage)
__device__ __forceinline__ float2 ld_dy2(const float* p) { return *(const float2*)p; }
__device__ __forceinline__ float2 ld_dy2(const bf16* p) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = *(const bf16x2*)p;
  return make_float2((float)v[0], (float)v[1]);
}

// Each wave walks rows two at a time (both rows' dy / x / dres loads issued before any math).
// DY = float or bf16 (the ViT engine's dgrad GEMMs hand over d(LN output) in bf16, half the bytes).
template <int V, typename DY>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const DY* __restrict__ dy, int lddy, const float* __restrict__ x,
                                                     int ldx, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const float* __restrict__ gamma,
                                                     const float* __restrict__ dres, int ldres, float* __restrict__ dx,
                                                     int lddx, bf16* __restrict__ dxb, int lddxb,
                                                     float* __restrict__ pg, float* __restrict__ pb, int M) {
  constexpr int D = V * 128, R = 2;
  __shared__ float red[2][4][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float2 ag[V], ab[V], gm[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    ag[j] = ab[j] = make_float2(0.f, 0.f);
    gm[j] = *(const float2*)(gamma + (j * 64 + lane) * 2);
  }
  // the next row pair's dy / x / dres / mean / rstd loads are issued before this pair's math (two pairs in
  // flight per wave); the arithmetic and its order are unchanged
  float2 d[R][V], xv[R][V], rv[R][V];
  float mean[R], rstd[R];
  auto load = [&](int r0) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = min(r0 + q, M - 1);
      mean[q] = mean_in[row];
      rstd[q] = rstd_in[row];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = (j * 64 + lane) * 2;
        d[q][j] = ld_dy2(dy + (size_t)row * lddy + c);
        xv[q][j] = *(const float2*)(x + (size_t)row * ldx + c);
        rv[q][j] = dres ? *(const float2*)(dres + (size_t)row * ldres + c) : make_float2(0.f, 0.f);
      }
    }
  };
  const int stride = gridDim.x * 4 * R;
  int row0 = (blockIdx.x * 4 + w) * R;
  if (row0 < M) load(row0);
  for (; row0 < M; row0 += stride) {
    float2 cd[R][V], cx[R][V], cr[R][V];
    float cm[R], cs[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      cm[q] = mean[q];
      cs[q] = rstd[q];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        cd[q][j] = d[q][j];
        cx[q][j] = xv[q][j];
        cr[q][j] = rv[q][j];
      }
    }
    if (row0 + stride < M) load(row0 + stride);
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int row = row0 + q;
      if (row >= M) break;
      float2 xh[V], gd[V];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        xh[j] = make_float2((cx[q][j].x - cm[q]) * cs[q], (cx[q][j].y - cm[q]) * cs[q]);
        gd[j] = make_float2(cd[q][j].x * gm[j].x, cd[q][j].y * gm[j].y);
        s1 += gd[j].x + gd[j].y;
        s2 += gd[j].x * xh[j].x + gd[j].y * xh[j].y;
        ag[j].x += cd[q][j].x * xh[j].x;
        ag[j].y += cd[q][j].y * xh[j].y;
        ab[j].x += cd[q][j].x;
        ab[j].y += cd[q][j].y;
      }
      s1 = warp_sum(s1) * (1.0f / D);
      s2 = warp_sum(s2) * (1.0f / D);
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const int c = (j * 64 + lane) * 2;
        const float2 o = make_float2(cs[q] * (gd[j].x - s1 - xh[j].x * s2) + cr[q][j].x,
                                     cs[q] * (gd[j].y - s1 - xh[j].y * s2) + cr[q][j].y);
        *(float2*)(dx + (size_t)row * lddx + c) = o;
        if (dxb) {
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
          bf16x2 ob = {(bf16)o.x, (bf16)o.y};
          *(bf16x2*)(dxb + (size_t)row * lddxb + c) = ob;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = (j * 64 + lane) * 2;
    red[0][w][c] = ag[j].x;
    red[0][w][c + 1] = ag[j].y;
    red[1][w][c] = ab[j].x;
    red[1][w][c + 1] = ab[j].y;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    pg[(size_t)blockIdx.x * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pb[(size_t)blockIdx.x * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

}  // namespace

namespace es_gemm {  // gemm.hip: dgamma and dbeta reductions in one launch (the LayerNorm backward's two tails)
int reduce_partials_pair(const float* P0, float* out0, const float* P1, float* out1, int G, int N, int accumulate,
                         hipStream_t stream);
struct RedPairEntry {
  const float* P;
  float *out0, *out1;
  int G, N, accumulate, blk0;
};
int reduce_partials_multi(const RedPairEntry* ents, int n, hipStream_t stream);
}

#define LN_DISPATCH(KER, V_, GRID, STREAM, ...)                                \
  switch (V_) {                                                                \
    case 1: hipLaunchKernelGGL(KER<1>, GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(KER<2>, GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(KER<3>, GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(KER<4>, GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 6: hipLaunchKernelGGL(KER<6>, GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    default: return ES_BAD_SHAPE;                                              \
  }
#define LN_BWD_DISPATCH(T_, V_, GRID, STREAM, ...)                                                  \
  switch (V_) {                                                                                     \
    case 1: hipLaunchKernelGGL(HIP_KERNEL_NAME(ln_bwd_kernel<1, T_>), GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 2: hipLaunchKernelGGL(HIP_KERNEL_NAME(ln_bwd_kernel<2, T_>), GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 3: hipLaunchKernelGGL(HIP_KERNEL_NAME(ln_bwd_kernel<3, T_>), GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 4: hipLaunchKernelGGL(HIP_KERNEL_NAME(ln_bwd_kernel<4, T_>), GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    case 6: hipLaunchKernelGGL(HIP_KERNEL_NAME(ln_bwd_kernel<6, T_>), GRID, 256, 0, STREAM, __VA_ARGS__); break; \
    default: return ES_BAD_SHAPE;                                                                   \
  }

template <typename DY>
static int ln_bwd_launch(const DY* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                         float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                         hipStream_t stream) {
  if (M <= 0 || D % 128 || blocks <= 0) return ES_BAD_SHAPE;
  // dgamma == dbeta == NULL: the per-block partials stay in the workspace (pg [grid][D], then pb) for a later
  // es_ln_param_grads_multi launch
  const bool defer = !dgamma && !dbeta;
  if (!dy || !x || !mean || !rstd || !gamma || !dx || (!defer && (!dgamma || !dbeta)) || !workspace) return ES_BAD_ARG;
  const int grid = blocks < (M + 7) / 8 ? blocks : (M + 7) / 8;
  float* pg = workspace;
  float* pb = workspace + (size_t)grid * D;
  LN_BWD_DISPATCH(DY, D / 128, grid, stream, dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx, (bf16*)dxb,
                  lddxb, pg, pb, M);
  if (hipGetLastError() != hipSuccess) return ES_HIP_ERROR;
  if (defer) return ES_OK;
  return es_gemm::reduce_partials_pair(pg, dgamma, pb, dbeta, grid, D, accumulate, stream);
}

// > 0 (default 2048): the grid-stride forward on this many workgroups when the one-shot grid would be larger;
// 0: the one-shot kernel.  F1 same box, interleaved three times (bench.py A/B, round 5): 0 30.51 ms/step
// mean, 1024 30.42, 2048 30.28, 4096 30.30; isolated at F1's LN2 (scripts/ln_bench.py, x L3-resident) the
// one-shot kernel is faster (35.1 vs 37.9 us): the gain is in the two-stream step, where 12,608 short-lived
// workgroups per launch interleave worse with the other stream's kernels
static int g_ln_fwd_grid = 2048;

extern "C" {

// tuning knob: LayerNorm forward grid (0 = one workgroup per 8 rows, the one-shot kernel; > 0 = the grid-stride
// kernel with the next row pair's loads in flight, on this many workgroups); returns the previous value
int es_set_ln_fwd_grid(int g) {
  const int old = g_ln_fwd_grid;
  g_ln_fwd_grid = g;
  return old;
}

int es_layernorm_fwd(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, float* mean,
                     float* rstd, int M, int D, float eps, hipStream_t stream) {
  if (M <= 0 || D % 128 || ldx % 2 || ldy % 2) return ES_BAD_SHAPE;
  if (!x || !gamma || !beta || !y || !mean || !rstd) return ES_BAD_ARG;
  const int grid = (M + 7) / 8;  // 4 waves x 2 rows
  if (g_ln_fwd_grid > 0 && grid > g_ln_fwd_grid) {
    LN_DISPATCH(ln_fwd_loop_kernel, D / 128, g_ln_fwd_grid, stream, x, ldx, gamma, beta, (bf16*)y, ldy, mean, rstd, M,
                eps);
  } else {
    LN_DISPATCH(ln_fwd_kernel, D / 128, grid, stream, x, ldx, gamma, beta, (bf16*)y, ldy, mean, rstd, M, eps);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// workspace: 2 * blocks * D floats.  dgamma / dbeta are accumulated (+=) when accumulate != 0.
int es_layernorm_bwd(const float* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                     const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                     float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                     hipStream_t stream) {
  return ln_bwd_launch(dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx, dxb, lddxb, dgamma, dbeta,
                       workspace, blocks, M, D, accumulate, stream);
}

// es_layernorm_bwd with dy in bf16 (the dgrad GEMM's output image)
// the partial-row count a backward over M rows on `blocks` workgroups leaves in its workspace
int es_layernorm_bwd_grid(int blocks, int M) { return blocks <= 0 || M <= 0 ? 0 : (blocks < (M + 7) / 8 ? blocks : (M + 7) / 8); }

// dgamma / dbeta of n deferred LayerNorm backwards in one launch: table = n host entries of
// es_ln_param_grads_entry_size() bytes {const float* workspace; float* dgamma; float* dbeta; int grid; int D;
// int accumulate; int pad} (grid = es_layernorm_bwd_grid of that backward); same sums, bit for bit, as the
// backwards' own reductions
int es_ln_param_grads_entry_size() { return (int)sizeof(es_gemm::RedPairEntry); }
int es_ln_param_grads_multi(const void* table, int n, hipStream_t stream) {
  return es_gemm::reduce_partials_multi((const es_gemm::RedPairEntry*)table, n, stream);
}

int es_layernorm_bwd_b16(const void* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                         float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                         hipStream_t stream) {
  return ln_bwd_launch((const bf16*)dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx, dxb, lddxb, dgamma,
                       dbeta, workspace, blocks, M, D, accumulate, stream);
}

}  // extern "C"
