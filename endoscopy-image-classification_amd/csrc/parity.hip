// fp32 parity mode of the ViT step (gfx950): every GEMM operand, activation and gradient in fp32.
//
// The production path keeps its GEMM operands in bf16 (gemm.hip, attention.hip, layernorm.hip),
// which moves ViT-S logits by ~5e-3 relative from the reference's fp32 arithmetic at depth 12 -- a
// gap no 1e-3 bar can see through.  These entry points take the SAME arguments as their bf16
// counterparts (include/endossl.h, suffix _f32) with fp32 storage wherever those read or write
// bf16, so endossl/vit.py's Engine runs its one forward / backward sequence in either precision
// (Engine(precision="fp32")) and the 12-layer orchestration is checked against the fp32 oracle at
// 1e-3 (tests/test_gpu_parity.py).  Not a performance path; still matrix-core code:
//
//  * GEMMs on v_mfma_f32_16x16x4_f32, which is bit for bit a k-ordered fp32 fmaf chain
//    (MI355X_MICROARCH.md, FP32-input MFMA): 64x64 output tile, 16-deep k step staged k-major in
//    LDS, 4 waves of 32x32.  One kernel covers NT (Linear forward / data gradient) and TN (weight
//    gradient) through a template choice of operand layout; split-K partials are reduced in a
//    fixed order (deterministic).
//  * attention as exact two-pass softmax (scores for all keys kept in LDS, T <= 1024), fp32 FMA;
//    backward as a query-block pass (dQ, delta) and a key-block pass (dK, dV) that recomputes P.
//  * LayerNorm / patches / embedding backward / weight packing: fp32 storage of the same maps.
//
// Reference ops: code/models/conformer.py:13-23 (Mlp), :35-50 (Attention), :58-72 (Block),
// timm PatchEmbed / VisionTransformer (code/build.py:196-197).
#include <algorithm>

#include "common.h"

namespace {

// ------------------------------------------------------------------------------------ GEMM
// C[i][j] = sum_k A(i,k) B(j,k);  A(i,k) = AK ? A[k*lda + i] : A[i*lda + k]  (same for B)
constexpr int PT = 64, PK = 16;

enum PEpi {
  P_PLAIN = 0, P_GELU = 1, P_RESID = 2, P_DGELU = 3, P_F32 = 4, P_PATCH = 5, P_GELU_ACT = 6, P_GELU_D = 7,
  P_MULAUX = 8, P_SLAB = 100  // raw accumulator into split-K slab z
};

struct PArgs {
  const float* A; const float* B; const float* bias;
  float* C; float* C2; const float* aux;
  int M, N, K, lda, ldb, ldc, ldaux, np, epi, kchunk;
};

__device__ __forceinline__ float gelu_exact(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_exact(float x) {
  return 0.5f * (1.0f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * expf(-0.5f * x * x);
}

__device__ __forceinline__ void p_store(const PArgs& p, int i, int j, float acc) {
  if (i >= p.M || j >= p.N) return;
  if (p.epi == P_SLAB) {
    p.C[(size_t)blockIdx.z * p.M * p.N + (size_t)i * p.N + j] = acc;
    return;
  }
  const float v = acc + (p.bias ? p.bias[j] : 0.f);
  const size_t o = (size_t)i * p.ldc + j;
  switch (p.epi) {
    case P_PLAIN:
    case P_F32: p.C[o] = v; break;
    case P_GELU: p.C[o] = v; p.C2[o] = gelu_exact(v); break;
    case P_RESID: p.C[o] = v + p.aux[(size_t)i * p.ldaux + j]; break;
    case P_DGELU: p.C[o] = v * gelu_grad_exact(p.aux[(size_t)i * p.ldaux + j]); break;
    case P_PATCH: {
      const int img = i / p.np, pi = i - img * p.np;
      p.C[((size_t)img * (p.np + 1) + 1 + pi) * p.ldc + j] = v + p.aux[(size_t)(1 + pi) * p.ldaux + j];
      break;
    }
    case P_GELU_ACT: p.C[o] = gelu_exact(v); break;
    case P_GELU_D: p.C[o] = gelu_grad_exact(v); p.C2[o] = gelu_exact(v); break;
    case P_MULAUX: p.C[o] = v * p.aux[(size_t)i * p.ldaux + j]; break;
    default: break;
  }
}

// stage a 64 x 16 (rows x k) operand tile k-major into S[k][row]
template <bool KMAJ>
__device__ __forceinline__ void p_stage(const float* __restrict__ X, int ld, int rows, int r0, int k0, int k1,
                                        float (*S)[PT + 1]) {
  const int t = threadIdx.x;
  if (KMAJ) {  // X[k*ld + r]: 64 consecutive rows per k, 4 k per pass
    const int r = t & 63, kq = t >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = kq + 4 * q, gr = r0 + r, gk = k0 + k;
      S[k][r] = (gr < rows && gk < k1) ? X[(size_t)gk * ld + gr] : 0.f;
    }
  } else {  // X[r*ld + k]: 16 consecutive k per row, 16 rows per pass
    const int k = t & 15, rq = t >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = rq + 16 * q, gr = r0 + r, gk = k0 + k;
      S[k][r] = (gr < rows && gk < k1) ? X[(size_t)gr * ld + gk] : 0.f;
    }
  }
}

template <bool AK, bool BK>
__global__ __launch_bounds__(256) void pgemm_kernel(PArgs p) {
  __shared__ float As[PK][PT + 1];
  __shared__ float Bs[PK][PT + 1];
  const int i0 = blockIdx.x * PT, j0 = blockIdx.y * PT;
  const int kb = blockIdx.z * p.kchunk, ke = min(p.K, kb + p.kchunk);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rb = (w >> 1) * 32, cb = (w & 1) * 32, lr = lane & 15, lk = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = kb; k0 < ke; k0 += PK) {
    p_stage<AK>(p.A, p.lda, p.M, i0, k0, ke, As);
    p_stage<BK>(p.B, p.ldb, p.N, j0, k0, ke, Bs);
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < PK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        a[q] = As[kk + lk][rb + q * 16 + lr];
        b[q] = Bs[kk + lk][cb + q * 16 + lr];
      }
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int q = 0; q < 4; ++q) p_store(p, i0 + rb + x * 16 + 4 * lk + q, j0 + cb + y * 16 + lr, acc[x][y][q]);
}

// out[idx] (+)= sum_s P[s][idx], s in order
__global__ void slab_reduce_kernel(const float* __restrict__ P, float* __restrict__ out, int S, long n, int accumulate) {
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < n; idx += (long)gridDim.x * blockDim.x) {
    float s = accumulate ? out[idx] : 0.f;
    for (int z = 0; z < S; ++z) s += P[(size_t)z * n + idx];
    out[idx] = s;
  }
}

// bias gradient partials: part[s][j] = sum over rows of split s of Y[m*ld + j]
__global__ void colsum_split_kernel(const float* __restrict__ Y, int ld, int M, int N, int chunk,
                                    float* __restrict__ part) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  if (j >= N) return;
  const int m0 = s * chunk, m1 = min(M, m0 + chunk);
  float acc = 0.f;
  for (int m = m0; m < m1; ++m) acc += Y[(size_t)m * ld + j];
  part[(size_t)s * N + j] = acc;
}

// kchunk: k range per grid.z slice (a multiple of PK)
int launch_pgemm(bool ak, bool bk, PArgs p, int kchunk, hipStream_t stream) {
  p.kchunk = kchunk;
  dim3 grid((p.M + PT - 1) / PT, (p.N + PT - 1) / PT, (p.K + kchunk - 1) / kchunk);
  if (!ak && !bk) hipLaunchKernelGGL(HIP_KERNEL_NAME(pgemm_kernel<false, false>), grid, 256, 0, stream, p);
  else if (ak && bk) hipLaunchKernelGGL(HIP_KERNEL_NAME(pgemm_kernel<true, true>), grid, 256, 0, stream, p);
  else return ES_BAD_ARG;
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// -------------------------------------------------------------------------------- attention
// qkv rows (img*T + t) of ldqkv floats: q at h*64, k at D + h*64, v at 2D + h*64 (timm's
// reshape(B, N, 3, H, hd)).  Tq queries per image (T, or 1 for the CLS-query form); o row of
// query i of image b is b*orows + i; lse[(b*H + h)*Tq + i].
constexpr int QB = 16, KT = 64;
struct PAttn {
  const float* qkv; float* o; float* lse; const float* dout; float* dqkv; float* delta;
  int ldqkv, ldo, lddo, lddqkv, T, Tq, H, orows;
  float scale;
};

__device__ __forceinline__ const float* qrow(const PAttn& a, int b, int t) { return a.qkv + ((size_t)b * a.T + t) * a.ldqkv; }

// one workgroup per (16-query block, head, image): scores for every key in LDS, exact softmax
__global__ __launch_bounds__(256) void pattn_fwd_kernel(PAttn a) {
  extern __shared__ float S[];  // [QB][Tp]
  __shared__ float Qs[QB][65];
  __shared__ float Ks[KT][65];
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * QB, t = threadIdx.x;
  const int D = a.H * 64, Tp = (a.T + KT - 1) / KT * KT;
  for (int e = t; e < QB * 64; e += 256) {
    const int q = e >> 6, d = e & 63;
    Qs[q][d] = (q0 + q < a.Tq) ? qrow(a, b, q0 + q)[h * 64 + d] : 0.f;
  }
  for (int k0 = 0; k0 < a.T; k0 += KT) {
    __syncthreads();
    for (int e = t; e < KT * 64; e += 256) {
      const int j = e >> 6, d = e & 63;
      Ks[j][d] = (k0 + j < a.T) ? qrow(a, b, k0 + j)[D + h * 64 + d] : 0.f;
    }
    __syncthreads();
    const int j = t & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = (t >> 6) + 4 * r;
      float s = 0.f;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) s = fmaf(Qs[q][d], Ks[j][d], s);
      S[q * Tp + k0 + j] = s * a.scale;
    }
  }
  __syncthreads();
  // softmax rows: wave w owns rows 4w .. 4w+3
  const int w = t >> 6, lane = t & 63;
  for (int r = 0; r < 4; ++r) {
    const int q = 4 * w + r;
    float mx = -INFINITY;
    for (int j = lane; j < a.T; j += 64) mx = fmaxf(mx, S[q * Tp + j]);
    mx = warp_max(mx);
    float sum = 0.f;
    for (int j = lane; j < a.T; j += 64) {
      const float e = expf(S[q * Tp + j] - mx);
      S[q * Tp + j] = e;
      sum += e;
    }
    sum = warp_sum(sum);
    const float inv = 1.0f / sum;
    for (int j = lane; j < a.T; j += 64) S[q * Tp + j] *= inv;
    if (lane == 0 && q0 + q < a.Tq) a.lse[((size_t)b * a.H + h) * a.Tq + q0 + q] = mx + logf(sum);
  }
  // O = P V
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int d = t & 63;
  for (int k0 = 0; k0 < a.T; k0 += KT) {
    __syncthreads();
    for (int e = t; e < KT * 64; e += 256) {
      const int j = e >> 6, dd = e & 63;
      Ks[j][dd] = (k0 + j < a.T) ? qrow(a, b, k0 + j)[2 * D + h * 64 + dd] : 0.f;
    }
    __syncthreads();
    const int jn = min(KT, a.T - k0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = (t >> 6) + 4 * r;
      for (int j = 0; j < jn; ++j) acc[r] = fmaf(S[q * Tp + k0 + j], Ks[j][d], acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = (t >> 6) + 4 * r;
    if (q0 + q < a.Tq) a.o[((size_t)b * a.orows + q0 + q) * a.ldo + h * 64 + d] = acc[r];
  }
}

// dQ pass: per query block, P recomputed from lse, dS = P (dO.V - delta), dQ = scale dS K
__global__ __launch_bounds__(256) void pattn_bwd_dq_kernel(PAttn a) {
  extern __shared__ float S[];  // [QB][Tp]
  __shared__ float Qs[QB][65], dOs[QB][65];
  __shared__ float Ks[KT][65];
  __shared__ float dl[QB], ls[QB];
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * QB, t = threadIdx.x;
  const int D = a.H * 64, Tp = (a.T + KT - 1) / KT * KT;
  const int w = t >> 6, lane = t & 63;
  for (int e = t; e < QB * 64; e += 256) {
    const int q = e >> 6, d = e & 63;
    const bool ok = q0 + q < a.Tq;
    Qs[q][d] = ok ? qrow(a, b, q0 + q)[h * 64 + d] : 0.f;
    dOs[q][d] = ok ? a.dout[((size_t)b * a.orows + q0 + q) * a.lddo + h * 64 + d] : 0.f;
  }
  __syncthreads();
  for (int r = 0; r < 4; ++r) {  // delta = rowsum(dO * O)
    const int q = 4 * w + r;
    const bool ok = q0 + q < a.Tq;
    const float ov = ok ? a.o[((size_t)b * a.orows + q0 + q) * a.ldo + h * 64 + lane] : 0.f;
    const float s = warp_sum(dOs[q][lane] * ov);
    if (lane == 0) {
      dl[q] = s;
      ls[q] = ok ? a.lse[((size_t)b * a.H + h) * a.Tq + q0 + q] : 0.f;
      if (ok && a.delta) a.delta[((size_t)b * a.H + h) * a.Tq + q0 + q] = s;
    }
  }
  for (int k0 = 0; k0 < a.T; k0 += KT) {  // P
    __syncthreads();
    for (int e = t; e < KT * 64; e += 256) {
      const int j = e >> 6, d = e & 63;
      Ks[j][d] = (k0 + j < a.T) ? qrow(a, b, k0 + j)[D + h * 64 + d] : 0.f;
    }
    __syncthreads();
    const int j = t & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = (t >> 6) + 4 * r;
      float s = 0.f;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) s = fmaf(Qs[q][d], Ks[j][d], s);
      S[q * Tp + k0 + j] = (k0 + j < a.T) ? expf(s * a.scale - ls[q]) : 0.f;
    }
  }
  for (int k0 = 0; k0 < a.T; k0 += KT) {  // dS
    __syncthreads();
    for (int e = t; e < KT * 64; e += 256) {
      const int j = e >> 6, d = e & 63;
      Ks[j][d] = (k0 + j < a.T) ? qrow(a, b, k0 + j)[2 * D + h * 64 + d] : 0.f;
    }
    __syncthreads();
    const int j = t & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = (t >> 6) + 4 * r;
      float dp = 0.f;
#pragma unroll 16
      for (int d = 0; d < 64; ++d) dp = fmaf(dOs[q][d], Ks[j][d], dp);
      S[q * Tp + k0 + j] *= (dp - dl[q]);
    }
  }
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int d = t & 63;
  for (int k0 = 0; k0 < a.T; k0 += KT) {  // dQ = scale dS K
    __syncthreads();
    for (int e = t; e < KT * 64; e += 256) {
      const int j = e >> 6, dd = e & 63;
      Ks[j][dd] = (k0 + j < a.T) ? qrow(a, b, k0 + j)[D + h * 64 + dd] : 0.f;
    }
    __syncthreads();
    const int jn = min(KT, a.T - k0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = (t >> 6) + 4 * r;
      for (int j = 0; j < jn; ++j) acc[r] = fmaf(S[q * Tp + k0 + j], Ks[j][d], acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = (t >> 6) + 4 * r;
    if (q0 + q < a.Tq) a.dqkv[((size_t)b * a.T + q0 + q) * a.lddqkv + h * 64 + d] = acc[r] * a.scale;
  }
}

// dK / dV pass: per 16-key block, over query tiles of 64: P and dS recomputed (delta from O, dO);
// also zeroes the dQ columns of token rows >= Tq (the CLS-query form has no query there)
constexpr int KB = 16, QT = 64;
__global__ __launch_bounds__(256) void pattn_bwd_dkv_kernel(PAttn a) {
  __shared__ float Kb[KB][65], Vb[KB][65];
  __shared__ float Qt[QT][65], dOt[QT][65];
  __shared__ float Ps[KB][QT + 1], dSs[KB][QT + 1];
  __shared__ float lq[QT], dq[QT];
  const int b = blockIdx.z, h = blockIdx.y, j0 = blockIdx.x * KB, t = threadIdx.x;
  const int D = a.H * 64;
  for (int e = t; e < KB * 64; e += 256) {
    const int j = e >> 6, d = e & 63;
    const bool ok = j0 + j < a.T;
    Kb[j][d] = ok ? qrow(a, b, j0 + j)[D + h * 64 + d] : 0.f;
    Vb[j][d] = ok ? qrow(a, b, j0 + j)[2 * D + h * 64 + d] : 0.f;
    if (ok && j0 + j >= a.Tq) a.dqkv[((size_t)b * a.T + j0 + j) * a.lddqkv + h * 64 + d] = 0.f;
  }
  float gk[4] = {0.f, 0.f, 0.f, 0.f}, gv[4] = {0.f, 0.f, 0.f, 0.f};
  const int w = t >> 6, lane = t & 63;
  for (int i0 = 0; i0 < a.Tq; i0 += QT) {
    __syncthreads();
    for (int e = t; e < QT * 64; e += 256) {
      const int i = e >> 6, d = e & 63;
      const bool ok = i0 + i < a.Tq;
      Qt[i][d] = ok ? qrow(a, b, i0 + i)[h * 64 + d] : 0.f;
      dOt[i][d] = ok ? a.dout[((size_t)b * a.orows + i0 + i) * a.lddo + h * 64 + d] : 0.f;
    }
    __syncthreads();
    for (int r = 0; r < QT / 4; ++r) {  // delta and lse of the tile's queries: wave w rows w, w+4, ...
      const int i = w + 4 * r;
      const bool ok = i0 + i < a.Tq;
      const float ov = ok ? a.o[((size_t)b * a.orows + i0 + i) * a.ldo + h * 64 + lane] : 0.f;
      const float s = warp_sum(dOt[i][lane] * ov);
      if (lane == 0) {
        dq[i] = s;
        lq[i] = ok ? a.lse[((size_t)b * a.H + h) * a.Tq + i0 + i] : 0.f;
      }
    }
    __syncthreads();
    {
      const int i = t & 63;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = (t >> 6) + 4 * r;
        float s = 0.f, dp = 0.f;
#pragma unroll 16
        for (int d = 0; d < 64; ++d) {
          s = fmaf(Qt[i][d], Kb[j][d], s);
          dp = fmaf(dOt[i][d], Vb[j][d], dp);
        }
        const float pv = (i0 + i < a.Tq) ? expf(s * a.scale - lq[i]) : 0.f;
        Ps[j][i] = pv;
        dSs[j][i] = pv * (dp - dq[i]);
      }
    }
    __syncthreads();
    const int d = t & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = (t >> 6) + 4 * r;
      for (int i = 0; i < QT; ++i) {
        gv[r] = fmaf(Ps[j][i], dOt[i][d], gv[r]);
        gk[r] = fmaf(dSs[j][i], Qt[i][d], gk[r]);
      }
    }
  }
  const int d = t & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = (t >> 6) + 4 * r;
    if (j0 + j < a.T) {
      float* row = a.dqkv + ((size_t)b * a.T + j0 + j) * a.lddqkv;
      row[D + h * 64 + d] = gk[r] * a.scale;
      row[2 * D + h * 64 + d] = gv[r];
    }
  }
}

int attn_fwd_launch(PAttn a, int nimg, hipStream_t stream) {
  const int Tp = (a.T + KT - 1) / KT * KT;
  const size_t lds = (size_t)QB * Tp * 4;
  allow_lds(pattn_fwd_kernel, lds + (QB + KT) * 65 * 4);
  dim3 grid((a.Tq + QB - 1) / QB, a.H, nimg);
  hipLaunchKernelGGL(pattn_fwd_kernel, grid, 256, lds, stream, a);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int attn_bwd_launch(PAttn a, int nimg, hipStream_t stream) {
  const int Tp = (a.T + KT - 1) / KT * KT;
  const size_t lds = (size_t)QB * Tp * 4;
  allow_lds(pattn_bwd_dq_kernel, lds + (2 * QB + KT) * 65 * 4 + 2 * QB * 4);
  dim3 g1((a.Tq + QB - 1) / QB, a.H, nimg);
  hipLaunchKernelGGL(pattn_bwd_dq_kernel, g1, 256, lds, stream, a);
  dim3 g2((a.T + KB - 1) / KB, a.H, nimg);
  hipLaunchKernelGGL(pattn_bwd_dkv_kernel, g2, 256, 0, stream, a);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// ------------------------------------------------------------------------------- LayerNorm
template <int V>  // D = 64 V, one wave per row
__global__ __launch_bounds__(256) void pln_fwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ g,
                                                      const float* __restrict__ bt, float* __restrict__ y, int ldy,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int M, float eps) {
  constexpr int D = V * 64;
  const int lane = threadIdx.x & 63, row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[V], s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    v[j] = x[(size_t)row * ldx + j * 64 + lane];
    s += v[j];
  }
  const float mean = warp_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) ss += (v[j] - mean) * (v[j] - mean);
  const float rstd = 1.0f / sqrtf(warp_sum(ss) / D + eps);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int c = j * 64 + lane;
    y[(size_t)row * ldy + c] = (v[j] - mean) * rstd * g[c] + bt[c];
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <int V>
__global__ __launch_bounds__(256) void pln_bwd_kernel(const float* __restrict__ dy, int lddy, const float* __restrict__ x,
                                                      int ldx, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, const float* __restrict__ g,
                                                      const float* __restrict__ dres, int ldres, float* __restrict__ dx,
                                                      int lddx, float* __restrict__ dxb, int lddxb,
                                                      float* __restrict__ pg, float* __restrict__ pb, int M) {
  constexpr int D = V * 64;
  __shared__ float red[2][4][D];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float ag[V], ab[V];
#pragma unroll
  for (int j = 0; j < V; ++j) ag[j] = ab[j] = 0.f;
  for (int row = blockIdx.x * 4 + w; row < M; row += gridDim.x * 4) {
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[V], gd[V], d[V], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = j * 64 + lane;
      d[j] = dy[(size_t)row * lddy + c];
      xh[j] = (x[(size_t)row * ldx + c] - mean) * rstd;
      gd[j] = d[j] * g[c];
      s1 += gd[j];
      s2 += gd[j] * xh[j];
      ag[j] += d[j] * xh[j];
      ab[j] += d[j];
    }
    s1 = warp_sum(s1) / D;
    s2 = warp_sum(s2) / D;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      const int c = j * 64 + lane;
      const float o = rstd * (gd[j] - s1 - xh[j] * s2) + (dres ? dres[(size_t)row * ldres + c] : 0.f);
      dx[(size_t)row * lddx + c] = o;
      if (dxb) dxb[(size_t)row * lddxb + c] = o;
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) {
    red[0][w][j * 64 + lane] = ag[j];
    red[1][w][j * 64 + lane] = ab[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    pg[(size_t)blockIdx.x * D + c] = red[0][0][c] + red[0][1][c] + red[0][2][c] + red[0][3][c];
    pb[(size_t)blockIdx.x * D + c] = red[1][0][c] + red[1][1][c] + red[1][2][c] + red[1][3][c];
  }
}

#define PV_DISPATCH(KER, V_, GRID, STREAM, ...)                                      \
  switch (V_) {                                                                      \
    case 2: hipLaunchKernelGGL(KER<2>, GRID, 256, 0, STREAM, __VA_ARGS__); break;    \
    case 4: hipLaunchKernelGGL(KER<4>, GRID, 256, 0, STREAM, __VA_ARGS__); break;    \
    case 6: hipLaunchKernelGGL(KER<6>, GRID, 256, 0, STREAM, __VA_ARGS__); break;    \
    case 8: hipLaunchKernelGGL(KER<8>, GRID, 256, 0, STREAM, __VA_ARGS__); break;    \
    case 12: hipLaunchKernelGGL(KER<12>, GRID, 256, 0, STREAM, __VA_ARGS__); break;  \
    default: return ES_BAD_SHAPE;                                                    \
  }

// ------------------------------------------------------------------------ patches / embedding
struct PNorm {
  float mean[3], std[3];
  int u8;
};
__global__ void pim2col_kernel(const void* __restrict__ img, float* __restrict__ out, int n, int S, int P, PNorm nm) {
  const int G = S / P, np = G * G, K = 3 * P * P;
  const long total = (long)n * np * K;
  for (long id = blockIdx.x * (long)blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const int k = (int)(id % K);
    const long row = id / K;
    const int im = (int)(row / np), pi = (int)(row % np);
    const int py = pi / G, px = pi % G, c = k / (P * P), ky = (k / P) % P, kx = k % P;
    const size_t src = (((size_t)im * 3 + c) * S + py * P + ky) * S + px * P + kx;
    float v;
    if (nm.u8) {
      const float mu = c == 0 ? nm.mean[0] : (c == 1 ? nm.mean[1] : nm.mean[2]);
      const float sd = c == 0 ? nm.std[0] : (c == 1 ? nm.std[1] : nm.std[2]);
      v = ((float)((const uint8_t*)img)[src] / 255.0f - mu) / sd;
    } else {
      v = ((const float*)img)[src];
    }
    out[row * K + k] = v;
  }
}

__global__ void pembed_bwd_kernel(const float* __restrict__ dx, int lddx, float* __restrict__ dpatch, int ldp,
                                  float* __restrict__ dpos, float* __restrict__ dcls, int n, int T, int D,
                                  int accumulate) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= T * D) return;
  const int t = id / D, d = id % D;
  float s = 0.f;
  for (int im = 0; im < n; ++im) {
    const float v = dx[((size_t)im * T + t) * lddx + d];
    s += v;
    if (t > 0) dpatch[((size_t)im * (T - 1) + t - 1) * ldp + d] = v;
  }
  dpos[id] = accumulate ? dpos[id] + s : s;
  if (t == 0) dcls[d] = accumulate ? dcls[d] + s : s;
}

struct PPackEntry {  // layout of optim.hip's PackEntry, fp32 images
  long src;
  float* dst;
  float* dstT;
  int N, K;
};
__global__ void ppack_kernel(const float* __restrict__ flat, const PPackEntry* __restrict__ tab) {
  const PPackEntry e = tab[blockIdx.y];
  const long total = (long)e.N * e.K;
  for (long id = blockIdx.x * (long)blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const int nn = (int)(id / e.K), kk = (int)(id % e.K);
    const float v = flat[e.src + id];
    if (e.dst) e.dst[id] = v;
    if (e.dstT) e.dstT[(size_t)kk * e.N + nn] = v;
  }
}

}  // namespace

extern "C" int es_reduce_partials(const float* P, float* out, int G, int N, int accumulate, hipStream_t stream);

extern "C" {

int es_gemm_nt_f32(int epi, const void* A, int lda, const void* B, int ldb, const float* bias, void* C, int ldc,
                   void* C2, const void* aux, int ldaux, int M, int N, int K, int np, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || epi < 0 || epi > 8) return ES_BAD_SHAPE;
  if (!A || !B || !C) return ES_BAD_ARG;
  if (((epi == P_GELU || epi == P_GELU_D) && !C2) ||
      ((epi == P_RESID || epi == P_DGELU || epi == P_MULAUX || epi == P_PATCH) && !aux) || (epi == P_PATCH && np <= 0))
    return ES_BAD_ARG;
  PArgs p{(const float*)A, (const float*)B, bias, (float*)C, (float*)C2, (const float*)aux,
          M, N, K, lda, ldb, ldc, ldaux, np, epi, 0};
  return launch_pgemm(false, false, p, (K + PK - 1) / PK * PK, stream);
}

// splits <= 0: automatic (enough 64 x 64 tiles x splits to fill the chip, >= 1024 tokens per split)
static int ptn_auto_splits(int M, int N1, int N2) {
  const int tiles = ((N1 + PT - 1) / PT) * ((N2 + PT - 1) / PT);
  return std::max(1, std::min(std::max(1, 1024 / tiles), std::max(1, M / 1024)));
}

size_t es_gemm_tn_f32_workspace(int N1, int N2, int splits) {
  if (splits <= 0) splits = std::max(1, 1024 / (((N1 + PT - 1) / PT) * ((N2 + PT - 1) / PT)));
  return (size_t)splits * N1 * N2 + (size_t)splits * N1;
}

int es_gemm_tn_f32(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
                   float* workspace, float* out, int accumulate, float* bias_out, hipStream_t stream) {
  if (M <= 0 || N1 <= 0 || N2 <= 0) return ES_BAD_SHAPE;
  if (!A1 || !A2 || !out || !workspace) return ES_BAD_ARG;
  if (splits <= 0) splits = ptn_auto_splits(M, N1, N2);
  // each split covers a whole number of 16-deep k steps; the slab count is what the grid covers
  const int kchunk = ((M + splits - 1) / splits + PK - 1) / PK * PK;
  const int S = (M + kchunk - 1) / kchunk;
  PArgs p{(const float*)A1, (const float*)A2, nullptr, workspace, nullptr, nullptr,
          N1, N2, M, ld1, ld2, N2, 0, 0, P_SLAB, 0};
  int rc = launch_pgemm(true, true, p, kchunk, stream);
  if (rc) return rc;
  const long n = (long)N1 * N2;
  hipLaunchKernelGGL(slab_reduce_kernel, (int)std::min<long>((n + 255) / 256, 4096), 256, 0, stream, workspace, out,
                     S, n, accumulate);
  if (bias_out) {
    float* part = workspace + (size_t)S * N1 * N2;
    dim3 g((N1 + 255) / 256, S);
    hipLaunchKernelGGL(colsum_split_kernel, g, 256, 0, stream, (const float*)A1, ld1, M, N1, kchunk, part);
    hipLaunchKernelGGL(slab_reduce_kernel, (N1 + 255) / 256, 256, 0, stream, part, bias_out, S, (long)N1, accumulate);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_attn_fwd_f32(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                    hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 1024 || H <= 0) return ES_BAD_SHAPE;
  if (!qkv || !o || !lse) return ES_BAD_ARG;
  PAttn a{(const float*)qkv, (float*)o, lse, nullptr, nullptr, nullptr, ldqkv, ldo, 0, 0, T, T, H, T, scale};
  return attn_fwd_launch(a, nimg, stream);
}

int es_attn_bwd_f32(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, float* delta,
                    const void* dout, int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale,
                    hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 1024 || H <= 0) return ES_BAD_SHAPE;
  if (!qkv || !o || !lse || !dout || !dqkv) return ES_BAD_ARG;
  PAttn a{(const float*)qkv, (float*)o, (float*)lse, (const float*)dout, (float*)dqkv, delta,
          ldqkv, ldo, lddo, lddqkv, T, T, H, T, scale};
  return attn_bwd_launch(a, nimg, stream);
}

int es_attn_cls_fwd_f32(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                        hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 1024 || H <= 0) return ES_BAD_SHAPE;
  if (!qkv || !o || !lse) return ES_BAD_ARG;
  PAttn a{(const float*)qkv, (float*)o, lse, nullptr, nullptr, nullptr, ldqkv, ldo, 0, 0, T, 1, H, 1, scale};
  return attn_fwd_launch(a, nimg, stream);
}

int es_attn_cls_bwd_f32(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, const void* dout,
                        int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 1024 || H <= 0) return ES_BAD_SHAPE;
  if (!qkv || !o || !lse || !dout || !dqkv) return ES_BAD_ARG;
  PAttn a{(const float*)qkv, (float*)o, (float*)lse, (const float*)dout, (float*)dqkv, nullptr,
          ldqkv, ldo, lddo, lddqkv, T, 1, H, 1, scale};
  return attn_bwd_launch(a, nimg, stream);
}

int es_layernorm_fwd_f32(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, float* mean,
                         float* rstd, int M, int D, float eps, hipStream_t stream) {
  if (M <= 0 || D % 64) return ES_BAD_SHAPE;
  if (!x || !gamma || !beta || !y || !mean || !rstd) return ES_BAD_ARG;
  PV_DISPATCH(pln_fwd_kernel, D / 64, (M + 3) / 4, stream, x, ldx, gamma, beta, (float*)y, ldy, mean, rstd, M, eps);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_layernorm_bwd_f32(const float* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                         float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                         hipStream_t stream) {
  if (M <= 0 || D % 64 || blocks <= 0) return ES_BAD_SHAPE;
  if (!dy || !x || !mean || !rstd || !gamma || !dx || !dgamma || !dbeta || !workspace) return ES_BAD_ARG;
  const int grid = std::min(blocks, (M + 3) / 4);
  float* pg = workspace;
  float* pb = workspace + (size_t)grid * D;
  PV_DISPATCH(pln_bwd_kernel, D / 64, grid, stream, dy, lddy, x, ldx, mean, rstd, gamma, dres, ldres, dx, lddx,
              (float*)dxb, lddxb, pg, pb, M);
  if (hipGetLastError() != hipSuccess) return ES_HIP_ERROR;
  int rc = es_reduce_partials(pg, dgamma, grid, D, accumulate, stream);
  if (rc) return rc;
  return es_reduce_partials(pb, dbeta, grid, D, accumulate, stream);
}

int es_patch_im2col_f32(const float* img, void* patches, int n, int S, int P, hipStream_t stream) {
  if (n <= 0 || P <= 0 || S % P) return ES_BAD_SHAPE;
  if (!img || !patches) return ES_BAD_ARG;
  const long total = (long)n * (S / P) * (S / P) * 3 * P * P;
  const PNorm nm{{0, 0, 0}, {1, 1, 1}, 0};
  hipLaunchKernelGGL(pim2col_kernel, (int)std::min<long>((total + 255) / 256, 65536), 256, 0, stream, img,
                     (float*)patches, n, S, P, nm);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_patch_im2col_u8_f32(const void* img, float mean0, float mean1, float mean2, float std0, float std1, float std2,
                           void* patches, int n, int S, int P, hipStream_t stream) {
  if (n <= 0 || P <= 0 || S % P) return ES_BAD_SHAPE;
  if (!img || !patches) return ES_BAD_ARG;
  const long total = (long)n * (S / P) * (S / P) * 3 * P * P;
  const PNorm nm{{mean0, mean1, mean2}, {std0, std1, std2}, 1};
  hipLaunchKernelGGL(pim2col_kernel, (int)std::min<long>((total + 255) / 256, 65536), 256, 0, stream, img,
                     (float*)patches, n, S, P, nm);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_embed_bwd_f32(const float* dx, int lddx, void* dpatch, int ldp, float* dpos, float* dcls, int n, int T, int D,
                     int accumulate, hipStream_t stream) {
  if (n <= 0 || T <= 1 || D <= 0) return ES_BAD_SHAPE;
  if (!dx || !dpatch || !dpos || !dcls) return ES_BAD_ARG;
  hipLaunchKernelGGL(pembed_bwd_kernel, (T * D + 255) / 256, 256, 0, stream, dx, lddx, (float*)dpatch, ldp, dpos, dcls,
                     n, T, D, accumulate);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_pack_weights_f32(const float* flat, const void* entries, int nmat, hipStream_t stream) {
  if (nmat <= 0) return ES_BAD_SHAPE;
  if (!flat || !entries) return ES_BAD_ARG;
  dim3 grid(256, nmat);
  hipLaunchKernelGGL(ppack_kernel, grid, 256, 0, stream, flat, (const PPackEntry*)entries);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_copy_f32(const float* x, void* y, long n, hipStream_t stream) {
  if (n < 0) return ES_BAD_SHAPE;
  if (n && (!x || !y)) return ES_BAD_ARG;
  return hipMemcpyAsync(y, x, (size_t)n * 4, hipMemcpyDeviceToDevice, stream) == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
