// Optimizer-side HBM-streaming kernels (gfx950): Adam + EMA in one pass, the reference-exact
// multi-tensor EMA, and the bf16 weight images the GEMMs read.
//
//  es_adam_ema_step    torch.optim.Adam(betas=(0.9,0.999), eps=1e-8, weight_decay=0)
//                      (code/optimizer.py:50-51, single-tensor update order) fused with the EMA
//                      e <- d*e + (1-d)*theta (code/ema.py:51-59) over the flat parameter buffer:
//                      one read of (p, g, m, v, e), one write of (p, m, v, e) per parameter.
//  es_ema_update_multi ModelEMA.update over an arbitrary list of state_dict tensors, fp32 and
//                      int64 (BatchNorm num_batches_tracked: blended in fp32, truncated on copy_).
//  es_pack_weights     fp32 master [N,K] -> bf16 [N,K] (forward operand) and bf16 [K,N] (dgrad
//                      operand, so dgrad is also an NT GEMM), one launch for every matrix.
// The reference evaluates `d*e + (1-d)*m` as three separately rounded fp32 ops (no FMA);
// `#pragma clang fp contract(off)` keeps that order bit-for-bit here.
#include "common.h"

namespace {

__global__ void adam_ema_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, float* __restrict__ e, long n, float one_minus_b1, float b2,
                                float one_minus_b2, float neg_step, float bc2_sqrt, float eps, float decay,
                                float one_minus_decay, float grad_scale) {
#pragma clang fp contract(off)
  const long n4 = n >> 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i], mv = ((f32x4*)m)[i], vv = ((f32x4*)v)[i];
    if (grad_scale != 1.0f) gv *= grad_scale;  // data-parallel mean of summed grads
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // exp_avg.lerp_(grad, 1-beta1)  (weight < 0.5 branch: self + w*(end-self))
      mv[k] = mv[k] + one_minus_b1 * (gv[k] - mv[k]);
      // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1-beta2)
      vv[k] = vv[k] * b2 + one_minus_b2 * gv[k] * gv[k];
      // denom = (exp_avg_sq.sqrt() / bias_correction2_sqrt).add_(eps); p.addcdiv_(m, denom, -step)
      const float denom = sqrtf(vv[k]) / bc2_sqrt + eps;
      pv[k] = pv[k] + neg_step * (mv[k] / denom);
    }
    ((f32x4*)p)[i] = pv;
    ((f32x4*)m)[i] = mv;
    ((f32x4*)v)[i] = vv;
    if (e) {
      f32x4 ev = ((f32x4*)e)[i];
#pragma unroll
      for (int k = 0; k < 4; ++k) ev[k] = decay * ev[k] + one_minus_decay * pv[k];
      ((f32x4*)e)[i] = ev;
    }
  }
}

struct EmaEntry {
  void* e; const void* m; long n; int dtype; int pad;  // dtype 0 = fp32, 1 = int64
};

// chunk table: (entry, start) pairs, one block per chunk of up to 4096 elements
__global__ void ema_multi_kernel(const EmaEntry* __restrict__ tab, const int2* __restrict__ chunks, float decay,
                                 float one_minus_decay) {
#pragma clang fp contract(off)
  const int2 ch = chunks[blockIdx.x];
  const EmaEntry en = tab[ch.x];
  const long s = (long)ch.y * 4096;
  const long end = min(s + 4096, en.n);
  for (long i = s + threadIdx.x; i < end; i += blockDim.x) {
    if (en.dtype == 0) {
      float* e = (float*)en.e;
      const float mv = ((const float*)en.m)[i];
      e[i] = decay * e[i] + one_minus_decay * mv;
    } else {
      int64_t* e = (int64_t*)en.e;
      const float r = decay * (float)e[i] + one_minus_decay * (float)((const int64_t*)en.m)[i];
      e[i] = (int64_t)r;  // copy_ into an integer tensor truncates toward zero
    }
  }
}

struct PackEntry {
  long src;     // float offset into the flat parameter buffer
  bf16* dst;    // [N][K] or null
  bf16* dstT;   // [K][N] or null
  int N, K;
};

// grid.y = matrix, grid.x strides over 64x64 tiles of that matrix.  N, K multiples of 4 (every ViT / Conformer
// Linear): 16-B loads of the fp32 master rows, 8-B bf16 stores of W rows and, through the LDS tile, of W^T rows;
// otherwise element-wise.
__global__ void pack_kernel(const float* __restrict__ flat, const PackEntry* __restrict__ tab) {
  __shared__ float tile[64][65];
  const PackEntry en = tab[blockIdx.y];
  const int tn = (en.N + 63) / 64, tk = (en.K + 63) / 64;
  const float* src = flat + en.src;
  const bool vec = (en.N % 4 == 0) && (en.K % 4 == 0);
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  for (int t = blockIdx.x; t < tn * tk; t += gridDim.x) {
    const int n0 = (t / tk) * 64, k0 = (t % tk) * 64;
    if (vec) {
      for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
        const int rr = i / 16, c4 = (i % 16) * 4;
        const int n = n0 + rr, k = k0 + c4;
        const bool ok = n < en.N && k < en.K;
        const f32x4 x = ok ? *(const f32x4*)(src + (size_t)n * en.K + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[rr][c4 + j] = x[j];
        if (en.dst && ok)
          *(bf16x4_t*)(en.dst + (size_t)n * en.K + k) = bf16x4_t{(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3]};
      }
      __syncthreads();
      if (en.dstT) {
        for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) {
          const int kk = i / 16, n4 = (i % 16) * 4;
          const int n = n0 + n4, k = k0 + kk;
          if (n < en.N && k < en.K)
            *(bf16x4_t*)(en.dstT + (size_t)k * en.N + n) =
                bf16x4_t{(bf16)tile[n4][kk], (bf16)tile[n4 + 1][kk], (bf16)tile[n4 + 2][kk], (bf16)tile[n4 + 3][kk]};
        }
      }
    } else {
      for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
        const int rr = i / 64, cc = i % 64;
        const int n = n0 + rr, k = k0 + cc;
        const float x = (n < en.N && k < en.K) ? src[(size_t)n * en.K + k] : 0.f;
        tile[rr][cc] = x;
        if (en.dst && n < en.N && k < en.K) en.dst[(size_t)n * en.K + k] = (bf16)x;
      }
      __syncthreads();
      if (en.dstT) {
        for (int i = threadIdx.x; i < 64 * 64; i += blockDim.x) {
          const int kk = i / 64, nn = i % 64;
          const int n = n0 + nn, k = k0 + kk;
          if (n < en.N && k < en.K) en.dstT[(size_t)k * en.N + n] = (bf16)tile[nn][kk];
        }
      }
    }
    __syncthreads();
  }
}

__global__ void cast_kernel(const float* __restrict__ x, bf16* __restrict__ y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = (bf16)x[i];
}

// y += x over n floats (n % 4 == 0, 16-byte aligned): the two-lane backward's second flat gradient
__global__ void add_f32_kernel(float* __restrict__ y, const float* __restrict__ x, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 a = ((const f32x4*)y)[i];
    a += ((const f32x4*)x)[i];
    ((f32x4*)y)[i] = a;
  }
}

}  // namespace

extern "C" {

int es_add_f32(float* y, const float* x, long n, hipStream_t stream) {
  if (n <= 0 || n % 4) return ES_BAD_SHAPE;
  if (!y || !x || ((uintptr_t)y & 15) || ((uintptr_t)x & 15)) return ES_BAD_ARG;
  long grid = (n / 4 + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(add_f32_kernel, (int)grid, 256, 0, stream, y, x, n / 4);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_cast_f32_bf16(const float* x, void* y, long n, hipStream_t stream) {
  if (n <= 0) return ES_BAD_SHAPE;
  long grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(cast_kernel, (int)grid, 256, 0, stream, x, (bf16*)y, n);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// n % 4 == 0 and 16-byte aligned buffers.  neg_step = -lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t)
// (host computes them in double exactly as torch.optim.Adam does).  ema may be null.
int es_adam_ema_step(float* p, const float* g, float* m, float* v, float* ema, long n, float beta1, float beta2,
                     float eps, float neg_step, float bc2_sqrt, float decay, float one_minus_decay,
                     float grad_scale, hipStream_t stream) {
  if (n <= 0 || n % 4) return ES_BAD_SHAPE;
  if (!p || !g || !m || !v) return ES_BAD_ARG;
  long grid = (n / 4 + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(adam_ema_kernel, (int)grid, 256, 0, stream, p, g, m, v, ema, n, 1.0f - beta1, beta2,
                     1.0f - beta2, neg_step, bc2_sqrt, eps, decay, one_minus_decay, grad_scale);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// entries: device array of {e, m, n, dtype}; chunks: device array of int2 {entry, chunk_index}
int es_ema_update_multi(const void* entries, const void* chunks, int nchunks, float decay, float one_minus_decay,
                        hipStream_t stream) {
  if (nchunks <= 0) return ES_BAD_SHAPE;
  if (!entries || !chunks) return ES_BAD_ARG;
  hipLaunchKernelGGL(ema_multi_kernel, nchunks, 256, 0, stream, (const EmaEntry*)entries, (const int2*)chunks,
                     decay, one_minus_decay);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_ema_entry_size(void) { return (int)sizeof(EmaEntry); }
int es_pack_entry_size(void) { return (int)sizeof(PackEntry); }

int es_pack_weights(const float* flat, const void* entries, int nmat, hipStream_t stream) {
  if (nmat <= 0) return ES_BAD_SHAPE;
  if (!flat || !entries) return ES_BAD_ARG;
  dim3 grid(128, nmat);
  hipLaunchKernelGGL(pack_kernel, grid, 256, 0, stream, flat, (const PackEntry*)entries);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
