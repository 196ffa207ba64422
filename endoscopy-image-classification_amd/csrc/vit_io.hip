// ViT input and output ends: patch extraction, CLS/pos-embed rows, embedding backward, and the
// fused final-LayerNorm + classifier head on the CLS token (gfx950).
//
// timm 0.5.4 VisionTransformer (reference build path code/build.py:196-197; same pattern as
// code/models/conformer.py:337,420,430,442-443):
//   x = PatchEmbed(img)            Conv2d(3, D, 16, 16): stride == kernel -> im2col is a pure
//                                  permutation; the projection is an MFMA GEMM (gemm.hip, EPI_PATCH)
//   x = cat(cls_token, x) + pos_embed
//   ...blocks...
//   logits = head(norm(x)[:, 0])   only the CLS row reaches the loss
#include "common.h"
#include <cstdlib>

namespace {

// img fp32 [n, 3, S, S] -> patches bf16 [n*G*G, 3*P*P], column k = c*P*P + ky*P + kx (Conv2d weight order)
template <int P>
__global__ void im2col_kernel(const float* __restrict__ img, bf16* __restrict__ out, int n, int S) {
  const int G = S / P, np = G * G, K = 3 * P * P;
  const long total = (long)n * np * (K / 8);
  for (long id = blockIdx.x * (long)blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const int k8 = (int)(id % (K / 8));
    const long row = id / (K / 8);
    const int im = (int)(row / np), pi = (int)(row % np);
    const int py = pi / G, px = pi % G;
    const int k = k8 * 8, c = k / (P * P), ky = (k / P) % P, kx = k % P;
    const float* src = img + (((size_t)im * 3 + c) * S + py * P + ky) * S + px * P + kx;
    const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
    bf16x8 o = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
    *(bf16x8*)(out + row * K + k) = o;
  }
}

// Same permutation from uint8 images [n, 3, S, S] (the host pipeline's un-normalised pixels): each
// value goes through torchvision's ToTensor (x / 255) and Normalize ((x - mean[c]) / std[c]) in fp32
// with IEEE divisions, exactly as code/dataset.py:49-51 runs them on the host, so the bf16 patches
// equal those of the fp32 path bit for bit -- with a quarter of the bytes over PCIe and from HBM.
struct ChanNorm {
  float mean[3], std[3];
};
template <int P>
__global__ void im2col_u8_kernel(const uint8_t* __restrict__ img, bf16* __restrict__ out, int n, int S, ChanNorm nm) {
  const int G = S / P, np = G * G, K = 3 * P * P;
  const long total = (long)n * np * (K / 8);
  for (long id = blockIdx.x * (long)blockDim.x + threadIdx.x; id < total; id += (long)gridDim.x * blockDim.x) {
    const int k8 = (int)(id % (K / 8));
    const long row = id / (K / 8);
    const int im = (int)(row / np), pi = (int)(row % np);
    const int py = pi / G, px = pi % G;
    const int k = k8 * 8, c = k / (P * P), ky = (k / P) % P, kx = k % P;
    const uint8_t* src = img + (((size_t)im * 3 + c) * S + py * P + ky) * S + px * P + kx;
    const uint2 raw = *(const uint2*)src;
    const float mu = c == 0 ? nm.mean[0] : (c == 1 ? nm.mean[1] : nm.mean[2]);
    const float sd = c == 0 ? nm.std[0] : (c == 1 ? nm.std[1] : nm.std[2]);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned b = ((j < 4 ? raw.x : raw.y) >> (8 * (j & 3))) & 255u;
      o[j] = (bf16)(((float)b / 255.0f - mu) / sd);
    }
    *(bf16x8*)(out + row * K + k) = o;
  }
}

// The same values, one workgroup per (image, patch row): the band's 3 x 16 image rows arrive with 16-B loads
// (whole rows, coalesced) into LDS, and the band's G consecutive output rows leave as 16-B stores in order
// (every wave-instruction one contiguous KiB).  S % 16 == 0 (16-B source rows), dynamic LDS 48 x S bytes.
__global__ __launch_bounds__(256) void im2col_u8_band_kernel(const uint8_t* __restrict__ img, bf16* __restrict__ out,
                                                             int S, ChanNorm nm) {
  extern __shared__ __attribute__((aligned(16))) uint8_t band[];  // [3][16][S]
  constexpr int P = 16, K = 3 * P * P;
  const int G = S / P, im = blockIdx.x / G, py = blockIdx.x - im * G;
  const int cpr = S / 16;  // 16-B chunks per image row
  for (int i = threadIdx.x; i < 48 * cpr; i += blockDim.x) {
    const int rr = i / cpr, ch = i - rr * cpr, c = rr >> 4, ky = rr & 15;
    *(uint4*)(band + rr * S + ch * 16) =
        *(const uint4*)(img + (((size_t)im * 3 + c) * S + py * P + ky) * S + ch * 16);
  }
  __syncthreads();
  bf16* dst = out + (size_t)blockIdx.x * G * K;  // rows (im * G + py) * G .. + G - 1
  for (int i = threadIdx.x; i < G * (K / 8); i += blockDim.x) {
    const int px = i / (K / 8), k = (i - px * (K / 8)) * 8;
    const int c = k / (P * P), ky = (k / P) % P, kx = k % P;
    const uint2 raw = *(const uint2*)(band + (c * 16 + ky) * S + px * P + kx);
    const float mu = c == 0 ? nm.mean[0] : (c == 1 ? nm.mean[1] : nm.mean[2]);
    const float sd = c == 0 ? nm.std[0] : (c == 1 ? nm.std[1] : nm.std[2]);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const unsigned b = ((j < 4 ? raw.x : raw.y) >> (8 * (j & 3))) & 255u;
      o[j] = (bf16)(((float)b / 255.0f - mu) / sd);
    }
    *(bf16x8*)(dst + (size_t)i * 8) = o;
  }
}

// x[img*T + 0][d] = cls[d] + pos[0][d]
__global__ void cls_init_kernel(float* __restrict__ x, int ldx, const float* __restrict__ cls,
                                const float* __restrict__ pos, int n, int T, int D) {
  const int total = n * D;
  for (int id = blockIdx.x * blockDim.x + threadIdx.x; id < total; id += gridDim.x * blockDim.x) {
    const int im = id / D, d = id % D;
    x[(size_t)im * T * ldx + d] = cls[d] + pos[d];
  }
}

// dx fp32 [n*T, D] -> dpatch bf16 [n*(T-1), D]; dpos[t][d] (+)= sum_img dx; dcls[d] (+)= dpos[0][d].
// Block = 64 features x 4 image groups; the 4 partial sums meet in LDS.  The image loop is unrolled
// so 8 loads per thread are in flight ahead of the in-order adds.
__global__ __launch_bounds__(256) void embed_bwd_kernel(const float* __restrict__ dx, int lddx,
                                                        bf16* __restrict__ dpatch, int ldp, float* __restrict__ dpos,
                                                        float* __restrict__ dcls, int n, int T, int D, int accumulate) {
  __shared__ float red[4][64];
  const int id = blockIdx.x * 64 + (threadIdx.x & 63), ig = threadIdx.x >> 6;
  const int total = T * D;
  float s0 = 0.f, s1 = 0.f;
  int t = 0, d = 0;
  if (id < total) {
    t = id / D;
    d = id % D;
    int im = ig;
#pragma unroll 4
    for (; im + 4 < n; im += 8) {
      const float v0 = dx[((size_t)im * T + t) * lddx + d];
      const float v1 = dx[((size_t)(im + 4) * T + t) * lddx + d];
      s0 += v0;
      s1 += v1;
      if (t > 0) {
        dpatch[((size_t)im * (T - 1) + t - 1) * ldp + d] = (bf16)v0;
        dpatch[((size_t)(im + 4) * (T - 1) + t - 1) * ldp + d] = (bf16)v1;
      }
    }
    for (; im < n; im += 4) {
      const float v = dx[((size_t)im * T + t) * lddx + d];
      s0 += v;
      if (t > 0) dpatch[((size_t)im * (T - 1) + t - 1) * ldp + d] = (bf16)v;
    }
  }
  red[ig][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (ig == 0 && id < total) {
    const int l = threadIdx.x & 63;
    const float s = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    dpos[id] = accumulate ? dpos[id] + s : s;
    if (t == 0) dcls[d] = accumulate ? dcls[d] + s : s;
  }
}

// embed_bwd_kernel with four consecutive features per lane (D, lddx, ldp multiples of 4): 16-B loads of dx,
// 8-B bf16 stores of dpatch; every feature's image sums run in the same order, so the results are bit-identical.
__global__ __launch_bounds__(256) void embed_bwd_vec_kernel(const float* __restrict__ dx, int lddx,
                                                            bf16* __restrict__ dpatch, int ldp, float* __restrict__ dpos,
                                                            float* __restrict__ dcls, int n, int T, int D,
                                                            int accumulate) {
  __shared__ f32x4 red[4][64];
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  const int id = (blockIdx.x * 64 + (threadIdx.x & 63)) * 4, ig = threadIdx.x >> 6;
  const int total = T * D;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  int t = 0, d = 0;
  if (id < total) {
    t = id / D;
    d = id % D;
    int im = ig;
#pragma unroll 4
    for (; im + 4 < n; im += 8) {
      const f32x4 v0 = *(const f32x4*)(dx + ((size_t)im * T + t) * lddx + d);
      const f32x4 v1 = *(const f32x4*)(dx + ((size_t)(im + 4) * T + t) * lddx + d);
      s0 += v0;
      s1 += v1;
      if (t > 0) {
        *(bf16x4_t*)(dpatch + ((size_t)im * (T - 1) + t - 1) * ldp + d) =
            bf16x4_t{(bf16)v0[0], (bf16)v0[1], (bf16)v0[2], (bf16)v0[3]};
        *(bf16x4_t*)(dpatch + ((size_t)(im + 4) * (T - 1) + t - 1) * ldp + d) =
            bf16x4_t{(bf16)v1[0], (bf16)v1[1], (bf16)v1[2], (bf16)v1[3]};
      }
    }
    for (; im < n; im += 4) {
      const f32x4 v = *(const f32x4*)(dx + ((size_t)im * T + t) * lddx + d);
      s0 += v;
      if (t > 0)
        *(bf16x4_t*)(dpatch + ((size_t)im * (T - 1) + t - 1) * ldp + d) =
            bf16x4_t{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
    }
  }
  red[ig][threadIdx.x & 63] = s0 + s1;
  __syncthreads();
  if (ig == 0 && id < total) {
    const int l = threadIdx.x & 63;
    const f32x4 sv = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dpos[id + j] = accumulate ? dpos[id + j] + sv[j] : sv[j];
      if (t == 0) dcls[d + j] = accumulate ? dcls[d + j] + sv[j] : sv[j];
    }
  }
}

// One wave per image: y = LN(x_cls) (eps), logits = y W^T + b.  Saves xhat (pre-affine) + rstd.
template <int V>
__global__ __launch_bounds__(256) void cls_head_fwd_kernel(const float* __restrict__ x, int ldx, int T,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ W, const float* __restrict__ b,
                                                           float* __restrict__ logits, int ldl,
                                                           float* __restrict__ xhat, float* __restrict__ rstd_out,
                                                           int n, int C, float eps) {
  constexpr int D = V * 64;
  const int lane = threadIdx.x & 63;
  const int im = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (im >= n) return;
  const float* xr = x + (size_t)im * T * ldx;
  float v[V], s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    v[j] = xr[j * 64 + lane];
    s += v[j];
  }
  const float mean = warp_sum(s) * (1.0f / D);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) ss += (v[j] - mean) * (v[j] - mean);
  const float rstd = 1.0f / sqrtf(warp_sum(ss) * (1.0f / D) + eps);
  float y[V];
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int d = j * 64 + lane;
    const float xh = (v[j] - mean) * rstd;
    xhat[(size_t)im * D + d] = xh;
    y[j] = xh * gamma[d] + beta[d];
  }
  if (lane == 0) rstd_out[im] = rstd;
  for (int c = 0; c < C; ++c) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < V; ++j) acc += y[j] * W[(size_t)c * D + j * 64 + lane];
    acc = warp_sum(acc);
    if (lane == 0) logits[(size_t)im * ldl + c] = acc + b[c];
  }
}

// One wave per image: dy = dlogits . W; dx_cls = LN'(dy) written to dx row img*T (other rows untouched).
template <int V>
__global__ __launch_bounds__(256) void cls_head_bwd_kernel(const float* __restrict__ dl, int lddl,
                                                           const float* __restrict__ W,
                                                           const float* __restrict__ gamma,
                                                           const float* __restrict__ xhat,
                                                           const float* __restrict__ rstd_in,
                                                           float* __restrict__ dyn, float* __restrict__ dx, int lddx,
                                                           int T, int n, int C) {
  constexpr int D = V * 64;
  const int lane = threadIdx.x & 63;
  const int im = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (im >= n) return;
  float dy[V];
#pragma unroll
  for (int j = 0; j < V; ++j) dy[j] = 0.f;
  for (int c = 0; c < C; ++c) {
    const float g = dl[(size_t)im * lddl + c];
#pragma unroll
    for (int j = 0; j < V; ++j) dy[j] += g * W[(size_t)c * D + j * 64 + lane];
  }
  float xh[V], gd[V], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int d = j * 64 + lane;
    dyn[(size_t)im * D + d] = dy[j];
    xh[j] = xhat[(size_t)im * D + d];
    gd[j] = dy[j] * gamma[d];
    s1 += gd[j];
    s2 += gd[j] * xh[j];
  }
  s1 = warp_sum(s1) * (1.0f / D);
  s2 = warp_sum(s2) * (1.0f / D);
  const float rstd = rstd_in[im];
#pragma unroll
  for (int j = 0; j < V; ++j) dx[(size_t)im * T * lddx + j * 64 + lane] = rstd * (gd[j] - s1 - xh[j] * s2);
}

// Parameter grads of the head + final norm, summed over images in a fixed order (run-to-run reproducible):
//  dW[c][d] += sum_i dl[i][c] * y[i][d], db[c] += sum_i dl[i][c], dgamma[d] += sum_i dyn*xhat, dbeta += sum_i dyn
// Workgroup (x, r): columns d = 64x .. 64x + 63 of row r (r < C: dW row c = r; C: dgamma; C + 1: dbeta); wave w
// sums images w, w + 4, .. per lane, the four wave sums are added in wave order; db[c] by wave 0 of workgroup
// (0, c) over lanes, then a fixed shuffle tree.
__global__ __launch_bounds__(256) void cls_head_wgrad_kernel(const float* __restrict__ dl, int lddl,
                                                             const float* __restrict__ xhat,
                                                             const float* __restrict__ dyn,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, float* __restrict__ dW,
                                                             float* __restrict__ db, float* __restrict__ dgamma,
                                                             float* __restrict__ dbeta, int n, int C, int D,
                                                             int accumulate) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int d = blockIdx.x * 64 + lane, r = blockIdx.y;
  float s = 0.f;
  if (r < C) {
    const float g = gamma[d], b = beta[d];
    for (int i = w; i < n; i += 4) s += dl[(size_t)i * lddl + r] * (xhat[(size_t)i * D + d] * g + b);
  } else if (r == C) {
    for (int i = w; i < n; i += 4) s += dyn[(size_t)i * D + d] * xhat[(size_t)i * D + d];
  } else {
    for (int i = w; i < n; i += 4) s += dyn[(size_t)i * D + d];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    const float t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    float* dst = r < C ? dW + (size_t)r * D : (r == C ? dgamma : dbeta);
    dst[d] = accumulate ? dst[d] + t : t;
    if (blockIdx.x == 0 && r < C) {
      float sb = 0.f;
      for (int i = lane; i < n; i += 64) sb += dl[(size_t)i * lddl + r];
      sb = warp_sum(sb);
      if (lane == 0) db[r] = accumulate ? db[r] + sb : sb;
    }
  }
}

// CoMatch features: one wave per image, fts = LN(x_cls) (the ModelwEmb `fts` over a ViT trunk,
// code/models/custom_model.py:207-209); xhat / rstd saved for the backward.
template <int V>
__global__ __launch_bounds__(256) void cls_ln_fwd_kernel(const float* __restrict__ x, int ldx, int T,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, float* __restrict__ fts,
                                                         int ldf, float* __restrict__ xhat,
                                                         float* __restrict__ rstd_out, int n, float eps) {
  constexpr int D = V * 64;
  const int lane = threadIdx.x & 63;
  const int im = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (im >= n) return;
  const float* xr = x + (size_t)im * T * ldx;
  float v[V], s = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    v[j] = xr[j * 64 + lane];
    s += v[j];
  }
  const float mean = warp_sum(s) * (1.0f / D);
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) ss += (v[j] - mean) * (v[j] - mean);
  const float rstd = 1.0f / sqrtf(warp_sum(ss) * (1.0f / D) + eps);
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int d = j * 64 + lane;
    const float xh = (v[j] - mean) * rstd;
    xhat[(size_t)im * D + d] = xh;
    fts[(size_t)im * ldf + d] = xh * gamma[d] + beta[d];
  }
  if (lane == 0) rstd_out[im] = rstd;
}

// dx_cls = LN'(dfts) into row img*T of dx (other rows untouched); dgamma / dbeta partials per
// 4-image workgroup folded with fp32 atomics (the grad buffer is zeroed per step).
template <int V>
__global__ __launch_bounds__(256) void cls_ln_bwd_kernel(const float* __restrict__ dfts, int lddf,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ xhat,
                                                         const float* __restrict__ rstd_in, float* __restrict__ dx,
                                                         int lddx, int T, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta, int n) {
  constexpr int D = V * 64;
  const int lane = threadIdx.x & 63;
  const int im = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (im >= n) return;
  float dy[V], xh[V], gd[V], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const int d = j * 64 + lane;
    dy[j] = dfts[(size_t)im * lddf + d];
    xh[j] = xhat[(size_t)im * D + d];
    gd[j] = dy[j] * gamma[d];
    s1 += gd[j];
    s2 += gd[j] * xh[j];
    atomicAdd(dgamma + d, dy[j] * xh[j]);
    atomicAdd(dbeta + d, dy[j]);
  }
  s1 = warp_sum(s1) * (1.0f / D);
  s2 = warp_sum(s2) * (1.0f / D);
  const float rstd = rstd_in[im];
#pragma unroll
  for (int j = 0; j < V; ++j) dx[(size_t)im * T * lddx + j * 64 + lane] = rstd * (gd[j] - s1 - xh[j] * s2);
}

}  // namespace

extern "C" {

int es_patch_im2col(const float* img, void* patches, int n, int S, int P, hipStream_t stream) {
  if (n <= 0 || P != 16 || S % P) return ES_BAD_SHAPE;
  if (!img || !patches) return ES_BAD_ARG;
  const long total = (long)n * (S / P) * (S / P) * (3 * P * P / 8);
  long grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  hipLaunchKernelGGL(im2col_kernel<16>, (int)grid, 256, 0, stream, img, (bf16*)patches, n, S);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_patch_im2col_u8(const void* img, float mean0, float mean1, float mean2, float std0, float std1, float std2,
                       void* patches, int n, int S, int P, hipStream_t stream) {
  if (n <= 0 || P != 16 || S % P) return ES_BAD_SHAPE;
  if (!img || !patches || ((uintptr_t)img & 7)) return ES_BAD_ARG;
  const long total = (long)n * (S / P) * (S / P) * (3 * P * P / 8);
  long grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  const ChanNorm nm{{mean0, mean1, mean2}, {std0, std1, std2}};
  if (S % 16 == 0 && !((uintptr_t)img & 15) && 48 * S <= 65536) {
    hipLaunchKernelGGL(im2col_u8_band_kernel, n * (S / 16), 256, 48 * S, stream, (const uint8_t*)img, (bf16*)patches,
                       S, nm);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  hipLaunchKernelGGL(im2col_u8_kernel<16>, (int)grid, 256, 0, stream, (const uint8_t*)img, (bf16*)patches, n, S, nm);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_cls_init(float* x, int ldx, const float* cls, const float* pos, int n, int T, int D, hipStream_t stream) {
  if (n <= 0 || T <= 0 || D <= 0) return ES_BAD_SHAPE;
  const int grid = (n * D + 255) / 256;
  hipLaunchKernelGGL(cls_init_kernel, grid, 256, 0, stream, x, ldx, cls, pos, n, T, D);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_embed_bwd(const float* dx, int lddx, void* dpatch, int ldp, float* dpos, float* dcls, int n, int T, int D,
                 int accumulate, hipStream_t stream) {
  if (n <= 0 || T <= 1 || D <= 0) return ES_BAD_SHAPE;
  if (D % 4 == 0 && lddx % 4 == 0 && ldp % 4 == 0 && !((uintptr_t)dx & 15) && !((uintptr_t)dpatch & 7)) {
    hipLaunchKernelGGL(embed_bwd_vec_kernel, (T * D / 4 + 63) / 64, 256, 0, stream, dx, lddx, (bf16*)dpatch, ldp, dpos,
                       dcls, n, T, D, accumulate);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  const int grid = (T * D + 63) / 64;
  hipLaunchKernelGGL(embed_bwd_kernel, grid, 256, 0, stream, dx, lddx, (bf16*)dpatch, ldp, dpos, dcls, n, T, D,
                     accumulate);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

#define HEAD_DISPATCH(KER, V_, GRID, STREAM, ...)                                  \
  switch (V_) {                                                                    \
    case 2: hipLaunchKernelGGL(KER<2>, GRID, 256, 0, STREAM, __VA_ARGS__); break;  \
    case 4: hipLaunchKernelGGL(KER<4>, GRID, 256, 0, STREAM, __VA_ARGS__); break;  \
    case 6: hipLaunchKernelGGL(KER<6>, GRID, 256, 0, STREAM, __VA_ARGS__); break;  \
    case 8: hipLaunchKernelGGL(KER<8>, GRID, 256, 0, STREAM, __VA_ARGS__); break;  \
    case 12: hipLaunchKernelGGL(KER<12>, GRID, 256, 0, STREAM, __VA_ARGS__); break;\
    default: return ES_BAD_SHAPE;                                                  \
  }

int es_cls_head_fwd(const float* x, int ldx, int T, const float* gamma, const float* beta, const float* W,
                    const float* b, float* logits, int ldl, float* xhat, float* rstd, int n, int D, int C, float eps,
                    hipStream_t stream) {
  if (n <= 0 || D % 64 || C <= 0) return ES_BAD_SHAPE;
  const int grid = (n + 3) / 4;
  HEAD_DISPATCH(cls_head_fwd_kernel, D / 64, grid, stream, x, ldx, T, gamma, beta, W, b, logits, ldl, xhat, rstd, n,
                C, eps);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// dx rows img*T receive the CLS gradient (caller zeroes the other rows); dW/db/dgamma/dbeta are summed over
// the batch in a fixed order and then ADDED to the buffers (es_cls_head_bwd) or WRITTEN over them
// (es_cls_head_bwd_ex, accumulate = 0: the step's first writer of those entries, so the flat gradient needs no
// zeroing launch); dyn: scratch [n, D].
int es_cls_head_bwd_ex(const float* dl, int lddl, const float* W, const float* gamma, const float* beta,
                       const float* xhat, const float* rstd, float* dyn, float* dx, int lddx, int T, float* dW,
                       float* db, float* dgamma, float* dbeta, int n, int D, int C, int accumulate, hipStream_t stream) {
  if (n <= 0 || D % 64 || C <= 0 || C > 256) return ES_BAD_SHAPE;
  const int grid = (n + 3) / 4;
  HEAD_DISPATCH(cls_head_bwd_kernel, D / 64, grid, stream, dl, lddl, W, gamma, xhat, rstd, dyn, dx, lddx, T, n, C);
  dim3 g2(D / 64, C + 2);
  hipLaunchKernelGGL(cls_head_wgrad_kernel, g2, 256, 0, stream, dl, lddl, xhat, dyn, gamma, beta, dW, db, dgamma,
                     dbeta, n, C, D, accumulate ? 1 : 0);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}
int es_cls_head_bwd(const float* dl, int lddl, const float* W, const float* gamma, const float* beta,
                    const float* xhat, const float* rstd, float* dyn, float* dx, int lddx, int T, float* dW, float* db,
                    float* dgamma, float* dbeta, int n, int D, int C, hipStream_t stream) {
  return es_cls_head_bwd_ex(dl, lddl, W, gamma, beta, xhat, rstd, dyn, dx, lddx, T, dW, db, dgamma, dbeta, n, D, C, 1,
                            stream);
}

// CoMatch feature path: fts [n, D] = LN(x_cls) and its backward (dgamma / dbeta accumulated)
int es_cls_ln_fwd(const float* x, int ldx, int T, const float* gamma, const float* beta, float* fts, int ldf,
                  float* xhat, float* rstd, int n, int D, float eps, hipStream_t stream) {
  if (n <= 0 || D % 64) return ES_BAD_SHAPE;
  if (!x || !gamma || !beta || !fts || !xhat || !rstd) return ES_BAD_ARG;
  const int grid = (n + 3) / 4;
  HEAD_DISPATCH(cls_ln_fwd_kernel, D / 64, grid, stream, x, ldx, T, gamma, beta, fts, ldf, xhat, rstd, n, eps);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_cls_ln_bwd(const float* dfts, int lddf, const float* gamma, const float* xhat, const float* rstd, float* dx,
                  int lddx, int T, float* dgamma, float* dbeta, int n, int D, hipStream_t stream) {
  if (n <= 0 || D % 64) return ES_BAD_SHAPE;
  if (!dfts || !gamma || !xhat || !rstd || !dx || !dgamma || !dbeta) return ES_BAD_ARG;
  const int grid = (n + 3) / 4;
  HEAD_DISPATCH(cls_ln_bwd_kernel, D / 64, grid, stream, dfts, lddf, gamma, xhat, rstd, dx, lddx, T, dgamma, dbeta, n);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
