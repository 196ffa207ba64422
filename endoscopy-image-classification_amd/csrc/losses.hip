// Fused FixMatch loss kernels: forward value AND d(loss)/d(logits) in one launch (gfx950).
//
//  es_fm_consistency_fwd_bwd  code/loss.py:126-164 (consistency_loss, name='ce', hard labels):
//      p = softmax(detach(l_w)); (max_p, idx) = max(p, -1)   [first index on ties]
//      mask = (max_p >= tau)                                 [inclusive]
//      loss = mean_i( CE(l_s[i], idx[i]) * mask[i] ),  mask_mean = mean(mask)   (T unused)
//      d loss / d l_s[i][c] = mask[i] * (softmax(l_s[i])_c - [c == idx[i]]) * grad_scale
//  es_poly_ce_fwd_bwd         code/loss.py:103-114,308-364 (PolyLoss, softmax=True, epsilon=2):
//      loss = mean_i( w[y_i] * CE_i + eps * (1 - p_i[y_i]) )   (plain mean, not weight-normalised)
//      d/d l[i][c] = grad_scale * (w[y_i] + eps * p_i[y_i]) * (p_i[c] - [c == y_i])
// The logits are tiny ([448,23] / [64,23]); one workgroup handles all rows, staging each row's
// logits in registers, and emits int32 pseudo-labels, the uint8 mask, per-row losses and the two
// means -- no host sync and no intermediate tensors.
#include "common.h"

namespace {

constexpr int MAXC = 64;

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(256) void fm_consistency_kernel(const float* __restrict__ lw, int ldw,
                                                             const float* __restrict__ ls, int lds_, int n, int C,
                                                             float tau, float grad_scale, int* __restrict__ pl,
                                                             uint8_t* __restrict__ mask_out,
                                                             float* __restrict__ row_loss, float* __restrict__ dls,
                                                             int lddls, float* __restrict__ out) {
  __shared__ float red[16];
  float sum_loss = 0.f, sum_mask = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    // pseudo-label from the weak view (logits re-read from L1 instead of a private array)
    const float* wr = lw + (size_t)i * ldw;
    const float* sr = ls + (size_t)i * lds_;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, wr[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(wr[c] - mx);
    const float inv = 1.0f / se;
    float pmax = -1.f;
    int idx = 0;
    for (int c = 0; c < C; ++c) {
      const float p = __expf(wr[c] - mx) * inv;
      if (p > pmax) {
        pmax = p;
        idx = c;
      }
    }
    const float m = pmax >= tau ? 1.f : 0.f;
    // CE of the strong view against idx
    float mxs = -INFINITY;
    for (int c = 0; c < C; ++c) mxs = fmaxf(mxs, sr[c]);
    float ses = 0.f;
    for (int c = 0; c < C; ++c) ses += __expf(sr[c] - mxs);
    const float lse = mxs + __logf(ses);
    const float ce = lse - sr[idx];
    const float rl = ce * m;
    const float invs = 1.0f / ses;
    for (int c = 0; c < C; ++c) {
      const float p = __expf(sr[c] - mxs) * invs;
      dls[(size_t)i * lddls + c] = m * (p - (c == idx ? 1.f : 0.f)) * grad_scale;
    }
    if (pl) pl[i] = idx;
    if (mask_out) mask_out[i] = (uint8_t)m;
    if (row_loss) row_loss[i] = rl;
    sum_loss += rl;
    sum_mask += m;
  }
  sum_loss = block_sum(sum_loss, red);
  sum_mask = block_sum(sum_mask, red);
  if (threadIdx.x == 0) {
    out[0] = sum_loss / (float)n;
    out[1] = sum_mask / (float)n;
  }
}

__global__ __launch_bounds__(256) void poly_ce_kernel(const float* __restrict__ l, int ldl,
                                                      const int64_t* __restrict__ y, const float* __restrict__ w,
                                                      int n, int C, float eps, float grad_scale,
                                                      float* __restrict__ dl, int lddl, float* __restrict__ out) {
  __shared__ float red[16];
  float sum = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* lr = l + (size_t)i * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, lr[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(lr[c] - mx);
    const float lse = mx + __logf(se);
    const int yi = (int)y[i];
    if ((unsigned)yi >= (unsigned)C) {  // invalid target: NaN loss, no gradient, no out-of-range read
      sum += __int_as_float(0x7fc00000);
      for (int c = 0; c < C; ++c) dl[(size_t)i * lddl + c] = 0.f;
      continue;
    }
    const float wy = w ? w[yi] : 1.f;
    const float py = __expf(lr[yi] - lse);
    sum += wy * (lse - lr[yi]) + eps * (1.f - py);
    const float coef = grad_scale * (wy + eps * py);
    for (int c = 0; c < C; ++c) {
      const float p = __expf(lr[c] - lse);
      dl[(size_t)i * lddl + c] = coef * (p - (c == yi ? 1.f : 0.f));
    }
  }
  sum = block_sum(sum, red);
  if (threadIdx.x == 0) out[0] = sum / (float)n;
}

// F.cross_entropy(logits, y, weight=w, reduction='mean') = sum_i w[y_i] l_i / sum_i w[y_i]
// (code/loss.py:118, the SemiFormer heads' loss, code/semiformer.py:125-126); one workgroup.
__global__ __launch_bounds__(256) void ce_weighted_kernel(const float* __restrict__ l, int ldl,
                                                          const int64_t* __restrict__ y, const float* __restrict__ w,
                                                          const float* __restrict__ wsum_global, int n, int C,
                                                          float grad_scale, float* __restrict__ dl, int lddl,
                                                          float* __restrict__ out) {
  __shared__ float red[16];
  float ws = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int yi = (int)y[i];
    ws += (unsigned)yi >= (unsigned)C ? __int_as_float(0x7fc00000) : (w ? w[yi] : 1.f);
  }
  float W = block_sum(ws, red);
  __syncthreads();
  if (wsum_global) W = *wsum_global;  // the whole batch's weight sum over every rank (data-parallel step)
  const float invW = 1.0f / W;
  float sum = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* lr = l + (size_t)i * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, lr[c]);
    float se = 0.f;
    for (int c = 0; c < C; ++c) se += __expf(lr[c] - mx);
    const float lse = mx + __logf(se);
    const int yi = (int)y[i];
    if ((unsigned)yi >= (unsigned)C) {  // invalid target: NaN loss (via the weight sum), no gradient
      for (int c = 0; c < C; ++c) dl[(size_t)i * lddl + c] = 0.f;
      continue;
    }
    const float wy = w ? w[yi] : 1.f;
    sum += wy * (lse - lr[yi]);
    const float coef = grad_scale * wy * invW;
    for (int c = 0; c < C; ++c) {
      const float p = __expf(lr[c] - lse);
      dl[(size_t)i * lddl + c] = coef * (p - (c == yi ? 1.f : 0.f));
    }
  }
  sum = block_sum(sum, red);
  if (threadIdx.x == 0) out[0] = sum * invW;
}

__global__ __launch_bounds__(256) void ce_weight_sum_kernel(const int64_t* __restrict__ y, const float* __restrict__ w,
                                                            int n, int C, float* __restrict__ out) {
  __shared__ float red[16];
  float ws = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int yi = (int)y[i];
    ws += (unsigned)yi >= (unsigned)C ? __int_as_float(0x7fc00000) : (w ? w[yi] : 1.f);
  }
  ws = block_sum(ws, red);
  if (threadIdx.x == 0) out[0] = ws;
}

}  // namespace

extern "C" {

// out[0] = weighted-mean CE (weights nullable -> plain mean); dl = grad_scale * d(out[0])/d logits
int es_ce_weighted_fwd_bwd(const float* logits, int ldl, const int64_t* targets, const float* weights, int n, int C,
                           float grad_scale, float* dlogits, int lddl, float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0) return ES_BAD_SHAPE;
  if (!logits || !targets || !dlogits || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(ce_weighted_kernel, 1, 256, 0, stream, logits, ldl, targets, weights, nullptr, n, C, grad_scale,
                     dlogits, lddl, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// out[0] = sum_i w[y_i] (the local weight sum of the weighted mean; weights nullable -> n)
int es_ce_weight_sum(const int64_t* targets, const float* weights, int n, int C, float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0) return ES_BAD_SHAPE;
  if (!targets || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(ce_weight_sum_kernel, 1, 256, 0, stream, targets, weights, n, C, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// The data-parallel form: the rows are this rank's shard, *wsum_global the weight sum over every
// rank's rows (es_ce_weight_sum + a SUM all-reduce), so out[0] = this shard's share of the global
// weighted mean, sum_{i in shard} w l_i / W_global, and dl = grad_scale * d(out[0])/d logits.
int es_ce_weighted_fwd_bwd_global(const float* logits, int ldl, const int64_t* targets, const float* weights,
                                  const float* wsum_global, int n, int C, float grad_scale, float* dlogits, int lddl,
                                  float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0) return ES_BAD_SHAPE;
  if (!logits || !targets || !dlogits || !out || !wsum_global) return ES_BAD_ARG;
  hipLaunchKernelGGL(ce_weighted_kernel, 1, 256, 0, stream, logits, ldl, targets, weights, wsum_global, n, C,
                     grad_scale, dlogits, lddl, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// out[0] = loss (mean over n of masked CE), out[1] = mask mean.  dls = d(grad_scale*loss*n)/d l_s
// i.e. pass grad_scale = lambda_u / n for d(lambda_u * loss).  pl / mask_out / row_loss nullable.
int es_fm_consistency_fwd_bwd(const float* logits_w, int ldw, const float* logits_s, int lds, int n, int C,
                              float tau, float grad_scale, int* pseudo_label, uint8_t* mask, float* row_loss,
                              float* dlogits_s, int lddls, float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0 || C > MAXC) return ES_BAD_SHAPE;
  if (!logits_w || !logits_s || !dlogits_s || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(fm_consistency_kernel, 1, 256, 0, stream, logits_w, ldw, logits_s, lds, n, C, tau, grad_scale,
                     pseudo_label, mask, row_loss, dlogits_s, lddls, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// out[0] = poly loss (mean over n); dl = grad_scale * n * d(loss)/d l  (grad_scale = 1/n for d loss)
int es_poly_ce_fwd_bwd(const float* logits, int ldl, const int64_t* targets, const float* weights, int n, int C,
                       float epsilon, float grad_scale, float* dlogits, int lddl, float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0 || C > MAXC) return ES_BAD_SHAPE;
  if (!logits || !targets || !dlogits || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(poly_ce_kernel, 1, 256, 0, stream, logits, ldl, targets, weights, n, C, epsilon, grad_scale,
                     dlogits, lddl, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
