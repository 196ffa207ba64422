// CoMatch on the MI355X (gfx950): ModelwEmb heads over the ViT features and the CoMatch step's
// pseudo-labelling / losses (code/comatch.py:141-222, code/models/custom_model.py:107-145,201-213).
//
//  Heads (fp32, rows = images; tiny next to the backbone):
//    fc       = Linear(D, D/4) -> ReLU -> Dropout(0.2) -> BatchNorm1d(D/4) -> Linear(D/4, C)
//    head_emb = Linear(D, 3L) -> LeakyReLU(0.1) -> Linear(3L, L) -> Normalize(2)
//  es_dense_fwd / es_dense_bwd   Linear (+ activation, + replayed dropout keep-mask)
//  es_bn1d_fwd / es_bn1d_bwd     BatchNorm1d over the batch rows (training statistics, running
//                                buffers with momentum 0.1 and the unbiased variance, as nn.BatchNorm1d)
//  es_l2norm_fwd / _bwd          Normalize(2): v / sqrt(sum v^2)
//  Step (code/comatch.py:162-220):
//  es_comatch_pseudo             softmax(weak) -> distribution alignment over <= 32 batch means
//                                (device ring) -> memory smoothing against the bank
//                                A = exp(z_w . bank^T / T) / rowsum, p = a p + (1-a) A . bank_probs
//                                -> max / first-index argmax / mask (>= thres)
//  es_comatch_bank_write         the gated ring write of [z_w; z_x] and [p_orig; onehot(y)]
//  es_comatch_contrastive_fwd_bwd  sim = exp(z0 z1^T / T) row-normalised, Q = p p^T (diag 1,
//                                >= th, row-normalised), L_c = -mean_i sum_j Q log(sim + 1e-7),
//                                and dL_c / dz0, dz1
//  es_comatch_focal_fwd_bwd      logp = -sum log_softmax(l) p * mask, L_u = mean((1-e^-logp)^g logp)
#include "common.h"

namespace {

constexpr int DR = 16;  // rows per dense workgroup

// Y[i][c] = act(X[i] . W[c] + b[c]) (* keep[i][c] * keep_scale); 16 rows per workgroup staged in
// LDS, one output column per thread with 16 row accumulators.
// act: 0 none, 1 ReLU, 2 LeakyReLU(slope)
__global__ __launch_bounds__(256) void dense_fwd_kernel(const float* __restrict__ X, int ldx,
                                                        const float* __restrict__ W,
                                                        const float* __restrict__ b, float* __restrict__ Y, int ldy,
                                                        int n, int K, int N, int act, float slope,
                                                        const uint8_t* __restrict__ keep, float keep_scale) {
  extern __shared__ float xs[];  // [DR][K]
  const int r0 = blockIdx.x * DR;
  const int rows = min(DR, n - r0);
  for (int id = threadIdx.x; id < DR * K; id += blockDim.x) {
    const int r = id / K, k = id - r * K;
    xs[id] = r < rows ? X[(size_t)(r0 + r) * ldx + k] : 0.f;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    float acc[DR];
#pragma unroll
    for (int r = 0; r < DR; ++r) acc[r] = 0.f;
    const float* w = W + (size_t)c * K;
    for (int k = 0; k < K; ++k) {
      const float wk = w[k];
#pragma unroll
      for (int r = 0; r < DR; ++r) acc[r] = fmaf(xs[r * K + k], wk, acc[r]);
    }
    const float bc = b ? b[c] : 0.f;
    for (int r = 0; r < rows; ++r) {
      float v = acc[r] + bc;
      if (act == 1) v = fmaxf(v, 0.f);
      else if (act == 2) v = v > 0.f ? v : v * slope;
      if (keep) v = v * ((float)keep[(size_t)(r0 + r) * N + c] * keep_scale);
      Y[(size_t)(r0 + r) * ldy + c] = v;
    }
  }
}

// The same Y for few output columns (N < 64: a classifier head, e.g. ResNet-18's 512 -> 23 at B = 16, where
// dense_fwd_kernel keeps N of a workgroup's 256 threads busy over a serial K loop): one wave per output, lanes
// strided over K, a fixed-order wave reduction (deterministic; another summation order than dense_fwd_kernel)
__global__ __launch_bounds__(256) void dense_fwd_small_kernel(const float* __restrict__ X, int ldx,
                                                              const float* __restrict__ W,
                                                              const float* __restrict__ b, float* __restrict__ Y,
                                                              int ldy, int n, int K, int N, int act, float slope,
                                                              const uint8_t* __restrict__ keep, float keep_scale) {
  const int o = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (o >= n * N) return;  // wave-uniform
  const int r = o / N, c = o - r * N;
  const float* x = X + (size_t)r * ldx;
  const float* w = W + (size_t)c * K;
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) acc = fmaf(x[k], w[k], acc);
  acc = warp_sum(acc);
  if (lane == 0) {
    float v = acc + (b ? b[c] : 0.f);
    if (act == 1) v = fmaxf(v, 0.f);
    else if (act == 2) v = v > 0.f ? v : v * slope;
    if (keep) v = v * ((float)keep[(size_t)r * N + c] * keep_scale);
    Y[(size_t)r * ldy + c] = v;
  }
}

// dpre[i][c] = dY[i][c] * act'(Yact[i][c]) (* keep * scale).  The activation derivative is read
// off the stored output: ReLU / LeakyReLU(slope > 0) outputs are > 0 exactly where their inputs
// are, and a dropped element's gradient is 0 whatever the sign.
__global__ void dense_dpre_kernel(const float* __restrict__ dY, int lddy, const float* __restrict__ Yact, int ldya,
                                  int act, float slope, const uint8_t* __restrict__ keep, float keep_scale,
                                  float* __restrict__ dpre, int n, int N) {
  const int id = blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= n * N) return;
  const int i = id / N, c = id - i * N;
  float g = dY[(size_t)i * lddy + c];
  if (keep) g *= (float)keep[id] * keep_scale;
  if (act) {
    const float y = Yact[(size_t)i * ldya + c];
    if (!(y > 0.f)) g = act == 1 ? 0.f : g * slope;
  }
  dpre[id] = g;
}

// dX[i][k] (+)= sum_c dpre[i][c] W[c][k]: 16 rows of dpre in LDS, one column k per thread.
__global__ __launch_bounds__(256) void dense_dx_kernel(const float* __restrict__ dpre, const float* __restrict__ W,
                                                       float* __restrict__ dX, int lddx, int n, int K, int N,
                                                       int accumulate) {
  extern __shared__ float ds[];  // [DR][N]
  const int r0 = blockIdx.x * DR;
  const int rows = min(DR, n - r0);
  for (int id = threadIdx.x; id < DR * N; id += blockDim.x) {
    const int r = id / N;
    ds[id] = r < rows ? dpre[(size_t)r0 * N + id] : 0.f;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x) {
    float acc[DR];
#pragma unroll
    for (int r = 0; r < DR; ++r) acc[r] = 0.f;
    for (int c = 0; c < N; ++c) {
      const float w = W[(size_t)c * K + k];
#pragma unroll
      for (int r = 0; r < DR; ++r) acc[r] = fmaf(ds[r * N + c], w, acc[r]);
    }
    for (int r = 0; r < rows; ++r) {
      float* o = dX + (size_t)(r0 + r) * lddx + k;
      *o = accumulate ? *o + acc[r] : acc[r];
    }
  }
}

// dW[c][k] = sum_i dpre[i][c] X[i][k] (column c per blockIdx.y, k over threads); db[c] = sum_i dpre[i][c],
// summed in row order beside the dW loop (which loads dpre[i][c] anyway) and written by thread 0 of
// the first x-block: one serial pass of dependent loads after the loop took ~200 us at n = 960.
__global__ __launch_bounds__(256) void dense_dw_kernel(const float* __restrict__ dpre, const float* __restrict__ X,
                                                       int ldx, float* __restrict__ dW, float* __restrict__ db, int n,
                                                       int K, int N) {
  const int c = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  const bool want_db = db && blockIdx.x == 0 && threadIdx.x == 0;
  if (k < K || want_db) {
    const int kk = k < K ? k : 0;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, sb = 0.f;
    int i = 0;
    for (; i + 4 <= n; i += 4) {
      const float d0 = dpre[(size_t)i * N + c], d1 = dpre[(size_t)(i + 1) * N + c];
      const float d2 = dpre[(size_t)(i + 2) * N + c], d3 = dpre[(size_t)(i + 3) * N + c];
      a0 = fmaf(d0, X[(size_t)i * ldx + kk], a0);
      a1 = fmaf(d1, X[(size_t)(i + 1) * ldx + kk], a1);
      a2 = fmaf(d2, X[(size_t)(i + 2) * ldx + kk], a2);
      a3 = fmaf(d3, X[(size_t)(i + 3) * ldx + kk], a3);
      sb += d0;
      sb += d1;
      sb += d2;
      sb += d3;
    }
    for (; i < n; ++i) {
      const float d = dpre[(size_t)i * N + c];
      a0 = fmaf(d, X[(size_t)i * ldx + kk], a0);
      sb += d;
    }
    if (k < K) dW[(size_t)c * K + k] = (a0 + a1) + (a2 + a3);
    if (want_db) db[c] = sb;
  }
}

// BatchNorm1d over rows, one workgroup per feature: batch mean / biased variance (two passes),
// y = xhat * gamma + beta; running stats <- (1-m) r + m (mean, unbiased var); eval uses them.
__global__ __launch_bounds__(256) void bn1d_fwd_kernel(const float* __restrict__ U, int ldu,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float* running_mean,
                                                       float* running_var, long long* nbt, float momentum, float eps,
                                                       int train, float* __restrict__ Y, int ldy,
                                                       float* __restrict__ xhat, float* __restrict__ rstd_out, int n,
                                                       int F) {
  __shared__ float red[256];
  const int f = blockIdx.x, t = threadIdx.x;
  float mean, rstd;
  if (train) {
    float s = 0.f;
    for (int i = t; i < n; i += blockDim.x) s += U[(size_t)i * ldu + f];
    red[t] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    mean = red[0] / n;
    __syncthreads();
    float ss = 0.f;
    for (int i = t; i < n; i += blockDim.x) {
      const float d = U[(size_t)i * ldu + f] - mean;
      ss += d * d;
    }
    red[t] = ss;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    const float var = red[0] / n;
    rstd = 1.0f / sqrtf(var + eps);
    if (t == 0) {
      running_mean[f] = (1.f - momentum) * running_mean[f] + momentum * mean;
      running_var[f] = (1.f - momentum) * running_var[f] + momentum * (n > 1 ? var * n / (n - 1) : var);
      if (f == 0 && nbt) *nbt += 1;
      rstd_out[f] = rstd;
    }
  } else {
    mean = running_mean[f];
    rstd = 1.0f / sqrtf(running_var[f] + eps);
  }
  const float g = gamma[f], bt = beta[f];
  for (int i = t; i < n; i += blockDim.x) {
    const float xh = (U[(size_t)i * ldu + f] - mean) * rstd;
    if (xhat) xhat[(size_t)i * F + f] = xh;
    Y[(size_t)i * ldy + f] = xh * g + bt;
  }
}

// dU = gamma * rstd * (dY - mean(dY) - xhat * mean(dY * xhat)); dgamma = sum dY xhat, dbeta = sum dY
__global__ __launch_bounds__(256) void bn1d_bwd_kernel(const float* __restrict__ dY, int lddy,
                                                       const float* __restrict__ xhat,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma, float* __restrict__ dU,
                                                       int lddu, float* __restrict__ dgamma,
                                                       float* __restrict__ dbeta, int n, int F) {
  __shared__ float r1[256], r2[256];
  const int f = blockIdx.x, t = threadIdx.x;
  float s1 = 0.f, s2 = 0.f;
  for (int i = t; i < n; i += blockDim.x) {
    const float g = dY[(size_t)i * lddy + f];
    s1 += g;
    s2 += g * xhat[(size_t)i * F + f];
  }
  r1[t] = s1;
  r2[t] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      r1[t] += r1[t + o];
      r2[t] += r2[t + o];
    }
    __syncthreads();
  }
  const float sdy = r1[0], sdyx = r2[0];
  if (t == 0) {
    dgamma[f] = sdyx;
    dbeta[f] = sdy;
  }
  const float k = gamma[f] * rstd[f], m1 = sdy / n, m2 = sdyx / n;
  for (int i = t; i < n; i += blockDim.x)
    dU[(size_t)i * lddu + f] = k * (dY[(size_t)i * lddy + f] - m1 - xhat[(size_t)i * F + f] * m2);
}

// ---- SyncBatchNorm1d pieces (the data-parallel CoMatch head: BatchNorm1d statistics over the global
// batch, as one process would compute them on the concatenated batch).  The caller all-reduces the
// per-feature sums between launches: S1 = sum x, then S2 = sum (x - S1/N)^2 (the same two-pass
// variance as bn1d_fwd_kernel), and in the backward sum dY, sum dY xhat.
__device__ __forceinline__ float wg_sum256(float v, float* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  const float r = red[0];
  __syncthreads();
  return r;
}

// out[f] = sum_i U[i][f]  (S1 == null)  or  sum_i (U[i][f] - S1[f] / N)^2
__global__ __launch_bounds__(256) void bn1d_sums_kernel(const float* __restrict__ U, int ldu, const float* S1, float N,
                                                        float* __restrict__ out, int n) {
  __shared__ float red[256];
  const int f = blockIdx.x;
  const float c = S1 ? S1[f] / N : 0.f;
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = U[(size_t)i * ldu + f] - c;
    s += S1 ? d * d : d;
  }
  s = wg_sum256(s, red);
  if (threadIdx.x == 0) out[f] = s;
}

__global__ __launch_bounds__(256) void bn1d_fwd_global_kernel(const float* __restrict__ U, int ldu,
                                                              const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, const float* S1,
                                                              const float* S2, float N, float* running_mean,
                                                              float* running_var, long long* nbt, float momentum,
                                                              float eps, float* __restrict__ Y, int ldy,
                                                              float* __restrict__ xhat, float* __restrict__ rstd_out,
                                                              int n, int F) {
  const int f = blockIdx.x, t = threadIdx.x;
  const float mean = S1[f] / N, var = S2[f] / N;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (t == 0) {
    running_mean[f] = (1.f - momentum) * running_mean[f] + momentum * mean;
    running_var[f] = (1.f - momentum) * running_var[f] + momentum * (N > 1.f ? var * N / (N - 1.f) : var);
    if (f == 0 && nbt) *nbt += 1;
    rstd_out[f] = rstd;
  }
  const float g = gamma[f], bt = beta[f];
  for (int i = t; i < n; i += blockDim.x) {
    const float xh = (U[(size_t)i * ldu + f] - mean) * rstd;
    xhat[(size_t)i * F + f] = xh;
    Y[(size_t)i * ldy + f] = xh * g + bt;
  }
}

// out[f] = sum_i dY[i][f], out[F + f] = sum_i dY[i][f] xhat[i][f]  (this rank's rows)
__global__ __launch_bounds__(256) void bn1d_bwd_sums_kernel(const float* __restrict__ dY, int lddy,
                                                            const float* __restrict__ xhat, float* __restrict__ out,
                                                            int n, int F) {
  __shared__ float red[256];
  const int f = blockIdx.x;
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float g = dY[(size_t)i * lddy + f];
    s1 += g;
    s2 += g * xhat[(size_t)i * F + f];
  }
  s1 = wg_sum256(s1, red);
  s2 = wg_sum256(s2, red);
  if (threadIdx.x == 0) {
    out[f] = s1;
    out[F + f] = s2;
  }
}

// dU = gamma rstd (dY - Sg[f]/N - xhat Sg[F+f]/N) with the all-reduced sums Sg; dgamma / dbeta = this
// rank's sums Sl (the gradient all-reduce adds the other ranks')
__global__ __launch_bounds__(256) void bn1d_bwd_global_kernel(const float* __restrict__ dY, int lddy,
                                                              const float* __restrict__ xhat,
                                                              const float* __restrict__ rstd,
                                                              const float* __restrict__ gamma, const float* Sg,
                                                              const float* Sl, float N, float* __restrict__ dU,
                                                              int lddu, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, int n, int F) {
  const int f = blockIdx.x;
  if (threadIdx.x == 0) {
    dgamma[f] = Sl[F + f];
    dbeta[f] = Sl[f];
  }
  const float k = gamma[f] * rstd[f], m1 = Sg[f] / N, m2 = Sg[F + f] / N;
  for (int i = threadIdx.x; i < n; i += blockDim.x)
    dU[(size_t)i * lddu + f] = k * (dY[(size_t)i * lddy + f] - m1 - xhat[(size_t)i * F + f] * m2);
}

// Normalize(2): one wave per row, L <= 256
__global__ __launch_bounds__(256) void l2norm_fwd_kernel(const float* __restrict__ V, int ldv, float* __restrict__ Z,
                                                         int ldz, float* __restrict__ nrm, int n, int L) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  float s = 0.f;
  for (int c = lane; c < L; c += 64) {
    const float v = V[(size_t)i * ldv + c];
    s += v * v;
  }
  const float nv = sqrtf(warp_sum(s));
  for (int c = lane; c < L; c += 64) Z[(size_t)i * ldz + c] = V[(size_t)i * ldv + c] / nv;
  if (lane == 0) nrm[i] = nv;
}

// dV = (dZ - Z (Z . dZ)) / norm
__global__ __launch_bounds__(256) void l2norm_bwd_kernel(const float* __restrict__ dZ, int lddz,
                                                         const float* __restrict__ Z, int ldz,
                                                         const float* __restrict__ nrm, float* __restrict__ dV,
                                                         int lddv, int n, int L) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  float s = 0.f;
  for (int c = lane; c < L; c += 64) s += Z[(size_t)i * ldz + c] * dZ[(size_t)i * lddz + c];
  s = warp_sum(s);
  const float inv = 1.0f / nrm[i];
  for (int c = lane; c < L; c += 64)
    dV[(size_t)i * lddv + c] = (dZ[(size_t)i * lddz + c] - Z[(size_t)i * ldz + c] * s) * inv;
}

// ---- CoMatch pseudo-labels (code/comatch.py:162-185) -------------------------------------------
// Stage 1 (one workgroup): softmax of the weak logits, the batch mean appended to the DA ring
// (hist[pos]), prob_avg = mean of the ring's len entries oldest -> newest, p /= prob_avg,
// p /= rowsum -> probs_orig.
__global__ __launch_bounds__(256) void comatch_da_kernel(const float* __restrict__ lw, int ldl, int nu, int C,
                                                         float* __restrict__ hist, int cap, int len, int pos,
                                                         int hist_given, float* __restrict__ probs_orig) {
  __shared__ float colsum[256];
  __shared__ float avg[256];
  const int t = threadIdx.x;
  // softmax rows: one thread per row (C <= 256 is tiny)
  for (int i = t; i < nu; i += blockDim.x) {
    const float* l = lw + (size_t)i * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, l[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(l[c] - mx);
    for (int c = 0; c < C; ++c) probs_orig[(size_t)i * C + c] = expf(l[c] - mx) / s;
  }
  __syncthreads();
  if (t < C && !hist_given) {  // hist_given: the entry was written by the caller (all-ranks mean)
    float s = 0.f;
    for (int i = 0; i < nu; ++i) s += probs_orig[(size_t)i * C + t];
    hist[(size_t)pos * C + t] = s / nu;
  }
  __syncthreads();
  if (t < C) {
    float s = 0.f;
    for (int j = 0; j < len; ++j) {
      int e = pos - (len - 1) + j;
      e = e < 0 ? e + cap : e;
      s += hist[(size_t)e * C + t];
    }
    avg[t] = s / len;
  }
  __syncthreads();
  for (int i = t; i < nu; i += blockDim.x) {
    float* p = probs_orig + (size_t)i * C;
    float s = 0.f;
    for (int c = 0; c < C; ++c) {
      p[c] = p[c] / avg[c];
      s += p[c];
    }
    for (int c = 0; c < C; ++c) p[c] = p[c] / s;
  }
  (void)colsum;
}

// Stage 2: memory smoothing partials on the fp32 matrix cores (v_mfma_f32_16x16x4_f32, a k-ordered
// fmaf chain, so S is bit-identical to an fp32 dot product).  Workgroup (chunk, row group): SB bank
// rows staged in LDS (features [SB][L+1], probabilities [SB][32] zero-padded), 4 waves x 16 weak
// rows.  Per 16-bank-row tile a wave computes S^T = F . Z^T (A = bank features from LDS, B = its
// rows' embeddings held in registers for the whole chunk), e = exp(S / T), S_e += e, and
// S_p += E . bank_probs with E straight from the first product's accumulator: lane (g, r) holds
// S^T[bank 4g + q][row r] = E[row r][bank 4g + q], which is the A operand of k-step q when the
// B operand (bank_probs, from LDS) uses the same bank order.  Partials [chunk][row][C+1].
constexpr int SB = 128;
__global__ __launch_bounds__(256) void comatch_smooth_partial_kernel(const float* __restrict__ zw, int ldz, int nu,
                                                                     int L, const float* __restrict__ bf,
                                                                     const float* __restrict__ bp, int Q, int C,
                                                                     float temperature, float* __restrict__ part) {
  extern __shared__ float sm[];
  const int LP = L + 1;
  float* fs = sm;            // [SB][L + 1]
  float* ps = sm + SB * LP;  // [SB][32]
  const int chunk = blockIdx.x, j0 = chunk * SB, nb = min(SB, Q - j0);
  for (int id = threadIdx.x; id < SB * L; id += blockDim.x) {
    const int jj = id / L, k = id - jj * L;
    fs[jj * LP + k] = jj < nb ? bf[(size_t)(j0 + jj) * L + k] : 0.f;
  }
  for (int id = threadIdx.x; id < SB * 32; id += blockDim.x) {
    const int jj = id >> 5, c = id & 31;
    ps[id] = (jj < nb && c < C) ? bp[(size_t)(j0 + jj) * C + c] : 0.f;
  }
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lg = lane >> 4;
  const int r0 = blockIdx.y * 64 + w * 16;
  const int ksteps = (L + 3) >> 2;
  float zb[16];  // B operand of S^T = F . Z^T: zb[s] = Z[r0 + lr][4s + lg]  (L <= 64)
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const int k = 4 * st + lg;
    zb[st] = (r0 + lr < nu && k < L) ? zw[(size_t)(r0 + lr) * ldz + k] : 0.f;
  }
  f32x4 pacc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float se = 0.f;
  for (int jt = 0; jt * 16 < nb; ++jt) {
    f32x4 sv = {0.f, 0.f, 0.f, 0.f};
    const float* frow = fs + (jt * 16 + lr) * LP;
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      if (st < ksteps) {
        const int k = 4 * st + lg;
        sv = __builtin_amdgcn_mfma_f32_16x16x4f32(k < L ? frow[k] : 0.f, zb[st], sv, 0, 0, 0);
      }
    }
    float e[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      e[q] = jt * 16 + 4 * lg + q < nb ? expf(sv[q] / temperature) : 0.f;
      se += e[q];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* prow = ps + (jt * 16 + 4 * lg + q) * 32;
      pacc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(e[q], prow[lr], pacc[0], 0, 0, 0);
      pacc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(e[q], prow[16 + lr], pacc[1], 0, 0, 0);
    }
  }
  // S_e of weak row r0 + lr: the 4 lane groups hold disjoint bank rows of it
  se += __shfl_xor(se, 16, 64);
  se += __shfl_xor(se, 32, 64);
  // pacc[nt] lane holds S_p[row r0 + 4 lg + q][class 16 nt + lr]
#pragma unroll
  for (int nt = 0; nt < 2; ++nt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = r0 + 4 * lg + q, c = nt * 16 + lr;
      if (r < nu && c < C) part[((size_t)chunk * nu + r) * (C + 1) + c] = pacc[nt][q];
    }
  if (lg == 0 && r0 + lr < nu) part[((size_t)chunk * nu + r0 + lr) * (C + 1) + C] = se;
}

// Stage 3 (one workgroup per weak row): the C+1 chunk sums in a fixed-order block reduction, then
// p = a p_orig + (1-a) S_p / S_e; score / first-index argmax / mask.
__global__ __launch_bounds__(256) void comatch_pseudo_final_kernel(const float* __restrict__ probs_orig,
                                                                   const float* __restrict__ part, int nchunks,
                                                                   int nu, int C, float alpha, float thres,
                                                                   float* __restrict__ probs, int* __restrict__ pl,
                                                                   float* __restrict__ mask) {
  __shared__ float red[33][256];
  const int i = blockIdx.x, t = threadIdx.x;
  float acc[33];
#pragma unroll
  for (int c = 0; c < 33; ++c) acc[c] = 0.f;
  for (int k = t; k < nchunks; k += 256) {
    const float* pr = part + ((size_t)k * nu + i) * (C + 1);
#pragma unroll
    for (int c = 0; c < 33; ++c)
      if (c <= C) acc[c] += pr[c];
  }
#pragma unroll
  for (int c = 0; c < 33; ++c) red[c][t] = acc[c];
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h)
#pragma unroll
      for (int c = 0; c < 33; ++c) red[c][t] += red[c][t + h];
    __syncthreads();
  }
  if (t != 0) return;
  const float se = red[C][0];
  float best = -INFINITY;
  int bi = 0;
  for (int c = 0; c < C; ++c) {
    const float v = alpha * probs_orig[(size_t)i * C + c] + (1.f - alpha) * (red[c][0] / se);
    probs[(size_t)i * C + c] = v;
    if (v > best) {  // strict: first index on ties (torch.max)
      best = v;
      bi = c;
    }
  }
  pl[i] = bi;
  mask[i] = best >= thres ? 1.f : 0.f;
}

// bank rows [ptr, ptr + nu) <- z_w, probs_orig; [ptr + nu, ptr + nu + bt) <- z_x, onehot(y)
__global__ void comatch_bank_write_kernel(const float* __restrict__ zw, int ldzw, int nu,
                                          const float* __restrict__ zx, int ldzx, int bt, int L,
                                          const float* __restrict__ probs_orig, const long long* __restrict__ y,
                                          int C, float* __restrict__ bf, float* __restrict__ bp, int ptr) {
  const int i = blockIdx.x;  // bank row offset
  const int row = ptr + i;
  for (int c = threadIdx.x; c < L; c += blockDim.x)
    bf[(size_t)row * L + c] = i < nu ? zw[(size_t)i * ldzw + c] : zx[(size_t)(i - nu) * ldzx + c];
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    bp[(size_t)row * C + c] = i < nu ? probs_orig[(size_t)i * C + c] : (y[i - nu] == c ? 1.f : 0.f);
}

// ---- contrastive (code/comatch.py:199-213) ------------------------------------------------------
// One workgroup per anchor row i (nr local rows, global index row_off + i) against nc columns
// (the global batch: all-gathered z1 / probs at world > 1): sim_ij = exp((z0_i . z1_j) / T),
// P = sim / rowsum; Q_ij = p_i . p_j with Q_ii = 1 (the row's own column), zeroed below th,
// row-normalised; loss_i = -sum_j Q_ij log(P_ij + 1e-7).
// dloss_i/ds_ik = P_ik sum_j w_ij - w_ik with w_ij = Q_ij P_ij / (P_ij + 1e-7); the rows of
// G = scale * dloss/ds / T feed dz0 = G z1 and dz1 = G^T z0.
__global__ __launch_bounds__(256) void contrast_rows_kernel(const float* __restrict__ z0, int ldz0,
                                                            const float* __restrict__ z1, int ldz1,
                                                            const float* __restrict__ probs_r,
                                                            const float* __restrict__ probs_c, int nr, int nc,
                                                            int row_off, int L, int C, float temperature, float th,
                                                            float scale, float* __restrict__ G,
                                                            float* __restrict__ row_loss) {
  extern __shared__ float sm[];  // sim [nc], q [nc], z0_i [L], p_i [C]
  __shared__ float red[256];
  float* sim = sm;
  float* q = sm + nc;
  float* zi = q + nc;
  float* pi = zi + L;
  const int i = blockIdx.x, t = threadIdx.x;
  for (int c = t; c < L; c += blockDim.x) zi[c] = z0[(size_t)i * ldz0 + c];
  for (int c = t; c < C; c += blockDim.x) pi[c] = probs_r[(size_t)i * C + c];
  __syncthreads();
  float ssum = 0.f, qsum = 0.f;
  for (int j = t; j < nc; j += blockDim.x) {
    float d = 0.f;
    for (int c = 0; c < L; ++c) d = fmaf(zi[c], z1[(size_t)j * ldz1 + c], d);
    const float e = expf(d / temperature);
    sim[j] = e;
    ssum += e;
    float qq = 0.f;
    for (int c = 0; c < C; ++c) qq = fmaf(pi[c], probs_c[(size_t)j * C + c], qq);
    if (j == row_off + i) qq = 1.f;
    qq = qq >= th ? qq : 0.f;
    q[j] = qq;
    qsum += qq;
  }
  auto block_sum = [&](float v) {
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if (t < o) red[t] += red[t + o];
      __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
  };
  ssum = block_sum(ssum);
  qsum = block_sum(qsum);
  float lsum = 0.f, wsum = 0.f;
  for (int j = t; j < nc; j += blockDim.x) {
    const float P = sim[j] / ssum, Qn = q[j] / qsum;
    lsum -= logf(P + 1e-7f) * Qn;
    const float w = Qn * P / (P + 1e-7f);
    sim[j] = P;
    q[j] = w;
    wsum += w;
  }
  lsum = block_sum(lsum);
  wsum = block_sum(wsum);
  const float k = scale / temperature;
  for (int j = t; j < nc; j += blockDim.x) G[(size_t)i * nc + j] = k * (sim[j] * wsum - q[j]);
  if (t == 0) row_loss[i] = lsum;
}

// dz0[r] = sum_k G[r][k] z1[k] over the nc columns (blockIdx.y = 0, r < nr) and dz1[r] = sum_i G[i][r]
// z0[i] over the nr local rows (blockIdx.y = 1, r < nc): one wave per output row, lanes over L
__global__ __launch_bounds__(256) void contrast_dz_kernel(const float* __restrict__ G, const float* __restrict__ z0,
                                                          int ldz0, const float* __restrict__ z1, int ldz1,
                                                          float* __restrict__ dz0, int lddz0, float* __restrict__ dz1,
                                                          int lddz1, int nr, int nc, int L) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const bool t1 = blockIdx.y == 1;
  if (r >= (t1 ? nc : nr)) return;
  for (int c = lane; c < L; c += 64) {
    float acc = 0.f;
    if (!t1) {
      for (int k = 0; k < nc; ++k) acc = fmaf(G[(size_t)r * nc + k], z1[(size_t)k * ldz1 + c], acc);
      dz0[(size_t)r * lddz0 + c] = acc;
    } else {
      for (int i = 0; i < nr; ++i) acc = fmaf(G[(size_t)i * nc + r], z0[(size_t)i * ldz0 + c], acc);
      dz1[(size_t)r * lddz1 + c] = acc;
    }
  }
}

// sum of per-row values / div (one workgroup) -> out[0]
__global__ __launch_bounds__(256) void row_mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out,
                                                       float div) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  float s = 0.f;
  for (int i = t; i < n; i += blockDim.x) s += v[i];
  red[t] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  if (t == 0) out[0] = red[0] / div;
}

// ---- focal unsupervised loss (code/comatch.py:215-220) ------------------------------------------
// One thread per row: logp = -mask * sum_c log_softmax(l)_c p_c, q = exp(-logp),
// loss = (1-q)^g logp; dloss/dl_c = scale * dL/dlogp * (-mask) (p_c - softmax_c sum p),
// dL/dlogp = g (1-q)^(g-1) q logp + (1-q)^g.  Row losses -> row_loss.
__global__ void focal_kernel(const float* __restrict__ ls, int ldl, const float* __restrict__ probs,
                             const float* __restrict__ mask, int nu, int C, float gamma, float scale,
                             float* __restrict__ dls, int lddl, float* __restrict__ row_loss) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nu) return;
  const float* l = ls + (size_t)i * ldl;
  const float* p = probs + (size_t)i * C;
  float mx = -INFINITY;
  for (int c = 0; c < C; ++c) mx = fmaxf(mx, l[c]);
  float se = 0.f;
  for (int c = 0; c < C; ++c) se += expf(l[c] - mx);
  const float lse = mx + logf(se);
  float dot = 0.f, psum = 0.f;
  for (int c = 0; c < C; ++c) {
    dot += (l[c] - lse) * p[c];
    psum += p[c];
  }
  const float m = mask[i];
  const float logp = -dot * m;
  const float q = expf(-logp);
  const float om = 1.f - q;
  const float pw = gamma == 2.f ? om * om : powf(om, gamma);
  row_loss[i] = pw * logp;
  const float dpw = gamma == 2.f ? 2.f * om : gamma * powf(om, gamma - 1.f);
  const float dL = dpw * q * logp + pw;
  for (int c = 0; c < C; ++c) {
    const float sm = expf(l[c] - lse);
    dls[(size_t)i * lddl + c] = scale * dL * (-m) * (p[c] - sm * psum);
  }
}

// Dropout keep-mask: counter-based (splitmix64 of seed + element index), keep = u >= p with u the
// top 24 bits as a uniform [0, 1) -- reproducible for a (seed, offset) pair, no RNG state.
__global__ void dropout_keep_kernel(uint8_t* __restrict__ keep, long n, float p, unsigned long long seed,
                                    unsigned long long offset) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned long long z = seed + 0x9E3779B97F4A7C15ull * (offset + (unsigned long long)i + 1ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
  keep[i] = u >= p ? 1 : 0;
}

}  // namespace

extern "C" {

// Dropout(p) keep-mask for n elements (uint8 0/1); the kept values are scaled by 1/(1-p) by the
// consumer (es_dense_fwd keep_scale)
int es_dropout_keep(void* keep, long n, float p, unsigned long long seed, unsigned long long offset,
                    hipStream_t stream) {
  if (n < 0 || !(p >= 0.f && p < 1.f)) return ES_BAD_SHAPE;
  if (!keep) return ES_BAD_ARG;
  if (n == 0) return ES_OK;
  hipLaunchKernelGGL(dropout_keep_kernel, (unsigned)((n + 255) / 256), 256, 0, stream, (uint8_t*)keep, n, p, seed,
                     offset);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}


int es_dense_fwd(const float* X, int ldx, const float* W, const float* b, float* Y, int ldy, int n, int K, int N,
                 int act, float slope, const void* keep, float keep_scale, hipStream_t stream) {
  if (n <= 0 || K <= 0 || N <= 0 || K > 2048 || act < 0 || act > 2) return ES_BAD_SHAPE;
  if (!X || !W || !Y) return ES_BAD_ARG;
  if (N < 64) {
    const long outs = (long)n * N;
    hipLaunchKernelGGL(dense_fwd_small_kernel, (unsigned)((outs + 3) / 4), 256, 0, stream, X, ldx, W, b, Y, ldy, n, K, N,
                       act, slope, (const uint8_t*)keep, keep_scale);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  const size_t lds = (size_t)DR * K * 4;
  allow_lds(dense_fwd_kernel, lds);
  hipLaunchKernelGGL(dense_fwd_kernel, (n + DR - 1) / DR, 256, lds, stream, X, ldx, W, b, Y, ldy, n, K, N, act, slope,
                     (const uint8_t*)keep, keep_scale);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

size_t es_dense_bwd_workspace(int n, int N) { return (size_t)n * N; }

// Backward of Y = act(X W^T + b) (* keep * scale): dW, db (overwritten), dX (+)= when dX != null.
// workspace: es_dense_bwd_workspace(n, N) floats.
int es_dense_bwd(const float* dY, int lddy, const float* Yact, int ldya, int act, float slope, const void* keep,
                 float keep_scale, const float* X, int ldx, const float* W, float* dX, int lddx, int accumulate_dx,
                 float* dW, float* db, int n, int K, int N, float* workspace, hipStream_t stream) {
  if (n <= 0 || K <= 0 || N <= 0 || N > 2048 || act < 0 || act > 2) return ES_BAD_SHAPE;
  if (!dY || !X || !W || !dW || !workspace || (act && !Yact)) return ES_BAD_ARG;
  hipLaunchKernelGGL(dense_dpre_kernel, (n * N + 255) / 256, 256, 0, stream, dY, lddy, Yact, ldya, act, slope,
                     (const uint8_t*)keep, keep_scale, workspace, n, N);
  hipLaunchKernelGGL(dense_dw_kernel, dim3((K + 255) / 256, N), 256, 0, stream, workspace, X, ldx, dW, db, n, K, N);
  if (dX) {
    const size_t lds = (size_t)DR * N * 4;
    allow_lds(dense_dx_kernel, lds);
    hipLaunchKernelGGL(dense_dx_kernel, (n + DR - 1) / DR, 256, lds, stream, workspace, W, dX, lddx, n, K, N,
                       accumulate_dx);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// BatchNorm1d over n rows x F features (nn.BatchNorm1d semantics).  train: batch statistics,
// running buffers updated (num_batches_tracked += 1 when nbt != null), xhat / rstd saved;
// eval: running statistics.
int es_bn1d_fwd(const float* U, int ldu, const float* gamma, const float* beta, float* running_mean, float* running_var,
                void* num_batches_tracked, float momentum, float eps, int train, float* Y, int ldy, float* xhat,
                float* rstd, int n, int F, hipStream_t stream) {
  if (n <= 0 || F <= 0) return ES_BAD_SHAPE;
  if (!U || !gamma || !beta || !running_mean || !running_var || !Y || (train && (!xhat || !rstd))) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_fwd_kernel, F, 256, 0, stream, U, ldu, gamma, beta, running_mean, running_var,
                     (long long*)num_batches_tracked, momentum, eps, train, Y, ldy, xhat, rstd, n, F);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_bn1d_bwd(const float* dY, int lddy, const float* xhat, const float* rstd, const float* gamma, float* dU,
                int lddu, float* dgamma, float* dbeta, int n, int F, hipStream_t stream) {
  if (n <= 0 || F <= 0) return ES_BAD_SHAPE;
  if (!dY || !xhat || !rstd || !gamma || !dU || !dgamma || !dbeta) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_bwd_kernel, F, 256, 0, stream, dY, lddy, xhat, rstd, gamma, dU, lddu, dgamma, dbeta, n, F);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// SyncBatchNorm1d (data-parallel CoMatch head), see the kernels above.  N = global row count.
int es_bn1d_sums(const float* U, int ldu, int n, int F, const float* S1, float N, float* out, hipStream_t stream) {
  if (n <= 0 || F <= 0 || N < (float)n) return ES_BAD_SHAPE;
  if (!U || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_sums_kernel, F, 256, 0, stream, U, ldu, S1, N, out, n);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_bn1d_fwd_global(const float* U, int ldu, const float* gamma, const float* beta, const float* S1,
                       const float* S2, float N, float* running_mean, float* running_var, void* num_batches_tracked,
                       float momentum, float eps, float* Y, int ldy, float* xhat, float* rstd, int n, int F,
                       hipStream_t stream) {
  if (n <= 0 || F <= 0 || N < (float)n) return ES_BAD_SHAPE;
  if (!U || !gamma || !beta || !S1 || !S2 || !running_mean || !running_var || !Y || !xhat || !rstd) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_fwd_global_kernel, F, 256, 0, stream, U, ldu, gamma, beta, S1, S2, N, running_mean,
                     running_var, (long long*)num_batches_tracked, momentum, eps, Y, ldy, xhat, rstd, n, F);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_bn1d_bwd_sums(const float* dY, int lddy, const float* xhat, int n, int F, float* out, hipStream_t stream) {
  if (n <= 0 || F <= 0) return ES_BAD_SHAPE;
  if (!dY || !xhat || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_bwd_sums_kernel, F, 256, 0, stream, dY, lddy, xhat, out, n, F);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_bn1d_bwd_global(const float* dY, int lddy, const float* xhat, const float* rstd, const float* gamma,
                       const float* sums_global, const float* sums_local, float N, float* dU, int lddu,
                       float* dgamma, float* dbeta, int n, int F, hipStream_t stream) {
  if (n <= 0 || F <= 0 || N < (float)n) return ES_BAD_SHAPE;
  if (!dY || !xhat || !rstd || !gamma || !sums_global || !sums_local || !dU || !dgamma || !dbeta) return ES_BAD_ARG;
  hipLaunchKernelGGL(bn1d_bwd_global_kernel, F, 256, 0, stream, dY, lddy, xhat, rstd, gamma, sums_global, sums_local,
                     N, dU, lddu, dgamma, dbeta, n, F);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_l2norm_fwd(const float* V, int ldv, float* Z, int ldz, float* norm, int n, int L, hipStream_t stream) {
  if (n <= 0 || L <= 0) return ES_BAD_SHAPE;
  if (!V || !Z || !norm) return ES_BAD_ARG;
  hipLaunchKernelGGL(l2norm_fwd_kernel, (n + 3) / 4, 256, 0, stream, V, ldv, Z, ldz, norm, n, L);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_l2norm_bwd(const float* dZ, int lddz, const float* Z, int ldz, const float* norm, float* dV, int lddv, int n,
                  int L, hipStream_t stream) {
  if (n <= 0 || L <= 0) return ES_BAD_SHAPE;
  if (!dZ || !Z || !norm || !dV) return ES_BAD_ARG;
  hipLaunchKernelGGL(l2norm_bwd_kernel, (n + 3) / 4, 256, 0, stream, dZ, lddz, Z, ldz, norm, dV, lddv, n, L);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

size_t es_comatch_pseudo_workspace(int nu, int C, int Q) {
  const int nchunks = (Q + SB - 1) / SB;
  return (size_t)nchunks * nu * (C + 1);
}

// out[c] = mean_i softmax(l_i)[c]: the DA batch mean, for the data-parallel path (all-reduced
// across ranks, then handed to es_comatch_pseudo_ex with hist_given = 1)
__global__ __launch_bounds__(256) void softmax_colmean_kernel(const float* __restrict__ lw, int ldl, int n, int C,
                                                              float* __restrict__ out) {
  __shared__ float acc[32];
  if (threadIdx.x < 32) acc[threadIdx.x] = 0.f;
  __syncthreads();
  float loc[32];
  for (int c = 0; c < C; ++c) loc[c] = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* l = lw + (size_t)i * ldl;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, l[c]);
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += expf(l[c] - mx);
    for (int c = 0; c < C; ++c) loc[c] += expf(l[c] - mx) / s;
  }
  for (int c = 0; c < C; ++c) atomicAdd(&acc[c], loc[c]);
  __syncthreads();
  if (threadIdx.x < C) out[threadIdx.x] = acc[threadIdx.x] / n;
}

int es_softmax_colmean(const float* logits, int ldl, int n, int C, float* out, hipStream_t stream) {
  if (n <= 0 || C <= 0 || C > 32) return ES_BAD_SHAPE;
  if (!logits || !out) return ES_BAD_ARG;
  hipLaunchKernelGGL(softmax_colmean_kernel, 1, 256, 0, stream, logits, ldl, n, C, out);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_comatch_pseudo_ex(const float* logits_w, int ldl, int nu, int C, float* hist, int hist_cap, int hist_len,
                         int hist_pos, int hist_given, const float* z_w, int ldz, int L, const float* bank_feats,
                         const float* bank_probs, int Q, float temperature, float alpha, float thres, float* probs,
                         float* probs_orig, int* pl, float* mask, float* workspace, hipStream_t stream);

// Pseudo-labels of the weak rows: DA (append this batch's mean to hist[hist_pos], average the
// hist_len newest entries of the hist_cap ring), memory smoothing against the bank (Q rows),
// argmax / mask.  probs_orig is the DA output (what the bank stores), probs the smoothed one.
int es_comatch_pseudo(const float* logits_w, int ldl, int nu, int C, float* hist, int hist_cap, int hist_len,
                      int hist_pos, const float* z_w, int ldz, int L, const float* bank_feats, const float* bank_probs,
                      int Q, float temperature, float alpha, float thres, float* probs, float* probs_orig, int* pl,
                      float* mask, float* workspace, hipStream_t stream) {
  return es_comatch_pseudo_ex(logits_w, ldl, nu, C, hist, hist_cap, hist_len, hist_pos, 0, z_w, ldz, L, bank_feats,
                              bank_probs, Q, temperature, alpha, thres, probs, probs_orig, pl, mask, workspace, stream);
}

// as es_comatch_pseudo; hist_given = 1: hist[hist_pos] already holds this step's batch mean (the
// data-parallel path writes the all-ranks mean there) and is not recomputed from the local rows
int es_comatch_pseudo_ex(const float* logits_w, int ldl, int nu, int C, float* hist, int hist_cap, int hist_len,
                         int hist_pos, int hist_given, const float* z_w, int ldz, int L, const float* bank_feats,
                         const float* bank_probs, int Q, float temperature, float alpha, float thres, float* probs,
                         float* probs_orig, int* pl, float* mask, float* workspace, hipStream_t stream) {
  if (nu <= 0 || C <= 0 || C > 32 || L <= 0 || L > 64 || Q <= 0 || hist_cap <= 0 || hist_len <= 0 ||
      hist_len > hist_cap || hist_pos < 0 || hist_pos >= hist_cap)
    return ES_BAD_SHAPE;
  if (!logits_w || !hist || !z_w || !bank_feats || !bank_probs || !probs || !probs_orig || !pl || !mask || !workspace)
    return ES_BAD_ARG;
  hipLaunchKernelGGL(comatch_da_kernel, 1, 256, 0, stream, logits_w, ldl, nu, C, hist, hist_cap, hist_len, hist_pos,
                     hist_given, probs_orig);
  const int nchunks = (Q + SB - 1) / SB;
  const size_t lds = (size_t)SB * (L + 1 + 32) * 4;
  allow_lds(comatch_smooth_partial_kernel, lds);
  hipLaunchKernelGGL(comatch_smooth_partial_kernel, dim3(nchunks, (nu + 63) / 64), 256, lds, stream, z_w, ldz, nu, L,
                     bank_feats, bank_probs, Q, C, temperature, workspace);
  hipLaunchKernelGGL(comatch_pseudo_final_kernel, nu, 256, 0, stream, probs_orig, workspace, nchunks, nu, C, alpha,
                     thres, probs, pl, mask);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_comatch_bank_write(const float* z_w, int ldzw, int nu, const float* z_x, int ldzx, int bt, int L,
                          const float* probs_orig, const void* y_int64, int C, float* bank_feats, float* bank_probs,
                          int ptr, int Q, hipStream_t stream) {
  if (nu < 0 || bt < 0 || L <= 0 || C <= 0 || ptr < 0 || ptr + nu + bt > Q) return ES_BAD_SHAPE;
  if (!z_w || !z_x || !probs_orig || !y_int64 || !bank_feats || !bank_probs) return ES_BAD_ARG;
  if (nu + bt == 0) return ES_OK;
  hipLaunchKernelGGL(comatch_bank_write_kernel, nu + bt, 64, 0, stream, z_w, ldzw, nu, z_x, ldzx, bt, L, probs_orig,
                     (const long long*)y_int64, C, bank_feats, bank_probs, ptr);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

size_t es_comatch_contrastive_workspace(int nu) { return (size_t)nu * nu + nu; }
size_t es_comatch_contrastive_ex_workspace(int nr, int nc) { return (size_t)nr * nc + nr; }

static int contrastive_launch(const float* z0, int ldz0, const float* z1, int ldz1, const float* probs_r,
                              const float* probs_c, int nr, int nc, int row_off, int L, int C, float temperature,
                              float contrast_th, float grad_scale, float loss_div, float* loss_out, float* dz0,
                              int lddz0, float* dz1, int lddz1, float* workspace, hipStream_t stream) {
  if (nr <= 0 || nc < nr || nc > 8192 || row_off < 0 || row_off + nr > nc || L <= 0 || C <= 0) return ES_BAD_SHAPE;
  if (!z0 || !z1 || !probs_r || !probs_c || !loss_out || !dz0 || !dz1 || !workspace) return ES_BAD_ARG;
  float* G = workspace;
  float* row_loss = workspace + (size_t)nr * nc;
  const size_t lds = (size_t)(2 * nc + L + C) * 4;
  allow_lds(contrast_rows_kernel, lds);
  hipLaunchKernelGGL(contrast_rows_kernel, nr, 256, lds, stream, z0, ldz0, z1, ldz1, probs_r, probs_c, nr, nc, row_off,
                     L, C, temperature, contrast_th, grad_scale, G, row_loss);
  hipLaunchKernelGGL(contrast_dz_kernel, dim3((nc + 3) / 4, 2), 256, 0, stream, G, z0, ldz0, z1, ldz1, dz0, lddz0, dz1,
                     lddz1, nr, nc, L);
  hipLaunchKernelGGL(row_mean_kernel, 1, 256, 0, stream, row_loss, nr, loss_out, loss_div);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// loss_out[0] = L_c = mean_i L_i (unscaled); dz0 / dz1 = grad_scale * d(sum_i L_i) / dz (overwritten)
int es_comatch_contrastive_fwd_bwd(const float* z0, int ldz0, const float* z1, int ldz1, const float* probs, int nu,
                                   int L, int C, float temperature, float contrast_th, float grad_scale,
                                   float* loss_out, float* dz0, int lddz0, float* dz1, int lddz1, float* workspace,
                                   hipStream_t stream) {
  return contrastive_launch(z0, ldz0, z1, ldz1, probs, probs, nu, nu, 0, L, C, temperature, contrast_th, grad_scale,
                            (float)nu, loss_out, dz0, lddz0, dz1, lddz1, workspace, stream);
}

// The data-parallel form: this rank's nr anchor rows (global rows row_off .. row_off + nr - 1)
// against the nc global columns (z1_all / probs_all: the all-gathered batch).  loss_out[0] =
// sum over the local rows / loss_div (pass the global row count: the ranks' values then sum to L_c);
// dz0 [nr, L] for the local rows, dz1 [nc, L] this rank's share of d/dz1 for EVERY column (the
// caller sums the shares over ranks and keeps its own rows).
int es_comatch_contrastive_fwd_bwd_ex(const float* z0, int ldz0, const float* z1_all, int ldz1,
                                      const float* probs_rows, const float* probs_all, int nr, int nc, int row_off,
                                      int L, int C, float temperature, float contrast_th, float grad_scale,
                                      float loss_div, float* loss_out, float* dz0, int lddz0, float* dz1_all,
                                      int lddz1, float* workspace, hipStream_t stream) {
  return contrastive_launch(z0, ldz0, z1_all, ldz1, probs_rows, probs_all, nr, nc, row_off, L, C, temperature,
                            contrast_th, grad_scale, loss_div, loss_out, dz0, lddz0, dz1_all, lddz1, workspace, stream);
}

// loss_out[0] = L_u = mean_i L_i (unscaled); dls = grad_scale * d(sum_i L_i) / dlogits_s0 (overwritten);
// workspace nu floats
int es_comatch_focal_fwd_bwd(const float* ls, int ldl, const float* probs, const float* mask, int nu, int C,
                             float gamma, float grad_scale, float* loss_out, float* dls, int lddl, float* workspace,
                             hipStream_t stream) {
  if (nu <= 0 || C <= 0) return ES_BAD_SHAPE;
  if (!ls || !probs || !mask || !loss_out || !dls || !workspace) return ES_BAD_ARG;
  hipLaunchKernelGGL(focal_kernel, (nu + 255) / 256, 256, 0, stream, ls, ldl, probs, mask, nu, C, gamma, grad_scale,
                     dls, lddl, workspace);
  hipLaunchKernelGGL(row_mean_kernel, 1, 256, 0, stream, workspace, nu, loss_out, (float)nu);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
