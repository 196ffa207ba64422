// Fused multi-head self-attention forward / backward for one ViT block (gfx950).
//
// Replaces code/models/conformer.py:40-50 (timm 0.5.4 Attention):
//   qkv.reshape(B,N,3,H,hd).permute -> attn = softmax(q k^T * hd^-0.5) -> (attn @ v) -> [B,N,H*hd]
// One workgroup per (image, head): the whole head (N <= 256 tokens, hd = 64) lives in LDS, so the
// softmax is exact (no online rescale) and K/V are read from HBM once per head.
//
// Layout: qkv bf16 [tokens, 3*D] with per-token column order [3][H][64] (the reference reshape);
// o / dout bf16 [tokens, D] with column h*64+d; lse fp32 [image][head][token].
//
// MFMA orientation (v_mfma_f32_16x16x32_bf16, maps in common.h):
//   fwd / dQ : S^T = K . Q^T  -> lane owns one query, keys in registers ("query on the lane"),
//              so row max / sum are register reductions + 2 shuffles, and P^T is directly the
//              B operand of O^T = V^T . P^T and dS^T the B operand of dQ^T = K^T . dS^T.
//   dK / dV  : S = Q . K^T     -> lane owns one key; P and dS are the B operands of
//              dV^T = dO^T . P and dK^T = Q^T . dS.
// The "^T" A operands (V^T, K^T, dO^T, Q^T) are ds_read_b64_tr_b16 transposed reads of the
// row-major [token][64] LDS images.  LDS row = 128 B; chunk c of row r is stored at
// c ^ (((r >> 1) & 3) << 1), which is conflict-free for both the row reads (ds_read_b128) and the
// transposed reads used here.
#include "common.h"

namespace {

struct AttnArgs {
  const bf16* qkv; bf16* o; float* lse; float* delta;
  const bf16* dout; bf16* dqkv;
  int ldqkv, ldo, lddo, lddqkv;
  int T, H;
  float scale;
};

__device__ __forceinline__ int aswz(int r, int c) { return c ^ (((r >> 1) & 3) << 1); }

// [TP][64] bf16 tile of rows [0, T) of `src` (row stride ld), zero rows >= T.
__device__ __forceinline__ void load_head_tile(char* lds, const bf16* src, int ld, int T, int TP) {
  for (int id = threadIdx.x; id < TP * 8; id += blockDim.x) {
    const int r = id >> 3, c = id & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < T) v = *(const uint4*)(src + (size_t)r * ld + c * 8);
    *(uint4*)(lds + r * 128 + aswz(r, c) * 16) = v;
  }
}

__device__ __forceinline__ bf16x8 lds_row8(const char* lds, int row, int chunk) {
  return *(const bf16x8*)(lds + row * 128 + aswz(row, chunk) * 16);
}

// A operand X^T[row d0+t][k in {base+4g+q, base+16+4g+q}] from a [token][64] image:
// elements 0..3 = rows base+4g..+3, elements 4..7 = rows base+16+4g..+3, column d0 + t.
__device__ __forceinline__ bf16x8 lds_trT(const char* lds, int base, int d0, int g, int t) {
  const int q = t >> 2, p4 = t & 3;
  const int c = (d0 >> 3) + (p4 >> 1), off = (p4 & 1) * 8;
  const int r1 = base + 4 * g + q, r2 = r1 + 16;
  return cat8(lds_tr4(lds + r1 * 128 + aswz(r1, c) * 16 + off),
              lds_tr4(lds + r2 * 128 + aswz(r2, c) * 16 + off));
}

__device__ __forceinline__ bf16x8 ld_row8(const bf16* p, bool valid) {
  if (!valid) return bf16x8{};
  return *(const bf16x8*)p;
}

template <int NKC>  // 32-key chunks: T <= 32*NKC
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NKC * 32;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  load_head_tile(Ks, base + D + h * 64, a.ldqkv, T, TP);
  load_head_tile(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const float sl = a.scale * 1.44269504088896341f;
  for (int qb = w; qb < nqt; qb += 4) {
    const int q = qb * 16 + r;
    const bool qv = q < T;
    const bf16* qrow = base + (size_t)q * a.ldqkv + h * 64;
    const bf16x8 qf0 = ld_row8(qrow + 8 * g, qv), qf1 = ld_row8(qrow + 32 + 8 * g, qv);

    // scores in log2 units (scale * log2 e folded in): p = exp2(s - max) is one v_exp_f32; keys
    // are masked only in the partial last tile (the branch is uniform per tile).
    f32x4 s[2 * NKC];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2 * NKC; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = mfma16(lds_row8(Ks, t * 16 + r, g), qf0, acc);
      acc = mfma16(lds_row8(Ks, t * 16 + r, 4 + g), qf1, acc);
      acc *= sl;
      if (t * 16 + 16 > T) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (t * 16 + 4 * g + i >= T) acc[i] = -INFINITY;
      }
      mx = fmaxf(mx, fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])));
      s[t] = acc;
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 2 * NKC; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = __builtin_amdgcn_exp2f(s[t][i] - mx);
        s[t][i] = pv;
        l += pv;
      }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);

    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sc = 0; sc < NKC; ++sc) {
      bf16x8 pf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[i] = (bf16)s[2 * sc][i];
        pf[4 + i] = (bf16)s[2 * sc + 1][i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(lds_trT(Vs, sc * 32, dt * 16, g, r), pf, o[dt]);
    }
    if (qv) {
      const float inv = 1.0f / l;
      bf16* orow = a.o + (size_t)(img * T + q) * a.ldo + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 v = {(bf16)(o[dt][0] * inv), (bf16)(o[dt][1] * inv), (bf16)(o[dt][2] * inv), (bf16)(o[dt][3] * inv)};
        *(bf16x4*)(orow + dt * 16 + 4 * g) = v;
      }
      if (g == 0) a.lse[(size_t)bh * T + q] = (mx + __log2f(l)) * 0.69314718055994531f;  // natural log
    }
  }
}

// dQ: query on the lane; delta = rowsum(dO * O) computed in-register for the wave's queries.
template <int NKC>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NKC * 32;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  load_head_tile(Ks, base + D + h * 64, a.ldqkv, T, TP);
  load_head_tile(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  for (int qb = w; qb < nqt; qb += 4) {
    const int q = qb * 16 + r;
    const bool qv = q < T;
    const size_t tok = (size_t)img * T + q;
    const bf16* qrow = base + (size_t)q * a.ldqkv + h * 64;
    const bf16* dorow = a.dout + tok * a.lddo + h * 64;
    const bf16* orow = a.o + tok * a.ldo + h * 64;
    const bf16x8 qf0 = ld_row8(qrow + 8 * g, qv), qf1 = ld_row8(qrow + 32 + 8 * g, qv);
    const bf16x8 df0 = ld_row8(dorow + 8 * g, qv), df1 = ld_row8(dorow + 32 + 8 * g, qv);
    const bf16x8 of0 = ld_row8(orow + 8 * g, qv), of1 = ld_row8(orow + 32 + 8 * g, qv);
    float delta = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) delta += (float)df0[j] * (float)of0[j] + (float)df1[j] * (float)of1[j];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    if (qv && g == 0) a.delta[(size_t)bh * T + q] = delta;  // consumed by attn_bwd_dkv_kernel
    const float lq = qv ? a.lse[(size_t)bh * T + q] * 1.44269504088896341f : 0.f;  // log2 units
    const float sl = a.scale * 1.44269504088896341f;

    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int sc = 0; sc < NKC; ++sc) {
      bf16x8 dsf;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int t = 2 * sc + hf;
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        sv = mfma16(lds_row8(Ks, t * 16 + r, g), qf0, sv);
        sv = mfma16(lds_row8(Ks, t * 16 + r, 4 + g), qf1, sv);
        dp = mfma16(lds_row8(Vs, t * 16 + r, g), df0, dp);
        dp = mfma16(lds_row8(Vs, t * 16 + r, 4 + g), df1, dp);
        f32x4 pv;
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[i] = __builtin_amdgcn_exp2f(sv[i] * sl - lq);
        if (t * 16 + 16 > T) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (t * 16 + 4 * g + i >= T) pv[i] = 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) dsf[4 * hf + i] = (bf16)(pv[i] * (dp[i] - delta));
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(lds_trT(Ks, sc * 32, dt * 16, g, r), dsf, dq[dt]);
    }
    if (qv) {
      bf16* drow = a.dqkv + tok * a.lddqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 v = {(bf16)(dq[dt][0] * a.scale), (bf16)(dq[dt][1] * a.scale), (bf16)(dq[dt][2] * a.scale),
                    (bf16)(dq[dt][3] * a.scale)};
        *(bf16x4*)(drow + dt * 16 + 4 * g) = v;
      }
    }
  }
}

// dK, dV: key on the lane; Q and dO of the whole head in LDS with lse / delta per query.
template <int NKC>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NKC * 32;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Qs = smem;
  char* Ds = smem + TP * 128;
  float* lse_s = (float*)(smem + 2 * TP * 128);
  float* del_s = lse_s + TP;
  load_head_tile(Qs, base + h * 64, a.ldqkv, T, TP);
  load_head_tile(Ds, a.dout + (size_t)img * T * a.lddo + h * 64, a.lddo, T, TP);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  // lse in log2 units; padded queries get +inf so their probabilities are exactly 0
  for (int t = threadIdx.x; t < TP; t += blockDim.x)
    lse_s[t] = t < T ? a.lse[(size_t)bh * T + t] * 1.44269504088896341f : INFINITY;
  const float sl = a.scale * 1.44269504088896341f;
  for (int t = threadIdx.x; t < TP; t += blockDim.x) del_s[t] = t < T ? a.delta[(size_t)bh * T + t] : 0.f;
  __syncthreads();

  const int nkt = (T + 15) >> 4;
  for (int kb = w; kb < nkt; kb += 4) {
    const int key = kb * 16 + r;
    const bool kv = key < T;
    const bf16* krow = base + (size_t)key * a.ldqkv + D + h * 64;
    const bf16* vrow = krow + D;
    const bf16x8 kf0 = ld_row8(krow + 8 * g, kv), kf1 = ld_row8(krow + 32 + 8 * g, kv);
    const bf16x8 vf0 = ld_row8(vrow + 8 * g, kv), vf1 = ld_row8(vrow + 32 + 8 * g, kv);
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int sc = 0; sc < NKC; ++sc) {
      bf16x8 pf, dsf;
#pragma unroll
      for (int hf = 0; hf < 2; ++hf) {
        const int u = 2 * sc + hf;
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
        sv = mfma16(lds_row8(Qs, u * 16 + r, g), kf0, sv);
        sv = mfma16(lds_row8(Qs, u * 16 + r, 4 + g), kf1, sv);
        dp = mfma16(lds_row8(Ds, u * 16 + r, g), vf0, dp);
        dp = mfma16(lds_row8(Ds, u * 16 + r, 4 + g), vf1, dp);
        const f32x4 l4 = *(const f32x4*)(lse_s + u * 16 + 4 * g);
        const f32x4 d4 = *(const f32x4*)(del_s + u * 16 + 4 * g);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float pv = __builtin_amdgcn_exp2f(sv[i] * sl - l4[i]);
          pf[4 * hf + i] = (bf16)pv;
          dsf[4 * hf + i] = (bf16)(pv * (dp[i] - d4[i]));
        }
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(lds_trT(Ds, sc * 32, dt * 16, g, r), pf, dv[dt]);
        dk[dt] = mfma16(lds_trT(Qs, sc * 32, dt * 16, g, r), dsf, dk[dt]);
      }
    }
    if (kv) {
      bf16* drow = a.dqkv + ((size_t)img * T + key) * a.lddqkv + D + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        bf16x4 vk = {(bf16)(dk[dt][0] * a.scale), (bf16)(dk[dt][1] * a.scale), (bf16)(dk[dt][2] * a.scale),
                     (bf16)(dk[dt][3] * a.scale)};
        bf16x4 vv = {(bf16)dv[dt][0], (bf16)dv[dt][1], (bf16)dv[dt][2], (bf16)dv[dt][3]};
        *(bf16x4*)(drow + dt * 16 + 4 * g) = vk;
        *(bf16x4*)(drow + D + dt * 16 + 4 * g) = vv;
      }
    }
  }
}

#define ATTN_DISPATCH(KERNEL, NKC_, GRID, LDS, STREAM, ARGS)                         \
  switch (NKC_) {                                                                    \
    case 1: allow_lds(KERNEL<1>, LDS); hipLaunchKernelGGL(KERNEL<1>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 2: allow_lds(KERNEL<2>, LDS); hipLaunchKernelGGL(KERNEL<2>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 3: allow_lds(KERNEL<3>, LDS); hipLaunchKernelGGL(KERNEL<3>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 4: allow_lds(KERNEL<4>, LDS); hipLaunchKernelGGL(KERNEL<4>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 5: allow_lds(KERNEL<5>, LDS); hipLaunchKernelGGL(KERNEL<5>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 6: allow_lds(KERNEL<6>, LDS); hipLaunchKernelGGL(KERNEL<6>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 7: allow_lds(KERNEL<7>, LDS); hipLaunchKernelGGL(KERNEL<7>, GRID, 256, LDS, STREAM, ARGS); break;      \
    case 8: allow_lds(KERNEL<8>, LDS); hipLaunchKernelGGL(KERNEL<8>, GRID, 256, LDS, STREAM, ARGS); break;      \
    default: return ES_BAD_SHAPE;                                                    \
  }

}  // namespace

extern "C" {

// qkv [nimg*T, ldqkv] -> o [nimg*T, ldo], lse [nimg*H*T]; head dim 64, T <= 256.
int es_attn_fwd(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 256 || H <= 0 || ldqkv < 3 * H * 64 || ldo < H * 64 || (ldqkv % 8) || (ldo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse) return ES_BAD_ARG;
  AttnArgs a{(const bf16*)qkv, (bf16*)o, lse, nullptr, nullptr, nullptr, ldqkv, ldo, 0, 0, T, H, scale};
  const int nkc = (T + 31) / 32;
  const size_t lds = 2 * (size_t)nkc * 32 * 128;
  ATTN_DISPATCH(attn_fwd_kernel, nkc, nimg * H, lds, stream, a);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// dout [nimg*T, lddo] + forward (qkv, o, lse) -> dqkv [nimg*T, lddqkv] (q, k and v parts).
// delta: workspace [nimg*H*T] fp32 (rowsum(dO*O), written by the dQ pass, read by the dK/dV pass).
int es_attn_bwd(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, float* delta, const void* dout,
                int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 256 || H <= 0 || ldqkv < 3 * H * 64 || lddqkv < 3 * H * 64 || (ldqkv % 8) ||
      (lddqkv % 8) || (ldo % 8) || (lddo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse || !delta || !dout || !dqkv) return ES_BAD_ARG;
  AttnArgs a{(const bf16*)qkv, (bf16*)o, (float*)lse, delta, (const bf16*)dout, (bf16*)dqkv, ldqkv, ldo, lddo,
             lddqkv, T, H, scale};
  const int nkc = (T + 31) / 32;
  const size_t lds_dq = 2 * (size_t)nkc * 32 * 128;
  const size_t lds_dkv = lds_dq + 2 * (size_t)nkc * 32 * 4;
  ATTN_DISPATCH(attn_bwd_dq_kernel, nkc, nimg * H, lds_dq, stream, a);
  ATTN_DISPATCH(attn_bwd_dkv_kernel, nkc, nimg * H, lds_dkv, stream, a);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
