// Fused MLP forward for inference rows (gfx950): out = resid + fc2(gelu(fc1(h))), the [tokens, 4D]
// activation never written to HBM.
//
// Replaces Block.mlp (timm Mlp: fc1 -> GELU -> fc2, code/models/conformer.py:13-23) plus the
// residual add of Block.forward (:58-60) on the rows whose activations the backward does not need:
// the FixMatch weak forward (its logits are detached, code/loss.py:144) and evaluation.  The train
// forward keeps GELU'(pre) and the activation for the backward and runs the two GEMMs unfused.
//
// One workgroup = 4 waves = 128 tokens (32 per wave).  Per hidden chunk of 32 units:
//   fc1:  X = W1c . h^T      X [32 hidden x 32 tokens], v_mfma_f32_32x32x16_bf16, K = D
//   X = bf16(gelu(X + b1))   (the GELU epilogue of the unfused EPI_GELU_ACT GEMM)
//   fc2:  acc^T[n][tok] += W2[n][chunk] . X   -- the fc1 accumulator IS the fc2 B operand
//         (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"): registers
//         8s..8s+7 of X, packed to bf16, are k-step s of the B fragment; element j of lane half h
//         is X row 16s + 8(j>>2) + 4h + (j&3).  The fc1 A operand loads W1 row pi(row) with pi
//         swapping row bits 2 and 3, so that X row rho holds hidden unit pi(rho) and the fc2 A
//         fragment reads 8 CONSECUTIVE hidden units (one ds_read_b128): hidden 16s + 8h + j.
// Each wave keeps its 32 tokens' h rows (D bf16) as fc1 B fragments in registers for the whole
// launch; W1c / W2c chunks (2 x 32 x D bf16) are staged by LDS-DMA through a 3-deep ring shared by
// the 4 waves (counted vmcnt, raw s_barrier); b1 is copied to LDS once (a plain global load inside
// the glds pipeline would make hipcc drain it).  fp32 accumulation throughout; the output epilogue
// adds b2 and the fp32 residual in the fc2 GEMM's order ((acc + b2) + resid).
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr int HC = 32;   // hidden units per chunk
constexpr int NST = 3;   // ring depth
constexpr int TOKS = 128;

template <int D>
struct MlpGeo {
  static constexpr int W1B = HC * D * 2;          // W1 chunk [32][D] bf16
  static constexpr int W2B = D * HC * 2;          // W2 chunk [D][32] bf16
  static constexpr int STAGE = W1B + W2B;
  static constexpr int G1 = W1B / 1024 / 4;       // glds per wave for W1c
  static constexpr int G2 = W2B / 1024 / 4;       // glds per wave for W2c
  static constexpr int PER = G1 + G2;             // glds per wave per chunk
  static constexpr int KS = D / 16;               // fc1 k-steps
  static constexpr int NT = D / 32;               // fc2 output tiles
  static constexpr int ROWB = 2 * D;              // W1c row bytes
};

struct MlpArgs {
  const bf16* h; const bf16* w1; const float* b1; const bf16* w2; const float* b2;
  const float* resid; float* out;
  int M, Hd, ldh, ldr, ldo;
};

template <int D>
__global__ __launch_bounds__(256, 1) void mlp_fwd_kernel(MlpArgs p) {
  using G = MlpGeo<D>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* b1s = (float*)(smem + NST * G::STAGE);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int tok = blockIdx.x * TOKS + w * 32 + r;  // this lane's token (fc1 B column / fc2 output row)
  const int nch = p.Hd / HC;

  // h rows as fc1 B fragments: k-step ks, lane (r, h) holds h[tok][16 ks + 8 h + j]
  bf16x8 hf[G::KS];
#pragma unroll
  for (int ks = 0; ks < G::KS; ++ks) hf[ks] = *(const bf16x8*)(p.h + (size_t)tok * p.ldh + ks * 16 + 8 * h);
  for (int i = tid; i < p.Hd; i += 256) b1s[i] = p.b1[i];

  // Ring stage k (k = -1 .. nch-1) = { W1 chunk k+1, W2 chunk k } in slot (k+1) % NST: iteration c
  // runs fc1 of chunk c+1 beside the GELU of chunk c (independent: the VALU fills the MFMA gaps of a
  // single wave per SIMD) and then fc2 of chunk c, so it reads exactly one stage.  Stage -1 holds
  // W1 chunk 0 (and a dummy W2 chunk 0), the last stage a dummy W1 chunk 0: every stage is PER glds
  // per wave, so the counted waits are uniform.
  // W1c rows (contiguous in W1 [Hd][D]): 16-B chunk q of row rw at q ^ (rw & 15); W2c = chunk c of
  // the chunk-major W2 image [Hd/32][D][32] (contiguous 24 KiB: column slices of W2 [D][Hd] read
  // 64 B per row and ran the staging at ~18 GB/s per CU), 64-B rows, chunk q of row n at
  // q ^ ((n >> 2) & 3) (both conflict-free for the ds_read_b128 lane groups, MI355X_MICROARCH.md §LDS).
  auto issue = [&](int k) {
    char* S = smem + ((k + 1) % NST) * G::STAGE;
    const int c1 = k + 1 < nch ? k + 1 : 0, c2 = k >= 0 ? k : 0;
#pragma unroll
    for (int i = 0; i < G::G1; ++i) {
      const int ins = w * G::G1 + i;
      const int byte = ins * 1024 + lane * 16;
      const int rw = byte / G::ROWB, pq = (byte % G::ROWB) >> 4;
      glds16(p.w1 + (size_t)(c1 * HC + rw) * D + ((pq ^ (rw & 15)) << 3), S + ins * 1024);
    }
#pragma unroll
    for (int i = 0; i < G::G2; ++i) {
      const int ins = w * G::G2 + i;
      const int n = ins * 16 + (lane >> 2), pq = lane & 3;
      glds16(p.w2 + ((size_t)c2 * D + n) * HC + ((pq ^ ((n >> 2) & 3)) << 3), S + G::W1B + ins * 1024);
    }
  };

  f32x16 acc[G::NT];
#pragma unroll
  for (int t = 0; t < G::NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // fc1 A row for MFMA row r: W1c row pi(r) (bits 2 and 3 swapped)
  const int arow = (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1);
  // fc1 of one chunk from the W1 part of a slot; A fragments read 4 k-steps ahead of their MFMAs
  auto fc1 = [&](const char* W1c) {
    f32x16 X;
#pragma unroll
    for (int i = 0; i < 16; ++i) X[i] = 0.f;
    auto w1frag = [&](int ks) {
      return *(const bf16x8*)(W1c + arow * G::ROWB + (((2 * ks + h) ^ (arow & 15)) << 4));
    };
    bf16x8 fa[2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fa[0][j] = w1frag(j);
#pragma unroll
    for (int kb = 0; kb < G::KS / 4; ++kb) {
      if (kb + 1 < G::KS / 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) fa[(kb + 1) & 1][j] = w1frag(4 * (kb + 1) + j);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) X = mfma32(fa[kb & 1][j], hf[4 * kb + j], X);
    }
    return X;
  };

  issue(-1);
  issue(0);
  // h / b1 loads and stage -1 retired (stage 0 may stay in flight)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::PER) : "memory");
  __syncthreads();  // b1s (ds_write) + stage -1 visible to every wave
  f32x16 X = fc1(smem);
  if (nch > 1) issue(1);
  for (int c = 0; c < nch; ++c) {
    // stage c landed (stage c+1 may stay in flight); every wave is past iteration c-1, so the slot
    // of stage c-1 is free for stage c+2
    if (c + 1 < nch) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::PER) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (c + 2 < nch) issue(c + 2);
    const char* S = smem + ((c + 1) % NST) * G::STAGE;
    // ---- bias + GELU of chunk c -> bf16 B fragments (register 8s + j = hidden c*32 + 16s + 8h + j)
    bf16x8 xb[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const f32x4 bl = *(const f32x4*)(b1s + c * HC + 16 * s + 8 * h);
      const f32x4 bh = *(const f32x4*)(b1s + c * HC + 16 * s + 8 * h + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        xb[s][j] = (bf16)gelu_f(X[8 * s + j] + bl[j]);
        xb[s][4 + j] = (bf16)gelu_f(X[8 * s + 4 + j] + bh[j]);
      }
    }
    // ---- fc1 of chunk c+1 (independent of the GELU above)
    if (c + 1 < nch) X = fc1(S);
    // ---- fc2 of chunk c: acc[t]^T[n = 32t + ..][token] += W2[n][hidden] . act
    const char* W2c = S + G::W1B;
    auto w2frag = [&](int t, int s) {
      const int n = t * 32 + r;
      return *(const bf16x8*)(W2c + n * 64 + (((2 * s + h) ^ ((n >> 2) & 3)) << 4));
    };
    bf16x8 fb[2][2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[0][j][0] = w2frag(j, 0);
      fb[0][j][1] = w2frag(j, 1);
    }
#pragma unroll
    for (int tb = 0; tb < G::NT / 2; ++tb) {
      if (tb + 1 < G::NT / 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          fb[(tb + 1) & 1][j][0] = w2frag(2 * (tb + 1) + j, 0);
          fb[(tb + 1) & 1][j][1] = w2frag(2 * (tb + 1) + j, 1);
        }
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc[2 * tb + j] = mfma32(fb[tb & 1][j][s], xb[s], acc[2 * tb + j]);
    }
  }

  // ---- epilogue: out[tok][n] = (acc + b2[n]) + resid[tok][n]; register i of tile t holds
  // n = 32t + 8(i>>2) + 4h + (i&3): four consecutive columns per (t, i>>2)
  if (tok < p.M) {
    const float* rr = p.resid + (size_t)tok * p.ldr;
    float* orow = p.out + (size_t)tok * p.ldo;
#pragma unroll
    for (int t = 0; t < G::NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int n = t * 32 + 8 * q + 4 * h;
        const f32x4 bb = *(const f32x4*)(p.b2 + n);
        const f32x4 rv = *(const f32x4*)(rr + n);
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (acc[t][4 * q + j] + bb[j]) + rv[j];
        *(f32x4*)(orow + n) = o;
      }
  }
}

// dst [K/32][N][32] <- src [N][K] (bf16), one 16-B piece per thread
__global__ void pack_chunk32_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst, int N, int K) {
  const int total = N * (K >> 3);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int n = i / (K >> 3), k8 = i - n * (K >> 3);
    const int c = k8 >> 2, j = k8 & 3;
    *(bf16x8*)(dst + ((size_t)c * N + n) * 32 + j * 8) = *(const bf16x8*)(src + (size_t)n * K + k8 * 8);
  }
}

}  // namespace

extern "C" {

// dst [K/32, N, 32] = src [N, K] in 32-column chunks (the fc2 weight image es_mlp_fwd_infer reads);
// K % 32 == 0.
int es_pack_chunk32(const void* src, void* dst, int N, int K, hipStream_t stream) {
  if (N <= 0 || K <= 0 || K % 32) return ES_BAD_SHAPE;
  if (!src || !dst) return ES_BAD_ARG;
  const int total = N * (K / 8);
  int grid = (total + 255) / 256;
  grid = grid > 4096 ? 4096 : grid;
  hipLaunchKernelGGL(pack_chunk32_kernel, grid, 256, 0, stream, (const bf16*)src, (bf16*)dst, N, K);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}


// out [M, D] fp32 = resid + fc2(gelu(fc1(h))) for inference rows.  h [M', D] bf16 with
// M' = ceil(M / 128) * 128 readable rows (the engine's token buffers are padded to 256 rows);
// w1 [Hd, D] bf16 (the forward weight image), w2c [Hd/32, D, 32] bf16 = fc2.weight [D, Hd] in
// 32-column chunks (es_pack_chunk32), b1 [Hd], b2 [D] fp32; D in {128, 384},
// Hd % 32 == 0, Hd <= 4096.  out may not alias resid.
int es_mlp_fwd_infer(const void* h, int ldh, const void* w1, const float* b1, const void* w2, const float* b2,
                     const float* resid, int ldr, float* out, int ldo, int M, int D, int Hd, hipStream_t stream) {
  if (M <= 0 || Hd <= 0 || Hd % HC || Hd > 4096 || (ldh % 8) || (ldr % 4) || (ldo % 4) || ldh < D || ldr < D ||
      ldo < D)
    return ES_BAD_SHAPE;
  if (!h || !w1 || !b1 || !w2 || !b2 || !resid || !out || (const void*)resid == (const void*)out) return ES_BAD_ARG;
  MlpArgs a{(const bf16*)h, (const bf16*)w1, b1, (const bf16*)w2, b2, resid, out, M, Hd, ldh, ldr, ldo};
  const int grid = (M + TOKS - 1) / TOKS;
  switch (D) {
    case 384: {
      const size_t lds = NST * MlpGeo<384>::STAGE + (size_t)Hd * 4;
      allow_lds(mlp_fwd_kernel<384>, lds);
      hipLaunchKernelGGL(mlp_fwd_kernel<384>, grid, 256, lds, stream, a);
      break;
    }
    case 128: {
      const size_t lds = NST * MlpGeo<128>::STAGE + (size_t)Hd * 4;
      allow_lds(mlp_fwd_kernel<128>, lds);
      hipLaunchKernelGGL(mlp_fwd_kernel<128>, grid, 256, lds, stream, a);
      break;
    }
    default:
      return ES_BAD_SHAPE;
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
