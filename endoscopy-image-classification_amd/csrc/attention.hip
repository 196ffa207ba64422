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
// Head tiles are padded to NT16*16 rows (208 for T = 197: 26 KiB each; the forward stages Q, K and
// V, 78 KiB, two heads per CU; the backward kernels two tiles, three per CU) and staged by LDS-DMA
// (global_load_lds_dwordx4, 8 rows per wave-instruction); pad rows re-read token T-1, so they hold
// finite values whose probabilities are exactly zero.  Key (or query) chunks are 32 wide for the P.V-type products; an odd last
// 16-row tile uses the K=16 MFMA (v_mfma_f32_16x16x16_bf16), whose operand maps are the first
// half of the K=32 ones.
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
#include <type_traits>

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

// [TP][64] bf16 image of rows [0, TP) of `src` (row stride ld) by LDS-DMA: wave-instruction i moves
// rows 8i..8i+7 (lane -> row 8i + lane/8, physical chunk lane%8 holding logical chunk
// aswz(row, lane%8)); rows >= T re-read row T-1.  Caller waits (vmcnt) and barriers.
template <int NW = 4>  // waves of the workgroup
__device__ __forceinline__ void stage_head(char* lds, const bf16* src, int ld, int T, int TP) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = w; i < TP / 8; i += NW) {
    const int row = i * 8 + (lane >> 3);
    const int sr = row < T ? row : T - 1;
    glds16(src + (size_t)sr * ld + aswz(row, lane & 7) * 8, lds + i * 1024);
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

// first half of lds_trT: rows base+4g..+3 of column d0 + t (A operand of the K=16 MFMA)
__device__ __forceinline__ bf16x4 lds_trT4(const char* lds, int base, int d0, int g, int t) {
  const int q = t >> 2, p4 = t & 3;
  const int c = (d0 >> 3) + (p4 >> 1), off = (p4 & 1) * 8;
  const int r1 = base + 4 * g + q;
  return lds_tr4(lds + r1 * 128 + aswz(r1, c) * 16 + off);
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16k16(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a), __builtin_bit_cast(s16x4, b), c, 0,
                                                   0, 0);
}

__device__ __forceinline__ bf16x8 ld_row8(const bf16* p, bool valid) {
  if (!valid) return bf16x8{};
  return *(const bf16x8*)p;
}

// The left or right half of tile_rows_out's tile (acc[0..1]: columns dt*16 + 4g .. + 3 of 32): through 1 KiB
// of the wave's slot (64-B rows, 16-B chunk c of row i at c ^ ((i >> 1) & 3)) and out as one 16-B store per
// lane (64-B row segments).  Same values as tile_rows_out's.
__device__ __forceinline__ void half_rows_out(char* slot, const f32x4* acc, float s, bf16* dst, size_t ld, int nrows) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
    *(bf16x4*)(slot + r * 64 + (((2 * dt + (g >> 1)) ^ ((r >> 1) & 3)) * 16) + (g & 1) * 8) =
        bf16x4{(bf16)(acc[dt][0] * s), (bf16)(acc[dt][1] * s), (bf16)(acc[dt][2] * s), (bf16)(acc[dt][3] * s)};
  __builtin_amdgcn_wave_barrier();
  const int rr = lane >> 2, ch = lane & 3;
  const bf16x8 x = *(const bf16x8*)(slot + rr * 64 + ((ch ^ ((rr >> 1) & 3)) * 16));
  if (rr < nrows) *(bf16x8*)(dst + rr * ld + ch * 8) = x;
  __builtin_amdgcn_wave_barrier();
}

// A 16 x 64 output tile in the MFMA C layout (lane (g, r) holds row r, columns dt*16 + 4g .. +3 of acc[dt]),
// bf16(acc * s) out to rows dst + i * ld, i < nrows.  Direct stores would write 16 rows x 32 B per
// instruction (partial lines: the forward's WRITE_SIZE was 137 MB per F1 launch against 80 MB of o + lse),
// so the tile goes through `slot` (SLOT_ROWS x 128 B of LDS read and written only by this wave; 16-B chunk
// c of slot row i at c ^ (i & 7)) and out as 16-B lanes, each instruction writing whole 128-B row segments.
// SLOT_ROWS = 8 (1 KiB, where the LDS is full) moves the tile in two halves.
template <int SLOT_ROWS = 16>
__device__ __forceinline__ void tile_rows_out(char* slot, const f32x4* acc, float s, bf16* dst, size_t ld,
                                              int nrows) {
  const int lane = threadIdx.x & 63, g = lane >> 4, r = lane & 15;
  bf16x4 v[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
    v[dt] = bf16x4{(bf16)(acc[dt][0] * s), (bf16)(acc[dt][1] * s), (bf16)(acc[dt][2] * s), (bf16)(acc[dt][3] * s)};
#pragma unroll
  for (int p = 0; p < 16 / SLOT_ROWS; ++p) {
    const int sr = r - p * SLOT_ROWS;  // this lane's row in the slot
    if (SLOT_ROWS == 16 || (unsigned)sr < (unsigned)SLOT_ROWS) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
        *(bf16x4*)(slot + sr * 128 + ((2 * dt + (g >> 1)) ^ (sr & 7)) * 16 + (g & 1) * 8) = v[dt];
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int hf = 0; hf < SLOT_ROWS / 8; ++hf) {
      const int rr = hf * 8 + (lane >> 3), ch = lane & 7, row = p * SLOT_ROWS + rr;
      const bf16x8 x = *(const bf16x8*)(slot + rr * 128 + (ch ^ (rr & 7)) * 16);
      if (row < nrows) *(bf16x8*)(dst + row * ld + ch * 8) = x;
    }
    __builtin_amdgcn_wave_barrier();  // the slot is rewritten by the next half / the wave's next tile
  }
}

// NW waves per workgroup: 4, or 7 (13 query tiles of T = 197 over 7 waves: at most 2 each, where 4 waves
// take 4 / 3 / 3 / 3; two 7-wave workgroups per CU = 14 waves at <= 128 VGPRs)
template <int NT16, int OCC, int NW = 4>  // 16-key tiles: T <= 16*NT16; OCC workgroups per CU (register budget)
__global__ __launch_bounds__(NW * 64, OCC) void attn_fwd_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  char* Qs = smem + 2 * TP * 128;  // Q staged with K and V: one wait, no per-tile global latency
  stage_head<NW>(Ks, base + D + h * 64, a.ldqkv, T, TP);
  stage_head<NW>(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  stage_head<NW>(Qs, base + h * 64, a.ldqkv, T, TP);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const float sl = a.scale * 1.44269504088896341f;
  for (int qb = w; qb < nqt; qb += NW) {
    const int q = qb * 16 + r;
    const bool qv = q < T;
    const bf16x8 qf0 = lds_row8(Qs, q, g), qf1 = lds_row8(Qs, q, 4 + g);

    // scores in log2 units (scale * log2 e folded in): p = exp2(s - max) is one v_exp_f32; keys
    // are masked only in the last tile, the only one that can be partial (the launcher picks
    // NT16 = ceil(T / 16)): a compile-time choice -- a runtime test per tile made the compiler
    // precompute all 4 x NT16 key masks into SGPR pairs spilled to VGPR lanes.
    f32x4 s[NT16];
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < NT16; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = mfma16(lds_row8(Ks, t * 16 + r, g), qf0, acc);
      acc = mfma16(lds_row8(Ks, t * 16 + r, 4 + g), qf1, acc);
      acc *= sl;
      if (t == NT16 - 1) {
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
    for (int t = 0; t < NT16; ++t)
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
    for (int sc = 0; sc < NT16 / 2; ++sc) {
      bf16x8 pf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[i] = (bf16)s[2 * sc][i];
        pf[4 + i] = (bf16)s[2 * sc + 1][i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(lds_trT(Vs, sc * 32, dt * 16, g, r), pf, o[dt]);
    }
    if constexpr (NT16 & 1) {
      const bf16x4 pf = {(bf16)s[NT16 - 1][0], (bf16)s[NT16 - 1][1], (bf16)s[NT16 - 1][2], (bf16)s[NT16 - 1][3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16k16(lds_trT4(Vs, (NT16 - 1) * 16, dt * 16, g, r), pf, o[dt]);
    }
    // O through this query tile's own Q rows in LDS (read only by this wave, whose Q fragments are in
    // registers), whole-row stores
    tile_rows_out(Qs + (qb * 16) * 128, o, 1.0f / l, a.o + (size_t)(img * T + qb * 16) * a.ldo + h * 64, a.ldo,
                  T - qb * 16);
    if (qv && g == 0) a.lse[(size_t)bh * T + q] = (mx + __log2f(l)) * 0.69314718055994531f;  // natural log
  }
}

// ---- long sequences (256 < T <= 640: ViT/16 at 384^2, T = 577) ------------------------------------
// K and V of the head staged in LDS (2 x 74 KiB at T = 577; Q can no longer ride along), Q fragments
// straight from HBM, eight waves per workgroup.  The scores of a 16-query block are taken over key
// chunks of FCH 16-key tiles with an online softmax (running max / sum, the output rescaled when the
// max grows), so the registers hold FCH tiles instead of all NT16.  Rounding points as the short
// kernel: scores in log2 units, bf16(P) into P.V, fp32 accumulation; P is exp2(s - running max).
constexpr int FCH = 8;

// MASK: the chunk holds key rows >= T (only the last chunk(s) of the head).  Unmasked chunks are straight-line
// code, so the compiler issues all of the chunk's K fragment reads ahead of its MFMAs; a per-tile branch on the
// padding (round 4) split the chunk into blocks and exposed each tile's LDS and MFMA latency.
template <int NT, bool MASK>
__device__ __forceinline__ void fwd_long_chunk(const char* Ks, const char* Vs, int t0, int T, float sl, int g, int r,
                                               const bf16x8& qf0, const bf16x8& qf1, float& m, float& l, f32x4* o) {
  f32x4 s[NT];
  float cm = -INFINITY;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int kt = t0 + t;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    acc = mfma16(lds_row8(Ks, kt * 16 + r, g), qf0, acc);
    acc = mfma16(lds_row8(Ks, kt * 16 + r, 4 + g), qf1, acc);
    acc *= sl;
    if constexpr (MASK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = kt * 16 + 4 * g + i >= T ? -INFINITY : acc[i];
    }
    s[t] = acc;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) cm = fmaxf(cm, fmaxf(fmaxf(s[t][0], s[t][1]), fmaxf(s[t][2], s[t][3])));
  cm = fmaxf(cm, __shfl_xor(cm, 16, 64));
  cm = fmaxf(cm, __shfl_xor(cm, 32, 64));
  const float mn = fmaxf(m, cm);
  const float alpha = __builtin_amdgcn_exp2f(m - mn);  // 0 on the first chunk (m = -inf)
  l *= alpha;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
  m = mn;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pv = __builtin_amdgcn_exp2f(s[t][i] - mn);
      s[t][i] = pv;
      l += pv;
    }
#pragma unroll
  for (int sc = 0; sc < NT / 2; ++sc) {
    bf16x8 pf;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pf[i] = (bf16)s[2 * sc][i];
      pf[4 + i] = (bf16)s[2 * sc + 1][i];
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16(lds_trT(Vs, (t0 + 2 * sc) * 16, dt * 16, g, r), pf, o[dt]);
  }
  if constexpr (NT & 1) {
    const bf16x4 pf = {(bf16)s[NT - 1][0], (bf16)s[NT - 1][1], (bf16)s[NT - 1][2], (bf16)s[NT - 1][3]};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = mfma16k16(lds_trT4(Vs, (t0 + NT - 1) * 16, dt * 16, g, r), pf, o[dt]);
  }
}

template <int NT16>
__global__ __launch_bounds__(512) void attn_fwd_long_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  {  // stage K and V with all eight waves (stage_head assumes four)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = w; i < 2 * (TP / 8); i += 8) {
      const int which = i >= TP / 8, ii = which ? i - TP / 8 : i;
      const int row = ii * 8 + (lane >> 3);
      const int sr = row < T ? row : T - 1;
      glds16(base + (which ? 2 * D : D) + h * 64 + (size_t)sr * a.ldqkv + aswz(row, lane & 7) * 8,
             (which ? Vs : Ks) + ii * 1024);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const float sl = a.scale * 1.44269504088896341f;
  // the query block's Q fragments come from HBM one block ahead of their use (their latency hides behind the
  // current block's chunks)
  auto load_qf = [&](int qb, bf16x8& f0, bf16x8& f1) {
    const int q = qb * 16 + r;
    const bf16* qrow = base + (size_t)(q < T ? q : T - 1) * a.ldqkv + h * 64;
    f0 = *(const bf16x8*)(qrow + 8 * g);
    f1 = *(const bf16x8*)(qrow + 32 + 8 * g);
  };
  bf16x8 nq0, nq1;
  if (w < nqt) load_qf(w, nq0, nq1);
  for (int qb = w; qb < nqt; qb += 8) {
    const int q = qb * 16 + r;
    const bool qv = q < T;
    const bf16x8 qf0 = nq0, qf1 = nq1;
    if (qb + 8 < nqt) load_qf(qb + 8, nq0, nq1);
    float m = -INFINITY, l = 0.f;
    f32x4 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int c = 0; c < NT16 / FCH; ++c) {
      if ((c + 1) * FCH * 16 <= T) fwd_long_chunk<FCH, false>(Ks, Vs, c * FCH, T, sl, g, r, qf0, qf1, m, l, o);
      else fwd_long_chunk<FCH, true>(Ks, Vs, c * FCH, T, sl, g, r, qf0, qf1, m, l, o);
    }
    if constexpr (NT16 % FCH)
      fwd_long_chunk<NT16 % FCH, true>(Ks, Vs, NT16 - NT16 % FCH, T, sl, g, r, qf0, qf1, m, l, o);
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    // whole-row stores through the wave's 1-KiB slot past K and V (two halves: the LDS is full)
    tile_rows_out<8>(smem + 2 * TP * 128 + w * 1024, o, 1.0f / l, a.o + (size_t)(img * T + qb * 16) * a.ldo + h * 64,
                     a.ldo, T - qb * 16);
    if (qv && g == 0) a.lse[(size_t)bh * T + q] = (m + __log2f(l)) * 0.69314718055994531f;  // natural log
  }
}

// dQ: query on the lane; delta = rowsum(dO * O) computed in-register for the wave's queries.
template <int NT16>
__global__ __launch_bounds__(256, 3) void attn_bwd_dq_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  stage_head(Ks, base + D + h * 64, a.ldqkv, T, TP);
  stage_head(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const float sl = a.scale * 1.44269504088896341f;
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

    // dS^T tile t (keys 16t + 4g + i on this lane's query), in fp32
    auto ds_tile = [&](int t) {
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
      f32x4 ds;
#pragma unroll
      for (int i = 0; i < 4; ++i) ds[i] = pv[i] * (dp[i] - delta);
      return ds;
    };

    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int sc = 0; sc < NT16 / 2; ++sc) {
      const f32x4 d0 = ds_tile(2 * sc), d1 = ds_tile(2 * sc + 1);
      bf16x8 dsf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dsf[i] = (bf16)d0[i];
        dsf[4 + i] = (bf16)d1[i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(lds_trT(Ks, sc * 32, dt * 16, g, r), dsf, dq[dt]);
    }
    if constexpr (NT16 & 1) {
      const f32x4 d0 = ds_tile(NT16 - 1);
      const bf16x4 dsf = {(bf16)d0[0], (bf16)d0[1], (bf16)d0[2], (bf16)d0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16k16(lds_trT4(Ks, (NT16 - 1) * 16, dt * 16, g, r), dsf, dq[dt]);
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
template <int NT16, bool SELF_DELTA = false>
__global__ __launch_bounds__(256) void attn_bwd_dkv_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Qs = smem;
  char* Ds = smem + TP * 128;
  float* lse_s = (float*)(smem + 2 * TP * 128);
  float* del_s = lse_s + TP;
  stage_head(Qs, base + h * 64, a.ldqkv, T, TP);
  stage_head(Ds, a.dout + (size_t)img * T * a.lddo + h * 64, a.lddo, T, TP);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  // lse in log2 units; padded queries get +inf so their probabilities are exactly 0
  for (int t = threadIdx.x; t < TP; t += blockDim.x)
    lse_s[t] = t < T ? a.lse[(size_t)bh * T + t] * 1.44269504088896341f : INFINITY;
  if constexpr (!SELF_DELTA) {
    for (int t = threadIdx.x; t < TP; t += blockDim.x) del_s[t] = t < T ? a.delta[(size_t)bh * T + t] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    // delta = rowsum(dO * O) for every query of the head, here instead of in the dQ pass, so the
    // dQ and dK/dV passes are independent launches (they can run on two streams): dO from its LDS
    // image, O from HBM, 4 lanes per query
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t0 = 0; t0 < TP; t0 += 64) {
      const int tq = t0 + (threadIdx.x >> 2), part = threadIdx.x & 3;
      float dsum = 0.f;
      if (tq < T) {
        const bf16* orow = a.o + ((size_t)img * T + tq) * a.ldo + h * 64 + part * 16;
        const bf16x8 o0 = *(const bf16x8*)orow, o1 = *(const bf16x8*)(orow + 8);
        const bf16x8 d0 = lds_row8(Ds, tq, 2 * part), d1 = lds_row8(Ds, tq, 2 * part + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)d0[j] * (float)o0[j] + (float)d1[j] * (float)o1[j];
      }
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      if (part == 0 && tq < TP) del_s[tq] = tq < T ? dsum : 0.f;
    }
    __syncthreads();
  }
  const float sl = a.scale * 1.44269504088896341f;

  const int nkt = (T + 15) >> 4;
  for (int kb = w; kb < nkt; kb += 4) {
    const int key = kb * 16 + r;
    const bool kv = key < T;
    const bf16* krow = base + (size_t)key * a.ldqkv + D + h * 64;
    const bf16* vrow = krow + D;
    const bf16x8 kf0 = ld_row8(krow + 8 * g, kv), kf1 = ld_row8(krow + 32 + 8 * g, kv);
    const bf16x8 vf0 = ld_row8(vrow + 8 * g, kv), vf1 = ld_row8(vrow + 32 + 8 * g, kv);
    // P and dS for query tile u (queries 16u + 4g + i, this lane's key)
    auto p_ds = [&](int u, f32x4& p, f32x4& ds) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      sv = mfma16(lds_row8(Qs, u * 16 + r, g), kf0, sv);
      sv = mfma16(lds_row8(Qs, u * 16 + r, 4 + g), kf1, sv);
      dp = mfma16(lds_row8(Ds, u * 16 + r, g), vf0, dp);
      dp = mfma16(lds_row8(Ds, u * 16 + r, 4 + g), vf1, dp);
      const f32x4 l4 = *(const f32x4*)(lse_s + u * 16 + 4 * g);
      const f32x4 d4 = *(const f32x4*)(del_s + u * 16 + 4 * g);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[i] = __builtin_amdgcn_exp2f(sv[i] * sl - l4[i]);
        ds[i] = p[i] * (dp[i] - d4[i]);
      }
    };
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dk[dt] = dv[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int sc = 0; sc < NT16 / 2; ++sc) {
      f32x4 p0, p1, s0, s1;
      p_ds(2 * sc, p0, s0);
      p_ds(2 * sc + 1, p1, s1);
      bf16x8 pf, dsf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[i] = (bf16)p0[i];
        pf[4 + i] = (bf16)p1[i];
        dsf[i] = (bf16)s0[i];
        dsf[4 + i] = (bf16)s1[i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(lds_trT(Ds, sc * 32, dt * 16, g, r), pf, dv[dt]);
        dk[dt] = mfma16(lds_trT(Qs, sc * 32, dt * 16, g, r), dsf, dk[dt]);
      }
    }
    if constexpr (NT16 & 1) {
      f32x4 p0, s0;
      p_ds(NT16 - 1, p0, s0);
      const bf16x4 pf = {(bf16)p0[0], (bf16)p0[1], (bf16)p0[2], (bf16)p0[3]};
      const bf16x4 dsf = {(bf16)s0[0], (bf16)s0[1], (bf16)s0[2], (bf16)s0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16k16(lds_trT4(Ds, (NT16 - 1) * 16, dt * 16, g, r), pf, dv[dt]);
        dk[dt] = mfma16k16(lds_trT4(Qs, (NT16 - 1) * 16, dt * 16, g, r), dsf, dk[dt]);
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

// dK, dV with the query-pair loop software-pipelined: the LDS fragments of pair sc+1 (Q and dO rows
// for the S / dP products, lse / delta) and the transposed dO / Q fragments of pair sc are issued
// before pair sc's MFMAs and VALU, into separate registers, so every ds_read's latency hides behind
// the previous pair's work (the straight loop waited lgkmcnt(0) in front of each of its 16 MFMAs:
// one register set, each LDS round trip exposed).  Same operands, same MFMAs, same rounding points
// (bf16(P) into dV, bf16(dS) into dK) and the same fp32 accumulation order as attn_bwd_dkv_kernel.
struct DkvPair {
  bf16x8 qa0, qa1, da0, da1, qb0, qb1, db0, db1;  // rows of query tiles u = 2sc (a) and 2sc+1 (b)
  f32x4 la, dla, lb, dlb;                          // lse (log2 units) and delta of those queries
};

template <int NT16, bool SELF_DELTA = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkv_pipe_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  constexpr int NP = NT16 / 2;  // full query-tile pairs
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Qs = smem;
  char* Ds = smem + TP * 128;
  float* lse_s = (float*)(smem + 2 * TP * 128);
  float* del_s = lse_s + TP;
  stage_head(Qs, base + h * 64, a.ldqkv, T, TP);
  stage_head(Ds, a.dout + (size_t)img * T * a.lddo + h * 64, a.lddo, T, TP);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  for (int t = threadIdx.x; t < TP; t += blockDim.x)
    lse_s[t] = t < T ? a.lse[(size_t)bh * T + t] * 1.44269504088896341f : INFINITY;
  if constexpr (!SELF_DELTA) {
    for (int t = threadIdx.x; t < TP; t += blockDim.x) del_s[t] = t < T ? a.delta[(size_t)bh * T + t] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t0 = 0; t0 < TP; t0 += 64) {
      const int tq = t0 + (threadIdx.x >> 2), part = threadIdx.x & 3;
      float dsum = 0.f;
      if (tq < T) {
        const bf16* orow = a.o + ((size_t)img * T + tq) * a.ldo + h * 64 + part * 16;
        const bf16x8 o0 = *(const bf16x8*)orow, o1 = *(const bf16x8*)(orow + 8);
        const bf16x8 d0 = lds_row8(Ds, tq, 2 * part), d1 = lds_row8(Ds, tq, 2 * part + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)d0[j] * (float)o0[j] + (float)d1[j] * (float)o1[j];
      }
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      if (part == 0 && tq < TP) del_s[tq] = tq < T ? dsum : 0.f;
    }
    __syncthreads();
  }
  const float sl = a.scale * 1.44269504088896341f;

  auto load_pair = [&](int sc) {
    DkvPair o;
    const int ua = 2 * sc * 16 + r, ub = ua + 16;
    o.qa0 = lds_row8(Qs, ua, g); o.qa1 = lds_row8(Qs, ua, 4 + g);
    o.da0 = lds_row8(Ds, ua, g); o.da1 = lds_row8(Ds, ua, 4 + g);
    o.qb0 = lds_row8(Qs, ub, g); o.qb1 = lds_row8(Qs, ub, 4 + g);
    o.db0 = lds_row8(Ds, ub, g); o.db1 = lds_row8(Ds, ub, 4 + g);
    o.la = *(const f32x4*)(lse_s + 2 * sc * 16 + 4 * g);
    o.dla = *(const f32x4*)(del_s + 2 * sc * 16 + 4 * g);
    o.lb = *(const f32x4*)(lse_s + 2 * sc * 16 + 16 + 4 * g);
    o.dlb = *(const f32x4*)(del_s + 2 * sc * 16 + 16 + 4 * g);
    return o;
  };

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
    // P and dS of one query tile from its operands (query rows on the B side, this lane's key)
    auto p_ds = [&](bf16x8 q0, bf16x8 q1, bf16x8 d0, bf16x8 d1, f32x4 l4, f32x4 d4, f32x4& p, f32x4& ds) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      sv = mfma16(q0, kf0, sv);
      sv = mfma16(q1, kf1, sv);
      dp = mfma16(d0, vf0, dp);
      dp = mfma16(d1, vf1, dp);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[i] = __builtin_amdgcn_exp2f(sv[i] * sl - l4[i]);
        ds[i] = p[i] * (dp[i] - d4[i]);
      }
    };
    DkvPair cur = load_pair(0);
#pragma unroll 2
    for (int sc = 0; sc < NP; ++sc) {
      DkvPair nxt = cur;
      if (sc + 1 < NP) nxt = load_pair(sc + 1);
      // this pair's transposed dO / Q fragments (the A operands of dV^T / dK^T)
      bf16x8 tdo[4], tq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tdo[dt] = lds_trT(Ds, sc * 32, dt * 16, g, r);
        tq[dt] = lds_trT(Qs, sc * 32, dt * 16, g, r);
      }
      f32x4 p0, p1, s0, s1;
      p_ds(cur.qa0, cur.qa1, cur.da0, cur.da1, cur.la, cur.dla, p0, s0);
      p_ds(cur.qb0, cur.qb1, cur.db0, cur.db1, cur.lb, cur.dlb, p1, s1);
      bf16x8 pf, dsf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pf[i] = (bf16)p0[i];
        pf[4 + i] = (bf16)p1[i];
        dsf[i] = (bf16)s0[i];
        dsf[4 + i] = (bf16)s1[i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16(tdo[dt], pf, dv[dt]);
        dk[dt] = mfma16(tq[dt], dsf, dk[dt]);
      }
      cur = nxt;
    }
    if constexpr (NT16 & 1) {
      const int u = NT16 - 1;
      f32x4 p0, s0;
      p_ds(lds_row8(Qs, u * 16 + r, g), lds_row8(Qs, u * 16 + r, 4 + g), lds_row8(Ds, u * 16 + r, g),
           lds_row8(Ds, u * 16 + r, 4 + g), *(const f32x4*)(lse_s + u * 16 + 4 * g),
           *(const f32x4*)(del_s + u * 16 + 4 * g), p0, s0);
      const bf16x4 pf = {(bf16)p0[0], (bf16)p0[1], (bf16)p0[2], (bf16)p0[3]};
      const bf16x4 dsf = {(bf16)s0[0], (bf16)s0[1], (bf16)s0[2], (bf16)s0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma16k16(lds_trT4(Ds, u * 16, dt * 16, g, r), pf, dv[dt]);
        dk[dt] = mfma16k16(lds_trT4(Qs, u * 16, dt * 16, g, r), dsf, dk[dt]);
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

// dQ with the key-pair loop software-pipelined (as attn_bwd_dkv_pipe_kernel): pair sc+1's K / V row
// fragments and pair sc's transposed K fragments are in flight while pair sc's MFMAs and VALU run.
// Same operands, MFMAs, rounding points and fp32 accumulation order as attn_bwd_dq_kernel.
struct DqPair {
  bf16x8 ka0, ka1, va0, va1, kb0, kb1, vb0, vb1;  // rows of key tiles 2sc (a) and 2sc+1 (b)
};

template <int NT16>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_pipe_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  constexpr int NP = NT16 / 2;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  stage_head(Ks, base + D + h * 64, a.ldqkv, T, TP);
  stage_head(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const float sl = a.scale * 1.44269504088896341f;
  auto load_pair = [&](int sc) {
    DqPair o;
    const int ta = 2 * sc * 16 + r, tb = ta + 16;
    o.ka0 = lds_row8(Ks, ta, g); o.ka1 = lds_row8(Ks, ta, 4 + g);
    o.va0 = lds_row8(Vs, ta, g); o.va1 = lds_row8(Vs, ta, 4 + g);
    o.kb0 = lds_row8(Ks, tb, g); o.kb1 = lds_row8(Ks, tb, 4 + g);
    o.vb0 = lds_row8(Vs, tb, g); o.vb1 = lds_row8(Vs, tb, 4 + g);
    return o;
  };
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
    if (qv && g == 0) a.delta[(size_t)bh * T + q] = delta;  // consumed by the dK/dV pass
    const float lq = qv ? a.lse[(size_t)bh * T + q] * 1.44269504088896341f : 0.f;  // log2 units

    // dS^T tile t (keys 16t + 4g + i on this lane's query), in fp32
    auto ds_tile = [&](int t, bf16x8 k0, bf16x8 k1, bf16x8 v0, bf16x8 v1) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      sv = mfma16(k0, qf0, sv);
      sv = mfma16(k1, qf1, sv);
      dp = mfma16(v0, df0, dp);
      dp = mfma16(v1, df1, dp);
      f32x4 pv;
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = __builtin_amdgcn_exp2f(sv[i] * sl - lq);
      if (t * 16 + 16 > T) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (t * 16 + 4 * g + i >= T) pv[i] = 0.f;
      }
      f32x4 ds;
#pragma unroll
      for (int i = 0; i < 4; ++i) ds[i] = pv[i] * (dp[i] - delta);
      return ds;
    };

    f32x4 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    DqPair cur = load_pair(0);
#pragma unroll 2
    for (int sc = 0; sc < NP; ++sc) {
      DqPair nxt = cur;
      if (sc + 1 < NP) nxt = load_pair(sc + 1);
      bf16x8 tk[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) tk[dt] = lds_trT(Ks, sc * 32, dt * 16, g, r);
      const f32x4 d0 = ds_tile(2 * sc, cur.ka0, cur.ka1, cur.va0, cur.va1);
      const f32x4 d1 = ds_tile(2 * sc + 1, cur.kb0, cur.kb1, cur.vb0, cur.vb1);
      bf16x8 dsf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dsf[i] = (bf16)d0[i];
        dsf[4 + i] = (bf16)d1[i];
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16(tk[dt], dsf, dq[dt]);
      cur = nxt;
    }
    if constexpr (NT16 & 1) {
      const int t = NT16 - 1;
      const f32x4 d0 = ds_tile(t, lds_row8(Ks, t * 16 + r, g), lds_row8(Ks, t * 16 + r, 4 + g),
                               lds_row8(Vs, t * 16 + r, g), lds_row8(Vs, t * 16 + r, 4 + g));
      const bf16x4 dsf = {(bf16)d0[0], (bf16)d0[1], (bf16)d0[2], (bf16)d0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma16k16(lds_trT4(Ks, t * 16, dt * 16, g, r), dsf, dq[dt]);
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

// dK, dV with TWO key tiles per wave item (32 keys): every Q / dO row fragment, lse / delta vector and
// transposed dO / Q fragment read from LDS feeds both tiles' MFMAs, halving the LDS bytes per MFMA -- the
// one-tile form (attn_bwd_dkv_pipe_kernel) moves ~17 KiB through LDS per 16 MFMAs, more than the 256 B/clk
// a CU's LDS delivers beside two waves per SIMD of matrix work.  Items: key-tile pairs (2kp, 2kp+1); a
// second tile past the head (odd tile count) computes on zero K / V rows and stores nothing.  Per key
// tile the operands, MFMAs, rounding points and fp32 accumulation order are those of
// attn_bwd_dkv_kernel: bit-identical dK / dV.
template <int NT16, bool SELF_DELTA = false, int NW = 4>  // NW waves: 4, or 6 for the 37-tile heads
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_dkv2_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  constexpr int SLOT_ROWS = NT16 <= 16 ? 16 : 8;  // + NW x 2 KiB of LDS (1 KiB per wave at 37 tiles)
  constexpr int NP = NT16 / 2;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Qs = smem;
  char* Ds = smem + TP * 128;
  float* lse_s = (float*)(smem + 2 * TP * 128);
  float* del_s = lse_s + TP;
  stage_head<NW>(Qs, base + h * 64, a.ldqkv, T, TP);
  stage_head<NW>(Ds, a.dout + (size_t)img * T * a.lddo + h * 64, a.lddo, T, TP);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  for (int t = threadIdx.x; t < TP; t += blockDim.x)
    lse_s[t] = t < T ? a.lse[(size_t)bh * T + t] * 1.44269504088896341f : INFINITY;
  if constexpr (!SELF_DELTA) {
    for (int t = threadIdx.x; t < TP; t += blockDim.x) del_s[t] = t < T ? a.delta[(size_t)bh * T + t] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t0 = 0; t0 < TP; t0 += NW * 16) {
      const int tq = t0 + (threadIdx.x >> 2), part = threadIdx.x & 3;
      float dsum = 0.f;
      if (tq < T) {
        const bf16* orow = a.o + ((size_t)img * T + tq) * a.ldo + h * 64 + part * 16;
        const bf16x8 o0 = *(const bf16x8*)orow, o1 = *(const bf16x8*)(orow + 8);
        const bf16x8 d0 = lds_row8(Ds, tq, 2 * part), d1 = lds_row8(Ds, tq, 2 * part + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += (float)d0[j] * (float)o0[j] + (float)d1[j] * (float)o1[j];
      }
      dsum += __shfl_xor(dsum, 1, 64);
      dsum += __shfl_xor(dsum, 2, 64);
      if (part == 0 && tq < TP) del_s[tq] = tq < T ? dsum : 0.f;
    }
    __syncthreads();
  }
  const float sl = a.scale * 1.44269504088896341f;

  // P and dS of one query tile (operands q0, q1, d0, d1 = its Q / dO rows, l4 / d4 its lse / delta)
  // against one key tile (kf0, kf1, vf0, vf1)
  auto p_ds = [&](bf16x8 q0, bf16x8 q1, bf16x8 d0, bf16x8 d1, f32x4 l4, f32x4 d4, bf16x8 kf0, bf16x8 kf1,
                  bf16x8 vf0, bf16x8 vf1, f32x4& p, f32x4& ds) {
    f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
    sv = mfma16(q0, kf0, sv);
    sv = mfma16(q1, kf1, sv);
    dp = mfma16(d0, vf0, dp);
    dp = mfma16(d1, vf1, dp);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p[i] = __builtin_amdgcn_exp2f(sv[i] * sl - l4[i]);
      ds[i] = p[i] * (dp[i] - d4[i]);
    }
  };

  const int nkt = (T + 15) >> 4;
  const int nitems = (nkt + 1) >> 1;
  for (int kp = w; kp < nitems; kp += NW) {
    const int keyA = kp * 32 + r, keyB = keyA + 16;
    const bool kvA = keyA < T, kvB = keyB < T;
    const bf16* krA = base + (size_t)keyA * a.ldqkv + D + h * 64;
    const bf16* krB = base + (size_t)keyB * a.ldqkv + D + h * 64;
    const bf16x8 kA0 = ld_row8(krA + 8 * g, kvA), kA1 = ld_row8(krA + 32 + 8 * g, kvA);
    const bf16x8 vA0 = ld_row8(krA + D + 8 * g, kvA), vA1 = ld_row8(krA + D + 32 + 8 * g, kvA);
    const bf16x8 kB0 = ld_row8(krB + 8 * g, kvB), kB1 = ld_row8(krB + 32 + 8 * g, kvB);
    const bf16x8 vB0 = ld_row8(krB + D + 8 * g, kvB), vB1 = ld_row8(krB + D + 32 + 8 * g, kvB);
    f32x4 dkA[4], dvA[4], dkB[4], dvB[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dkA[dt] = dvA[dt] = dkB[dt] = dvB[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int sc = 0; sc < NP; ++sc) {
      const int ua = 2 * sc * 16 + r, ub = ua + 16;
      const bf16x8 qa0 = lds_row8(Qs, ua, g), qa1 = lds_row8(Qs, ua, 4 + g);
      const bf16x8 da0 = lds_row8(Ds, ua, g), da1 = lds_row8(Ds, ua, 4 + g);
      const bf16x8 qb0 = lds_row8(Qs, ub, g), qb1 = lds_row8(Qs, ub, 4 + g);
      const bf16x8 db0 = lds_row8(Ds, ub, g), db1 = lds_row8(Ds, ub, 4 + g);
      const f32x4 la = *(const f32x4*)(lse_s + 2 * sc * 16 + 4 * g);
      const f32x4 dla = *(const f32x4*)(del_s + 2 * sc * 16 + 4 * g);
      const f32x4 lb = *(const f32x4*)(lse_s + 2 * sc * 16 + 16 + 4 * g);
      const f32x4 dlb = *(const f32x4*)(del_s + 2 * sc * 16 + 16 + 4 * g);
      bf16x8 tdo[4], tq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tdo[dt] = lds_trT(Ds, sc * 32, dt * 16, g, r);
        tq[dt] = lds_trT(Qs, sc * 32, dt * 16, g, r);
      }
      {  // key tile A
        f32x4 p0, p1, s0, s1;
        p_ds(qa0, qa1, da0, da1, la, dla, kA0, kA1, vA0, vA1, p0, s0);
        p_ds(qb0, qb1, db0, db1, lb, dlb, kA0, kA1, vA0, vA1, p1, s1);
        bf16x8 pf, dsf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pf[i] = (bf16)p0[i];
          pf[4 + i] = (bf16)p1[i];
          dsf[i] = (bf16)s0[i];
          dsf[4 + i] = (bf16)s1[i];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dvA[dt] = mfma16(tdo[dt], pf, dvA[dt]);
          dkA[dt] = mfma16(tq[dt], dsf, dkA[dt]);
        }
      }
      {  // key tile B
        f32x4 p0, p1, s0, s1;
        p_ds(qa0, qa1, da0, da1, la, dla, kB0, kB1, vB0, vB1, p0, s0);
        p_ds(qb0, qb1, db0, db1, lb, dlb, kB0, kB1, vB0, vB1, p1, s1);
        bf16x8 pf, dsf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pf[i] = (bf16)p0[i];
          pf[4 + i] = (bf16)p1[i];
          dsf[i] = (bf16)s0[i];
          dsf[4 + i] = (bf16)s1[i];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dvB[dt] = mfma16(tdo[dt], pf, dvB[dt]);
          dkB[dt] = mfma16(tq[dt], dsf, dkB[dt]);
        }
      }
    }
    if constexpr (NT16 & 1) {
      const int u = NT16 - 1;
      const bf16x8 q0 = lds_row8(Qs, u * 16 + r, g), q1 = lds_row8(Qs, u * 16 + r, 4 + g);
      const bf16x8 d0 = lds_row8(Ds, u * 16 + r, g), d1 = lds_row8(Ds, u * 16 + r, 4 + g);
      const f32x4 l4 = *(const f32x4*)(lse_s + u * 16 + 4 * g), d4 = *(const f32x4*)(del_s + u * 16 + 4 * g);
      bf16x4 tdo4[4], tq4[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tdo4[dt] = lds_trT4(Ds, u * 16, dt * 16, g, r);
        tq4[dt] = lds_trT4(Qs, u * 16, dt * 16, g, r);
      }
      f32x4 p0, s0;
      p_ds(q0, q1, d0, d1, l4, d4, kA0, kA1, vA0, vA1, p0, s0);
      bf16x4 pf = {(bf16)p0[0], (bf16)p0[1], (bf16)p0[2], (bf16)p0[3]};
      bf16x4 dsf = {(bf16)s0[0], (bf16)s0[1], (bf16)s0[2], (bf16)s0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dvA[dt] = mfma16k16(tdo4[dt], pf, dvA[dt]);
        dkA[dt] = mfma16k16(tq4[dt], dsf, dkA[dt]);
      }
      p_ds(q0, q1, d0, d1, l4, d4, kB0, kB1, vB0, vB1, p0, s0);
      pf = bf16x4{(bf16)p0[0], (bf16)p0[1], (bf16)p0[2], (bf16)p0[3]};
      dsf = bf16x4{(bf16)s0[0], (bf16)s0[1], (bf16)s0[2], (bf16)s0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dvB[dt] = mfma16k16(tdo4[dt], pf, dvB[dt]);
        dkB[dt] = mfma16k16(tq4[dt], dsf, dkB[dt]);
      }
    }
    {  // whole-row stores through the wave's LDS slot (dV: bf16(x * 1) = bf16(x))
      char* slot = smem + 2 * TP * 128 + 2 * TP * 4 + w * (SLOT_ROWS * 128);
      bf16* d0 = a.dqkv + ((size_t)img * T + kp * 32) * a.lddqkv + D + h * 64;
      tile_rows_out<SLOT_ROWS>(slot, dkA, a.scale, d0, a.lddqkv, T - kp * 32);
      tile_rows_out<SLOT_ROWS>(slot, dvA, 1.0f, d0 + D, a.lddqkv, T - kp * 32);
      tile_rows_out<SLOT_ROWS>(slot, dkB, a.scale, d0 + 16 * (size_t)a.lddqkv, a.lddqkv, T - kp * 32 - 16);
      tile_rows_out<SLOT_ROWS>(slot, dvB, 1.0f, d0 + 16 * (size_t)a.lddqkv + D, a.lddqkv, T - kp * 32 - 16);
    }
  }
}

// dQ with TWO query tiles per wave item (32 queries): the K / V row fragments and transposed K fragments
// read from LDS for a key pair feed both query tiles' MFMAs (half the LDS bytes per MFMA of
// attn_bwd_dq_kernel).  A second tile past the head (odd tile count) runs on zero rows and stores nothing.
// Per query tile: the operands, MFMAs, rounding points and fp32 order of attn_bwd_dq_kernel (bit-identical).
template <int NT16, int NW = 4>  // NW waves: 4, or 8 for the 37-tile heads (1-KiB output slots there)
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_bwd_dq2_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16;
  constexpr int NP = NT16 / 2;
  const int bh = blockIdx.x, img = bh / a.H, h = bh - img * a.H;
  const int D = a.H * 64, T = a.T;
  const bf16* base = a.qkv + (size_t)img * T * a.ldqkv;
  char* Ks = smem;
  char* Vs = smem + TP * 128;
  stage_head<NW>(Ks, base + D + h * 64, a.ldqkv, T, TP);
  stage_head<NW>(Vs, base + 2 * D + h * 64, a.ldqkv, T, TP);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, r = lane & 15;
  const int nqt = (T + 15) >> 4;
  const int nitems = (nqt + 1) >> 1;
  const float sl = a.scale * 1.44269504088896341f;
  struct QOps {
    bf16x8 qf0, qf1, df0, df1;
    float delta, lq;
    int q;
    bool qv;
  };
  // a query tile's rows from HBM (issued one wave item ahead of their use: their latency hides behind the
  // current item's MFMAs), then finished -- delta = rowsum(dO * O) -- when the item starts
  struct QRaw {
    bf16x8 qf0, qf1, df0, df1, of0, of1;
    float lse;
    int q;
    bool qv;
  };
  auto load_raw = [&](int qb) {
    QRaw o;
    o.q = qb * 16 + r;
    o.qv = o.q < T;
    const size_t tok = (size_t)img * T + o.q;
    const bf16* qrow = base + (size_t)o.q * a.ldqkv + h * 64;
    const bf16* dorow = a.dout + tok * a.lddo + h * 64;
    const bf16* orow = a.o + tok * a.ldo + h * 64;
    o.qf0 = ld_row8(qrow + 8 * g, o.qv);
    o.qf1 = ld_row8(qrow + 32 + 8 * g, o.qv);
    o.df0 = ld_row8(dorow + 8 * g, o.qv);
    o.df1 = ld_row8(dorow + 32 + 8 * g, o.qv);
    o.of0 = ld_row8(orow + 8 * g, o.qv);
    o.of1 = ld_row8(orow + 32 + 8 * g, o.qv);
    o.lse = o.qv ? a.lse[(size_t)bh * T + o.q] : 0.f;
    return o;
  };
  auto finish_q = [&](const QRaw& x) {
    QOps o;
    o.q = x.q;
    o.qv = x.qv;
    o.qf0 = x.qf0;
    o.qf1 = x.qf1;
    o.df0 = x.df0;
    o.df1 = x.df1;
    float delta = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) delta += (float)x.df0[j] * (float)x.of0[j] + (float)x.df1[j] * (float)x.of1[j];
    delta += __shfl_xor(delta, 16, 64);
    delta += __shfl_xor(delta, 32, 64);
    o.delta = delta;
    if (o.qv && g == 0) a.delta[(size_t)bh * T + o.q] = delta;  // consumed by the dK/dV pass
    o.lq = o.qv ? x.lse * 1.44269504088896341f : 0.f;            // log2 units
    return o;
  };
  // dS^T tile t (keys 16t + 4g + i on this lane's query) from the key tile's K / V rows.  maskc: whether the
  // tile may hold key rows >= T (std::true_type only for the head's last tile / pair: the other pairs are
  // straight-line code, so their LDS reads and MFMAs interleave -- a per-tile branch split them into blocks)
  auto ds_tile = [&](auto maskc, const QOps& Q, int t, bf16x8 k0, bf16x8 k1, bf16x8 v0, bf16x8 v1) {
    f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
    sv = mfma16(k0, Q.qf0, sv);
    sv = mfma16(k1, Q.qf1, sv);
    dp = mfma16(v0, Q.df0, dp);
    dp = mfma16(v1, Q.df1, dp);
    f32x4 pv;
#pragma unroll
    for (int i = 0; i < 4; ++i) pv[i] = __builtin_amdgcn_exp2f(sv[i] * sl - Q.lq);
    if constexpr (decltype(maskc)::value) {
#pragma unroll
      for (int i = 0; i < 4; ++i) pv[i] = t * 16 + 4 * g + i >= T ? 0.f : pv[i];
    }
    f32x4 ds;
#pragma unroll
    for (int i = 0; i < 4; ++i) ds[i] = pv[i] * (dp[i] - Q.delta);
    return ds;
  };
  auto store = [&](const QOps& Q, const f32x4* dq) {  // whole-row stores through the wave's 2-KiB LDS slot
    const int q0 = Q.q - r;
    constexpr int SR = NW == 4 ? 16 : 8;  // slot rows: 2 KiB per wave, 1 KiB with eight waves
    tile_rows_out<SR>(smem + 2 * TP * 128 + w * SR * 128, dq, a.scale,
                      a.dqkv + ((size_t)img * T + q0) * a.lddqkv + h * 64, a.lddqkv, T - q0);
  };

  QRaw rA = load_raw(2 * w), rB = load_raw(2 * w + 1);
  for (int it = w; it < nitems; it += NW) {
    const QOps QA = finish_q(rA), QB = finish_q(rB);
    if (it + NW < nitems) {
      rA = load_raw(2 * (it + NW));
      rB = load_raw(2 * (it + NW) + 1);
    }
    f32x4 dqA[4], dqB[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dqA[dt] = dqB[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto pair = [&](auto maskc, int sc) {
      const int ta = 2 * sc * 16 + r, tb = ta + 16;
      const bf16x8 ka0 = lds_row8(Ks, ta, g), ka1 = lds_row8(Ks, ta, 4 + g);
      const bf16x8 va0 = lds_row8(Vs, ta, g), va1 = lds_row8(Vs, ta, 4 + g);
      const bf16x8 kb0 = lds_row8(Ks, tb, g), kb1 = lds_row8(Ks, tb, 4 + g);
      const bf16x8 vb0 = lds_row8(Vs, tb, g), vb1 = lds_row8(Vs, tb, 4 + g);
      bf16x8 tk[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) tk[dt] = lds_trT(Ks, sc * 32, dt * 16, g, r);
      {
        const f32x4 d0 = ds_tile(maskc, QA, 2 * sc, ka0, ka1, va0, va1);
        const f32x4 d1 = ds_tile(maskc, QA, 2 * sc + 1, kb0, kb1, vb0, vb1);
        bf16x8 dsf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dsf[i] = (bf16)d0[i];
          dsf[4 + i] = (bf16)d1[i];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dqA[dt] = mfma16(tk[dt], dsf, dqA[dt]);
      }
      {
        const f32x4 d0 = ds_tile(maskc, QB, 2 * sc, ka0, ka1, va0, va1);
        const f32x4 d1 = ds_tile(maskc, QB, 2 * sc + 1, kb0, kb1, vb0, vb1);
        bf16x8 dsf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          dsf[i] = (bf16)d0[i];
          dsf[4 + i] = (bf16)d1[i];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dqB[dt] = mfma16(tk[dt], dsf, dqB[dt]);
      }
    };
#pragma unroll 1
    for (int sc = 0; sc < NP; ++sc) {
      if ((2 * sc + 2) * 16 <= T) pair(std::false_type{}, sc);
      else pair(std::true_type{}, sc);
    }
    if constexpr (NT16 & 1) {
      const int t = NT16 - 1;
      const bf16x8 k0 = lds_row8(Ks, t * 16 + r, g), k1 = lds_row8(Ks, t * 16 + r, 4 + g);
      const bf16x8 v0 = lds_row8(Vs, t * 16 + r, g), v1 = lds_row8(Vs, t * 16 + r, 4 + g);
      bf16x4 tk4[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) tk4[dt] = lds_trT4(Ks, t * 16, dt * 16, g, r);
      f32x4 d0 = ds_tile(std::true_type{}, QA, t, k0, k1, v0, v1);
      bf16x4 dsf = {(bf16)d0[0], (bf16)d0[1], (bf16)d0[2], (bf16)d0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dqA[dt] = mfma16k16(tk4[dt], dsf, dqA[dt]);
      d0 = ds_tile(std::true_type{}, QB, t, k0, k1, v0, v1);
      dsf = bf16x4{(bf16)d0[0], (bf16)d0[1], (bf16)d0[2], (bf16)d0[3]};
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dqB[dt] = mfma16k16(tk4[dt], dsf, dqB[dt]);
    }
    store(QA, dqA);
    store(QB, dqB);
  }
}

// ---- single-pass backward (T in (192, 208]: 13 tiles) ------------------------------------------------
// One persistent workgroup per CU (eight waves, 148 KiB of LDS), heads bh = blockIdx.x, + gridDim.x, ...
// HBM is touched once per operand: Q, dO and K of a head by LDS-DMA, O and lse into registers (delta, the
// log2 lse), the K / V rows of phase 1 into registers, and dQ, dK, dV written once -- where the two-pass
// form (attn_bwd_dq2_kernel + attn_bwd_dkv2_kernel) read Q, K, V, dO twice and wrote / re-read delta.
// A head runs in two rounds over its queries (tiles 0..7, then 8..12):
//   phase 1, key on the lane (wave w < 7 owns key tiles 2w, 2w + 1 and their K / V rows): S, P, dP and dS of
//     the round's query pairs exactly as attn_bwd_dkv2_kernel, dV / dK accumulated in registers, and
//     bf16(dS) written to LDS as [key][query] images (64 queries per 128-B row; within a 32-query segment
//     column 8g + i holds query 4g + i of the first tile (i < 4) and 16 + 4g + i - 4 of the second, so the
//     lane's packed dK operand goes out as one 16-B store; 8-B pieces swizzled by sws);
//   phase 2, query on the lane (one query tile per wave): dQ^T = K^T . dS^T from the K image and the dS
//     images (both transposed reads), attn_bwd_dq2_kernel's MFMAs without recomputing S and dP.
// dK / dV are stored after the second round's phase 1.  The next head's Q / dO rows are DMA'd into the rows
// a round's phase 1 has finished with, its K after the last phase 2, and its O / lse / K / V fragments are
// loaded into registers during the last phase 2: only the first head's loads are exposed.  The DMAs are
// inline asm (hipcc would otherwise drain them in front of every transposed read) retired by counted waits;
// the barriers wait for LDS only, so a prefetch stays in flight across them.
// Rounding points and fp32 accumulation orders are attn_bwd_dq2_kernel's (delta, dQ) and
// attn_bwd_dkv2_kernel's (dK, dV): phase 1's S and dP are the transposed MFMA products of dq2's, the same
// fp32 dot products.

// dS image row k: logical 8-B piece p (= 2 x chunk + half) at piece p ^ sws(k).  Conflict-free both for the
// transposed reads (a 32-lane group: rows k0..k0+7, four chunks, one half) and for the 16-B row stores (8 lanes:
// rows k0..k0+7, one chunk): bits 1-3 of sws are a bijection of k & 7, and bits 0 and 3 differ over the four
// rows of one parity.
__device__ __forceinline__ int sws(int k) { return ((k & 4) << 1) | ((k & 1) << 2) | (((k >> 1) & 1) * 3); }

// dS^T fragment (B operand of dQ^T = K^T . dS^T) of query tile `half` of a 32-query segment of a dS image:
// elements 0..3 = keys base + 4g .. + 3, elements 4..7 = keys base + 16 + 4g .. + 3 (lds_trT's k order)
__device__ __forceinline__ bf16x8 lds_trS(const char* img, int base, int seg, int half, int g, int t) {
  const int p = 2 * (seg * 4 + (t & 3)) + half;
  const int r1 = base + 4 * g + (t >> 2), r2 = r1 + 16;
  return cat8(lds_tr4(img + r1 * 128 + (p ^ sws(r1)) * 8), lds_tr4(img + r2 * 128 + (p ^ sws(r2)) * 8));
}
__device__ __forceinline__ bf16x4 lds_trS4(const char* img, int base, int seg, int half, int g, int t) {
  const int p = 2 * (seg * 4 + (t & 3)) + half;
  const int r1 = base + 4 * g + (t >> 2);
  return lds_tr4(img + r1 * 128 + (p ^ sws(r1)) * 8);
}

// LDS byte address of a pointer into LDS (a non-template function: see glds16)
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// bl16_asm with the LDS destination already a wave-uniform 32-bit LDS address (no generic pointer formed)
__device__ __forceinline__ void bl16_m0(i32x4 rsrc, unsigned voff, unsigned soff, unsigned lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(lds_byte), "s"(soff)
               : "memory");
}

// LDS writes visible to the workgroup; VMEM (DMA, stores) left in flight
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NT16>
__global__ __launch_bounds__(512) void attn_bwd_fused_kernel(AttnArgs a, int nbh) {
  static_assert(NT16 == 13, "rounds of 8 + 5 query tiles, 7 key-tile pairs over 8 waves");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TP = NT16 * 16, IMG = TP * 128, NP = NT16 / 2, PA = 4, NG = TP / 8;
  char* Qs = smem;
  char* Ds = smem + IMG;
  char* Ks = smem + 2 * IMG;
  char* Ss = smem + 3 * IMG;  // two dS images
  float* lse_s = (float*)(smem + 5 * IMG);
  float* del_s = lse_s + TP;
  // the wave index in a scalar register: wave-uniform branches and loop trips stay scalar
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  char* slot = (char*)(del_s + TP) + w * 2048;
  const unsigned lds0 = lds_addr(smem);  // LDS byte address of the dynamic allocation
  const int D = a.H * 64, T = a.T;
  const float sl = a.scale * 1.44269504088896341f;
  // the lane index as an opaque value: each phase derives its LDS addresses from a fresh copy, so hipcc
  // cannot hoist them all out of the head loop (two dozen loop-invariant addresses live across every phase
  // were spilled to scratch, and every reload's vmcnt wait drained the prefetch DMAs)
  auto fresh_lane = [&]() {
    int l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
  };

  // whole-tensor buffer resources (the launcher keeps every tensor under 2 GiB): per-head offsets are 32-bit
  // scalars, so no 64-bit head pointer is ever formed in (and spilled from) vector registers
  const int nrows = nbh / a.H * T;
  const i32x4 sQKV = rsrc_i4(a.qkv, (unsigned)nrows * a.ldqkv * 2u);
  const i32x4 sDO = rsrc_i4(a.dout, (unsigned)nrows * a.lddo * 2u);
  const auto bQKV = buf_rsrc(a.qkv, (unsigned)nrows * a.ldqkv * 2u);
  const auto bO = buf_rsrc(a.o, (unsigned)nrows * a.ldo * 2u);
  const auto bLSE = buf_rsrc(a.lse, (unsigned)nbh * T * 4u);

  // 8-row groups [i0, i1) of a head image (rows >= T re-read row T - 1; colb: the head's byte column, ldb: the
  // row pitch in bytes, base: the image's first byte), by waves w0 .. w0 + nw - 1: this wave's share groups
  // i0 + w - w0, + nw, ..
  auto stage = [&](const char* lds, i32x4 rs, unsigned base, unsigned colb, unsigned ldb, int i0, int i1, int w0,
                   int nw) {
    const int l = fresh_lane();
    const unsigned dst = lds0 + (unsigned)(lds - smem);
    for (int i = i0 + w - w0; w >= w0 && w < w0 + nw && i < i1; i += nw) {
      const int row = i * 8 + (l >> 3);
      const int sr = row < T ? row : T - 1;
      bl16_m0(rs, (unsigned)sr * ldb + colb + aswz(row, l & 7) * 16, base, dst + i * 1024);
    }
  };
  auto stage_qdo = [&](int bh, int i0, int i1, int w0, int nw) {
    const int img = bh / a.H, h = bh - img * a.H;
    stage(Qs, sQKV, (unsigned)img * T * a.ldqkv * 2u, h * 128, a.ldqkv * 2, i0, i1, w0, nw);
    stage(Ds, sDO, (unsigned)img * T * a.lddo * 2u, h * 128, a.lddo * 2, i0, i1, w0, nw);
  };
  auto stage_k = [&](int bh) {
    const int img = bh / a.H, h = bh - img * a.H;
    stage(Ks, sQKV, (unsigned)img * T * a.ldqkv * 2u, (D + h * 64) * 2, a.ldqkv * 2, 0, NG, 0, 8);
  };

  // register operands of a head: O rows of the wave's delta tiles (w, w + 8), V rows of its key tiles
  // (2w, 2w + 1; the K rows come from the K image), the lse of query threadIdx.x -- buffer loads, rows past
  // T read as zero
  struct Pre {
    bf16x8 o[2][2];
    bf16x8 v[4];
    float lse;
  };
  auto prefetch = [&](int bh) {
    Pre p;
    const int l = fresh_lane(), g = l >> 4, r = l & 15;
    const int img = bh / a.H, h = bh - img * a.H;
    // in order of use (lse and O by the deltas, V by phase 1)
    const int tq = l + 64 * w;
    p.lse = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                          bLSE, tq < T ? (unsigned)(bh * T + tq) * 4u : ES_OOB, 0, 0));
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = (w + 8 * j) * 16 + r;
      const unsigned off = q < T ? (unsigned)((img * T + q) * a.ldo + h * 64 + 8 * g) * 2u : ES_OOB;
      p.o[j][0] = __builtin_bit_cast(bf16x8, buf_load16(bO, off));
      p.o[j][1] = __builtin_bit_cast(bf16x8, buf_load16(bO, off + 64));
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = w * 32 + 16 * t + r;
      const unsigned off = key < T ? (unsigned)((img * T + key) * a.ldqkv + 2 * D + h * 64 + 8 * g) * 2u : ES_OOB;
      p.v[2 * t + 0] = __builtin_bit_cast(bf16x8, buf_load16(bQKV, off));
      p.v[2 * t + 1] = __builtin_bit_cast(bf16x8, buf_load16(bQKV, off + 64));
    }
    return p;
  };
  // delta = rowsum(dO * O) with attn_bwd_dq2_kernel's lane split and order; lse in log2 units
  auto deltas = [&](const Pre& p) {
    const int l = fresh_lane(), g = l >> 4, r = l & 15;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tile = w + 8 * j;
      if (tile < NT16) {
        const int q = tile * 16 + r;
        const bf16x8 d0 = lds_row8(Ds, q, g), d1 = lds_row8(Ds, q, 4 + g);
        float delta = 0.f;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          delta += (float)d0[jj] * (float)p.o[j][0][jj] + (float)d1[jj] * (float)p.o[j][1][jj];
        delta += __shfl_xor(delta, 16, 64);
        delta += __shfl_xor(delta, 32, 64);
        if (g == 0) del_s[q] = q < T ? delta : 0.f;
      }
    }
    if ((int)threadIdx.x < TP) lse_s[threadIdx.x] = (int)threadIdx.x < T ? p.lse * 1.44269504088896341f : INFINITY;
  };

  // P and dS of one query tile against one key tile (attn_bwd_dkv2_kernel's p_ds)
  auto p_ds = [&](bf16x8 q0, bf16x8 q1, bf16x8 d0, bf16x8 d1, f32x4 l4, f32x4 d4, bf16x8 kf0, bf16x8 kf1,
                  bf16x8 vf0, bf16x8 vf1, f32x4& p, f32x4& ds) {
    f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
    sv = mfma16(q0, kf0, sv);
    sv = mfma16(q1, kf1, sv);
    dp = mfma16(d0, vf0, dp);
    dp = mfma16(d1, vf1, dp);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p[i] = __builtin_amdgcn_exp2f(sv[i] * sl - l4[i]);
      ds[i] = p[i] * (dp[i] - d4[i]);
    }
  };
  const bf16x8 zero8 = {};
  const bf16x4 zero4 = {};
  // phase 1 over query pairs [s0, s1) (+ the odd tile NT16 - 1), dS written for queries qbase..
  auto phase1 = [&](const bf16x8 (&kv)[8], f32x4 (&dk)[2][4], f32x4 (&dv)[2][4], int s0, int s1, bool odd,
                    int qbase) {
    const int l = fresh_lane(), g = l >> 4, r = l & 15;
    const int keyA = w * 32 + r, keyB = keyA + 16;
    const bool wrB = w * 32 + 16 < TP;  // the phantom tile past the head (keys 208..223) is not written
#pragma unroll 1
    for (int sc = s0; sc < s1; ++sc) {
      const int ua = 2 * sc * 16 + r, ub = ua + 16;
      const bf16x8 qa0 = lds_row8(Qs, ua, g), qa1 = lds_row8(Qs, ua, 4 + g);
      const bf16x8 da0 = lds_row8(Ds, ua, g), da1 = lds_row8(Ds, ua, 4 + g);
      const bf16x8 qb0 = lds_row8(Qs, ub, g), qb1 = lds_row8(Qs, ub, 4 + g);
      const bf16x8 db0 = lds_row8(Ds, ub, g), db1 = lds_row8(Ds, ub, 4 + g);
      const f32x4 la = *(const f32x4*)(lse_s + 2 * sc * 16 + 4 * g);
      const f32x4 dla = *(const f32x4*)(del_s + 2 * sc * 16 + 4 * g);
      const f32x4 lb = *(const f32x4*)(lse_s + 2 * sc * 16 + 16 + 4 * g);
      const f32x4 dlb = *(const f32x4*)(del_s + 2 * sc * 16 + 16 + 4 * g);
      bf16x8 tdo[4], tq[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tdo[dt] = lds_trT(Ds, sc * 32, dt * 16, g, r);
        tq[dt] = lds_trT(Qs, sc * 32, dt * 16, g, r);
      }
      const int ql = sc * 32 - qbase;
      char* img = Ss + (ql >> 6) * IMG;
      const int c = ((ql >> 5) & 1) * 4 + g;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x4 p0, p1, s0_, s1_;
        p_ds(qa0, qa1, da0, da1, la, dla, kv[4 * kt], kv[4 * kt + 1], kv[4 * kt + 2], kv[4 * kt + 3], p0, s0_);
        p_ds(qb0, qb1, db0, db1, lb, dlb, kv[4 * kt], kv[4 * kt + 1], kv[4 * kt + 2], kv[4 * kt + 3], p1, s1_);
        bf16x8 pf, dsf;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pf[i] = (bf16)p0[i];
          pf[4 + i] = (bf16)p1[i];
          dsf[i] = (bf16)s0_[i];
          dsf[4 + i] = (bf16)s1_[i];
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[kt][dt] = mfma16(tdo[dt], pf, dv[kt][dt]);
          dk[kt][dt] = mfma16(tq[dt], dsf, dk[kt][dt]);
        }
        const int key = kt ? keyB : keyA, f = sws(key);
        const bf16x8 sw = (f & 1) ? __builtin_shufflevector(dsf, dsf, 4, 5, 6, 7, 0, 1, 2, 3) : dsf;
        if (kt == 0 || wrB) *(bf16x8*)(img + key * 128 + (c ^ (f >> 1)) * 16) = key < T ? sw : zero8;
      }
    }
    if (odd) {
      const int u = NT16 - 1;
      const bf16x8 q0 = lds_row8(Qs, u * 16 + r, g), q1 = lds_row8(Qs, u * 16 + r, 4 + g);
      const bf16x8 d0 = lds_row8(Ds, u * 16 + r, g), d1 = lds_row8(Ds, u * 16 + r, 4 + g);
      const f32x4 l4 = *(const f32x4*)(lse_s + u * 16 + 4 * g), d4 = *(const f32x4*)(del_s + u * 16 + 4 * g);
      bf16x4 tdo4[4], tq4[4];
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        tdo4[dt] = lds_trT4(Ds, u * 16, dt * 16, g, r);
        tq4[dt] = lds_trT4(Qs, u * 16, dt * 16, g, r);
      }
      const int ql = u * 16 - qbase;
      char* img = Ss + (ql >> 6) * IMG;
      const int c = ((ql >> 5) & 1) * 4 + g;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x4 p0, s0_;
        p_ds(q0, q1, d0, d1, l4, d4, kv[4 * kt], kv[4 * kt + 1], kv[4 * kt + 2], kv[4 * kt + 3], p0, s0_);
        const bf16x4 pf = {(bf16)p0[0], (bf16)p0[1], (bf16)p0[2], (bf16)p0[3]};
        const bf16x4 dsf = {(bf16)s0_[0], (bf16)s0_[1], (bf16)s0_[2], (bf16)s0_[3]};
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          dv[kt][dt] = mfma16k16(tdo4[dt], pf, dv[kt][dt]);
          dk[kt][dt] = mfma16k16(tq4[dt], dsf, dk[kt][dt]);
        }
        const int key = kt ? keyB : keyA;
        if (kt == 0 || wrB) *(bf16x4*)(img + key * 128 + ((2 * c) ^ sws(key)) * 8) = key < T ? dsf : zero4;
      }
    }
  };
  // phase 2: dQ of query tile `tile` (queries qbase.. in the dS images), out through the wave's slot
  // NDT = 4: the whole tile; NDT = 2: its dims 32 hd .. + 31 (the second round, where five tiles meet eight
  // waves, runs ten halves).  Per 16-dim block the same MFMAs in the same order either way.
  auto phase2 = [&](auto ndt_tag, int bh, int tile, int hd, int qbase) {
    constexpr int NDT = decltype(ndt_tag)::value;
    const int l = fresh_lane(), g = l >> 4, r = l & 15;
    const int ql = tile * 16 - qbase;
    const char* img = Ss + (ql >> 6) * IMG;
    const int seg = (ql >> 5) & 1, half = (ql >> 4) & 1, d0 = NDT == 4 ? 0 : 2 * hd;
    f32x4 dq[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) dq[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
    for (int sc = 0; sc < NP; ++sc) {
      bf16x8 tk[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) tk[dt] = lds_trT(Ks, sc * 32, (d0 + dt) * 16, g, r);
      const bf16x8 dsf = lds_trS(img, sc * 32, seg, half, g, r);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) dq[dt] = mfma16(tk[dt], dsf, dq[dt]);
    }
    {
      const int t = NT16 - 1;
      bf16x4 tk4[NDT];
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) tk4[dt] = lds_trT4(Ks, t * 16, (d0 + dt) * 16, g, r);
      const bf16x4 dsf = lds_trS4(img, t * 16, seg, half, g, r);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) dq[dt] = mfma16k16(tk4[dt], dsf, dq[dt]);
    }
    const int img_i = bh / a.H, h = bh - img_i * a.H, q0 = tile * 16;
    bf16* dst = a.dqkv + ((size_t)img_i * T + q0) * a.lddqkv + h * 64 + d0 * 16;
    if constexpr (NDT == 4) tile_rows_out(slot, dq, a.scale, dst, a.lddqkv, T - q0);
    else half_rows_out(slot, dq, a.scale, dst, a.lddqkv, T - q0);
  };
  using Whole = std::integral_constant<int, 4>;
  using Half = std::integral_constant<int, 2>;

  int bh = blockIdx.x;
  stage_qdo(bh, 0, NG, 0, 8);
  stage_k(bh);
  Pre pre = prefetch(bh);
  const int nk = (NG - w + 7) / 8;  // this wave's K pieces: the youngest VMEM ops at the top of a head
  for (;;) {
    const int img = bh / a.H, h = bh - img * a.H;
    const int nx = bh + gridDim.x;
    const bool more = nx < nbh;
    if (nk == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // Q / dO landed (K may be in flight)
    else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    lds_barrier();
    deltas(pre);
    // this head's K image (DMA'd behind the previous head's last phase) and the register prefetch; the builtin
    // (a vmcnt(0) hipcc sees) retires the prefetch on every path, so no later counted wait of hipcc's drains
    // the DMAs issued below
    __builtin_amdgcn_s_waitcnt(0x0F70);
    lds_barrier();
    f32x4 dk[2][4], dv[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) dk[t][dt] = dv[t][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 kv[8];  // per key tile t: K dims 8g.. / 32 + 8g.., V the same (zero past T)
    {
      const int l = fresh_lane(), g = l >> 4, r = l & 15;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int key = w * 32 + 16 * t + r;
        const bf16x8 k0 = lds_row8(Ks, key < TP ? key : 0, g), k1 = lds_row8(Ks, key < TP ? key : 0, 4 + g);
        kv[4 * t + 0] = key < T ? k0 : zero8;
        kv[4 * t + 1] = key < T ? k1 : zero8;
        kv[4 * t + 2] = pre.v[2 * t];
        kv[4 * t + 3] = pre.v[2 * t + 1];
      }
    }
    if (w < (NT16 + 1) / 2) phase1(kv, dk, dv, 0, PA, false, 0);
    lds_barrier();
    if (more) stage_qdo(nx, 0, PA * 32 / 8, 0, 8);  // rows 0..127: phase 1 is done with them
    phase2(Whole{}, bh, w, 0, 0);
    lds_barrier();
    if (w < (NT16 + 1) / 2) phase1(kv, dk, dv, PA, NP, true, 2 * PA * 16);
    lds_barrier();
    // every wave's loads issue before its dK / dV stores (stores issue at ~14 B/clk per CU: VMEM ops behind
    // them would wait); the round-2 dQ as ten half tiles: waves 0..6 one each beside their dK / dV stores,
    // wave 7 (no key tiles) three
    if (more) stage_qdo(nx, PA * 32 / 8, NG, 0, 8);
    // unconditional (the last head re-reads its own rows): a conditional assignment would keep the old
    // operands live through the phases for the join
    pre = prefetch(more ? nx : bh);
    static_assert(2 * (NT16 - 2 * PA) == 10, "ten half tiles");
    if (w < 7) {
      phase2(Half{}, bh, 2 * PA + (w >> 1), w & 1, 2 * PA * 16);
    } else {
      phase2(Half{}, bh, 2 * PA + 3, 1, 2 * PA * 16);
      phase2(Half{}, bh, 2 * PA + 4, 0, 2 * PA * 16);
      phase2(Half{}, bh, 2 * PA + 4, 1, 2 * PA * 16);
    }
    if (w < (NT16 + 1) / 2) {
      bf16* d0 = a.dqkv + ((size_t)img * T + w * 32) * a.lddqkv + D + h * 64;
      tile_rows_out(slot, dk[0], a.scale, d0, a.lddqkv, T - w * 32);
      tile_rows_out(slot, dv[0], 1.0f, d0 + D, a.lddqkv, T - w * 32);
      tile_rows_out(slot, dk[1], a.scale, d0 + 16 * (size_t)a.lddqkv, a.lddqkv, T - w * 32 - 16);
      tile_rows_out(slot, dv[1], 1.0f, d0 + 16 * (size_t)a.lddqkv + D, a.lddqkv, T - w * 32 - 16);
    }
    lds_barrier();
    if (!more) break;
    stage_k(nx);
    bh = nx;
  }
}

// ---- CLS-query attention (the last block: only the CLS rows reach the head) ---------------------
// One wave per (image, head).  Lane (c = lane & 7, jg = lane >> 3) holds dims 8c..8c+7 and walks keys
// j = jg, jg + 8, ...: each 8-lane group reads whole 128-B K / V rows (coalesced) and completes a
// dot product with 3 xor-shuffles.  Same rounding points as attn_fwd_kernel / the backward kernels
// (scores in log2 units, bf16(P) into P.V, bf16(dS) into dQ / dK, bf16(P) into dV); only the fp32
// summation order differs.  Outputs are compact: o / do [img][D], lse [img][head].
constexpr int CLS_KMAX = 32;       // keys per lane group: T <= 256
constexpr int CLS_KMAX_LONG = 80;  // T <= 640 (ViT/16 at 384^2: 577)

__device__ __forceinline__ float grp8_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  return v;
}

__device__ __forceinline__ void ld8f(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}

template <int KMAX>
__global__ __launch_bounds__(64) void attn_cls_fwd_kernel(const bf16* __restrict__ qkv, int ldqkv, bf16* __restrict__ o,
                                                          int ldo, float* __restrict__ lse, int T, int H, float scale) {
  const int bh = blockIdx.x, img = bh / H, h = bh - img * H, D = H * 64;
  const int lane = threadIdx.x, c = lane & 7, jg = lane >> 3;
  const bf16* base = qkv + (size_t)img * T * ldqkv;
  float q[8];
  ld8f(base + h * 64 + 8 * c, q);
  const float sl = scale * 1.44269504088896341f;
  float s[KMAX];
  float mx = -INFINITY;
#pragma unroll
  for (int it = 0; it < KMAX; ++it) {
    const int j = it * 8 + jg;
    float part = 0.f;
    if (j < T) {
      float k[8];
      ld8f(base + (size_t)j * ldqkv + D + h * 64 + 8 * c, k);
#pragma unroll
      for (int i = 0; i < 8; ++i) part = fmaf(q[i], k[i], part);
    }
    const float dot = grp8_sum(part);
    s[it] = j < T ? dot * sl : -INFINITY;
    mx = fmaxf(mx, s[it]);
  }
  mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int it = 0; it < KMAX; ++it) {
    const int j = it * 8 + jg;
    if (j < T) {
      const float p = __builtin_amdgcn_exp2f(s[it] - mx);
      l += p;
      const float pb = (float)(bf16)p;
      float v[8];
      ld8f(base + (size_t)j * ldqkv + 2 * D + h * 64 + 8 * c, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(pb, v[i], acc[i]);
    }
  }
#pragma unroll
  for (int m = 8; m < 64; m <<= 1) {
    l += __shfl_xor(l, m, 64);
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] += __shfl_xor(acc[i], m, 64);
  }
  if (jg == 0) {
    const float inv = 1.0f / l;
    bf16x8 ov;
#pragma unroll
    for (int i = 0; i < 8; ++i) ov[i] = (bf16)(acc[i] * inv);
    *(bf16x8*)(o + (size_t)img * ldo + h * 64 + 8 * c) = ov;
    if (c == 0) lse[bh] = (mx + __log2f(l)) * 0.69314718055994531f;
  }
}

// dQ (CLS row), dK / dV (every key) and zeros for the Q part of the other rows: the whole dqkv of
// the block's tokens, so the qkv data / weight gradient GEMMs read it as written by es_attn_bwd.
template <int KMAX>
__global__ __launch_bounds__(64) void attn_cls_bwd_kernel(const bf16* __restrict__ qkv, int ldqkv,
                                                          const bf16* __restrict__ o, int ldo,
                                                          const float* __restrict__ lse,
                                                          const bf16* __restrict__ dout, int lddo,
                                                          bf16* __restrict__ dqkv, int lddqkv, int T, int H,
                                                          float scale) {
  const int bh = blockIdx.x, img = bh / H, h = bh - img * H, D = H * 64;
  const int lane = threadIdx.x, c = lane & 7, jg = lane >> 3;
  const bf16* base = qkv + (size_t)img * T * ldqkv;
  bf16* dbase = dqkv + (size_t)img * T * lddqkv;
  float q[8], dq_o[8], ov[8];
  ld8f(base + h * 64 + 8 * c, q);
  ld8f(dout + (size_t)img * lddo + h * 64 + 8 * c, dq_o);
  ld8f(o + (size_t)img * ldo + h * 64 + 8 * c, ov);
  float dpart = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) dpart += dq_o[i] * ov[i];
  const float delta = grp8_sum(dpart);
  const float sl = scale * 1.44269504088896341f;
  const float lq = lse[bh] * 1.44269504088896341f;
  float dqa[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16x8 zero8 = {};
  for (int it = 0; it < KMAX; ++it) {
    const int j = it * 8 + jg;
    if (it * 8 >= T) break;
    float k[8], v[8];
    float sp = 0.f, dpp = 0.f;
    if (j < T) {
      ld8f(base + (size_t)j * ldqkv + D + h * 64 + 8 * c, k);
      ld8f(base + (size_t)j * ldqkv + 2 * D + h * 64 + 8 * c, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sp = fmaf(q[i], k[i], sp);
        dpp = fmaf(dq_o[i], v[i], dpp);
      }
    }
    const float sv = grp8_sum(sp), dp = grp8_sum(dpp);
    if (j < T) {
      const float p = __builtin_amdgcn_exp2f(sv * sl - lq);
      const float ds = p * (dp - delta);
      const float pb = (float)(bf16)p, dsb = (float)(bf16)ds;
      bf16x8 dk8, dv8;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        dk8[i] = (bf16)(dsb * q[i] * scale);
        dv8[i] = (bf16)(pb * dq_o[i]);
        dqa[i] = fmaf(dsb, k[i], dqa[i]);
      }
      bf16* drow = dbase + (size_t)j * lddqkv + h * 64 + 8 * c;
      *(bf16x8*)(drow + D) = dk8;
      *(bf16x8*)(drow + 2 * D) = dv8;
      if (j > 0) *(bf16x8*)drow = zero8;
    }
  }
#pragma unroll
  for (int m = 8; m < 64; m <<= 1)
#pragma unroll
    for (int i = 0; i < 8; ++i) dqa[i] += __shfl_xor(dqa[i], m, 64);
  if (jg == 0) {
    bf16x8 d8;
#pragma unroll
    for (int i = 0; i < 8; ++i) d8[i] = (bf16)(dqa[i] * scale);
    *(bf16x8*)(dbase + h * 64 + 8 * c) = d8;
  }
}

#define ATTN_CASE(KERNEL, N_, GRID, LDS, STREAM, ARGS) \
  case N_: allow_lds(KERNEL<N_>, LDS); hipLaunchKernelGGL(KERNEL<N_>, GRID, 256, LDS, STREAM, ARGS); break;

#define ATTN_DISPATCH(KERNEL, NT16_, GRID, LDS, STREAM, ARGS)                                               \
  switch (NT16_) {                                                                                        \
    ATTN_CASE(KERNEL, 1, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 2, GRID, LDS, STREAM, ARGS)            \
    ATTN_CASE(KERNEL, 3, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 4, GRID, LDS, STREAM, ARGS)            \
    ATTN_CASE(KERNEL, 5, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 6, GRID, LDS, STREAM, ARGS)            \
    ATTN_CASE(KERNEL, 7, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 8, GRID, LDS, STREAM, ARGS)            \
    ATTN_CASE(KERNEL, 9, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 10, GRID, LDS, STREAM, ARGS)           \
    ATTN_CASE(KERNEL, 11, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 12, GRID, LDS, STREAM, ARGS)          \
    ATTN_CASE(KERNEL, 13, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 14, GRID, LDS, STREAM, ARGS)          \
    ATTN_CASE(KERNEL, 15, GRID, LDS, STREAM, ARGS) ATTN_CASE(KERNEL, 16, GRID, LDS, STREAM, ARGS)          \
    ATTN_CASE(KERNEL, 37, GRID, LDS, STREAM, ARGS)                                                        \
    default: return ES_BAD_SHAPE;                                                                         \
  }

#define FWD_CASE(N_, OCC_, GRID, LDS, STREAM, ARGS)                                                  \
  case N_:                                                                                          \
    allow_lds(attn_fwd_kernel<N_, OCC_>, LDS);                                                      \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_fwd_kernel<N_, OCC_>), GRID, 256, LDS, STREAM, ARGS);   \
    break;
#define FWD_DISPATCH(NT16_, OCC_, GRID, LDS, STREAM, ARGS)                                            \
  switch (NT16_) {                                                                                  \
    FWD_CASE(1, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(2, OCC_, GRID, LDS, STREAM, ARGS)            \
    FWD_CASE(3, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(4, OCC_, GRID, LDS, STREAM, ARGS)            \
    FWD_CASE(5, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(6, OCC_, GRID, LDS, STREAM, ARGS)            \
    FWD_CASE(7, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(8, OCC_, GRID, LDS, STREAM, ARGS)            \
    FWD_CASE(9, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(10, OCC_, GRID, LDS, STREAM, ARGS)           \
    FWD_CASE(11, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(12, OCC_, GRID, LDS, STREAM, ARGS)          \
    FWD_CASE(13, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(14, OCC_, GRID, LDS, STREAM, ARGS)          \
    FWD_CASE(15, OCC_, GRID, LDS, STREAM, ARGS) FWD_CASE(16, OCC_, GRID, LDS, STREAM, ARGS)          \
    default: return ES_BAD_SHAPE;                                                                   \
  }

// forward occupancy target (workgroups per CU the register budget is sized for): 2 = no cap
// (measured faster: 108 vs 150 us at the F1 shape, scripts/attn_bench.py),
// 3 = 168 VGPRs (three 52-KiB heads per CU, small spill), 7 (default) = variant 2 with seven waves per
// workgroup at 13 tiles (T = 197): 0.0851 / 0.0836 -> 0.0731 / 0.0728 ms at the F1 head batch,
// bit-identical (scripts/attn_bench.py; 14 waves per CU instead of 8, no 4-tile wave)
int g_attn_fwd_occ = 7;
// backward kernels: 1 = the software-pipelined dQ / dK-dV loops (attn_bwd_*_pipe_kernel), 2 = the pipelined dQ
// and the two-key-tiles-per-wave dK / dV (attn_bwd_dkv2_kernel), 3 = two query tiles per wave for dQ
// (attn_bwd_dq2_kernel) and dkv2, 4 = the single pass (attn_bwd_fused_kernel; 13-tile heads, others as 3),
// 0 = the plain loops (all bit-identical).  Default 4: F1 head batch 0.2015 vs 0.2419 ms (3) isolated, 633 vs
// 941 MB; inside the two-stream step on g_attn_bwd_grid's default grid (one workgroup per CU: worse than 3).
// Round 3: 3 at 0.257 vs 0.269 (1) and 0.289 (0)
int g_attn_bwd_pipe = 4;
// the same variants for T = 577 (the 37-tile kernels: one 151-KiB head per CU, four waves)
int g_attn_bwd_long = 1;
// the single pass's grid: -1 (default) = max(CUs, heads / 4), 0 = one persistent workgroup per CU, else this
// many.  Inside the two-stream F1 step (profiles/r04_attn_bwd_live_ab.txt) a head
// or two per workgroup lets the side stream's weight-gradient launches take CUs between them, twelve per
// workgroup (one per CU) holds the CUs: 3072 heads on 768 workgroups 30.78-30.80 ms/step, 1024: 30.86-30.90,
// 1536: 30.80-30.87, 3072: 31.05-31.09, 256: +0.5 ms, the two-pass kernels 30.95-31.03 (one box)
int g_attn_bwd_grid = -1;

}  // namespace

extern "C" {

// tuning knob: forward attention workgroups per CU the register budget targets (2 or 3)
int es_set_attn_variant(int occ) {
  const int old = g_attn_fwd_occ;
  g_attn_fwd_occ = occ;
  return old;
}

// tuning knob: attention backward loops (0 plain, 1 pipelined, 2 pipelined dQ + dkv2, 3 dq2 + dkv2,
// 4 = default: the single-pass kernel for 13-tile heads, else as 3); returns the previous value, or
// ES_BAD_ARG (state unchanged) for any other value
int es_set_attn_bwd_variant(int v) {
  if (v < 0 || v > 4) return ES_BAD_ARG;
  const int old = g_attn_bwd_pipe;
  g_attn_bwd_pipe = v;
  return old;
}

// tuning knob: the single-pass backward's workgroups (-1 = max(CUs, heads / 4), 0 = one per CU); returns the
// previous value
int es_set_attn_bwd_grid(int workgroups) {
  const int old = g_attn_bwd_grid;
  g_attn_bwd_grid = workgroups < -1 ? -1 : workgroups;
  return old;
}

// tuning knob: 1 = es_set_attn_bwd_variant's variant also at T > 256 (37 tiles), 0 = the plain loops there
int es_set_attn_bwd_long(int v) {
  const int old = g_attn_bwd_long;
  g_attn_bwd_long = v;
  return old;
}


// 16-key tiles of a head: exact for T <= 256; one 37-tile instantiation (592 rows: two staged heads
// fit the 160 KiB of LDS) covers 256 < T <= 592 (ViT/16 at 384^2, T = 577), rows past T masked
static int attn_tiles(int T) { return T <= 256 ? (T + 15) / 16 : 37; }
constexpr int ATTN_TMAX = 592;

// qkv [nimg*T, ldqkv] -> o [nimg*T, ldo], lse [nimg*H*T]; head dim 64, T <= 592.
int es_attn_fwd(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > ATTN_TMAX || H <= 0 || ldqkv < 3 * H * 64 || ldo < H * 64 || (ldqkv % 8) ||
      (ldo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse) return ES_BAD_ARG;
  AttnArgs a{(const bf16*)qkv, (bf16*)o, lse, nullptr, nullptr, nullptr, ldqkv, ldo, 0, 0, T, H, scale};
  if (T > 256) {  // online softmax over key chunks, K / V staged, eight waves
    const size_t lds = 2 * (size_t)37 * 16 * 128 + 8 * 1024;  // K, V + eight 1-KiB output slots
    allow_lds(attn_fwd_long_kernel<37>, lds);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_fwd_long_kernel<37>), nimg * H, 512, lds, stream, a);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  const int nt16 = (T + 15) / 16;
  const size_t lds = 3 * (size_t)nt16 * 16 * 128;  // K, V, Q head tiles (two heads per CU at T = 197)
  if (g_attn_fwd_occ == 7 && nt16 == 13) {
    allow_lds(attn_fwd_kernel<13, 2, 7>, lds);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_fwd_kernel<13, 2, 7>), nimg * H, 448, lds, stream, a);
  } else if (g_attn_fwd_occ == 2 || g_attn_fwd_occ == 7) {
    FWD_DISPATCH(nt16, 2, nimg * H, lds, stream, a);
  } else {
    FWD_DISPATCH(nt16, 3, nimg * H, lds, stream, a);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// dout [nimg*T, lddo] + forward (qkv, o, lse) -> dqkv [nimg*T, lddqkv] (q, k and v parts).
// delta: workspace [nimg*H*T] fp32 (rowsum(dO*O), written by the dQ pass, read by the dK/dV pass).
int es_attn_bwd(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, float* delta, const void* dout,
                int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > ATTN_TMAX || H <= 0 || ldqkv < 3 * H * 64 || lddqkv < 3 * H * 64 || (ldqkv % 8) ||
      (lddqkv % 8) || (ldo % 8) || (lddo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse || !delta || !dout || !dqkv) return ES_BAD_ARG;
  AttnArgs a{(const bf16*)qkv, (bf16*)o, (float*)lse, delta, (const bf16*)dout, (bf16*)dqkv, ldqkv, ldo, lddo,
             lddqkv, T, H, scale};
  const int nt16 = attn_tiles(T);
  const size_t lds_dq = 2 * (size_t)nt16 * 16 * 128;
  const size_t lds_dkv = lds_dq + 2 * (size_t)nt16 * 16 * 4;
  // dq2 / dkv2 output slots; the 37-tile heads (one 148-KiB head per CU) run 8 / 6 waves, so each SIMD holds
  // two of them (four waves left one per SIMD with nothing to hide the LDS latency behind)
  const int nw_dq = nt16 == 37 ? 8 : 4, nw_dkv = nt16 == 37 ? 6 : 4;
  const size_t slots_dq = nw_dq * (nw_dq == 4 ? 2048 : 1024), slots_dkv = nw_dkv * (nt16 <= 16 ? 2048 : 1024);
  // ViT/16 at 224^2 (T = 197, 13 tiles) and at 384^2 (T = 577, the 37-tile instantiation): the pipelined /
  // two-tile loops (bit-identical to the plain ones)
#define BWD_VARIANTS(N_)                                                                                    \
  if (g_attn_bwd_pipe >= 3) {                                                                               \
    if (nw_dq == 8) {                                                                                       \
      allow_lds(attn_bwd_dq2_kernel<N_, 8>, lds_dq + slots_dq);                                             \
      hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dq2_kernel<N_, 8>), nimg * H, 512, lds_dq + slots_dq, stream, a); \
    } else {                                                                                                \
      allow_lds(attn_bwd_dq2_kernel<N_>, lds_dq + slots_dq);                                                \
      hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dq2_kernel<N_>), nimg * H, 256, lds_dq + slots_dq, stream, a); \
    }                                                                                                       \
  } else {                                                                                                  \
    allow_lds(attn_bwd_dq_pipe_kernel<N_>, lds_dq);                                                         \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dq_pipe_kernel<N_>), nimg * H, 256, lds_dq, stream, a);     \
  }                                                                                                         \
  if (g_attn_bwd_pipe >= 2) {                                                                               \
    if (nw_dkv == 6) {                                                                                      \
      allow_lds(attn_bwd_dkv2_kernel<N_, false, 6>, lds_dkv + slots_dkv);                                   \
      hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dkv2_kernel<N_, false, 6>), nimg * H, 384, lds_dkv + slots_dkv, \
                         stream, a);                                                                        \
    } else {                                                                                                \
      allow_lds(attn_bwd_dkv2_kernel<N_>, lds_dkv + slots_dkv);                                             \
      hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dkv2_kernel<N_>), nimg * H, 256, lds_dkv + slots_dkv, stream, a); \
    }                                                                                                       \
  } else {                                                                                                  \
    allow_lds(attn_bwd_dkv_pipe_kernel<N_>, lds_dkv);                                                       \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_dkv_pipe_kernel<N_>), nimg * H, 256, lds_dkv, stream, a);   \
  }                                                                                                         \
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  if (g_attn_bwd_pipe == 4 && nt16 == 13 &&
      (size_t)nimg * T * std::max(std::max(ldqkv, ldo), lddo) * 2 < ((size_t)1 << 31)) {
    static int cus = 0;
    if (!cus) {
      int dev = 0;
      (void)hipGetDevice(&dev);
      if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    }
    const size_t lds = 5 * (size_t)13 * 16 * 128 + 2 * 13 * 16 * 4 + 8 * 2048;
    allow_lds(attn_bwd_fused_kernel<13>, lds);
    const int heads = nimg * H;
    const int grid = std::min(g_attn_bwd_grid > 0 ? g_attn_bwd_grid
                                                  : (g_attn_bwd_grid == 0 ? cus : std::max(cus, (heads + 3) / 4)),
                              heads);
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_bwd_fused_kernel<13>), grid, 512, lds, stream, a, nimg * H);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  if (g_attn_bwd_pipe && nt16 == 13) { BWD_VARIANTS(13) }
  if (g_attn_bwd_pipe && nt16 == 37 && g_attn_bwd_long) { BWD_VARIANTS(37) }
#undef BWD_VARIANTS
  ATTN_DISPATCH(attn_bwd_dq_kernel, nt16, nimg * H, lds_dq, stream, a);
  ATTN_DISPATCH(attn_bwd_dkv_kernel, nt16, nimg * H, lds_dkv, stream, a);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}


// CLS-query attention of a block whose non-CLS outputs are unused (the ViT's last block): qkv
// [nimg*T, ldqkv] -> o [nimg, ldo] (the CLS rows only, compact), lse [nimg*H].
int es_attn_cls_fwd(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                    hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 8 * CLS_KMAX_LONG || H <= 0 || ldqkv < 3 * H * 64 || ldo < H * 64 || (ldqkv % 8) ||
      (ldo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse) return ES_BAD_ARG;
  if (T <= 8 * CLS_KMAX)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_cls_fwd_kernel<CLS_KMAX>), nimg * H, 64, 0, stream, (const bf16*)qkv, ldqkv,
                       (bf16*)o, ldo, lse, T, H, scale);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_cls_fwd_kernel<CLS_KMAX_LONG>), nimg * H, 64, 0, stream, (const bf16*)qkv,
                       ldqkv, (bf16*)o, ldo, lse, T, H, scale);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// Backward of es_attn_cls_fwd: dout [nimg, lddo] (CLS rows) -> dqkv [nimg*T, lddqkv] for every token
// (q part zero except the CLS rows).
int es_attn_cls_bwd(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, const void* dout, int lddo,
                    void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream) {
  if (nimg <= 0 || T <= 0 || T > 8 * CLS_KMAX_LONG || H <= 0 || ldqkv < 3 * H * 64 || lddqkv < 3 * H * 64 ||
      ldo < H * 64 || lddo < H * 64 || (ldqkv % 8) || (lddqkv % 8) || (ldo % 8) || (lddo % 8))
    return ES_BAD_SHAPE;
  if (!qkv || !o || !lse || !dout || !dqkv) return ES_BAD_ARG;
  if (T <= 8 * CLS_KMAX)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_cls_bwd_kernel<CLS_KMAX>), nimg * H, 64, 0, stream, (const bf16*)qkv, ldqkv,
                       (const bf16*)o, ldo, lse, (const bf16*)dout, lddo, (bf16*)dqkv, lddqkv, T, H, scale);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(attn_cls_bwd_kernel<CLS_KMAX_LONG>), nimg * H, 64, 0, stream, (const bf16*)qkv,
                       ldqkv, (const bf16*)o, ldo, lse, (const bf16*)dout, lddo, (bf16*)dqkv, lddqkv, T, H, scale);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
