// bf16 MFMA GEMMs for the ViT step (gfx950).
//
//  gemm_nt : C[M,N] = A[M,K] . B[N,K]^T (+ fused epilogue)      -- forward Linear / conv and dgrad
//            (dgrad uses the transposed bf16 weight image W^T [K_in, N_out] that the optimizer
//             writes, so it is an NT product too)
//  gemm_tn : P[s][N1,N2] = sum_{m in split s} A1[m,N1]^T . A2[m,N2] -- wgrad, split over tokens
//  splitk_reduce, colsum_partial : fp32 slab reductions (wgrad partials, bias grads)
//
// Replaces the reference's implicit aten::addmm / mm / conv2d calls on the ViT path
// (code/models/conformer.py:13-23,35-50 Linear layers; timm PatchEmbed Conv2d(3,D,16,16)).
//
// Tiling (both kernels): 128x128 output tile, 64-deep K step, 256 threads = 4 waves in a 2x2
// arrangement, each wave 64x64 = 4x4 MFMA 16x16x32 tiles.  Operand tiles are staged HBM->LDS with
// global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear destination), XOR-swizzled on
// the SOURCE address so the fragment reads are bank-conflict free; two LDS stages; the stage for
// step k+1 is issued before the MFMAs of step k.
#include <algorithm>
#include <cstdlib>

#include <hip/hip_ext.h>

#include "common.h"

namespace es_gemm {

constexpr int BM = 128, BN = 128, BK = 64;

enum Epi {
  EPI_BF16 = 0,       // C bf16 = acc (+bias)
  EPI_GELU = 1,       // C bf16 = acc+bias (pre-activation), C2 bf16 = gelu(acc+bias)
  EPI_F32_RESID = 2,  // C f32 = acc (+bias) + aux_f32
  EPI_DGELU = 3,      // C bf16 = acc * gelu'(aux_bf16)
  EPI_F32 = 4,        // C f32 = acc (+bias)
  EPI_PATCH = 5,      // C f32 at token row (img*(np+1)+1+p) = acc + bias + pos[1+p]
  EPI_GELU_ACT = 6,   // C bf16 = gelu(acc+bias) only (inference: no pre-activation kept)
  EPI_GELU_D = 7,     // C bf16 = gelu'(acc+bias), C2 bf16 = gelu(acc+bias): the derivative the backward
                      // needs instead of the pre-activation (it shares the erf's exp; no erf in the backward)
  EPI_MULAUX = 8,     // C bf16 = acc * aux_bf16 (the backward of EPI_GELU_D: dpre = dact * gelu')
};

struct NTArgs {
  const bf16* A; const bf16* B; const float* bias;
  void* C; void* C2; const void* aux;
  int M, N, K, lda, ldb, ldc, ldaux, np;
};

// 128-byte rows (64 bf16), 16-byte chunk c of row r stored at chunk c ^ ((r >> 1) & 7).
__device__ __forceinline__ int swz128(int r, int c) { return c ^ ((r >> 1) & 7); }
// 64-byte rows (32 bf16), chunk c of row r at c ^ ((-(r >> 2)) & 3): conflict-free fragment reads.
__device__ __forceinline__ int swz64(int r, int c) { return c ^ ((4 - ((r >> 2) & 3)) & 3); }

// ---- fused epilogue on 8-column row segments ------------------------------------------------
// Operands an epilogue reads besides the accumulator: per lane, the bias of its 8 columns (loaded
// once -- a lane's columns do not change across row chunks) and per segment the row-dependent
// aux (fp32 residual, bf16 pre-activation, fp32 position embedding), issued one row chunk ahead
// of the stores.  All aux loads and C stores are buffer operations on range-checked resources
// with rows >= M mapped to ES_OOB (no branches: vmcnt counts loads and stores together on gfx9,
// and straight-line code lets the compiler count instead of draining).
template <int EPI>
struct EpiCtx {
  __amdgpu_buffer_rsrc_t c, c2, aux;
  int esz;  // bytes per C element
};

template <int EPI>
__device__ __forceinline__ EpiCtx<EPI> epi_ctx(const NTArgs& p) {
  EpiCtx<EPI> x;
  constexpr bool f32out = (EPI == EPI_F32_RESID || EPI == EPI_F32 || EPI == EPI_PATCH);
  x.esz = f32out ? 4 : 2;
  const unsigned crows = EPI == EPI_PATCH ? (unsigned)(p.M / p.np) * (p.np + 1) : (unsigned)p.M;
  x.c = buf_rsrc(p.C, crows * p.ldc * x.esz);
  x.c2 = buf_rsrc((EPI == EPI_GELU || EPI == EPI_GELU_D) ? p.C2 : p.C, crows * p.ldc * x.esz);
  if constexpr (EPI == EPI_F32_RESID) x.aux = buf_rsrc(p.aux, (unsigned)p.M * p.ldaux * 4);
  else if constexpr (EPI == EPI_DGELU || EPI == EPI_MULAUX) x.aux = buf_rsrc(p.aux, (unsigned)p.M * p.ldaux * 2);
  else if constexpr (EPI == EPI_PATCH) x.aux = buf_rsrc(p.aux, (unsigned)(p.np + 1) * p.ldaux * 4);
  else x.aux = x.c;
  return x;
}

struct EpiAuxRegs { u32x4 a0, a1; };

template <int EPI>
__device__ __forceinline__ EpiAuxRegs epi_load_aux(const NTArgs& p, const EpiCtx<EPI>& x, int m, int n) {
  EpiAuxRegs r;
  const bool ok = m < p.M;
  if constexpr (EPI == EPI_F32_RESID) {
    const unsigned off = ok ? (unsigned)(m * p.ldaux + n) * 4u : ES_OOB;
    r.a0 = buf_load16(x.aux, off);
    r.a1 = buf_load16(x.aux, off + 16);
  } else if constexpr (EPI == EPI_PATCH) {
    const int pi = m - (m / p.np) * p.np;
    const unsigned off = ok ? (unsigned)((1 + pi) * p.ldaux + n) * 4u : ES_OOB;
    r.a0 = buf_load16(x.aux, off);
    r.a1 = buf_load16(x.aux, off + 16);
  } else if constexpr (EPI == EPI_DGELU || EPI == EPI_MULAUX) {
    r.a0 = buf_load16(x.aux, ok ? (unsigned)(m * p.ldaux + n) * 2u : ES_OOB);
  }
  return r;
}

__device__ __forceinline__ u32x4 pack_bf16x8(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
  return __builtin_bit_cast(u32x4, o);
}

// 8 consecutive outputs C[m][n .. n+7]: v0, v1 = accumulator + bias.
template <int EPI, int STAUX = 0>
__device__ __forceinline__ void epi_store8(const NTArgs& p, const EpiCtx<EPI>& x, int m, int n, f32x4 v0, f32x4 v1,
                                           const EpiAuxRegs& a) {
  auto buf_store16 = [](u32x4 v, __amdgpu_buffer_rsrc_t r, unsigned off) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, STAUX);
  };
  const bool ok = m < p.M;
  int crow = m;
  if constexpr (EPI == EPI_PATCH) {
    const int img = m / p.np;
    crow = img * (p.np + 1) + 1 + (m - img * p.np);
  }
  const unsigned off = ok ? (unsigned)(crow * p.ldc + n) * (unsigned)x.esz : ES_OOB;
  float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  if constexpr (EPI == EPI_BF16) {
    buf_store16(pack_bf16x8(v), x.c, off);
  } else if constexpr (EPI == EPI_GELU_D) {
    float g[8], d[8];
    gelu_and_grad_f8(v, g, d);
    buf_store16(pack_bf16x8(d), x.c, off);
    buf_store16(pack_bf16x8(g), x.c2, off);
  } else if constexpr (EPI == EPI_MULAUX) {
    const bf16x8 gp = __builtin_bit_cast(bf16x8, a.a0);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = v[i] * (float)gp[i];
    buf_store16(pack_bf16x8(o), x.c, off);
  } else if constexpr (EPI == EPI_GELU || EPI == EPI_GELU_ACT) {
    float g[8], d[8];  // d unused: its two ops are dead code
    gelu_and_grad_f8(v, g, d);
    if constexpr (EPI == EPI_GELU) {
      buf_store16(pack_bf16x8(v), x.c, off);
      buf_store16(pack_bf16x8(g), x.c2, off);
    } else {
      buf_store16(pack_bf16x8(g), x.c, off);
    }
  } else if constexpr (EPI == EPI_F32_RESID || EPI == EPI_PATCH) {
    buf_store16(__builtin_bit_cast(u32x4, v0 + __builtin_bit_cast(f32x4, a.a0)), x.c, off);
    buf_store16(__builtin_bit_cast(u32x4, v1 + __builtin_bit_cast(f32x4, a.a1)), x.c, off + 16);
  } else if constexpr (EPI == EPI_DGELU) {
    const bf16x8 pre = __builtin_bit_cast(bf16x8, a.a0);
    float o[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = v[i] * gelu_grad_f((float)pre[i]);
    buf_store16(pack_bf16x8(o), x.c, off);
  } else if constexpr (EPI == EPI_F32) {
    buf_store16(__builtin_bit_cast(u32x4, v0), x.c, off);
    buf_store16(__builtin_bit_cast(u32x4, v1), x.c, off + 16);
  }
}

// Per-lane epilogue operands that do not depend on the accumulators -- segment coordinates, the bias
// of the lane's columns and the first row chunk's aux (residual / GELU' / position rows) -- loaded
// by epi_prefetch at kernel start, so their HBM latency hides behind the K loop.
template <int EPI, int NF>
struct EpiPre {
  static constexpr int SEGR = NF * 2, SEGS = 16 * SEGR, IT = (SEGS + 63) / 64;
  int srow[IT], scol[IT];
  f32x4 b0[IT], b1[IT];
  EpiAuxRegs aux0[IT];
};

template <int EPI, int NF>
__device__ __forceinline__ EpiPre<EPI, NF> epi_prefetch(const NTArgs& p, int mw0, int nw0, int lane) {
  using E = EpiPre<EPI, NF>;
  constexpr bool kAux = (EPI == EPI_F32_RESID || EPI == EPI_PATCH || EPI == EPI_DGELU || EPI == EPI_MULAUX);
  E e;
  const EpiCtx<EPI> x = epi_ctx<EPI>(p);
#pragma unroll
  for (int it = 0; it < E::IT; ++it) {
    const int sg = it * 64 + lane;
    const bool valid = (E::SEGS % 64 == 0) || sg < E::SEGS;
    e.srow[it] = valid ? sg / E::SEGR : (1 << 20);  // an invalid segment lands past M: dropped
    e.scol[it] = valid ? (sg % E::SEGR) * 8 : 0;
    e.b0[it] = f32x4{0.f, 0.f, 0.f, 0.f};
    e.b1[it] = e.b0[it];
    if (p.bias) {
      e.b0[it] = *(const f32x4*)(p.bias + nw0 + e.scol[it]);
      e.b1[it] = *(const f32x4*)(p.bias + nw0 + e.scol[it] + 4);
    }
    if constexpr (kAux) e.aux0[it] = epi_load_aux<EPI>(p, x, mw0 + e.srow[it], nw0 + e.scol[it]);
  }
  return e;
}

// A wave's (MF*16) x (NF*16) fp32 accumulator tile goes through its private LDS region 16 rows
// at a time (rows padded by 16 B so each 16-row ds_write_b128 is conflict-free), read back as
// 8-column row segments (2 x ds_read_b128) and stored with 16-B accesses (each wave store
// instruction covers whole row segments).  Row chunk mi + 1's aux is loaded during chunk mi.
template <int NF>
__host__ __device__ constexpr int epi_wave_bytes() { return 16 * (NF * 64 + 16); }
constexpr int EPI_WAVE_BYTES = epi_wave_bytes<4>();  // 4352

template <int EPI, int MF, int NF, int STAUX = 0>
__device__ __forceinline__ void staged_epilogue_g(const NTArgs& p, char* wlds, const f32x4 (&acc)[MF][NF], int mw0,
                                                  int nw0, int lane, const EpiPre<EPI, NF>& e) {
  using E = EpiPre<EPI, NF>;
  constexpr int ROWB = NF * 64 + 16;
  constexpr int IT = E::IT;
  constexpr bool kAux = (EPI == EPI_F32_RESID || EPI == EPI_PATCH || EPI == EPI_DGELU || EPI == EPI_MULAUX);
  const int g = lane >> 4, r = lane & 15;
  const EpiCtx<EPI> x = epi_ctx<EPI>(p);
  EpiAuxRegs aux[2][IT];
  if constexpr (kAux) {
#pragma unroll
    for (int it = 0; it < IT; ++it) aux[0][it] = e.aux0[it];
  }
#pragma unroll
  for (int mi = 0; mi < MF; ++mi) {
#pragma unroll
    for (int ni = 0; ni < NF; ++ni) *(f32x4*)(wlds + r * ROWB + (ni * 16 + 4 * g) * 4) = acc[mi][ni];
    __builtin_amdgcn_wave_barrier();
    f32x4 v[IT][2];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int rr = min(e.srow[it], 15);
      v[it][0] = *(const f32x4*)(wlds + rr * ROWB + e.scol[it] * 4);
      v[it][1] = *(const f32x4*)(wlds + rr * ROWB + e.scol[it] * 4 + 16);
    }
    __builtin_amdgcn_wave_barrier();
    if constexpr (kAux) {
      if (mi + 1 < MF) {
#pragma unroll
        for (int it = 0; it < IT; ++it)
          aux[(mi + 1) & 1][it] = epi_load_aux<EPI>(p, x, mw0 + (mi + 1) * 16 + e.srow[it], nw0 + e.scol[it]);
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it)
      epi_store8<EPI, STAUX>(p, x, mw0 + mi * 16 + e.srow[it], nw0 + e.scol[it], v[it][0] + e.b0[it],
                             v[it][1] + e.b1[it], aux[mi & 1][it]);
  }
}

// chunk swizzle for a BKT-deep K step: 128-B rows (BKT 64) or 64-B rows (BKT 32)
template <int BKT>
__device__ __forceinline__ int swzk(int r, int c) {
  if constexpr (BKT == 64) return c ^ ((r >> 1) & 7);
  else return swz64(r, c);
}

// vmcnt immediates must be literals: counted waits for the stage pipelines below.
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
#define ES_VMC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    ES_VMC(1) ES_VMC(2) ES_VMC(3) ES_VMC(4) ES_VMC(5) ES_VMC(6) ES_VMC(7) ES_VMC(8) ES_VMC(9) ES_VMC(10)
    ES_VMC(12) ES_VMC(15) ES_VMC(16) ES_VMC(18) ES_VMC(20) ES_VMC(24)
#undef ES_VMC
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// v2: 256x128 output tile, 8 waves (4 M x 2 N, 64x64 each), 3-stage LDS ring (48 KiB per stage,
// 144 KiB total: one workgroup per CU).  Stage k+2 is issued right after the barrier that
// publishes stage k, so two stages stay in flight behind the MFMAs; the wait for stage k is a
// COUNTED vmcnt (6 = the younger stage's glds) and the barrier is a raw s_barrier, never
// __syncthreads() (which would drain every glds -- cdna_hip_programming.md §5).
constexpr int BM2 = 256;
constexpr int STAGE2 = (BM2 + BN) * BK * 2;  // 49152 B

template <int EPI>
__global__ __launch_bounds__(512, 1) void gemm_nt256_kernel(NTArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntn = p.N / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * BM2, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int g = lane >> 4, r = lane & 15;

  const EpiPre<EPI, 4> epre = epi_prefetch<EPI, 4>(p, m0 + wm * 64, n0 + wn * 64, lane);

  const bf16* ga[4];
  const bf16* gb[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = (w * 4 + j) * 8 + (lane >> 3);
    ga[j] = p.A + (size_t)(m0 + row) * p.lda + swz128(row, lane & 7) * 8;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = (w * 2 + j) * 8 + (lane >> 3);
    gb[j] = p.B + (size_t)(n0 + row) * p.ldb + swz128(row, lane & 7) * 8;
  }
  auto issue = [&](int buf, int k0) {
    char* As = smem + buf * STAGE2;
    char* Bs = As + BM2 * BK * 2;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      __builtin_amdgcn_global_load_lds(ga[j] + k0, LDS_PTR(As + (w * 4 + j) * 1024), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds(gb[j] + k0, LDS_PTR(Bs + (w * 2 + j) * 1024), 16, 0, 0);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BK;
  issue(0, 0);
  if (nk > 1) issue(1, BK);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(buf == 0 ? 2 : buf - 1, (kt + 2) * BK);
    const char* As = smem + buf * STAGE2;
    const char* Bs = As + BM2 * BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ra = wm * 64 + i * 16 + r;
        af[i] = *(const bf16x8*)(As + ra * 128 + swz128(ra, kk * 4 + g) * 16);
        const int rb = wn * 64 + i * 16 + r;
        bfr[i] = *(const bf16x8*)(Bs + rb * 128 + swz128(rb, kk * 4 + g) * 16);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(bfr[ni], af[mi], acc[mi][ni]);
      __builtin_amdgcn_s_setprio(0);
    }
    buf = buf == 2 ? 0 : buf + 1;
  }

  __builtin_amdgcn_s_barrier();
  staged_epilogue_g<EPI, 4, 4, 2>(p, smem + w * EPI_WAVE_BYTES, acc, m0 + wm * 64, n0 + wn * 64, lane, epre);
}


// Big-tile family: (WM*MF*16) x ((8/WM)*NF*16) output tile, 8 waves (WM along M), one
// workgroup per CU.  K step BKT (32: 64-B LDS rows, swz64; 64: 128-B rows, swz128), NST-stage
// glds ring: stage k+NST-1 is issued right after the barrier that publishes stage k, so NST-1
// stages stay in flight ACROSS the barriers (counted vmcnt, raw s_barrier --
// cdna_hip_programming.md §5 T3/T4).  128-row wave tiles (WM=2) read 12 KiB of LDS per 32 MFMAs
// instead of 16 KiB for 64x64 tiles.  With BKT = 32 the B tile may need a half glds instruction
// per wave (BN = 192: 24 rows per wave); the instruction count per wave stays uniform so the
// vmcnt arithmetic holds for every wave.
// OCC: waves per SIMD the register budget is sized for (launch_bounds' second argument; 4: <= 128
// VGPRs, so two 8-wave workgroups share a CU and one's epilogue runs beside the other's main loop).
// PROBE (measurement variants 13..15 only): 1 = operand stream alone, 2 = MFMAs alone (no DMA),
// 3 = no epilogue (main loop only), 4 = operand stream alone without the epilogue, 5 = epilogue alone;
// 0 = the kernel.
// STAUX: cache-policy bits of the epilogue's C stores (0 plain, 2 nt, 16 sc1).  nt by default in every NT
// family: isolated at the F1 shapes (r03, scripts/gemm_bench.py) the qkv forward 138 -> 122.5 us, proj
// forward 92.6 -> 78.7, fc1 forward 254 -> 195 (256x128 tile), qkv data gradient 131 -> 107 (128x128 BK64);
// sc1 (write-through, dropped from L2) was slower than plain.
template <int EPI, int WM, int MF, int NF, int NST, int BKT, int OCC = 1, int PROBE = 0, int STAUX = 2>
__global__ __launch_bounds__(512, OCC) void gemm_nt_big_kernel(NTArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int WN = 8 / WM;
  constexpr int TBM = WM * MF * 16, TBN = WN * NF * 16;
  constexpr int ROWB = BKT * 2, RPI = 1024 / ROWB, CPR = ROWB / 16;  // row bytes, rows / chunks per glds
  constexpr int RPW = 8 * RPI;                   // rows per round of 8 waves
  constexpr int IA = TBM / RPW;                  // full glds per wave for A
  constexpr int IBF = TBN / RPW;                 // full glds per wave for B
  constexpr int IBH = (TBN % RPW) ? 1 : 0;       // plus one half (RPI/2 rows, lanes 0..31)
  static_assert(TBM % RPW == 0 && (TBN % RPW == 0 || TBN % RPW == RPW / 2), "tile");
  static_assert(BKT == 32 || BKT == 64, "K step");
  constexpr int PER = IA + IBF + IBH;
  constexpr int TA = TBM * ROWB, STAGE = (TBM + TBN) * ROWB;
  const int ntn = p.N / TBN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * TBM, n0 = (wg % ntn) * TBN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WN, wn = w % WN;
  const int g = lane >> 4, r = lane & 15;

  // bias / first aux chunk prefetched at kernel start (one workgroup per CU: nothing else hides their
  // latency); at two per CU they are loaded after the K loop instead, keeping 32 registers out of it
  EpiPre<EPI, NF> epre;
  if constexpr (OCC < 4) epre = epi_prefetch<EPI, NF>(p, m0 + wm * MF * 16, n0 + wn * NF * 16, lane);

  const bf16* ga[IA];
  const bf16* gb[IBF + IBH];
  int da[IA], db[IBF + IBH];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = (j * 8 + w) * RPI + lane / CPR;
    ga[j] = p.A + (size_t)(m0 + row) * p.lda + swzk<BKT>(row, lane % CPR) * 8;
    da[j] = (j * 8 + w) * 1024;
  }
#pragma unroll
  for (int j = 0; j < IBF; ++j) {
    const int row = (j * 8 + w) * RPI + lane / CPR;
    gb[j] = p.B + (size_t)(n0 + row) * p.ldb + swzk<BKT>(row, lane % CPR) * 8;
    db[j] = TA + (j * 8 + w) * 1024;
  }
  if constexpr (IBH) {
    const int row = IBF * RPW + w * (RPI / 2) + (lane & 31) / CPR;
    gb[IBF] = p.B + (size_t)(n0 + row) * p.ldb + swzk<BKT>(row, lane % CPR) * 8;
    db[IBF] = TA + IBF * RPW * ROWB + w * 512;
  }
#define BIG_ISSUE(BUF, K0)                                                        \
  {                                                                               \
    char* S_ = smem + (BUF) * STAGE;                                              \
    if constexpr (PROBE != 2 && PROBE != 5) {                                     \
    _Pragma("unroll") for (int j = 0; j < IA; ++j) glds16(ga[j] + (K0), S_ + da[j]); \
    _Pragma("unroll") for (int j = 0; j < IBF; ++j) glds16(gb[j] + (K0), S_ + db[j]); \
    if constexpr (IBH) {                                                          \
      if (lane < 32) glds16(gb[IBF] + (K0), S_ + db[IBF]);                        \
    }                                                                             \
    }                                                                             \
  }

  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BKT;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) BIG_ISSUE(st, st * BKT)
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt(min(NST - 2, nk - 1 - kt) * PER);
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nk) {
      int nb = buf + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      BIG_ISSUE(nb, (kt + NST - 1) * BKT)
    }
    const char* As = smem + buf * STAGE;
    const char* Bs = As + TA;
#pragma unroll
    for (int kk = 0; kk < ((PROBE == 1 || PROBE >= 4) ? 0 : BKT / 32); ++kk) {
      bf16x8 af[MF], bfr[NF];
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int rb = wn * NF * 16 + j * 16 + r;
        bfr[j] = *(const bf16x8*)(Bs + rb * ROWB + swzk<BKT>(rb, kk * 4 + g) * 16);
      }
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int ra = wm * MF * 16 + i * 16 + r;
        af[i] = *(const bf16x8*)(As + ra * ROWB + swzk<BKT>(ra, kk * 4 + g) * 16);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
    buf = buf + 1 == NST ? 0 : buf + 1;
  }
#undef BIG_ISSUE
  if constexpr (PROBE == 3 || PROBE == 4) {
    if (acc[0][0][0] == 1.2345f) ((float*)p.C)[tid] = acc[MF - 1][NF - 1][3];  // keeps the MFMAs live
    return;
  }
  if constexpr (OCC >= 4) epre = epi_prefetch<EPI, NF>(p, m0 + wm * MF * 16, n0 + wn * NF * 16, lane);
  __builtin_amdgcn_s_barrier();
  staged_epilogue_g<EPI, MF, NF, STAUX>(p, smem + w * epi_wave_bytes<NF>(), acc, m0 + wm * MF * 16,
                                        n0 + wn * NF * 16, lane, epre);
}

// v0 family: 128x128 output tile, 4 waves (2x2, 64x64 each), K step BKT in {32, 64}, NST-stage
// LDS ring.  Stage k+NST-1 is issued right after the barrier that publishes stage k; the wait
// for stage k is a counted vmcnt (the younger stages' glds stay in flight), the barrier a raw
// s_barrier.  Small footprints (BKT=32: 16 KiB per stage) let 3-4 workgroups share a CU, so one
// tile's epilogue overlaps other tiles' MFMAs.
//   BKT=64: 128-B LDS rows, chunk c of row r at c ^ ((r>>1)&7)
//   BKT=32:  64-B LDS rows, chunk c of row r at c ^ ((-(r>>2))&3)   (both conflict-free for the
//            16-row x 16-B fragment reads under the ds_read_b128 lane groups of
//            MI355X_MICROARCH.md §LDS; the plain c ^ ((r>>2)&3) is 2-way conflicted there)

// GELU epilogues: 4 waves per SIMD (<= 128 VGPRs incl. the 64 accumulators), i.e. 4 workgroups
// per CU at the 32-KiB two-stage footprint; the packed GELU would otherwise take a few more
// registers and drop to 3 (measured slower).  The other epilogues fit without the bound.
template <int EPI>
constexpr int nt_min_waves() { return (EPI == EPI_GELU || EPI == EPI_GELU_ACT || EPI == EPI_GELU_D) ? 4 : 1; }
// TBM: output rows per workgroup -- 128 (waves 64 x 64) or 64 (waves 32 x 64: twice the workgroups for a
// rank's small token shard, where 128-row tiles leave most CUs with one tile and a few with two).
template <int EPI, int BKT, int NST, int TBM = 128, int STAUX = 2>
__global__ __launch_bounds__(256, nt_min_waves<EPI>()) void gemm_nt_kernel(NTArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ROWB = BKT * 2;              // bytes per LDS row
  constexpr int RPI = 1024 / ROWB;           // rows per 1-KiB glds instruction
  constexpr int CPR = ROWB / 16;             // 16-B chunks per row
  constexpr int MF = TBM / 32;               // A fragments per wave (wave tile TBM/2 x 64)
  constexpr int IPA = (TBM / RPI) / 4;       // glds instructions per wave per stage: A operand
  constexpr int IPB = (BN / RPI) / 4;        //                                     B operand
  constexpr int PER = IPA + IPB;             // per stage per wave
  constexpr int TILEA = TBM * ROWB;          // bytes of the A tile
  constexpr int STAGE = TILEA + BN * ROWB;
  static_assert(IPA >= 1 && IPB >= 1, "tile");
  const int ntn = p.N / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (wg / ntn) * TBM, n0 = (wg % ntn) * BN;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int g = lane >> 4, r = lane & 15;

  const EpiPre<EPI, 4> epre = epi_prefetch<EPI, 4>(p, m0 + wm * (TBM / 2), n0 + wn * 64, lane);

  const bf16* ga[IPA];
  const bf16* gb[IPB];
#pragma unroll
  for (int j = 0; j < IPA; ++j) {
    const int row = (w * IPA + j) * RPI + lane / CPR;
    ga[j] = p.A + (size_t)(m0 + row) * p.lda + swzk<BKT>(row, lane % CPR) * 8;
  }
#pragma unroll
  for (int j = 0; j < IPB; ++j) {
    const int row = (w * IPB + j) * RPI + lane / CPR;
    gb[j] = p.B + (size_t)(n0 + row) * p.ldb + swzk<BKT>(row, lane % CPR) * 8;
  }
#define NT_ISSUE(BUF, K0)                                                                           \
  {                                                                                                 \
    char* As_ = smem + (BUF) * STAGE;                                                               \
    _Pragma("unroll") for (int j = 0; j < IPA; ++j) glds16(ga[j] + (K0), As_ + (w * IPA + j) * 1024); \
    _Pragma("unroll") for (int j = 0; j < IPB; ++j) glds16(gb[j] + (K0), As_ + TILEA + (w * IPB + j) * 1024); \
  }

  f32x4 acc[MF][4];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = p.K / BKT;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) NT_ISSUE(st, st * BKT)
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int younger = min(NST - 2, nk - 1 - kt);
    wait_vmcnt(younger * PER);
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nk) {
      int nb = buf + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      NT_ISSUE(nb, (kt + NST - 1) * BKT)
    }
    const char* As = smem + buf * STAGE;
    const char* Bs = As + TILEA;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 af[MF], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < MF) {
          const int ra = wm * (TBM / 2) + i * 16 + r;
          af[i] = *(const bf16x8*)(As + ra * ROWB + swzk<BKT>(ra, kk * 4 + g) * 16);
        }
        const int rb = wn * 64 + i * 16 + r;
        bfr[i] = *(const bf16x8*)(Bs + rb * ROWB + swzk<BKT>(rb, kk * 4 + g) * 16);
      }
#pragma unroll
      for (int mi = 0; mi < MF; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(bfr[ni], af[mi], acc[mi][ni]);
    }
    buf = buf + 1 == NST ? 0 : buf + 1;
  }

  // ---- epilogue through LDS (stage buffers are free once every wave passed the last MFMA) ----
  __builtin_amdgcn_s_barrier();
  staged_epilogue_g<EPI, MF, 4, STAUX>(p, smem + w * EPI_WAVE_BYTES, acc, m0 + wm * (TBM / 2), n0 + wn * 64, lane,
                                       epre);
}
#undef NT_ISSUE

// ---------------------------------------------------------------------------------------------
// TN (wgrad): 256-byte LDS rows (128 bf16 of the N1 / N2 axis), read with ds_read_b64_tr_b16.
// Chunk c of row r stored at c ^ f(r), f(r) = ((r&3)<<1) | (((r>>3)&1)<<3): the 8 rows x 32 B that
// one 32-lane half of a transposed read touches land on 16 distinct bank slots.
__device__ __forceinline__ int swz256(int r, int c) { return c ^ (((r & 3) << 1) | (((r >> 3) & 1) << 3)); }

struct TNArgs {
  const bf16* A1; const bf16* A2; float* P; float* PB;
  int M, N1, N2, ld1, ld2, mchunk;
};

// BKM-deep token steps (32 or 64), NST-stage glds ring (asm DMA: glds16_asm, retired by the counted
// vmcnt + barrier at the top of each step), counted vmcnt.  With PB != null the
// workgroups of the first N2 tile also sum their A1 (= dY) tile columns from LDS: the bias
// gradient of the same Linear, written as per-split partials PB[split][N1].
template <int BKM, int NST>
__device__ __forceinline__ void gemm_tn_body(const TNArgs& p, int split, int tile, char* smem) {
  constexpr int IPW = (BKM / 4) / 4;    // 1-KiB glds (4 rows of 256 B) per wave per operand per stage
  constexpr int PER = 2 * IPW;
  constexpr int TILE = BKM * BM * 2;     // bytes per operand tile
  constexpr int STAGE = 2 * TILE;
  const int nt2 = p.N2 / BN;
  const int n1_0 = (tile / nt2) * BM, n2_0 = (tile % nt2) * BN;
  const bool do_bias = p.PB != nullptr && (tile % nt2) == 0;
  const int mbeg = split * p.mchunk;
  const int mend = min(mbeg + p.mchunk, (p.M + BKM - 1) / BKM * BKM);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wa = w >> 1, wb = w & 1;
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p4 = t & 3;

  const bf16* g1[IPW];
  const bf16* g2[IPW];
#pragma unroll
  for (int j = 0; j < IPW; ++j) {
    const int row = (w * IPW + j) * 4 + (lane >> 4);
    const int lc = swz256(row, lane & 15);
    g1[j] = p.A1 + (size_t)(mbeg + row) * p.ld1 + n1_0 + lc * 8;
    g2[j] = p.A2 + (size_t)(mbeg + row) * p.ld2 + n2_0 + lc * 8;
  }
#define TN_ISSUE(BUF, MO)                                                        \
  {                                                                              \
    char* T1_ = smem + (BUF) * STAGE;                                            \
    _Pragma("unroll") for (int j = 0; j < IPW; ++j) {                            \
      glds16_asm(g1[j] + (size_t)(MO) * p.ld1, T1_ + (w * IPW + j) * 1024);      \
      glds16_asm(g2[j] + (size_t)(MO) * p.ld2, T1_ + TILE + (w * IPW + j) * 1024); \
    }                                                                            \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;
  const int bc = tid & 127, bh = tid >> 7;  // bias: column, row half

  const int nk = (mend - mbeg) / BKM;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) TN_ISSUE(st, st * BKM)
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const int younger = min(NST - 2, nk - 1 - kt);
    wait_vmcnt(younger * PER);
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nk) {
      int nb = buf + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      TN_ISSUE(nb, (kt + NST - 1) * BKM)
    }
    const char* T1 = smem + buf * STAGE;
    const char* T2 = T1 + TILE;
#pragma unroll
    for (int hh = 0; hh < BKM / 32; ++hh) {
      bf16x8 af[4], bfr[4];
      const int r1 = hh * 32 + 8 * g + q, r2 = r1 + 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ca = (wa * 64 + i * 16) / 8 + (p4 >> 1);
        const int off = (p4 & 1) * 8;
        af[i] = cat8(lds_tr4(T2 + r1 * 256 + swz256(r1, ca) * 16 + off),
                     lds_tr4(T2 + r2 * 256 + swz256(r2, ca) * 16 + off));
        const int cb = (wb * 64 + i * 16) / 8 + (p4 >> 1);
        bfr[i] = cat8(lds_tr4(T1 + r1 * 256 + swz256(r1, cb) * 16 + off),
                      lds_tr4(T1 + r2 * 256 + swz256(r2, cb) * 16 + off));
      }
#pragma unroll
      for (int ai = 0; ai < 4; ++ai)
#pragma unroll
        for (int bi = 0; bi < 4; ++bi) acc[ai][bi] = mfma16(af[ai], bfr[bi], acc[ai][bi]);
    }
    if (do_bias) {
#pragma unroll 8
      for (int rr = bh * (BKM / 2); rr < (bh + 1) * (BKM / 2); ++rr)
        bsum += (float)*(const bf16*)(T1 + rr * 256 + swz256(rr, bc >> 3) * 16 + (bc & 7) * 2);
    }
    buf = buf + 1 == NST ? 0 : buf + 1;
  }
#undef TN_ISSUE

  // lane holds D[n2 = .. + 4g + i][n1 = .. + t]  ->  P[split][n1][n2 .. n2+3]
  float* P = p.P + (size_t)split * p.N1 * p.N2;
#pragma unroll
  for (int bi = 0; bi < 4; ++bi) {
    const int n1 = n1_0 + wb * 64 + bi * 16 + t;
#pragma unroll
    for (int ai = 0; ai < 4; ++ai) {
      const int n2 = n2_0 + wa * 64 + ai * 16 + 4 * g;
      *(f32x4*)(P + (size_t)n1 * p.N2 + n2) = acc[ai][bi];
    }
  }
  if (do_bias) {
    __builtin_amdgcn_s_barrier();
    float* red = (float*)smem;
    if (bh == 1) red[bc] = bsum;
    __syncthreads();
    if (bh == 0) p.PB[(size_t)split * p.N1 + n1_0 + bc] = bsum + red[bc];
  }
}

template <int BKM, int NST>
__global__ __launch_bounds__(256) void gemm_tn_kernel(TNArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntiles = (p.N1 / BM) * (p.N2 / BN);
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles;
  gemm_tn_body<BKM, NST>(p, split, wg - split * ntiles, smem);
}

// Grouped weight gradients: one launch over many independent TN problems, each tile over its
// problem's whole token axis (no split-K: no fp32 slabs, no reduction launches).  Entry g's tiles
// are the global tile indices [tile0_g, tile0_g + tiles_g); entries sorted by tile0.
struct TNGroupEntry {
  TNArgs a;
  int tile0, pad;
};
template <int BKM, int NST>
__global__ __launch_bounds__(256) void gemm_tn_grouped_kernel(const TNGroupEntry* __restrict__ grp, int ng) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int e = 0;
  while (e + 1 < ng && grp[e + 1].tile0 <= wg) ++e;
  const TNArgs a = grp[e].a;
  gemm_tn_body<BKM, NST>(a, 0, wg - grp[e].tile0, smem);
}

// ---- weight gradient on a 384 x 192 output tile (N1 x N2) per 8-wave workgroup -----------------
// The 128x128 kernel above brings 16 KiB into LDS per 32-token step for 1 MFLOP: at 64 FLOP/B the
// L2 -> LDS stream, not the matrix cores, sets its pace (rocprofv3: 63 % of wave cycles parked in
// s_waitcnt, no LDS bank conflicts).  Here a workgroup owns a 384 (N1, from A1 = dY) x 192 (N2,
// from A2 = X) tile -- 128 FLOP/B -- as 8 waves of 96 x 96 (4 along N1 x 2 along N2), each 6 x 6
// v_mfma_f32_16x16x32_bf16 per 32 tokens from 12 A2 + 12 A1 transposed fragment reads (0.67
// ds_read_b64_tr_b16 per MFMA, was 1.0).  Every ViT-S / ViT-B Linear satisfies N1 % 384 == 0 and
// N2 % 192 == 0.  Operand rows are 768 B (A1) and 384 B (A2) of 16-B chunks, written by LDS-DMA
// pieces that cross rows; conflict-free transposed reads via source-side XOR swizzles:
//   A1 (row stride = 0 mod 64 banks): chunk c of row r at c ^ (((r & 3) << 1) | (((r >> 3) & 1) << 3))
//   A2 (row stride = 32 mod 64 banks: odd rows shift by half the banks):
//                                     chunk c of row r at c ^ ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2))
// The bias gradient (column sums of A1) rides on the matrix cores: the N2-tile-0 workgroups' w2 = 0
// waves issue one extra MFMA per A1 fragment against an all-ones A operand.
constexpr int TB1 = 384, TB2 = 192;
__device__ __forceinline__ int swz384(int r, int c) { return c ^ ((((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2)); }

// PROBE (measurement variants only, es_gemm_tn_ex 10..13): 1 = the operand stream alone (no transposed
// reads, no MFMAs), 2 = the MFMAs alone on whatever the ring holds (no DMA); 0 = the kernel.
template <int BKM, int NST, bool ASM = true, int PROBE = 0>
__device__ __forceinline__ void tn_big_body(const TNArgs& p, int split, int tile, char* smem) {
  constexpr int R1B = TB1 * 2, R2B = TB2 * 2;          // LDS row bytes: 768, 384
  constexpr int C1 = R1B / 16, C2 = R2B / 16;           // 16-B chunks per row: 48, 24
  constexpr int T1B = BKM * R1B, T2B = BKM * R2B;
  constexpr int STAGE = T1B + T2B;
  constexpr int F1 = T1B / 1024 / 8;                    // full 1-KiB pieces per wave, A1
  constexpr int F2 = T2B / 1024 / 8;                    // ... A2
  constexpr int H2 = ((T2B / 1024) % 8) ? 1 : 0;        // plus one half piece (lanes 0..31)
  static_assert((T1B / 1024) % 8 == 0 && ((T2B / 1024) % 8 == 0 || (T2B / 1024) % 8 == 4), "pieces");
  constexpr int PER = F1 + F2 + H2;
  const int nt2 = p.N2 / TB2;
  const int n1_0 = (tile / nt2) * TB1, n2_0 = (tile % nt2) * TB2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int w1 = w >> 1, w2 = w & 1;
  // the bias gradient's 6 extra MFMAs per A1 fragment row are split between the two w2 waves (3 each), so
  // every SIMD of a bias workgroup carries the same MFMA count (waves 0, 2, 4, 6 sit on SIMDs 0 / 1 and
  // 1, 3, 5, 7 on SIMDs 2 / 3: with the bias on the w2 = 0 waves alone two SIMDs ran 84 MFMAs per 32
  // tokens against 72)
  const bool do_bias = p.PB != nullptr && (tile % nt2) == 0;
  const int mbeg = split * p.mchunk;
  const int mend = min(mbeg + p.mchunk, (p.M + BKM - 1) / BKM * BKM);
  const int g = lane >> 4, t = lane & 15, q = t >> 2, p4 = t & 3;

  // per-lane byte offsets of the DMA sources within one token step (row-major tile, swizzled chunk)
  unsigned o1[F1], o2[F2 + H2];
#pragma unroll
  for (int j = 0; j < F1; ++j) {
    const int L = (j * 8 + w) * 64 + lane, row = L / C1;
    o1[j] = (unsigned)row * p.ld1 * 2u + (unsigned)swz256(row, L - row * C1) * 16u;
  }
#pragma unroll
  for (int j = 0; j < F2 + H2; ++j) {
    const int L = j < F2 ? (j * 8 + w) * 64 + lane : F2 * 512 + w * 32 + (lane & 31), row = L / C2;
    o2[j] = (unsigned)row * p.ld2 * 2u + (unsigned)swz384(row, L - row * C2) * 16u;
  }
  const char* b1 = (const char*)(p.A1 + (size_t)mbeg * p.ld1 + n1_0);
  const char* b2 = (const char*)(p.A2 + (size_t)mbeg * p.ld2 + n2_0);
  const size_t s1 = (size_t)BKM * p.ld1 * 2, s2 = (size_t)BKM * p.ld2 * 2;
#define TNB_ISSUE(BUF, KT)                                                                       \
  {                                                                                              \
    char* S_ = smem + (BUF) * STAGE;                                                             \
    const char* x1 = b1 + (size_t)(KT) * s1;                                                     \
    const char* x2 = b2 + (size_t)(KT) * s2;                                                     \
    if constexpr (PROBE != 2) {                                                                  \
    _Pragma("unroll") for (int j = 0; j < F1; ++j) GLDS(x1 + o1[j], S_ + (j * 8 + w) * 1024);  \
    _Pragma("unroll") for (int j = 0; j < F2; ++j) GLDS(x2 + o2[j], S_ + T1B + (j * 8 + w) * 1024); \
    if constexpr (H2) {                                                                          \
      if (lane < 32) GLDS(x2 + o2[F2], S_ + T1B + F2 * 8192 + w * 512);                          \
    }                                                                                            \
    }                                                                                            \
  }

  // ASM: the ring's DMA as inline asm (glds16_asm), so the transposed reads of the current stage are
  // not preceded by a compiler drain of the next stage's DMA; retired by the counted waits below
  auto GLDS = [](const char* src, char* dst) {
    if constexpr (ASM) glds16_asm(src, dst);
    else glds16(src, dst);
  };
  f32x4 acc[6][6], bacc[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) bacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;

  const int nk = (mend - mbeg) / BKM;
#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) TNB_ISSUE(st, st)
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    wait_vmcnt(min(NST - 2, nk - 1 - kt) * PER);
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nk) {
      int nb = buf + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      TNB_ISSUE(nb, kt + NST - 1)
    }
    const char* T1 = smem + buf * STAGE;
    const char* T2 = T1 + T1B;
#pragma unroll
    for (int hh = 0; hh < (PROBE == 1 ? 0 : BKM / 32); ++hh) {
      const int r1 = hh * 32 + 8 * g + q, r2 = r1 + 4;
      const int off = (p4 & 1) * 8;
      bf16x8 bfr[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        const int cb = (w1 * 96 + i * 16) / 8 + (p4 >> 1);
        bfr[i] = cat8(lds_tr4(T1 + r1 * R1B + swz256(r1, cb) * 16 + off),
                      lds_tr4(T1 + r2 * R1B + swz256(r2, cb) * 16 + off));
      }
      if (do_bias) {
        if (w2 == 0) {
#pragma unroll
          for (int i = 0; i < 3; ++i) bacc[i] = mfma16(ones, bfr[i], bacc[i]);
        } else {
#pragma unroll
          for (int i = 0; i < 3; ++i) bacc[i] = mfma16(ones, bfr[3 + i], bacc[i]);
        }
      }
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        const int ca = (w2 * 96 + a * 16) / 8 + (p4 >> 1);
        const bf16x8 af = cat8(lds_tr4(T2 + r1 * R2B + swz384(r1, ca) * 16 + off),
                               lds_tr4(T2 + r2 * R2B + swz384(r2, ca) * 16 + off));
#pragma unroll
        for (int i = 0; i < 6; ++i) acc[a][i] = mfma16(af, bfr[i], acc[a][i]);
      }
    }
    buf = buf + 1 == NST ? 0 : buf + 1;
  }
#undef TNB_ISSUE
  // lane holds D[n2 = .. + 4g + e][n1 = .. + t]  ->  P[split][n1][n2 .. n2+3]
  float* P = p.P + (size_t)split * p.N1 * p.N2;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int n1 = n1_0 + w1 * 96 + i * 16 + t;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      const int n2 = n2_0 + w2 * 96 + a * 16 + 4 * g;
      *(f32x4*)(P + (size_t)n1 * p.N2 + n2) = acc[a][i];
    }
  }
  if (do_bias && g == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p.PB[(size_t)split * p.N1 + n1_0 + w1 * 96 + (w2 * 3 + i) * 16 + t] = bacc[i][0];
  }
}

template <int BKM, int NST, bool ASM = true, int PROBE = 0>
__global__ __launch_bounds__(512, 1) void gemm_tn_big_kernel(TNArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ntiles = (p.N1 / TB1) * (p.N2 / TB2);
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int split = wg / ntiles;
  tn_big_body<BKM, NST, ASM, PROBE>(p, split, wg - split * ntiles, smem);
}

// ---- a Linear layer's weight gradients as ONE split-K launch on the 384 x 192 tile ----------------
// Entry e owns the workgroups [wg0_e, wg0_e + splits_e * ntiles_e), split-major (the tiles of one token
// range are consecutive, so xcd_remap puts them on one XCD and they share that range's dY / X rows in its
// L2).  Every tile of every entry is the same 384 x 192 output over the same number of tokens per split,
// so the workgroups carry equal work; the few splits per problem that a whole layer's tiles (fc1 8 + fc2 8
// + qkv 6 + proj 2 = 24 at ViT-S) need to fill the granted CUs keep the fp32 slabs small (S x the layer's
// outputs, vs ~16-32 slabs per GEMM when each GEMM alone fills them).
struct TNBigEntry {
  TNArgs a;
  int wg0, ntiles, pad0, pad1;
};
// The table travels in the kernel arguments (no device copy to make or keep in sync: the tensors'
// pointers may change every step, and a hipGraph capture records the arguments by value).
constexpr int TNG_MAX = 8;
struct TNBigTable {
  TNBigEntry e[TNG_MAX];
  int ng, pad;
};
// 64-token steps in a two-stage ring (147 KiB of LDS).  Round 5 measured 32-token steps in four- and three-stage
// rings (bit-identical): F1 30.94 / 30.87 vs 30.73 ms, the live launch 1.02-1.03 / 1.006 vs 1.028 ms -- removed.
template <int BKM = 64, int NST = 2>
__global__ __launch_bounds__(512, 1) void gemm_tn_big_grouped_kernel(const TNBigTable t) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  int e = 0;
  while (e + 1 < t.ng && t.e[e + 1].wg0 <= wg) ++e;
  const TNArgs a = t.e[e].a;
  const int local = wg - t.e[e].wg0, nt = t.e[e].ntiles;
  const int split = local / nt;
  tn_big_body<BKM, NST, true, 0>(a, split, local - split * nt, smem);
}

// out[i] = sum_s P[s][i] for every entry of a table (the grouped launch's weight slabs and bias
// partials): block b belongs to the entry with the largest blk0 <= b and sums 1,024 of its floats with
// splitk_reduce_kernel's chains and order (4 interleaved chains over s, (s0 + s1) + (s2 + s3)).
struct TNRedEntry {
  const float* P;
  float* out;
  int S, n, blk0, pad;
};
struct TNRedTable {
  TNRedEntry r[2 * TNG_MAX];
  int nr, pad;
};
__global__ __launch_bounds__(256) void splitk_reduce_grouped_kernel(const TNRedTable t) {
  const TNRedEntry* red = t.r;
  const int nr = t.nr;
  int e = 0;
  while (e + 1 < nr && red[e + 1].blk0 <= (int)blockIdx.x) ++e;
  const float* P = red[e].P;
  const int S = red[e].S, n = red[e].n;
  const int i = ((int)blockIdx.x - red[e].blk0) * 256 + (int)threadIdx.x;
  if (i >= (n >> 2)) return;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
  int k = 0;
#pragma unroll 4
  for (; k + 4 <= S; k += 4) {
    s0 += ((const f32x4*)(P + (size_t)k * n))[i];
    s1 += ((const f32x4*)(P + (size_t)(k + 1) * n))[i];
    s2 += ((const f32x4*)(P + (size_t)(k + 2) * n))[i];
    s3 += ((const f32x4*)(P + (size_t)(k + 3) * n))[i];
  }
  for (; k < S; ++k) s0 += ((const f32x4*)(P + (size_t)k * n))[i];
  ((f32x4*)red[e].out)[i] = (s0 + s1) + (s2 + s3);
}

// out[i] = (accumulate ? out[i] : 0) + sum_s P[s][i]   (n % 4 == 0); 4 independent partial sums
// per thread keep 4 slab loads in flight.
__global__ void splitk_reduce_kernel(const float* __restrict__ P, float* __restrict__ out, int S, int n,
                                     int accumulate) {
  const int n4 = n >> 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    int k = 0;
    // unrolled: 16 slab loads in flight ahead of the four in-order accumulation chains (same sums)
#pragma unroll 4
    for (; k + 4 <= S; k += 4) {
      s0 += ((const f32x4*)(P + (size_t)k * n))[i];
      s1 += ((const f32x4*)(P + (size_t)(k + 1) * n))[i];
      s2 += ((const f32x4*)(P + (size_t)(k + 2) * n))[i];
      s3 += ((const f32x4*)(P + (size_t)(k + 3) * n))[i];
    }
    for (; k < S; ++k) s0 += ((const f32x4*)(P + (size_t)k * n))[i];
    f32x4 s = (s0 + s1) + (s2 + s3);
    if (accumulate) s += ((const f32x4*)out)[i];
    ((f32x4*)out)[i] = s;
  }
}

// Column sums of a bf16 [M, N] matrix (bias gradients), HBM-streaming: each thread owns one
// 8-column chunk (16-B loads) of a row group and keeps 4 rows in flight; per-block partials P[block][N].
__global__ __launch_bounds__(256) void colsum_partial_kernel(const bf16* __restrict__ Y, int ld, int M, int N,
                                                             int rows_per, float* __restrict__ P) {
  __shared__ float red[256 * 8];
  const int nc = N >> 3;        // 8-column chunks (<= 256)
  const int groups = 256 / nc;  // row groups per block
  const int t = threadIdx.x, c = t % nc, rg = t / nc;
  const int m0 = blockIdx.x * rows_per, m1 = min(m0 + rows_per, M);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rg < groups) {
    int m = m0 + rg;
    for (; m + 3 * groups < m1; m += 4 * groups) {
      const bf16x8 v0 = *(const bf16x8*)(Y + (size_t)m * ld + c * 8);
      const bf16x8 v1 = *(const bf16x8*)(Y + (size_t)(m + groups) * ld + c * 8);
      const bf16x8 v2 = *(const bf16x8*)(Y + (size_t)(m + 2 * groups) * ld + c * 8);
      const bf16x8 v3 = *(const bf16x8*)(Y + (size_t)(m + 3 * groups) * ld + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += ((float)v0[j] + (float)v1[j]) + ((float)v2[j] + (float)v3[j]);
    }
    for (; m < m1; m += groups) {
      const bf16x8 v = *(const bf16x8*)(Y + (size_t)m * ld + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[t * 8 + j] = acc[j];
  __syncthreads();
  for (int col = t; col < N; col += 256) {
    const int cc = col >> 3, j = col & 7;
    float sum = 0.f;
    for (int gg = 0; gg < groups; ++gg) sum += red[(gg * nc + cc) * 8 + j];
    P[(size_t)blockIdx.x * N + col] = sum;
  }
}

// out[n] (+)= sum_g P[g][n]: CW columns x (256 / CW) row-groups per block (4 loads in flight per
// thread), then a fixed-order LDS combine (deterministic).  Narrow blocks (CW = 4) for short rows so
// a 384-column reduction still spreads over ~100 workgroups.
template <int CW>
__device__ __forceinline__ void reduce_partials_body(const float* __restrict__ P, float* __restrict__ out, int G,
                                                     int N, int accumulate, int blk) {
  constexpr int RG = 256 / CW;
  __shared__ float red[RG][CW + 1];
  const int cl = threadIdx.x % CW, rg = threadIdx.x / CW;
  const int col = blk * CW + cl;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    int g = rg;
#pragma unroll 4
    for (; g + 3 * RG < G; g += 4 * RG) {
      s0 += P[(size_t)g * N + col];
      s1 += P[(size_t)(g + RG) * N + col];
      s2 += P[(size_t)(g + 2 * RG) * N + col];
      s3 += P[(size_t)(g + 3 * RG) * N + col];
    }
    for (; g < G; g += RG) s0 += P[(size_t)g * N + col];
  }
  red[rg][cl] = (s0 + s1) + (s2 + s3);
  __syncthreads();
#pragma unroll
  for (int h = RG / 2; h >= 1; h >>= 1) {
    if (rg < h) red[rg][cl] += red[rg + h][cl];
    __syncthreads();
  }
  if (rg == 0 && col < N) {
    const float sum = red[0][cl];
    out[col] = accumulate ? out[col] + sum : sum;
  }
}

template <int CW>
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ P, float* __restrict__ out,
                                                              int G, int N, int accumulate) {
  reduce_partials_body<CW>(P, out, G, N, accumulate, blockIdx.x);
}

// two independent reductions of the same shape in one launch (a LayerNorm backward's dgamma and dbeta):
// blocks [0, nb) reduce P0 -> out0, blocks [nb, 2 nb) P1 -> out1, each column as reduce_partials_kernel
template <int CW>
__global__ __launch_bounds__(256) void reduce_partials_pair_kernel(const float* __restrict__ P0, float* __restrict__ out0,
                                                                   const float* __restrict__ P1, float* __restrict__ out1,
                                                                   int G, int N, int accumulate, int nb) {
  const bool second = (int)blockIdx.x >= nb;
  reduce_partials_body<CW>(second ? P1 : P0, second ? out1 : out0, G, N, accumulate, blockIdx.x - (second ? nb : 0));
}

// launch: 4-column blocks when that still leaves <= 512 blocks, else 16-column blocks
inline void launch_reduce_partials(const float* P, float* out, int G, int N, int accumulate, hipStream_t stream) {
  if (N <= 2048 && G >= 64)
    hipLaunchKernelGGL(reduce_partials_kernel<4>, (N + 3) / 4, 256, 0, stream, P, out, G, N, accumulate);
  else
    hipLaunchKernelGGL(reduce_partials_kernel<16>, (N + 15) / 16, 256, 0, stream, P, out, G, N, accumulate);
}

// out0 (+)= sum_g P0[g], out1 (+)= sum_g P1[g] in one launch; bit-identical to two es_reduce_partials calls
int reduce_partials_pair(const float* P0, float* out0, const float* P1, float* out1, int G, int N, int accumulate,
                         hipStream_t stream) {
  if (G <= 0 || N <= 0) return ES_BAD_SHAPE;
  if (N <= 2048 && G >= 64) {
    const int nb = (N + 3) / 4;
    hipLaunchKernelGGL(reduce_partials_pair_kernel<4>, 2 * nb, 256, 0, stream, P0, out0, P1, out1, G, N, accumulate, nb);
  } else {
    const int nb = (N + 15) / 16;
    hipLaunchKernelGGL(reduce_partials_pair_kernel<16>, 2 * nb, 256, 0, stream, P0, out0, P1, out1, G, N, accumulate,
                       nb);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// many LayerNorm backwards' dgamma / dbeta reductions in one launch (es_ln_param_grads_multi): entry e owns
// blocks [blk0_e, blk0_e + 2 nb), the first nb reducing P_e -> out0_e, the next nb P_e + G N -> out1_e, every
// column as reduce_partials_kernel<CW> (bit-identical to the per-LayerNorm reduce_partials_pair launches)
struct RedPairEntry {
  const float* P;
  float *out0, *out1;
  int G, N, accumulate, blk0;
};
constexpr int RPM_MAX = 32;
struct RedPairTable {
  RedPairEntry e[RPM_MAX];
  int n, pad;
};
template <int CW>
__global__ __launch_bounds__(256) void reduce_partials_multi_kernel(const RedPairTable t) {
  int e = 0;
  while (e + 1 < t.n && t.e[e + 1].blk0 <= (int)blockIdx.x) ++e;
  const RedPairEntry& r = t.e[e];
  const int nb = (r.N + CW - 1) / CW, b = blockIdx.x - r.blk0;
  const bool second = b >= nb;
  reduce_partials_body<CW>(second ? r.P + (size_t)r.G * r.N : r.P, second ? r.out1 : r.out0, r.G, r.N, r.accumulate,
                           b - (second ? nb : 0));
}

// entries {P (= pg [G][N] then pb [G][N]), out0, out1, G, N, accumulate}: one launch; every entry must take the
// same column width as reduce_partials_pair would (N <= 2048 && G >= 64 -> 4 columns, else 16)
int reduce_partials_multi(const RedPairEntry* ents, int n, hipStream_t stream) {
  if (!ents || n <= 0) return ES_BAD_ARG;
  if (n > RPM_MAX) return ES_BAD_SHAPE;
  RedPairTable t{};
  const bool narrow = ents[0].N <= 2048 && ents[0].G >= 64;
  const int CW = narrow ? 4 : 16;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    const RedPairEntry& r = ents[i];
    if (!r.P || !r.out0 || !r.out1) return ES_BAD_ARG;
    if (r.G <= 0 || r.N <= 0 || ((r.N <= 2048 && r.G >= 64) != narrow)) return ES_BAD_SHAPE;
    t.e[i] = r;
    t.e[i].blk0 = blk;
    blk += 2 * ((r.N + CW - 1) / CW);
  }
  t.n = n;
  if (narrow) hipLaunchKernelGGL(reduce_partials_multi_kernel<4>, blk, 256, 0, stream, t);
  else hipLaunchKernelGGL(reduce_partials_multi_kernel<16>, blk, 256, 0, stream, t);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// ---------------------------------------------------------------------------------------------
// Weight-stationary NT GEMM for K = 384 (round 6, es_gemm_nt variant 12).
//
// Every tiled NT kernel above re-reads its operands from L2 into LDS once per output tile: a 256 x 128 tile at
// K = 384 moves (256 + 128) x 768 B for 32 K outputs, 9 B per output, and the K = 384 GEMMs of the ViT step
// measured their L2 -> LDS operand stream at ~14 TB/s (~23 B/clk/CU), which -- not the matrix cores -- set
// their pace.  Here one persistent 8-wave workgroup per CU owns a 384-column group of C and
// keeps that group's weight rows in REGISTERS for the whole launch: wave w holds W[n0 + 48 w .. + 48][0 .. 384)
// as the MFMA A operand (3 column fragments x 12 K fragments of v_mfma_f32_16x16x32_bf16 = 144 VGPRs).  The
// workgroup walks 32-row tiles of A; each tile is staged into LDS once by LDS-DMA (4-stage ring, 24 KiB per
// stage, source-side XOR swizzle: chunk c of row r at chunk c ^ (r & 15), conflict-free fragment reads) and
// consumed by all eight waves, so the L2 -> LDS stream carries 768 B per 384 outputs (2 B per output).
//   Accumulation: each output is the same chain of 12 MFMAs in K order, with the same operand roles (weights as
// the A operand, activations as B) as the tiled kernels, so the fp32 accumulators -- and every epilogue's
// outputs -- are bit-identical to variants 0 / 5 / 10 (tested).
//   Epilogue: straight from the MFMA layout, one 16-row block at a time, interleaved with the other block's
//   MFMAs by wave role (see the step body).  An LDS-staged epilogue (whole 768-B row stretches per store,
//   double-buffered staging tiles) was built and measured too: bit-identical, but slower (qkv forward 133.7
//   vs 122 us direct); so was the first version, a single fp32 staging tile behind a second barrier per step
//   (119-126 us).
//   Work distribution: row tiles are claimed dynamically, in chunks of 2, from per-(XCD range, column group)
//   counters (agent-scope atomics on a code-object array, one counter block per HIP stream; the last workgroup
//   to finish resets it), three chunks ahead of use.  A static split would be wrong for this engine: the
//   data-gradient GEMMs share the chip with the weight-gradient launches of the side stream (3/8 of the CUs for
//   ~1 ms), so a workgroup that only gets a CU late must find the work already taken instead of extending the
//   launch.  All ring DMA is inline asm (glds16_asm): the explicit counted vmcnt at the top of each step retires
//   it (the count follows every VMEM op this wave issued since, in issue order: claim atomics, DMA pieces, C
//   stores).
//   Measured (scripts/ws_bench.py, default rules vs variant 12, us): qkv forward 108 / 123, weak qkv 91 / 100,
//   fc1 forward 190 / 246, weak fc1 154 / 162, proj dgrad 40 / 51, fp32-out N = 384 61 / 50.  So variant 12
//   stays opt-in: per-step stamps (PROBE 7) show a wave's step ~6.4 K cycles with ~1.9 K waiting on its ring
//   stage and each MFMA half ~1 K, and a no-MFMA probe streams the same bytes in 67 us -- the chain of ring
//   wait, fragment reads and MFMAs per 32-row step, not HBM, sets the pace, and one workgroup per CU (the
//   weights fill the registers) leaves no second workgroup to cover it.
namespace wsg {
constexpr int R = 32;                      // output rows per step (one A tile)
constexpr int KD = 384;                    // reduction depth
constexpr int NG = 384;                    // output columns per workgroup (8 waves x 48)
constexpr int ROWB = KD * 2;               // A row bytes in the ring
constexpr int STAGE = R * ROWB;            // 24 KiB
constexpr int NST = 4;                     // ring stages (three tiles in flight behind the current one)
constexpr int PIECES = STAGE / 1024 / 8;   // LDS-DMA instructions per wave per stage
constexpr int CH = 2;                      // row tiles per claimed chunk
constexpr int QN = 8;                      // chunk-index ring (LDS)
constexpr int SLOTS = 64, SLOT_INTS = 64;  // counter blocks (one per stream): heads [xcd * 8 + cg], [63] done
constexpr int LDS = NST * STAGE + QN * 4 + 16 + NG * 4;  // ring, chunk ring, scratch, the column group's bias
}  // namespace wsg
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ int g_ws_ctr[wsg::SLOTS * wsg::SLOT_INTS];
// measurement build (PROBE 7): per-step s_memtime stamps of workgroup 0's waves 0 and 4 (endossl_ws_debug_stamps)
constexpr int WS_DBG = 2 * 64 * 8;
__device__ unsigned long long g_ws_dbg[WS_DBG];

// A chunk claim: one lane's returning agent-scope add (the same instruction hipcc emits for
// __hip_atomic_fetch_add(.., __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)), as inline asm so that hipcc neither
// waits for it nor moves the result to an SGPR right away; the caller retires it with a counted vmcnt before
// ws_publish_asm reads the result (cdna_hip_programming.md §5.7 item 1, form ii: the destination is named again
// by the consuming statement; audited in the .s: no copy of it between the two).
__device__ __forceinline__ void ws_claim_asm(int* head, int& ret) {
  unsigned long long save;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "s_nop 4\n\t"
      "global_atomic_add %0, %2, %3, off sc0\n\t"
      "s_mov_b64 exec, %1"
      : "=&v"(ret), "=&s"(save)
      : "v"(head), "v"(1)
      : "memory");
}
// lane 0 stores the claimed chunk index to the LDS ring (the other lanes store nothing)
__device__ __forceinline__ void ws_publish_asm(int* slot_lds, int& v, int lane) {
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)slot_lds;
  unsigned long long save;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "s_nop 4\n\t"
      "ds_write_b32 %2, %0\n\t"
      "s_mov_b64 exec, %1"
      : "+v"(v), "=&s"(save)
      : "v"(a)
      : "memory");
  (void)lane;
}

// The MFMA phase of a step: 24 activation fragments (2 row blocks x 12 K steps), each feeding 3 MFMAs, read by
// inline-asm ds_read_b128 kept WS_PF ahead (hipcc, at ~240 VGPRs, issued each read right before its MFMAs and
// waited for it: one LDS round trip per 3 MFMAs).  Each wait names its fragment ("+v", cdna_hip_programming.md
// §5.7 item 1 form ii) so no MFMA is scheduled above it; LDS returns in order, so lgkmcnt(reads issued after
// fragment t) retires fragment t.  Chunk 4 kk + g of row r sits at chunk (4 kk + g) ^ r =
// 16 (kk >> 2) + 4 ((kk & 3) ^ (r >> 2)) + (g ^ (r & 3)): four per-lane bases (kk & 3) plus constants.
constexpr int WS_PF = 4;
__device__ __forceinline__ void ws_ds_read(bf16x8& x, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(x) : "v"(addr) : "memory");
}
template <int N>
__device__ __forceinline__ void ws_lgkm_wait(bf16x8& x) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(x) : "i"(N) : "memory");
}
template <int T>
__device__ __forceinline__ unsigned ws_frag_addr(const unsigned (&xb4)[4]) {
  constexpr int kk = T % 12;
  return xb4[kk & 3] + (T / 12) * 16 * wsg::ROWB + (kk >> 2) * 256;
}
template <int A, int T>
__device__ __forceinline__ void ws_mfma_loop(f32x4 (&acc)[2][3], const bf16x8 (&wf)[3][12], const unsigned (&xb4)[4],
                                             bf16x8 (&xs)[WS_PF]) {
  if constexpr (T < 12) {
    constexpr int after = (11 - T) < (WS_PF - 1) ? (11 - T) : (WS_PF - 1);
    ws_lgkm_wait<after>(xs[T % WS_PF]);
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[A][j] = mfma16(wf[j][T], xs[T % WS_PF], acc[A][j]);
    if constexpr (T + WS_PF < 12) ws_ds_read(xs[T % WS_PF], ws_frag_addr<A * 12 + T + WS_PF>(xb4));
    ws_mfma_loop<A, T + 1>(acc, wf, xb4, xs);
  }
}
// row block A (16 rows) of a step: 12 fragments x 3 MFMAs
template <int A>
__device__ __forceinline__ void ws_mfma_half(f32x4 (&acc)[2][3], const bf16x8 (&wf)[3][12], const unsigned (&xb4)[4]) {
  static_assert(WS_PF == 4, "prologue reads");
#pragma unroll
  for (int j = 0; j < 3; ++j) acc[A][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 xs[WS_PF];
  ws_ds_read(xs[0], ws_frag_addr<A * 12 + 0>(xb4));
  ws_ds_read(xs[1], ws_frag_addr<A * 12 + 1>(xb4));
  ws_ds_read(xs[2], ws_frag_addr<A * 12 + 2>(xb4));
  ws_ds_read(xs[3], ws_frag_addr<A * 12 + 3>(xb4));
  ws_mfma_loop<A, 0>(acc, wf, xb4, xs);
}

// Row chunks are split into 8 contiguous ranges, one per XCD: a workgroup claims from its own XCD's range of its
// column group first (the column groups of one XCD then stream the same A rows, which its L2 serves to all but
// the first), then from the next XCDs' ranges once its own is exhausted.  One lane; blocking (the prologue's claims
// and the rare range switch at the end of a range).
__device__ __forceinline__ int ws_range_lo(int xr, int nch) { return (xr * nch) >> 3; }
__device__ int ws_claim_blocking(int* heads, int cg, int& xr, int& visited, int nch) {
  while (visited < 8) {
    const int lo = ws_range_lo(xr, nch), len = ws_range_lo(xr + 1, nch) - lo;
    const int r = __hip_atomic_fetch_add(heads + xr * 8 + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (r < len) return lo + r;
    xr = (xr + 1) & 7;
    ++visited;
  }
  return nch;
}

template <int EPI>
constexpr bool ws_epi_ok() {
  return EPI == EPI_BF16 || EPI == EPI_GELU || EPI == EPI_GELU_ACT || EPI == EPI_GELU_D || EPI == EPI_F32;
}
// C stores per wave per epilogue (6 items of 4 outputs per lane; two outputs for GELU / GELU_D)
template <int EPI>
constexpr int ws_nstore() {
  return (EPI == EPI_GELU || EPI == EPI_GELU_D) ? 12 : 6;
}

template <int EPI, int STAUX, int PROBE = 0>
__global__ __launch_bounds__(512, 2) void gemm_nt_ws_kernel(NTArgs p, int ncg, int slot) {
  using namespace wsg;
  static_assert(ws_epi_ok<EPI>(), "epilogue");
  static_assert(NST == 4 && CH == 2, "the claim lookahead below is written for 4 stages and 2-tile chunks");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* const qring = (int*)(smem + NST * STAGE);
  float* const bias_lds = (float*)(qring + QN + 4);  // the column group's bias (after 4 scratch words)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int cg = blockIdx.x % ncg;
  int* const ctr = g_ws_ctr + slot * SLOT_INTS;
  const int nrt = (p.M + R - 1) / R, nch = (nrt + CH - 1) / CH;
  const int n0 = cg * NG, nw = n0 + w * 48;
  const bool late = w >= 4;  // waves 4..7 interleave their epilogue differently (see the step body)

  // claim state (wave 0): the XCD range claimed from and how many ranges were found exhausted
  int xr;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xr));
  xr &= 7;
  int visited = 0;
  // the first three chunks: blocking claims (their latency hides behind the weight loads below)
  if (tid == 0) {
    if constexpr (PROBE == 5) {  // measurement: static chunks rs, rs + nrs, ... (no claims)
      const int rs = blockIdx.x / ncg, nrs = gridDim.x / ncg;
      qring[0] = rs; qring[1] = rs + nrs; qring[2] = rs + 2 * nrs;
    } else {
      qring[0] = ws_claim_blocking(ctr, cg, xr, visited, nch);
      qring[1] = ws_claim_blocking(ctr, cg, xr, visited, nch);
      qring[2] = ws_claim_blocking(ctr, cg, xr, visited, nch);
      qring[QN + 0] = xr;  // (the bias follows the ring: these two words are scratch before it is written)
      qring[QN + 1] = visited;
    }
  }
  bf16x8 wf[3][12];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int kk = 0; kk < 12; ++kk)
      wf[j][kk] = *(const bf16x8*)(p.B + (size_t)(nw + 16 * j + r) * p.ldb + 32 * kk + 8 * g);
  if (tid < NG / 4)
    *(f32x4*)(bias_lds + 4 * tid) = p.bias ? *(const f32x4*)(p.bias + n0 + 4 * tid) : f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // weights, bias and the first claims retired (no compiler-counted load crosses into the loop)
  if constexpr (PROBE != 5) {
    xr = __builtin_amdgcn_readfirstlane(qring[QN + 0]);
    visited = __builtin_amdgcn_readfirstlane(qring[QN + 1]);
  }
  int cur = __builtin_amdgcn_readfirstlane(qring[0]);  // chunk of the current iteration, and the two after it
  int n1 = __builtin_amdgcn_readfirstlane(qring[1]);
  int n2 = __builtin_amdgcn_readfirstlane(qring[2]);

  // LDS-DMA source offsets of this wave's pieces within a tile (bytes from the tile's first row)
  unsigned so[PIECES];
#pragma unroll
  for (int j = 0; j < PIECES; ++j) {
    const int off = ((j * 8 + w) * 64 + lane) * 16, row = off / ROWB, c = (off % ROWB) >> 4;
    so[j] = (unsigned)(row * p.lda * 2 + ((c ^ (row & 15)) << 4));
  }
  auto dma = [&](int st, int tile) {
    const char* src = (const char*)(p.A + (size_t)tile * R * p.lda);
#pragma unroll
    for (int j = 0; j < PIECES; ++j) glds16_asm(src + so[j], smem + st * STAGE + (j * 8 + w) * 1024);
  };
  int xbase[4];  // per-lane byte offsets of the activation fragments within a stage (ws_mfma_phase)
#pragma unroll
  for (int k = 0; k < 4; ++k) xbase[k] = r * ROWB + ((4 * (k ^ (r >> 2)) + (g ^ (r & 3))) << 4);

  // Epilogue straight from the MFMA layout: acc[a][j] holds C[m0 + 16 a + r][nw + 16 j + 4 g + 0..3] (the
  // accumulator of D = W X^T: 4 consecutive columns of one row per lane), so each store instruction writes
  // 16 rows x 32 (bf16) / 64 (fp32) contiguous bytes and a wave's 3 stores per row block cover 96 / 192 B;
  // the L2 merges the eight waves' pieces of each row (plain stores: written back as whole lines).
  constexpr bool f32out = EPI == EPI_F32;
  const unsigned crows = (unsigned)p.M;
  const __amdgpu_buffer_rsrc_t rc = buf_rsrc(p.C, crows * p.ldc * (f32out ? 4u : 2u));
  const __amdgpu_buffer_rsrc_t rc2 = buf_rsrc((EPI == EPI_GELU || EPI == EPI_GELU_D) ? p.C2 : p.C, crows * p.ldc * 2u);
  auto epilogue = [&](const f32x4 (&acc)[2][3], int tile, int a) {  // row block a of tile
    const int m0 = tile * R;
    f32x4 bj[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) bj[j] = *(const f32x4*)(bias_lds + w * 48 + 16 * j + 4 * g);
    auto st8 = [&](const float* v, __amdgpu_buffer_rsrc_t rr, unsigned o) {  // 4 bf16 = 8 B
      const bf16x4 b = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, b), rr, o, 0, STAUX);
    };
#pragma unroll
    for (int j = 0; j < 3; ++j) {  // column fragment j: 4 consecutive outputs of one row
      const f32x4 x = acc[a][j] + bj[j];
      float v[4] = {x[0], x[1], x[2], x[3]};
      const int m = m0 + 16 * a + r;
      const unsigned off = m < p.M ? (unsigned)(m * p.ldc + nw + 16 * j + 4 * g) * (f32out ? 4u : 2u) : ES_OOB;
      if constexpr (EPI == EPI_F32) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), rc, off, 0, STAUX);
      } else if constexpr (EPI == EPI_BF16) {
        st8(v, rc, off);
      } else {
        float gg[4], dd[4];
        gelu_and_grad_f4(v, gg, dd);
        if constexpr (EPI == EPI_GELU_ACT) {
          st8(gg, rc, off);
        } else if constexpr (EPI == EPI_GELU) {
          st8(v, rc, off);
          st8(gg, rc2, off);
        } else {  // EPI_GELU_D: C = gelu', C2 = gelu
          st8(dd, rc, off);
          st8(gg, rc2, off);
        }
      }
    }
  };

  if (cur < nch) {
    // vmcnt bookkeeping: this wave's VMEM ops since the loop started, in issue order
    int seq = 0;
    auto dma_valid = [&](int ch, int k) { return ch < nch && ch * CH + k < nrt; };
    dma(0, cur * CH);  // positions 0, 1 (chunk cur) and 2 (chunk n1)
    seq += PIECES;
    int after_a = seq;  // seq right after the DMA of position i (retired at the top of step i), i + 1, i + 2
    if (dma_valid(cur, 1)) {
      dma(1, cur * CH + 1);
      seq += PIECES;
    }
    int after_b = seq;
    if (dma_valid(n1, 0)) {
      dma(2, n1 * CH);
      seq += PIECES;
    }
    int after_c = seq;
    int st = 0;  // ring stage of the current position
    int nstep = 0;
    auto top = [&]() {
      if constexpr (PROBE == 7) {
        if (blockIdx.x == 0 && (w == 0 || w == 4) && lane == 0 && nstep < 64)
          g_ws_dbg[((w >> 2) * 64 + nstep) * 8 + 7] = __builtin_amdgcn_s_memtime();
      }
      wait_vmcnt_any(seq - after_a);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // stage of this position landed for every wave
    };
    // One step: the DMA three positions ahead (tile tdma, or none), then the MFMAs and epilogue of this position
    // (tile tcur), one 16-row block at a time.  Each SIMD holds one wave of each half of the workgroup; waves 0..3
    // run [MFMA 0][MFMA 1][epilogue 0][epilogue 1], waves 4..7 [MFMA 0][epilogue 0][MFMA 1][epilogue 1], so
    // each wave's epilogue (VALU, stores) runs beside its partner's MFMAs instead of both partners alternating
    // the two in step (MI355X_MICROARCH.md, two waves per SIMD, item 9: split roles by wave number >= 4).
    auto stamp = [&](int k) {
      if constexpr (PROBE == 7) {
        if (blockIdx.x == 0 && (w == 0 || w == 4) && lane == 0 && nstep < 64)
          g_ws_dbg[((w >> 2) * 64 + nstep) * 8 + k] = __builtin_amdgcn_s_memtime();
      }
    };
    auto body = [&](bool do_dma, int tdma, int tcur, auto&& tail) {
      stamp(0);
      int st3 = st + 3;
      st3 = st3 >= NST ? st3 - NST : st3;
      after_a = after_b;
      after_b = after_c;
      if (do_dma) {
        dma(st3, tdma);
        seq += PIECES;
      }
      after_c = seq;
      f32x4 acc[2][3];
      unsigned xb4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        xb4[k] = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)(smem + st * STAGE + xbase[k]);
      stamp(1);
      ws_mfma_half<0>(acc, wf, xb4);
      stamp(2);
      if (late) {
        epilogue(acc, tcur, 0);
        stamp(3);
        ws_mfma_half<1>(acc, wf, xb4);
      } else {
        ws_mfma_half<1>(acc, wf, xb4);
        stamp(3);
        epilogue(acc, tcur, 0);
      }
      stamp(4);
      epilogue(acc, tcur, 1);
      stamp(5);
      seq += ws_nstore<EPI>();
      tail();
      stamp(6);
      st = st + 1 == NST ? 0 : st + 1;
      ++nstep;
    };
    // one iteration = one chunk (positions 2 lc, 2 lc + 1).  The claim for chunk lc + 3 is issued at the first
    // position and consumed (published to LDS) at the end of the second, inside the iteration; the DMA of the
    // first tile of chunk lc + 3 is issued at position 2 lc + 3, after the next iteration's first barrier.
    for (int lc = 0;; ++lc) {
      top();
      if (lc > 0) {
        cur = n1;
        n1 = n2;
        n2 = __builtin_amdgcn_readfirstlane(qring[(lc + 2) & (QN - 1)]);
        if (cur >= nch) break;
      }
      const bool live = n2 < nch;
      const bool claimer = live && w == 0;  // wave-uniform
      int claimed = nch, after_claim = 0;
      if (claimer) {
        if constexpr (PROBE == 5) {
          claimed = (int)(blockIdx.x / ncg) + (lc + 3) * (int)(gridDim.x / ncg);
        } else {
          ws_claim_asm(ctr + xr * 8 + cg, claimed);
          seq += 1;
        }
        after_claim = seq;
      }
      body(dma_valid(n1, 1), n1 * CH + 1, cur * CH, [] {});
      top();
      if (cur * CH + 1 >= nrt) break;
      body(dma_valid(n2, 0), n2 * CH, cur * CH + 1, [&] {
        if (w == 0) {  // publish chunk lc + 3 (nch: none claimed) for the iterations after this one
          int chunk = nch;
          if (claimer) {
            wait_vmcnt_any(seq - after_claim);
            asm volatile("" : "+v"(claimed));  // (ordered after the wait: the claim's data is in lane 0)
            const int raw = __builtin_amdgcn_readfirstlane(claimed);
            if constexpr (PROBE == 5) {
              chunk = raw;
            } else {
              const int lo = ws_range_lo(xr, nch), len = ws_range_lo(xr + 1, nch) - lo;
              if (raw < len) {
                chunk = lo + raw;
              } else {  // this XCD's range is exhausted: the next ones (blocking; once per range at its end)
                xr = (xr + 1) & 7;
                ++visited;
                int c2 = nch, x2 = xr, v2 = visited;
                if (lane == 0) c2 = ws_claim_blocking(ctr, cg, x2, v2, nch);
                chunk = __builtin_amdgcn_readfirstlane(c2);
                xr = __builtin_amdgcn_readfirstlane(x2);
                visited = __builtin_amdgcn_readfirstlane(v2);
              }
            }
          }
          if (lane == 0) qring[(lc + 3) & (QN - 1)] = chunk;
        }
      });
    }
  }
  // every claim of this workgroup has landed; the last workgroup out resets the counter block
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tid == 0) {
    const int d = __hip_atomic_fetch_add(ctr + SLOT_INTS - 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (int)gridDim.x - 1) {
      for (int x = 0; x < 8; ++x)
        for (int c = 0; c < ncg; ++c) __hip_atomic_store(ctr + x * 8 + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + SLOT_INTS - 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The attention projection with its residual add AND the LayerNorm that follows it (round 6,
// es_gemm_nt_resid_ln): x = o W^T + b + x_in (fp32), h = LN(x) (bf16), mean / rstd -- for D = 384
// (ViT-S: N = K = 384).  Replaces es_gemm_nt(EPI_F32_RESID) + es_layernorm_fwd (code/models/conformer.py:
// 65-66: x = x + attn(norm1(x)); norm2(x)) in one pass: x is never re-read from memory for its
// statistics.  The weight-stationary body of gemm_nt_ws_kernel (W in registers, one persistent 8-wave
// workgroup per CU, 32-row tiles) with whole rows per workgroup (one column group), so the row
// statistics need no cross-workgroup exchange:
//   ring (2 stages): the A tile (24 KiB, swizzled as in gemm_nt_ws_kernel) and the residual tile (32 rows x
//     1,536 B, 16-B chunk c of row r at chunk c ^ (r & 15): conflict-free both for the MFMA-layout reads of
//     the epilogue and for the LayerNorm's row reads), both by LDS-DMA one tile ahead;
//   per step: [vmcnt: tile i landed] [barrier] [DMA tile i + 1] [claim tile i + 2] [MFMAs] [x = acc + bias +
//     residual, written over the residual tile in place] [barrier] [LayerNorm: one wave per row, 4 rows per
//     wave, ln_fwd_kernel's lane map, warp sums and rounding as compiled (see the statistics below), so h /
//     mean / rstd are its bits for the same x] [x, h, mean, rstd stores] [the claim retired, published for
//     step i + 2].
// x's bits equal es_gemm_nt(EPI_F32_RESID)'s (the same MFMA chain, (acc + bias) + residual) and h's equal
// es_layernorm_fwd's on that x (tested).
namespace rlg {
constexpr int R = 32, KD = 384, D = 384;
constexpr int ROWA = KD * 2, TA = R * ROWA;        // A tile: 24 KiB
constexpr int ROWX = D * 4, TX = R * ROWX;         // residual / x tile: 48 KiB
constexpr int STAGE = TA + TX, NST = 2;
constexpr int PA = TA / 1024 / 8, PX = TX / 1024 / 8;  // LDS-DMA instructions per wave per stage (3 + 6)
constexpr int QN = 4;
constexpr int LDS = NST * STAGE + QN * 4 + 16 + D * 4 * 3;  // ring, claim ring, scratch, bias, gamma, beta
constexpr int SLOTS = 64, SLOT_INTS = 4;                    // per stream: [0] head, [3] done
}  // namespace rlg
__device__ int g_rl_ctr[rlg::SLOTS * rlg::SLOT_INTS];

// a a + b b with both products rounded (no contraction: __fmul_rn is a plain multiply in this HIP, so the
// pragma is what keeps hipcc from fusing), and fma(a, a, b b)
__device__ __forceinline__ float sq2_rounded(float a, float b) {
#pragma clang fp contract(off)
  return a * a + b * b;
}
__device__ __forceinline__ float sq2_fused(float a, float b) {
#pragma clang fp contract(off)
  return __builtin_fmaf(a, a, b * b);
}
__device__ __forceinline__ float mul_rounded(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}

struct RLArgs {
  const float* gamma; const float* beta;
  bf16* h; float* mean; float* rstd;
  int ldh; float eps;
};

__global__ __launch_bounds__(512, 1) void gemm_resid_ln_kernel(NTArgs p, RLArgs l, int slot) {
  using namespace rlg;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* const qring = (int*)(smem + NST * STAGE);
  float* const bias_lds = (float*)(qring + QN + 4);
  float* const gam_lds = bias_lds + D;
  float* const bet_lds = gam_lds + D;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  int* const ctr = g_rl_ctr + slot * SLOT_INTS;
  const int nt = (p.M + R - 1) / R;
  if (tid == 0) {  // the first two tiles: blocking claims (their latency hides behind the weight loads)
    qring[0] = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    qring[1] = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  bf16x8 wf[3][12];
  const int nw = w * 48;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int kk = 0; kk < 12; ++kk)
      wf[j][kk] = *(const bf16x8*)(p.B + (size_t)(nw + 16 * j + r) * p.ldb + 32 * kk + 8 * g);
  if (tid < D / 4) {
    *(f32x4*)(bias_lds + 4 * tid) = p.bias ? *(const f32x4*)(p.bias + 4 * tid) : f32x4{0.f, 0.f, 0.f, 0.f};
    *(f32x4*)(gam_lds + 4 * tid) = *(const f32x4*)(l.gamma + 4 * tid);
    *(f32x4*)(bet_lds + 4 * tid) = *(const f32x4*)(l.beta + 4 * tid);
  }
  __syncthreads();  // weights, parameters and the first claims retired before the loop's counted waits
  int cur = __builtin_amdgcn_readfirstlane(qring[0]);
  int nxt = __builtin_amdgcn_readfirstlane(qring[1]);

  // LDS-DMA pieces: A (row, 16-B chunk) and residual (row, chunk) of this wave's instructions within a tile
  int ar[PA], ac[PA], xr[PX], xc[PX];
#pragma unroll
  for (int j = 0; j < PA; ++j) {
    const int off = ((j * 8 + w) * 64 + lane) * 16;
    ar[j] = off / ROWA;
    ac[j] = ((off % ROWA) >> 4) ^ (ar[j] & 15);
  }
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    const int P = (j * 8 + w) * 64 + lane;  // physical chunk of the tile (contiguous per instruction)
    xr[j] = P / (ROWX / 16);
    xc[j] = (P % (ROWX / 16)) ^ (xr[j] & 15);  // the logical chunk it holds
  }
  auto dma = [&](int st, int tile) {  // rows past M re-read row M - 1 (finite, never stored)
    const int m0 = tile * R, lim = p.M - 1 - m0;
    const char* a = (const char*)(p.A + (size_t)m0 * p.lda);
    const char* x = (const char*)((const float*)p.aux + (size_t)m0 * p.ldaux);
    char* S = smem + st * STAGE;
#pragma unroll
    for (int j = 0; j < PA; ++j)
      glds16_asm(a + (size_t)min(ar[j], lim) * p.lda * 2 + ac[j] * 16, S + (j * 8 + w) * 1024);
#pragma unroll
    for (int j = 0; j < PX; ++j)
      glds16_asm(x + (size_t)min(xr[j], lim) * p.ldaux * 4 + xc[j] * 16, S + TA + (j * 8 + w) * 1024);
  };
  int xbase[4];  // the activation fragments' per-lane offsets (gemm_nt_ws_kernel's layout)
#pragma unroll
  for (int k = 0; k < 4; ++k) xbase[k] = r * ROWA + ((4 * (k ^ (r >> 2)) + (g ^ (r & 3))) << 4);

  const unsigned rows = (unsigned)p.M;
  const __amdgpu_buffer_rsrc_t rx = buf_rsrc(p.C, rows * p.ldc * 4u);
  const __amdgpu_buffer_rsrc_t rh = buf_rsrc(l.h, rows * l.ldh * 2u);
  const __amdgpu_buffer_rsrc_t rm = buf_rsrc(l.mean, rows * 4u);
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(l.rstd, rows * 4u);

  if (cur < nt) {
    int seq = 0, after_cur = 0, after_nxt = 0;
    dma(0, cur);
    seq += PA + PX;
    after_cur = seq;
    if (nxt < nt) {
      dma(1, nxt);
      seq += PA + PX;
    }
    after_nxt = seq;
    int st = 0;
    for (int it = 0;; ++it) {
      if (it > 0) {  // this step's tile: the one DMA'd last step (claims only grow, so past the end stays past it)
        cur = nxt;
        after_cur = after_nxt;
        if (cur >= nt) break;
      }
      wait_vmcnt_any(seq - after_cur);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // tile `cur` landed for every wave; the other stage and the claim ring free
      if (it > 0) {  // the next step's tile (published at the end of the last step) into the other stage
        nxt = __builtin_amdgcn_readfirstlane(qring[(it + 1) & (QN - 1)]);
        if (nxt < nt) {
          dma(st ^ 1, nxt);
          seq += PA + PX;
        }
        after_nxt = seq;
      }
      // claim the tile of step it + 2 (one lane of wave 0; retired by a counted wait at the end of the step)
      int claimed = nt, after_claim = 0;
      const bool claimer = w == 0;
      if (claimer) {
        ws_claim_asm(ctr, claimed);
        seq += 1;
        after_claim = seq;
      }
      char* S = smem + st * STAGE;
      unsigned xb4[4];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        xb4[k] = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)(S + xbase[k]);
      f32x4 acc[2][3];
      ws_mfma_half<0>(acc, wf, xb4);
      ws_mfma_half<1>(acc, wf, xb4);
      // x = (acc + bias) + residual in the MFMA layout (lane: row 16 a + r, columns nw + 16 j + 4 g .. + 3),
      // written over the residual
      char* X = S + TA;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int row = 16 * a + r, c = w * 12 + 4 * j + g;
          f32x4* q = (f32x4*)(X + row * ROWX + ((c ^ r) << 4));
          const f32x4 v = acc[a][j] + *(const f32x4*)(bias_lds + nw + 16 * j + 4 * g);
          *q = v + *q;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // the x tile complete
      // LayerNorm, one wave per row (ln_fwd_kernel's map: lane holds columns (j * 64 + lane) * 2, + 1)
      const int m0 = cur * R;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = w * 4 + q;
        float2 v[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int cc = (j * 64 + lane) >> 1;
          v[j] = *(const float2*)(X + row * ROWX + ((cc ^ (row & 15)) << 4) + (lane & 1) * 8);
        }
        // the statistics with the rounding of ln_fwd_kernel / ln_fwd_loop_kernel as hipcc (ROCm 7.2) compiles
        // them, which differs between the two rows a wave holds: their ISA sums the three column pairs' squares
        // as fma(a0, a0, b0 b0) + (a1 a1 + b1 b1) + fma(a2, a2, b2 b2) for the even row and with no fma for the
        // odd row, left to right, fuses the variance scale with eps and forms the output as fma(g, (x - mean)
        // rstd, b).  Written out here because where hipcc contracts a * b + c depends on the surrounding code
        // (the same source expression gave rstd 1 ulp apart on ~2 % of rows); the bit-identity test
        // (test_gemm_resid_ln_matches_two_launches_bit_for_bit) pins it to the LayerNorm kernels' build.
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 3; ++j) s += v[j].x + v[j].y;
        const float mean = warp_sum(s) * (1.0f / D);
        float a[3], b[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          a[j] = v[j].x - mean;
          b[j] = v[j].y - mean;
        }
        const bool even = (q & 1) == 0;  // the row's place in ln_fwd_kernel's row pair (m0 and w * 4 are even)
        const float t0 = even ? sq2_fused(a[0], b[0]) : sq2_rounded(a[0], b[0]);
        const float t1 = sq2_rounded(a[1], b[1]);
        const float t2 = even ? sq2_fused(a[2], b[2]) : sq2_rounded(a[2], b[2]);
        const float ss = (t0 + t1) + t2;
        const float rstd = 1.0f / sqrtf(__builtin_fmaf(warp_sum(ss), 1.0f / D, l.eps));
        const int m = m0 + row;
        const bool ok = m < p.M;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int c = (j * 64 + lane) * 2;
          const float2 gm = *(const float2*)(gam_lds + c), bt = *(const float2*)(bet_lds + c);
          typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
          bf16x2 o = {(bf16)__builtin_fmaf(mul_rounded(a[j], rstd), gm.x, bt.x),
                      (bf16)__builtin_fmaf(mul_rounded(b[j], rstd), gm.y, bt.y)};
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[j]), rx,
                                                ok ? (unsigned)(m * p.ldc + c) * 4u : ES_OOB, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, o), rh,
                                                ok ? (unsigned)(m * l.ldh + c) * 2u : ES_OOB, 0, 0);
        }
        const bool one = ok && lane == 0;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, mean), rm, one ? (unsigned)m * 4u : ES_OOB,
                                              0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, rstd), rs, one ? (unsigned)m * 4u : ES_OOB,
                                              0, 0);
      }
      seq += 4 * 8;
      if (claimer) {  // publish the tile of step it + 2
        wait_vmcnt_any(seq - after_claim);
        asm volatile("" : "+v"(claimed));
        const int c2 = __builtin_amdgcn_readfirstlane(claimed);
        if (lane == 0) qring[(it + 2) & (QN - 1)] = c2;
      }
      st ^= 1;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (tid == 0) {
    const int d = __hip_atomic_fetch_add(ctr + SLOT_INTS - 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (int)gridDim.x - 1) {
      __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + SLOT_INTS - 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Launcher with every specialisation spelled out and launched by name (HIP_KERNEL_NAME keeps the
// template commas out of the launch macro; a kernel referenced only through a function pointer
// gets no host stub).
#define NT_LAUNCH(E, BKT_, NST_, TBM_, ...)                                             \
  {                                                                                        \
    const size_t lds = std::max((size_t)NST_ * (TBM_ + BN) * BKT_ * 2, (size_t)4 * EPI_WAVE_BYTES); \
    allow_lds(gemm_nt_kernel<E, BKT_, NST_, TBM_, ##__VA_ARGS__>, lds);                   \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_nt_kernel<E, BKT_, NST_, TBM_, ##__VA_ARGS__>), dim3(grid), dim3(256), lds, stream, a); \
    return ES_OK;                                                                          \
  }
#define NT_EPIS(BKT_, NST_, TBM_, ...)                                            \
  switch (epi) {                                                                  \
    case EPI_BF16: NT_LAUNCH(EPI_BF16, BKT_, NST_, TBM_, ##__VA_ARGS__)           \
    case EPI_GELU: NT_LAUNCH(EPI_GELU, BKT_, NST_, TBM_, ##__VA_ARGS__)           \
    case EPI_F32_RESID: NT_LAUNCH(EPI_F32_RESID, BKT_, NST_, TBM_, ##__VA_ARGS__) \
    case EPI_DGELU: NT_LAUNCH(EPI_DGELU, BKT_, NST_, TBM_, ##__VA_ARGS__)         \
    case EPI_F32: NT_LAUNCH(EPI_F32, BKT_, NST_, TBM_, ##__VA_ARGS__)             \
    case EPI_PATCH: NT_LAUNCH(EPI_PATCH, BKT_, NST_, TBM_, ##__VA_ARGS__)         \
    case EPI_GELU_ACT: NT_LAUNCH(EPI_GELU_ACT, BKT_, NST_, TBM_, ##__VA_ARGS__)   \
    case EPI_GELU_D: NT_LAUNCH(EPI_GELU_D, BKT_, NST_, TBM_, ##__VA_ARGS__)       \
    case EPI_MULAUX: NT_LAUNCH(EPI_MULAUX, BKT_, NST_, TBM_, ##__VA_ARGS__)       \
    default: return ES_BAD_ARG;                                                   \
  }
// The residual-stream outputs (EPI_F32_RESID: the proj / fc2 forward's x + f(x), read right away by the
// next LayerNorm) keep plain, cacheable C stores instead of nt: F1 30.82 / 30.84 -> 30.59 / 30.66 ms on one
// box (bench.py A/B, round 3); plain stores for the qkv (EPI_BF16) or fc1 (EPI_GELU_D) outputs were
// slower (30.90 / 31.03 ms).
int launch_nt(int cfg, int epi, int grid, hipStream_t stream, const NTArgs& a) {
  if (cfg == 11 && epi == EPI_F32_RESID) NT_LAUNCH(EPI_F32_RESID, 64, 2, 64, 0)
  switch (cfg) {
    case 0: NT_EPIS(64, 2, 128)
    case 5: NT_EPIS(32, 2, 128)
    case 11: NT_EPIS(64, 2, 64)
    default: NT_EPIS(32, 3, 128)  // 2
  }
}
#undef NT_EPIS
#undef NT_LAUNCH

#define BIG_LAUNCH(E, WM_, MF_, NF_, NST_, BKT_, OCC_, ...)                                        \
  {                                                                                                 \
    const size_t lds = (size_t)NST_ * (WM_ * MF_ * 16 + (8 / WM_) * NF_ * 16) * BKT_ * 2;            \
    allow_lds(gemm_nt_big_kernel<E, WM_, MF_, NF_, NST_, BKT_, OCC_, ##__VA_ARGS__>, lds);          \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_nt_big_kernel<E, WM_, MF_, NF_, NST_, BKT_, OCC_, ##__VA_ARGS__>), dim3(grid), \
                       dim3(512), lds, stream, a);                                                  \
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;                                  \
  }
#define BIG_EPIS2(WM_, MF_, NF_, NST_, BKT_, OCC_)                                        \
  switch (epi) {                                                                          \
    case EPI_BF16: BIG_LAUNCH(EPI_BF16, WM_, MF_, NF_, NST_, BKT_, OCC_)                  \
    case EPI_GELU: BIG_LAUNCH(EPI_GELU, WM_, MF_, NF_, NST_, BKT_, OCC_)                  \
    case EPI_F32_RESID: BIG_LAUNCH(EPI_F32_RESID, WM_, MF_, NF_, NST_, BKT_, OCC_)        \
    case EPI_DGELU: BIG_LAUNCH(EPI_DGELU, WM_, MF_, NF_, NST_, BKT_, OCC_)                \
    case EPI_F32: BIG_LAUNCH(EPI_F32, WM_, MF_, NF_, NST_, BKT_, OCC_)                    \
    case EPI_PATCH: BIG_LAUNCH(EPI_PATCH, WM_, MF_, NF_, NST_, BKT_, OCC_)                \
    case EPI_GELU_ACT: BIG_LAUNCH(EPI_GELU_ACT, WM_, MF_, NF_, NST_, BKT_, OCC_)          \
    case EPI_GELU_D: BIG_LAUNCH(EPI_GELU_D, WM_, MF_, NF_, NST_, BKT_, OCC_)              \
    case EPI_MULAUX: BIG_LAUNCH(EPI_MULAUX, WM_, MF_, NF_, NST_, BKT_, OCC_)              \
    default: return ES_BAD_ARG;                                                           \
  }
#define BIG_EPIS(WM_, MF_, NF_, NST_, BKT_) BIG_EPIS2(WM_, MF_, NF_, NST_, BKT_, 1)
int launch_big(int cfg, int epi, int grid, hipStream_t stream, const NTArgs& a) {
  if (cfg == 10 && epi == EPI_F32_RESID) BIG_LAUNCH(EPI_F32_RESID, 4, 4, 4, 3, 32, 4, 0, 0)  // plain stores
  switch (cfg) {
    case 10: BIG_EPIS2(4, 4, 4, 3, 32, 4)  // 256x128, BK32, 3 stages (72 KiB), two workgroups per CU
    default: BIG_EPIS(2, 8, 4, 2, 64)      // 6: 256x256, BK64, 2 stages (128 KiB)
  }
}
#undef BIG_EPIS
#undef BIG_EPIS2
#undef BIG_LAUNCH

// The weight-stationary kernel's counter block for a stream: launches on one stream never overlap, so one block
// per stream is never shared by two running launches (64 streams; beyond that streams share blocks by hash,
// which is only wrong if two of them then run such GEMMs at the same time).
static int ws_slot(hipStream_t s) {
  static hipStream_t tab[wsg::SLOTS];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (tab[i] == s) return i;
  if (n < wsg::SLOTS) {
    tab[n] = s;
    return n++;
  }
  return (int)(((uintptr_t)s >> 6) % wsg::SLOTS);
}
static bool ws_fits(int epi, int N, int K) {
  const bool e = epi == EPI_BF16 || epi == EPI_GELU || epi == EPI_GELU_ACT || epi == EPI_GELU_D || epi == EPI_F32;
  return e && K == wsg::KD && N % wsg::NG == 0 && N / wsg::NG <= 8;
}
#define WS_LAUNCH(E, AUX_, ...)                                                                                   \
  {                                                                                                                \
    allow_lds(gemm_nt_ws_kernel<E, AUX_, ##__VA_ARGS__>, (size_t)wsg::LDS);                                       \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_nt_ws_kernel<E, AUX_, ##__VA_ARGS__>), dim3(grid), dim3(512), wsg::LDS, \
                       stream, a, ncg, slot);                                                                      \
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;                                                 \
  }
int launch_ws(int epi, hipStream_t stream, const NTArgs& a) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  const int ncg = a.N / wsg::NG;
  const int nrt = (a.M + wsg::R - 1) / wsg::R, nch = (nrt + wsg::CH - 1) / wsg::CH;
  const int per = std::max(1, std::min(cus / ncg, nch));  // workgroups per column group
  const int grid = per * ncg;
  const int slot = ws_slot(stream);
  static const int probe = getenv("ENDOSSL_WS_PROBE") ? atoi(getenv("ENDOSSL_WS_PROBE")) : 0;  // measurement only
  if (probe == 5 && epi == EPI_BF16) WS_LAUNCH(EPI_BF16, 0, 5)
  if (probe == 7 && epi == EPI_BF16) WS_LAUNCH(EPI_BF16, 0, 7)
  switch (epi) {
    case EPI_BF16: WS_LAUNCH(EPI_BF16, 0)
    case EPI_GELU: WS_LAUNCH(EPI_GELU, 0)
    case EPI_GELU_ACT: WS_LAUNCH(EPI_GELU_ACT, 0)
    case EPI_GELU_D: WS_LAUNCH(EPI_GELU_D, 0)
    case EPI_F32: WS_LAUNCH(EPI_F32, 0)
    default: return ES_BAD_ARG;
  }
}
#undef WS_LAUNCH

int launch_resid_ln(hipStream_t stream, const NTArgs& a, const RLArgs& l) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  const int nt = (a.M + rlg::R - 1) / rlg::R;
  const int grid = std::max(1, std::min(cus, nt));
  allow_lds(gemm_resid_ln_kernel, (size_t)rlg::LDS);
  hipLaunchKernelGGL(gemm_resid_ln_kernel, dim3(grid), dim3(512), rlg::LDS, stream, a, l, ws_slot(stream));
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // namespace es_gemm
using namespace es_gemm;

// ----------------------------------------------------------------- C-ABI entry points
static int g_gemm_variant = -1;
static int g_tn_variant = -1;
static int g_small_tile = 1;  // the 64 x 128 tile rules (es_set_gemm_small_tile; 0 = without them)


extern "C" {

// measurement builds only (ENDOSSL_WS_PROBE=7): the weight-stationary kernel's step stamps (not part of the es_ ABI)
int endossl_ws_debug_stamps(unsigned long long* host, int n) {
  if (n > WS_DBG) n = WS_DBG;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ws_dbg), n * sizeof(unsigned long long)) == hipSuccess ? 0 : -3;
}

int es_gemm_tn_ex(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
                  float* workspace, float* out, int accumulate, float* bias_out, int variant, hipStream_t stream);

int es_gemm_nt(int epi, const void* A, int lda, const void* B, int ldb, const float* bias, void* C,
               int ldc, void* C2, const void* aux, int ldaux, int M, int N, int K, int np,
               hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || (N % BN) || (K % BK) || (lda % 8) || (ldb % 8) || (ldc % 4))  // NOLINT
    return ES_BAD_SHAPE;
  if (!A || !B || !C) return ES_BAD_ARG;
  if (((epi == EPI_GELU || epi == EPI_GELU_D) && !C2) ||
      ((epi == EPI_F32_RESID || epi == EPI_DGELU || epi == EPI_MULAUX || epi == EPI_PATCH) && !aux))
    return ES_BAD_ARG;
  if (epi == EPI_PATCH && np <= 0) return ES_BAD_ARG;
  NTArgs a{(const bf16*)A, (const bf16*)B, bias, C, C2, aux, M, N, K, lda, ldb, ldc, ldaux, np};
  // variant -1 (default): per-shape choice measured on MI355X (scripts/gemm_bench.py, isolated launches at
  // the F1 shapes and at 1/2, 1/4, 1/8 of the batch -- a rank's share at N GPUs, --shard; r03 sweep with the
  // nt C stores, profiles/r03_nt_sweep.txt):
  //  * N = 384 outputs on the 64 x 128 tile (variant 11: twice the workgroups of the 128 x 128 tile): the
  //    residual proj forward (K = 384) at every size (F1 78.7 -> 69.9 us, weak 77.7 -> 63.4) and every
  //    N = 384 output of a rank's small shard (M < 32,768: fc2 forward, the fc1 / qkv / proj data
  //    gradients, 0.85-0.93x), and the weak fc1 (GELU) there;
  //  * the long-K N = 384 data gradients (fc1 / qkv dgrad) at F1: 128x128 BK64 (qkv dgrad 116.5 -> 101 us);
  //  * the plain / residual / MULAUX / GELU_D epilogues at F1's long token axis (the qkv forward, the fc1
  //    forward with its GELU' output, the fc2 forward and data gradient): the 256 x 128 two-workgroups-per-CU
  //    kernel (variant 10; fc1 forward 204 -> 196 us vs the 128 x 128 kernel);
  //  * the GELU epilogues otherwise (weak fc1): 128x128 BK32 two-stage at 4-5 workgroups/CU for K <= 384;
  //  * the other K <= 384 GEMMs: 128x128 BK64 two-stage (variant 0) below M = 65,536 (qkv forward at a
  //    rank's half share 73 -> 61 us) and for N <= 384, else BK32;
  //  * the patch embedding (EPI_PATCH): 128x128 BK64 at every size (r04: 0.74 / 0.68x the 256x128 BK64 kernel);
  //  * ViT-B / Conformer-B widths (K >= 768, N % 256 == 0: every S1 transformer GEMM): the 256x256
  //    tile, 710-930 vs 620-900 TF/s (--s1) -- except the erf-per-element EPI_DGELU epilogue, serial
  //    behind the 8 waves' K loop at one workgroup per CU (S1 fc2 dgrad 1.97 vs 1.65 ms on the ring).
  //  es_set_gemm_small_tile(0) drops the 64 x 128 rules.
  int variant = g_gemm_variant;
  const bool two_wg = true;
  if (variant == 12) {  // the weight-stationary kernel where it applies, the per-shape rules elsewhere
    if (ws_fits(epi, N, K)) return launch_ws(epi, stream, a);
    variant = -1;
  }
  if (variant < 0) {
    const bool gelu = epi == EPI_GELU || epi == EPI_GELU_ACT || epi == EPI_GELU_D;
    const bool plain = epi == EPI_BF16 || epi == EPI_F32 || epi == EPI_F32_RESID || epi == EPI_MULAUX;
    if (g_small_tile && N <= 384 && ((K <= 384 && epi == EPI_F32_RESID) || (M < 32768 && (plain || epi == EPI_GELU_ACT))))
      variant = 11;
    else if (g_small_tile && M < 32768 && epi == EPI_GELU_ACT)
      variant = 11;
    else if (two_wg && M >= 65536 && K >= 768 && N == 384 && epi == EPI_BF16)
      variant = 0;
    else if (two_wg && (plain || epi == EPI_GELU_D) && M >= 65536 && ((K <= 384 && N >= 384) || (K >= 768 && N == 384)))
      variant = 10;
    else if (K <= 384 && N % 256 == 0 && epi == EPI_MULAUX)
      variant = M < 65536 ? 0 : 6;
    else if (K >= 768 && N % 256 == 0 && epi != EPI_DGELU)
      variant = 6;
    else if (epi == EPI_PATCH)  // the patch embedding (K = 768): F1 88.9 vs 120.0 us on nt256, weak 76.5 vs 111.7
      variant = 0;
    else if (gelu)
      variant = K <= 384 ? 5 : 1;
    else if (K <= 384)
      variant = (epi == EPI_F32_RESID || N <= 384 || M < 65536) ? 0 : (epi == EPI_DGELU ? 2 : 5);
    else
      variant = M < 65536 ? 0 : 1;
  }
  if (variant == 1) {
    const int grid = ((M + BM2 - 1) / BM2) * (N / BN);
    const size_t lds = 3 * STAGE2;
#define L2(E) allow_lds(gemm_nt256_kernel<E>, lds); hipLaunchKernelGGL(gemm_nt256_kernel<E>, grid, 512, lds, stream, a); break;
    switch (epi) {
      case EPI_BF16: L2(EPI_BF16)
      case EPI_GELU: L2(EPI_GELU)
      case EPI_F32_RESID: L2(EPI_F32_RESID)
      case EPI_DGELU: L2(EPI_DGELU)
      case EPI_F32: L2(EPI_F32)
      case EPI_PATCH: L2(EPI_PATCH)
      case EPI_GELU_ACT: L2(EPI_GELU_ACT)
      case EPI_GELU_D: L2(EPI_GELU_D)
      case EPI_MULAUX: L2(EPI_MULAUX)
      default: return ES_BAD_ARG;
    }
#undef L2
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  if (variant == 6 || variant == 10) {
    const int tbn = variant == 6 ? 256 : 128;
    if (N % tbn) return ES_BAD_SHAPE;
    return launch_big(variant, epi, ((M + 255) / 256) * (N / tbn), stream, a);
  }
  if (variant != 0 && variant != 2 && variant != 5 && variant != 11) return ES_BAD_ARG;  // es_set_gemm_variant checks
  const int tbm = variant == 11 ? 64 : BM;
  const int grid = ((M + tbm - 1) / tbm) * (N / BN);
  const int rc = launch_nt(variant, epi, grid, stream, a);
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// x = A B^T + bias + aux (fp32 residual), h = LayerNorm(x) (bf16) with its per-row mean / rstd, for N = K = 384
// (gemm_resid_ln_kernel): es_gemm_nt(EPI_F32_RESID) followed by es_layernorm_fwd in one launch, the same bits.
int es_gemm_nt_resid_ln(const void* A, int lda, const void* B, int ldb, const float* bias, float* C, int ldc,
                        const float* aux, int ldaux, const float* gamma, const float* beta, void* h, int ldh,
                        float* mean, float* rstd, int M, int N, int K, float eps, hipStream_t stream) {
  if (M <= 0 || N != rlg::D || K != rlg::KD || (lda % 8) || (ldb % 8) || (ldc % 2) || (ldaux % 4) || (ldh % 2) ||
      (size_t)M * (size_t)std::max(ldc, ldaux) * 4 >= (1u << 31))
    return ES_BAD_SHAPE;
  if (!A || !B || !C || !aux || !gamma || !beta || !h || !mean || !rstd) return ES_BAD_ARG;
  // 16-B pieces by LDS-DMA (A, aux), 16-B weight / parameter loads, 8-B x and 4-B h stores
  if ((((uintptr_t)A | (uintptr_t)aux | (uintptr_t)B | (uintptr_t)gamma | (uintptr_t)beta) & 15) ||
      (bias && ((uintptr_t)bias & 15)) || ((uintptr_t)C & 7) || ((uintptr_t)h & 3))
    return ES_BAD_ARG;
  NTArgs a{(const bf16*)A, (const bf16*)B, bias, C, nullptr, aux, M, N, K, lda, ldb, ldc, ldaux, 0};
  RLArgs l{gamma, beta, (bf16*)h, mean, rstd, ldh, eps};
  return launch_resid_ln(stream, a, l);
}

// Tuning knob: which NT kernel family es_gemm_nt launches (-1 = per-shape default, 0 = 128x128
// BK64 2-stage, 1 = 256x128 BK64 3-stage, 2 = 128x128 BK32 3-stage, 5 = 128x128 BK32 2-stage;
// 6 = 256x256 BK64 2-stage (8 waves of 128x64, one workgroup per CU, N % 256 == 0); 10 = 256x128 BK32
// 3-stage, 64x64 per wave, two workgroups per CU (N % 128 == 0); 11 = 64x128 (waves of 32x64) BK64
// 2-stage).  Returns the previous value, or ES_BAD_ARG (state unchanged) for a family that does not
// exist (the others were measured slower and removed in round 4).
static bool gemm_variant_ok(int v) {
  return v == -1 || v == 0 || v == 1 || v == 2 || v == 5 || v == 6 || v == 10 || v == 11 || v == 12;
}
int es_set_gemm_variant(int v) {
  if (!gemm_variant_ok(v)) return ES_BAD_ARG;
  const int old = g_gemm_variant;
  g_gemm_variant = v;
  return old;
}

// Tuning knob: 1 (default) = the 64 x 128 tile for small token shards in the per-shape rules, 0 = without it.
// Returns the previous value.
int es_set_gemm_small_tile(int v) {
  const int old = g_small_tile;
  g_small_tile = v;
  return old;
}

// Tuning knob for es_gemm_tn: -1 = default, 0 = the 128x128 tile (32-token steps, two stages), 7 = the
// 384x192 tile (64-token steps, two stages; shapes that do not tile fall back to 0).  A pin (>= 0) also
// overrides the variant es_gemm_tn_ex callers name (an A/B run pins every weight gradient).  Returns the
// previous value, or ES_BAD_ARG (state unchanged) for any other value (the other ring depths and step
// sizes were measured slower and removed in round 4).
int es_set_tn_variant(int v) {
  if (v != -1 && v != 0 && v != 7) return ES_BAD_ARG;
  const int old = g_tn_variant;
  g_tn_variant = v;
  return old;
}

// es_gemm_tn kernel choice and split-K sizing (splits <= 0: auto).  Kernels: 0 the 128 x 128
// four-wave tile, 7 the 384 x 192 eight-wave tile (where the shape tiles).  Auto: the big tile
// for long token axes (M >= 65536: 15-25 % faster alone at the F1 shapes, scripts/gemm_bench.py),
// the 128 x 128 tile below that (more tiles to spread a short axis over).  Splits: enough
// workgroups to fill the chip (target), but at least TN_MIN_SPLIT_TOKENS tokens per split -- each
// split writes and the reduction re-reads a full fp32 N1 x N2 slab.  Measured at a per-GPU shard of
// 64 images (M = 12,608, scripts/gemm_bench.py --m-train): 16-24 splits of the 128 x 128 kernel are
// fastest (fc1 / fc2 / qkv / proj weight gradients 44 / 44 / 38 / 28 us; 64 splits of the big tile
// 48 + 26 us of reduction; 4 splits 108 us).
constexpr int TN_MIN_SPLIT_TOKENS = 512;
static bool tn_big_ok(int N1, int N2, int ld1, int ld2) {
  return N1 % TB1 == 0 && N2 % TB2 == 0 && ld1 % 8 == 0 && ld2 % 8 == 0;
}
static int tn_pick(int M, int N1, int N2, int ld1, int ld2, int v) {
  if (!(N1 % BM == 0 && N2 % BN == 0)) return 7;  // only the big tile covers N2 = 192 (caller checked)
  if (v == 7) return tn_big_ok(N1, N2, ld1, ld2) ? 7 : 0;
  if (v >= 0) return 0;
  return (tn_big_ok(N1, N2, ld1, ld2) && M >= 65536) ? 7 : 0;
}
static int tn_target(int v) { return v == 7 ? 256 : 768; }
static int tn_tiles(int v, int N1, int N2) { return v == 7 ? (N1 / TB1) * (N2 / TB2) : (N1 / BM) * (N2 / BN); }
static int tn_auto_splits(int v, int M, int N1, int N2) {
  const int by_fill = std::max(1, tn_target(v) / tn_tiles(v, N1, N2));
  const int by_len = std::max(1, M / TN_MIN_SPLIT_TOKENS);
  return std::min(by_fill, by_len);
}

// workspace floats needed by es_gemm_tn for `splits` splits (slabs + bias partials); splits <= 0:
// the most any kernel choice's automatic split count can use
size_t es_gemm_tn_workspace(int N1, int N2, int splits) {
  if (splits <= 0) {
    splits = std::max(1, 768 / std::max(1, (N1 / BM) * (N2 / BN)));
    if (N1 % TB1 == 0 && N2 % TB2 == 0) splits = std::max(splits, 512 / std::max(1, (N1 / TB1) * (N2 / TB2)));
  }
  return (size_t)splits * N1 * N2 + (size_t)splits * N1;
}

int es_gemm_tn(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
               float* workspace, float* out, int accumulate, float* bias_out, hipStream_t stream) {
  return es_gemm_tn_ex(A1, ld1, A2, ld2, M, N1, N2, splits, workspace, out, accumulate, bias_out, -1, stream);
}

// es_gemm_tn with the kernel chosen by the caller (variant >= 0, as es_set_tn_variant; shapes the
// chosen tile does not cover fall back as there) instead of the default (variant -1); a process-wide pin
// (es_set_tn_variant >= 0, an A/B run) wins over the caller's choice.
int es_gemm_tn_ex(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
                  float* workspace, float* out, int accumulate, float* bias_out, int variant, hipStream_t stream) {
  if (M <= 0 || (ld1 % 8) || (ld2 % 8)) return ES_BAD_SHAPE;
  if (!tn_big_ok(N1, N2, ld1, ld2) && ((N1 % BM) || (N2 % BN))) return ES_BAD_SHAPE;
  if (!A1 || !A2 || !out || !workspace) return ES_BAD_ARG;
  if (variant != -1 && variant != 0 && variant != 7) return ES_BAD_ARG;
  const int v = tn_pick(M, N1, N2, ld1, ld2, g_tn_variant >= 0 ? g_tn_variant : variant);
  const int BKM = v == 7 ? 64 : 32;
  const int msteps = (M + BKM - 1) / BKM;
  if (splits <= 0) splits = tn_auto_splits(v, M, N1, N2);
  splits = std::min(splits, msteps);
  const int per = (msteps + splits - 1) / splits;
  const int S = (msteps + per - 1) / per;
  const bool direct = (S == 1 && !accumulate);
  float* P = direct ? out : workspace;
  float* PB = bias_out ? workspace + (size_t)S * N1 * N2 : nullptr;
  TNArgs a{(const bf16*)A1, (const bf16*)A2, P, PB, M, N1, N2, ld1, ld2, per * BKM};
  const int grid = S * tn_tiles(v, N1, N2);
#define TN_LAUNCH(BKM_, NST_)                                                                           \
  {                                                                                                   \
    const size_t lds = (size_t)NST_ * 2 * BKM_ * BM * 2;                                              \
    allow_lds(gemm_tn_kernel<BKM_, NST_>, lds);                                                       \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_tn_kernel<BKM_, NST_>), dim3(grid), dim3(256), lds, stream, a); \
  }
#define TNB_LAUNCH(BKM_, NST_, ASM_, ...)                                                               \
  {                                                                                                   \
    const size_t lds = (size_t)NST_ * BKM_ * (TB1 + TB2) * 2;                                         \
    allow_lds(gemm_tn_big_kernel<BKM_, NST_, ASM_, ##__VA_ARGS__>, lds);                              \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_tn_big_kernel<BKM_, NST_, ASM_, ##__VA_ARGS__>), dim3(grid), dim3(512), lds, stream, a); \
  }
  switch (v) {
    case 7: TNB_LAUNCH(64, 2, true) break;
    default: TN_LAUNCH(32, 2) break;  // 0
  }
#undef TN_LAUNCH
#undef TNB_LAUNCH
  if (!direct) {
    const int n = N1 * N2;
    int rg = (n / 4 + 255) / 256;
    rg = rg > 2048 ? 2048 : rg;
    hipLaunchKernelGGL(splitk_reduce_kernel, rg, 256, 0, stream, P, out, S, n, accumulate);
  }
  if (bias_out)
    launch_reduce_partials(PB, bias_out, S, N1, accumulate, stream);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// ---- grouped weight gradients (es_tn_problem, include/endossl.h) ----
static_assert(sizeof(TNGroupEntry) == 64, "es_tn_problem layout");
size_t es_tn_problem_size(void) { return sizeof(TNGroupEntry); }

// Validate a host copy of the table and fill its tile0 / mchunk fields; returns the total tile
// count (the grid), or a negative status.
int es_gemm_tn_grouped_prepare(void* host_table, int count) {
  if (!host_table || count <= 0) return ES_BAD_ARG;
  TNGroupEntry* t = (TNGroupEntry*)host_table;
  int tiles = 0;
  for (int i = 0; i < count; ++i) {
    TNArgs& a = t[i].a;
    if (!a.A1 || !a.A2 || !a.P) return ES_BAD_ARG;
    if (a.M <= 0 || a.N1 % BM || a.N2 % BN || a.ld1 % 8 || a.ld2 % 8) return ES_BAD_SHAPE;
    a.mchunk = (a.M + 31) / 32 * 32;
    t[i].tile0 = tiles;
    t[i].pad = 0;
    tiles += (a.N1 / BM) * (a.N2 / BN);
  }
  return tiles;
}

// out_g = dY_g^T X_g (+ bias_g = column sums of dY_g) for every entry of a device table prepared by
// es_gemm_tn_grouped_prepare (same count, total_tiles its return value).  Outputs overwritten.
int es_gemm_tn_grouped(const void* device_table, int count, int total_tiles, hipStream_t stream) {
  if (!device_table || count <= 0 || total_tiles <= 0) return ES_BAD_ARG;
  const size_t lds = (size_t)2 * 2 * 32 * BM * 2;
  allow_lds(gemm_tn_grouped_kernel<32, 2>, lds);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_tn_grouped_kernel<32, 2>), dim3(total_tiles), dim3(256), lds, stream,
                     (const TNGroupEntry*)device_table, count);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// ---- a layer's weight gradients as one split-K launch on the 384 x 192 tile (include/endossl.h) ----
static_assert(sizeof(TNBigEntry) == 72 && sizeof(TNRedEntry) == 32, "grouped big-tile table layout");
// 64-token steps per split when a problem of M tokens gets (at most) S0 splits
static int tn_group_per(int M, int S0) {
  const int msteps = (M + 63) / 64, s = std::min(S0, msteps);
  return (msteps + s - 1) / s;
}
size_t es_gemm_tn_big_grouped_table_bytes(int count) {
  return count <= 0 ? 0 : (size_t)count * (sizeof(TNBigEntry) + 2 * sizeof(TNRedEntry));
}
size_t es_gemm_tn_big_grouped_workspace(const void* problems, int count, int target_wgs) {
  if (!problems || count <= 0) return 0;
  const TNGroupEntry* q = (const TNGroupEntry*)problems;
  int tiles = 0;
  for (int i = 0; i < count; ++i) tiles += (q[i].a.N1 / TB1) * (q[i].a.N2 / TB2);
  const int S0 = std::max(1, target_wgs / std::max(1, tiles));
  size_t f = 0;
  for (int i = 0; i < count; ++i) {
    const int per = tn_group_per(q[i].a.M, S0), S = ((q[i].a.M + 63) / 64 + per - 1) / per;
    if (S > 1) f += (size_t)S * ((size_t)q[i].a.N1 * q[i].a.N2 + (q[i].a.PB ? q[i].a.N1 : 0));
  }
  return f;
}

// Build the device table of es_gemm_tn_big_grouped from `count` es_tn_problem entries (dy, x, out,
// bias_out, M, N1, N2, ld1, ld2; the other fields ignored): splits = target_wgs / (the problems' 384 x 192
// tiles) for every problem (at most one per 64 tokens), slabs and bias partials carved from `workspace`
// in problem order.  Writes TNBigEntry[count] then TNRedEntry[nred] to `table` (es_gemm_tn_big_grouped_
// table_bytes(count) bytes) and {workgroups, reduce blocks, reduce entries} to dims[0..2].
int es_gemm_tn_big_grouped_prepare(const void* problems, int count, int target_wgs, float* workspace,
                                   size_t workspace_floats, void* table, int* dims) {
  if (!problems || count <= 0 || !workspace || !table || !dims || target_wgs <= 0) return ES_BAD_ARG;
  if (count > TNG_MAX) return ES_BAD_SHAPE;
  const TNGroupEntry* q = (const TNGroupEntry*)problems;
  int tiles = 0;
  for (int i = 0; i < count; ++i) {
    const TNArgs& a = q[i].a;
    if (!a.A1 || !a.A2 || !a.P) return ES_BAD_ARG;
    if (a.M <= 0 || !tn_big_ok(a.N1, a.N2, a.ld1, a.ld2)) return ES_BAD_SHAPE;
    tiles += (a.N1 / TB1) * (a.N2 / TB2);
  }
  const int S0 = std::max(1, target_wgs / tiles);
  TNBigEntry* g = (TNBigEntry*)table;
  TNRedEntry* r = (TNRedEntry*)(g + count);
  size_t off = 0;
  int wg = 0, blk = 0, nr = 0;
  for (int i = 0; i < count; ++i) {
    const TNArgs& a = q[i].a;
    const int msteps = (a.M + 63) / 64;
    const int per = tn_group_per(a.M, S0);
    const int S = (msteps + per - 1) / per;
    const size_t nslab = (size_t)a.N1 * a.N2;
    const size_t need = S == 1 ? 0 : (size_t)S * nslab + (q[i].a.PB ? (size_t)S * a.N1 : 0);
    if (off + need > workspace_floats) return ES_BAD_SHAPE;
    // one split: the tile writes the weight and bias gradients in place (no slab, no reduce entry)
    float* P = S == 1 ? (float*)a.P : workspace + off;
    float* PB = q[i].a.PB ? (S == 1 ? q[i].a.PB : P + (size_t)S * nslab) : nullptr;
    off += need;
    const int nt = (a.N1 / TB1) * (a.N2 / TB2);
    g[i].a = TNArgs{a.A1, a.A2, P, PB, a.M, a.N1, a.N2, a.ld1, a.ld2, per * 64};
    g[i].wg0 = wg;
    g[i].ntiles = nt;
    g[i].pad0 = S;
    g[i].pad1 = 0;
    wg += S * nt;
    if (S == 1) continue;
    r[nr] = TNRedEntry{P, (float*)a.P, S, (int)nslab, blk, 0};
    blk += (int)((nslab / 4 + 255) / 256);
    ++nr;
    if (PB) {
      r[nr] = TNRedEntry{PB, q[i].a.PB, S, a.N1, blk, 0};
      blk += (a.N1 / 4 + 255) / 256;
      ++nr;
    }
  }
  dims[0] = wg;
  dims[1] = blk;
  dims[2] = nr;
  return ES_OK;
}

// out_g = dY_g^T X_g and bias_g = column sums of dY_g (both overwritten) for every problem of the
// (host) table es_gemm_tn_big_grouped_prepare wrote: the split-K GEMM launch, then one reduce launch
// over every problem's slabs and bias partials.  The table is passed by value in the kernel arguments.
static int tn_big_grouped_launch(const void* table, int count, const int* dims, hipStream_t stream, hipEvent_t e0,
                                 hipEvent_t e1) {
  if (!table || count <= 0 || !dims || dims[0] <= 0 || dims[1] < 0 || dims[2] < 0) return ES_BAD_ARG;
  if (count > TNG_MAX || dims[2] > 2 * TNG_MAX) return ES_BAD_SHAPE;
  const TNBigEntry* g = (const TNBigEntry*)table;
  TNBigTable bt{};
  for (int i = 0; i < count; ++i) bt.e[i] = g[i];
  bt.ng = count;
  // with events: hipExtLaunchKernelGGL stamps them at the kernels' own start / end (what rocprofv3's kernel
  // trace reports), not where the stream reaches a hipEventRecord
#define TNG_LAUNCH(BKM_, NST_)                                                                              \
  {                                                                                                       \
    const size_t lds = (size_t)NST_ * BKM_ * (TB1 + TB2) * 2;                                             \
    allow_lds(gemm_tn_big_grouped_kernel<BKM_, NST_>, lds);                                               \
    if (e0 || e1)                                                                                         \
      hipExtLaunchKernelGGL(HIP_KERNEL_NAME(gemm_tn_big_grouped_kernel<BKM_, NST_>), dim3(dims[0]), dim3(512), \
                            (uint32_t)lds, stream, e0, dims[2] > 0 ? nullptr : e1, 0, bt);                \
    else                                                                                                  \
      hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_tn_big_grouped_kernel<BKM_, NST_>), dim3(dims[0]), dim3(512), lds, \
                         stream, bt);                                                                     \
  }
  TNG_LAUNCH(64, 2)
#undef TNG_LAUNCH
  if (dims[2] > 0) {
    TNRedTable rt{};
    const TNRedEntry* r = (const TNRedEntry*)(g + count);
    for (int i = 0; i < dims[2]; ++i) rt.r[i] = r[i];
    rt.nr = dims[2];
    if (e1)
      hipExtLaunchKernelGGL(splitk_reduce_grouped_kernel, dim3(dims[1]), dim3(256), 0, stream, nullptr, e1, 0, rt);
    else
      hipLaunchKernelGGL(splitk_reduce_grouped_kernel, dim3(dims[1]), dim3(256), 0, stream, rt);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_gemm_tn_big_grouped(const void* table, int count, const int* dims, hipStream_t stream) {
  return tn_big_grouped_launch(table, count, dims, stream, nullptr, nullptr);
}

// es_gemm_tn_big_grouped with timing: `start` takes the grouped kernel's start, `stop` the end of the reduce
// launch (or of the kernel when there is none).  Events from es_event_create.
int es_gemm_tn_big_grouped_timed(const void* table, int count, const int* dims, void* start, void* stop,
                                 hipStream_t stream) {
  if (!start || !stop) return ES_BAD_ARG;
  return tn_big_grouped_launch(table, count, dims, stream, (hipEvent_t)start, (hipEvent_t)stop);
}

// timing events for the *_timed launches: created with timing enabled; elapsed = stop - start in ms after the
// stop event completed (it waits for it)
int es_event_create(void** ev) {
  if (!ev) return ES_BAD_ARG;
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return ES_HIP_ERROR;
  *ev = (void*)e;
  return ES_OK;
}

int es_event_elapsed(void* start, void* stop, float* ms) {
  if (!start || !stop || !ms) return ES_BAD_ARG;
  if (hipEventSynchronize((hipEvent_t)stop) != hipSuccess) return ES_HIP_ERROR;
  return hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop) == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_event_destroy(void* ev) {
  if (!ev) return ES_BAD_ARG;
  return hipEventDestroy((hipEvent_t)ev) == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_splitk_reduce(const float* P, float* out, int S, int n, int accumulate, hipStream_t stream) {
  if (n % 4 || S <= 0) return ES_BAD_SHAPE;
  int rg = (n / 4 + 255) / 256;
  rg = rg > 2048 ? 2048 : rg;
  hipLaunchKernelGGL(splitk_reduce_kernel, rg, 256, 0, stream, P, out, S, n, accumulate);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// bias gradient: out[n] (+)= sum_m Y[m][n]; workspace >= blocks*N floats.  N % 8 == 0, N <= 2048.
int es_colsum(const void* Y, int ld, int M, int N, float* workspace, int blocks, float* out, int accumulate,
              hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 8 || N > 2048 || ld % 8 || blocks <= 0) return ES_BAD_SHAPE;
  if (!Y || !workspace || !out) return ES_BAD_ARG;
  const int rows_per = (M + blocks - 1) / blocks;
  const int G = (M + rows_per - 1) / rows_per;
  hipLaunchKernelGGL(colsum_partial_kernel, G, 256, 0, stream, (const bf16*)Y, ld, M, N, rows_per, workspace);
  launch_reduce_partials(workspace, out, G, N, accumulate, stream);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// out[n] (+)= sum_g P[g][n]  (partials of the LayerNorm / colsum kernels)
int es_reduce_partials(const float* P, float* out, int G, int N, int accumulate, hipStream_t stream) {
  if (G <= 0 || N <= 0) return ES_BAD_SHAPE;
  launch_reduce_partials(P, out, G, N, accumulate, stream);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

}  // extern "C"
