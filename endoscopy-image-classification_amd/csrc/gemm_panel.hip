// Activation-stationary bf16 MFMA GEMM for the K = 384 Linear layers of the ViT-S step (gfx950).
//
//   C[M, N] = A[M, 384] . B[N, 384]^T (+ the gemm.hip epilogues), B = a weight image (W or W^T)
//
// Replaces, for K = 384, the reference's aten::addmm of the qkv / fc1 Linear forwards and of the fc2 / proj
// data gradients (code/models/conformer.py:13-23,35-50 via timm's Block).
//
// Why a different kernel family for K = 384: the output-tiled kernels of gemm.hip
// re-stream both operands through LDS for every output tile.  At K = 384 a 256 x 128 tile brings 85 FLOP
// per LDS-DMA byte, so the qkv forward moved 1.05 GB from L2 into LDS for 89 GFLOP.  Here the ACTIVATION
// rows stay in registers for the whole K: each wave holds 32 rows x 384 of A as MFMA fragments (96 VGPRs,
// loaded once from HBM) and the workgroup walks every output column of its 128-row panel, streaming the
// weight (L2-resident, <= 1.2 MB) through an LDS ring in 32-column chunks.  A is read from HBM exactly
// once, C written exactly once; the LDS-DMA stream is the weight alone.  Each chunk's epilogue runs one
// step late, after the next chunk's MFMAs, so a wave's stores and VALU work sit beside the other
// workgroup's matrix work on the same SIMDs.
//
// Layout: 512 threads = 8 waves (two per SIMD), one workgroup per CU: a 256-row panel, so every weight chunk
// brought into LDS feeds 256 rows (qkv forward: 0.35 GB of LDS-DMA per launch).  Persistent grid: the
// (panel, chunk) steps are cut into equal contiguous ranges, one per workgroup; adjacent ranges share their
// boundary panel and run in opposite directions (they reach it at the same time, on one XCD).
//
// MFMA v_mfma_f32_16x16x32_bf16 with the weight fragment as the A operand: lane (g, r) accumulates
// C[row0 + r][col0 + perm(16 nt + 4 g + i)].  The chunk's weight rows are stored in LDS permuted so that
// perm(16 nt + 4 g + i) = 8 g + 4 nt + i: a lane's two 16 x 16 tiles are EIGHT CONSECUTIVE output columns,
// so every output leaves as one 16-B (bf16) or two 16-B (fp32) stores per lane and row, and every epilogue
// operand arrives the same way.  Weight chunk in LDS: 12 k-blocks of [32 rows][64 B] (hsw below: conflict-free
// ds_read_b128 fragment reads under gfx950's 16-lane groups, MI355X_MICROARCH.md §LDS, at kk-independent lane
// addresses), then the chunk's 32 bias values.
//
// Memory-counter discipline.  Every global load inside the loop is LDS-DMA issued as inline asm
// (glds16_asm): the weight chunk (shared: barrier) and the epilogue's aux rows (per wave: each lane later
// reads back exactly the 16 B it fetched).  The compiler sees none of them, and a wave retires them with
// counted waits computed from a running count of the vector-memory operations it has issued, so no wait
// ever covers more than the operation it is for: a store's write-back latency (~1-3 us under load) never
// enters the step's critical path.  The A rows are the only compiler-visible loads: they are issued after a
// segment's last MFMAs and drained (vmcnt(0), a wait the compiler's bookkeeping sees) at the panel switch.
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace es_panel {

enum {
  EPI_BF16 = 0, EPI_GELU = 1, EPI_F32_RESID = 2, EPI_DGELU = 3, EPI_F32 = 4, EPI_PATCH = 5,
  EPI_GELU_ACT = 6, EPI_GELU_D = 7, EPI_MULAUX = 8
};

constexpr int KT = 12;             // K / 32
constexpr int ROWB = KT * 64;      // LDS bytes of one weight row (768)
constexpr int WAVES = 8;
constexpr int RW = 32;             // activation rows per wave
constexpr int PANEL = WAVES * RW;  // 256
constexpr int NC = 32;             // output columns per step
constexpr int WB = NC * ROWB;      // weight bytes of a step (24 KiB)
constexpr int SLOT = WB + NC * 4;  // + the step's bias
constexpr int PD = WB / 1024 / WAVES;  // weight LDS-DMA pieces per wave per step (3)

struct PArgs {
  const bf16* A; const bf16* B; const float* bias;
  void* C; void* C2; const void* aux;
  int M, N, lda, ldb, ldc, ldaux;
  int CH;  // chunks per panel (N / NC)
  int S;   // steps = panels x CH
};

template <int EPI>
constexpr bool f32_out() { return EPI == EPI_F32 || EPI == EPI_F32_RESID; }
template <int EPI>
constexpr int aux_pieces() {  // per wave per step: 16-B aux loads per lane (bf16: 8 values, fp32: 4)
  return EPI == EPI_F32_RESID ? 4 : ((EPI == EPI_MULAUX || EPI == EPI_DGELU) ? 2 : 0);
}
template <int EPI>
constexpr int stores_per_row() {  // 16-B C stores per lane per 16-row tile
  return (EPI == EPI_GELU || EPI == EPI_GELU_D || f32_out<EPI>()) ? 2 : 1;
}
// ring depth: three weight slots (plus two per-wave aux stages when the epilogue reads aux rows)
template <int EPI>
constexpr int ring_of() { return 3; }
template <int EPI>
constexpr int lds_bytes() { return ring_of<EPI>() * SLOT + 2 * WAVES * aux_pieces<EPI>() * 1024; }

__device__ __forceinline__ u32x4 pack8(const float* v) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)v[i];
  return __builtin_bit_cast(u32x4, o);
}

// k-block-major weight chunk: the 16 B of k-chunk (4 kk + g) of LDS row q at kk * 2048 + q * 64 +
// (g ^ hsw(q)) * 16.  With hsw = [0, 2, 3, 1] over (q >> 2) & 3 the 16 lanes of every ds_read_b128 lane group
// ({0-3, 12-15, 20-27}, ...) hit 16 distinct 16-B bank slots, and the lane's address is kk-independent: the
// k-step and tile offsets are instruction immediates.
__device__ __forceinline__ int hsw(int q) { return (0x78 >> (2 * ((q >> 2) & 3))) & 3; }

// PROBE (measurement only, variants 41..44): 1 no epilogue stores, 2 no weight DMA in the loop, 3 no barrier,
// 4 no fragment reads / MFMAs
template <int EPI, int STAUX, int PROBE = 0>
__global__ __launch_bounds__(512, 2) void gemm_panel_kernel(PArgs p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int R = ring_of<EPI>();
  constexpr int PA = aux_pieces<EPI>();
  constexpr bool F32O = f32_out<EPI>();
  constexpr int ESZ = F32O ? 4 : 2;
  constexpr int EST = 2 * stores_per_row<EPI>();  // stores per lane per step (two 16-row tiles)
  char* const auxs = smem + R * SLOT;              // per-wave aux stages: [stage][wave][PA KiB]
  const int G = gridDim.x;
  const int wl = xcd_remap(blockIdx.x, G);
  const int s0 = (int)(((long long)wl * p.S) / G), s1 = (int)(((long long)(wl + 1) * p.S) / G);
  const int n = s1 - s0;
  if (n <= 0) return;
  const bool rev = wl & 1;  // odd ranges walk backwards: they meet their left neighbour at the shared panel
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int fo = r * 64 + ((g ^ hsw(r)) << 4);  // the lane's fragment offset within a k-block

  const __amdgpu_buffer_rsrc_t ra = buf_rsrc(p.A, (unsigned)p.M * p.lda * 2u);
  const __amdgpu_buffer_rsrc_t rc = buf_rsrc(p.C, (unsigned)p.M * p.ldc * ESZ);
  const __amdgpu_buffer_rsrc_t rc2 = buf_rsrc((EPI == EPI_GELU || EPI == EPI_GELU_D) ? p.C2 : p.C,
                                              (unsigned)p.M * p.ldc * ESZ);

  // weight-chunk DMA: piece j of wave w covers the slot's 16-B units L = (j * 4 + w) * 64 + lane; unit L is
  // k-block kk = L / 128, LDS row q = (L % 128) / 4 (weight row perm(q)), position u = L % 4, which holds the
  // k-chunk 4 kk + (u ^ hsw(q))
  unsigned ob[PD];  // byte offsets within a chunk's weight rows
#pragma unroll
  for (int j = 0; j < PD; ++j) {
    const int L = (j * WAVES + w) * 64 + lane, kk = L >> 7, q = (L >> 2) & 31, u = L & 3;
    const int row = 8 * ((q >> 2) & 3) + 4 * (q >> 4) + (q & 3);
    ob[j] = (unsigned)(row * p.ldb + (4 * kk + (u ^ hsw(q))) * 8) * 2u;
  }
  const i32x4 rB = rsrc_i4(p.B, (unsigned)p.N * p.ldb * 2u);
  // a null bias: a zero-size resource, every piece reads zeros
  const i32x4 rBias = rsrc_i4(p.bias ? (const void*)p.bias : (const void*)p.B, p.bias ? (unsigned)p.N * 4u : 0u);
  constexpr int AESZ = PA == 4 ? 4 : 2;  // aux element bytes
  const i32x4 rX = rsrc_i4(PA ? p.aux : (const void*)p.B, PA ? (unsigned)p.M * p.ldaux * AESZ : 0u);

  // Step descriptors, advanced incrementally (no divisions in the loop): chunk and panel of a step.
  struct Pos { int ch, panel; };
  auto adv = [&](Pos q) {
    if (!rev) return q.ch + 1 == p.CH ? Pos{0, q.panel + 1} : Pos{q.ch + 1, q.panel};
    return q.ch == 0 ? Pos{p.CH - 1, q.panel - 1} : Pos{q.ch - 1, q.panel};
  };
  const int sf = rev ? s1 - 1 : s0;
  const Pos first{sf % p.CH, sf / p.CH};

  int issued = 0;  // vector-memory operations this wave has issued (loads, DMA, stores): the slow-path waits
  // the weight chunk + bias of a step into slot `slot`: one asm block, M0 stepped by 4 KiB between the pieces
  auto issue_w = [&](Pos q, int slot) {
    const unsigned so = (unsigned)(q.ch * NC * p.ldb) * 2u;
    const unsigned dst = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)(smem + slot * SLOT + w * 1024));
    static_assert(PD == 3 && WAVES == 8, "issue_w pieces");
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %4, %6 offen lds\n\ts_add_u32 m0, m0, 8192\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %2, %4, %6 offen lds\n\ts_add_u32 m0, m0, 8192\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %3, %4, %6 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(ob[0]), "v"(ob[1]), "v"(ob[2]), "s"(rB), "s"(dst), "s"(so)
        : "memory", "scc");
    // 128 B of bias from lanes 0..7 (the same bytes from every wave)
    if (lane < 8) bl16_asm(rBias, lane * 16u, (unsigned)(q.ch * NC) * 4u, smem + slot * SLOT + WB);
    issued += PD + 1;
  };
  // the aux rows of a step's epilogue: lane (g, r) fetches row (16 mt + r), columns 8 g .. + 8 (bf16) or
  // 8 g + 4 h .. + 4 (fp32, h = 0, 1) into its own 16 B of the wave's stage (rows past M are out of the
  // resource's range: zeros, their outputs dropped)
  auto lane_row = [&](int panel, int mt, int ld, int esz) {
    const int m = panel * PANEL + w * RW + 16 * mt + r;
    return m < p.M ? (unsigned)(m * ld + 8 * g) * (unsigned)esz : ES_OOB;
  };
  auto issue_aux = [&](Pos q, int stage) {
    if constexpr (PA > 0) {
      char* dst = auxs + (stage * WAVES + w) * PA * 1024;
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int mt = PA == 2 ? j : (j >> 1), h = PA == 2 ? 0 : (j & 1);
        bl16_asm(rX, lane_row(q.panel, mt, p.ldaux, AESZ) + 16u * h, (unsigned)(q.ch * NC) * AESZ, dst + j * 1024);
      }
      issued += PA;
    }
  };

  // A fragments: a[mt][kk] = A[row0 + 16 mt + r][32 kk + 8 g .. + 8]
  bf16x8 a[2][KT];
  auto load_a = [&](int panel) {
    const int m0 = panel * PANEL + w * RW;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = m0 + mt * 16 + r;
      const unsigned base = m < p.M ? (unsigned)(m * p.lda + 8 * g) * 2u : ES_OOB;
#pragma unroll
      for (int kk = 0; kk < KT; ++kk) a[mt][kk] = __builtin_bit_cast(bf16x8, buf_load16(ra, base + kk * 64u));
    }
    issued += 2 * KT;
  };

  // the epilogue of a step (q) from its accumulators, the bias values the lane read from its slot, and the
  // wave's aux stage (a segment's last epilogue runs in the next segment's first step: its rows come from q)
  auto epilogue = [&](Pos q, const f32x4 (&acc)[2][2], const f32x4 (&bias)[2], int stage) {
    const unsigned cofs = (unsigned)(q.ch * NC) * (unsigned)ESZ;
    const char* as = auxs + (stage * WAVES + w) * PA * 1024 + lane * 16;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const unsigned off = lane_row(q.panel, mt, p.ldc, ESZ) + cofs;
      const f32x4 v0 = acc[mt][0] + bias[0], v1 = acc[mt][1] + bias[1];
      float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      auto st = [&](__amdgpu_buffer_rsrc_t rr, unsigned o, u32x4 d) {
        if constexpr (PROBE == 1) {
          if (d[0] == 0x12345u && d[1] == 0x777u) __builtin_amdgcn_raw_buffer_store_b128(d, rr, o, 0, STAUX);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(d, rr, o, 0, STAUX);
        }
      };
      if constexpr (EPI == EPI_BF16) {
        st(rc, off, pack8(v));
      } else if constexpr (EPI == EPI_F32) {
        st(rc, off, __builtin_bit_cast(u32x4, v0));
        st(rc, off + 16, __builtin_bit_cast(u32x4, v1));
      } else if constexpr (EPI == EPI_F32_RESID) {
        const f32x4 x0 = *(const f32x4*)(as + (2 * mt) * 1024), x1 = *(const f32x4*)(as + (2 * mt + 1) * 1024);
        st(rc, off, __builtin_bit_cast(u32x4, v0 + x0));
        st(rc, off + 16, __builtin_bit_cast(u32x4, v1 + x1));
      } else if constexpr (EPI == EPI_MULAUX || EPI == EPI_DGELU) {
        const bf16x8 qq = *(const bf16x8*)(as + mt * 1024);
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = EPI == EPI_MULAUX ? v[i] * (float)qq[i] : v[i] * gelu_grad_f((float)qq[i]);
        st(rc, off, pack8(o));
      } else {  // GELU family: the same packed routine as gemm.hip's epilogues (bit-identical outputs)
        float gv[8], dv[8];
        gelu_and_grad_f8(v, gv, dv);
        if constexpr (EPI == EPI_GELU_ACT) {
          st(rc, off, pack8(gv));
        } else if constexpr (EPI == EPI_GELU_D) {
          st(rc, off, pack8(dv));
          st(rc2, off, pack8(gv));
        } else {  // EPI_GELU: pre-activation + activation
          st(rc, off, pack8(v));
          st(rc2, off, pack8(gv));
        }
      }
    }
    issued += EST;
  };

  // Steady-state wait counts (every step of the window issued all its operations), per step k in issue
  // order [DMA(k + R - 1): PD + 1][aux(k): PA][MFMAs][epilogue(k - 1): EST]:
  //   DMA(k), issued in step k - R + 1: R = 3: aux(k - 2) + epi(k - 3) + DMA(k + 1) + aux(k - 1) + epi(k - 2);
  //                                     R = 2: aux(k - 1) + epi(k - 2)
  //   aux(k - 1), issued in step k - 1: epi(k - 2) + DMA(k + R - 1) + aux(k)
  constexpr int NW = R == 3 ? 2 * PA + 2 * EST + PD + 1 : PA + EST;
  constexpr int NX = EST + PD + 1 + PA;
  static_assert(NW <= 63 && NX <= 63, "vmcnt");
  int mw0 = 0, mw1 = 0, mx = 0;  // slow path: `issued` after DMA(k), DMA(k + 1) (R = 3), aux(k - 1)

  // one step k at position qk (qe: position of step k - 1, qd: of step k + R - 1).  FIRST (compile-time): step
  // 0, no epilogue before it -- no compiler-visible load and its wait sit on different conditional paths
  // (the compiler's wait bookkeeping is path-insensitive).  accC / biasC: this step's; accP / biasP: the
  // previous step's (two register sets, alternated by the caller: no copies).
  auto step = [&](auto first_tag, int k, Pos qk, Pos qe, Pos qd, f32x4 (&accC)[2][2], f32x4 (&accP)[2][2],
                  f32x4 (&biasC)[2], f32x4 (&biasP)[2]) {
    constexpr bool FIRST = decltype(first_tag)::value;
    const bool steady = k >= R + 1 && k + R - 2 < n;
    if (steady) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NW) : "memory");
    else wait_vmcnt_any(min(issued - mw0, 63));  // this wave's pieces of DMA(k); the barrier: every wave's
    if constexpr (PROBE != 3) __builtin_amdgcn_s_barrier();
    if (PROBE != 2 && k + R - 1 < n) issue_w(qd, (k + R - 1) % R);  // slot (k - 1) % R: read in step k - 1, which all left
    if constexpr (R == 3) {
      mw0 = mw1;
      mw1 = issued;
    } else {
      mw0 = issued;
    }
    const int mx_prev = mx;
    issue_aux(qk, k & 1);
    mx = issued;
    const char* Bs = smem + (k % R) * SLOT + fo;
    {  // the bias of this step's columns (the lane's eight): DMA(k + R) reuses the slot before the epilogue
      const char* bs = smem + (k % R) * SLOT + WB + 32 * g;
      biasC[0] = *(const f32x4*)bs;
      biasC[1] = *(const f32x4*)(bs + 16);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) accC[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fragments two k-steps ahead (three register sets); the group barriers pin the order [2 fragment reads
    // of step kk + 2][4 MFMAs of step kk]
    bf16x8 b[3][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) b[kk][nt] = *(const bf16x8*)(Bs + kk * 2048 + nt * 1024);
#pragma unroll
    for (int kk = 0; kk < (PROBE == 4 ? 0 : KT); ++kk) {
      if (kk + 2 < KT) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) b[(kk + 2) % 3][nt] = *(const bf16x8*)(Bs + (kk + 2) * 2048 + nt * 1024);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) accC[mt][nt] = mfma16(b[kk % 3][nt], a[mt][kk], accC[mt][nt]);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!FIRST) {
      if constexpr (PA > 0) {  // this wave's aux(k - 1)
        if (k >= 2 && k + R - 1 < n) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NX) : "memory");
        else wait_vmcnt_any(min(issued - mx_prev, 63));
      }
      epilogue(qe, accP, biasP, (k - 1) & 1);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  f32x4 acc0[2][2], acc1[2][2], bias0[2], bias1[2];
  // panel segments: a segment's rows are loaded into registers at its first step and drained with a wait the
  // compiler sees (vmcnt(0)), so no A load is pending inside the steps.  (Loading the next panel's rows
  // during the previous segment's last step needs 96 more registers than two waves per SIMD leave.)
  // Positions: qe (step k - 1), qk (k), q1 (k + 1), q2 (k + 2); the DMA of step k targets k + R - 1.
  Pos qe = first, qk = first, q1 = adv(first), q2 = adv(q1);
  int panel = qk.panel;
  load_a(panel);
  issue_w(qk, 0);
  mw0 = issued;
  if constexpr (R == 3) {
    if (n > 1) issue_w(q1, 1);
    mw1 = issued;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  step(T_{}, 0, qk, qe, R == 3 ? q2 : q1, acc0, acc1, bias0, bias1);
  for (int k = 1; k < n; ++k) {
    qe = qk;
    qk = q1;
    q1 = q2;
    q2 = adv(q2);
    if (qk.panel != panel) {
      panel = qk.panel;
      load_a(panel);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    }
    const Pos qd = R == 3 ? q2 : q1;
    if (k & 1) step(F_{}, k, qk, qe, qd, acc1, acc0, bias1, bias0);
    else step(F_{}, k, qk, qe, qd, acc0, acc1, bias0, bias1);
  }
  if constexpr (PA > 0) wait_vmcnt_any(min(issued - mx, 63));
  if ((n - 1) & 1) epilogue(qk, acc1, bias1, (n - 1) & 1);
  else epilogue(qk, acc0, bias0, (n - 1) & 1);
}

}  // namespace es_panel

// C-ABI-internal launcher for es_gemm_nt (gemm.hip): K must be 384, N a multiple of 32.  Returns an
// EsStatus; ES_BAD_SHAPE when the shape or epilogue is not covered (the caller then uses another kernel).
extern "C" int es_panel_gemm(int epi, const void* A, int lda, const void* B, int ldb, const float* bias, void* C,
                             int ldc, void* C2, const void* aux, int ldaux, int M, int N, int K, int stores_nt,
                             hipStream_t stream) {
  const int probe = stores_nt >= 41 ? stores_nt - 40 : 0;
  using namespace es_panel;
  if (K != KT * 32 || N % NC || M <= 0 || (lda % 8) || (ldb % 8) || (ldc % 8) || (ldaux % 8)) return ES_BAD_SHAPE;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  PArgs a{(const bf16*)A, (const bf16*)B, bias, C, C2, aux, M, N, lda, ldb, ldc, ldaux, N / NC, 0};
  a.S = ((M + PANEL - 1) / PANEL) * a.CH;
  const int grid = std::min(cus, a.S);
#define PL(E, X)                                                                                       \
  {                                                                                                    \
    allow_lds(gemm_panel_kernel<E, X>, lds_bytes<E>());                                                \
    hipLaunchKernelGGL(HIP_KERNEL_NAME(gemm_panel_kernel<E, X>), dim3(grid), dim3(512), lds_bytes<E>(), stream, a); \
    break;                                                                                             \
  }
#define PLE(E) \
  if (stores_nt) PL(E, 2) else PL(E, 0)
  if (probe) {  // measurement variants 41..44 (EPI_BF16 only)
    constexpr int E = EPI_BF16;
    auto go = [&](auto kern) {
      allow_lds(kern, lds_bytes<E>());
      hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds_bytes<E>(), stream, a);
    };
    if (probe == 1) go(gemm_panel_kernel<E, 2, 1>);
    else if (probe == 2) go(gemm_panel_kernel<E, 2, 2>);
    else if (probe == 3) go(gemm_panel_kernel<E, 2, 3>);
    else go(gemm_panel_kernel<E, 2, 4>);
    return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
  }
  switch (epi) {
    case EPI_BF16: PLE(EPI_BF16)
    case EPI_F32: PLE(EPI_F32)
    case EPI_GELU: PLE(EPI_GELU)
    case EPI_GELU_ACT: PLE(EPI_GELU_ACT)
    case EPI_GELU_D: PLE(EPI_GELU_D)
    case EPI_MULAUX: PLE(EPI_MULAUX)
    case EPI_DGELU: PLE(EPI_DGELU)
    case EPI_F32_RESID: PLE(EPI_F32_RESID)
    default: return ES_BAD_SHAPE;
  }
#undef PLE
#undef PL
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}
