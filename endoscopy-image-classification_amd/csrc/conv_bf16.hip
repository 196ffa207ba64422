// bf16-operand MFMA convolutions for the Conformer CNN branch at ViT-B scale (SURVEY.md §8(a) a20;
// code/models/conformer.py:75-200 ConvBlock / FCUDown / FCUUp / trans_patch_conv Conv2d calls).
//
//  es_conv2d_pack_bf16              weights [Cout][Cin][kh][kw] fp32 -> wp [Cout][kh kw][Cin] bf16
//                                   (forward operand) and / or wt [Cin][kh kw][Cout] bf16 (data grad)
//  es_conv2d_fwd_bf16               y (+)= conv(x)              implicit GEMM, rows = output pixels
//  es_conv2d_bwd_data_bf16          dx (+)= conv^T(dy)          implicit GEMM per stride phase
//  es_conv2d_bwd_weight_bf16        dw (+)= sum_pixels dy x im2col(x)   split over pixels + reduce
//
// Numerical contract (the transformer GEMMs' one): the conv OPERANDS -- the gathered activation /
// gradient tile and the weights -- are bf16 (rounded as they are staged into LDS when the map is fp32),
// products accumulate in fp32 on v_mfma_f32_16x16x32_bf16 (8x the fp32 MFMA rate conv.hip's kernels run
// at).  The maps themselves are fp32 or bf16 per operand (the _ex entry points' flags): the Conformer's
// CNN branch keeps its activation and gradient maps in bf16 when every conv of the branch runs here
// (conformer.NativeConformer.map_bf16), halving the map traffic of the HBM-bound 1x1 convs and
// BatchNorms; outputs are rounded once from the fp32 accumulators (an accumulating store adds in fp32
// and rounds once).  BatchNorm statistics in the epilogue come from the fp32 accumulators.  The fp32
// kernels of conv.hip remain the parity mode and the path for convs these do not take (channel
// counts not multiples of 32: the 3-channel stem, Conformer-Ti's 16-channel bottlenecks).
//
// Tiling.  Forward / data grad: 128 output pixels x BN (64 | 128) output channels per 256-thread
// workgroup, 4 waves 2 x 2 (64 x BN/2 each), 32-deep K steps that each cover ONE kernel tap and 32
// consecutive channels (C % 32 == 0), so a step's gather is one 128-byte channel run per pixel:
// two threads per pixel, four 16-byte loads each, converted to bf16 and written to a 64-byte LDS
// row (XOR-swizzled 16-byte chunks: conflict-free ds_read_b128 fragment reads).  The next step's
// gathers are issued before this step's MFMAs (register double buffering, two LDS stages, one
// barrier per step).  Weight gradient: a TN product over pixels -- 32-pixel steps, dy and im2col(x)
// tiles stored pixel-major ([32 rows][256 B], the TN GEMM's swizzle) and read as transposed
// fragments (ds_read_b64_tr_b16); fp32 partial slabs per pixel split, reduced in a fixed order.
#include "common.h"

namespace {

// 64-byte rows (32 bf16): chunk c of row r at c ^ ((-(r >> 2)) & 3) (gemm.hip swz64)
__device__ __forceinline__ int cswz64(int r, int c) { return c ^ ((4 - ((r >> 2) & 3)) & 3); }
// 256-byte rows read transposed (gemm.hip swz256)
__device__ __forceinline__ int cswz256(int r, int c) { return c ^ (((r & 3) << 1) | (((r >> 3) & 1) << 3)); }

__device__ __forceinline__ u32x4 f8_to_bf16x8(f32x4 a, f32x4 b) {
  bf16x8 o;
  o[0] = (bf16)a[0]; o[1] = (bf16)a[1]; o[2] = (bf16)a[2]; o[3] = (bf16)a[3];
  o[4] = (bf16)b[0]; o[5] = (bf16)b[1]; o[6] = (bf16)b[2]; o[7] = (bf16)b[3];
  return __builtin_bit_cast(u32x4, o);
}

// 4 map elements by a range-checked buffer load (out-of-range offsets read zeros): no branch around the load
template <typename T> __device__ __forceinline__ typename Q4<T>::t q4_buf_load(__amdgpu_buffer_rsrc_t r, unsigned off);
template <> __device__ __forceinline__ f32x4 q4_buf_load<float>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
template <> __device__ __forceinline__ bf16x4 q4_buf_load<bf16>(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
}

struct NTConv {
  const void* src;    // gathered operand (fp32 or bf16 map): x (forward) or dy (data grad), channel stride 1
  const bf16* wp;     // packed weights [Ncol][kh kw][C]
  const float* bias;  // [Ncol] or null
  void* out;          // fp32 or bf16 map
  int N, C, Ncol, Hs, Ws;  // C = gathered channels (Cin | Cout), Ncol = output channels (Cout | Cin)
  long ssn, ssh, ssw;
  int kh, kw, s, p;
  int Ho, Wo;  // output map dims: forward y (Ho, Wo); data grad x (H, W)
  long osn, osh, osw;
  int accumulate;
  float* stats;  // forward only, nullable: per 128-pixel block [sum | M2] of every output channel
  // forward only (INBN): the gathered map is a train-mode BatchNorm's INPUT; each in-range gathered channel
  // quad becomes relu(bn_affine(x)) in the map's type -- the normalised map itself is never written
  const float* bnm; const float* bnr; const float* bng; const float* bnb;
  // the output pixel m lives at out + m * osw (a dense NHWC map and no stride phase): the epilogue skips the
  // per-row (n, h, w) decomposition -- four integer divisions by run-time values per stored row
  int olin;
  // the gathered map's and the packed weights' byte extents when both are under 2 GiB (else 0): the staged
  // kernel's gathers are then branch-free buffer loads (out-of-range offsets read zeros)
  unsigned sbytes, wbytes;
};

constexpr int NT_BM = 128, NT_BK = 32;

// sum over the 16 lanes of each row of 16 (every lane gets its row's sum): DPP quad swaps, then the half-row and
// row mirrors -- the same pairwise tree for every lane, no LDS traffic (__shfl_xor is ds_bpermute_b32)
__device__ __forceinline__ float row16_sum(float t) {
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0xB1, 0xF, 0xF, true));  // [1,0,3,2]
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x4E, 0xF, 0xF, true));  // [2,3,0,1]
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x141, 0xF, 0xF, true));  // half mirror
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x140, 0xF, 0xF, true));  // row mirror
  return t;
}

// The forward / data-grad epilogue shared by the register-staged and the ring kernels: BatchNorm statistics of
// the tile (forward, STATS), then the outputs through LDS as whole-row quads.
template <int BN, bool DX, bool STATS, typename TO>
__device__ __forceinline__ void nt_tail(const NTConv& a, f32x4 (&acc)[4][BN / 32], int M, int m0, int n0, int Hm,
                                        int Wm, int om, int oa0, int ob0, char* smem) {
  constexpr int NF = BN / 32;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int wm = w >> 1, wn = w & 1;
  // BatchNorm statistics of this tile (forward, STATS: a separate instantiation, so the plain
  // forward keeps its registers): per output channel the block's sum and its
  // centred sum of squares M2 over the valid pixels of the 128-pixel block (Chan's parallel form;
  // es_bn2d_fwd_partials combines the blocks).  Lane (g, r) holds rows wm 64 + 16 i + r of the 4
  // channels wn BN/2 + 16 j + 4 g + q: sums over i in-lane, over r by xor shuffles within each
  // 16-lane group, over the two row waves (wm) through LDS.
  if constexpr (STATS && !DX) {
    // the bias shifts a channel's values uniformly: M2 is computed on the accumulators alone and the
    // sum gets nb bias[col] added once (no per-lane bias registers: the plain instantiation's occupancy)
    float* red = (float*)smem;  // [2 (wm)][BN] partial sums, then [2][BN] partial M2
    const int nb = min(NT_BM, M - m0);
    bool rv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) rv[i] = m0 + wm * 64 + i * 16 + r < M;
    float mu[NF][4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float t = 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = pass == 0 ? acc[i][j][q] : acc[i][j][q] - mu[j][q];
            t += rv[i] ? (pass == 0 ? d : d * d) : 0.f;
          }
          t = row16_sum(t);
          if (r == 0) red[wm * BN + wn * (BN / 2) + j * 16 + 4 * g + q] = t;
        }
      __syncthreads();
      const bool wr = tid < BN && n0 + tid < a.Ncol;
      if (pass == 0) {
#pragma unroll
        for (int j = 0; j < NF; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int cl = wn * (BN / 2) + j * 16 + 4 * g + q;
            mu[j][q] = (red[cl] + red[BN + cl]) / (float)nb;
          }
        if (wr)
          a.stats[(long)blockIdx.x * 2 * a.Ncol + n0 + tid] =
              red[tid] + red[BN + tid] + (a.bias ? (float)nb * a.bias[n0 + tid] : 0.f);
        __syncthreads();
      } else if (wr) {
        a.stats[(long)blockIdx.x * 2 * a.Ncol + a.Ncol + n0 + tid] = red[tid] + red[BN + tid];
      }
    }
    __syncthreads();
  }

  // Epilogue through LDS (the stage buffers are free after the loop's last barrier): lane holds
  // out[pixel m0 + wm 64 + 16 i + r][col wn BN/2 + 16 j + 4 g .. + 3]; per 16-pixel chunk the wave
  // writes its [16][BN/2] tile to its LDS region and reads it back as whole-row quads, so every store
  // instruction covers RPI pixel rows x BN/2 contiguous channels (256 B per row at BN = 128).
  constexpr int NCOL = BN / 2, QPR = NCOL / 4, RPI = 64 / QPR, ROWF = NCOL + 4;
  float* wl = (float*)smem + w * 16 * ROWF;
  const int eq = lane % QPR, er = lane / QPR;
  const int ecol = n0 + wn * NCOL + eq * 4;
  const bool ecol_ok = ecol < a.Ncol;
  const f32x4 bv = (a.bias && ecol_ok) ? *(const f32x4*)(a.bias + ecol) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < NF; ++j) *(f32x4*)(wl + r * ROWF + j * 16 + 4 * g) = acc[i][j];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 16 / RPI; ++it) {
      const int row = er + it * RPI;
      const f32x4 v0 = *(const f32x4*)(wl + row * ROWF + eq * 4);
      const int m = m0 + wm * 64 + i * 16 + row;
      if (m < M && ecol_ok) {
        TO* o;
        if (a.olin) {
          o = (TO*)a.out + (long)m * a.osw + ecol;
        } else {
          const int bb = m % Wm, t = m / Wm, aa = t % Hm, n = t / Hm;
          o = (TO*)a.out + (long)n * a.osn + (long)(aa * om + oa0) * a.osh + (long)(bb * om + ob0) * a.osw + ecol;
        }
        f32x4 v = v0 + bv;
        if (a.accumulate) v += q4_f32(q4_load(o));
        q4_store(o, v);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// out[pixel][col] (+)= bias[col] + sum_{tap, c} src[gathered pixel(tap)][c] . wp[col][tap][c]
// DX = false: pixels (n, ho, wo); source (n, ho s - p + ky, wo s - p + kx).
// DX = true:  blockIdx.z = stride phase (py, px); pixels (n, hq, wq) -> x pixel (hq s + py, wq s + px);
//             taps ky = ky0 + s kyq (the only ones that reach this phase); source dy pixel
//             (hq + qh - kyq, wq + qw - kxq) (conv.hip conv_dx_kernel's decomposition).
// TS / TO: element types of the gathered map and of the output map (float or bf16).
// INBN (forward): BatchNorm + ReLU applied to every in-range gathered quad (padding stays zero).
// BUFL: the gathers as branch-free buffer loads (NTConv sbytes / wbytes set), else the branchy loads
template <int BN, bool DX, bool STATS, typename TS, typename TO, bool INBN = false, bool BUFL = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void convb_nt_kernel(NTConv a) {
  constexpr int NF = BN / 32;       // 16-col fragments per wave (wave covers BN / 2 cols)
  constexpr int BJ = BN / 64;       // 16-byte weight loads per thread per step
  constexpr int ABYTES = NT_BM * 64, BBYTES = BN * 64, STAGE = ABYTES + BBYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  int Hm, Wm, ra, ca, cb, sy, twx, twy, by0, bx0, bs, om, oa0, ob0;
  if constexpr (!DX) {
    Hm = a.Ho; Wm = a.Wo; ra = a.s; ca = -a.p; cb = -a.p; sy = 1; twy = a.kh; twx = a.kw;
    by0 = 0; bx0 = 0; bs = 1; om = 1; oa0 = 0; ob0 = 0;
  } else {
    const int s = a.s, py = blockIdx.z / s, px = blockIdx.z - py * s;
    Hm = (a.Ho - py + s - 1) / s;
    Wm = (a.Wo - px + s - 1) / s;
    const int ky0 = (py + a.p) % s, kx0 = (px + a.p) % s;
    twy = a.kh > ky0 ? (a.kh - ky0 + s - 1) / s : 0;
    twx = a.kw > kx0 ? (a.kw - kx0 + s - 1) / s : 0;
    ca = (py + a.p - ky0) / s; cb = (px + a.p - kx0) / s; ra = 1; sy = -1;
    by0 = ky0; bx0 = kx0; bs = s; om = s; oa0 = py; ob0 = px;
  }
  const int M = a.N * Hm * Wm;
  const int m0 = blockIdx.x * NT_BM, n0 = blockIdx.y * BN;
  if (m0 >= M) return;  // a smaller stride phase (block-uniform)
  const int nk = twy * twx * (a.C / NT_BK);
  const int Kfull = a.kh * a.kw * a.C;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, r = lane & 15;

  // gather slots: 8 lanes per pixel (one channel quad each -- 16 bytes of fp32, 8 of bf16: a wave
  // instruction reads 8 whole channel runs), pixel rows arow0 + 32 j
  const int ac = tid & 7, arow0 = tid >> 3;
  long abase[4];
  int ahb[4], awb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int am = m0 + arow0 + 32 * j;
    abase[j] = 0;
    ahb[j] = -(1 << 28);  // a pixel row past M gathers zeros (its h is far out of range)
    awb[j] = 0;
    if (am < M) {
      const int bb = am % Wm, t = am / Wm, aa = t % Hm, n = t / Hm;
      abase[j] = (long)n * a.ssn + ac * 4;
      ahb[j] = aa * ra + ca;
      awb[j] = bb * ra + cb;
    }
  }
  const int bchunk = tid & 3, brow0 = tid >> 2;

  const TS* src = (const TS*)a.src;
  const __amdgpu_buffer_rsrc_t srs = buf_rsrc(a.src, a.sbytes), wrs = buf_rsrc(a.wp, a.wbytes);
  typename Q4<TS>::t ra4[4];
  u32x4 rb[BJ];
  // INBN: the step's BatchNorm channel quad and which gathered rows are in range (padding stays zero); the
  // affine map + ReLU is applied in store(), after this step's MFMAs, so the loads stay in flight behind them
  f32x4 bm, br, bg, bb;
  bool aok[4];
  auto load = [&](int kt) {
    const int k0 = kt * NT_BK;
    const int tq = k0 / a.C, c0 = k0 - tq * a.C;
    const int tyq = tq / twx, txq = tq - tyq * twx;
    if constexpr (INBN) {  // this step's channel quad of the BatchNorm (c0 + ac * 4: abase carries ac * 4)
      const int cq = c0 + ac * 4;
      bm = *(const f32x4*)(a.bnm + cq);
      br = *(const f32x4*)(a.bnr + cq);
      bg = *(const f32x4*)(a.bng + cq);
      bb = *(const f32x4*)(a.bnb + cq);
    }
    const int btap = (by0 + tyq * bs) * a.kw + bx0 + txq * bs;
    if constexpr (BUFL) {  // branch-free: a branch around each load made the waitcnt pass drain them at its join
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = ahb[j] + sy * tyq, ww = awb[j] + sy * txq;
        aok[j] = (unsigned)h < (unsigned)a.Hs && (unsigned)ww < (unsigned)a.Ws;
        const long e = abase[j] + (long)h * a.ssh + (long)ww * a.ssw + c0;
        ra4[j] = q4_buf_load<TS>(srs, aok[j] ? (unsigned)(e * (long)sizeof(TS)) : ES_OOB);
      }
#pragma unroll
      for (int j = 0; j < BJ; ++j) {
        const int col = n0 + brow0 + 64 * j;
        const long e = (long)col * Kfull + btap * a.C + c0 + bchunk * 8;
        rb[j] = buf_load16(wrs, col < a.Ncol ? (unsigned)(e * 2) : ES_OOB);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int h = ahb[j] + sy * tyq, ww = awb[j] + sy * txq;
        ra4[j] = q4_zero<TS>();
        aok[j] = (unsigned)h < (unsigned)a.Hs && (unsigned)ww < (unsigned)a.Ws;
        if (aok[j]) ra4[j] = q4_load(src + abase[j] + (long)h * a.ssh + (long)ww * a.ssw + c0);
      }
#pragma unroll
      for (int j = 0; j < BJ; ++j) {
        const int col = n0 + brow0 + 64 * j;
        rb[j] = col < a.Ncol ? *(const u32x4*)(a.wp + (long)col * Kfull + btap * a.C + c0 + bchunk * 8)
                             : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + ABYTES;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = arow0 + 32 * j;
      typename Q4<TS>::t v = ra4[j];
      if constexpr (INBN) v = aok[j] ? q4_bn_relu(v, bm, br, bg, bb) : q4_zero<TS>();
      *(bf16x4*)(As + row * 64 + cswz64(row, ac >> 1) * 16 + (ac & 1) * 8) = q4_b16(v);
    }
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      const int br = brow0 + 64 * j;
      *(u32x4*)(Bs + br * 64 + cswz64(br, bchunk) * 16) = rb[j];
    }
  };

  const int wm = w >> 1, wn = w & 1;
  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load(0);  // a pixel row past M gathers zeros (its h base is far out of range)
    store(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + ABYTES;
    bf16x8 af[4], bfr[NF];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = wm * 64 + i * 16 + r;
      af[i] = *(const bf16x8*)(As + rr * 64 + cswz64(rr, g) * 16);
    }
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int rr = wn * (BN / 2) + j * 16 + r;
      bfr[j] = *(const bf16x8*)(Bs + rr * 64 + cswz64(rr, g) * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  nt_tail<BN, DX, STATS, TO>(a, acc, M, m0, n0, Hm, Wm, om, oa0, ob0, smem);
}

// The same forward / data-grad convolution for a bf16 gathered map with the operand tiles brought in by LDS-DMA
// (buffer_load ... lds: a padding or past-M pixel is an out-of-range offset and reads as zeros) through an
// NST-stage ring, stage k + NST - 1 issued right after the barrier that publishes stage k (counted vmcnt, raw
// s_barrier) -- the register-staged kernel above keeps ONE step of gathers in flight behind 16 MFMAs per wave,
// which leaves the 1 x 1 / 3 x 3 convs at 3-5x their HBM floors.  Same LDS images (cswz64: the DMA lane writing
// physical chunk p of row r fetches logical chunk cswz64(r, p)), same fragments and MFMAs, same epilogue:
// bit-identical outputs.
template <int P3>
__device__ __forceinline__ void conv_wait_vmcnt(int n) {
  switch (n) {
#define ES_CVM(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    ES_CVM(1) ES_CVM(2) ES_CVM(3) ES_CVM(4) ES_CVM(5) ES_CVM(6) ES_CVM(8) ES_CVM(9) ES_CVM(12)
#undef ES_CVM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <int BN, bool DX, bool STATS, typename TO, int NST = 4>
__global__ __launch_bounds__(256) void convb_nt_ring_kernel(NTConv a) {
  constexpr int NF = BN / 32;
  constexpr int ABYTES = NT_BM * 64, BBYTES = BN * 64, STAGE = ABYTES + BBYTES;
  constexpr int IA = 2, IB = BN / 64, PER = IA + IB;  // 1-KiB DMA pieces per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];

  int Hm, Wm, ra, ca, cb, sy, twx, twy, by0, bx0, bs, om, oa0, ob0;
  if constexpr (!DX) {
    Hm = a.Ho; Wm = a.Wo; ra = a.s; ca = -a.p; cb = -a.p; sy = 1; twy = a.kh; twx = a.kw;
    by0 = 0; bx0 = 0; bs = 1; om = 1; oa0 = 0; ob0 = 0;
  } else {
    const int s = a.s, py = blockIdx.z / s, px = blockIdx.z - py * s;
    Hm = (a.Ho - py + s - 1) / s;
    Wm = (a.Wo - px + s - 1) / s;
    const int ky0 = (py + a.p) % s, kx0 = (px + a.p) % s;
    twy = a.kh > ky0 ? (a.kh - ky0 + s - 1) / s : 0;
    twx = a.kw > kx0 ? (a.kw - kx0 + s - 1) / s : 0;
    ca = (py + a.p - ky0) / s; cb = (px + a.p - kx0) / s; ra = 1; sy = -1;
    by0 = ky0; bx0 = kx0; bs = s; om = s; oa0 = py; ob0 = px;
  }
  const int M = a.N * Hm * Wm;
  const int m0 = blockIdx.x * NT_BM, n0 = blockIdx.y * BN;
  if (m0 >= M) return;  // a smaller stride phase (block-uniform)
  const int nk = twy * twx * (a.C / NT_BK);
  const int Kfull = a.kh * a.kw * a.C;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, r = lane & 15;

  // A pieces: wave w, piece j covers tile rows (4 j + w) 16 .. + 15; lane -> row + lane / 4, physical chunk lane % 4
  const i32x4 srs = rsrc_i4(a.src, (unsigned)(((long)(a.N - 1) * a.ssn + (long)(a.Hs - 1) * a.ssh +
                                                (long)(a.Ws - 1) * a.ssw + a.C) * 2));
  long abase[IA];
  int ahb[IA], awb[IA], alc[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = (4 * j + w) * 16 + (lane >> 2);
    alc[j] = cswz64(row, lane & 3) * 8;  // the logical channel chunk this lane's physical chunk holds
    const int am = m0 + row;
    abase[j] = 0;
    ahb[j] = -(1 << 28);  // a pixel row past M: every tap out of range, zeros
    awb[j] = 0;
    if (am < M) {
      const int bb = am % Wm, t = am / Wm, aa = t % Hm, n = t / Hm;
      abase[j] = (long)n * a.ssn;
      ahb[j] = aa * ra + ca;
      awb[j] = bb * ra + cb;
    }
  }
  // B pieces: weight rows (4 j + w) 16 .. (BN = 128: j < 2; BN = 64: j = 0); rows past Ncol read zeros
  const i32x4 wrs = rsrc_i4(a.wp, (unsigned)((long)a.Ncol * Kfull * 2));
  unsigned bofs[IB];
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int row = (4 * j + w) * 16 + (lane >> 2);
    const int col = n0 + row;
    bofs[j] = col < a.Ncol ? (unsigned)(((long)col * Kfull + cswz64(row, lane & 3) * 8) * 2) : ES_OOB;
  }
  auto issue = [&](int buf, int kt) {
    const int k0 = kt * NT_BK;
    const int tq = k0 / a.C, c0 = k0 - tq * a.C;
    const int tyq = tq / twx, txq = tq - tyq * twx;
    char* As = smem + buf * STAGE;
    char* Bs = As + ABYTES;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int h = ahb[j] + sy * tyq, ww = awb[j] + sy * txq;
      const bool ok = (unsigned)h < (unsigned)a.Hs && (unsigned)ww < (unsigned)a.Ws;
      const unsigned off = ok ? (unsigned)((abase[j] + (long)h * a.ssh + (long)ww * a.ssw + c0 + alc[j]) * 2) : ES_OOB;
      bl16_asm(srs, off, 0u, As + (4 * j + w) * 1024);
    }
    const int btap = (by0 + tyq * bs) * a.kw + bx0 + txq * bs;
    const unsigned bsoff = (unsigned)((btap * a.C + c0) * 2);
#pragma unroll
    for (int j = 0; j < IB; ++j)
      bl16_asm(wrs, bofs[j] == ES_OOB ? ES_OOB : bofs[j] + bsoff, 0u, Bs + (4 * j + w) * 1024);
  };

  const int wm = w >> 1, wn = w & 1;
  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NST - 1; ++st)
    if (st < nk) issue(st, st);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    conv_wait_vmcnt<0>(min(NST - 2, nk - 1 - kt) * PER);
    __builtin_amdgcn_s_barrier();
    if (kt + NST - 1 < nk) {
      int nb = buf + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      issue(nb, kt + NST - 1);
    }
    const char* As = smem + buf * STAGE;
    const char* Bs = As + ABYTES;
    bf16x8 af[4], bfr[NF];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rr = wm * 64 + i * 16 + r;
      af[i] = *(const bf16x8*)(As + rr * 64 + cswz64(rr, g) * 16);
    }
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int rr = wn * (BN / 2) + j * 16 + r;
      bfr[j] = *(const bf16x8*)(Bs + rr * 64 + cswz64(rr, g) * 16);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    buf = buf + 1 == NST ? 0 : buf + 1;
  }
  __syncthreads();  // every wave's last fragment reads are done before the tail reuses the ring as scratch
  nt_tail<BN, DX, STATS, TO>(a, acc, M, m0, n0, Hm, Wm, om, oa0, ob0, smem);
}

// ---- weight gradient -------------------------------------------------------------------------
struct DWConv {
  const void* x;    // [N, H, W, Cin] at (sxn, sxh, sxw), channel stride 1 (fp32 or bf16 map)
  const void* dy;   // [N, Ho, Wo, Cout] at (syn, syh, syw), channel stride 1 (fp32 or bf16 map)
  float* P;         // [splits][Cout][kh kw Cin] partials, column k' = tap Cin + ci
  int N, H, W, Cin, Ho, Wo, Cout, kh, kw, s, p;
  long sxn, sxh, sxw, syn, syh, syw;
  int M, mchunk;
  const float* bnm; const float* bnr; const float* bng; const float* bnb;  // INBN: x is a BatchNorm's input
  // branch-free loads (BUF kernels): the maps' byte extents (< 2 GiB: 32-bit buffer offsets) and the pixel walk's
  // per-step advance 32 = wdq Wo + wdr (one wrap of wo and of ho per step at most when wdq + 1 < Ho)
  unsigned xbytes, ybytes;
  int wdq, wdr;
};

// pixel index -> (n, ho, wo), advanced without division
struct PixWalk {
  int n, ho, wo;
  __device__ void init(int m, int Ho, int Wo) {
    wo = m % Wo;
    const int t = m / Wo;
    ho = t % Ho;
    n = t / Ho;
  }
  __device__ void advance(int d, int Ho, int Wo) {
    wo += d;
    while (wo >= Wo) {
      wo -= Wo;
      if (++ho == Ho) {
        ho = 0;
        ++n;
      }
    }
  }
  // the same +32 pixels as selects (DWConv wdq / wdr; valid while wdq + 1 < Ho): no loop, no branch
  __device__ void advance32(int dq, int dr, int Ho, int Wo) {
    wo += dr;
    ho += dq;
    const bool cw = wo >= Wo;
    wo = cw ? wo - Wo : wo;
    ho = cw ? ho + 1 : ho;
    const bool ch = ho >= Ho;
    ho = ch ? ho - Ho : ho;
    n = ch ? n + 1 : n;
  }
};



// P[split][co][k'] = sum_{pixels m of the split} dy[m][co] . im2col(x)[m][k'], tile B1 (co) x B2 (k')
// INBN: x is a train-mode BatchNorm's input; the gathered quads get its affine map + ReLU (as the forward's)
// BUF: branch-free loads (buffer loads, out-of-range offsets for the rows past the split / padding taps) and the
// select-only pixel walk; the branchy form (maps >= 2 GiB, or maps too small for one wrap per step) otherwise
template <int B1, int B2, typename TX, typename TD, bool INBN = false, bool BUF = true>
__global__ __launch_bounds__(256) void convb_dw_kernel(DWConv a) {
  constexpr int WA = (B1 == 128 && B2 == 64) ? 4 : (B1 == 64 && B2 == 128) ? 1 : 2, WB = 4 / WA;
  constexpr int F1 = B1 / WA / 16, F2 = B2 / WB / 16;  // fragments per wave along co / k'
  constexpr int QP1 = B1 / 4, RP1 = 256 / QP1, J1 = 32 / RP1;  // dy tile: quads per row, rows per pass
  constexpr int QP2 = B2 / 4, RP2 = 256 / QP2, J2 = 32 / RP2;  // im2col tile
  constexpr int TILE = 32 * 256, STAGE = 2 * TILE;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int K = a.kh * a.kw * a.Cin;
  const int co0 = blockIdx.x * B1, k0 = blockIdx.y * B2, split = blockIdx.z;
  const int mbeg = split * a.mchunk, mend = min(mbeg + a.mchunk, a.M);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane >> 4, t16 = lane & 15, q = t16 >> 2, p4 = t16 & 3;

  // dy slots: channel quad q1, rows r1 + RP1 j
  const int q1 = tid % QP1, r1 = tid / QP1;
  const int co = co0 + 4 * q1;
  const bool co_ok = co < a.Cout;
  // im2col slots: column quad q2 -> (tap, ci) fixed for the kernel
  const int q2 = tid % QP2, r2 = tid / QP2;
  const int kc = k0 + 4 * q2;
  const bool kc_ok = kc < K;
  int ky = 0, kx = 0, ci = 0;
  if (kc_ok) {
    const int tap = kc / a.Cin;
    ci = kc - tap * a.Cin;
    ky = tap / a.kw;
    kx = tap - ky * a.kw;
  }
  f32x4 bm = {0.f, 0.f, 0.f, 0.f}, br = bm, bg = bm, bb = bm;
  if constexpr (INBN) {
    if (kc_ok) {  // a thread's im2col columns keep one channel quad for the whole kernel
      bm = *(const f32x4*)(a.bnm + ci);
      br = *(const f32x4*)(a.bnr + ci);
      bg = *(const f32x4*)(a.bng + ci);
      bb = *(const f32x4*)(a.bnb + ci);
    }
  }
  PixWalk pw1[J1], pw2[J2];
#pragma unroll
  for (int j = 0; j < J1; ++j) pw1[j].init(mbeg + r1 + RP1 * j, a.Ho, a.Wo);
#pragma unroll
  for (int j = 0; j < J2; ++j) pw2[j].init(mbeg + r2 + RP2 * j, a.Ho, a.Wo);

  const TX* xs = (const TX*)a.x;
  const TD* dys = (const TD*)a.dy;
  typename Q4<TD>::t v1[J1];
  typename Q4<TX>::t v2[J2];
  bool xok[J2];  // INBN: in-range im2col rows (the BatchNorm is applied in store(), padding stays zero)
  const __amdgpu_buffer_rsrc_t yr = buf_rsrc(a.dy, BUF ? a.ybytes : 0u), xr = buf_rsrc(a.x, BUF ? a.xbytes : 0u);
  auto load = [&](int mm) {
    if constexpr (BUF) {
#pragma unroll
      for (int j = 0; j < J1; ++j) {
        const int m = mm + r1 + RP1 * j;
        const bool ok = m < mend && co_ok;
        const long e = (long)pw1[j].n * a.syn + (long)pw1[j].ho * a.syh + (long)pw1[j].wo * a.syw + co;
        v1[j] = q4_buf_load<TD>(yr, ok ? (unsigned)(e * (long)sizeof(TD)) : ES_OOB);
        pw1[j].advance32(a.wdq, a.wdr, a.Ho, a.Wo);
      }
#pragma unroll
      for (int j = 0; j < J2; ++j) {
        const int m = mm + r2 + RP2 * j;
        const int h = pw2[j].ho * a.s - a.p + ky, ww = pw2[j].wo * a.s - a.p + kx;
        xok[j] = m < mend && kc_ok && (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
        const long e = (long)pw2[j].n * a.sxn + (long)h * a.sxh + (long)ww * a.sxw + ci;
        v2[j] = q4_buf_load<TX>(xr, xok[j] ? (unsigned)(e * (long)sizeof(TX)) : ES_OOB);
        pw2[j].advance32(a.wdq, a.wdr, a.Ho, a.Wo);
      }
    } else {
#pragma unroll
      for (int j = 0; j < J1; ++j) {
        const int m = mm + r1 + RP1 * j;
        v1[j] = q4_zero<TD>();
        if (m < mend && co_ok)
          v1[j] = q4_load(dys + (long)pw1[j].n * a.syn + (long)pw1[j].ho * a.syh + (long)pw1[j].wo * a.syw + co);
        pw1[j].advance(32, a.Ho, a.Wo);
      }
#pragma unroll
      for (int j = 0; j < J2; ++j) {
        const int m = mm + r2 + RP2 * j;
        v2[j] = q4_zero<TX>();
        xok[j] = false;
        if (m < mend && kc_ok) {
          const int h = pw2[j].ho * a.s - a.p + ky, ww = pw2[j].wo * a.s - a.p + kx;
          xok[j] = (unsigned)h < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
          if (xok[j]) v2[j] = q4_load(xs + (long)pw2[j].n * a.sxn + (long)h * a.sxh + (long)ww * a.sxw + ci);
        }
        pw2[j].advance(32, a.Ho, a.Wo);
      }
    }
  };
  auto store = [&](int buf) {
    char* T1 = smem + buf * STAGE;
    char* T2 = T1 + TILE;
#pragma unroll
    for (int j = 0; j < J1; ++j) {
      const int row = r1 + RP1 * j;
      *(bf16x4*)(T1 + row * 256 + cswz256(row, q1 >> 1) * 16 + (q1 & 1) * 8) = q4_b16(v1[j]);
    }
#pragma unroll
    for (int j = 0; j < J2; ++j) {
      const int row = r2 + RP2 * j;
      typename Q4<TX>::t v = v2[j];
      if constexpr (INBN) v = xok[j] ? q4_bn_relu(v, bm, br, bg, bb) : q4_zero<TX>();
      *(bf16x4*)(T2 + row * 256 + cswz256(row, q2 >> 1) * 16 + (q2 & 1) * 8) = q4_b16(v);
    }
  };

  const int wa = w / WB, wb = w % WB;
  f32x4 acc[F2][F1];
#pragma unroll
  for (int i = 0; i < F2; ++i)
#pragma unroll
    for (int j = 0; j < F1; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = mend > mbeg ? (mend - mbeg + 31) / 32 : 0;
  if (nk > 0) {
    load(mbeg);
    store(0);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(mbeg + (kt + 1) * 32);
    const char* T1 = smem + buf * STAGE;
    const char* T2 = T1 + TILE;
    const int ra_ = 8 * g + q, rb_ = ra_ + 4;
    const int off = (p4 & 1) * 8;
    bf16x8 af[F2], bfr[F1];
#pragma unroll
    for (int i = 0; i < F2; ++i) {
      const int c = (wb * (B2 / WB) + i * 16) / 8 + (p4 >> 1);
      af[i] = cat8(lds_tr4(T2 + ra_ * 256 + cswz256(ra_, c) * 16 + off),
                   lds_tr4(T2 + rb_ * 256 + cswz256(rb_, c) * 16 + off));
    }
#pragma unroll
    for (int j = 0; j < F1; ++j) {
      const int c = (wa * (B1 / WA) + j * 16) / 8 + (p4 >> 1);
      bfr[j] = cat8(lds_tr4(T1 + ra_ * 256 + cswz256(ra_, c) * 16 + off),
                    lds_tr4(T1 + rb_ * 256 + cswz256(rb_, c) * 16 + off));
    }
#pragma unroll
    for (int i = 0; i < F2; ++i)
#pragma unroll
      for (int j = 0; j < F1; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // lane holds D[k' = .. + 4 g + e][co = .. + t16] -> P[split][co][k' .. k'+3]
  float* P = a.P + (long)split * a.Cout * K;
#pragma unroll
  for (int j = 0; j < F1; ++j) {
    const int c = co0 + wa * (B1 / WA) + j * 16 + t16;
    if (c >= a.Cout) continue;
#pragma unroll
    for (int i = 0; i < F2; ++i) {
      const int kk = k0 + wb * (B2 / WB) + i * 16 + 4 * g;
      if (kk < K) *(f32x4*)(P + (long)c * K + kk) = acc[i][j];
    }
  }
}

// dw[co][ci][tap] (+)= sum_s P[s][co][tap Cin + ci]: 64 column quads x 4 split lanes per workgroup,
// lanes combined in a fixed order (deterministic)
__global__ __launch_bounds__(256) void convb_dw_reduce_kernel(const float* __restrict__ P, int S, int Cout, int Cin,
                                                              int T, float* __restrict__ dw, int accumulate) {
  __shared__ f32x4 red[4][64];
  const long n = (long)Cout * T * Cin;
  const int nq = (int)(n / 4);
  const int cq = blockIdx.x * 64 + (threadIdx.x & 63), sl = threadIdx.x >> 6;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (cq < nq) {
#pragma unroll 4
    for (int k = sl; k < S; k += 4) s += *(const f32x4*)(P + (long)k * n + (long)cq * 4);
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
  if (sl != 0 || cq >= nq) return;
  s = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
  const int K = T * Cin;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long idx = (long)cq * 4 + e;
    const int c = (int)(idx / K), kk = (int)(idx - (long)c * K);
    const int tap = kk / Cin, cc = kk - tap * Cin;
    float* o = dw + (long)c * K + (long)cc * T + tap;
    *o = accumulate ? *o + s[e] : s[e];
  }
}

// wp[co][tap][ci] = bf16(w[co][ci][tap]); wt[ci][tap][co] = bf16(w[co][ci][tap])
__global__ void convb_pack_kernel(const float* __restrict__ w, int Cout, int Cin, int T, bf16* __restrict__ wp,
                                  bf16* __restrict__ wt) {
  const long n = (long)Cout * Cin * T;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int tap = (int)(i % T);
    const long t2 = i / T;
    const int ci = (int)(t2 % Cin), co = (int)(t2 / Cin);
    const bf16 v = (bf16)w[i];
    if (wp) wp[((long)co * T + tap) * Cin + ci] = v;
    if (wt) wt[((long)ci * T + tap) * Cout + co] = v;
  }
}

// Every conv weight of a model in one launch (es_conv2d_pack_bf16_multi): workgroup row y packs entry y,
// the same element mapping as convb_pack_kernel
struct ConvPackEntry {
  const float* w;
  bf16 *wp, *wt;
  int Cout, Cin, T, pad;
};
// Stores coalesced on both images: wp in its own element order (each thread gathers its source element: the
// rows of w it reads are L2-resident), and wt -- w viewed as [Cout][K = Cin T] transposed to [K][Cout] -- through
// 64 x 64 LDS tiles.  The same bf16 values as convb_pack_kernel.
__global__ __launch_bounds__(256) void convb_pack_multi_kernel(const ConvPackEntry* __restrict__ tab) {
  __shared__ float tile[64][65];
  const ConvPackEntry e = tab[blockIdx.y];
  const int K = e.Cin * e.T;
  const long n = (long)e.Cout * K;
  if (e.wp) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
      const int ci = (int)(i % e.Cin);  // i = (co T + tap) Cin + ci
      const long t2 = i / e.Cin;
      const int tap = (int)(t2 % e.T), co = (int)(t2 / e.T);
      e.wp[i] = (bf16)e.w[((long)co * e.Cin + ci) * e.T + tap];
    }
  }
  if (!e.wt) return;
  const int tco = (e.Cout + 63) / 64, tk = (K + 63) / 64;
  const int c = threadIdx.x & 63, r0 = threadIdx.x >> 6;
  for (int t = blockIdx.x; t < tco * tk; t += gridDim.x) {
    const int co0 = (t / tk) * 64, k0 = (t % tk) * 64;
    __syncthreads();  // the previous tile's reads are done
#pragma unroll 4
    for (int r = r0; r < 64; r += 4)
      if (co0 + r < e.Cout && k0 + c < K) tile[r][c] = e.w[(long)(co0 + r) * K + k0 + c];
    __syncthreads();
#pragma unroll 4
    for (int r = r0; r < 64; r += 4)  // r: the k row of wt, c: the co column
      if (k0 + r < K && co0 + c < e.Cout) e.wt[(long)(k0 + r) * e.Cout + co0 + c] = (bf16)tile[c][r];
  }
}

inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }
inline bool st4(long a, long b, long c) { return a % 4 == 0 && b % 4 == 0 && c % 4 == 0; }

// ~8 workgroups per CU over the pixel splits (the small-tile shapes are load-latency bound: occupancy hides
// it); every split writes an fp32 slab of the whole weight gradient that convb_dw_reduce_kernel sums, so
// fewer, longer splits trade occupancy for slab traffic (es_set_conv_dw_target).  S1, one box, interleaved
// twice (bench.py --workload s1, round 4): 2048 -> 144.4 / 145.4 ms/step, 1024 -> 143.0 / 143.8, 512 -> 143.2 / 142.6
int g_dw_target_wg = 512;
constexpr int DW_MAX_SPLITS = 1024;

inline void dw_tile(int Cout, int K, int& b1, int& b2) {
  b1 = Cout <= 64 ? 64 : 128;
  b2 = K <= 64 ? 64 : 128;
}
inline int dw_tiles(int Cout, int K) {
  int b1, b2;
  dw_tile(Cout, K, b1, b2);
  return ((Cout + b1 - 1) / b1) * ((K + b2 - 1) / b2);
}
inline int dw_splits(int M, int Cout, int K, int splits) {
  if (splits <= 0) {
    const int tiles = dw_tiles(Cout, K);
    splits = (g_dw_target_wg + tiles - 1) / tiles;
    const int maxs = (M + 127) / 128;  // at least 4 pixel steps per split
    splits = splits < maxs ? splits : maxs;
  }
  if (splits > DW_MAX_SPLITS) splits = DW_MAX_SPLITS;
  return splits < 1 ? 1 : splits;
}

// the _ex entry points' map element-type flags: bit 0 = the gathered / input map is bf16, bit 1 = the
// output map (bwd_weight: dy) is bf16

template <int BN, bool DX, bool STATS, bool INBN, bool BUFL>
void launch_nt_b(dim3 grid, int flags, const NTConv& a, hipStream_t stream) {
  switch (flags & 3) {
    case 0: hipLaunchKernelGGL((convb_nt_kernel<BN, DX, STATS, float, float, INBN, BUFL>), grid, 256, 0, stream, a); break;
    case 1: hipLaunchKernelGGL((convb_nt_kernel<BN, DX, STATS, bf16, float, INBN, BUFL>), grid, 256, 0, stream, a); break;
    case 2: hipLaunchKernelGGL((convb_nt_kernel<BN, DX, STATS, float, bf16, INBN, BUFL>), grid, 256, 0, stream, a); break;
    default: hipLaunchKernelGGL((convb_nt_kernel<BN, DX, STATS, bf16, bf16, INBN, BUFL>), grid, 256, 0, stream, a); break;
  }
}
template <int BN, bool DX, bool STATS, bool INBN = false>
void launch_nt(dim3 grid, int flags, const NTConv& a, hipStream_t stream) {
  if (a.sbytes) launch_nt_b<BN, DX, STATS, INBN, true>(grid, flags, a, stream);
  else launch_nt_b<BN, DX, STATS, INBN, false>(grid, flags, a, stream);
}

template <int B1, int B2, bool INBN, bool BUF>
void launch_dw_b(dim3 grid, int flags, const DWConv& a, hipStream_t stream) {
  switch (flags & 3) {
    case 0: hipLaunchKernelGGL((convb_dw_kernel<B1, B2, float, float, INBN, BUF>), grid, 256, 0, stream, a); break;
    case 1: hipLaunchKernelGGL((convb_dw_kernel<B1, B2, bf16, float, INBN, BUF>), grid, 256, 0, stream, a); break;
    case 2: hipLaunchKernelGGL((convb_dw_kernel<B1, B2, float, bf16, INBN, BUF>), grid, 256, 0, stream, a); break;
    default: hipLaunchKernelGGL((convb_dw_kernel<B1, B2, bf16, bf16, INBN, BUF>), grid, 256, 0, stream, a); break;
  }
}
// the branch-free kernel when both maps are under 2 GiB and a 32-pixel step wraps the walk at most once per
// dimension (es_set_conv_dw_buf 0: always the branchy one)
int g_conv_dw_buf = 1;
template <int B1, int B2, bool INBN = false>
void launch_dw(dim3 grid, int flags, const DWConv& a, hipStream_t stream) {
  if (g_conv_dw_buf && a.xbytes && a.ybytes && a.wdq + 1 < a.Ho) launch_dw_b<B1, B2, INBN, true>(grid, flags, a, stream);
  else launch_dw_b<B1, B2, INBN, false>(grid, flags, a, stream);
}

// the staged kernel's branch-free gathers: both operands' byte extents when under 2 GiB (es_set_conv_dw_buf 0:
// the branchy loads here too)
inline void nt_extents(NTConv& a, int flags) {
  const long sb = ((long)(a.N - 1) * a.ssn + (long)(a.Hs - 1) * a.ssh + (long)(a.Ws - 1) * a.ssw + a.C) *
                  ((flags & 1) ? 2 : 4);
  const long wb = (long)a.Ncol * a.kh * a.kw * a.C * 2;
  const bool ok = g_conv_dw_buf && sb < 0x7fff0000L && wb < 0x7fff0000L;
  a.sbytes = ok ? (unsigned)sb : 0u;
  a.wbytes = ok ? (unsigned)wb : 0u;
}

// bf16 gathered maps on the LDS-DMA ring (convb_nt_ring_kernel): 0 = off (the register-staged kernel), else its
// stage count (3 or 4); es_set_conv_ring.  Isolated at the Conformer-B/384 shapes (r05, scripts/convb_bench.py
// --bnin --all-shapes, ring 0 / 3 / 4): every data gradient is 7-20 % faster on 3 stages (48 KiB: three workgroups
// per CU; 4 stages hold two), and so is every forward that does not widen the channels (the 3 x 3, the 1 x 1
// reductions, FCUUp: 146 vs 163 us at stage 1's conv1); the widening 1 x 1 forwards (conv3, the strided residual
// conv) lose 5-15 % on it (a 2-8-step K loop cannot use the ring; the staged kernel's 32 KiB fit more tiles)
int g_conv_ring = 3;
// the 128-channel tile leaves most CUs idle on a small map (P0's layer 4: 784 pixels x 512 channels = 28
// workgroups over a 4,608-deep reduction): below g_conv_small workgroups the 64-channel tile runs instead
// (twice the workgroups, the same per-element reduction order); es_set_conv_small, 0 = off
static int g_conv_small = 128;
static inline bool conv_small_grid(long wgs) { return wgs < g_conv_small; }


template <int BN, bool DX, bool STATS, int NST>
void launch_ring_n(dim3 grid, int flags, const NTConv& a, hipStream_t stream) {
  const size_t lds = (size_t)NST * (NT_BM + BN) * 64;
  if (flags & 2) hipLaunchKernelGGL((convb_nt_ring_kernel<BN, DX, STATS, bf16, NST>), grid, 256, lds, stream, a);
  else hipLaunchKernelGGL((convb_nt_ring_kernel<BN, DX, STATS, float, NST>), grid, 256, lds, stream, a);
}
// true when the ring kernel took the launch: a bf16 source map under 2 GiB (32-bit DMA offsets), no input BatchNorm
template <int BN, bool DX, bool STATS>
bool launch_ring(dim3 grid, int flags, const NTConv& a, hipStream_t stream) {
  const long src_bytes = ((long)(a.N - 1) * a.ssn + (long)(a.Hs - 1) * a.ssh + (long)(a.Ws - 1) * a.ssw + a.C) * 2;
  const long w_bytes = (long)a.Ncol * a.kh * a.kw * a.C * 2;
  if (!g_conv_ring || !(flags & 1) || a.bnm || src_bytes >= 0x7fff0000L || w_bytes >= 0x7fff0000L) return false;
  if (!DX && a.Ncol > a.C) return false;  // a widening forward: the staged kernel
  if (g_conv_ring == 3) launch_ring_n<BN, DX, STATS, 3>(grid, flags, a, stream);
  else launch_ring_n<BN, DX, STATS, 4>(grid, flags, a, stream);
  return true;
}

// the forward / weight-gradient launches with or without the input BatchNorm
template <int BN, bool STATS>
void launch_fwd(dim3 grid, int flags, const NTConv& a, hipStream_t stream) {
  if (launch_ring<BN, false, STATS>(grid, flags, a, stream)) return;
  if (a.bnm) launch_nt<BN, false, STATS, true>(grid, flags, a, stream);
  else launch_nt<BN, false, STATS, false>(grid, flags, a, stream);
}
template <int B1, int B2>
void launch_dw_bn(dim3 grid, int flags, const DWConv& a, hipStream_t stream) {
  if (a.bnm) launch_dw<B1, B2, true>(grid, flags, a, stream);
  else launch_dw<B1, B2, false>(grid, flags, a, stream);
}

}  // namespace

extern "C" {

// 1 if the bf16 kernels take a conv of these channel counts (both multiples of 32)
// tuning knob: the workgroup count the bf16 weight gradient's automatic pixel split aims at (default 512);
// returns the previous value (v <= 0: unchanged)
// tuning knob: the bf16-map data-gradient convs and the forwards that do not widen the channels on the LDS-DMA
// ring kernel with this many stages (3 or 4, default 3), or 0 = the register-staged kernel (bit-identical);
// returns the previous value, or ES_BAD_ARG (unchanged) for any other value
int es_set_conv_ring(int v) {
  if (v != 0 && v != 3 && v != 4) return ES_BAD_ARG;
  const int old = g_conv_ring;
  g_conv_ring = v;
  return old;
}

// tuning knob: 1 (default) = the register-staged conv kernels' branch-free loads (weight gradient: and pixel walk)
// where they apply, 0 = the branchy loads everywhere (bit-identical); returns the previous value, or ES_BAD_ARG
// (unchanged) otherwise
int es_set_conv_dw_buf(int v) {
  if (v != 0 && v != 1) return ES_BAD_ARG;
  const int old = g_conv_dw_buf;
  g_conv_dw_buf = v;
  return old;
}

// tuning knob: a bf16 conv forward / data gradient whose 128-channel tiling would launch fewer than `wgs`
// workgroups runs on the 64-channel tile (default 128; 0 = never; bit-identical); returns the previous value,
// or -2 (unchanged) for a negative value
int es_set_conv_small(int wgs) {
  if (wgs < 0) return ES_BAD_ARG;
  const int old = g_conv_small;
  g_conv_small = wgs;
  return old;
}

int es_set_conv_dw_target(int v) {
  const int old = g_dw_target_wg;
  if (v > 0) g_dw_target_wg = v;
  return old;
}

int es_conv2d_bf16_eligible(int Cin, int Cout, int kh, int kw) {
  return Cin > 0 && Cout > 0 && Cin % 32 == 0 && Cout % 32 == 0 && kh > 0 && kw > 0 && kh * kw <= 64;
}

int es_conv2d_pack_bf16(const float* w, int Cout, int Cin, int kh, int kw, void* wp, void* wt, hipStream_t stream) {
  if (!w || (!wp && !wt)) return ES_BAD_ARG;
  if (Cout <= 0 || Cin <= 0 || kh <= 0 || kw <= 0) return ES_BAD_SHAPE;
  const long n = (long)Cout * Cin * kh * kw;
  long b = (n + 255) / 256;
  hipLaunchKernelGGL(convb_pack_kernel, (unsigned)(b > 4096 ? 4096 : b), 256, 0, stream, w, Cout, Cin, kh * kw, (bf16*)wp,
                     (bf16*)wt);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_conv_pack_entry_size() { return (int)sizeof(ConvPackEntry); }

// es_conv2d_pack_bf16 over n weights in one launch: table = n device-resident entries of
// es_conv_pack_entry_size() bytes {const float* w; bf16* wp; bf16* wt; int Cout, Cin, kh * kw, 0};
// max_elems = the largest Cout * Cin * kh * kw among them (sizes the grid)
int es_conv2d_pack_bf16_multi(const void* table, int n, long max_elems, hipStream_t stream) {
  if (!table) return ES_BAD_ARG;
  if (n <= 0 || n > 65535 || max_elems <= 0) return ES_BAD_SHAPE;
  const long b = (max_elems + 255) / 256;
  hipLaunchKernelGGL(convb_pack_multi_kernel, dim3((unsigned)(b > 1024 ? 1024 : b), n), 256, 0, stream,
                     (const ConvPackEntry*)table);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

// y[n, ho, wo, co] (+)= bias[co] + conv(x) with wp = es_conv2d_pack_bf16's forward image.  Same geometry
// arguments as es_conv2d_fwd; requires es_conv2d_bf16_eligible, sxc == 1, 16-byte aligned pointers and
// element strides % 4 == 0.  flags: 1 = x is a bf16 map, 2 = y is a bf16 map (else fp32).  bn_partials
// (nullable, accumulate 0 only): y's BatchNorm statistics per 128-pixel block (es_conv2d_bnstats_size
// floats; from the fp32 accumulators).
static int conv_fwd_bf16_impl(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                              const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad, void* y,
                              long syn, long syh, long syw, int accumulate, float* bn_partials, int flags,
                              const float* bnm, const float* bnr, const float* bng, const float* bnb,
                              hipStream_t stream) {
  if (!x || !wp || !y) return ES_BAD_ARG;
  if (!es_conv2d_bf16_eligible(Cin, Cout, kh, kw) || N <= 0 || H <= 0 || W <= 0 || stride <= 0 || pad < 0 ||
      (flags & ~3))
    return ES_BAD_SHAPE;
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || sxc != 1 || !st4(sxn, sxh, sxw) || !st4(syn, syh, syw) || !al16(x) || !al16(y) || !al16(wp) ||
      (bias && !al16(bias)))
    return ES_BAD_SHAPE;
  if (bnm && (!bnr || !bng || !bnb || !al16(bnm) || !al16(bnr) || !al16(bng) || !al16(bnb))) return ES_BAD_ARG;
  NTConv a{x, (const bf16*)wp, bias, y, N, Cin, Cout, H, W, sxn, sxh, sxw, kh, kw, stride, pad, Ho, Wo, syn, syh, syw,
           accumulate, bn_partials, bnm, bnr, bng, bnb, syh == (long)Wo * syw && syn == (long)Ho * syh};
  nt_extents(a, flags);
  if (bn_partials && accumulate) return ES_BAD_ARG;
  const int M = N * Ho * Wo;
  const dim3 g128((M + 127) / 128, Cout / 128), g64((M + 127) / 128, (Cout + 63) / 64);
  if (Cout % 128 == 0 && !conv_small_grid((long)g128.x * g128.y)) {
    if (bn_partials) launch_fwd<128, true>(g128, flags, a, stream);
    else launch_fwd<128, false>(g128, flags, a, stream);
  } else {
    if (bn_partials) launch_fwd<64, true>(g64, flags, a, stream);
    else launch_fwd<64, false>(g64, flags, a, stream);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_conv2d_fwd_bf16_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                          const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad, void* y,
                          long syn, long syh, long syw, int accumulate, float* bn_partials, int flags,
                          hipStream_t stream) {
  return conv_fwd_bf16_impl(x, N, H, W, Cin, sxn, sxh, sxw, sxc, wp, bias, Cout, kh, kw, stride, pad, y, syn, syh, syw,
                            accumulate, bn_partials, flags, nullptr, nullptr, nullptr, nullptr, stream);
}

// es_conv2d_fwd_bf16_ex whose input map x is a train-mode BatchNorm + ReLU's INPUT: the conv reads
// relu((x - mean) rstd gamma + beta) (rounded to x's map type, exactly as es_bn2d_fwd*_ex would have stored
// it) as it gathers, so the normalised map is never written.  mean / rstd from es_bn2d_fwd_partials_ex with
// y = NULL; all four per-channel arrays 16-byte aligned.
int es_conv2d_fwd_bf16_bnin_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                               const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                               void* y, long syn, long syh, long syw, int accumulate, float* bn_partials, int flags,
                               const float* in_mean, const float* in_rstd, const float* in_gamma,
                               const float* in_beta, hipStream_t stream) {
  if (!in_mean) return ES_BAD_ARG;
  return conv_fwd_bf16_impl(x, N, H, W, Cin, sxn, sxh, sxw, sxc, wp, bias, Cout, kh, kw, stride, pad, y, syn, syh, syw,
                            accumulate, bn_partials, flags, in_mean, in_rstd, in_gamma, in_beta, stream);
}

int es_conv2d_fwd_bf16(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                       const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad, float* y,
                       long syn, long syh, long syw, int accumulate, hipStream_t stream) {
  return es_conv2d_fwd_bf16_ex(x, N, H, W, Cin, sxn, sxh, sxw, sxc, wp, bias, Cout, kh, kw, stride, pad, y, syn, syh,
                               syw, accumulate, nullptr, 0, stream);
}

// floats of es_conv2d_fwd_bf16_bnstats' partials for M = N Ho Wo output pixels
size_t es_conv2d_bnstats_size(int M, int Cout) {
  return M > 0 && Cout > 0 ? (size_t)((M + NT_BM - 1) / NT_BM) * 2 * Cout : 0;
}

// es_conv2d_fwd_bf16 (accumulate 0) that also writes the BatchNorm statistics of y: per 128-pixel
// block b, partials[b][0][c] = sum of y[., c] and partials[b][1][c] = sum of (y - block mean)^2 over
// the block's pixels -- es_bn2d_fwd_partials turns them into the batch statistics without re-reading y.
int es_conv2d_fwd_bf16_bnstats(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                               const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                               float* y, long syn, long syh, long syw, float* partials, hipStream_t stream) {
  if (!partials) return ES_BAD_ARG;
  return es_conv2d_fwd_bf16_ex(x, N, H, W, Cin, sxn, sxh, sxw, sxc, wp, bias, Cout, kh, kw, stride, pad, y, syn, syh,
                               syw, 0, partials, 0, stream);
}

// dx[n, h, w, ci] (+)= conv^T(dy) with wt = es_conv2d_pack_bf16's transposed image.  Same geometry
// arguments as es_conv2d_bwd_data.  flags: 1 = dy is a bf16 map, 2 = dx is a bf16 map.
int es_conv2d_bwd_data_bf16_ex(const void* dy, long syn, long syh, long syw, const void* wt, int N, int H, int W,
                               int Cin, int Cout, int kh, int kw, int stride, int pad, void* dx, long sxn, long sxh,
                               long sxw, long sxc, int accumulate, int flags, hipStream_t stream) {
  if (!dy || !wt || !dx) return ES_BAD_ARG;
  if (!es_conv2d_bf16_eligible(Cin, Cout, kh, kw) || N <= 0 || H <= 0 || W <= 0 || stride <= 0 || pad < 0 ||
      (flags & ~3))
    return ES_BAD_SHAPE;
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || sxc != 1 || !st4(sxn, sxh, sxw) || !st4(syn, syh, syw) || !al16(dy) || !al16(dx) ||
      !al16(wt))
    return ES_BAD_SHAPE;
  NTConv a{dy, (const bf16*)wt, nullptr, dx, N, Cout, Cin, Ho, Wo, syn, syh, syw, kh, kw, stride, pad, H, W, sxn, sxh,
           sxw, accumulate, nullptr, nullptr, nullptr, nullptr, nullptr,
           stride == 1 && sxh == (long)W * sxw && sxn == (long)H * sxh};
  nt_extents(a, flags);
  const int Mq = N * ((H + stride - 1) / stride) * ((W + stride - 1) / stride);  // largest phase
  const unsigned ph = (unsigned)(stride * stride);
  if (Cin % 128 == 0 && !conv_small_grid((long)((Mq + 127) / 128) * (Cin / 128) * ph)) {
    const dim3 gr((Mq + 127) / 128, Cin / 128, ph);
    if (!launch_ring<128, true, false>(gr, flags, a, stream)) launch_nt<128, true, false>(gr, flags, a, stream);
  } else {
    const dim3 gr((Mq + 127) / 128, (Cin + 63) / 64, ph);
    if (!launch_ring<64, true, false>(gr, flags, a, stream)) launch_nt<64, true, false>(gr, flags, a, stream);
  }
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_conv2d_bwd_data_bf16(const float* dy, long syn, long syh, long syw, const void* wt, int N, int H, int W,
                            int Cin, int Cout, int kh, int kw, int stride, int pad, float* dx, long sxn, long sxh,
                            long sxw, long sxc, int accumulate, hipStream_t stream) {
  return es_conv2d_bwd_data_bf16_ex(dy, syn, syh, syw, wt, N, H, W, Cin, Cout, kh, kw, stride, pad, dx, sxn, sxh, sxw,
                                    sxc, accumulate, 0, stream);
}

// fp32 workspace floats of es_conv2d_bwd_weight_bf16 for M = N Ho Wo output pixels (splits <= 0: auto)
size_t es_conv2d_bwd_weight_bf16_workspace(int M, int Cout, int Cin, int kh, int kw, int splits) {
  if (M <= 0 || Cout <= 0 || Cin <= 0 || kh <= 0 || kw <= 0) return 0;
  const int K = Cin * kh * kw;
  return (size_t)dw_splits(M, Cout, K, splits) * Cout * K;
}

// dw[co, ci, ky, kx] (+)= sum over output pixels of dy x im2col(x) (bf16 operands, fp32 sums); same
// geometry arguments as es_conv2d_bwd_weight; splits <= 0 sizes the pixel split for the chip.
// flags: 1 = x is a bf16 map, 2 = dy is a bf16 map.
static int conv_dw_bf16_impl(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                             const void* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride, int pad,
                             int splits, float* workspace, float* dw, int accumulate, int flags, const float* bnm,
                             const float* bnr, const float* bng, const float* bnb, hipStream_t stream) {
  if (!x || !dy || !dw || !workspace) return ES_BAD_ARG;
  if (!es_conv2d_bf16_eligible(Cin, Cout, kh, kw) || N <= 0 || H <= 0 || W <= 0 || stride <= 0 || pad < 0 ||
      (flags & ~3))
    return ES_BAD_SHAPE;
  const int Ho = (H + 2 * pad - kh) / stride + 1, Wo = (W + 2 * pad - kw) / stride + 1;
  if (Ho <= 0 || Wo <= 0 || sxc != 1 || !st4(sxn, sxh, sxw) || !st4(syn, syh, syw) || !al16(x) || !al16(dy) ||
      !al16(workspace))
    return ES_BAD_SHAPE;
  if (bnm && (!bnr || !bng || !bnb || !al16(bnm) || !al16(bnr) || !al16(bng) || !al16(bnb))) return ES_BAD_ARG;
  const int M = N * Ho * Wo, K = Cin * kh * kw;
  const int S0 = dw_splits(M, Cout, K, splits);
  int chunk = (M + S0 - 1) / S0;
  chunk = (chunk + 31) / 32 * 32;
  const int S = (M + chunk - 1) / chunk;
  const long xb = ((long)(N - 1) * sxn + (long)(H - 1) * sxh + (long)(W - 1) * sxw + Cin) * ((flags & 1) ? 2 : 4);
  const long yb = ((long)(N - 1) * syn + (long)(Ho - 1) * syh + (long)(Wo - 1) * syw + Cout) * ((flags & 2) ? 2 : 4);
  DWConv a{x, dy, workspace, N, H, W, Cin, Ho, Wo, Cout, kh, kw, stride, pad, sxn, sxh, sxw, syn, syh, syw, M, chunk,
           bnm, bnr, bng, bnb, xb < 0x7fff0000L ? (unsigned)xb : 0u, yb < 0x7fff0000L ? (unsigned)yb : 0u, 32 / Wo,
           32 % Wo};
  int b1, b2;
  dw_tile(Cout, K, b1, b2);
  const dim3 grid((Cout + b1 - 1) / b1, (K + b2 - 1) / b2, S);
  if (b1 == 128 && b2 == 128) launch_dw_bn<128, 128>(grid, flags, a, stream);
  else if (b1 == 64 && b2 == 128) launch_dw_bn<64, 128>(grid, flags, a, stream);
  else if (b1 == 128) launch_dw_bn<128, 64>(grid, flags, a, stream);
  else launch_dw_bn<64, 64>(grid, flags, a, stream);
  const long n = (long)Cout * K;
  hipLaunchKernelGGL(convb_dw_reduce_kernel, (unsigned)((n / 4 + 63) / 64), 256, 0, stream, workspace, S, Cout, Cin,
                     kh * kw, dw, accumulate);
  return hipGetLastError() == hipSuccess ? ES_OK : ES_HIP_ERROR;
}

int es_conv2d_bwd_weight_bf16_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                                 const void* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride,
                                 int pad, int splits, float* workspace, float* dw, int accumulate, int flags,
                                 hipStream_t stream) {
  return conv_dw_bf16_impl(x, N, H, W, Cin, sxn, sxh, sxw, sxc, dy, syn, syh, syw, Cout, kh, kw, stride, pad, splits,
                           workspace, dw, accumulate, flags, nullptr, nullptr, nullptr, nullptr, stream);
}

// es_conv2d_bwd_weight_bf16_ex for the conv of es_conv2d_fwd_bf16_bnin_ex: x is the BatchNorm's input and the
// im2col gather applies the same affine map + ReLU
int es_conv2d_bwd_weight_bf16_bnin_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw,
                                      long sxc, const void* dy, long syn, long syh, long syw, int Cout, int kh, int kw,
                                      int stride, int pad, int splits, float* workspace, float* dw, int accumulate,
                                      int flags, const float* in_mean, const float* in_rstd, const float* in_gamma,
                                      const float* in_beta, hipStream_t stream) {
  if (!in_mean) return ES_BAD_ARG;
  return conv_dw_bf16_impl(x, N, H, W, Cin, sxn, sxh, sxw, sxc, dy, syn, syh, syw, Cout, kh, kw, stride, pad, splits,
                           workspace, dw, accumulate, flags, in_mean, in_rstd, in_gamma, in_beta, stream);
}

int es_conv2d_bwd_weight_bf16(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                              const float* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride,
                              int pad, int splits, float* workspace, float* dw, int accumulate, hipStream_t stream) {
  return es_conv2d_bwd_weight_bf16_ex(x, N, H, W, Cin, sxn, sxh, sxw, sxc, dy, syn, syh, syw, Cout, kh, kw, stride, pad,
                                      splits, workspace, dw, accumulate, 0, stream);
}

}  // extern "C"
