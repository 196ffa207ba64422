// Shared device helpers for the endossl gfx950 (CDNA4 / MI355X) kernels.
//
// Conventions used by every kernel in this library:
//  * wave = 64 lanes; lane = threadIdx.x & 63; g = lane >> 4 (16-lane group), r = lane & 15.
//  * MFMA is v_mfma_f32_16x16x32_bf16.  Operand maps (cdna_hip_programming.md §3):
//      A: lane holds A[row r][k = 8g + j], j = 0..7     B: lane holds B[k = 8g + j][col r]
//      D: lane holds D[row 4g + i][col r], i = 0..3
//  * Token-major activation buffers are padded to a multiple of 256 rows; pad rows are zero and
//    are never written, so GEMM tiles may read them freely (DESIGN.md "HBM layout").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  Kept in a non-template function: inside a
// kernel template the address-space-3 cast of a value-dependent pointer fails host-side template
// substitution and hipcc then silently emits no host stub for the kernel.
__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, LDS_PTR(lds), 16, 0, 0);
}

// The same DMA as inline asm (cdna_hip_programming.md §5.7 LDS-DMA recipe: M0 written and restored in the
// statement).  For loops that keep LDS-DMA in flight while they read other ring stages with
// ds_read_b64_tr_b16: hipcc cannot prove that such a transposed read does not alias a pending
// global_load_lds and drains every one of them (s_waitcnt vmcnt(0)) in front of the first read -- measured
// in the weight-gradient kernels, where it serialised each stage's load with the previous stage's MFMAs.
// An asm DMA is invisible to hipcc's waitcnt bookkeeping, so the CALLER retires it: a counted
// s_waitcnt vmcnt(N) and a barrier before any wave reads the stage (extra compiler-counted VMEM ops only
// make hipcc's own waits stricter, never looser).  No VGPR destination: register-safe.
__device__ __forceinline__ void glds16_asm(const void* src, char* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(src), "s"(dst)
               : "memory");
}

// Buffer-addressed 16-byte LDS-DMA (buffer_load_dwordx4 ... offen lds), inline asm like glds16_asm: the
// source is resource + voff (per lane, 32 bit) + soff (wave-uniform), so a loop that walks a tensor keeps one
// VGPR per piece instead of a 64-bit address.  Out-of-range pieces read as zero.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 rsrc_i4(const void* base, unsigned bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  return i32x4{__builtin_amdgcn_readfirstlane((int)(uint32_t)b), __builtin_amdgcn_readfirstlane((int)(b >> 32)),
               __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}
__device__ __forceinline__ void bl16_asm(i32x4 rsrc, unsigned voff, unsigned soff, char* lds) {
  const unsigned dst = __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(rsrc), "s"(dst), "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory");
}

// Raw buffer access (range-checked by the resource: out-of-range loads return 0, out-of-range
// stores are dropped).  Epilogues map rows past M to an out-of-range offset with a select instead
// of branching, which keeps the code straight-line so the waitcnt pass can count (a divergent
// branch around a store makes it fall back to vmcnt(0) at every join).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned ES_OOB = 0x7ffffff0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ void buf_store16(u32x4 v, __amdgpu_buffer_rsrc_t r, unsigned off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

enum EsStatus {
  ES_OK = 0,
  ES_BAD_SHAPE = -1,
  ES_BAD_ARG = -2,
  ES_HIP_ERROR = -3,
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ds_read_b64_tr_b16: within each 16-lane group, lane 4q+p supplies &tile[row q][col 4p];
// lane t of the group receives column t of the 4 rows (row q in element q).
__device__ __forceinline__ bf16x4 lds_tr4(const void* lds_byte_addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (__attribute__((address_space(3))) bf16x4*)(lds_byte_addr));
}

__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  bf16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// ---- activation-map element types (the CNN branch keeps its NHWC maps in fp32 or in bf16) ----------
// Q4<T>::t: 4 consecutive map elements as loaded (16 bytes of fp32, 8 of bf16); q4_f32 widens them,
// q4_b16 rounds them to the bf16 operand form (exact for bf16 maps), q4_store rounds fp32 values to T.
template <typename T> struct Q4;
template <> struct Q4<float> { typedef f32x4 t; };
template <> struct Q4<bf16> { typedef bf16x4 t; };
template <typename T> __device__ __forceinline__ typename Q4<T>::t q4_zero();
template <> __device__ __forceinline__ f32x4 q4_zero<float>() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
template <> __device__ __forceinline__ bf16x4 q4_zero<bf16>() {
  const bf16 z = (bf16)0.f;
  return bf16x4{z, z, z, z};
}
__device__ __forceinline__ f32x4 q4_f32(f32x4 v) { return v; }
__device__ __forceinline__ f32x4 q4_f32(bf16x4 v) { return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; }
__device__ __forceinline__ bf16x4 q4_b16(bf16x4 v) { return v; }
__device__ __forceinline__ bf16x4 q4_b16(f32x4 v) { return bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]}; }
template <typename T> __device__ __forceinline__ typename Q4<T>::t q4_load(const T* p) {
  return *(const typename Q4<T>::t*)p;
}
__device__ __forceinline__ void q4_store(float* p, f32x4 v) { *(f32x4*)p = v; }
__device__ __forceinline__ void q4_store(bf16* p, f32x4 v) { *(bf16x4*)p = q4_b16(v); }
// The BatchNorm affine map of the forward, (x - mean) * rstd * gamma + beta, with its one rounding point pinned
// (an explicit fma): shared by conv.hip's bn_apply / mask-rebuilding backward kernels and by the bf16 convs'
// gathers that apply a BatchNorm + ReLU to their input map on the fly (conv_bf16.hip, INBN), so the fused
// gather reproduces the normalised map's bits exactly.
__device__ __forceinline__ float bn_affine(float x, float mu, float rs, float ga, float be) {
  return __builtin_fmaf((x - mu) * rs, ga, be);
}
// relu(bn_affine) of 4 consecutive channels, in the map's element type (bf16 maps: rounded once, as bn_apply
// stores its output)
__device__ __forceinline__ f32x4 bn_relu4(f32x4 x, f32x4 mu, f32x4 rs, f32x4 ga, f32x4 be) {
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = fmaxf(bn_affine(x[j], mu[j], rs[j], ga[j], be[j]), 0.f);
  return o;
}
__device__ __forceinline__ f32x4 q4_bn_relu(f32x4 x, f32x4 mu, f32x4 rs, f32x4 ga, f32x4 be) {
  return bn_relu4(x, mu, rs, ga, be);
}
__device__ __forceinline__ bf16x4 q4_bn_relu(bf16x4 x, f32x4 mu, f32x4 rs, f32x4 ga, f32x4 be) {
  return q4_b16(bn_relu4(q4_f32(x), mu, rs, ga, be));
}

// scalar forms
__device__ __forceinline__ float m_f32(float v) { return v; }
__device__ __forceinline__ float m_f32(bf16 v) { return (float)v; }
__device__ __forceinline__ void m_store(float* p, float v) { *p = v; }
__device__ __forceinline__ void m_store(bf16* p, float v) { *p = (bf16)v; }

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// erf for the GELU epilogues: Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7 absolute (30x below
// half a bf16 ulp at 1.0, so the bf16 outputs match torch's exact erf), ~12 VALU ops with one
// v_exp and one v_rcp instead of ocml's piecewise erff -- the GELU epilogue runs beside MFMAs.
// The reciprocal is the raw v_rcp_f32 (1 ulp): __frcp_rn / 1.f/x compile to a correctly rounded
// division (div_scale x2, div_fmas, div_fixup, Newton steps), ~6 extra VALU per element.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  y = 1.0f - y * t * __expf(-ax * ax);
  return copysignf(y, x);
}

// exact-erf GELU, nn.GELU() default (code/models/conformer.py:9,14)
__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.0f + erf_fast(x * 0.70710678118654752f));
}
// gelu(x) and gelu'(x) together: one rcp, one exp (the erf's exp(-x^2 / 2) is the density's too)
__device__ __forceinline__ void gelu_and_grad_f(float x, float& g, float& d) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  const float e = __expf(-az * az);
  const float cdf = 0.5f * (1.0f + copysignf(1.0f - y * t * e, z));
  g = x * cdf;
  d = fmaf(x, 0.39894228040143268f * e, cdf);
}

// gelu_and_grad_f on 8 elements as 4 pairs with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32: two
// lanes' worth per instruction), each step over all 4 pairs so that dependent packed ops are not
// back to back (gfx950 pads those with s_nop).  Same operations in the same order as the scalar
// form: bit-identical results; only v_rcp / v_exp stay per element.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_and_grad_f8(const float* x, float* g, float* d) {
  f32x2 xv[4], z[4], t[4], y[4], e[4], cdf[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    xv[i] = f32x2{x[2 * i], x[2 * i + 1]};
    z[i] = xv[i] * 0.70710678118654752f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 den = __builtin_elementwise_fma(f32x2(0.3275911f), __builtin_elementwise_abs(z[i]), f32x2(1.0f));
    t[i] = f32x2{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    const f32x2 az = __builtin_elementwise_abs(z[i]);
    const f32x2 q = -az * az;
    e[i] = f32x2{__expf(q[0]), __expf(q[1])};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(f32x2(1.061405429f), t[i], f32x2(-1.453152027f));
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(1.421413741f));
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(-0.284496736f));
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(0.254829592f));
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = f32x2(1.0f) - y[i] * t[i] * e[i];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    cdf[i] = 0.5f * (f32x2(1.0f) + f32x2{copysignf(y[i][0], z[i][0]), copysignf(y[i][1], z[i][1])});
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 gv = xv[i] * cdf[i];
    const f32x2 dv = __builtin_elementwise_fma(xv[i], 0.39894228040143268f * e[i], cdf[i]);
    g[2 * i] = gv[0]; g[2 * i + 1] = gv[1];
    d[2 * i] = dv[0]; d[2 * i + 1] = dv[1];
  }
}

// the same on 4 elements (2 pairs): fewer live temporaries for register-tight epilogues; bit-identical
__device__ __forceinline__ void gelu_and_grad_f4(const float* x, float* g, float* d) {
  f32x2 xv[2], z[2], t[2], y[2], e[2], cdf[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    xv[i] = f32x2{x[2 * i], x[2 * i + 1]};
    z[i] = xv[i] * 0.70710678118654752f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x2 den = __builtin_elementwise_fma(f32x2(0.3275911f), __builtin_elementwise_abs(z[i]), f32x2(1.0f));
    t[i] = f32x2{__builtin_amdgcn_rcpf(den[0]), __builtin_amdgcn_rcpf(den[1])};
    const f32x2 az = __builtin_elementwise_abs(z[i]);
    const f32x2 q = -az * az;
    e[i] = f32x2{__expf(q[0]), __expf(q[1])};
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = __builtin_elementwise_fma(f32x2(1.061405429f), t[i], f32x2(-1.453152027f));
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(1.421413741f));
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(-0.284496736f));
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], f32x2(0.254829592f));
#pragma unroll
  for (int i = 0; i < 2; ++i) y[i] = f32x2(1.0f) - y[i] * t[i] * e[i];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    cdf[i] = 0.5f * (f32x2(1.0f) + f32x2{copysignf(y[i][0], z[i][0]), copysignf(y[i][1], z[i][1])});
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x2 gv = xv[i] * cdf[i];
    const f32x2 dv = __builtin_elementwise_fma(xv[i], 0.39894228040143268f * e[i], cdf[i]);
    g[2 * i] = gv[0]; g[2 * i + 1] = gv[1];
    d[2 * i] = dv[0]; d[2 * i + 1] = dv[1];
  }
}

// gelu'(x) = Phi(x) + x phi(x).  erf_fast's exp(-z^2), z = x / sqrt(2), IS exp(-x^2 / 2): one v_exp
// serves both the erf and the density.
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float z = x * 0.70710678118654752f;
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  const float e = __expf(-az * az);
  const float erfv = copysignf(1.0f - y * t * e, z);
  return fmaf(x, 0.39894228040143268f * e, 0.5f * (1.0f + erfv));
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 share an XCD; give each XCD a contiguous range of logical tile ids so that
// neighbouring tiles (which share an operand panel) hit the same L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// vmcnt immediates 0..63 (counted waits computed at run time)
__device__ __forceinline__ void wait_vmcnt_any(int n) {
  switch (n) {
#define ES_VM1(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
#define ES_VM8(B) ES_VM1(B) ES_VM1(B + 1) ES_VM1(B + 2) ES_VM1(B + 3) ES_VM1(B + 4) ES_VM1(B + 5) ES_VM1(B + 6) ES_VM1(B + 7)
    ES_VM8(1) ES_VM8(9) ES_VM8(17) ES_VM8(25) ES_VM8(33) ES_VM8(41) ES_VM8(49) ES_VM1(57) ES_VM1(58) ES_VM1(59)
    ES_VM1(60) ES_VM1(61) ES_VM1(62) ES_VM1(63)
#undef ES_VM8
#undef ES_VM1
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// Opt a kernel into more than 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU).  Set once per kernel
// and size (a per-function attribute, remembered per kernel address): the launchers then issue no
// host-side runtime call beyond the launch itself, which keeps them capturable into a hipGraph
// (endossl/fixmatch.py).
inline bool lds_grant_needed(const void* kernel, size_t bytes) {
  static const void* ks[256];
  static size_t bs[256];
  static int n = 0;
  for (int i = 0; i < n; ++i)
    if (ks[i] == kernel) {
      if (bs[i] >= bytes) return false;
      bs[i] = bytes;
      return true;
    }
  if (n < 256) {
    ks[n] = kernel;
    bs[n++] = bytes;
  }
  return true;
}
template <typename K>
inline void allow_lds(K kernel, size_t bytes) {
  if (bytes > 65536 && lds_grant_needed((const void*)kernel, bytes))
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}
