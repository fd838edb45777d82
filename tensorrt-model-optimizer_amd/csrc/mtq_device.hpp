// mtq_device.hpp — gfx950 (CDNA4) device helpers shared by the fake-quant kernels.
//
// Numerics notes (why each helper looks the way it does):
//  * All arithmetic is fp32, as in the reference kernels and ATen fallback
//    (modelopt/torch/quantization/tensor_quant.py:620-645, tensor_quant_gpu.cu:43-56).
//  * `div_rn` is the correctly rounded fp32 quotient q/s computed from a correctly rounded
//    reciprocal r = RN(1/s) with one FMA correction (Markstein).  Exhaustively checked on
//    the host for every fp32 significand of s at 7 exponents x every q in [-128, 127] and
//    for 16-bit q on every 64th significand (scripts/check_div_rn.c, run sliced by tests/test_div_rn_check.py): bit-identical to q / s.  It replaces two
//    ~12-instruction IEEE divisions per element by 3 instructions, which keeps the INT-n
//    qdq kernels HBM-bound (SURVEY.md §8a a9 requires `/scale`, not `*inv_scale`).
//  * Clamps are written as compare-selects so NaN propagates like torch.clamp / the
//    reference kernel's ternaries (v_max_f32/v_min_f32 would return the non-NaN operand).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtq {

constexpr float kEps = 1.0f / (1 << 24);  // tensor_quant.py:626, tensor_quant_gpu.cu:26
constexpr float kE4M3Max = 448.0f;
constexpr float kE5M2Max = 57344.0f;

// ---- element traits ---------------------------------------------------------------------
template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(float v) { return v; }
  static __device__ __forceinline__ float st(float v) { return v; }
};
template <> struct Elem<_Float16> {
  static __device__ __forceinline__ float ld(_Float16 v) { return (float)v; }
  // The empty asm pins v as an fp32 register value: without it the backend folds
  // fptrunc(fma(a, b, c)) / fptrunc(fmul) into v_fma_mixlo_f16, a single rounding straight to
  // f16 instead of the reference's fp32-then-f16 double rounding (observed on gfx950 at f16 ties).
  static __device__ __forceinline__ _Float16 st(float v) {
    asm("" : "+v"(v));
    return (_Float16)v;
  }
};
template <> struct Elem<__bf16> {
  static __device__ __forceinline__ float ld(__bf16 v) { return (float)v; }
  static __device__ __forceinline__ __bf16 st(float v) {  // v_cvt_pk_bf16_f32, RNE
    asm("" : "+v"(v));
    return (__bf16)v;
  }
};
template <> struct Elem<double> {
  static __device__ __forceinline__ float ld(double v) { return (float)v; }
  static __device__ __forceinline__ double st(float v) { return (double)v; }
};

// 16-byte vector of T, the widest coalesced per-lane access (cdna_hip_programming.md G13).
template <typename T> struct Vec {
  static constexpr int N = 16 / sizeof(T);
  union {
    uint4 raw;
    T e[N];
  };
};

template <typename T>
__device__ __forceinline__ Vec<T> ldg_vec(const T *p) {
  Vec<T> v;
  v.raw = *reinterpret_cast<const uint4 *>(p);
  return v;
}
template <typename T>
__device__ __forceinline__ void stg_vec(T *p, const Vec<T> &v) {
  *reinterpret_cast<uint4 *>(p) = v.raw;
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// streaming (non-temporal) forms: the data is touched exactly once
template <typename T>
__device__ __forceinline__ Vec<T> ldg_vec_nt(const T *p) {
  u32x4 r = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  Vec<T> v;
  v.raw = make_uint4(r.x, r.y, r.z, r.w);
  return v;
}
template <typename T>
__device__ __forceinline__ void stg_vec_nt(T *p, const Vec<T> &v) {
  u32x4 r = {v.raw.x, v.raw.y, v.raw.z, v.raw.w};
  __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(p));
}

// amax pointer of any dtype -> fp32 (reference: amax.to(at::ScalarType::Float)).
__device__ __forceinline__ float load_as_float(const void *p, int dtype, int64_t i) {
  switch (dtype) {
  case 1: return (float)reinterpret_cast<const _Float16 *>(p)[i];
  case 2: return (float)reinterpret_cast<const __bf16 *>(p)[i];
  case 3: return (float)reinterpret_cast<const double *>(p)[i];
  default: return reinterpret_cast<const float *>(p)[i];
  }
}

// ---- arithmetic helpers -------------------------------------------------------------------
// s > 0 always here, so the quotient carries q's sign; copysign (one v_bfi_b32) keeps a -0
// numerator's sign, which the final fma (+0 + -0 = +0) would otherwise drop.
__device__ __forceinline__ float div_rn(float q, float s, float r) {
  float y0 = q * r;
  float e = __builtin_fmaf(-y0, s, q);
  return __builtin_copysignf(__builtin_fmaf(e, r, y0), q);
}

__device__ __forceinline__ float clamp_nan(float v, float lo, float hi) {
  v = v > hi ? hi : v;
  v = v < lo ? lo : v;
  return v;
}

// compute_max_* clamp, tensor_quant_mx.cu:191-193: inf -> FLT_MAX, NaN kept (fmaxf then skips it)
__device__ __forceinline__ float clamp_flt_max(float a) { return a > 3.402823466e38f ? 3.402823466e38f : a; }

// Running max of magnitudes that skips NaN of either kind, on the bit patterns: a float form
// (fmaxf, or `a > m ? a : m`, which LLVM folds to v_max_f32 against a constant) lets a
// signalling NaN -- e.g. a bf16 sNaN pattern widened to fp32 -- through as a quiet NaN, where the
// reference's block max skips it (tensor_quant_mx.cu:240-294; the oracle maps NaN to 0).
// m and a are magnitudes (>= 0 or NaN); non-negative floats order like their bit patterns.
__device__ __forceinline__ uint32_t abs_bits_nonan(float v) {  // |v| bits, NaN -> +0
  const uint32_t b = __float_as_uint(v) & 0x7fffffffu;
  return b > 0x7f800000u ? 0u : b;
}
__device__ __forceinline__ float max_skip_nan(float m, float a) {
  const uint32_t mb = __float_as_uint(m), ab = abs_bits_nonan(a);
  return __uint_as_float(ab > mb ? ab : mb);
}
__device__ __forceinline__ float abs_or_zero(float v) { return __uint_as_float(abs_bits_nonan(v)); }

__device__ __forceinline__ float pow2f(int k) {  // 2^k for k in the normal range
  return __uint_as_float((uint32_t)(k + 127) << 23);
}

// ---- INT-n quant parameters -----------------------------------------------------------------
struct IntQ {
  float s;    // scale (0 when amax <= eps)
  float d;    // divisor (s, or 1 when amax <= eps)
  float r;    // RN(1/d)
  float lo, hi;
};

__device__ __forceinline__ IntQ make_intq(float amax, float max_bound, float min_bound) {
  IntQ q;
  q.lo = min_bound;
  q.hi = max_bound;
  // tensor_quant.py:625-640: scale = max_bound / amax; amax <= eps -> scale 0 for the
  // multiply and 1 for the divide.
  if (amax <= kEps) {
    q.s = 0.f;
    q.d = 1.f;
  } else {
    q.s = max_bound / amax;
    q.d = q.s;
  }
  q.r = 1.0f / q.d;
  return q;
}

__device__ __forceinline__ float int_qdq(float x, const IntQ &q) {
  float v = __builtin_rintf(x * q.s);  // torch.round_: half to even (v_rndne_f32)
  v = clamp_nan(v, q.lo, q.hi);
  return div_rn(v, q.d, q.r);
}

// ---- FP8 e4m3 qdq -------------------------------------------------------------------------
struct Fp8Q {
  float s, inv;
};
__device__ __forceinline__ Fp8Q make_fp8q(float amax) {
  // tensor_quant.py:50-54: safe_amax = where(amax <= eps, 1, amax); scale = 448.0 / safe_amax;
  // scale_inv = 1 / scale.  A Python scalar divided by a tensor is Tensor.__rtruediv__ =
  // reciprocal(t) * scalar, so scale = RN(RN(1/safe) * 448), not RN(448/safe) (the C++ ext's
  // `448.f / safe_amax`, tensor_quant_gpu_fp8.cu:97, is the same ATen scalar/tensor operator).
  Fp8Q q;
  float safe = amax <= kEps ? 1.0f : amax;
  q.s = (1.0f / safe) * kE4M3Max;
  q.inv = 1.0f / q.s;
  return q;
}

// Two elements at a time through the packed gfx950 converts (OCP e4m3fn, RNE).
__device__ __forceinline__ void fp8_qdq2(float &a, float &b, const Fp8Q &q) {
  float va = a * q.s, vb = b * q.s;
  float ca = clamp_nan(va, -kE4M3Max, kE4M3Max);
  float cb = clamp_nan(vb, -kE4M3Max, kE4M3Max);
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(ca, cb, 0, false);
  a = __builtin_amdgcn_cvt_f32_fp8(p, 0) * q.inv;
  b = __builtin_amdgcn_cvt_f32_fp8(p, 1) * q.inv;
}

// ---- element-format conversion (reference tensor_quant_mx.h:61-188) --------------------------
// Saturating round-to-nearest for the table formats.  The reference walks a value/bound table
// (round_to_even / round_away_from_zero, tensor_quant_mx.h:81-120); these formats are regular
// minifloats, so the same result is rint(v / q) * q with the quantum q = 2^(max(e, emin) - m),
// ties-to-even-index == ties-to-even-mantissa.  v >= 0; inf/NaN saturate to the max (:127-129).
struct TableFmt {
  int m;        // mantissa bits
  int emin;     // exponent of the smallest normal
  float vmax;   // largest magnitude
  bool away;    // E3M0 rounds ties away from zero (tensor_quant_mx.h:143-158)
};

__device__ __forceinline__ TableFmt table_fmt(int fmt) {
  switch (fmt) {
  case 3: return {3, 3, 7.0f, false};     // E0M3: 0..7
  case 4: return {2, 1, 3.5f, false};     // E1M2: 0..3.5 step 0.5
  case 5: return {0, -2, 16.0f, true};    // E3M0: 0, 0.25 .. 16
  case 7: return {2, -2, 28.0f, false};   // E3M2
  case 8: return {3, 0, 7.5f, false};     // E2M3
  default: return {1, 0, 6.0f, false};    // E2M1: 0 .. 6
  }
}

__device__ __forceinline__ float round_table(float v, const TableFmt &f) {
  v = fminf(v, f.vmax);  // fminf(NaN, max) = max: NaN saturates like the table path
  int e = (int)((__float_as_uint(v) >> 23) & 0xff) - 127;
  e = e < f.emin ? f.emin : e;
  int k = e - f.m;
  float t = v * pow2f(-k);
  float r = f.away ? __builtin_floorf(t + 0.5f) : __builtin_rintf(t);
  return fminf(r * pow2f(k), f.vmax);
}

// convert_to_types for v = |x| * scale >= 0 (tensor_quant_mx.h:161-188).
__device__ __forceinline__ float convert_fmt(float v, int fmt) {
  switch (fmt) {
  case 0: {  // E4M3: __nv_fp8_e4m3 (satfinite, RNE)
    float c = v != v ? v : fminf(v, kE4M3Max);
    int p = __builtin_amdgcn_cvt_pk_fp8_f32(c, c, 0, false);
    return __builtin_amdgcn_cvt_f32_fp8(p, 0);
  }
  case 1: {  // E5M2
    float c = v != v ? v : fminf(v, kE5M2Max);
    int p = __builtin_amdgcn_cvt_pk_bf8_f32(c, c, 0, false);
    return __builtin_amdgcn_cvt_f32_bf8(p, 0);
  }
  case 2: {  // INT8 symmetric: rint, clamp to +-127
    float r = __builtin_rintf(v);
    return fminf(r, 127.0f);
  }
  case 9: return 0.0f;  // E8M0 is not an element format (convert_to_types default)
  default: return round_table(v, table_fmt(fmt));
  }
}

__device__ __forceinline__ float format_max(int fmt) {  // get_format_max, tensor_quant_mx.h:190-213
  switch (fmt) {
  case 0: return 448.f;
  case 1: return 57344.f;
  case 2: return 127.f;
  case 6: return 6.f;
  case 3: return 7.f;
  case 5: return 16.f;
  case 4: return 3.5f;
  case 7: return 28.f;
  case 8: return 7.5f;
  default: return 0.f;
  }
}

// E8M0 "NV" scale (tensor_quant_mx.cu:104-137): unscale = 2^ceil(log2(amax / emax)) from the
// bits of the RN ratio; amax in {0, inf, NaN} -> (1, 1) (compute_scale, :139-145).
__device__ __forceinline__ void e8m0_scale(float amax, float emax, float &scale,
                                           float &unscale) {
  if (amax == 0.f || __builtin_isinf(amax) || amax != amax) {
    scale = 1.f;
    unscale = 1.f;
    return;
  }
  float ratio = amax / emax;
  uint32_t b = __float_as_uint(ratio);
  uint32_t ex = (b >> 23) & 0xff, sig = b & 0x7fffff;
  int ue = (sig > 0 && ex != 0xfe && !(ex == 0 && sig <= 0x400000)) ? (int)ex - 126 : (int)ex - 127;
  scale = __builtin_ldexpf(1.f, -ue);
  unscale = __builtin_ldexpf(1.f, ue);
}

// Non-E8M0 scale formats: compute_scale / compute_scale_with_global (tensor_quant_mx.cu:139-183).
__device__ __forceinline__ void generic_scale(float amax, int fmt, int sfmt, float &scale,
                                              float &unscale) {
  if (amax == 0.f || __builtin_isinf(amax) || amax != amax) {
    scale = 1.f;
    unscale = 1.f;
    return;
  }
  const float emax = format_max(fmt);
  double sc = (double)(emax / amax);
  double inv = (double)convert_fmt(fabsf((float)(1.0 / sc)), sfmt);
  sc = 1.0 / inv;
  scale = (float)sc;
  unscale = (float)inv;
}

__device__ __forceinline__ void global_scale(float gamax, float lamax, int fmt, int sfmt,
                                             float &scale, float &unscale) {
  bool li = lamax == 0.f || __builtin_isinf(lamax) || lamax != lamax;
  bool gi = gamax == 0.f || __builtin_isinf(gamax) || gamax != gamax;
  if (li || gi) {
    scale = 1.f;
    unscale = 1.f;
    return;
  }
  const float em = format_max(fmt), sm = format_max(sfmt);
  const float local_unscale = lamax / em;
  const double two_level = (double)sm * (double)(em / gamax);
  const double luq =
      (double)convert_fmt(fabsf((float)((double)local_unscale * two_level)), sfmt) / two_level;
  scale = (float)(1.0 / luq);
  unscale = (float)luq;
}

// ---- native CDNA4 FP4 (E2M1) converts on packed 16-bit pairs ---------------------------------
// v_cvt_scalef32_pk_fp4_{bf16,f16} converts two 16-bit floats to E2M1 codes of x / 2^e(s) and
// v_cvt_scalef32_pk_{bf16,f16}_fp4 back to code * 2^e(s) (e(s) = s's exponent field).  Measured
// on gfx950 (scripts/probe_fp4_cvt*.hip, profiles/r02/fp4_convert_probe.txt): for every bf16 /
// f16 pattern and every power-of-two scale 2^-130..2^130 they equal the fp32 converts composed
// with an exact widening / an RNE narrowing, and the fp32 down-convert equals the reference E2M1
// rounding (tensor_quant_mx.h:104-141: nearest, ties to the even code, saturating at 6) of x / s
// for every finite value, sign included (-tiny -> -0).  They differ from the reference only on
// x = -0 (-0 where the reference gives +0) and NaN (signed +-6 where MX gives +6 and NVFP4 -6),
// which the kernels route to the emulated path.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));

template <typename T> struct Fp4Native;
template <> struct Fp4Native<__bf16> {
  static constexpr uint32_t kInfBits = 0x7f80u;  // |x| patterns above this are NaN
  static __device__ __forceinline__ uint32_t down(uint32_t w, float s) {
    return __builtin_amdgcn_cvt_scalef32_pk_fp4_bf16(0u, __builtin_bit_cast(bf16x2_t, w), s, 0);
  }
  static __device__ __forceinline__ uint32_t up(uint32_t p, float s) {
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(p, s, 0));
  }
};
template <> struct Fp4Native<_Float16> {
  static constexpr uint32_t kInfBits = 0x7c00u;
  static __device__ __forceinline__ uint32_t down(uint32_t w, float s) {
    return __builtin_amdgcn_cvt_scalef32_pk_fp4_f16(0u, __builtin_bit_cast(f16x2_t, w), s, 0);
  }
  static __device__ __forceinline__ uint32_t up(uint32_t p, float s) {
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(p, s, 0));
  }
};

// ---- native CDNA4 FP8 (E4M3) scaled converts on packed 16-bit pairs -------------------------------
// v_cvt_scalef32_pk_fp8_{bf16,f16}: two 16-bit floats -> two E4M3 bytes of x / 2^e(s), written to
// the low or high 16 bits of the destination (word_sel); v_cvt_scalef32_pk_{bf16,f16}_fp8: two E4M3
// bytes (low / high half) -> code * 2^e(s).  Used only where the MX E4M3 block scale keeps
// |x| / 2^e <= 448 (e8m0_scale) and the exponents in the range tests/test_gpu_mx_native.py checks
// exhaustively against the emulated mx_vec_kernel path (every 16-bit pattern at every scale).
typedef short i16x2_t __attribute__((ext_vector_type(2)));
template <typename T> struct Fp8Native;
template <> struct Fp8Native<__bf16> {
  // w0, w1: two packed pairs -> four E4M3 bytes
  static __device__ __forceinline__ uint32_t down(uint32_t w0, uint32_t w1, float s) {
    i16x2_t p = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16((i16x2_t){0, 0}, __builtin_bit_cast(bf16x2_t, w0), s, false);
    p = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(p, __builtin_bit_cast(bf16x2_t, w1), s, true);
    return __builtin_bit_cast(uint32_t, p);
  }
  static __device__ __forceinline__ uint32_t up(uint32_t p, float s, bool hi) {
    return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(p, s, true)
                                           : __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(p, s, false));
  }
};
template <> struct Fp8Native<_Float16> {
  static __device__ __forceinline__ uint32_t down(uint32_t w0, uint32_t w1, float s) {
    i16x2_t p = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16((i16x2_t){0, 0}, __builtin_bit_cast(f16x2_t, w0), s, false);
    p = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(p, __builtin_bit_cast(f16x2_t, w1), s, true);
    return __builtin_bit_cast(uint32_t, p);
  }
  static __device__ __forceinline__ uint32_t up(uint32_t p, float s, bool hi) {
    return __builtin_bit_cast(uint32_t, hi ? __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(p, s, true)
                                           : __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(p, s, false));
  }
};

// Per-lane scan of 4 packed 16-bit pairs: the largest |x| pattern (NaN patterns sort above inf)
// and whether any element is -0 (pattern 0x8000), two packed u16 ops per pair.
struct PairScan {
  uint32_t max_abs;
  bool neg_zero;
};
__device__ __forceinline__ PairScan scan_pairs(const uint32_t (&w)[4]) {
  u16x2_t mx = {0, 0}, mn = {0xffff, 0xffff};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mx = __builtin_elementwise_max(mx, __builtin_bit_cast(u16x2_t, w[j] & 0x7fff7fffu));
    mn = __builtin_elementwise_min(mn, __builtin_bit_cast(u16x2_t, w[j] ^ 0x80008000u));
  }
  const uint32_t m = mx.x > mx.y ? mx.x : mx.y;
  return {m, mn.x == 0 || mn.y == 0};
}

// 16-bit pattern -> fp32 value
template <typename T> __device__ __forceinline__ float half_bits_to_float(uint32_t b) {
  return Elem<T>::ld(__builtin_bit_cast(T, (uint16_t)b));
}

// ---- reductions -----------------------------------------------------------------------------
// |x| bit patterns compare like the magnitudes and NaN (exponent all ones, mantissa != 0) sorts
// above +inf, so an unsigned max propagates NaN the way torch.max does.
__device__ __forceinline__ uint32_t abs_bits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

template <typename T> __device__ __forceinline__ uint32_t abs_bits_t(T v) {
  return abs_bits(Elem<T>::ld(v));
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t t = (uint32_t)__shfl_xor((int)v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

// max over aligned groups of G consecutive lanes (G power of two <= 64)
// Cross-lane moves inside a row of 16 lanes on the DPP path of the VALU (no LDS round trip, no
// lgkmcnt wait): xor 1 / xor 2 as quad permutations, then the half-row and row mirrors (lane i
// <- 7 - i / 15 - i), which pair every lane with one of the other half once the smaller groups are
// reduced -- enough for a max.  Groups of 32 / 64 keep __shfl_xor (ds_bpermute).
template <int CTRL> __device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int G> __device__ __forceinline__ uint32_t group_max_u32(uint32_t v) {
  if constexpr (G <= 16) {
    if constexpr (G >= 2) v = max(v, dpp_u32<0xB1>(v));   // quad_perm [1, 0, 3, 2]
    if constexpr (G >= 4) v = max(v, dpp_u32<0x4E>(v));   // quad_perm [2, 3, 0, 1]
    if constexpr (G >= 8) v = max(v, dpp_u32<0x141>(v));  // row_half_mirror
    if constexpr (G >= 16) v = max(v, dpp_u32<0x140>(v)); // row_mirror
    return v;
  } else {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) {
      uint32_t t = (uint32_t)__shfl_xor((int)v, o, 64);
      v = t > v ? t : v;
    }
    return v;
  }
}

template <int G> __device__ __forceinline__ float group_max_f(float v) {
  if constexpr (G <= 16) {
    if constexpr (G >= 2) v = fmaxf(v, __uint_as_float(dpp_u32<0xB1>(__float_as_uint(v))));
    if constexpr (G >= 4) v = fmaxf(v, __uint_as_float(dpp_u32<0x4E>(__float_as_uint(v))));
    if constexpr (G >= 8) v = fmaxf(v, __uint_as_float(dpp_u32<0x141>(__float_as_uint(v))));
    if constexpr (G >= 16) v = fmaxf(v, __uint_as_float(dpp_u32<0x140>(__float_as_uint(v))));
    return v;
  } else {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
  }
}

// ---- fast unsigned division by a run-time constant (Granlund-Montgomery), n < 2^31 ----------
// l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, n / d = (umulhi(n, m) + n) >> l.
struct FastDiv {
  uint32_t d, m, s;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv &f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}
__device__ __forceinline__ uint32_t fmod_(uint32_t n, uint32_t q, const FastDiv &f) {
  return n - q * f.d;
}

// ---- dispatch registry (host side): one relaxed atomic increment per launch of the kernel
// families below, read through mtq_dispatch_counts (which kernel a call reached is otherwise
// invisible to a caller: the launchers pick among vector / group / row-wave / persistent forms
// by shape and alignment).  Names in mtq_dispatch_name; the order is the ABI.
enum DispatchId {
  kDispEwVec, kDispEwGroupSk, kDispEwGroup, kDispEwRowwave, kDispAmaxPersist, kDispAmaxRowsU,
  kDispAmaxRowsShort, kDispAmaxColsWide, kDispBlockQuantDyn, kDispHistValue, kDispHistValueChunked,
  kDispMxVec, kDispMxE2m1Native, kDispNvfp4NativeU, kDispAwqSearchPp, kDispAwqPrescale, kDispAwqMseMulti,
  kDispHistValueNz, kDispMxE4m3Native, kDispAwqSearchW4, kDispCount
};
void count_dispatch(int id);

}  // namespace mtq
