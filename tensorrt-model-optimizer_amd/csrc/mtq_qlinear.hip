// mtq_qlinear.hip — the QuantLinear simulated GEMM for short inputs on MFMA (gfx950).
//
// Reference: a fake-quantised nn.Linear evaluates F.linear(qdq(x), qdq(W), b)
// (nn/modules/quant_module.py:257-278 + quant_linear.py:38-53): the weight quantizer writes a
// full dequantised copy of W to HBM on every forward and the GEMM reads it back, so for
// decode-shaped inputs (a few tokens) the linear costs three passes over W (read, write, read)
// where the GEMM itself needs one.  Here the weight fake quant is applied to the B fragments in
// registers, between the global load and the MFMA: one pass over W.
//
// y[M, N] = x[M, K] · qdq(W)[N, K]^T (+ bias), bf16/f16 in and out, fp32 accumulate on
// v_mfma_f32_16x16x32_{bf16,f16}.  qdq(W) is element for element the weight fake quant of
// mtq_fake_tensor_quant_with_axis / mtq_fake_e4m3fy_with_axis (same make_intq / make_fp8q scale
// derivation, same rounding steps), so the dequantised weight values are equal to the unfused
// path's; only the GEMM summation order differs (as between any two GEMM libraries).  The one
// liberty taken: a -0 weight may come out as +0 (no copysign), which no sum starting from +0 can
// observe.
//
// Streaming kernel (qlinear_stream_kernel).  A unit is one 16-row tile of W times one chunk of
// K steps (32 columns a step); every wave owns one unit, so a launch has tiles x S waves and the
// small projections (k/v: 64 tiles) are spread over the whole chip by splitting K (S chunks)
// instead of leaving 3/4 of the CUs idle.  Lane l holds W row n0 + (l & 15) and the 8 K-elements
// 8 (l >> 4) .. +7 of each step (the B layout of mfma_f32_16x16x32); U steps form a batch whose
// W, x and amax loads are issued before the previous batch is quantised (register double
// buffer, late vmcnt: the guide's GEMV recipe).  Loads go through a buffer descriptor over the
// wave's 16 rows (32-bit lane offsets, scalar step offsets: no VALU address arithmetic).  x rows
// >= M are not zero-filled: lanes of such rows re-read row M-1, and the MFMA output rows they
// feed are never stored.  qdq runs on fp32 pairs (v_pk_mul/v_pk_fma, v_maximum3/v_minimum3
// NaN-propagating clamps, v_cvt_pk_bf16_f32), ~6.5 VALU per weight for INT-n, ~5.5 for FP8.
// S > 1 writes fp32 partial tiles to a workspace and qlinear_splitk_finish sums them in chunk
// order (deterministic), adds the bias in fp32 and rounds once.
//
// qlinear_wg_kernel (the first version: one workgroup per 16-row tile, waves splitting K, LDS
// reduce) remains for amax blocks that do not line up with the U-step batches (e.g. block 96).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"

using namespace mtq;

namespace mtq {
int host_check_launch();
int host_num_cus();
}

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename T> struct Mfma;
template <> struct Mfma<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  typedef __bf16 v2 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  // two packed bf16 -> fp32 pair (exact: a shift and a mask)
  static __device__ __forceinline__ f2 unpack(uint32_t w) {
    return f2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  }
  // fp32 pair -> two packed bf16, RNE (v_cvt_pk_bf16_f32)
  static __device__ __forceinline__ uint32_t pack(f2 v) {
    asm("" : "+v"(v));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, v2));
  }
};
template <> struct Mfma<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  typedef _Float16 v2 __attribute__((ext_vector_type(2)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ f2 unpack(uint32_t w) {
    return __builtin_convertvector(__builtin_bit_cast(v2, w), f2);
  }
  // v_cvt_pk_f16_f32 (RNE); the asm pins the fp32 values so no mixed-precision fma folds the
  // final fp32 rounding away (see Elem<_Float16>::st)
  static __device__ __forceinline__ uint32_t pack(f2 v) {
    asm("" : "+v"(v));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, v2));
  }
};

template <typename T>
__device__ __forceinline__ typename Mfma<T>::v8 as_v8(const Vec<T> &v) {
  typename Mfma<T>::v8 r;
  __builtin_memcpy(&r, &v.raw, 16);
  return r;
}
template <typename T>
__device__ __forceinline__ typename Mfma<T>::v8 as_v8(const u32x4 &v) {
  return __builtin_bit_cast(typename Mfma<T>::v8, v);
}

struct QlParams {
  const void *amax;
  int amax_dtype;
  int64_t amax_numel;  // 1: per tensor; else one amax per `block` consecutive elements of W
  int64_t block;
  float max_bound, min_bound;  // INT
};

// KIND 0: INT-n (IntQ), 1: FP8 e4m3 (Fp8Q)
template <int KIND> struct QParam;
template <> struct QParam<0> {
  IntQ q;
  __device__ __forceinline__ void make(float a, const QlParams &p) { q = make_intq(a, p.max_bound, p.min_bound); }
  template <typename T> __device__ __forceinline__ void apply(Vec<T> &v) const {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; ++j) v.e[j] = Elem<T>::st(int_qdq(Elem<T>::ld(v.e[j]), q));
  }
  // two packed 16-bit weights: rint(w * s), NaN-propagating clamp, RN(v / d) (Markstein with
  // r = RN(1/d), mtq_device.hpp div_rn without the -0 copysign), packed back
  template <typename T> __device__ __forceinline__ uint32_t pair(uint32_t w) const {
    f2 v = Mfma<T>::unpack(w) * f2{q.s, q.s};
    v.x = __builtin_rintf(v.x);
    v.y = __builtin_rintf(v.y);
    v.x = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v.x, q.lo), q.hi);
    v.y = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v.y, q.lo), q.hi);
    const f2 r = {q.r, q.r}, d = {q.d, q.d};
    const f2 y0 = v * r;
    const f2 e = __builtin_elementwise_fma(-y0, d, v);
    return Mfma<T>::pack(__builtin_elementwise_fma(e, r, y0));
  }
};
template <> struct QParam<1> {
  Fp8Q q;
  __device__ __forceinline__ void make(float a, const QlParams &) { q = make_fp8q(a); }
  template <typename T> __device__ __forceinline__ void apply(Vec<T> &v) const {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; j += 2) {
      float a = Elem<T>::ld(v.e[j]), b = Elem<T>::ld(v.e[j + 1]);
      fp8_qdq2(a, b, q);
      v.e[j] = Elem<T>::st(a);
      v.e[j + 1] = Elem<T>::st(b);
    }
  }
  // fp8_qdq2 on a packed pair: clamp(w * s, +-448) (NaN kept) -> e4m3 (RNE) -> fp32 -> * inv
  template <typename T> __device__ __forceinline__ uint32_t pair(uint32_t w) const {
    f2 v = Mfma<T>::unpack(w) * f2{q.s, q.s};
    v.x = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v.x, -kE4M3Max), kE4M3Max);
    v.y = __builtin_elementwise_minimum(__builtin_elementwise_maximum(v.y, -kE4M3Max), kE4M3Max);
    const int p8 = __builtin_amdgcn_cvt_pk_fp8_f32(v.x, v.y, 0, false);
    const f2 f = __builtin_amdgcn_cvt_pk_f32_fp8(p8, false);
    return Mfma<T>::pack(f * f2{q.inv, q.inv});
  }
};

// ---- streaming kernel ---------------------------------------------------------------------
constexpr int kStreamWaves = 4;  // waves per workgroup (each wave independent)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void *base, uint32_t bytes) {
  // descriptor inputs made provably wave-uniform (guide T20): no waterfall loops
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// PT: per-tensor amax.  SPB: 0 = amax blocks hold a whole number of U-step batches (one amax per
// batch per lane), else K steps per amax block (SPB divides U: U / SPB amax per batch).
template <typename T, int KIND, int U, bool PT, int SPB>
__global__ __launch_bounds__(kStreamWaves * 64) void qlinear_stream_kernel(
    const T *__restrict__ x, const T *__restrict__ w, T *__restrict__ y, const T *__restrict__ bias,
    float *__restrict__ part, int M, int N, int K, int tiles, int S, int kcs, QlParams p) {
  constexpr int NA = PT ? 0 : (SPB == 0 ? 1 : U / SPB);  // amax values per batch per lane
  const int lane = threadIdx.x & 63;
  // the wave id made provably uniform: every index below is then scalar (SGPR soffsets)
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * kStreamWaves + (threadIdx.x >> 6));
  if (unit >= tiles * S) return;  // wave-uniform; the kernel has no barrier
  const int tile = unit % tiles, chunk = unit / tiles;  // a workgroup's waves: adjacent tiles
  const int r = lane & 15, qd = lane >> 4;
  const int nsteps = K >> 5;
  const int s0 = chunk * kcs;
  const int s1 = s0 + kcs < nsteps ? s0 + kcs : nsteps;
  const int n0 = tile * 16;

  // W: descriptor over the wave's 16 rows; lane offset row r, columns 8 qd..; step s at s*64 B
  const __amdgpu_buffer_rsrc_t wr = wave_rsrc(w + (int64_t)n0 * K, (uint32_t)(16u * (uint32_t)K * 2u));
  const uint32_t wlane = (uint32_t)(r * K + qd * 8) * 2u;
  const int xr = r < M ? r : M - 1;
  const __amdgpu_buffer_rsrc_t xrs = wave_rsrc(x, (uint32_t)((uint32_t)M * (uint32_t)K * 2u));
  const uint32_t xlane = (uint32_t)(xr * K + qd * 8) * 2u;
  // amax of W row n0 + r, block b: amax[(n0 + r) * (K / block) + b]
  const int spb = PT ? nsteps : (int)(p.block >> 5);
  const int64_t row_blk = PT ? 0 : (int64_t)(n0 + r) * (K / p.block);

  const float *amax = reinterpret_cast<const float *>(p.amax);  // fp32 (host-checked)
  QParam<KIND> qp;
  if (PT) qp.make(amax[0], p);

  // amax block of the batch being loaded, tracked incrementally (no per-batch division); a
  // dummy tail batch may step one block past the row, so the index is clamped
  const int nblk = PT ? 1 : (int)(K / p.block);
  int lkb = PT ? 0 : s0 / spb, lrem = PT ? 0 : s0 % spb;
  auto load = [&](int s, u32x4 *wv, u32x4 *xv, float *av) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int st = s + u < s1 ? s + u : s1 - 1;  // scalar clamp: the tail re-reads a valid step
      wv[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wlane, st * 64, 2));
      xv[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, xlane, st * 64, 0));
    }
    if constexpr (NA > 0) {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        int kb = SPB == 0 ? lkb : (s + i * SPB) / SPB;  // SPB > 0: s0 and U are multiples of SPB
        kb = kb < nblk - 1 ? kb : nblk - 1;
        av[i] = amax[row_blk + kb];
      }
      if (SPB == 0) {
        lrem += U;
        if (lrem >= spb) {
          lrem -= spb;
          ++lkb;
        }
      }
    }
  };

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t cur = 0;
  auto compute = [&](int s, const u32x4 *wv, const u32x4 *xv, const float *av) {
    if (SPB == 0 && !PT && __float_as_uint(av[0]) != cur) {  // per lane: a new block of its row
      cur = __float_as_uint(av[0]);
      qp.make(av[0], p);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u >= s1) break;  // wave-uniform
      if (SPB > 0 && u % (SPB > 0 ? SPB : 1) == 0) qp.make(av[u / (SPB > 0 ? SPB : 1)], p);
      u32x4 b;
      b.x = qp.template pair<T>(wv[u].x);
      b.y = qp.template pair<T>(wv[u].y);
      b.z = qp.template pair<T>(wv[u].z);
      b.w = qp.template pair<T>(wv[u].w);
      acc = Mfma<T>::mma(as_v8<T>(xv[u]), as_v8<T>(b), acc);
    }
  };

  // ping-pong between two register sets (a copy of in-flight load destinations would wait for
  // them): batch A is quantised while B loads, then B while A loads
  u32x4 wa[U], xa[U], wb[U], xb[U];
  float aa[NA > 0 ? NA : 1], ab[NA > 0 ? NA : 1];
  load(s0, wa, xa, aa);
  if (SPB == 0 && !PT) {
    cur = __float_as_uint(aa[0]);
    qp.make(aa[0], p);
  }
  for (int s = s0; s < s1; s += 2 * U) {
    load(s + U, wb, xb, ab);
    compute(s, wa, xa, aa);
    if (s + U >= s1) break;
    load(s + 2 * U, wa, xa, aa);
    compute(s + U, wb, xb, ab);
  }
  // D layout of mfma_f32_16x16x32: col = lane & 15 (n), row = 4 (lane >> 4) + i (m)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = qd * 4 + i;
    if (m >= M) break;
    if (S == 1) {
      float v = acc[i];
      if (bias) v += Elem<T>::ld(bias[n0 + r]);
      y[(int64_t)m * N + n0 + r] = Elem<T>::st(v);
    } else {
      part[((int64_t)chunk * M + m) * N + n0 + r] = acc[i];
    }
  }
}

// ---- LDS-DMA streaming kernel ----------------------------------------------------------------
// Same units, lane layout and qdq as qlinear_stream_kernel, but every operand reaches the MFMA
// through LDS.  A register load of the B fragment reads 16 rows x 64 B per instruction, and that
// shape alone capped the weight stream at ~4.3 TB/s (loads-only probe; 1 KB-contiguous
// instructions of the same bytes: ~5.9).  Here a batch (U = 4 steps = 128 columns) is one group
// of buffer_load ... lds instructions into a per-wave ring slot:
//   W     4 x (4 rows x 256 B: whole 128 B lines), chunk c of row r at c ^ (r & 7) (the swizzle
//         goes on the source side, LDS-DMA writes lane-linear), so each 8-lane group of a
//         fragment read hits 8 distinct 16 B bank groups;
//   x     M == 1: one dword-per-lane DMA of the row's 256 B; else XI = ceil(M/4) DMAs of 4 rows
//         (rows past M re-read row M-1; the MFMA rows they feed are never stored);
//   amax  (per-row / per-block amax) one dword per lane, lane l -> row l & 15's block.
// The slot is read back with ds_read_b128 / ds_read_b32 in one asm statement.  No operand has a
// register destination in flight, so hipcc inserts no vmcnt of its own and the loop's only
// wait is the counted one: R - 1 groups ahead, vmcnt((R - 1) x group size) retires this batch's
// group and leaves the next R - 1 in flight (past the end, the group's descriptors have no
// records: the DMAs move nothing but keep the count).
constexpr int kSlotW = 4096;
constexpr int kSlotA = 256;

// buffer_load ... lds (LDS-DMA through a buffer descriptor).  The builtin only exists for the
// device pass: named in a kernel body seen by the host pass, it silently drops that kernel's
// host stub (an undefined __device_stub__ at load time), hence the device-pass guard.
#if defined(__HIP_DEVICE_COMPILE__)
#define MTQ_DMA(rsrc, lds, bytes, voff, soff, aux) \
  __builtin_amdgcn_raw_ptr_buffer_load_lds((rsrc), (__attribute__((address_space(3))) void *)(lds), bytes, (voff), (soff), 0, aux)
#else
#define MTQ_DMA(rsrc, lds, bytes, voff, soff, aux) ((void)(rsrc), (void)(lds), (void)(voff), (void)(soff))
#endif

template <int N> __device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// XM: x rows class, 1 (M == 1), 4, 8 or 16; R ring slots per wave
template <int XM> struct XLayout {
  static constexpr int dmas = XM == 1 ? 1 : XM / 4;             // x DMA instructions per batch
  static constexpr int bytes = XM == 1 ? 256 : (XM / 4) * 1024;  // x bytes per slot
  static constexpr int slot = kSlotW + bytes + kSlotA;
  // ring slots: 2.  Measured (gate_proj 14336 x 4096, FP8 per tensor, M = 1): 4 slots (two
  // workgroups per CU) 24.2 us, 3 slots 22.3, 2 slots (four workgroups, 16 waves per CU) 20.0 --
  // more waves to overlap one wave's qdq with another's DMA beat a deeper ring per wave
  static constexpr int ring = 2;
};

// One unit (16-row tile x K chunk) of one linear; `unit` and `wave` wave-uniform.
template <typename T, int KIND, bool PT, int XM>
__device__ __forceinline__ void qlinear_dma_unit(
    const T *__restrict__ x, const T *__restrict__ w, T *__restrict__ y, const T *__restrict__ bias,
    float *__restrict__ part, int M, int N, int K, int tiles, int S, int kcs, const QlParams &p,
    int unit, int wave) {
  constexpr int U = 4;
  using XL = XLayout<XM>;
  constexpr int R = XL::ring, SLOT = XL::slot;
  constexpr int GROUP = 4 + XL::dmas + (PT ? 0 : 1);  // DMA instructions per batch
  __shared__ __attribute__((aligned(16))) unsigned char lds[kStreamWaves * R * SLOT];
  const int lane = threadIdx.x & 63;
  const int tile = unit % tiles, chunk = unit / tiles;
  const int r = lane & 15, qd = lane >> 4;
  const int nsteps = K >> 5;
  const int s0 = chunk * kcs;
  const int s1 = s0 + kcs < nsteps ? s0 + kcs : nsteps;
  const int nb = (s1 - s0 + U - 1) / U;
  const int n0 = tile * 16;

  // descriptors (wave-uniform inputs) and the null descriptor of the tail groups
  const __amdgpu_buffer_rsrc_t wr = wave_rsrc(w + (int64_t)n0 * K, (uint32_t)(16u * (uint32_t)K * 2u));
  const __amdgpu_buffer_rsrc_t xrs = wave_rsrc(x, (uint32_t)((uint32_t)M * (uint32_t)K * 2u));
  const __amdgpu_buffer_rsrc_t nul = wave_rsrc(w, 0u);
  const int spb = PT ? nsteps : (int)(p.block >> 5);
  const int nblk = PT ? 1 : (int)(K / p.block);
  const __amdgpu_buffer_rsrc_t ars =
      wave_rsrc(p.amax, PT ? 4u : (uint32_t)((uint32_t)N * (uint32_t)nblk * 4u));

  // per-lane DMA offsets.  W instruction i: row 4i + (lane >> 4), source chunk (lane & 15) ^ (row & 7)
  uint32_t wv_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = 4 * i + (lane >> 4), c = lane & 15;
    wv_off[i] = (uint32_t)(row * K * 2 + ((c ^ (row & 7)) << 4));
  }
  uint32_t xv_off[XL::dmas];
#pragma unroll
  for (int i = 0; i < XL::dmas; ++i) {
    if (XM == 1) {
      xv_off[i] = (uint32_t)lane * 4u;  // 64 dwords = the row's 256 B
    } else {
      int row = 4 * i + (lane >> 4);
      const int c = lane & 15;
      const int src = row < M ? row : M - 1;
      xv_off[i] = (uint32_t)(src * K * 2 + ((c ^ (row & 7)) << 4));
    }
  }
  const uint32_t av_off = PT ? 0u : (uint32_t)((n0 + r) * nblk) * 4u;

  unsigned char *const ring = lds + wave * (R * SLOT);
  const uint32_t lds_base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) unsigned char *)ring);
  // read offsets within a slot: B fragment of step u (row r, chunk 4u + qd, swizzled), A
  // fragment of step u (x row r, clamped to the rows the DMAs wrote), the row's amax
  uint32_t wr_off[U], xr_off[U];
  const int xrr = XM == 1 ? 0 : (r < XM ? r : XM - 1);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    wr_off[u] = (uint32_t)(r * 256 + (((4 * u + qd) ^ (r & 7)) << 4));
    xr_off[u] = (uint32_t)(kSlotW + (XM == 1 ? (u * 64 + qd * 16) : (xrr * 256 + (((4 * u + qd) ^ (xrr & 7)) << 4))));
  }
  const uint32_t ar_off = (uint32_t)(kSlotW + XL::bytes + r * 4);

  QParam<KIND> qp;
  if (PT) qp.make(reinterpret_cast<const float *>(p.amax)[0], p);

  // group of batch b into slot b % R (slot index tracked by the caller)
  int lkb = PT ? 0 : s0 / spb, lrem = PT ? 0 : s0 % spb;  // amax block of the next group
  auto issue = [&](int b, int slot) {
    const bool live = b < nb;  // wave-uniform
    const int s = s0 + (live ? b : 0) * U;
    unsigned char *sl = ring + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 4; ++i) MTQ_DMA(live ? wr : nul, sl + i * 1024, 16, wv_off[i], s * 64, 2);
#pragma unroll
    for (int i = 0; i < XL::dmas; ++i) {
      if (XM == 1)
        MTQ_DMA(live ? xrs : nul, sl + kSlotW, 4, xv_off[i], s * 64, 0);
      else
        MTQ_DMA(live ? xrs : nul, sl + kSlotW + i * 1024, 16, xv_off[i], s * 64, 0);
    }
    if (!PT) {
      const int kb = lkb < nblk - 1 ? lkb : nblk - 1;
      MTQ_DMA(live ? ars : nul, sl + kSlotW + XL::bytes, 4, av_off, kb * 4, 0);
      lrem += U;  // spb is a multiple of U (host-checked): one block per batch
      if (lrem >= spb) {
        lrem -= spb;
        ++lkb;
      }
    }
  };

  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t cur = 0;
  bool have = false;
  auto compute = [&](int b, int slot) {
    const uint32_t sb = lds_base + (uint32_t)(slot * SLOT);
    u32x4 wf[U], xf[U];
    float am;
    // the whole slot in one statement (reads + their lgkmcnt): hipcc never sees an LDS read it
    // could order behind the DMAs in flight
    asm volatile(
        "ds_read_b128 %0, %9\n\tds_read_b128 %1, %10\n\tds_read_b128 %2, %11\n\tds_read_b128 %3, %12\n\t"
        "ds_read_b128 %4, %13\n\tds_read_b128 %5, %14\n\tds_read_b128 %6, %15\n\tds_read_b128 %7, %16\n\t"
        "ds_read_b32 %8, %17\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(wf[0]), "=&v"(wf[1]), "=&v"(wf[2]), "=&v"(wf[3]), "=&v"(xf[0]), "=&v"(xf[1]), "=&v"(xf[2]),
          "=&v"(xf[3]), "=&v"(am)
        : "v"(sb + wr_off[0]), "v"(sb + wr_off[1]), "v"(sb + wr_off[2]), "v"(sb + wr_off[3]),
          "v"(sb + xr_off[0]), "v"(sb + xr_off[1]), "v"(sb + xr_off[2]), "v"(sb + xr_off[3]),
          "v"(sb + (PT ? 0u : ar_off))
        : "memory");
    if (!PT && (!have || __float_as_uint(am) != cur)) {  // per lane: a new block of its row
      cur = __float_as_uint(am);
      have = true;
      qp.make(am, p);
    }
    const int s = s0 + b * U;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u >= s1) break;  // wave-uniform
      u32x4 bq;
      bq.x = qp.template pair<T>(wf[u].x);
      bq.y = qp.template pair<T>(wf[u].y);
      bq.z = qp.template pair<T>(wf[u].z);
      bq.w = qp.template pair<T>(wf[u].w);
      acc = Mfma<T>::mma(as_v8<T>(xf[u]), as_v8<T>(bq), acc);
    }
  };

#pragma unroll
  for (int b = 0; b < R - 1; ++b) issue(b, b);
  int slot = 0, ahead = R - 1;  // slot of batch b, slot of batch b + R - 1
  for (int b = 0; b < nb; ++b) {
    issue(b + R - 1, ahead);
    __builtin_amdgcn_sched_barrier(0);
    wait_vmcnt<(R - 1) * GROUP>();
    __builtin_amdgcn_sched_barrier(0);
    compute(b, slot);
    __builtin_amdgcn_sched_barrier(0);
    slot = slot + 1 == R ? 0 : slot + 1;
    ahead = ahead + 1 == R ? 0 : ahead + 1;
  }
  // D layout of mfma_f32_16x16x32: col = lane & 15 (n), row = 4 (lane >> 4) + i (m)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = qd * 4 + i;
    if (m >= M) break;
    if (S == 1) {
      float v = acc[i];
      if (bias) v += Elem<T>::ld(bias[n0 + r]);
      y[(int64_t)m * N + n0 + r] = Elem<T>::st(v);
    } else {
      part[((int64_t)chunk * M + m) * N + n0 + r] = acc[i];
    }
  }
}

template <typename T, int KIND, bool PT, int XM>
__global__ __launch_bounds__(kStreamWaves * 64) void qlinear_dma_kernel(
    const T *__restrict__ x, const T *__restrict__ w, T *__restrict__ y, const T *__restrict__ bias,
    float *__restrict__ part, int M, int N, int K, int tiles, int S, int kcs, QlParams p) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * kStreamWaves) + wave;
  if (unit >= tiles * S) return;  // wave-uniform; the kernel has no barrier
  qlinear_dma_unit<T, KIND, PT, XM>(x, w, y, bias, part, M, N, K, tiles, S, kcs, p, unit, wave);
}

// Several linears of the same input length M and depth K in one launch (the q/k/v projections of
// a decode step: 8 MB k/v weight streams alone cannot fill the chip or amortise a launch).  The
// units of linear i are [uend[i-1], uend[i]); every linear splits K the same way (S, kcs).
constexpr int kMaxGroup = 4;
struct QlGroupArgs {
  const void *x[kMaxGroup], *w[kMaxGroup], *bias[kMaxGroup];
  void *y[kMaxGroup];
  float *part[kMaxGroup];
  int N[kMaxGroup], uend[kMaxGroup];
  QlParams p[kMaxGroup];
  int n, M, K, S, kcs;
};

template <typename T, int KIND, bool PT, int XM>
__global__ __launch_bounds__(kStreamWaves * 64) void qlinear_dma_group_kernel(QlGroupArgs g) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int unit = __builtin_amdgcn_readfirstlane(blockIdx.x * kStreamWaves) + wave;
  if (unit >= g.uend[g.n - 1]) return;  // wave-uniform
  int i = 0, base = 0;
#pragma unroll
  for (int j = 0; j < kMaxGroup - 1; ++j)
    if (j < g.n - 1 && unit >= g.uend[j]) {
      i = j + 1;
      base = g.uend[j];
    }
  const int N = g.N[i];
  qlinear_dma_unit<T, KIND, PT, XM>(reinterpret_cast<const T *>(g.x[i]), reinterpret_cast<const T *>(g.w[i]),
                                    reinterpret_cast<T *>(g.y[i]), reinterpret_cast<const T *>(g.bias[i]),
                                    g.part[i], g.M, N, g.K, N / 16, g.S, g.kcs, g.p[i], unit - base, wave);
}

// y[m, n] = sum over chunks in order of part[c, m, n] (+ bias[n]), one rounding
template <typename T>
__global__ __launch_bounds__(256) void qlinear_splitk_finish(const float *__restrict__ part,
                                                             const T *__restrict__ bias,
                                                             T *__restrict__ y, int MN, int N, int S) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= MN) return;
  // chunk order kept; the loads of four chunks are issued before their adds
  float v = 0.f;
  int c = 0;
  for (; c + 4 <= S; c += 4) {
    const float p0 = part[(int64_t)c * MN + i], p1 = part[(int64_t)(c + 1) * MN + i];
    const float p2 = part[(int64_t)(c + 2) * MN + i], p3 = part[(int64_t)(c + 3) * MN + i];
    v += p0;
    v += p1;
    v += p2;
    v += p3;
  }
  for (; c < S; ++c) v += part[(int64_t)c * MN + i];
  if (bias) v += Elem<T>::ld(bias[i % N]);
  y[i] = Elem<T>::st(v);
}

struct QlFinishGroupArgs {
  const float *part[kMaxGroup];
  const void *bias[kMaxGroup];
  void *y[kMaxGroup];
  int N[kMaxGroup], mnend[kMaxGroup];
  int n, M, S;
};
// the split-K finish of every linear of a group in one launch (same fixed chunk order)
template <typename T>
__global__ __launch_bounds__(256) void qlinear_splitk_finish_group(QlFinishGroupArgs a) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= a.mnend[a.n - 1]) return;
  int k = 0, base = 0;
#pragma unroll
  for (int j = 0; j < kMaxGroup - 1; ++j)
    if (j < a.n - 1 && t >= a.mnend[j]) {
      k = j + 1;
      base = a.mnend[j];
    }
  const int i = t - base, MN = a.M * a.N[k];
  const float *part = a.part[k];
  float v = 0.f;
  for (int c = 0; c < a.S; ++c) v += part[(int64_t)c * MN + i];
  const T *bias = reinterpret_cast<const T *>(a.bias[k]);
  if (bias) v += Elem<T>::ld(bias[i % a.N[k]]);
  reinterpret_cast<T *>(a.y[k])[i] = Elem<T>::st(v);
}

// ---- workgroup-per-tile kernel (blocks not aligned to the stream kernel's batches) ----------
template <typename T, int KIND, int MT, int kQlWaves, int kQlU>
__global__ __launch_bounds__(kQlWaves * 64) void qlinear_wg_kernel(
    const T *__restrict__ x, const T *__restrict__ w, const T *__restrict__ bias,
    T *__restrict__ y, int64_t M, int64_t N, int64_t K, QlParams p) {
  using V = Vec<T>;
  __shared__ float red[kQlWaves * MT * 16 * 17];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, qd = lane >> 4;
  const int64_t n0 = (int64_t)blockIdx.x * 16;
  const int64_t nsteps = K / 32;
  const int64_t per = (nsteps + kQlWaves - 1) / kQlWaves;
  const int64_t s0 = (int64_t)wv * per;
  int64_t s1 = s0 + per;
  s1 = s1 < nsteps ? s1 : nsteps;

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the amax index of a W element is row_blk + s / spb (blocks tile whole K steps, so every
  // lane of a step shares the K block and s / spb is wave-uniform)
  const int64_t spb = p.amax_numel == 1 ? nsteps : p.block / 32;  // K steps per amax block
  const int64_t row_blk = p.amax_numel == 1 ? 0 : (n0 + r) * (K / p.block);
  const T *wp = w + (n0 + r) * K + qd * 8 + s0 * 32;
  const bool xrow = r < M;
  const T *xp = x + (xrow ? r : 0) * K + qd * 8 + s0 * 32;
  int64_t cur = -1;
  QParam<KIND> qp;
  for (int64_t s = s0; s < s1; s += kQlU) {
    V wvec[kQlU], xvec[kQlU];
#pragma unroll
    for (int u = 0; u < kQlU; ++u) {
      if (s + u < s1) {
        wvec[u] = ldg_vec_nt(wp + u * 32);
        if (xrow)
          xvec[u] = ldg_vec(xp + u * 32);
        else
          xvec[u].raw = make_uint4(0, 0, 0, 0);
      }
    }
    wp += kQlU * 32;
    xp += kQlU * 32;
#pragma unroll
    for (int u = 0; u < kQlU; ++u) {
      if (s + u >= s1) break;
      const int64_t kb = (s + u) / spb;  // wave-uniform
      if (kb != cur) {
        qp.make(load_as_float(p.amax, p.amax_dtype, row_blk + kb), p);
        cur = kb;
      }
      qp.template apply<T>(wvec[u]);
      acc[0] = Mfma<T>::mma(as_v8<T>(xvec[u]), as_v8<T>(wvec[u]), acc[0]);
    }
  }
  // D layout of mfma_f32_16x16x32: col = lane & 15 (n), row = (lane >> 4) * 4 + i (m)
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      red[((wv * MT + t) * 16 + qd * 4 + i) * 17 + r] = acc[t][i];
  __syncthreads();
  for (int o = threadIdx.x; o < MT * 256; o += kQlWaves * 64) {
    const int t = o >> 8, row = (o >> 4) & 15, col = o & 15;
    const int64_t m = (int64_t)t * 16 + row;
    if (m >= M) continue;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < kQlWaves; ++k) sum += red[((k * MT + t) * 16 + row) * 17 + col];
    if (bias) sum += Elem<T>::ld(bias[n0 + col]);
    y[m * N + n0 + col] = Elem<T>::st(sum);
  }
}

// ---- host ----------------------------------------------------------------------------------
constexpr int kU = 4;  // K steps per batch (4 x 16 B of W per lane in flight, double-buffered)

// waves a launch aims for: split K until tiles x S reaches it (8 per CU, two per SIMD)
int64_t target_waves() { return 8 * (int64_t)mtq::host_num_cus(); }

struct Split {
  int S, kcs;
};
Split choose_split(int64_t N, int64_t K, bool allow_split) {
  const int64_t tiles = N / 16, nsteps = K / 32;
  int64_t S = 1;
  if (allow_split) {
    S = (target_waves() + tiles - 1) / tiles;
    const int64_t max_s = nsteps / (2 * kU);  // at least two batches per chunk
    S = S < max_s ? S : max_s;
    S = S < 1 ? 1 : S;
  }
  int64_t kcs = (nsteps + S - 1) / S;
  kcs = (kcs + kU - 1) / kU * kU;
  S = (nsteps + kcs - 1) / kcs;
  return {(int)S, (int)kcs};
}

// (the stream kernel reads fp32 amax: a dtype switch next to its loads would drain them)
// -1: the stream kernel cannot take this amax layout; else 0 (per-tensor / batch-aligned) or the
// steps per block (dividing kU)
int stream_spb(int64_t amax_numel, int64_t block, int64_t K) {
  if (amax_numel == 1) return 0;
  const int64_t spb = block / 32, nsteps = K / 32;
  if (spb == nsteps || spb % kU == 0) return 0;
  if (kU % spb == 0) return (int)spb;
  return -1;
}

template <typename T, int KIND, int XM>
void launch_dma(unsigned g, bool pt, hipStream_t stream, const T *x, const T *w, T *y, const T *bias,
                float *part, int M, int N, int K, int tiles, int S, int kcs, const QlParams &p) {
  if (pt)
    qlinear_dma_kernel<T, KIND, true, XM><<<g, kStreamWaves * 64, 0, stream>>>(x, w, y, bias, part, M, N, K,
                                                                              tiles, S, kcs, p);
  else
    qlinear_dma_kernel<T, KIND, false, XM><<<g, kStreamWaves * 64, 0, stream>>>(x, w, y, bias, part, M, N, K,
                                                                               tiles, S, kcs, p);
}

template <typename T, int KIND>
int launch_stream(const void *x, const void *w, const void *bias, void *y, float *part, int64_t M,
                  int64_t N, int64_t K, const QlParams &p, int spb, Split sp, hipStream_t stream) {
  const int tiles = (int)(N / 16);
  const unsigned g = (unsigned)(((int64_t)tiles * sp.S + kStreamWaves - 1) / kStreamWaves);
  const T *xt = reinterpret_cast<const T *>(x);
  const T *wt = reinterpret_cast<const T *>(w);
  const T *bt = reinterpret_cast<const T *>(bias);
  T *yt = reinterpret_cast<T *>(y);
  const bool pt = p.amax_numel == 1;
#define QL_ARGS xt, wt, yt, bt, part, (int)M, (int)N, (int)K, tiles, sp.S, sp.kcs, p
  if (pt || spb == 0) {
    if (M == 1)
      launch_dma<T, KIND, 1>(g, pt, stream, QL_ARGS);
    else if (M <= 4)
      launch_dma<T, KIND, 4>(g, pt, stream, QL_ARGS);
    else if (M <= 8)
      launch_dma<T, KIND, 8>(g, pt, stream, QL_ARGS);
    else
      launch_dma<T, KIND, 16>(g, pt, stream, QL_ARGS);
  } else if (spb == 1)
    qlinear_stream_kernel<T, KIND, kU, false, 1><<<g, kStreamWaves * 64, 0, stream>>>(QL_ARGS);
  else
    qlinear_stream_kernel<T, KIND, kU, false, 2><<<g, kStreamWaves * 64, 0, stream>>>(QL_ARGS);
#undef QL_ARGS
  int st = host_check_launch();
  if (st != MTQ_OK || sp.S == 1) return st;
  const int MN = (int)(M * N);
  qlinear_splitk_finish<T><<<(MN + 255) / 256, 256, 0, stream>>>(part, bt, yt, MN, (int)N, sp.S);
  return host_check_launch();
}

template <typename T, int KIND>
int launch_wg(const void *x, const void *w, const void *bias, void *y, int64_t M, int64_t N,
              int64_t K, const QlParams &p, hipStream_t stream) {
  const unsigned g = (unsigned)(N / 16);
  const T *xt = reinterpret_cast<const T *>(x);
  const T *wt = reinterpret_cast<const T *>(w);
  const T *bt = reinterpret_cast<const T *>(bias);
  T *yt = reinterpret_cast<T *>(y);
  // measured (r01 variant sweep): 16 waves when there are few 16-row tiles, 8 when many
  if ((int64_t)g >= 2 * (int64_t)mtq::host_num_cus())
    qlinear_wg_kernel<T, KIND, 1, 8, 4><<<g, 8 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p);
  else
    qlinear_wg_kernel<T, KIND, 1, 16, 4><<<g, 16 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p);
  return host_check_launch();
}

bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

int validate(const void *x, const void *w, const void *y, int64_t M, int64_t N, int64_t K, int dtype,
             const void *amax, int amax_dtype, int64_t amax_numel, int64_t block, int kind,
             int num_bits) {
  if (M < 1 || M > 16 || N < 16 || N % 16 != 0 || K < 32 || K % 32 != 0) return MTQ_ERR_INVALID_ARG;
  if (!x || !w || !y || !amax || amax_numel < 1) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (amax_dtype < 0 || amax_dtype > 3) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(w)) return MTQ_ERR_INVALID_ARG;
  // the stream kernel's 32-bit lane / step offsets within a 16-row tile (and int M, N, K)
  if (K >= (int64_t)1 << 26 || N >= (int64_t)1 << 30) return MTQ_ERR_INVALID_ARG;
  // per-tensor, or per-(row, block) with blocks that tile the 32-wide K steps
  if (amax_numel > 1 && (block < 32 || block % 32 != 0 || K % block != 0 || amax_numel * block != N * K))
    return MTQ_ERR_INVALID_ARG;
  if (kind != 0 && kind != 1) return MTQ_ERR_FORMAT;
  if (kind == 0 && (num_bits < 1 || num_bits > 31)) return MTQ_ERR_INVALID_ARG;
  return MTQ_OK;
}

}  // namespace

extern "C" size_t mtq_qlinear_small_m_workspace_bytes(int64_t M, int64_t N, int64_t K) {
  if (M < 1 || N < 16 || K < 32) return 0;
  const Split sp = choose_split(N, K, true);
  return sp.S > 1 ? (size_t)sp.S * (size_t)M * (size_t)N * sizeof(float) : 0;
}

extern "C" int mtq_qlinear_small_m_ws(const void *x, const void *w, const void *bias, void *y,
                                      int64_t M, int64_t N, int64_t K, int dtype, const void *amax,
                                      int amax_dtype, int64_t amax_numel, int64_t block, int kind,
                                      int num_bits, int is_unsigned, int narrow_range, void *ws,
                                      size_t ws_bytes, hipStream_t stream) {
  int st = validate(x, w, y, M, N, K, dtype, amax, amax_dtype, amax_numel, block, kind, num_bits);
  if (st != MTQ_OK) return st;
  QlParams p{amax, amax_dtype, amax_numel, block, 0.f, 0.f};
  if (kind == 0) {
    const float mb = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
    p.max_bound = mb;
    p.min_bound = is_unsigned ? 0.f : (narrow_range ? -mb : -mb - 1.f);
  }
  const int spb = stream_spb(amax_numel, block, K);
  const bool bf = dtype == MTQ_BF16;
  if (spb < 0 || amax_dtype != 0) {
    if (bf) return kind == 0 ? launch_wg<__bf16, 0>(x, w, bias, y, M, N, K, p, stream)
                             : launch_wg<__bf16, 1>(x, w, bias, y, M, N, K, p, stream);
    return kind == 0 ? launch_wg<_Float16, 0>(x, w, bias, y, M, N, K, p, stream)
                     : launch_wg<_Float16, 1>(x, w, bias, y, M, N, K, p, stream);
  }
  // split K only with a workspace big enough for the partial tiles
  Split sp = choose_split(N, K, ws != nullptr);
  if (sp.S > 1 && (!al16(ws) || ws_bytes < (size_t)sp.S * (size_t)M * (size_t)N * sizeof(float)))
    sp = choose_split(N, K, false);
  float *part = reinterpret_cast<float *>(ws);
  if (bf) return kind == 0 ? launch_stream<__bf16, 0>(x, w, bias, y, part, M, N, K, p, spb, sp, stream)
                           : launch_stream<__bf16, 1>(x, w, bias, y, part, M, N, K, p, spb, sp, stream);
  return kind == 0 ? launch_stream<_Float16, 0>(x, w, bias, y, part, M, N, K, p, spb, sp, stream)
                   : launch_stream<_Float16, 1>(x, w, bias, y, part, M, N, K, p, spb, sp, stream);
}

extern "C" int mtq_qlinear_small_m(const void *x, const void *w, const void *bias, void *y,
                                   int64_t M, int64_t N, int64_t K, int dtype, const void *amax,
                                   int amax_dtype, int64_t amax_numel, int64_t block, int kind,
                                   int num_bits, int is_unsigned, int narrow_range,
                                   hipStream_t stream) {
  return mtq_qlinear_small_m_ws(x, w, bias, y, M, N, K, dtype, amax, amax_dtype, amax_numel, block,
                                kind, num_bits, is_unsigned, narrow_range, nullptr, 0, stream);
}

namespace {

// the problems run as one grouped launch: same kind, fp32 amax of one class (per tensor, or
// per-row blocks aligned to the 128-column batches)
bool groupable(const mtq_qlinear_problem *pr, int n, int64_t K) {
  if (n < 1 || n > kMaxGroup) return false;
  const bool pt = pr[0].amax_numel == 1;
  for (int i = 0; i < n; ++i) {
    if (pr[i].kind != pr[0].kind || pr[i].amax_dtype != 0 || (pr[i].amax_numel == 1) != pt) return false;
    if (!pt && stream_spb(pr[i].amax_numel, pr[i].block, K) != 0) return false;
  }
  return true;
}

int64_t group_part_floats(const mtq_qlinear_problem *pr, int n, int64_t M, const Split &sp) {
  int64_t f = 0;
  for (int i = 0; i < n; ++i) f += sp.S > 1 ? (int64_t)sp.S * M * pr[i].N : 0;
  return f;
}

Split group_split(const int64_t *N, int n, int64_t K) {
  int64_t total = 0;
  for (int i = 0; i < n; ++i) total += N[i];
  return choose_split(total, K, true);
}

template <typename T, int KIND, bool PT, int XM>
void launch_group(const QlGroupArgs &g, unsigned grid, hipStream_t stream) {
  qlinear_dma_group_kernel<T, KIND, PT, XM><<<grid, kStreamWaves * 64, 0, stream>>>(g);
}

template <typename T, int KIND>
int run_group(const mtq_qlinear_problem *pr, int n, int64_t M, int64_t K, float *ws, Split sp,
              hipStream_t stream) {
  QlGroupArgs g{};
  g.n = n, g.M = (int)M, g.K = (int)K, g.S = sp.S, g.kcs = sp.kcs;
  QlFinishGroupArgs f{};
  f.n = n, f.M = (int)M, f.S = sp.S;
  int units = 0, mn = 0;
  int64_t off = 0;
  for (int i = 0; i < n; ++i) {
    g.x[i] = pr[i].x, g.w[i] = pr[i].w, g.bias[i] = pr[i].bias, g.y[i] = pr[i].y;
    g.N[i] = (int)pr[i].N;
    g.part[i] = sp.S > 1 ? ws + off : nullptr;
    off += sp.S > 1 ? (int64_t)sp.S * M * pr[i].N : 0;
    QlParams &p = g.p[i];
    p = QlParams{pr[i].amax, pr[i].amax_dtype, pr[i].amax_numel, pr[i].block, 0.f, 0.f};
    if (KIND == 0) {
      const float mb = (float)((1ll << (pr[i].num_bits - 1 + (pr[i].is_unsigned ? 1 : 0))) - 1);
      p.max_bound = mb;
      p.min_bound = pr[i].is_unsigned ? 0.f : (pr[i].narrow_range ? -mb : -mb - 1.f);
    }
    units += (int)(pr[i].N / 16) * sp.S;
    g.uend[i] = units;
    f.part[i] = g.part[i], f.bias[i] = pr[i].bias, f.y[i] = pr[i].y, f.N[i] = (int)pr[i].N;
    mn += (int)(M * pr[i].N);
    f.mnend[i] = mn;
  }
  const unsigned grid = (unsigned)((units + kStreamWaves - 1) / kStreamWaves);
  const bool pt = pr[0].amax_numel == 1;
#define QL_GROUP(XM)                                         \
  do {                                                       \
    if (pt)                                                  \
      launch_group<T, KIND, true, XM>(g, grid, stream);      \
    else                                                     \
      launch_group<T, KIND, false, XM>(g, grid, stream);     \
  } while (0)
  if (M == 1)
    QL_GROUP(1);
  else if (M <= 4)
    QL_GROUP(4);
  else if (M <= 8)
    QL_GROUP(8);
  else
    QL_GROUP(16);
#undef QL_GROUP
  int st = host_check_launch();
  if (st != MTQ_OK || sp.S == 1) return st;
  qlinear_splitk_finish_group<T><<<(unsigned)((mn + 255) / 256), 256, 0, stream>>>(f);
  return host_check_launch();
}

}  // namespace

extern "C" size_t mtq_qlinear_small_m_group_workspace_bytes(int64_t M, const int64_t *N, int n, int64_t K) {
  if (M < 1 || K < 32 || !N || n < 1 || n > kMaxGroup) return 0;
  int64_t Ns[kMaxGroup];
  size_t single = 0;
  for (int i = 0; i < n; ++i) {
    if (N[i] < 16) return 0;
    Ns[i] = N[i];
    const size_t b = mtq_qlinear_small_m_workspace_bytes(M, N[i], K);
    single = b > single ? b : single;  // the fallback runs the linears one after another
  }
  const Split sp = group_split(Ns, n, K);
  int64_t f = 0;
  for (int i = 0; i < n; ++i) f += sp.S > 1 ? (int64_t)sp.S * M * Ns[i] : 0;
  const size_t grouped = (size_t)f * sizeof(float);
  return grouped > single ? grouped : single;
}

extern "C" int mtq_qlinear_small_m_group(const mtq_qlinear_problem *pr, int n, int64_t M, int64_t K,
                                         int dtype, void *ws, size_t ws_bytes, hipStream_t stream) {
  if (!pr || n < 1 || n > kMaxGroup) return MTQ_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i) {
    const int st = validate(pr[i].x, pr[i].w, pr[i].y, M, pr[i].N, K, dtype, pr[i].amax, pr[i].amax_dtype,
                            pr[i].amax_numel, pr[i].block, pr[i].kind, pr[i].num_bits);
    if (st != MTQ_OK) return st;
  }
  int64_t Ns[kMaxGroup];
  for (int i = 0; i < n; ++i) Ns[i] = pr[i].N;
  Split sp = group_split(Ns, n, K);
  if (groupable(pr, n, K) && (sp.S == 1 || (ws && al16(ws) && ws_bytes >= (size_t)group_part_floats(pr, n, M, sp) * sizeof(float)))) {
    float *part = reinterpret_cast<float *>(ws);
    const bool bf = dtype == MTQ_BF16, k0 = pr[0].kind == 0;
    if (bf) return k0 ? run_group<__bf16, 0>(pr, n, M, K, part, sp, stream) : run_group<__bf16, 1>(pr, n, M, K, part, sp, stream);
    return k0 ? run_group<_Float16, 0>(pr, n, M, K, part, sp, stream) : run_group<_Float16, 1>(pr, n, M, K, part, sp, stream);
  }
  // not groupable: one launch per linear, in order (same results as separate calls)
  for (int i = 0; i < n; ++i) {
    const int st = mtq_qlinear_small_m_ws(pr[i].x, pr[i].w, pr[i].bias, pr[i].y, M, pr[i].N, K, dtype, pr[i].amax,
                                          pr[i].amax_dtype, pr[i].amax_numel, pr[i].block, pr[i].kind,
                                          pr[i].num_bits, pr[i].is_unsigned, pr[i].narrow_range, ws, ws_bytes,
                                          stream);
    if (st != MTQ_OK) return st;
  }
  return MTQ_OK;
}
