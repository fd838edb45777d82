// mtq_kernels.hip — MI355X (gfx950, CDNA4) fake-quantization and calibration kernels and the
// C ABI declared in include/mtq_amd.h.
//
// Design: every kernel here is HBM-bound (<= ~10 VALU ops per byte), so the
// kernels are built around 16-byte-per-lane coalesced loads/stores, a grid of
// min(work, 8 blocks x CUs) 256-thread blocks with a grid-stride loop and 4 vectors in flight
// per lane, per-tensor/per-channel constants computed on the device (no host ATen scale ops,
// unlike tensor_quant_gpu_fp8.cu:97-100), and wave64 shuffle reductions.  Reference citations
// are relative to the reference repository root.
#include <hip/hip_runtime.h>
#include <atomic>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
#include <type_traits>

#include "mtq_amd.h"
#include "mtq_device.hpp"

using namespace mtq;

namespace {

constexpr int kThreads = 256;

thread_local int g_last_hip_error = 0;

int num_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cu <= 0)
      cu = 256;
    cached[dev] = cu;
  }
  return cached[dev];
}


unsigned grid_for(int64_t work_items, int per_block) {
  int64_t blocks = (work_items + per_block - 1) / per_block;
  int64_t cap = (int64_t)num_cus() * 8;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  return (unsigned)blocks;
}

int check_launch() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_hip_error = (int)e;
    return MTQ_ERR_LAUNCH;
  }
  return MTQ_OK;
}

FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) l++;
  f.s = l;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  return f;
}

bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// ============================================================================================
// Element-wise driver: vectorised main body + scalar tail.  `Op` provides
//   init()                       per-thread constants (per-tensor scale etc.)
//   vec(Vec<T>&, int64_t vi)     quantise one 16-byte vector (vector index vi)
//   one(float x, int64_t i)      quantise one element (element index i)
// ============================================================================================
// Launch structure (measured with scripts/bw_probe.hip on MI355X, bf16 256 MiB in + out):
// one 16-byte vector per lane, each block a contiguous chunk of 256*U vectors, one chunk per
// block (no grid-stride loop), reaches 6.1 TB/s; a grid-stride loop with 4 vectors in flight per
// lane over 2048 blocks only 4.3-4.6 TB/s.  U = 1 with non-temporal loads / stores is the one
// shipped: best of the r01 sweep (scripts/sweep_ew.py: fp8 per-tensor 6.28 TB/s, fp8 block-128
// 6.0 TB/s vs 5.9 / 5.87 with temporal accesses; U = 2 / 4 no faster).
template <typename T, class Op, int U, bool NT>
__global__ __launch_bounds__(kThreads) void ew_vec_kernel(const T *__restrict__ x,
                                                           T *__restrict__ y, int64_t nvec,
                                                           Op op) {
  using V = Vec<T>;
  op.init();
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (i < nvec) v[u] = NT ? ldg_vec_nt(x + i * V::N) : ldg_vec(x + i * V::N);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (i < nvec) {
      op.vec(v[u], i);
      if (NT)
        stg_vec_nt(y + i * V::N, v[u]);
      else
        stg_vec(y + i * V::N, v[u]);
    }
  }
}

template <typename T, class Op>
__global__ __launch_bounds__(kThreads) void ew_scalar_kernel(const T *__restrict__ x,
                                                              T *__restrict__ y, int64_t begin,
                                                              int64_t n, Op op) {
  op.init();
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = begin + (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride)
    y[i] = Elem<T>::st(op.one(Elem<T>::ld(x[i]), i));
}

template <typename T, class Op>
int launch_ew(const void *xv, void *yv, int64_t n, Op op, hipStream_t stream) {
  const T *x = reinterpret_cast<const T *>(xv);
  T *y = reinterpret_cast<T *>(yv);
  if (n <= 0) return MTQ_OK;
  constexpr int N = Vec<T>::N;
  int64_t nvec = (aligned16(x) && aligned16(y)) ? n / N : 0;
  if (nvec > 0) {
    const unsigned blocks = (unsigned)((nvec + kThreads - 1) / kThreads);
    count_dispatch(kDispEwVec);
    ew_vec_kernel<T, Op, 1, true><<<blocks, kThreads, 0, stream>>>(x, y, nvec, op);
  }
  int64_t done = nvec * N;
  if (done < n) {
    unsigned g = grid_for(n - done, kThreads);
    ew_scalar_kernel<T, Op><<<g, kThreads, 0, stream>>>(x, y, done, n, op);
  }
  return check_launch();
}

// --------------------------------------------------------------------------------------------
// INT-n ops
// --------------------------------------------------------------------------------------------
struct IntBounds {
  float max_bound, min_bound;
};
IntBounds int_bounds(int num_bits, int is_unsigned, int narrow_range) {
  // tensor_quant.py:624-632 / tensor_quant_gpu.cu:38-41,67-69
  float mb = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
  float lo = is_unsigned ? 0.f : (narrow_range ? -mb : -mb - 1.f);
  return {mb, lo};
}

template <typename T> struct IntTensorOp {
  const void *amax;
  int amax_dtype;
  float max_bound, min_bound;
  IntQ q;
  __device__ __forceinline__ void init() {
    q = make_intq(load_as_float(amax, amax_dtype, 0), max_bound, min_bound);
  }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t) {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; ++j) v.e[j] = Elem<T>::st(int_qdq(Elem<T>::ld(v.e[j]), q));
  }
  __device__ __forceinline__ float one(float x, int64_t) { return int_qdq(x, q); }
};

// Channel of vector vi when `inner` is a multiple of the vector width: all elements of the
// vector share (vi / inner_vec) % axis_size.  Indices < 2^31 use the fast divider.
template <typename T> struct IntAxisVecOp {
  const void *amax;
  int amax_dtype;
  float max_bound, min_bound;
  FastDiv inner_vec, axis;
  bool small;
  int64_t inner_vec64, axis64;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ int64_t chan(int64_t vi) const {
    if (small) {
      uint32_t r = fdiv((uint32_t)vi, inner_vec);
      uint32_t q = fdiv(r, axis);
      return r - q * axis.d;
    }
    return (vi / inner_vec64) % axis64;
  }
  __device__ __forceinline__ IntQ qparam(int64_t vi) const {
    return make_intq(load_as_float(amax, amax_dtype, chan(vi)), max_bound, min_bound);
  }
  __device__ __forceinline__ IntQ qparam_from(float a) const { return make_intq(a, max_bound, min_bound); }
  __device__ __forceinline__ static void apply(Vec<T> &v, const IntQ &q) {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; ++j) v.e[j] = Elem<T>::st(int_qdq(Elem<T>::ld(v.e[j]), q));
  }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t vi) { apply(v, qparam(vi)); }
  __device__ __forceinline__ float one(float x, int64_t i) {
    int64_t c = (i / (inner_vec64 * Vec<T>::N)) % axis64;
    return int_qdq(x, make_intq(load_as_float(amax, amax_dtype, c), max_bound, min_bound));
  }
};

// Generic channel mapping (inner not a multiple of the vector width, e.g. axis = -1).
template <typename T> struct IntAxisElemOp {
  const void *amax;
  int amax_dtype;
  float max_bound, min_bound;
  int64_t inner, axis;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ float one(float x, int64_t i) {
    int64_t c = (i / inner) % axis;
    return int_qdq(x, make_intq(load_as_float(amax, amax_dtype, c), max_bound, min_bound));
  }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t vi) {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; ++j)
      v.e[j] = Elem<T>::st(one(Elem<T>::ld(v.e[j]), vi * Vec<T>::N + j));
  }
};

// --------------------------------------------------------------------------------------------
// FP8 ops
// --------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void fp8_vec(Vec<T> &v, const Fp8Q &q) {
#pragma unroll
  for (int j = 0; j < Vec<T>::N; j += 2) {
    float a = Elem<T>::ld(v.e[j]);
    float b = (j + 1 < Vec<T>::N) ? Elem<T>::ld(v.e[j + 1]) : 0.f;
    fp8_qdq2(a, b, q);
    v.e[j] = Elem<T>::st(a);
    if (j + 1 < Vec<T>::N) v.e[j + 1] = Elem<T>::st(b);
  }
}
__device__ __forceinline__ float fp8_one(float x, const Fp8Q &q) {
  float b = 0.f;
  fp8_qdq2(x, b, q);
  return x;
}

template <typename T> struct Fp8TensorOp {
  const void *amax;
  int amax_dtype;
  Fp8Q q;
  __device__ __forceinline__ void init() { q = make_fp8q(load_as_float(amax, amax_dtype, 0)); }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t) { fp8_vec(v, q); }
  __device__ __forceinline__ float one(float x, int64_t) { return fp8_one(x, q); }
};

template <typename T> struct Fp8AxisVecOp {
  const void *amax;
  int amax_dtype;
  FastDiv inner_vec, axis;
  bool small;
  int64_t inner_vec64, axis64;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ int64_t chan(int64_t vi) const {
    if (small) {
      uint32_t r = fdiv((uint32_t)vi, inner_vec);
      uint32_t q = fdiv(r, axis);
      return r - q * axis.d;
    }
    return (vi / inner_vec64) % axis64;
  }
  __device__ __forceinline__ Fp8Q qparam(int64_t vi) const {
    return make_fp8q(load_as_float(amax, amax_dtype, chan(vi)));
  }
  __device__ __forceinline__ Fp8Q qparam_from(float a) const { return make_fp8q(a); }
  __device__ __forceinline__ static void apply(Vec<T> &v, const Fp8Q &q) { fp8_vec(v, q); }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t vi) { fp8_vec(v, qparam(vi)); }
  __device__ __forceinline__ float one(float x, int64_t i) {
    int64_t c = (i / (inner_vec64 * Vec<T>::N)) % axis64;
    return fp8_one(x, make_fp8q(load_as_float(amax, amax_dtype, c)));
  }
};

template <typename T> struct Fp8AxisElemOp {
  const void *amax;
  int amax_dtype;
  int64_t inner, axis;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ float one(float x, int64_t i) {
    int64_t c = (i / inner) % axis;
    return fp8_one(x, make_fp8q(load_as_float(amax, amax_dtype, c)));
  }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t vi) {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; ++j)
      v.e[j] = Elem<T>::st(one(Elem<T>::ld(v.e[j]), vi * Vec<T>::N + j));
  }
};

// torch float8_e4m3fn cast (no clamp): |x| > 464 (the 448/480 midpoint) overflows to NaN.
template <typename T> struct Fp8CastOp {
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ static float ovf(float v) {
    return fabsf(v) > 464.0f ? __builtin_nanf("") : v;
  }
  __device__ __forceinline__ void vec(Vec<T> &v, int64_t) {
#pragma unroll
    for (int j = 0; j < Vec<T>::N; j += 2) {
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(ovf(Elem<T>::ld(v.e[j])),
                                              ovf(Elem<T>::ld(v.e[j + 1])), 0, false);
      v.e[j] = Elem<T>::st(__builtin_amdgcn_cvt_f32_fp8(p, 0));
      v.e[j + 1] = Elem<T>::st(__builtin_amdgcn_cvt_f32_fp8(p, 1));
    }
  }
  __device__ __forceinline__ float one(float x, int64_t) {
    int p = __builtin_amdgcn_cvt_pk_fp8_f32(ovf(x), 0.f, 0, false);
    return __builtin_amdgcn_cvt_f32_fp8(p, 0);
  }
};

// --------------------------------------------------------------------------------------------
// Block-grouped form of the axis ops for short channels (the static block view: one amax per
// `inner` = VB vectors, e.g. 16 bf16 vectors for block 128).  A lane takes U vectors of the SAME
// channel, so the per-channel parameters -- an amax load and two correctly rounded divisions for
// FP8 (make_fp8q), one for INT -- are paid once per U vectors instead of per vector.  The LPB =
// VB / U lanes of a channel read consecutive 16-byte vectors, so each load instruction still
// covers whole aligned 128-byte lines (LPB >= 8).  Each wave covers 64 * U vectors = 64 / LPB
// channels; one contiguous chunk of 256 * U vectors per block, non-temporal, as ew_vec_kernel.
// --------------------------------------------------------------------------------------------
template <typename T, class Op, int U>
__global__ __launch_bounds__(kThreads) void ew_group_kernel(const T *__restrict__ x,
                                                             T *__restrict__ y, int64_t nvec,
                                                             int lpb, Op op) {
  using V = Vec<T>;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t wb = ((int64_t)blockIdx.x * kThreads + (int64_t)w * 64) * U;
  const int k = lane / lpb, pos = lane - k * lpb;
  const int64_t v0 = wb + (int64_t)k * lpb * U + pos;  // first vector of this lane
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * lpb;
    if (i < nvec) v[u] = ldg_vec_nt(x + i * V::N);
  }
  if (v0 >= nvec) return;
  const auto q = op.qparam(v0);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * lpb;
    if (i < nvec) {
      Op::apply(v[u], q);
      stg_vec_nt(y + i * V::N, v[u]);
    }
  }
}

// Default for fp32 amax with channel = vector / VB (no wrap; the per-lane-load kernel above
// otherwise): the wave's 64 / LPB channel amax values arrive through
// scalar loads from one wave-uniform address (scalar cache, no vector-memory instruction, no
// per-lane address) and each lane selects its own.  FP8 block-128 bf16 [32768, 4096]: 88.3 ->
// 83.4-84.9 us (76.6 -> 79.7-81.1 % of HBM peak, profiles/r02/export/).
// TPB = 512 threads per workgroup: 0.5-0.8 % faster than 256 on the bench primary in interleaved
// A/Bs (83.1 vs 83.6 us; 1024: 86.2 us; scripts/exp/group_exp.hip, profiles/r05/group_tpb_ab_r05gx3.log)
constexpr int kGroupSkThreads = 512;
template <typename T, class Op, int U, int LPB>
__global__ __launch_bounds__(kGroupSkThreads) void ew_group_sk_kernel(const T *__restrict__ x,
                                                                       T *__restrict__ y, int64_t nvec,
                                                                       const float *__restrict__ amax,
                                                                       int64_t nchan, Op op) {
  using V = Vec<T>;
  constexpr int CPW = 64 / LPB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wb = ((int64_t)blockIdx.x * kGroupSkThreads + (int64_t)w * 64) * U;
  const int k = lane / LPB, pos = lane - k * LPB;
  const int64_t v0 = wb + (int64_t)k * LPB * U + pos;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    if (i < nvec) v[u] = ldg_vec_nt(x + i * V::N);
  }
  const int64_t c0 = wb / (LPB * U);
  float am = amax[c0 < nchan ? c0 : nchan - 1];
#pragma unroll
  for (int j = 1; j < CPW; ++j) {
    const float a = amax[c0 + j < nchan ? c0 + j : nchan - 1];
    am = k == j ? a : am;
  }
  // (r05: clamped unconditional loads with an unguarded whole-wave path put both loads and the
  // amax scalar loads ahead of every wait in the ISA, and measured 0.3 % slower than this form in
  // an interleaved A/B, scripts/exp/group_exp.hip)
  if (v0 >= nvec) return;
  const auto q = op.qparam_from(am);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    if (i < nvec) {
      Op::apply(v[u], q);
      stg_vec_nt(y + i * V::N, v[u]);
    }
  }
}

// Long channels of whole vectors (per-row weights: one amax per row of >= 128 vectors): a wave's
// 64 * U consecutive vectors lie in ONE channel when the channel length is a multiple of 64 * U,
// so the channel, its amax (one scalar load) and the qdq parameters are wave-uniform -- the
// per-vector channel division, per-lane amax load and per-vector scale computation of the
// element-wise kernel disappear.  Lane l of the wave takes vectors wb + l + 64 u (each load
// instruction covers 1 KiB contiguous).  Requires axis_size * vb == nvec (no outer wrap).
// A: the amax storage type -- fp32, or the input's own 16-bit type (a bf16 model's per-channel
// weight amax is bf16, reference tensor_quantizer.py `_get_amax` keeps the input dtype).
template <typename T, typename A, class Op, int U>
__global__ __launch_bounds__(kThreads) void ew_rowwave_kernel(const T *__restrict__ x,
                                                               T *__restrict__ y, int64_t nvec,
                                                               const A *__restrict__ amax,
                                                               int64_t vb, Op op) {
  using V = Vec<T>;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wb = ((int64_t)blockIdx.x * kThreads + (int64_t)w * 64) * U;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = wb + u * 64 + lane;
    if (i < nvec) v[u] = ldg_vec_nt(x + i * V::N);
  }
  if (wb >= nvec) return;
  const int64_t c = wb / vb;  // wave-uniform (scalar)
  float am;
  if constexpr (sizeof(A) == 2) {
    // a 16-bit amax through the scalar cache: the dword holding it (s_load_dword; gfx950 has no
    // 16-bit scalar load, and the vector load the compiler emits otherwise put a VMEM round trip
    // in front of every wave's first store: 0.746 vs 0.777 with an fp32 amax, r05n).  amax is
    // 4-byte aligned (the launcher checks), so the dword of an even-count tensor's last element
    // is inside it (the launcher takes this path for an even channel count only, so no dword
    // reaches past the tensor).
    const uint32_t wv = reinterpret_cast<const uint32_t *>(amax)[c >> 1];
    const uint16_t h = (uint16_t)((c & 1) ? (wv >> 16) : (wv & 0xFFFFu));
    am = Elem<A>::ld(__builtin_bit_cast(A, h));
  } else {
    am = (float)amax[c];
  }
  const auto q = op.qparam_from(am);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = wb + u * 64 + lane;
    if (i < nvec) {
      Op::apply(v[u], q);
      stg_vec_nt(y + i * V::N, v[u]);
    }
  }
}

// --------------------------------------------------------------------------------------------
// Axis dispatch shared by INT and FP8
// --------------------------------------------------------------------------------------------
template <typename T, template <typename> class VecOp, template <typename> class ElemOp,
          class Fill>
int launch_axis(const void *x, void *y, int64_t n, int64_t axis_size, int64_t inner,
                Fill fill, hipStream_t stream) {
  constexpr int N = Vec<T>::N;
  if (inner % N == 0) {
    VecOp<T> op;
    fill(op);
    op.inner_vec64 = inner / N;
    op.axis64 = axis_size;
    op.small = (n / N) < (1ll << 31) && op.inner_vec64 < (1ll << 31) && axis_size < (1ll << 31);
    if (op.small) {
      op.inner_vec = make_fastdiv((uint32_t)op.inner_vec64);
      op.axis = make_fastdiv((uint32_t)axis_size);
    }
    // short channels of whole vectors (static block quant): the grouped kernel, U = 2, when a
    // channel spans 16..64 vectors (LPB = 8..32 lanes) and the buffers are 16-byte aligned;
    // the vector tail n % N goes through the scalar kernel as in launch_ew.
    const int64_t vb = op.inner_vec64;
    if (vb >= 16 && vb <= 64 && (vb & (vb - 1)) == 0 && aligned16(x) && aligned16(y)) {
      // U = 2 vectors per lane (LPB = VB / 2 lanes per channel); U = 1 / 4 measured slower
      // (74 / 56 % vs ~80 %, profiles/r02/round_c/group_u_ab.json)
      constexpr int U = 2;
      const int64_t nvec = n / N;
      const unsigned g = (unsigned)((nvec + (int64_t)kThreads * U - 1) / ((int64_t)kThreads * U));
      const bool sk = op.amax_dtype == MTQ_F32 && op.small && axis_size * vb == nvec;
      if (nvec > 0 && sk) {
        auto go = [&](auto lc) {
          constexpr int L = decltype(lc)::value;
          count_dispatch(kDispEwGroupSk);
          const unsigned gsk =
              (unsigned)((nvec + (int64_t)kGroupSkThreads * U - 1) / ((int64_t)kGroupSkThreads * U));
          ew_group_sk_kernel<T, VecOp<T>, U, L><<<gsk, kGroupSkThreads, 0, stream>>>(
              reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec,
              reinterpret_cast<const float *>(op.amax), axis_size, op);
        };
        if (vb == 16)
          go(std::integral_constant<int, 8>{});
        else if (vb == 32)
          go(std::integral_constant<int, 16>{});
        else
          go(std::integral_constant<int, 32>{});
      } else if (nvec > 0) {
        count_dispatch(kDispEwGroup);
        ew_group_kernel<T, VecOp<T>, U><<<g, kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, (int)(vb / U), op);
      }
      const int64_t done = nvec * N;
      if (done < n) {
        unsigned gs = grid_for(n - done, kThreads);
        ew_scalar_kernel<T, VecOp<T>><<<gs, kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), done, n, op);
      }
      return check_launch();
    }
    // long channels (per-row weights): channel length a multiple of 128 vectors, fp32 amax,
    // 16-byte aligned, no outer wrap -> wave-uniform channel.  A 16-bit amax is read as the
    // dword holding it, so that form needs a 4-byte-aligned amax and an even channel count (the
    // last dword then ends at the tensor's end); odd counts take the element-wise kernel
    const bool amax_own = ((op.amax_dtype == MTQ_BF16 && __is_same(T, __bf16)) ||
                           (op.amax_dtype == MTQ_F16 && __is_same(T, _Float16))) &&
                          reinterpret_cast<uintptr_t>(op.amax) % 4 == 0 && axis_size % 2 == 0;
    if (vb >= 128 && vb % 128 == 0 && aligned16(x) && aligned16(y) &&
        (op.amax_dtype == MTQ_F32 || amax_own) && axis_size * vb == n / N && n % N == 0) {
      constexpr int U = 2;
      const int64_t nvec = n / N;
      const unsigned g = (unsigned)((nvec + (int64_t)kThreads * U - 1) / ((int64_t)kThreads * U));
      if (nvec > 0) {
        count_dispatch(kDispEwRowwave);
        if (op.amax_dtype == MTQ_F32)
          ew_rowwave_kernel<T, float, VecOp<T>, U><<<g, kThreads, 0, stream>>>(
              reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec,
              reinterpret_cast<const float *>(op.amax), vb, op);
        else
          ew_rowwave_kernel<T, T, VecOp<T>, U><<<g, kThreads, 0, stream>>>(
              reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec,
              reinterpret_cast<const T *>(op.amax), vb, op);
      }
      return check_launch();
    }
    return launch_ew<T>(x, y, n, op, stream);
  }
  ElemOp<T> op;
  fill(op);
  op.inner = inner;
  op.axis = axis_size;
  return launch_ew<T>(x, y, n, op, stream);
}

template <class F> int dispatch_dtype(int dtype, F &&f) {
  switch (dtype) {
  case MTQ_F32: return f(float{});
  case MTQ_F16: return f(_Float16{});
  case MTQ_BF16: return f(__bf16{});
  case MTQ_F64: return f(double{});
  default: return MTQ_ERR_DTYPE;
  }
}

template <class F> int dispatch_dtype_nof64(int dtype, F &&f) {
  switch (dtype) {
  case MTQ_F32: return f(float{});
  case MTQ_F16: return f(_Float16{});
  case MTQ_BF16: return f(__bf16{});
  default: return MTQ_ERR_DTYPE;
  }
}

bool valid_dtype(int d) { return d >= 0 && d <= 3; }

// ============================================================================================
// MX / dynamic-block kernel (amax_and_convert_kernel, tensor_quant_mx.cu:239-294)
// ============================================================================================
struct MxParams {
  int fmt, sfmt;
  const float *gamax;
  int per_channel;
  int64_t cols;
};

__device__ __forceinline__ void mx_block_scale(float bamax, int64_t row, const MxParams &p,
                                               float &scale, float &unscale) {
  if (p.gamax) {
    float g = p.gamax[p.per_channel ? row : 0];
    global_scale(g, bamax, p.fmt, p.sfmt, scale, unscale);
  } else if (p.sfmt == MTQ_E8M0) {
    e8m0_scale(bamax, format_max(p.fmt), scale, unscale);
  } else {
    generic_scale(bamax, p.fmt, p.sfmt, scale, unscale);
  }
}

// quantize(), tensor_quant_mx.cu:36-55: sign * convert(|x| * scale) * unscale.
__device__ __forceinline__ float mx_qdq(float x, float scale, float unscale, int fmt) {
  float a = fabsf(x) * scale;
  float c = convert_fmt(a, fmt) * unscale;
  return x < 0.f ? -c : c;
}

// Fast path: cols % bs == 0 and 16-byte aligned rows, so blocks never straddle rows and the
// tensor is a flat sequence of blocks.  LPB = lanes per block = bs / N (N elements per lane);
// the block amax is a shuffle-max over LPB adjacent lanes (<= 8 lanes: one DPP row).  FMT >= 0
// bakes the element format in at compile time (the per-element conversion is the kernel's only
// real ALU work: with a runtime format it was VALU-bound at ~4.3 TB/s); FMT = -1 reads p.fmt.
// U = 2 vectors per lane, both loads issued first (MXFP8 0.727 -> 0.754-0.766 of the HBM
// roofline over one vector per lane, profiles/r03/dyn_u/).
template <typename T, int BS, int FMT, int U>
__global__ __launch_bounds__(kThreads) void mx_vec_kernel(const T *__restrict__ x,
                                                           T *__restrict__ y, int64_t nvec,
                                                           MxParams p) {
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int LPB = BS / N >= 1 ? BS / N : 1;
  static_assert(BS % N == 0, "block must be a multiple of the vector");
  const int fmt = FMT >= 0 ? FMT : p.fmt;
  // nvec % LPB == 0 and kThreads % LPB == 0: the LPB lanes of an MX block are all live or all out
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  const int lead = threadIdx.x % LPB;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * N);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (i - lead >= nvec) continue;
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) m = max_skip_nan(m, clamp_flt_max(fabsf(Elem<T>::ld(v[u].e[j]))));
    m = group_max_f<LPB>(m);
    const int64_t blk = i / LPB;
    float scale, unscale;
    if (p.gamax == nullptr && p.sfmt == MTQ_E8M0) {
      e8m0_scale(m, format_max(fmt), scale, unscale);
    } else {
      const int64_t row = (blk * BS) / p.cols;
      mx_block_scale(m, row, p, scale, unscale);
    }
#pragma unroll
    for (int j = 0; j < N; ++j)
      v[u].e[j] = Elem<T>::st(mx_qdq(Elem<T>::ld(v[u].e[j]), scale, unscale, fmt));
    stg_vec_nt(y + i * N, v[u]);
  }
}

// MXFP4 (E2M1 elements, E8M0 scales, no global amax) on 16-bit inputs with the native CDNA4
// FP4 converts (mtq_device.hpp Fp4Native): per packed pair one down-convert by the block's
// unscale 2^e and one up-convert by it -- sign(x) * e2m1(|x| * scale) * unscale of
// tensor_quant_mx.cu:36-55 in 2 instructions per 2 elements instead of ~24 VALU of table
// emulation.  The block amax comes from packed u16 max of the |x| patterns (NaN detected from
// the same max); blocks with a NaN, lanes with a -0 and exponents outside [-125, 125] (where the
// converts' exponent-only scale operand or subnormal results could differ) take the emulated
// path of mx_vec_kernel, so every element is bit-identical to it.
template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void mx_e2m1_native_kernel(const T *__restrict__ x,
                                                                   T *__restrict__ y,
                                                                   int64_t nvec) {
  using V = Vec<T>;
  constexpr int N = V::N;
  static_assert(N == 8 && BS % N == 0, "16-bit elements, block a multiple of the vector");
  constexpr int LPB = BS / N;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i - (threadIdx.x % LPB) >= nvec) return;
  V v = ldg_vec_nt(x + i * N);
  uint32_t w[4] = {v.raw.x, v.raw.y, v.raw.z, v.raw.w};
  const PairScan sc = scan_pairs(w);
  const uint32_t mb = group_max_u32<LPB>(sc.max_abs);
  const bool block_nan = mb > Fp4Native<T>::kInfBits;  // uniform over the block's lanes
  float amax;
  if (!block_nan) {
    amax = mb == Fp4Native<T>::kInfBits ? 3.402823466e38f : half_bits_to_float<T>(mb);
  } else {  // NaN is skipped by the reference's block max, as in mx_vec_kernel
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < N; ++j) m = max_skip_nan(m, clamp_flt_max(fabsf(Elem<T>::ld(v.e[j]))));
    amax = group_max_f<LPB>(m);
  }
  float scale, unscale;
  e8m0_scale(amax, 6.0f, scale, unscale);
  const int ue = (int)((__float_as_uint(unscale) >> 23) & 0xff) - 127;
  if (!block_nan && !sc.neg_zero && ue >= -125 && ue <= 125) {
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = Fp4Native<T>::up(Fp4Native<T>::down(w[j], unscale), unscale);
    v.raw = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j)
      v.e[j] = Elem<T>::st(mx_qdq(Elem<T>::ld(v.e[j]), scale, unscale, MTQ_E2M1));
  }
  stg_vec_nt(y + i * N, v);
}

// MXFP8 (E4M3 elements, E8M0 scales, no global amax) on 16-bit inputs with the native CDNA4
// scaled FP8 converts (Fp8Native): per two packed pairs one down-convert pair by the block's
// unscale 2^e and one up-convert pair -- the emulated path's sign(x) * e4m3(|x| * scale) *
// unscale (tensor_quant_mx.cu:36-55) in 4 instructions per 4 elements.  Block amax from packed
// u16 max of the |x| patterns, as mx_e2m1_native_kernel; blocks with a NaN or an infinity, lanes
// with a -0 and block exponents outside [kLo, kHi] take the emulated path, so every element is
// bit-identical to mx_vec_kernel (checked exhaustively, tests/test_gpu_mx_native.py).  U = 2
// vectors per lane, both loads issued first.
template <typename T, int BS, int U>
__global__ __launch_bounds__(kThreads) void mx_e4m3_native_kernel(const T *__restrict__ x,
                                                                   T *__restrict__ y,
                                                                   int64_t nvec) {
  using V = Vec<T>;
  constexpr int N = V::N;
  static_assert(N == 8 && BS % N == 0, "16-bit elements, block a multiple of the vector");
  constexpr int LPB = BS / N;
  constexpr int kLo = sizeof(T) == 2 && __is_same(T, _Float16) ? -30 : -125;
  constexpr int kHi = sizeof(T) == 2 && __is_same(T, _Float16) ? 7 : 125;
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  const int lead = threadIdx.x % LPB;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * N);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (i - lead >= nvec) continue;
    uint32_t w[4] = {v[u].raw.x, v[u].raw.y, v[u].raw.z, v[u].raw.w};
    const PairScan sc = scan_pairs(w);
    const uint32_t mb = group_max_u32<LPB>(sc.max_abs);
    const bool block_nan = mb > Fp4Native<T>::kInfBits;  // uniform over the block's lanes
    float amax;
    if (!block_nan) {
      amax = mb == Fp4Native<T>::kInfBits ? 3.402823466e38f : half_bits_to_float<T>(mb);
    } else {  // NaN is skipped by the reference's block max, as in mx_vec_kernel
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) m = max_skip_nan(m, clamp_flt_max(fabsf(Elem<T>::ld(v[u].e[j]))));
      amax = group_max_f<LPB>(m);
    }
    float scale, unscale;
    e8m0_scale(amax, 448.0f, scale, unscale);
    const int ue = (int)((__float_as_uint(unscale) >> 23) & 0xff) - 127;
    // (a block holding +-inf: E4M3 has no infinity -- the convert gives NaN where the emulated
    // path saturates to 448 -- so it is emulated too)
    if (mb < Fp4Native<T>::kInfBits && !sc.neg_zero && ue >= kLo && ue <= kHi) {
      const uint32_t p0 = Fp8Native<T>::down(w[0], w[1], unscale);
      const uint32_t p1 = Fp8Native<T>::down(w[2], w[3], unscale);
      w[0] = Fp8Native<T>::up(p0, unscale, false);
      w[1] = Fp8Native<T>::up(p0, unscale, true);
      w[2] = Fp8Native<T>::up(p1, unscale, false);
      w[3] = Fp8Native<T>::up(p1, unscale, true);
      v[u].raw = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j)
        v[u].e[j] = Elem<T>::st(mx_qdq(Elem<T>::ld(v[u].e[j]), scale, unscale, MTQ_E4M3));
    }
    stg_vec_nt(y + i * N, v[u]);
  }
}

template <typename T, int BS>
void launch_mx_vec(const T *x, T *y, int64_t nvec, MxParams p, hipStream_t stream) {
  const unsigned g = (unsigned)((nvec + kThreads - 1) / kThreads);
  if constexpr (sizeof(T) == 2) {
    if (p.fmt == MTQ_E2M1 && p.gamax == nullptr && p.sfmt == MTQ_E8M0) {
      count_dispatch(kDispMxE2m1Native);
      mx_e2m1_native_kernel<T, BS><<<g, kThreads, 0, stream>>>(x, y, nvec);
      return;
    }
    if (p.fmt == MTQ_E4M3 && p.gamax == nullptr && p.sfmt == MTQ_E8M0) {
      count_dispatch(kDispMxE4m3Native);
      const unsigned g2 = (unsigned)((nvec + 2 * kThreads - 1) / (2 * kThreads));
      mx_e4m3_native_kernel<T, BS, 2><<<g2, kThreads, 0, stream>>>(x, y, nvec);
      return;
    }
  }
  const unsigned g2 = (unsigned)((nvec + 2 * kThreads - 1) / (2 * kThreads));
  auto go = [&](auto fmt_c) {
    constexpr int F = decltype(fmt_c)::value;
    count_dispatch(kDispMxVec);
    mx_vec_kernel<T, BS, F, 2><<<g2, kThreads, 0, stream>>>(x, y, nvec, p);
  };
  switch (p.fmt) {
  case MTQ_E2M1: go(std::integral_constant<int, MTQ_E2M1>{}); break;
  case MTQ_E4M3: go(std::integral_constant<int, MTQ_E4M3>{}); break;
  case MTQ_E5M2: go(std::integral_constant<int, MTQ_E5M2>{}); break;
  case MTQ_INT8: go(std::integral_constant<int, MTQ_INT8>{}); break;
  case MTQ_E3M2: go(std::integral_constant<int, MTQ_E3M2>{}); break;
  case MTQ_E2M3: go(std::integral_constant<int, MTQ_E2M3>{}); break;
  default: go(std::integral_constant<int, -1>{}); break;
  }
}

// General path: one lane per element of the zero-padded [rows, padded_cols] matrix; BS lanes
// per block (BS divides 64, so a block never straddles a wave).
template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void mx_scalar_kernel(const T *__restrict__ x,
                                                              T *__restrict__ y, int64_t rows,
                                                              int64_t cols, int64_t pcols,
                                                              MxParams p) {
  const int64_t total = rows * pcols;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x; idx - (threadIdx.x % BS) < total;
       idx += stride) {
    const bool live = idx < total;
    int64_t row = live ? idx / pcols : 0;
    int64_t col = live ? idx - row * pcols : 0;
    bool real = live && col < cols;
    float v = real ? Elem<T>::ld(x[row * cols + col]) : 0.f;
    float m = group_max_f<BS>(clamp_flt_max(abs_or_zero(v)));
    if (!real) continue;
    float scale, unscale;
    mx_block_scale(m, row, p, scale, unscale);
    y[row * cols + col] = Elem<T>::st(mx_qdq(v, scale, unscale, p.fmt));
  }
}

template <typename T>
int launch_mx(const void *xv, void *yv, int64_t rows, int64_t cols, int bs, MxParams p,
              hipStream_t stream) {
  const T *x = reinterpret_cast<const T *>(xv);
  T *y = reinterpret_cast<T *>(yv);
  if (rows <= 0 || cols <= 0) return MTQ_OK;
  constexpr int N = Vec<T>::N;
  const int64_t n = rows * cols;
  if (cols % bs == 0 && bs % N == 0 && aligned16(x) && aligned16(y)) {
    int64_t nvec = n / N;
    switch (bs) {
    case 8: launch_mx_vec<T, 8>(x, y, nvec, p, stream); break;
    case 16: launch_mx_vec<T, 16>(x, y, nvec, p, stream); break;
    case 32: launch_mx_vec<T, 32>(x, y, nvec, p, stream); break;
    default: return MTQ_ERR_BLOCKSIZE;
    }
    return check_launch();
  }
  int64_t pcols = (cols + bs - 1) / bs * bs;
  unsigned g = grid_for(rows * pcols, kThreads);
  switch (bs) {
  case 8: mx_scalar_kernel<T, 8><<<g, kThreads, 0, stream>>>(x, y, rows, cols, pcols, p); break;
  case 16: mx_scalar_kernel<T, 16><<<g, kThreads, 0, stream>>>(x, y, rows, cols, pcols, p); break;
  case 32: mx_scalar_kernel<T, 32><<<g, kThreads, 0, stream>>>(x, y, rows, cols, pcols, p); break;
  default: return MTQ_ERR_BLOCKSIZE;
  }
  return check_launch();
}

// ============================================================================================
// amax reductions (MaxCalibrator.collect / reduce_amax)
// ============================================================================================
template <typename T>
__device__ __forceinline__ uint32_t vec_absmax_bits(const Vec<T> &v) {
  uint32_t m = 0;
#pragma unroll
  for (int j = 0; j < Vec<T>::N; ++j) {
    uint32_t b = abs_bits_t<T>(v.e[j]);
    m = b > m ? b : m;
  }
  return m;
}

// Per-tensor (K = 1, Q = 1), grid-stride form (unaligned inputs): wave max, block max in LDS, one
// atomicMax per block on the fp32 bit pattern.
__device__ __forceinline__ void block_atomic_max(uint32_t m, uint32_t *out) {
  __shared__ uint32_t red[kThreads / 64];
  m = wave_max_u32(m);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < kThreads / 64; ++k) m = red[k] > m ? red[k] : m;
    atomicMax(out, m);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void amax_all_kernel(const T *__restrict__ x, int64_t n,
                                                             int64_t nvec, uint32_t *out) {
  using V = Vec<T>;
  uint32_t m = 0;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += stride) {
    uint32_t b = vec_absmax_bits(ldg_vec(x + i * V::N));
    m = b > m ? b : m;
  }
  // scalar tail (n % N elements, or all of them when unaligned)
  for (int64_t t = nvec * V::N + (int64_t)blockIdx.x * kThreads + threadIdx.x; t < n; t += stride) {
    uint32_t b = abs_bits_t<T>(x[t]);
    m = b > m ? b : m;
  }
  block_atomic_max(m, out);
}

// Per-tensor, persistent form (default): `grid` blocks of 1024 threads (a few per CU), each
// lane keeps U non-temporal 16 B loads in flight per round, one atomicMax per block at the end.
// Same-address atomics serialise at ~12 ns each on gfx950 (measured: a one-vector-per-lane
// grid of 16k blocks spends 190 us in them), so the block count, not the load pattern, is
// what bounds a single-output reduction: keep it at O(CUs).
constexpr int kAmaxThreads = 1024;
template <typename T, int U>
__global__ __launch_bounds__(kAmaxThreads) void amax_persist_kernel(const T *__restrict__ x,
                                                                     int64_t n, int64_t nvec,
                                                                     uint32_t *out) {
  using V = Vec<T>;
  constexpr int64_t CH = (int64_t)kAmaxThreads * U;
  uint32_t m = 0;
  int64_t c0 = (int64_t)blockIdx.x * CH;
  const int64_t step = (int64_t)gridDim.x * CH;
  for (; c0 + CH <= nvec; c0 += step) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ldg_vec_nt(x + (c0 + u * kAmaxThreads + threadIdx.x) * V::N);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      uint32_t bb = vec_absmax_bits(v[u]);
      m = bb > m ? bb : m;
    }
  }
  if (c0 < nvec) {  // this block's partial chunk
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = c0 + u * kAmaxThreads + threadIdx.x;
      if (i < nvec) {
        uint32_t bb = vec_absmax_bits(ldg_vec_nt(x + i * V::N));
        m = bb > m ? bb : m;
      }
    }
  }
  if (blockIdx.x == gridDim.x - 1) {
    for (int64_t t = nvec * V::N + threadIdx.x; t < n; t += kAmaxThreads) {
      uint32_t bb = abs_bits_t<T>(x[t]);
      m = bb > m ? bb : m;
    }
  }
  __shared__ uint32_t red[kAmaxThreads / 64];
  m = wave_max_u32(m);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 1; k < kAmaxThreads / 64; ++k) m = red[k] > m ? red[k] : m;
    atomicMax(out, m);
  }
}

template <typename T, int U>
int launch_amax_persist(const T *x, int64_t n, int64_t nvec, uint32_t *out, int per_cu,
                        hipStream_t stream) {
  int64_t blocks = (nvec + (int64_t)kAmaxThreads * U - 1) / ((int64_t)kAmaxThreads * U);
  const int64_t cap = (int64_t)num_cus() * per_cu;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  count_dispatch(kDispAmaxPersist);
  amax_persist_kernel<T, U><<<(unsigned)blocks, kAmaxThreads, 0, stream>>>(x, n, nvec, out);
  return check_launch();
}

// Calibration bookkeeping (mtq_amax_fill / _fold / _check): tiny launches that live in this code
// object so the calibration pass needs no kernel the model's forward has not loaded.
__global__ __launch_bounds__(kThreads) void amax_fill_kernel(float *__restrict__ out, int64_t n, float value) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) out[i] = value;
}

// dst = max(dst, src) with a NaN of either operand propagating, as torch.maximum (which NaN is
// kept when both are NaN is not part of the contract)
__global__ __launch_bounds__(kThreads) void amax_fold_kernel(float *__restrict__ dst, const float *__restrict__ src,
                                                             int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float a = dst[i], b = src[i];
    dst[i] = (a != a) ? a : (b != b) ? b : fmaxf(a, b);
  }
}

// one workgroup: grid-stride flags, wave OR, LDS OR, thread 0 writes all three
constexpr int kCheckThreads = 1024;
__device__ __forceinline__ int check_bits(float v) {
  return (v != v) | ((fabsf(v) == __builtin_inff()) << 1) | ((v < 0.f) << 2);
}

// bits of NaN / inf / negative over the block; MULTI: a grid-stride pass over 16-byte vectors
// (x aligned, n % N elements past the last whole vector by block 0), OR-ed into flags zeroed by
// amax_check_zero_kernel; else one block over scalars, writing flags
template <typename T, bool MULTI>
__global__ __launch_bounds__(kCheckThreads) void amax_check_kernel(const T *__restrict__ x, int64_t n,
                                                                  int32_t *__restrict__ flags) {
  int bits = 0;
  if constexpr (MULTI) {
    using V = Vec<T>;
    const int64_t nvec = n / V::N;
    const int64_t stride = (int64_t)gridDim.x * kCheckThreads;
    for (int64_t i = (int64_t)blockIdx.x * kCheckThreads + threadIdx.x; i < nvec; i += stride) {
      const V v = ldg_vec_nt(x + i * V::N);
#pragma unroll
      for (int j = 0; j < V::N; ++j) bits |= check_bits(Elem<T>::ld(v.e[j]));
    }
    if (blockIdx.x == 0)
      for (int64_t i = nvec * V::N + threadIdx.x; i < n; i += kCheckThreads) bits |= check_bits(Elem<T>::ld(x[i]));
  } else {
    for (int64_t i = threadIdx.x; i < n; i += kCheckThreads) bits |= check_bits(Elem<T>::ld(x[i]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) bits |= __shfl_xor(bits, o);
  __shared__ int red[kCheckThreads / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = bits;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kCheckThreads / 64; ++w) bits |= red[w];
    if constexpr (MULTI) {
      for (int k = 0; k < 3; ++k)
        if ((bits >> k) & 1) atomicOr(flags + k, 1);
    } else {
      flags[0] = bits & 1;
      flags[1] = (bits >> 1) & 1;
      flags[2] = (bits >> 2) & 1;
    }
  }
}

__global__ void amax_check_zero_kernel(int32_t *flags) {
  if (threadIdx.x < 3) flags[threadIdx.x] = 0;
}

// y[r, :] = x[r, :] if any of row r's k expert indices lies in [0, E), else +0 (the MoE shared
// input quantizer's masking of rows routed to no local expert, huggingface.py _QuantFusedExperts):
// one pass instead of the compare / and / any / where sequence.  VEC: 16-byte vectors (cols a
// multiple of the vector, 16-byte aligned), else one element per lane.
template <typename T, bool VEC>
__global__ __launch_bounds__(kThreads) void mask_rows_kernel(const T *__restrict__ x, T *__restrict__ y,
                                                             const int64_t *__restrict__ idx, int64_t rows,
                                                             int64_t cols, int k, int64_t experts) {
  constexpr int N = VEC ? Vec<T>::N : 1;
  const int64_t per_row = cols / N, total = rows * per_row;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += stride) {
    const int64_t r = i / per_row;
    bool routed = false;
    for (int j = 0; j < k; ++j) {
      const int64_t e = idx[r * k + j];
      routed |= (e >= 0) & (e < experts);
    }
    if constexpr (VEC) {
      Vec<T> v = ldg_vec(x + i * N);
      if (!routed) v.raw = make_uint4(0u, 0u, 0u, 0u);
      stg_vec(y + i * N, v);
    } else {
      y[i] = routed ? x[i] : Elem<T>::st(0.f);
    }
  }
}

// Generic: one element per lane, atomicMax per element (any P, K, Q, alignment).
template <typename T>
__global__ __launch_bounds__(kThreads) void amax_generic_kernel(const T *__restrict__ x,
                                                                 int64_t n, int64_t K, int64_t Q,
                                                                 uint32_t *out) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    int64_t k = (i / Q) % K;
    atomicMax(out + k, abs_bits_t<T>(x[i]));
  }
}

// Rows, unrolled form: one item = (row, chunk of <= G*U vectors) per group of G lanes, U
// non-temporal 16 B loads in flight per lane, one chunk per group (no grid-stride loop, the
// structure that reaches ~6 TB/s in ew_vec_kernel).  With one chunk per row and P == 1 every
// output word has exactly one writer in the launch, so the fold is a plain load-max-store
// instead of an atomic (R atomics to distinct words still cost ~10 us at R = 32k).
template <typename T, int G, int U, bool EXCL>
__global__ __launch_bounds__(kThreads) void amax_rows_u_kernel(const T *__restrict__ x,
                                                                int64_t R, int64_t Q, int64_t K,
                                                                int64_t chunks, uint32_t *out) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const int64_t qvec = Q / N;
  const int64_t item = (int64_t)blockIdx.x * (kThreads / G) + threadIdx.x / G;
  if (item >= R * chunks) return;  // whole G-lane groups exit together
  const int gl = threadIdx.x % G;
  const int64_t r = item / chunks, c = item - r * chunks;
  const int64_t v0 = c * (int64_t)(G * U);
  int64_t v1 = v0 + G * U;
  v1 = v1 < qvec ? v1 : qvec;
  const T *row = x + r * Q;
  // unconditional loads (a lane past the chunk re-reads its last vector, then contributes 0): a
  // load under a lane condition is waited with vmcnt(0) right behind it, serialising the U loads
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + gl + u * G;
    v[u] = ldg_vec_nt(row + (i < v1 ? i : v1 - 1) * N);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (v0 + gl + u * G >= v1) v[u].raw = make_uint4(0, 0, 0, 0);
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    uint32_t b = vec_absmax_bits(v[u]);
    m = b > m ? b : m;
  }
  m = group_max_u32<G>(m);
  if (gl == 0) {
    if (EXCL) {
      uint32_t o = out[r];
      out[r] = m > o ? m : o;
    } else {
      atomicMax(out + (r % K), m);
    }
  }
}

// Columns, wide form: 1024-thread blocks, `lpr` (<= 64) lanes across a column chunk and
// 1024 / lpr row lanes, U loads in flight per lane; row lanes fold in LDS, then one atomicMax
// per column per block.  Global atomics cost ~30 ns per thousand on gfx950 (measured: 1 M of
// them add ~35 us to a 44 us read), so the grid is kept to O(CUs) blocks and the atomic count
// to slabs x K with few slabs; 16 waves per block keep ~128 KB in flight per CU.
constexpr int kColsThreads = 1024;
template <typename T, int U>
__global__ __launch_bounds__(kColsThreads) void amax_cols_wide_kernel(
    const T *__restrict__ x, int64_t P, int64_t K, int lpr, int64_t nchunks,
    int64_t rows_per_slab, uint32_t *out) {
  using V = Vec<T>;
  constexpr int N = V::N;
  __shared__ uint32_t sh[64 * N];
  const int64_t kvec = K / N;
  const int64_t chunk = blockIdx.x % nchunks, slab = blockIdx.x / nchunks;
  const int tc = threadIdx.x % lpr, tr = threadIdx.x / lpr;
  const int rstep = kColsThreads / lpr;
  const int64_t kv = chunk * lpr + tc;
  const bool active = kv < kvec;
  for (int i = threadIdx.x; i < lpr * N; i += kColsThreads) sh[i] = 0;
  __syncthreads();
  uint32_t m[N];
#pragma unroll
  for (int j = 0; j < N; ++j) m[j] = 0;
  if (active) {
    const int64_t p0 = slab * rows_per_slab;
    int64_t p1 = p0 + rows_per_slab;
    p1 = p1 < P ? p1 : P;
    const T *base = x + kv * N;
    int64_t p = p0 + tr;
    for (; p + (int64_t)(U - 1) * rstep < p1; p += (int64_t)U * rstep) {
      V v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = ldg_vec_nt(base + (p + (int64_t)u * rstep) * K);
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < N; ++j) {
          uint32_t b = abs_bits_t<T>(v[u].e[j]);
          m[j] = b > m[j] ? b : m[j];
        }
    }
    for (; p < p1; p += rstep) {
      V v = ldg_vec_nt(base + p * K);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        uint32_t b = abs_bits_t<T>(v.e[j]);
        m[j] = b > m[j] ? b : m[j];
      }
    }
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (m[j]) atomicMax(sh + tc * N + j, m[j]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < lpr * N; i += kColsThreads) {
    const int64_t col = chunk * lpr * N + i;
    if (col < K && sh[i]) atomicMax(out + col, sh[i]);
  }
}

template <typename T>
int launch_amax_cols_wide(const T *x, int64_t P, int64_t K, uint32_t *out, int blocks_per_2cu,
                          hipStream_t stream) {
  constexpr int N = Vec<T>::N, U = 8;
  const int64_t kvec = K / N;
  const int lpr = (int)(kvec < 64 ? kvec : 64);
  const int64_t nchunks = (kvec + lpr - 1) / lpr;
  const int rstep = kColsThreads / lpr;
  // blocks_per_2cu == 0: 1 block per CU when every row lane then gets >= 4 unrolled rounds,
  // else 2 (measured: [32768, 4096] 45 vs 53 us, [8192, 4096] 19.7 vs 16.0 us).  The slab
  // count is rounded down so that the grid never spills a partial second round of blocks.
  if (blocks_per_2cu == 0) {
    const int64_t slabs1 = (int64_t)num_cus() / nchunks;
    blocks_per_2cu = (slabs1 >= 1 && P / slabs1 >= (int64_t)4 * U * rstep) ? 2 : 4;
  }
  const int64_t want = (int64_t)num_cus() * blocks_per_2cu / 2;
  int64_t slabs = want / nchunks;
  const int64_t max_slabs = (P + (int64_t)U * rstep - 1) / ((int64_t)U * rstep);
  if (slabs > max_slabs) slabs = max_slabs;
  if (slabs < 1) slabs = 1;
  const int64_t rows_per_slab = (P + slabs - 1) / slabs;
  slabs = (P + rows_per_slab - 1) / rows_per_slab;
  const unsigned g = (unsigned)(nchunks * slabs);
  count_dispatch(kDispAmaxColsWide);
  amax_cols_wide_kernel<T, U><<<g, kColsThreads, 0, stream>>>(x, P, K, lpr, nchunks,
                                                              rows_per_slab, out);
  return check_launch();
}

// Short rows (Q / N <= 64 vectors, e.g. the [rows * K / 128, 128] block view): a group of G
// lanes covers one row, and each group takes RU consecutive rows with one load per row in
// flight per lane; in exclusive mode the accumulator words are fetched before the data so
// their latency overlaps it.
template <typename T, int G, int RU, bool EXCL>
__global__ __launch_bounds__(kThreads) void amax_rows_short_kernel(const T *__restrict__ x,
                                                                    int64_t R, int64_t Q,
                                                                    int64_t K, uint32_t *out) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const int64_t qvec = Q / N;
  const int64_t r0 = ((int64_t)blockIdx.x * (kThreads / G) + threadIdx.x / G) * RU;
  if (r0 >= R) return;
  const int gl = threadIdx.x % G;
  uint32_t o[RU];
  if (EXCL && gl == 0) {
#pragma unroll
    for (int u = 0; u < RU; ++u) o[u] = r0 + u < R ? out[r0 + u] : 0;
  }
  V v[RU];
#pragma unroll
  for (int u = 0; u < RU; ++u) {  // unconditional (clamped) loads, as amax_rows_u_kernel
    const int64_t rr = r0 + u < R ? r0 + u : R - 1;
    v[u] = ldg_vec_nt(x + rr * Q + (int64_t)(gl < qvec ? gl : qvec - 1) * N);
  }
#pragma unroll
  for (int u = 0; u < RU; ++u)
    if (!(r0 + u < R && gl < qvec)) v[u].raw = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int u = 0; u < RU; ++u) {
    uint32_t m = group_max_u32<G>(vec_absmax_bits(v[u]));
    if (gl == 0 && r0 + u < R) {
      if (EXCL)
        out[r0 + u] = m > o[u] ? m : o[u];
      else
        atomicMax(out + ((r0 + u) % K), m);
    }
  }
}

template <typename T>
int launch_amax_rows_u(const T *x, int64_t P, int64_t K, int64_t Q, uint32_t *out,
                       hipStream_t stream) {
  constexpr int N = Vec<T>::N;
  const int64_t R = P * K, qvec = Q / N;
  if (qvec >= 64) {
    constexpr int G = 64, U = 8;
    const int64_t chunks = (qvec + G * U - 1) / (G * U);
    const int64_t items = R * chunks;
    const unsigned g = (unsigned)((items + kThreads / G - 1) / (kThreads / G));
    count_dispatch(kDispAmaxRowsU);
    if (chunks == 1 && P == 1)
      amax_rows_u_kernel<T, G, U, true><<<g, kThreads, 0, stream>>>(x, R, Q, K, chunks, out);
    else
      amax_rows_u_kernel<T, G, U, false><<<g, kThreads, 0, stream>>>(x, R, Q, K, chunks, out);
    return check_launch();
  }
  // short rows: the smallest power-of-two group covering the row, RU rows per group
  constexpr int RU = 4;
  auto go = [&](auto gtag) {
    constexpr int G = decltype(gtag)::value;
    const int64_t rows_per_block = (int64_t)(kThreads / G) * RU;
    const unsigned g = (unsigned)((R + rows_per_block - 1) / rows_per_block);
    count_dispatch(kDispAmaxRowsShort);
    if (P == 1)
      amax_rows_short_kernel<T, G, RU, true><<<g, kThreads, 0, stream>>>(x, R, Q, K, out);
    else
      amax_rows_short_kernel<T, G, RU, false><<<g, kThreads, 0, stream>>>(x, R, Q, K, out);
    return check_launch();
  };
  if (qvec > 32) return go(std::integral_constant<int, 64>{});
  if (qvec > 16) return go(std::integral_constant<int, 32>{});
  if (qvec > 8) return go(std::integral_constant<int, 16>{});
  if (qvec > 4) return go(std::integral_constant<int, 8>{});
  if (qvec > 2) return go(std::integral_constant<int, 4>{});
  if (qvec > 1) return go(std::integral_constant<int, 2>{});
  return go(std::integral_constant<int, 1>{});
}

template <typename T>
int launch_amax(const void *xv, int64_t P, int64_t K, int64_t Q, float *outf,
                hipStream_t stream) {
  const T *x = reinterpret_cast<const T *>(xv);
  uint32_t *out = reinterpret_cast<uint32_t *>(outf);
  const int64_t n = P * K * Q;
  if (n <= 0) return MTQ_OK;
  constexpr int N = Vec<T>::N;
  const bool al = aligned16(x);
  if (K == 1 && (Q == 1 || P == 1)) {  // per-tensor
    if (!al) {  // unaligned: the all-scalar grid-stride form
      unsigned g = grid_for(n / N + 1, kThreads * 4);
      amax_all_kernel<T><<<g, kThreads, 0, stream>>>(x, n, 0, out);
      return check_launch();
    }
    // persistent grid, 2 x 1024-thread blocks per CU, 8 loads in flight per lane (r01 sweep,
    // scripts/sweep_amax.py: 1 / 4 blocks per CU or 4 loads per lane no faster)
    return launch_amax_persist<T, 8>(x, n, n / N, out, 2, stream);
  }
  if (Q % N == 0 && al && Q >= N) return launch_amax_rows_u<T>(x, P, K, Q, out, stream);
  // per-column (axis -1 kept): 1024-thread wide-column kernel with the LDS fold; the block count
  // per CU is picked from the shape (launch_amax_cols_wide)
  if (Q == 1 && K % N == 0 && al) return launch_amax_cols_wide<T>(x, P, K, out, 0, stream);
  unsigned g = grid_for(n, kThreads);
  amax_generic_kernel<T><<<g, kThreads, 0, stream>>>(x, n, K, Q, out);
  return check_launch();
}

// ============================================================================================
// Dynamic INT-n block quant with optional per-column pre-quant scale (AWQ-lite weight side)
// ============================================================================================
// U vectors per lane, all U loads issued first
template <typename T, int BLK, int U>
__global__ __launch_bounds__(kThreads) void block_quant_dyn_kernel(
    const T *__restrict__ x, T *__restrict__ y, const T *__restrict__ pqs, int64_t nvec,
    int64_t cols, float max_bound, float min_bound) {
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int LPB = BLK / N;
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  const int lead = threadIdx.x % LPB;  // a block's LPB lanes are in range together
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * N);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (i - lead >= nvec) continue;
    if (pqs) {
      const int64_t col = (i * N) % cols;
      V s = ldg_vec(pqs + col);
#pragma unroll
      for (int j = 0; j < N; ++j) v[u].e[j] = Elem<T>::st(Elem<T>::ld(v[u].e[j]) * Elem<T>::ld(s.e[j]));
    }
    uint32_t m = group_max_u32<LPB>(vec_absmax_bits(v[u]));
    IntQ q = make_intq(__uint_as_float(m), max_bound, min_bound);
#pragma unroll
    for (int j = 0; j < N; ++j) v[u].e[j] = Elem<T>::st(int_qdq(Elem<T>::ld(v[u].e[j]), q));
    stg_vec_nt(y + i * N, v[u]);
  }
}

// ============================================================================================
// Histogram of |x| (torch.histc semantics, LDS-privatised)
// ============================================================================================
template <typename T>
__global__ __launch_bounds__(kThreads) void hist_kernel(const T *__restrict__ x, int64_t n,
                                                         const float *hmax, int bins,
                                                         int skip_zeros, uint32_t *counts,
                                                         int use_lds) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  float lo = 0.f, hi = *hmax;
  if (hi == lo) {  // histc_select_outer_bin_edges: widen a degenerate range by 1 on each side
    lo -= 1.f;
    hi += 1.f;
  }
  const float fb = (float)bins;
  const float span = hi - lo;
  if (use_lds) {
    for (int b = threadIdx.x; b < bins; b += kThreads) sh[b] = 0;
    __syncthreads();
  }
  uint32_t *dst = use_lds ? sh : counts;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    float v = fabsf(Elem<T>::ld(x[i]));
    if (skip_zeros && v == 0.f) continue;
    if (!(v >= lo && v <= hi)) continue;  // outside the range or NaN
    int b = (int)(((v - lo) * fb) / span);
    if (b == bins) b -= 1;
    atomicAdd(dst + b, 1u);
  }
  if (use_lds) {
    __syncthreads();
    for (int b = threadIdx.x; b < bins; b += kThreads)
      if (sh[b]) atomicAdd(counts + b, sh[b]);
  }
}

// Division form (default, any dtype): the per-element true division of the formula above is
// replaced by Markstein's correction q = fma(fma(-q0, span, t), y, q0), q0 = t * y,
// y = RN(1 / span), which is the correctly rounded t / span for normal operands (checked on
// the host against the IEEE division for every bf16 and f16 |x| at 20 000 random ranges and
// bin counts: 6.96e8 cases, no difference; scripts/check_hist_division.c).  4 VALU ops instead
// of the ~10 of a divide, no table read: one LDS add per element into REP interleaved copies.
constexpr int kHistDivThreads = 1024;
template <typename T, int REP, int U>
__global__ __launch_bounds__(kHistDivThreads) void hist_div_kernel(
    const T *__restrict__ x, int64_t nvec, int64_t vec_per_block, const float *hmax, int bins,
    int skip_zeros, uint32_t *counts) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  using V = Vec<T>;
  float lo = 0.f, hi = *hmax;
  if (hi == lo) {
    lo -= 1.f;
    hi += 1.f;
  }
  const float fb = (float)bins;
  const float span = hi - lo;
  const float y = 1.f / span;
  const uint32_t last = (uint32_t)bins - 1u;
  for (int b = threadIdx.x; b < bins * REP; b += kHistDivThreads) sh[b] = 0;
  __syncthreads();
  const int c = threadIdx.x % REP;
  const int64_t v0 = (int64_t)blockIdx.x * vec_per_block;
  int64_t v1 = v0 + vec_per_block;
  v1 = v1 < nvec ? v1 : nvec;
  for (int64_t i = v0 + threadIdx.x; i < v1; i += (int64_t)kHistDivThreads * U) {
    V v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = i + (int64_t)u * kHistDivThreads;
      if (k < v1)
        v[u] = ldg_vec_nt(x + k * V::N);
      else
        v[u].raw = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);  // NaN: dropped
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int j = 0; j < V::N; ++j) {
        const float a = fabsf(Elem<T>::ld(v[u].e[j]));
        // a >= 0 >= lo always; NaN fails the compare
        if (a <= hi && !(skip_zeros && a == 0.f)) {
          const float t = (a - lo) * fb;
          const float q0 = t * y;
          const float q = __builtin_fmaf(__builtin_fmaf(-q0, span, t), y, q0);
          uint32_t b = (uint32_t)(int)q;
          b = b < last ? b : last;  // q == bins -> last bin (histc); overflow guard
          atomicAdd(sh + b * REP + c, 1u);
        }
      }
    }
  }
  __syncthreads();
  for (int b = threadIdx.x; b < bins; b += kHistDivThreads) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < REP; ++k) s += sh[b * REP + k];
    if (s) atomicAdd(counts + b, s);
  }
}

// Value-histogram form (bf16 / f16, bins <= 8192; default for them).  |x| of a 16-bit float is
// one of 32768 bit patterns, so a block first counts the patterns themselves in LDS (one
// `and` + one `ds_add_u32` per element, no arithmetic), then folds the <= 32768 pattern counts
// into its bins with the same exact bin formula as hist_div_kernel, evaluated once per distinct
// pattern instead of once per element.  The bin of an element is a function of its pattern
// only, so the counts equal the per-element kernel's exactly.  Measured on hist_div_kernel
// (profiles/r02/histogram/): ~14 VALU instructions per element, LDS 46 % busy -- the per-element
// bin arithmetic, not the LDS, was what this form removes.  LDS: 128 KiB pattern counts + the
// bins, so one 1024-thread block per CU over one contiguous chunk.
constexpr int kHistValThreads = 1024;
constexpr int kHistPatterns = 32768;
//
// CHUNKED: the torch.histc chunk emulation.  Chunk c covers elements [e0, e1) (from `bounds`, or
// c * chunk_elems clipped to n_elems when bounds is null) and owns `bpc` consecutive workgroups;
// each workgroup stores its whole LDS bin row (plain non-temporal stores, no atomics) into its own
// row of the scratch, rows[block * bins, +bins); element bounds need not fall on vectors, so the
// two edge vectors of a chunk are counted separately (below).
//
// The rows are folded by a second, small launch (hist_fold_blocks_kernel): chunk c's count of bin
// b is the exact sum of its bpc workgroup rows, and hist[b] = sum_c min(fp32(count_c[b]), 2^24)
// in chunk order (+ an optional running histogram).  Every row is overwritten by every call, so
// the scratch needs no zeroing.  (r05: per-chunk rows filled by workgroup atomics and zeroed again
// by the fold measured 42.4 us against 41.0 us for this form, count + fold, bf16 [8192, 14336],
// 16 chunks, scripts/exp/hist_exp.hip; a fold inside the counting launch -- its last workgroup
// after an agent-scope check-in -- cost 12 us at the launch's tail.)
struct HistChunks {
  const int64_t *bounds;  // [chunks + 1] element offsets (device), or null: uniform chunks
  int64_t chunk_elems;
  int64_t n_elems;
  int bpc;  // workgroups per chunk
  int chunks;
  uint32_t *rows;  // [chunks * bpc, bins] per-workgroup counts, overwritten
};

// NZ (skip_zeros, r06): torch.histc's chunks of the compacted non-zero elements, counted in ONE
// read of the input.  The chunk boundaries depend on the non-zero count of everything before
// them, so the counting launch cannot know them; it counts uniform, slab-aligned workgroup ranges
// instead, storing per workgroup its bin row, its non-zero count and the non-zero count of each
// slab (one 2048-vector batch of its count loop, counted by wave ballots: no LDS traffic), and
// zeroes the boundary rows.  A boundary that falls strictly inside a workgroup's range is then
// resolved by hist_nz_recount_kernel: one workgroup per (boundary, slab) re-reads only the slabs
// of that range which hold non-zeros of the boundary's chunk-before segment (at most one
// workgroup range per boundary, ~1.5 % of the input at 16 threads) and adds their bins into
// rec[b]; hist_nz_fold_kernel assembles chunk c from whole rows, rec[c + 1] (its part of the
// workgroup its end cuts) and row - sum rec (its part of the workgroup its start cuts) -- all
// exact uint32 -- then clamps and adds the chunks in order as the CHUNKED fold does.  Replaces
// the r05 per-tile non-zero pass + per-boundary block scans (a second full read of the input).
struct HistNz {
  int64_t vpb;         // vectors per workgroup range (a multiple of the slab)
  int S;               // slabs per workgroup range
  uint32_t *rows;      // [G, bins]
  uint32_t *wg_tot;    // [G] non-zero elements per workgroup range
  uint32_t *slab_tot;  // [G, S] non-zero elements per slab
  uint32_t *rec;       // [threads, bins] boundary segment counts (zeroed by the count launch)
  int64_t rec_words;
};
constexpr int kHvCounts = 0, kHvChunked = 1, kHvNz = 2;

// workgroups per chunk of the chunked count: ~one 1024-thread workgroup per CU in total, at
// least kHistValThreads * 8 vectors each
int64_t hist_chunk_bpc(int64_t n, int chunks) {
  const int64_t cvec = (n / 8 + chunks - 1) / chunks;
  int64_t bpc = ((int64_t)num_cus() + chunks - 1) / chunks;
  const int64_t by_size = (cvec + (int64_t)kHistValThreads * 8 - 1) / ((int64_t)kHistValThreads * 8);
  bpc = bpc < by_size ? bpc : by_size;
  return bpc < 1 ? 1 : bpc;
}

// 1024 threads = 64 bins x 16 chunk lanes: a thread sums its chunk's bpc workgroup rows (exact,
// uint32), clamps at 2^24 in fp32; the chunk-0 lane of each bin adds the 16 clamped counts of the
// group in chunk order (torch.histc's thread-order fold of its fp32 per-thread counts), group
// after group, then + accum[b] for b < accum_n (the calibrator's running histogram,
// `hist[:old.numel()] += old`).
template <int BW>  // bins per workgroup; BW * 16 threads
__global__ __launch_bounds__(BW * 16) void hist_fold_blocks_kernel(const uint32_t *__restrict__ rows, int bpc,
                                                                   int chunks, int bins, const float *accum,
                                                                   int64_t accum_n, float *hist) {  // accum may alias hist
  __shared__ float part[16][BW];
  const int bl = threadIdx.x % BW, cl = threadIdx.x / BW, b = blockIdx.x * BW + bl;
  float h = 0.f;
  for (int c0 = 0; c0 < chunks; c0 += 16) {
    const int c = c0 + cl;
    if (c < chunks && b < bins) {
      const uint32_t *r = rows + (int64_t)c * bpc * bins + b;
      uint32_t sum = 0;
      // 16 rows' loads issued together (clamped to the chunk's last row, then masked): one round
      // trip for the usual bpc <= 16 (r05x trace: 4.75 us with two dependent groups of 8)
      for (int k0 = 0; k0 < bpc; k0 += 16) {
        uint32_t v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          v[k] = __builtin_nontemporal_load(r + (int64_t)(k0 + k < bpc ? k0 + k : bpc - 1) * bins);
#pragma unroll
        for (int k = 0; k < 16; ++k) sum += k0 + k < bpc ? v[k] : 0u;
      }
      part[cl][bl] = fminf((float)sum, 16777216.f);
    }
    __syncthreads();
    if (cl == 0 && b < bins) {
      const int m = chunks - c0 < 16 ? chunks - c0 : 16;
      for (int k = 0; k < m; ++k) h += part[k][bl];
    }
    __syncthreads();
  }
  if (cl == 0 && b < bins) {
    if (b < accum_n) h += accum[b];
    hist[b] = h;
  }
}

template <typename T, int U, int MODE = kHvCounts>
__global__ __launch_bounds__(kHistValThreads) void hist_value_kernel(
    const T *__restrict__ x, int64_t nvec, int64_t vec_per_block, const float *hmax, int bins,
    int skip_zeros, uint32_t *counts, HistChunks ch, HistNz nz) {
  constexpr bool CHUNKED = MODE == kHvChunked;
  static_assert(sizeof(T) == 2, "pattern histogram is for 16-bit floats");
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t *vh = sh;                  // [32768] counts per |x| bit pattern
  uint32_t *bh = sh + kHistPatterns;  // [bins]
  // the workgroup's vector range first, so its first loads are in flight before the hmax round
  // trip and the LDS zeroing below (r05: 41.8 -> 38.3 us with the A/B loop, bf16 [8192, 14336],
  // scripts/exp/hist_exp.hip v562)
  int64_t v0, v1, e0 = 0, e1 = 0;
  if constexpr (CHUNKED) {
    const int c = blockIdx.x / ch.bpc, s = blockIdx.x % ch.bpc;
    if (ch.bounds) {
      e0 = ch.bounds[c];
      e1 = ch.bounds[c + 1];
    } else {
      e0 = (int64_t)c * ch.chunk_elems;
      e0 = e0 < ch.n_elems ? e0 : ch.n_elems;
      e1 = e0 + ch.chunk_elems;
      e1 = e1 < ch.n_elems ? e1 : ch.n_elems;
    }
    // whole vectors inside [e0, e1) go through the hot loop unmasked; the (at most two) vectors a
    // chunk edge cuts are counted below by lane 0 of the chunk's first block (masking them at load
    // time made every prefetch wait for its data: 53 vs 41 us, r05d)
    const int64_t cv0 = (e0 + 7) / 8, cv1 = e1 / 8 > cv0 ? e1 / 8 : cv0;
    const int64_t per = (cv1 - cv0 + ch.bpc - 1) / ch.bpc;
    v0 = cv0 + (int64_t)s * per;
    v1 = v0 + per;
    v1 = v1 < cv1 ? v1 : cv1;
    v0 = v0 < v1 ? v0 : v1;
  } else {
    if constexpr (MODE == kHvNz) vec_per_block = nz.vpb;
    v0 = (int64_t)blockIdx.x * vec_per_block;
    v1 = v0 + vec_per_block;
    v1 = v1 < nvec ? v1 : nvec;
  }
  // Two named register batches (A, B) with unconditional loads clamped to the range's last vector
  // (vector 0 for an empty range; nvec >= 1): no load sits under a branch and no in-flight
  // register is copied, so the wait in front of each batch's count is vmcnt(U) -- the other
  // batch stays in flight -- where the earlier cur / next form, its next-batch load under a
  // condition, compiled to vmcnt(0) before every count (ISA).  Lanes past the range count a
  // per-lane NaN pattern (> phi, never folded) so the tail's dummy atomics do not all collide.
  const int64_t vlast = v1 > 0 ? v1 - 1 : 0;
  auto ld = [&](int64_t k) -> u32x4 {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(x + (k < vlast ? k : vlast) * 8));
  };
  const uint32_t dummy = 0x7FC0u + (threadIdx.x & 63u);
  auto count = [&](const u32x4 v, bool ok) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      atomicAdd(vh + (ok ? (w[j] & 0x7FFFu) : dummy), 1u);
      atomicAdd(vh + (ok ? ((w[j] >> 16) & 0x7FFFu) : dummy), 1u);
    }
  };
  constexpr int64_t kStep = (int64_t)kHistValThreads * U;
  int64_t i = v0 + threadIdx.x;
  u32x4 a[U], b[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = ld(i + (int64_t)u * kHistValThreads);

  float lo = 0.f, hi = *hmax;
  if (hi == lo) {
    lo -= 1.f;
    hi += 1.f;
  }
  // Only patterns p <= phi, the largest pattern whose value is <= hi, can land in a bin (the
  // patterns of non-negative floats are ordered as their values; NaN hi: none), so only those
  // counters are zeroed here and folded below; the count loop still increments every pattern, the
  // entries past phi are never read.  bf16 [32768, 4096] with |x| <= 96: 128 -> 68 KiB zeroed and
  // folded per block (r04: fixed cost 5.1 us of the 46.6 us launch, scripts/exp/hist_exp.hip).
  int phi;
  if (!(hi >= 0.f)) {
    phi = -1;
  } else if constexpr (__is_same(T, __bf16)) {
    const uint32_t hb = __float_as_uint(hi) >> 16;  // truncation = round toward zero
    phi = (int)(hb < 0x7F80u ? hb : 0x7F80u);
  } else {
    // round toward zero to f16 (v_cvt_pkrtz_f16_f32): the largest f16 <= hi (65504 above it)
    const auto h2 = __builtin_amdgcn_cvt_pkrtz(hi, 0.f);
    uint16_t hb;
    __builtin_memcpy(&hb, &h2, 2);
    phi = (int)(hb < 0x7C00u ? hb : 0x7C00u);
  }
  const int nz4 = (phi + 4) / 4;  // 16-byte words covering patterns [0, phi]
  for (int k = threadIdx.x; k < nz4; k += kHistValThreads)
    reinterpret_cast<uint4 *>(vh)[k] = make_uint4(0u, 0u, 0u, 0u);
  for (int k = threadIdx.x; k < bins; k += kHistValThreads) bh[k] = 0;
  uint32_t *slab_w = bh + bins;  // [S][16] per-wave non-zero counts of each slab (kHvNz)
  const int wave = threadIdx.x >> 6;
  if constexpr (MODE == kHvNz) {
    // this workgroup's share of the boundary rows, zeroed for the recount launch
    const int64_t per = (nz.rec_words + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = (int64_t)blockIdx.x * per;
    for (int64_t k = r0 + threadIdx.x; k < r0 + per && k < nz.rec_words; k += kHistValThreads) nz.rec[k] = 0u;
  }
  __syncthreads();  // LDS zeroed (the first batch's loads issued before)
  // (no branch around B's count either: with one, the compiler sank B's loads into it and waited
  // vmcnt(0) right behind them; a past-the-end B batch costs its lanes' dummy atomics instead)
  // kHvNz: a slab = one batch (kStep vectors, contiguous); the wave's non-zero halves of a batch
  // by ballots (wave-uniform, SALU popcounts), kept in lane `slab` of one VGPR (a lane select: no
  // LDS write and no branch in the loop -- a lane-0-only LDS write split the loop body and the
  // scheduler then waited vmcnt(0) for batch B before issuing the next A loads); S <= 64
  uint32_t slab_acc = 0u;
  auto slab_count = [&](const u32x4 *v, int64_t ib, int slab) {
    if constexpr (MODE == kHvNz) {
      int c = 0;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t okm = __ballot(ib + (int64_t)u * kHistValThreads < v1);
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t m = w[j] & 0x7FFF7FFFu;
          c += __popcll(__ballot((m & 0xFFFFu) != 0u) & okm);
          c += __popcll(__ballot(m > 0xFFFFu) & okm);
        }
      }
      slab_acc = (int)(threadIdx.x & 63) == slab ? (uint32_t)c : slab_acc;  // v_cmp + v_cndmask
    }
  };
  for (int it = 0; i < v1; i += 2 * kStep, ++it) {
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(i + kStep + (int64_t)u * kHistValThreads);
#pragma unroll
    for (int u = 0; u < U; ++u) count(a[u], i + (int64_t)u * kHistValThreads < v1);
    slab_count(a, i, 2 * it);
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(i + 2 * kStep + (int64_t)u * kHistValThreads);
#pragma unroll
    for (int u = 0; u < U; ++u) count(b[u], i + kStep + (int64_t)u * kHistValThreads < v1);
    slab_count(b, i + kStep, (2 * it + 1) & 63);  // a past-the-range B batch counts 0 (written, unread)
  }
  if constexpr (MODE == kHvNz) {
    if ((threadIdx.x & 63) < nz.S) slab_w[(threadIdx.x & 63) * 16 + wave] = slab_acc;
  }
  if constexpr (CHUNKED) {
    if (blockIdx.x % ch.bpc == 0 && threadIdx.x == 0 && e1 > e0) {
      // the chunk's cut edge vectors: the head one holding e0 (when e0 is not vector-aligned) and
      // the tail one holding e1 - 1 (when e1 is not, and it is another vector); their halves
      // outside [e0, e1) belong to the neighbouring chunks
      const int64_t hv = e0 / 8, tv = (e1 - 1) / 8;
      for (int64_t vv = hv; vv <= tv; vv += (tv > hv ? tv - hv : 1)) {
        if (vv * 8 >= e0 && vv * 8 + 8 <= e1) continue;  // a whole vector: the hot loop had it
        const uint16_t *h = reinterpret_cast<const uint16_t *>(x + vv * 8);
        for (int j = 0; j < 8; ++j) {
          const int64_t e = vv * 8 + j;
          if (e >= e0 && e < e1) atomicAdd(vh + (h[j] & 0x7FFFu), 1u);
        }
      }
    }
  }
  __syncthreads();
  // fold: pattern -> bin (torch.histc formula, hist_div_kernel's exact division)
  const float fb = (float)bins;
  const float span = hi - lo;
  const float y = 1.f / span;
  const uint32_t last = (uint32_t)bins - 1u;
  // four consecutive patterns per lane (one ds_read_b128, a wave reads 1 KiB contiguous); their
  // bins are non-decreasing, so the counts of equal bins are summed in registers and leave with
  // one LDS atomic per run (0.717 -> 0.747 of the HBM roofline on the bench input with the phi
  // limit above, scripts/exp/hist_exp.hip v41)
  for (int w = threadIdx.x; w < nz4; w += kHistValThreads) {
    const uint4 c4 = reinterpret_cast<const uint4 *>(vh)[w];
    const uint32_t cs[4] = {c4.x, c4.y, c4.z, c4.w};
    uint32_t run_b = 0xFFFFFFFFu, run_c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = 4 * w + j;
      if (cs[j] == 0u || p > phi) continue;
      const uint16_t bits = (uint16_t)p;
      T tv;
      __builtin_memcpy(&tv, &bits, 2);
      const float a = Elem<T>::ld(tv);
      if (!(a <= hi) || (skip_zeros && a == 0.f)) continue;  // NaN patterns fail the compare
      const float t = (a - lo) * fb;
      const float q0 = t * y;
      const float q = __builtin_fmaf(__builtin_fmaf(-q0, span, t), y, q0);
      uint32_t b = (uint32_t)(int)q;
      b = b < last ? b : last;
      if (b != run_b) {
        if (run_c) atomicAdd(bh + run_b, run_c);
        run_b = b;
        run_c = 0;
      }
      run_c += cs[j];
    }
    if (run_c) atomicAdd(bh + run_b, run_c);
  }
  __syncthreads();
  if constexpr (CHUNKED) {
    uint32_t *row = ch.rows + (int64_t)blockIdx.x * bins;
    for (int b = threadIdx.x; b < bins; b += kHistValThreads) __builtin_nontemporal_store(bh[b], row + b);
  } else if constexpr (MODE == kHvNz) {
    uint32_t *row = nz.rows + (int64_t)blockIdx.x * bins;
    for (int b = threadIdx.x; b < bins; b += kHistValThreads) __builtin_nontemporal_store(bh[b], row + b);
    // slab totals, and the workgroup's total through one LDS word (the pattern table is free now)
    if (threadIdx.x == 0) vh[0] = 0u;
    __syncthreads();
    for (int k = threadIdx.x; k < nz.S; k += kHistValThreads) {
      uint32_t t = 0;
#pragma unroll
      for (int w2 = 0; w2 < 16; ++w2) t += slab_w[k * 16 + w2];
      nz.slab_tot[(int64_t)blockIdx.x * nz.S + k] = t;
      atomicAdd(vh, t);
    }
    __syncthreads();
    if (threadIdx.x == 0) nz.wg_tot[blockIdx.x] = vh[0];
  } else {
    for (int b = threadIdx.x; b < bins; b += kHistValThreads)
      if (bh[b]) atomicAdd(counts + b, bh[b]);
  }
}

// skip_zeros: torch.histc counts the compacted non-zero elements, N of them, as
// at::parallel_for chunks: T' = min(T, ceil(N / grain)) threads, chunk = ceil(N / T'), chunk t =
// compacted ranks [t * chunk, (t + 1) * chunk).  r05 found the chunks' first elements on the
// device with a per-tile non-zero pass and one block per boundary (a second full read of the
// input, plus T + 1 blocks each re-summing every tile count); r06 counts in one read (kHvNz
// above) and resolves the boundaries afterwards (hist_nz_recount_kernel, hist_nz_fold_kernel).
constexpr int kNzThreads = 1024;

__device__ __forceinline__ int nz_halves(uint32_t w) {
  return ((w & 0x7FFFu) != 0u) + ((w & 0x7FFF0000u) != 0u);
}

__device__ __forceinline__ int nz_vec(const u32x4 &v) {
  return nz_halves(v.x) + nz_halves(v.y) + nz_halves(v.z) + nz_halves(v.w);
}

// exclusive prefix sum over the block (kNzThreads lanes); *total = the block's sum
__device__ __forceinline__ int64_t block_exscan(int64_t v, int64_t *sh_w, int64_t *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) sh_w[w] = inc;
  __syncthreads();
  int64_t base = 0, tot = 0;
  for (int k = 0; k < kNzThreads / 64; ++k) {
    base += k < w ? sh_w[k] : 0;
    tot += sh_w[k];
  }
  __syncthreads();  // sh_w reusable
  *total = tot;
  return base + inc - v;
}

// hist_nz_recount_kernel: grid (threads - 1) x S, workgroup (b - 1, p) = boundary b, slab p of
// the workgroup range that boundary b falls strictly inside (nothing to do otherwise).  The chunks
// are torch.histc's: N non-zeros (sum of wg_tot), T' = min(threads, ceil(N / grain)), chunk =
// ceil(N / T'), boundary b at compacted rank b * chunk.  Its segment is the non-zeros of that
// workgroup range with ranks in [max(R_w, (b - 1) * chunk), b * chunk) -- the part the range gives
// to chunk b - 1 -- and this workgroup adds the ones in slab p to rec[b].
// int64 block-prefix of the uint32 array v[0, n) into pre[0, n] (pre[n] = total), 1024 threads;
// each thread's contiguous slice is loaded 8 at a time, all 8 loads issued together (one round
// trip for n <= 8192 -- a plain loop over the slice waited for each load in turn, r06j)
__device__ void block_prefix_u32(const uint32_t *v, int64_t n, int64_t *pre, int64_t *sh_w) {
  const int64_t per = (n + kNzThreads - 1) / kNzThreads;
  const int64_t s0 = (int64_t)threadIdx.x * per, s1 = s0 + per < n ? s0 + per : n;
  int64_t mine = 0;
  for (int64_t k0 = s0; k0 < s1; k0 += 8) {
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = v[k0 + k < s1 ? k0 + k : s1 - 1];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k0 + k < s1) {
        pre[k0 + k] = mine;  // exclusive within the slice; the slice offset is added below
        mine += t[k];
      }
    }
  }
  int64_t tot;
  const int64_t off = block_exscan(mine, sh_w, &tot);
  for (int64_t k = s0; k < s1; ++k) pre[k] += off;
  if (threadIdx.x == 0) pre[n] = tot;
  __syncthreads();
}

struct NzChunking {
  int64_t N, teff, chunk;
  double inv;  // 1 / chunk, for chunk_of
};

// floor(r / chunk) without a 64-bit integer division (a ~100-instruction sequence on the GPU: the
// fold ran 15 us with two per workgroup range and lane, r06k): the double quotient is within one
// of it for r < 2^50, corrected by one multiply-compare each way
__device__ __forceinline__ int64_t chunk_of(int64_t r, const NzChunking &c) {
  int64_t q = (int64_t)((double)r * c.inv);
  if (q * c.chunk > r) --q;
  else if ((q + 1) * c.chunk <= r) ++q;
  return q;
}

__device__ __forceinline__ NzChunking nz_chunking(int64_t N, int threads, int64_t grain) {
  NzChunking c;
  c.N = N;
  const int64_t tq = (N + grain - 1) / grain;
  c.teff = (int64_t)threads < tq ? (int64_t)threads : tq;  // 0 when N == 0
  c.chunk = c.teff > 0 ? (N + c.teff - 1) / c.teff : 1;
  c.inv = 1.0 / (double)c.chunk;
  return c;
}

constexpr int kNzSlabVec = (int)kHistValThreads * 2;  // the count kernel's batch (U = 2)

template <typename T>
__global__ __launch_bounds__(kNzThreads) void hist_nz_recount_kernel(const u32x4 *__restrict__ x, int64_t nvec,
                                                                      HistNz nz, int G, int threads, int64_t grain,
                                                                      const float *hmax, int bins) {
  extern __shared__ __attribute__((aligned(16))) int64_t shq[];
  int64_t *R = shq;                    // [G + 1] workgroup rank prefix
  int64_t *Rs = R + G + 1;             // [S + 1] slab rank prefix inside the boundary's workgroup
  int64_t *sh_w = Rs + nz.S + 1;       // [16] scan scratch
  int64_t *sh_misc = sh_w + 16;        // [2]
  uint32_t *bh = reinterpret_cast<uint32_t *>(sh_misc + 2);  // [bins]
  const int b = blockIdx.x + 1, p = blockIdx.y;
  block_prefix_u32(nz.wg_tot, G, R, sh_w);
  const NzChunking ck = nz_chunking(R[G], threads, grain);
  const int64_t target = (int64_t)b * ck.chunk;
  if (b >= ck.teff || target >= ck.N) return;  // block-uniform
  if (threadIdx.x == 0) sh_misc[0] = -1;
  __syncthreads();
  for (int w = threadIdx.x; w < G; w += kNzThreads)
    if (R[w] < target && target < R[w + 1]) sh_misc[0] = w;  // at most one
  __syncthreads();
  const int64_t w = sh_misc[0];
  if (w < 0 || p >= nz.S) return;  // the boundary sits on a workgroup edge: no split
  const int64_t rw = R[w];
  const int64_t rank_lo = rw > target - ck.chunk ? rw : target - ck.chunk, rank_hi = target;
  block_prefix_u32(nz.slab_tot + w * nz.S, nz.S, Rs, sh_w);
  const int64_t s_lo = rw + Rs[p], s_hi = rw + Rs[p + 1];
  if (s_hi <= rank_lo || s_lo >= rank_hi) return;  // no rank of the segment in this slab
  for (int k = threadIdx.x; k < bins; k += kNzThreads) bh[k] = 0u;
  // the slab: vectors [v0, v1); lane l takes vectors v0 + 2l, + 1 (contiguous: ranks in lane order)
  const int64_t v0 = w * nz.vpb + (int64_t)p * kNzSlabVec;
  int64_t v1 = v0 + kNzSlabVec < (w + 1) * nz.vpb ? v0 + kNzSlabVec : (w + 1) * nz.vpb;
  v1 = v1 < nvec ? v1 : nvec;
  u32x4 v[2];
  int c = 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t k = v0 + 2 * (int64_t)threadIdx.x + u;
    v[u] = k < v1 ? x[k] : u32x4{0u, 0u, 0u, 0u};
    c += nz_vec(v[u]);
  }
  int64_t tot;
  int64_t rank = s_lo + block_exscan(c, sh_w, &tot);  // also orders the bh zeroing before the adds
  float lo = 0.f, hi = *hmax;
  if (hi == lo) {
    lo -= 1.f;
    hi += 1.f;
  }
  const float fb = (float)bins, span = hi - lo, y = 1.f / span;
  const uint32_t last = (uint32_t)bins - 1u;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const uint32_t w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const uint16_t bits = (uint16_t)((w4[h / 2] >> (16 * (h % 2))) & 0x7FFFu);
      if (bits == 0) continue;
      const bool in = rank >= rank_lo && rank < rank_hi;
      ++rank;
      T tv;
      __builtin_memcpy(&tv, &bits, 2);
      const float a = Elem<T>::ld(tv);
      if (!in || !(a <= hi)) continue;  // NaN fails the compare
      const float t = (a - lo) * fb;
      const float q0 = t * y;
      const float q = __builtin_fmaf(__builtin_fmaf(-q0, span, t), y, q0);
      uint32_t bn = (uint32_t)(int)q;
      bn = bn < last ? bn : last;
      atomicAdd(bh + bn, 1u);
    }
  }
  __syncthreads();
  uint32_t *rec = nz.rec + (int64_t)b * bins;
  for (int k = threadIdx.x; k < bins; k += kNzThreads)
    if (bh[k]) atomicAdd(rec + k, bh[k]);
}

// hist_nz_fold_kernel: BW bins x 16 lanes per workgroup; lane l of bin b loads the rows of
// workgroup ranges l, l + 16, ... for b -- issued first, together with the boundary rows, before
// the rank prefix is known, so the whole fold is one round trip -- then adds each range's part
// into LDS chunk accumulators (uint32, exact): a range inside one chunk gives its whole row; one
// that boundaries cut gives rec[c + 1] to every chunk c its ranks leave (the segment before the
// boundary) and row - sum of those to its last chunk.  Chunks in groups of 16: clamp at 2^24 and
// add in chunk order in fp32 (torch.histc's thread-order fold), + accum.
constexpr int kNzFoldMaxRec = 16;  // boundary rows staged in LDS per chunk group

template <int BW>
__global__ __launch_bounds__(BW * 16) void hist_nz_fold_kernel(HistNz nz, int G, int threads, int64_t grain,
                                                               int bins, const float *accum, int64_t accum_n,
                                                               float *hist) {  // accum may alias hist
  extern __shared__ __attribute__((aligned(16))) int64_t shq[];
  int64_t *R = shq;                                             // [G + 1]
  int64_t *sh_w = R + G + 1;                                    // [16]
  int64_t *cfl = sh_w + 16;                                     // [G][2] first / last chunk of each range
  uint32_t *acc = reinterpret_cast<uint32_t *>(cfl + 2 * G);    // [16][BW]
  uint32_t *recl = acc + 16 * BW;                               // [kNzFoldMaxRec][BW]
  const int bl = threadIdx.x % BW, gl = threadIdx.x / BW, bn = blockIdx.x * BW + bl;
  const int bnc = bn < bins ? bn : bins - 1;
  // this lane's rows: ranges 16 gl .. 16 gl + 15 (consecutive, so mostly one chunk: summed in a
  // register and added to LDS once per chunk change); G <= 256 in one batch of 16 loads
  const int wl = G <= 256 ? 16 : (G + 15) / 16;  // ranges per lane
  uint32_t v[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int w = gl * wl + k < G ? gl * wl + k : G - 1;
    v[k] = nz.rows[(int64_t)w * bins + bnc];
  }
  // the first group's boundary rows (rec[1 .. 16]) and the range totals, loaded beside the rows:
  // the whole fold waits for one round trip (the totals' scan after the rows' loads made it two)
  const int nrec0 = threads - 1 < 16 ? threads - 1 : 16;
  const uint32_t rec0 = nz.rec[(int64_t)(gl < nrec0 ? gl + 1 : 1) * bins + bnc];
  if (G <= BW * 16) {
    const uint32_t tot = nz.wg_tot[threadIdx.x < G ? threadIdx.x : G - 1];
    if (gl < nrec0) recl[gl * BW + bl] = rec0;
    int64_t all;
    const int64_t ex = block_exscan(threadIdx.x < G ? tot : 0u, sh_w, &all);
    if (threadIdx.x < G) R[threadIdx.x] = ex;
    if (threadIdx.x == 0) R[G] = all;
    __syncthreads();
  } else {
    if (gl < nrec0) recl[gl * BW + bl] = rec0;
    block_prefix_u32(nz.wg_tot, G, R, sh_w);  // also orders the recl stores before their reads
  }
  const NzChunking ck = nz_chunking(R[G], threads, grain);
  // each range's first / last chunk once per workgroup (the same for every bin; -1: no non-zeros)
  for (int w = threadIdx.x; w < G; w += BW * 16) {
    const int64_t rw = R[w], rz = R[w + 1];
    cfl[2 * w] = rz == rw ? -1 : chunk_of(rw, ck);
    cfl[2 * w + 1] = rz == rw ? -1 : chunk_of(rz - 1, ck);
  }
  float h = 0.f;
  for (int64_t g0 = 0; g0 < ck.teff; g0 += 16) {
    const int64_t g1 = g0 + 16 < ck.teff ? g0 + 16 : ck.teff;
    acc[gl * BW + bl] = 0u;
    // boundary rows g0 + 1 .. g1 (rec[c + 1] for the group's chunks), staged in LDS slot (c - g0)
    if (g0 > 0 && g0 + gl + 1 < ck.teff) recl[gl * BW + bl] = nz.rec[(g0 + gl + 1) * bins + bnc];
    __syncthreads();
    int64_t run_c = -1;
    uint32_t run = 0;
    for (int k0 = 0; k0 < wl; k0 += 16) {
      uint32_t vv[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k0 == 0) {
          vv[k] = v[k];
        } else {
          const int w = gl * wl + k0 + k;
          vv[k] = nz.rows[(int64_t)(w < G ? w : G - 1) * bins + bnc];
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int w = gl * wl + k0 + k;
        if (k0 + k >= wl || w >= G) break;
        const int64_t cf = cfl[2 * w], cl = cfl[2 * w + 1];  // first / last chunk of its ranks
        if (cf < 0 || cl < g0 || cf >= g1) continue;  // no non-zeros (an all-zero row), or another group
        if (cf == cl) {
          if (cf != run_c) {
            if (run_c >= 0) atomicAdd(acc + (run_c - g0) * BW + bl, run);
            run_c = cf;
            run = 0;
          }
          run += vv[k];
          continue;
        }
        uint32_t rest = vv[k];
        for (int64_t c = cf; c < cl; ++c) {  // the segment before boundary c + 1 goes to chunk c
          const uint32_t r = (c >= g0 && c < g1) ? recl[(c - g0) * BW + bl] : nz.rec[(c + 1) * bins + bnc];
          rest -= r;
          if (c >= g0 && c < g1) atomicAdd(acc + (c - g0) * BW + bl, r);
        }
        if (cl < g1) atomicAdd(acc + (cl - g0) * BW + bl, rest);
      }
    }
    if (run_c >= 0) atomicAdd(acc + (run_c - g0) * BW + bl, run);
    __syncthreads();
    if (gl == 0 && bn < bins)
      for (int64_t c = g0; c < g1; ++c) h += fminf((float)acc[(c - g0) * BW + bl], 16777216.f);
    __syncthreads();
  }
  if (gl == 0 && bn < bins) {
    if (bn < accum_n) h += accum[bn];
    hist[bn] = h;
  }
}

// hist[b] = accum[b] (b < accum_n) or 0: an empty call's result
__global__ void hist_fill_kernel(const float *accum, int64_t accum_n, int bins, float *hist) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < bins) hist[b] = b < accum_n ? accum[b] : 0.f;
}

// ============================================================================================
// AWQ-lite search helpers: column scale (x * s[col]) and the per-alpha MSE loss
// ============================================================================================
// y = T(x * s[col]) -- the reference's `inputs * pre_quant_scale` (fp32 product, one rounding).
template <typename T>
__global__ __launch_bounds__(kThreads) void mul_cols_kernel(const T *__restrict__ x,
                                                             const T *__restrict__ sc,
                                                             T *__restrict__ y, int64_t nvec,
                                                             int64_t cols) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nvec) return;
  V v = ldg_vec_nt(x + i * N);
  const int64_t c0 = (i * N) % cols;  // cols % N == 0: a vector never straddles rows
  V s = ldg_vec(sc + c0);
#pragma unroll
  for (int j = 0; j < N; ++j) v.e[j] = Elem<T>::st(Elem<T>::ld(v.e[j]) * Elem<T>::ld(s.e[j]));
  stg_vec_nt(y + i * N, v);
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// loss[0] += sum(float(T(a - b))^2) / n -- `(out - out_act).float().pow(2).mean()`
// (model_calib.py:1494) in one read of a and b.  Deterministic: the grid depends only on n and
// the CU count, each block stores its partial, and the last block to finish (agent-scope
// counter in workspace[0]) sums the partials in block order in double, then resets the counter.
constexpr int kMseU = 4;
constexpr int kMseThreads = 1024;
template <typename T>
__global__ __launch_bounds__(kMseThreads) void mse_kernel(const T *__restrict__ a,
                                                           const T *__restrict__ b, int64_t n,
                                                           int64_t nvec, unsigned *counter,
                                                           float *partials, float *loss) {
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int64_t CH = (int64_t)kMseThreads * kMseU;
  float acc = 0.f;
  for (int64_t c0 = (int64_t)blockIdx.x * CH; c0 < nvec; c0 += (int64_t)gridDim.x * CH) {
    V va[kMseU], vb[kMseU];
#pragma unroll
    for (int u = 0; u < kMseU; ++u) {
      const int64_t i = c0 + u * kMseThreads + threadIdx.x;
      if (i < nvec) {
        va[u] = ldg_vec_nt(a + i * N);
        vb[u] = ldg_vec_nt(b + i * N);
      }
    }
#pragma unroll
    for (int u = 0; u < kMseU; ++u) {
      const int64_t i = c0 + u * kMseThreads + threadIdx.x;
      if (i < nvec) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          float d = Elem<T>::ld(Elem<T>::st(Elem<T>::ld(va[u].e[j]) - Elem<T>::ld(vb[u].e[j])));
          acc += d * d;
        }
      }
    }
  }
  if (blockIdx.x == gridDim.x - 1) {
    for (int64_t t = nvec * N + threadIdx.x; t < n; t += kMseThreads) {
      float d = Elem<T>::ld(Elem<T>::st(Elem<T>::ld(a[t]) - Elem<T>::ld(b[t])));
      acc += d * d;
    }
  }
  __shared__ float red[kMseThreads / 64];
  __shared__ bool last;
  acc = wave_sum_f(acc);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float bs = 0.f;
#pragma unroll
    for (int k = 0; k < kMseThreads / 64; ++k) bs += red[k];
    __hip_atomic_store(partials + blockIdx.x, bs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned done = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = done == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (unsigned k = 0; k < gridDim.x; ++k)
      tot += (double)__hip_atomic_load(partials + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    loss[0] += (float)(tot / (double)n);
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int64_t mse_grid(int64_t n, int dtype) {
  const int N = dtype == MTQ_F32 ? 4 : 8;
  int64_t blocks = (n / N + (int64_t)kMseThreads * kMseU - 1) / ((int64_t)kMseThreads * kMseU);
  const int64_t cap = (int64_t)num_cus() * 2;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  return blocks;
}


// ============================================================================================
// NVFP4 two-level dynamic block fake quant (the reference's primary NVFP4 kernel,
// kernels/quantization/gemm/fp4_kernel_hopper.py:33-160 + common/nvfp4_quant.py)
// ============================================================================================
// gs = RN(global_amax / 2688) (1e-12 when not > 0); per block of BS along the last dim:
// s8 = min(RN(bmax / RN(6 gs)), 448); q = fp32(e4m3_rne(s8)) * gs (1 when < 1e-5);
// y = sign(x) * e2m1(RN(|x| / q)) * q, E2M1 = round-to-nearest-even on {0,.5,1,1.5,2,3,4,6},
// saturating (NaN -> 6 like the reference's comparison chain).  Divisions are correctly rounded
// (Markstein on RN(1/q)), as the reference's fp32 `/` is.
struct Nvfp4Block {
  float q, r;  // block scale and RN(1/q)
};

__device__ __forceinline__ Nvfp4Block nvfp4_block(float bmax, float gs) {
  const float six_gs = 6.0f * gs;
  float s8 = div_rn(bmax, six_gs, 1.0f / six_gs);
  s8 = s8 < 448.0f ? s8 : 448.0f;  // NaN -> 448 (tl.minimum returns the non-NaN operand)
  const int p = __builtin_amdgcn_cvt_pk_fp8_f32(s8, s8, 0, false);
  float q = __builtin_amdgcn_cvt_f32_fp8(p, 0) * gs;
  q = q >= 1e-5f ? q : 1.0f;
  return {q, 1.0f / q};
}

__device__ __forceinline__ float nvfp4_qdq(float x, const Nvfp4Block &b) {
  const float a = div_rn(fabsf(x), b.q, b.r);
  const float c = round_table(a, TableFmt{1, 0, 6.0f, false}) * b.q;
  return x >= 0.f ? c : -c;
}

__device__ __forceinline__ float nvfp4_global_scale(const float *gamax) {
  const float g = *gamax;
  const float gs = div_rn(g, 2688.0f, 1.0f / 2688.0f);
  return gs > 0.f ? gs : 1e-12f;
}

template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void nvfp4_vec_kernel(const T *__restrict__ x,
                                                              T *__restrict__ y, int64_t nvec,
                                                              const float *__restrict__ gamax) {
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int LPB = BS / N;
  static_assert(BS % N == 0, "block must be a multiple of the vector");
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i - (threadIdx.x % LPB) >= nvec) return;
  const float gs = nvfp4_global_scale(gamax);
  V v = ldg_vec_nt(x + i * N);
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) m = max_skip_nan(m, fabsf(Elem<T>::ld(v.e[j])));
  m = group_max_f<LPB>(m);
  const Nvfp4Block b = nvfp4_block(m, gs);
#pragma unroll
  for (int j = 0; j < N; ++j) v.e[j] = Elem<T>::st(nvfp4_qdq(Elem<T>::ld(v.e[j]), b));
  stg_vec_nt(y + i * N, v);
}

// NVFP4 on 16-bit inputs with the native E2M1 converts: per element a = RN(x / q) (signed,
// Markstein as nvfp4_qdq), the pair rounded to E2M1 by one v_cvt_scalef32_pk_fp4_f32 (scale 1)
// and widened back by one v_cvt_scalef32_pk_f32_fp4, times q.  Symmetric rounding makes the
// signed form equal to the reference's sign(x) * e2m1(|x| / q) * q except for x = -0 and NaN
// (mtq_device.hpp Fp4Native): blocks with a NaN and lanes with a -0 take nvfp4_qdq.
// U = 2 vectors per lane, both loads issued before the first block is converted, the per-thread
// constants (global scale, its 6x reciprocal) paid once per U vectors: 0.755-0.760 -> 0.772-0.774
// of the HBM roofline over one vector per lane, U = 4 slower (profiles/r03/nvfp4).
template <typename T, int BS, int U, int TPB = kThreads>
__global__ __launch_bounds__(TPB) void nvfp4_native_u_kernel(const T *__restrict__ x,
                                                              T *__restrict__ y, int64_t nvec,
                                                              const float *__restrict__ gamax) {
  using V = Vec<T>;
  constexpr int N = V::N;
  static_assert(N == 8 && BS % N == 0, "16-bit elements, block a multiple of the vector");
  constexpr int LPB = BS / N;
  const int64_t base = (int64_t)blockIdx.x * (TPB * U) + threadIdx.x;
  const int lead = threadIdx.x % LPB;  // a block's LPB lanes are in range together
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * TPB - lead < nvec) v[u] = ldg_vec_nt(x + (base + u * TPB) * N);
  const float gs = nvfp4_global_scale(gamax);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * TPB;
    if (i - lead >= nvec) continue;
    uint32_t w[4] = {v[u].raw.x, v[u].raw.y, v[u].raw.z, v[u].raw.w};
    const PairScan sc = scan_pairs(w);
    const uint32_t mb = group_max_u32<LPB>(sc.max_abs);
    const bool block_nan = mb > Fp4Native<T>::kInfBits;
    float bmax;
    if (!block_nan) {
      bmax = half_bits_to_float<T>(mb);
    } else {
      float m = 0.f;
#pragma unroll
      for (int j = 0; j < N; ++j) m = max_skip_nan(m, fabsf(Elem<T>::ld(v[u].e[j])));
      bmax = group_max_f<LPB>(m);
    }
    const Nvfp4Block b = nvfp4_block(bmax, gs);
    if (!block_nan && !sc.neg_zero) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a0 = div_rn(Elem<T>::ld(v[u].e[2 * j]), b.q, b.r);
        const float a1 = div_rn(Elem<T>::ld(v[u].e[2 * j + 1]), b.q, b.r);
        const uint32_t c = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, a0, a1, 1.0f, 0);
        const auto r = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(c, 1.0f, 0);
        v[u].e[2 * j] = Elem<T>::st(r[0] * b.q);
        v[u].e[2 * j + 1] = Elem<T>::st(r[1] * b.q);
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) v[u].e[j] = Elem<T>::st(nvfp4_qdq(Elem<T>::ld(v[u].e[j]), b));
    }
    stg_vec_nt(y + i * N, v[u]);
  }
}

// any shape: one lane per element of the zero-padded [rows, pcols] matrix, BS lanes per block
template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void nvfp4_scalar_kernel(const T *__restrict__ x,
                                                                 T *__restrict__ y, int64_t rows,
                                                                 int64_t cols, int64_t pcols,
                                                                 const float *__restrict__ gamax) {
  const float gs = nvfp4_global_scale(gamax);
  const int64_t total = rows * pcols;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t idx = (int64_t)blockIdx.x * kThreads + threadIdx.x; idx - (threadIdx.x % BS) < total;
       idx += stride) {
    const bool live = idx < total;
    const int64_t row = live ? idx / pcols : 0;
    const int64_t col = live ? idx - row * pcols : 0;
    const bool real = live && col < cols;
    const float v = real ? Elem<T>::ld(x[row * cols + col]) : 0.f;
    const float m = group_max_f<BS>(abs_or_zero(v));
    if (!real) continue;
    y[row * cols + col] = Elem<T>::st(nvfp4_qdq(v, nvfp4_block(m, gs)));
  }
}

template <typename T, int BS>
int launch_nvfp4(const T *x, T *y, int64_t rows, int64_t cols, const float *gamax,
                 hipStream_t stream) {
  constexpr int N = Vec<T>::N;
  if (cols % BS == 0 && BS % N == 0 && aligned16(x) && aligned16(y)) {
    const int64_t nvec = rows * cols / N;
    const unsigned g = (unsigned)((nvec + kThreads - 1) / kThreads);
    if constexpr (sizeof(T) == 2) {
      count_dispatch(kDispNvfp4NativeU);
      nvfp4_native_u_kernel<T, BS, 2><<<(unsigned)((nvec + 2 * kThreads - 1) / (2 * kThreads)), kThreads, 0,
                                        stream>>>(x, y, nvec, gamax);
      return check_launch();
    }
    nvfp4_vec_kernel<T, BS><<<g, kThreads, 0, stream>>>(x, y, nvec, gamax);
  } else {
    const int64_t pcols = (cols + BS - 1) / BS * BS;
    nvfp4_scalar_kernel<T, BS><<<grid_for(rows * pcols, kThreads), kThreads, 0, stream>>>(
        x, y, rows, cols, pcols, gamax);
  }
  return check_launch();
}


// Static NVFP4 element pass with precomputed per-block scales (static_blockwise_fp4_fake_quant
// kernel, kernels/quantization/gemm/fp4_kernel.py:193-214 -> nvfp4_scalar_quant,
// common/nvfp4_quant.py): scale 0 -> block of +0; NaN/inf scale -> 1; y = sign * e2m1(|x|/s) * s.
template <typename T>
__global__ __launch_bounds__(kThreads) void fp4_scaled_vec_kernel(const T *__restrict__ x,
                                                                   T *__restrict__ y,
                                                                   const float *__restrict__ sc,
                                                                   int64_t nvec, int block) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= nvec) return;
  V v = ldg_vec_nt(x + i * N);
  const float s = sc[(i * N) / block];  // block % N == 0: one scale per vector
  const bool zero = s == 0.f;
  const float ss = (zero || s != s || __builtin_isinf(s)) ? 1.0f : s;
  const Nvfp4Block b{ss, 1.0f / ss};
#pragma unroll
  for (int j = 0; j < N; ++j)
    v.e[j] = Elem<T>::st(zero ? 0.0f : nvfp4_qdq(Elem<T>::ld(v.e[j]), b));
  stg_vec_nt(y + i * N, v);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void fp4_scaled_scalar_kernel(const T *__restrict__ x,
                                                                      T *__restrict__ y,
                                                                      const float *__restrict__ sc,
                                                                      int64_t n, int block) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float s = sc[i / block];
    const bool zero = s == 0.f;
    const float ss = (zero || s != s || __builtin_isinf(s)) ? 1.0f : s;
    y[i] = Elem<T>::st(zero ? 0.0f : nvfp4_qdq(Elem<T>::ld(x[i]), Nvfp4Block{ss, 1.0f / ss}));
  }
}


// ============================================================================================
// Real-quant packing for checkpoint export (export/quant_utils.py to_quantized_weight and the
// qtensor quantize() routines).  All HBM-bound byte work: one read of the weight, one write of
// the packed bytes.
// ============================================================================================
// torch float -> float8_e4m3fn byte: RNE, |v| > 464 or NaN/inf -> NaN (0x7F | sign); the
// 448..464 band rounds to 448.
__device__ __forceinline__ uint32_t e4m3_byte(float v) {
  const uint32_t sign = (__float_as_uint(v) >> 24) & 0x80u;
  if (v != v || fabsf(v) > 464.0f) return 0x7Fu | sign;
  const float c = v > 448.f ? 448.f : (v < -448.f ? -448.f : v);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(c, c, 0, false) & 0xFFu;
}

// A NaN weight keeps its sign through the reference's division and its dtype re-rounding (torch
// CPU), where the device's bf16 round trip makes the NaN positive: the e4m3 NaN byte takes the
// weight's sign bit.
// The sign comes from the raw element bits: the widening convert of a 16-bit NaN does not keep it.
template <typename T> __device__ __forceinline__ uint32_t nan_sign_byte(T x) {
  const float f = Elem<T>::ld(x);
  if constexpr (sizeof(T) == 2)
    return f != f ? (uint32_t)(__builtin_bit_cast(uint16_t, x) >> 8) & 0x80u : 0u;
  else
    return f != f ? (__float_as_uint(f) >> 24) & 0x80u : 0u;
}

// weight / scale -> e4m3 bytes.  per_row: scale[row] (the division then happens in fp32, as torch
// promotes bf16 / fp32[rows, 1] to fp32); per-tensor: scale[0] and, with round_dtype, the quotient
// is first rounded to the weight dtype (torch keeps bf16 / 0-dim fp32 in bf16).
template <typename T>
__global__ __launch_bounds__(kThreads) void export_fp8_kernel(const T *__restrict__ x,
                                                               uint8_t *__restrict__ y, int64_t n,
                                                               int64_t cols,
                                                               const float *__restrict__ scale,
                                                               int per_row, int round_dtype) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const float s = scale[per_row ? i / cols : 0];
    const float xv = Elem<T>::ld(x[i]);
    float q = div_rn(xv, s, 1.0f / s);
    if (round_dtype) q = Elem<T>::ld(Elem<T>::st(q));
    y[i] = (uint8_t)(e4m3_byte(q) | nan_sign_byte(x[i]));
  }
}

// INT4 AWQ: q = clamp(rint(w / scale[row, col / block]), -8, 7); two consecutive ROWS share a
// byte (low nibble = even row): y[r/2, c] (pack_int4_in_uint8, export/quant_utils.py:792-833).
template <typename T>
__global__ __launch_bounds__(kThreads) void export_int4_kernel(const T *__restrict__ x,
                                                                uint8_t *__restrict__ y,
                                                                int64_t prow_count, int64_t cols,
                                                                const float *__restrict__ scale,
                                                                int64_t nblk, int block) {
  const int64_t n = prow_count * cols;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n; i += stride) {
    const int64_t pr = i / cols, c = i - pr * cols;
    uint32_t out = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t r = 2 * pr + h;
      const float s = scale[r * nblk + c / block];
      float q = __builtin_rintf(Elem<T>::ld(x[r * cols + c]) / s);  // IEEE: any s, +-inf
      q = q < -8.f ? -8.f : (q > 7.f ? 7.f : q);  // NaN stays NaN -> int8 cast below
      const int v = q != q ? 0 : (int)q;
      out |= ((uint32_t)v & 0xFu) << (4 * h);
    }
    y[i] = (uint8_t)out;
  }
}

// E2M1 code (sign << 3 | magnitude index) the way NVFP4QTensor._cast_fp4 computes it:
// searchsorted(right=False) over the midpoints + 1 on the odd midpoints (ties to even index);
// NaN -> 7, the sign bit from (v < 0).
__device__ __forceinline__ uint32_t nvfp4_code(float q) {
  const float a = fabsf(q);
  uint32_t ord;
  if (a != a) {
    ord = 7;
  } else {
    ord = (a > 0.25f) + (a > 0.75f) + (a > 1.25f) + (a > 1.75f) + (a > 2.5f) + (a > 3.5f) + (a > 5.0f);
    ord += (a == 0.75f) | (a == 1.75f) | (a == 3.5f);
  }
  return ((q < 0.f) ? 8u : 0u) + ord;
}

// NVFP4QTensor.quantize (qtensor/nvfp4_tensor.py:253-342): q = w / (fp32(scale_fp8[blk]) * s2),
// packed two per byte along the last dim (low nibble = even column).
template <typename T>
__global__ __launch_bounds__(kThreads) void export_nvfp4_kernel(const T *__restrict__ x,
                                                                 uint8_t *__restrict__ y,
                                                                 int64_t npairs, int64_t cols,
                                                                 const float *__restrict__ sblk,
                                                                 const float *__restrict__ s2,
                                                                 int block) {
  const float g = *s2;
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  const int64_t nb_row = cols / block;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < npairs; i += stride) {
    const int64_t e0 = 2 * i;
    const int64_t row = e0 / cols, c = e0 - row * cols;  // cols even: a pair never straddles rows
    const float d = sblk[row * nb_row + c / block] * g;
    const uint32_t lo = nvfp4_code(Elem<T>::ld(x[e0]) / d);  // IEEE: any d, +-inf
    const uint32_t hi = nvfp4_code(Elem<T>::ld(x[e0 + 1]) / d);
    y[i] = (uint8_t)(lo | (hi << 4));
  }
}

// ceil(max(log2(d), -127)) with log2 correctly rounded to fp32 (what torch.log2 gives): exact from
// the exponent bits unless the significand is within 2^-10 of a power of two, where the rounding
// of log2 can land on the integer -- only then is a double log2 taken.
__device__ __forceinline__ float mx_e8m0_exponent(float d) {
  const uint32_t b = __float_as_uint(d);
  const uint32_t m = b & 0x7fffffu;
  // positive normal d with m == 0 (log2 exact) or m > 64 (log2(d) = ex + log2(1 + m 2^-23) rounds
  // above ex for every such m; the largest m that rounds back to ex is 22: scripts/check_e8m0.c,
  // exhaustive): ceil = ex + (m != 0), one test and no nested branches -- all but 1 block in 2^17
  if ((b >> 23) - 1u < 0xFEu && (m == 0u || m > 64u)) return (float)((int)(b >> 23) - 127 + (m != 0u ? 1 : 0));
  if (d != d) return d;
  if (!(d > 0.f)) return -127.f;
  const float e = __builtin_ceilf((float)log2((double)d));  // subnormal d, or 0 < m <= 64
  return e > -127.f ? e : -127.f;
}

// MXFP4QTensor.quantize (qtensor/mxfp4_tensor.py:38-81): per block of `block` along the flat
// tensor, e = ceil(max(log2(amax / 6), -127)) (log2 correctly rounded to fp32), q = w / 2^e,
// code = #(bounds < |q|) (ties toward zero) + 8 * (sign(q) <= 0) -- zero encodes with the sign bit
// set, as torch.sign gives 0 there; bytes pack (even, odd) into (low, high); scale byte e + 127.
template <typename T>
__global__ __launch_bounds__(kThreads) void export_mxfp4_kernel(const T *__restrict__ x,
                                                                 uint8_t *__restrict__ y,
                                                                 uint8_t *__restrict__ sc,
                                                                 int64_t nblocks, int block) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  for (int64_t b = (int64_t)blockIdx.x * kThreads + threadIdx.x; b < nblocks; b += stride) {
    const T *xb = x + b * block;
    float amax = 0.f;
    for (int k = 0; k < block; ++k) {
      const float a = fabsf(Elem<T>::ld(xb[k]));
      amax = (a > amax || a != a) ? a : amax;  // torch.max propagates NaN
    }
    const float e = mx_e8m0_exponent(amax / 6.0f);
    sc[b] = (uint8_t)(int)(e + 127.f);
    const float p = (e == e) ? exp2f(e) : e;
    for (int k = 0; k < block; k += 2) {
      uint32_t code[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float q = Elem<T>::ld(xb[k + h]) / p;
        const float a = fabsf(q);
        const uint32_t ord = (a > 0.25f) + (a > 0.75f) + (a > 1.25f) + (a > 1.75f) + (a > 2.5f) +
                             (a > 3.5f) + (a > 5.0f);
        const uint32_t sb = (q > 0.f) ? 0u : 1u;  // sign(q) in {1, 0, -1, NaN}: (2 - sign) // 2
        code[h] = sb * 8u + ord;
      }
      y[(b * block + k) / 2] = (uint8_t)((code[0] & 0xFFu) + ((code[1] << 4) & 0xFFu));
    }
  }
}


// ---- vectorised export packing (one 16 B input vector per lane, chunked non-temporal) --------
// Index math: with IDX32 (every vector index < 2^31, true for any single weight up to 16 G
// elements of bf16) the row / block of a vector comes from a 32-bit multiply-high divider
// (make_fastdiv) instead of a 64-bit division (~40 VALU ops per lane); packed bytes go out with
// non-temporal stores like the fake-quant kernels' outputs.
typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st_packed_nt(uint8_t *p, uint32_t o) {
  __builtin_nontemporal_store(o, reinterpret_cast<uint32_t *>(p));
}
__device__ __forceinline__ void st_packed_nt(uint8_t *p, uint16_t o) {
  __builtin_nontemporal_store(o, reinterpret_cast<uint16_t *>(p));
}
__device__ __forceinline__ void st_packed_nt(uint8_t *p, uint32_t lo, uint32_t hi) {
  u32x2_t o = {lo, hi};
  __builtin_nontemporal_store(o, reinterpret_cast<u32x2_t *>(p));
}

template <bool IDX32>
__device__ __forceinline__ int64_t idx_div(int64_t n, int64_t d, const FastDiv &f) {
  if constexpr (IDX32)
    return (int64_t)fdiv((uint32_t)n, f);
  else
    return n / d;
}

// Native fast paths of the packers (`native` kernel argument, always 1 from the launchers; 0 =
// the emulated conversions only, the r01 packers): each lane first converts its vector with the gfx950 converts and a handful of
// VALU ops, checks the few inputs where the converter and the reference disagree, and only a lane
// that holds one of those redoes the vector on the exact emulated path above.  The emulated path
// costs ~25 VALU ops per element (seven threshold compares per E2M1 code), which made the packers
// VALU-bound at 38-52 % of the HBM roofline.

// E2M1 codes of two fp32 values through v_cvt_scalef32_pk_fp4_f32: x / 2^e(s), round to nearest
// with ties to the even code, saturating at +-6, -0 -> 8, NaN -> 7 | sign
// (profiles/r02/fp4_convert_probe.txt).
__device__ __forceinline__ uint32_t fp4_pair_hw(float a, float b, float s) {
  return __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, a, b, s, 0) & 0xFFu;
}

// correctly rounded q / s (div_rn) with a zero quotient always +0: the fma's own -0 from a
// negative underflow becomes +0 through the `+ 0.0f` (RN: -0 + +0 = +0), which is what the
// NVFP4 packer's sign rule (q < 0) gives for both zeros.
__device__ __forceinline__ float div_rn_pz(float q, float s, float r) {
  const float y0 = q * r;
  const float e = __builtin_fmaf(-y0, s, q);
  return __builtin_fmaf(e, r, y0) + 0.0f;
}

// div_rn on a pair through the packed fp32 ALU (v_pk_mul_f32 / v_pk_fma_f32: two lanes' worth of
// work per issue), and the pair's dtype re-rounding (bf16: one v_cvt_pk_bf16_f32).
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2_t div_rn2(f32x2_t q, float s, float r) {
  const f32x2_t sv = {s, s}, rv = {r, r};
  const f32x2_t y0 = q * rv;
  const f32x2_t e = __builtin_elementwise_fma(-y0, sv, q);
  const f32x2_t y = __builtin_elementwise_fma(e, rv, y0);
  return (f32x2_t){__builtin_copysignf(y.x, q.x), __builtin_copysignf(y.y, q.y)};
}
template <typename T> __device__ __forceinline__ f32x2_t round_pair(f32x2_t d) {
  if constexpr (std::is_same_v<T, __bf16>) {
    return __builtin_convertvector(__builtin_convertvector(d, bf16x2_t), f32x2_t);
  } else {
    return (f32x2_t){Elem<T>::ld(Elem<T>::st(d.x)), Elem<T>::ld(Elem<T>::st(d.y))};
  }
}

template <typename T>
__device__ __forceinline__ void export_fp8_pack_store(int64_t i, const Vec<T> &v, uint8_t *__restrict__ y, float s,
                                                      int round_dtype, int native);
template <typename T, bool IDX32>
__device__ __forceinline__ void export_fp8_vec_one(int64_t i, const T *__restrict__ x,
                                                                   uint8_t *__restrict__ y,
                                                                   int64_t nvec, int64_t cv,
                                                                   FastDiv fcv,
                                                                   const float *__restrict__ scale,
                                                                   int per_row, int round_dtype,
                                                                   int native, float s_t) {
  using V = Vec<T>;
  constexpr int N = V::N;
  if (i >= nvec) return;
  V v = ldg_vec_nt(x + i * N);
  // per-tensor: the scalar-loaded s_t (no per-lane load and its latency before the division)
  const float s = per_row ? scale[idx_div<IDX32>(i, cv, fcv)] : s_t;
  export_fp8_pack_store<T>(i, v, y, s, round_dtype, native);
}

// the E4M3 bytes of vector i of x (loaded in v) divided by s, stored at y + i * N: the packed RNE
// convert where every quotient of the vector is within +-448, the exact per-element path otherwise
template <typename T>
__device__ __forceinline__ void export_fp8_pack_store(int64_t i, const Vec<T> &v, uint8_t *__restrict__ y, float s,
                                                      int round_dtype, int native) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const float r = 1.0f / s;
  uint32_t b[N];
  if (native) {
    // |q| <= 448 (NaN fails the test): the packed RNE convert needs no clamp and no NaN patch, two
    // bytes per v_cvt_pk_fp8_f32.  Lanes with an overflow / NaN quotient take the exact path.
    float q[N];
    bool inrange = true;
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      f32x2_t d = div_rn2((f32x2_t){Elem<T>::ld(v.e[j]), Elem<T>::ld(v.e[j + 1])}, s, r);
      if (round_dtype) d = round_pair<T>(d);
      q[j] = d.x;
      q[j + 1] = d.y;
      inrange &= (fabsf(d.x) <= kE4M3Max) & (fabsf(d.y) <= kE4M3Max);
    }
    if (inrange) {
      uint32_t w[N / 4];
#pragma unroll
      for (int k = 0; k < N / 4; ++k) {
        int p = __builtin_amdgcn_cvt_pk_fp8_f32(q[4 * k], q[4 * k + 1], 0, false);
        w[k] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(q[4 * k + 2], q[4 * k + 3], p, true);
      }
      if constexpr (N == 8)
        st_packed_nt(y + i * N, w[0], w[1]);
      else
        st_packed_nt(y + i * N, w[0]);
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float xv = Elem<T>::ld(v.e[j]);
    float q = div_rn(xv, s, r);
    if (round_dtype) q = Elem<T>::ld(Elem<T>::st(q));
    b[j] = e4m3_byte(q) | nan_sign_byte(v.e[j]);
  }
  if constexpr (N == 8)
    st_packed_nt(y + i * N, b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24),
                 b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24));
  else
    st_packed_nt(y + i * N, (uint32_t)(b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)));
}

// two INT4 codes (rows 2p, 2p+1) of quotients: rint, clamp to [-8, 7], NaN -> 0 (int8 cast)
__device__ __forceinline__ uint32_t int4_pair(float d0, float d1) {
  float q0 = __builtin_rintf(d0), q1 = __builtin_rintf(d1);
  q0 = q0 < -8.f ? -8.f : (q0 > 7.f ? 7.f : q0);
  q1 = q1 < -8.f ? -8.f : (q1 > 7.f ? 7.f : q1);
  const int v0 = q0 != q0 ? 0 : (int)q0, v1 = q1 != q1 ? 0 : (int)q1;
  return ((uint32_t)v0 & 0xFu) | (((uint32_t)v1 & 0xFu) << 4);
}
// one INT4 code from a div_rn quotient d of weight x: a NaN d with a non-NaN x is an overflowing
// or infinite IEEE quotient, i.e. the clamp bound on x's side
__device__ __forceinline__ uint32_t int4_pair_nan(float d, float x) {
  float q = __builtin_rintf(d);
  q = q < -8.f ? -8.f : (q > 7.f ? 7.f : q);
  const int v = q == q ? (int)q : (x != x ? 0 : (x < 0.f ? -8 : 7));
  return (uint32_t)v & 0xFu;
}

// rows (2p, 2p+1) x N columns -> N bytes, in two phases so a thread's U vector pairs are all
// loaded before the first is packed (r05: with load and pack in one function per vector, the
// second pair's loads were issued only after the first pair's store)
template <typename T>
struct Int4Pair {
  Vec<T> lo, hi;
  float s0, s1;
  int64_t out;  // byte offset of the N packed bytes
};
template <typename T, bool IDX32>
__device__ __forceinline__ Int4Pair<T> export_int4_load(int64_t i, const T *__restrict__ x, int64_t cols,
                                                        FastDiv fcv, FastDiv fblk, const float *__restrict__ scale,
                                                        int64_t nblk, int block) {
  constexpr int N = Vec<T>::N;
  const int64_t cv = cols / N;
  const int64_t pr = idx_div<IDX32>(i, cv, fcv), c0 = (i - pr * cv) * N;
  Int4Pair<T> q;
  q.lo = ldg_vec_nt(x + (2 * pr) * cols + c0);
  q.hi = ldg_vec_nt(x + (2 * pr + 1) * cols + c0);
  const int64_t cb = idx_div<IDX32>(c0, block, fblk);
  q.s0 = scale[(2 * pr) * nblk + cb];
  q.s1 = scale[(2 * pr + 1) * nblk + cb];
  q.out = pr * cols + c0;
  return q;
}
template <typename T>
__device__ __forceinline__ void export_int4_pack(const Int4Pair<T> &q, uint8_t *__restrict__ y) {
  using V = Vec<T>;
  constexpr int N = V::N;
  const V &lo = q.lo, &hi = q.hi;
  const float s0 = q.s0, s1 = q.s1;
  const float r0 = 1.0f / s0, r1 = 1.0f / s1;
  // div_rn is the IEEE quotient except where that quotient overflows or is infinite (div_rn
  // gives NaN there, IEEE +-inf -> the clamp's -8 / 7, selected from the weight's sign) and where
  // 1/s is not finite (a zero, subnormal or non-finite scale: that lane, rare and uniform over its
  // vector, repacks with the IEEE division operator).
  uint32_t b[N];
  constexpr float kInf = __builtin_huge_valf();
  if (__builtin_expect(r0 < kInf && r1 < kInf && s0 < kInf && s1 < kInf, 1)) {
    // the (row 2p, row 2p+1) pair of column j on the packed ALU: div_rn of both quotients per
    // v_pk_mul / v_pk_fma (no copysign: a -0 quotient packs as 0 like +0), clamp to [-8, 7] by
    // v_med3_f32 (clamping before rounding is the same: the bounds are integers), then
    // RN-to-integer and the two's-complement nibble at once: q + 1.5 * 2^23 has ulp 1, so its low
    // mantissa bits ARE rint(q) mod 2^22 (one v_pk_add_f32 for the pair).  A NaN quotient (an
    // infinite weight, an overflowing quotient, a NaN weight) sends the lane to int4_pair_nan.
    const f32x2_t sv = {s0, s1}, rv = {r0, r1}, magic = {12582912.0f, 12582912.0f};
    f32x2_t d[N];
    bool nan = false;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const f32x2_t q = {Elem<T>::ld(lo.e[j]), Elem<T>::ld(hi.e[j])};
      const f32x2_t y0 = q * rv;
      const f32x2_t e = __builtin_elementwise_fma(-y0, sv, q);
      d[j] = __builtin_elementwise_fma(e, rv, y0);
      nan |= (d[j].x != d[j].x) | (d[j].y != d[j].y);
    }
    if (!nan) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const f32x2_t c = {__builtin_amdgcn_fmed3f(d[j].x, -8.f, 7.f), __builtin_amdgcn_fmed3f(d[j].y, -8.f, 7.f)};
        const f32x2_t t = c + magic;
        b[j] = (__float_as_uint(t.x) & 0xFu) | ((__float_as_uint(t.y) << 4) & 0xF0u);
      }
    } else {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const float x0 = Elem<T>::ld(lo.e[j]), x1 = Elem<T>::ld(hi.e[j]);
        b[j] = int4_pair_nan(d[j].x, x0) | (int4_pair_nan(d[j].y, x1) << 4);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j)
      b[j] = int4_pair(Elem<T>::ld(lo.e[j]) / s0, Elem<T>::ld(hi.e[j]) / s1);
  }
  if constexpr (N == 8)
    st_packed_nt(y + q.out, b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24),
                 b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24));
  else
    st_packed_nt(y + q.out, (uint32_t)(b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)));
}

// one 16 B vector (N elements of one block) -> N/2 bytes
template <typename T, bool IDX32>
__device__ __forceinline__ void export_nvfp4_vec_one(int64_t i, const T *__restrict__ x,
                                                                     uint8_t *__restrict__ y,
                                                                     int64_t nvec, int64_t vpb,
                                                                     FastDiv fvpb,
                                                                     const float *__restrict__ sblk,
                                                                     const float *__restrict__ s2,
                                                                     int native) {
  using V = Vec<T>;
  constexpr int N = V::N;
  if (i >= nvec) return;
  V v = ldg_vec_nt(x + i * N);
  const float d = sblk[idx_div<IDX32>(i, vpb, fvpb)] * (*s2);
  const float r = 1.0f / d;
  uint32_t o = 0;
  // Native: the converter's ties-to-even-code rounding with saturation is the reference's
  // searchsorted + odd-bound adjustment (nvfp4_tensor.py:230-250) for every finite q and +-inf;
  // -0 is made +0 by div_rn_pz, and a NaN quotient (or a non-positive / non-finite divisor)
  // sends the lane to the exact path.
  if (native && d > 0.f && r < __builtin_huge_valf() && d < __builtin_huge_valf()) {
    bool nan = false;
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const float q0 = div_rn_pz(Elem<T>::ld(v.e[j]), d, r);
      const float q1 = div_rn_pz(Elem<T>::ld(v.e[j + 1]), d, r);
      nan |= (q0 != q0) | (q1 != q1);
      o |= fp4_pair_hw(q0, q1, 1.0f) << (4 * j);
    }
    if (!nan) {
      if constexpr (N == 8)
        st_packed_nt(y + i * (N / 2), o);
      else
        st_packed_nt(y + i * (N / 2), (uint16_t)o);
      return;
    }
    o = 0;
  }
  if (native) {
    // exact lane: IEEE division handles what div_rn does not (+-inf / d, a zero or non-finite d)
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const uint32_t lo = nvfp4_code(Elem<T>::ld(v.e[j]) / d);
      const uint32_t hi = nvfp4_code(Elem<T>::ld(v.e[j + 1]) / d);
      o |= (lo | (hi << 4)) << (4 * j);
    }
  } else {  // the r01 emulated kernel, kept as the A/B baseline
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      const uint32_t lo = nvfp4_code(div_rn(Elem<T>::ld(v.e[j]), d, r));
      const uint32_t hi = nvfp4_code(div_rn(Elem<T>::ld(v.e[j + 1]), d, r));
      o |= (lo | (hi << 4)) << (4 * j);
    }
  }
  if constexpr (N == 8)
    st_packed_nt(y + i * (N / 2), o);
  else
    st_packed_nt(y + i * (N / 2), (uint16_t)o);
}

// MXFP4: LPB = block / N lanes per block, shuffle-max, every lane writes N/2 code bytes.  Scale
// bytes: with LDS, the block's first lane puts its byte into the workgroup's LDS line `sl` and the
// kernel writes the line once (export_mxfp4_vec_kernel); with 16-bit elements and block 32 (LPB 4)
// and a 4-byte aligned scale buffer (SC4), the bytes of 4 consecutive blocks are gathered into lane
// 16 k of each 16-lane row and leave as one dword store; otherwise the block's first lane writes
// its byte.  The caller loads the lane's vector (all of a thread's loads issued first).
template <typename T, int BLOCK, bool SC4, bool LDS = false>
__device__ __forceinline__ void export_mxfp4_vec_one(int64_t i, const Vec<T> &v, uint8_t *__restrict__ y,
                                                     uint8_t *__restrict__ sc, int64_t nvec, int native,
                                                     uint8_t *sl = nullptr) {
  using V = Vec<T>;
  constexpr int N = V::N;
  constexpr int LPB = BLOCK / N;
  if (i - (threadIdx.x % LPB) >= nvec) return;
  float amax = 0.f;
  if constexpr (N == 8) {
    // 16-bit elements: max of the |x| bit patterns, two per packed u16 op (NaN patterns sort
    // above inf, so a NaN propagates as torch.max does)
    const uint32_t w[4] = {v.raw.x, v.raw.y, v.raw.z, v.raw.w};
    const uint32_t m = group_max_u32<LPB>(scan_pairs(w).max_abs);
    amax = half_bits_to_float<T>(m);
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const float a = fabsf(Elem<T>::ld(v.e[j]));
      amax = (a > amax || a != a) ? a : amax;
    }
#pragma unroll
    for (int o = LPB / 2; o > 0; o >>= 1) {
      const float t = __shfl_xor(amax, o, 64);
      amax = (t > amax || t != t) ? t : amax;
    }
  }
  // amax / 6 correctly rounded without the IEEE division sequence for 16-bit elements: div_rn
  // with r = RN(1/6), bit-identical to the operator for every finite bf16 / f16 amax
  // (scripts/check_div6.c, exhaustive; tests/test_div_rn_check.py); inf / NaN amax keep the
  // operator's result (inf * RN(1/6) = inf).  fp32 elements keep the division.
  float d6;
  if constexpr (N == 8) {
    constexpr float kInv6 = 1.0f / 6.0f;
    d6 = amax <= 3.402823466e38f ? div_rn(amax, 6.0f, kInv6) : amax * kInv6;
  } else {
    d6 = amax / 6.0f;
  }
  const float e = mx_e8m0_exponent(d6);
  const uint32_t sbyte = (uint32_t)(int)(e + 127.f) & 0xFFu;
  if constexpr (LDS) {
    if (threadIdx.x % LPB == 0) sl[threadIdx.x / LPB] = (uint8_t)sbyte;
  } else if constexpr (SC4) {
    static_assert(LPB == 4, "dword scale stores: 4 lanes per block");
    // lanes 16k .. 16k+15 hold blocks 4k' .. 4k'+3 (vector index i is lane-consecutive and the
    // chunk base a multiple of 256): gather the three neighbour blocks' bytes into lane 16k
    const uint32_t b1 = (uint32_t)__shfl_down((int)sbyte, 4, 16);
    const uint32_t b2 = (uint32_t)__shfl_down((int)sbyte, 8, 16);
    const uint32_t b3 = (uint32_t)__shfl_down((int)sbyte, 12, 16);
    if ((threadIdx.x & 15) == 0) {
      const int64_t blk = i / LPB;
      if (i + 15 < nvec)
        __builtin_nontemporal_store(sbyte | (b1 << 8) | (b2 << 16) | (b3 << 24),
                                    reinterpret_cast<uint32_t *>(sc + blk));
      else  // the tensor's last, partial row of blocks
        for (int k = 0; k < 4 && i + 4 * k < nvec; ++k)
          sc[blk + k] = (uint8_t)(k == 0 ? sbyte : k == 1 ? b1 : k == 2 ? b2 : b3);
    }
  } else {
    if (threadIdx.x % LPB == 0) sc[i / LPB] = (uint8_t)sbyte;
  }
  uint32_t o = 0;
  if constexpr (N == 8) {
    // Native (16-bit elements, -100 <= e <= 127 so 2^e is a normal scale operand and no input the
    // converter might flush can reach a nonzero code): the reference counts strict `bounds < |q|`,
    // i.e. ties toward zero, where the converter rounds ties to the even code -- they differ on
    // |q| = 0.75, 1.75, 3.5.  A 16-bit x has at most 11 significant bits, so x minus one fp32 ulp
    // lies strictly between x and every other 16-bit value: it falls on the same side of every
    // midpoint as x does, except that a midpoint itself now rounds down.  A quotient x / 2^e that
    // is zero in fp32 -- x = +-0, or |x| <= 2^(e - 150) underflowing -- is code 8 in the reference
    // (torch.sign(0) = 0) where the converter sees a signed tiny value: those nibbles are patched.
    // A NaN element makes e NaN and takes the exact path.
    if (native && e >= -100.f && e <= 127.f) {
      const int ei = (int)e;
      const float s = __uint_as_float((uint32_t)(ei + 127) << 23);
      // largest |x| whose quotient rounds to zero: 2^(e - 150) (normal for e >= 24, subnormal
      // for 1 <= e <= 23; below every nonzero 16-bit value for e < 1)
      const float zthr = __uint_as_float(ei >= 24 ? (uint32_t)(ei - 23) << 23
                                                  : (ei >= 1 ? 1u << (ei - 1) : 0u));
      uint32_t zero = 0;
#pragma unroll
      for (int j = 0; j < N; j += 2) {
        const float f0 = Elem<T>::ld(v.e[j]), f1 = Elem<T>::ld(v.e[j + 1]);
        zero |= (fabsf(f0) <= zthr ? 0xFu : 0u) << (4 * j);
        zero |= (fabsf(f1) <= zthr ? 0xFu : 0u) << (4 * j + 4);
        o |= fp4_pair_hw(__uint_as_float(__float_as_uint(f0) - 1u),
                         __uint_as_float(__float_as_uint(f1) - 1u), s)
             << (4 * j);
      }
      o = (o & ~zero) | (zero & 0x88888888u);
      st_packed_nt(y + i * (N / 2), o);
      return;
    }
  }
  const float pinv = (e == e) ? exp2f(-e) : e;  // exact power of two: x * 2^-e == x / 2^e
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float q = Elem<T>::ld(v.e[j]) * pinv;
    const float a = fabsf(q);
    const uint32_t ord = (a > 0.25f) + (a > 0.75f) + (a > 1.25f) + (a > 1.75f) + (a > 2.5f) +
                         (a > 3.5f) + (a > 5.0f);
    o |= (((q > 0.f) ? 0u : 8u) + ord) << (4 * j);
  }
  if constexpr (N == 8)
    st_packed_nt(y + i * (N / 2), o);
  else
    st_packed_nt(y + i * (N / 2), (uint16_t)o);
}

// Per-tensor FP8 export (the unified-HF-export weight path): the scale and its reciprocal once per
// thread from the scalar-loaded amax (the per-vector IEEE 1/s sequence and its wait were ~1.3 VALU
// per element), the dtype re-rounding as a template parameter instead of a per-element select,
// and all U vectors of a lane loaded before the first is converted.  Same arithmetic as
// export_fp8_vec_one: div_rn on packed pairs, optional re-rounding, the native RNE convert for
// |q| <= 448, the exact per-element form for a lane with an overflowing or NaN quotient.
// the E4M3 bytes of one 16-bit vector (8 elements), packed in two dwords
template <typename T, bool ROUND>
__device__ __forceinline__ u32x2_t export_fp8_pt_pack(const Vec<T> &v, float s, float r) {
  static_assert(Vec<T>::N == 8, "16-bit vectors");
  constexpr int N = 8;
  float q[N];
  bool inrange = true;
#pragma unroll
  for (int j = 0; j < N; j += 2) {
    f32x2_t d = div_rn2((f32x2_t){Elem<T>::ld(v.e[j]), Elem<T>::ld(v.e[j + 1])}, s, r);
    if constexpr (ROUND) d = round_pair<T>(d);
    q[j] = d.x;
    q[j + 1] = d.y;
    inrange &= (fabsf(d.x) <= kE4M3Max) & (fabsf(d.y) <= kE4M3Max);
  }
  if (__builtin_expect(inrange, 1)) {
    uint32_t w[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(q[4 * k], q[4 * k + 1], 0, false);
      w[k] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(q[4 * k + 2], q[4 * k + 3], p, true);
    }
    return (u32x2_t){w[0], w[1]};
  }
  uint32_t b[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    float qq = div_rn(Elem<T>::ld(v.e[j]), s, r);
    if constexpr (ROUND) qq = Elem<T>::ld(Elem<T>::st(qq));
    b[j] = e4m3_byte(qq) | nan_sign_byte(v.e[j]);
  }
  return (u32x2_t){b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24), b[4] | (b[5] << 8) | (b[6] << 16) | (b[7] << 24)};
}

template <typename T, bool ROUND>
__device__ __forceinline__ void export_fp8_pt_one(int64_t i, const Vec<T> &v, uint8_t *__restrict__ y,
                                                  float s, float r) {
  constexpr int N = Vec<T>::N;
  if constexpr (N == 8) {
    const u32x2_t w = export_fp8_pt_pack<T, ROUND>(v, s, r);
    st_packed_nt(y + i * N, w.x, w.y);
    return;
  } else {
    float q[N];
    bool inrange = true;
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      f32x2_t d = div_rn2((f32x2_t){Elem<T>::ld(v.e[j]), Elem<T>::ld(v.e[j + 1])}, s, r);
      if constexpr (ROUND) d = round_pair<T>(d);
      q[j] = d.x;
      q[j + 1] = d.y;
      inrange &= (fabsf(d.x) <= kE4M3Max) & (fabsf(d.y) <= kE4M3Max);
    }
    if (__builtin_expect(inrange, 1)) {
      int p = __builtin_amdgcn_cvt_pk_fp8_f32(q[0], q[1], 0, false);
      st_packed_nt(y + i * N, (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(q[2], q[3], p, true));
      return;
    }
    uint32_t b[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      float qq = div_rn(Elem<T>::ld(v.e[j]), s, r);
      if constexpr (ROUND) qq = Elem<T>::ld(Elem<T>::st(qq));
      b[j] = e4m3_byte(qq) | nan_sign_byte(v.e[j]);
    }
    st_packed_nt(y + i * N, (uint32_t)(b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)));
  }
}

template <int U, typename T, bool ROUND>
__global__ __launch_bounds__(kThreads) void export_fp8_pt_kernel(const T *__restrict__ x,
                                                                  uint8_t *__restrict__ y,
                                                                  int64_t nvec,
                                                                  const float *__restrict__ scale) {
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  Vec<T> v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * Vec<T>::N);
  }
  // the scale after the data loads (the empty asm keeps the compiler from hoisting its scalar
  // load and wait above them): its round trip and 1/s overlap the data's
  asm volatile("" ::: "memory");
  const float s = scale[0];
  const float r = 1.0f / s;
  // a whole block in range (all but the last) converts unconditionally: with only the lane-guarded
  // form the compiler sank the first load into its guarded consumer and waited vmcnt(0) there
  if ((int64_t)(blockIdx.x + 1) * (kThreads * U) <= nvec) {
#pragma unroll
    for (int u = 0; u < U; ++u) export_fp8_pt_one<T, ROUND>(base + u * kThreads, v[u], y, s, r);
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u * kThreads < nvec) export_fp8_pt_one<T, ROUND>(base + u * kThreads, v[u], y, s, r);
  }
}

template <int U, typename T, bool IDX32>
__global__ __launch_bounds__(kThreads) void export_fp8_vec_kernel(const T *__restrict__ x,
                                                                   uint8_t *__restrict__ y,
                                                                   int64_t nvec, int64_t cv,
                                                                   FastDiv fcv,
                                                                   const float *__restrict__ scale,
                                                                   int per_row, int round_dtype,
                                                                   int native) {
  const float s_t = per_row ? 0.f : scale[0];
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u)
    export_fp8_vec_one<T, IDX32>(base + u * kThreads, x, y, nvec, cv, fcv, scale, per_row, round_dtype,
                                 native, s_t);
}
// FP8 with 2D block scales (FP8QTensor.quantize with {-1: bc, -2: br}, qtensor/fp8_tensor.py:40-117,
// the FP8_PB_WO export, export/quant_utils.py:874-877): vector i (N elements along a row, never
// across a column block: bc % N == 0) uses scale[(row / br) * ncb + col / bc] of the fp32 block
// grid; the fp32 quotient (input / expanded_scales promotes to fp32) converted as the per-row path.
// U vectors per lane, all loaded before the first scale index is formed (the one-vector form
// with three int64 divisions per vector ran at 0.62 of the roofline, r05); row / block indices
// from 32-bit multiply-high dividers when every index fits (IDX32).
template <int U, typename T, bool IDX32>
__global__ __launch_bounds__(kThreads) void export_fp8_blk2d_kernel(const T *__restrict__ x, uint8_t *__restrict__ y,
                                                                    int64_t nvec, int64_t cv, FastDiv fcv, int64_t br,
                                                                    FastDiv fbr, int64_t bcv, FastDiv fbcv, int64_t ncb,
                                                                    const float *__restrict__ scale, int round_dtype,
                                                                    int native) {
  constexpr int N = Vec<T>::N;
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  Vec<T> v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * N);
  }
  float sv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    int64_t i = base + u * kThreads;
    i = i < nvec ? i : nvec - 1;
    const int64_t row = idx_div<IDX32>(i, cv, fcv), cvec = i - row * cv;
    sv[u] = scale[idx_div<IDX32>(row, br, fbr) * ncb + idx_div<IDX32>(cvec, bcv, fbcv)];
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * kThreads < nvec) export_fp8_pack_store<T>(base + u * kThreads, v[u], y, sv[u], round_dtype, native);
}

template <int U, typename T, bool IDX32>
__global__ __launch_bounds__(kThreads) void export_int4_vec_kernel(const T *__restrict__ x,
                                                                    uint8_t *__restrict__ y,
                                                                    int64_t nvec, int64_t cols,
                                                                    FastDiv fcv, FastDiv fblk,
                                                                    const float *__restrict__ scale,
                                                                    int64_t nblk, int block) {
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  Int4Pair<T> q[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: see export_mxfp4_vec_kernel
    const int64_t i = base + u * kThreads;
    q[u] = export_int4_load<T, IDX32>(i < nvec ? i : nvec - 1, x, cols, fcv, fblk, scale, nblk, block);
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (base + u * kThreads < nvec) export_int4_pack<T>(q[u], y);
}
template <int U, typename T, bool IDX32>
__global__ __launch_bounds__(kThreads) void export_nvfp4_vec_kernel(const T *__restrict__ x,
                                                                     uint8_t *__restrict__ y,
                                                                     int64_t nvec, int64_t vpb,
                                                                     FastDiv fvpb,
                                                                     const float *__restrict__ sblk,
                                                                     const float *__restrict__ s2,
                                                                     int native) {
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; ++u)
    export_nvfp4_vec_one<T, IDX32>(base + u * kThreads, x, y, nvec, vpb, fvpb, sblk, s2, native);
}
template <int U, typename T, int BLOCK, bool SC4>
__global__ __launch_bounds__(kThreads) void export_mxfp4_vec_kernel(const T *__restrict__ x,
                                                                     uint8_t *__restrict__ y,
                                                                     uint8_t *__restrict__ sc,
                                                                     int64_t nvec, int native) {
  constexpr int LPB = BLOCK / Vec<T>::N;
  const int64_t base = (int64_t)blockIdx.x * (kThreads * U) + threadIdx.x;
  // every load of the thread issued before the first block is converted (the FP8 per-tensor
  // packer's lesson, 0.589 -> 0.666: a load behind the previous vector's stores was waited for)
  // The loads are unconditional (a lane past the end re-reads the last vector, n % block == 0 so
  // whole blocks are past it and export_mxfp4_vec_one drops them): a load under a lane condition
  // made the compiler wait vmcnt(0) right behind each one (the wait analysis is path-insensitive),
  // serialising the U loads.
  static_assert(LPB >= 1, "block holds whole vectors");
  Vec<T> v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * Vec<T>::N);
  }
  if constexpr (SC4) {
    // The workgroup's U * 64 scale bytes are consecutive: gathered in LDS and written as whole
    // dwords by the first U * 16 lanes (two 128 B lines for U = 4) instead of 8 waves x U
    // non-temporal 16 B fragments, each a partial-line write (0.643 -> 0.689 of the roofline at
    // U = 2, profiles/r04/export/export_mxfp4_store_ab_r04v.json).
    constexpr int NB = U * kThreads / LPB;
    static_assert(NB % 4 == 0, "whole dwords of scale bytes");
    __shared__ uint8_t sl[NB];
#pragma unroll
    for (int u = 0; u < U; ++u)
      export_mxfp4_vec_one<T, BLOCK, true, true>(base + u * kThreads, v[u], y, sc, nvec, native,
                                                 sl + u * (kThreads / LPB));
    __syncthreads();
    const int64_t b0 = (int64_t)blockIdx.x * NB, nblk = nvec / LPB;
    if (b0 + NB <= nblk) {
      if (threadIdx.x < NB / 4)
        __builtin_nontemporal_store(reinterpret_cast<const uint32_t *>(sl)[threadIdx.x],
                                    reinterpret_cast<uint32_t *>(sc + b0) + threadIdx.x);
    } else {
      for (int t = threadIdx.x; t < NB && b0 + t < nblk; t += kThreads) sc[b0 + t] = sl[t];
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u) export_mxfp4_vec_one<T, BLOCK, false>(base + u * kThreads, v[u], y, sc, nvec, native);
  }
}

// U = 2 consecutive 256-vector chunks per block (U = 1 / 4 within run-to-run noise,
// profiles/r02/export/export_u_ab.json)
template <class F> void with_export_u(F &&f) { f(std::integral_constant<int, 2>{}); }
unsigned export_grid(int64_t nvec, int u) { return (unsigned)((nvec + kThreads * u - 1) / (kThreads * u)); }

// MXFP8QTensor.quantize (qtensor/mxfp8_tensor.py:36-52 + 163-187): per 32-block along the rows,
// amax = max|x| (NaN propagates), descale = amax / 448 (IEEE), e = clamp(ceil(log2(descale)),
// -127, 127) with log2 correctly rounded and e = -127 where descale is not > 0 (0 or NaN, the
// reference's torch.where); q = e4m3(clamp(x * 2^-e, -448, 448)) (RNE, NaN kept); scale byte
// e + 127.  Four lanes per block, one 16-byte vector each; 8 e4m3 bytes per lane out.
template <typename T>
__global__ __launch_bounds__(kThreads) void export_mxfp8_kernel(const T *__restrict__ x,
                                                                 uint8_t *__restrict__ y,
                                                                 uint8_t *__restrict__ sc,
                                                                 int64_t nvec) {
  const int64_t v = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  const bool ok = v < nvec;
  Vec<T> xv;
  if (ok)
    xv = ldg_vec_nt(x + v * 8);
  else
    xv.raw = make_uint4(0, 0, 0, 0);
  float f[8];
  uint32_t m = 0;  // max of |x| bit patterns: NaN patterns sort above +inf
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    f[j] = Elem<T>::ld(xv.e[j]);
    const uint32_t b = __float_as_uint(f[j]) & 0x7fffffffu;
    m = b > m ? b : m;
  }
  m = group_max_u32<4>(m);
  const float amax = __uint_as_float(m > 0x7f800000u ? 0x7fc00000u : m);
  const float descale = amax / 448.0f;
  float e = descale > 0.f ? mx_e8m0_exponent(descale) : -127.f;
  e = e < 127.f ? e : 127.f;
  const float p = __builtin_ldexpf(1.0f, -(int)e);
  uint32_t w[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t packed = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)  // torch's cast: NaN -> 0x7F | sign
      packed |= e4m3_byte(clamp_nan(f[4 * h + j] * p, -kE4M3Max, kE4M3Max)) << (8 * j);
    w[h] = packed;
  }
  if (ok) {
    *reinterpret_cast<uint2 *>(y + v * 8) = make_uint2(w[0], w[1]);
    if ((threadIdx.x & 3) == 0) sc[v >> 2] = (uint8_t)(int)(e + 127.f);
  }
}

}  // namespace

// shared with the other translation units of libmtq_amd.so (mtq_search.hip)
namespace mtq {
int host_check_launch() { return check_launch(); }
int host_num_cus() { return num_cus(); }
static std::atomic<long long> g_dispatch[kDispCount];
void count_dispatch(int id) { g_dispatch[id].fetch_add(1, std::memory_order_relaxed); }
static const char *const kDispatchNames[kDispCount] = {
    "ew_vec", "ew_group_sk", "ew_group", "ew_rowwave", "amax_persist", "amax_rows_u", "amax_rows_short",
    "amax_cols_wide", "block_quant_dyn", "hist_value", "hist_value_chunked", "mx_vec", "mx_e2m1_native",
    "nvfp4_native_u", "awq_search_pp", "awq_prescale", "awq_mse_multi", "hist_value_nz", "mx_e4m3_native", "awq_search_w4"};
}  // namespace mtq

// ============================================================================================
// C ABI
// ============================================================================================
extern "C" {

int mtq_dispatch_counts(int64_t *counts, int n) {
  if (n < 0 || (n > 0 && !counts)) return -1;
  for (int i = 0; i < n && i < kDispCount; ++i) counts[i] = g_dispatch[i].load(std::memory_order_relaxed);
  return kDispCount;
}

const char *mtq_dispatch_name(int id) { return id >= 0 && id < kDispCount ? kDispatchNames[id] : nullptr; }

const char *mtq_status_string(int status) {
  switch (status) {
  case MTQ_OK: return "ok";
  case MTQ_ERR_INVALID_ARG: return "invalid argument";
  case MTQ_ERR_DTYPE: return "unsupported dtype";
  case MTQ_ERR_BLOCKSIZE: return "Blocksize for fused call must be one of {8, 16, 32}";
  case MTQ_ERR_FORMAT: return "unsupported quantization format";
  case MTQ_ERR_LAUNCH: return "HIP kernel launch failed";
  case MTQ_ERR_NO_DEVICE: return "no HIP device";
  default: return "unknown status";
  }
}

int mtq_last_hip_error(void) { return g_last_hip_error; }

int mtq_version(void) { return 100; }

int mtq_fake_tensor_quant(const void *x, void *y, int64_t n, int dtype, const void *amax,
                          int amax_dtype, int num_bits, int is_unsigned, int narrow_range,
                          hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !y || !amax)) || num_bits < 1 || num_bits > 31)
    return MTQ_ERR_INVALID_ARG;
  if (!valid_dtype(dtype) || !valid_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  IntBounds b = int_bounds(num_bits, is_unsigned, narrow_range);
  return dispatch_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    IntTensorOp<T> op{amax, amax_dtype, b.max_bound, b.min_bound, {}};
    return launch_ew<T>(x, y, n, op, stream);
  });
}

int mtq_fake_tensor_quant_with_axis(const void *x, void *y, int64_t n, int dtype,
                                    const void *amax, int amax_dtype, int64_t axis_size,
                                    int64_t inner, int num_bits, int is_unsigned,
                                    int narrow_range, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !y || !amax)) || axis_size < 1 || inner < 1 || num_bits < 1 ||
      num_bits > 31)
    return MTQ_ERR_INVALID_ARG;
  if (!valid_dtype(dtype) || !valid_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  IntBounds b = int_bounds(num_bits, is_unsigned, narrow_range);
  return dispatch_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    auto fill = [&](auto &op) {
      op.amax = amax;
      op.amax_dtype = amax_dtype;
      op.max_bound = b.max_bound;
      op.min_bound = b.min_bound;
    };
    return launch_axis<T, IntAxisVecOp, IntAxisElemOp>(x, y, n, axis_size, inner, fill, stream);
  });
}

int mtq_fake_e4m3fy(const void *x, void *y, int64_t n, int dtype, const void *amax,
                    int amax_dtype, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !y || !amax))) return MTQ_ERR_INVALID_ARG;
  if (!valid_dtype(dtype) || !valid_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  return dispatch_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    Fp8TensorOp<T> op{amax, amax_dtype, {}};
    return launch_ew<T>(x, y, n, op, stream);
  });
}

int mtq_fake_e4m3fy_with_axis(const void *x, void *y, int64_t n, int dtype, const void *amax,
                              int amax_dtype, int64_t axis_size, int64_t inner,
                              hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !y || !amax)) || axis_size < 1 || inner < 1)
    return MTQ_ERR_INVALID_ARG;
  if (!valid_dtype(dtype) || !valid_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  return dispatch_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    auto fill = [&](auto &op) {
      op.amax = amax;
      op.amax_dtype = amax_dtype;
    };
    return launch_axis<T, Fp8AxisVecOp, Fp8AxisElemOp>(x, y, n, axis_size, inner, fill, stream);
  });
}

int mtq_e4m3_cast(const void *x, void *y, int64_t n, int dtype, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!x || !y))) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    return launch_ew<T>(x, y, n, Fp8CastOp<T>{}, stream);
  });
}

int mtq_fused_amax_convert(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                           int block_size, int format, int scale_format,
                           const float *global_amax, int per_channel, hipStream_t stream) {
  if (rows < 0 || cols < 0 || ((rows * cols) > 0 && (!x || !y))) return MTQ_ERR_INVALID_ARG;
  if (block_size != 8 && block_size != 16 && block_size != 32) return MTQ_ERR_BLOCKSIZE;
  if (format < 0 || format > 9 || scale_format < 0 || scale_format > 9) return MTQ_ERR_FORMAT;
  MxParams p{format, scale_format, global_amax, per_channel, cols};
  return dispatch_dtype_nof64(dtype, [&](auto t) {
    using T = decltype(t);
    return launch_mx<T>(x, y, rows, cols, block_size, p, stream);
  });
}

int mtq_reduce_amax(const void *x, int64_t P, int64_t K, int64_t Q, int dtype, float *out,
                    hipStream_t stream) {
  if (P < 0 || K < 1 || Q < 0 || !out || (P * K * Q > 0 && !x)) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) {
    using T = decltype(t);
    return launch_amax<T>(x, P, K, Q, out, stream);
  });
}

int mtq_amax_fill(float *out, int64_t n, float value, hipStream_t stream) {
  if (n < 0 || (n > 0 && !out)) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  amax_fill_kernel<<<grid_for(n, kThreads), kThreads, 0, stream>>>(out, n, value);
  return check_launch();
}

int mtq_amax_fold(float *dst, const float *src, int64_t n, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!dst || !src))) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  amax_fold_kernel<<<grid_for(n, kThreads), kThreads, 0, stream>>>(dst, src, n);
  return check_launch();
}

int mtq_amax_check(const void *x, int64_t n, int dtype, int32_t *flags, hipStream_t stream) {
  if (n < 0 || !flags || (n > 0 && !x)) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    // one workgroup up to 1 M elements (one launch, no zeroing); above, the whole GPU (static
    // block scales concatenated over many quantizers reach 10^8 elements: ADVICE r04)
    if (n <= (1 << 20) || !aligned16(x)) {
      amax_check_kernel<T, false><<<1, kCheckThreads, 0, stream>>>(reinterpret_cast<const T *>(x), n, flags);
    } else {
      const int64_t nvec = n / Vec<T>::N;
      int64_t g = (nvec + (int64_t)kCheckThreads * 4 - 1) / ((int64_t)kCheckThreads * 4);
      const int64_t cap = (int64_t)num_cus() * 2;
      g = g < cap ? g : cap;
      amax_check_zero_kernel<<<1, 64, 0, stream>>>(flags);
      amax_check_kernel<T, true><<<(unsigned)g, kCheckThreads, 0, stream>>>(reinterpret_cast<const T *>(x), n, flags);
    }
    return check_launch();
  });
}

int mtq_mask_unrouted_rows(const void *x, void *y, const int64_t *idx, int64_t rows, int64_t cols, int k,
                           int64_t num_experts, int dtype, hipStream_t stream) {
  if (rows < 0 || cols < 0 || k < 1 || num_experts < 1) return MTQ_ERR_INVALID_ARG;
  if (rows == 0 || cols == 0) return MTQ_OK;
  if (!x || !y || !idx) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    const T *xt = reinterpret_cast<const T *>(x);
    T *yt = reinterpret_cast<T *>(y);
    if (cols % N == 0 && aligned16(x) && aligned16(y))
      mask_rows_kernel<T, true><<<grid_for(rows * cols / N, kThreads), kThreads, 0, stream>>>(xt, yt, idx, rows, cols, k,
                                                                                          num_experts);
    else
      mask_rows_kernel<T, false><<<grid_for(rows * cols, kThreads), kThreads, 0, stream>>>(xt, yt, idx, rows, cols, k,
                                                                                       num_experts);
    return check_launch();
  });
}

int mtq_block_quant_dynamic(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                            const void *pqs, int pqs_dtype, int block, int num_bits,
                            int is_unsigned, int narrow_range, hipStream_t stream) {
  if (rows < 0 || cols < 1 || num_bits < 1 || num_bits > 31) return MTQ_ERR_INVALID_ARG;
  if (rows == 0) return MTQ_OK;
  if (!x || !y) return MTQ_ERR_INVALID_ARG;
  if (pqs && pqs_dtype != dtype) return MTQ_ERR_DTYPE;
  IntBounds b = int_bounds(num_bits, is_unsigned, narrow_range);
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    if (cols % block != 0 || block % N != 0 || !aligned16(x) || !aligned16(y) ||
        (pqs && !aligned16(pqs)))
      return MTQ_ERR_INVALID_ARG;
    const int64_t nvec = rows * cols / N;
    const T *xt = reinterpret_cast<const T *>(x);
    T *yt = reinterpret_cast<T *>(y);
    const T *pt = reinterpret_cast<const T *>(pqs);
    // U = 2 vectors per lane, both loads first: 0.738 -> 0.766 of the HBM roofline over one
    // (profiles/r03/dyn_u/)
    auto go_u = [&](auto blk_c) {
      constexpr int BLK = decltype(blk_c)::value, U = 2;
      const unsigned gu = (unsigned)((nvec + (int64_t)kThreads * U - 1) / ((int64_t)kThreads * U));
      count_dispatch(kDispBlockQuantDyn);
      block_quant_dyn_kernel<T, BLK, U><<<gu, kThreads, 0, stream>>>(xt, yt, pt, nvec, cols, b.max_bound, b.min_bound);
    };
    switch (block) {
    case 32: go_u(std::integral_constant<int, 32>{}); break;
    case 64: go_u(std::integral_constant<int, 64>{}); break;
    case 128: go_u(std::integral_constant<int, 128>{}); break;
    case 256:
      if constexpr (N == 8) {
        go_u(std::integral_constant<int, 256>{});
        break;
      }
      return MTQ_ERR_BLOCKSIZE;
    default: return MTQ_ERR_BLOCKSIZE;
    }
    return check_launch();
  });
}

int mtq_histogram_abs(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                      int skip_zeros, uint32_t *counts, hipStream_t stream) {
  if (n < 0 || bins < 1 || !hmax || !counts || (n > 0 && !x)) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    const T *xt = reinterpret_cast<const T *>(x);
    const bool lds = bins <= 16384;
    const size_t shm = lds ? (size_t)bins * 4 : 0;
    // 16-bit dtypes: pattern histogram + per-block fold, U = 2 vectors per lane with a register
    // prefetch (bf16 [32768, 4096], 2048 bins: 46.9 us = 71.6 %; U 1 / 4 / 8 and no prefetch
    // measured no faster, profiles/r02/histogram/; r05: U 4 / 2 / 3 = 40.0 / 41.3 / 46.0 us on
    // bf16 [8192, 14336] (profiles/r05/hist/hist_u_ab_r05m.log) but 0.691 vs 0.73-0.74 on the
    // bench input and slower for the chunked form (r05n), so U stays 2).
    if constexpr (sizeof(T) == 2) {
      if (aligned16(x) && n % N == 0 && bins <= 8192) {
        const int64_t nvec = n / N;
        int64_t blocks = num_cus();
        const int64_t min_per_block = (int64_t)kHistValThreads * 8;
        int64_t vpb = (nvec + blocks - 1) / blocks;
        vpb = vpb < min_per_block ? min_per_block : vpb;
        blocks = (nvec + vpb - 1) / vpb;
        const size_t shr = ((size_t)kHistPatterns + (size_t)bins) * 4;
        auto kern = hist_value_kernel<T, 2>;
        static bool attr = false;
        if (!attr) {
          (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          attr = true;
        }
        count_dispatch(kDispHistValue);
        kern<<<(unsigned)blocks, kHistValThreads, shr, stream>>>(xt, nvec, vpb, hmax, bins, skip_zeros, counts,
                                                                    HistChunks{}, HistNz{});
        return check_launch();
      }
    }
    // fp32 (and > 8192 bins): REP interleaved LDS copies of the bins (REP 4 while bins * REP fits
    // 16384 words), 2 blocks per CU (scripts/sweep_reduce.py: 4.3 TB/s on bf16 [32768, 4096]
    // against 2.4 TB/s for one copy; REP 8 / 1 block per CU no faster)
    if (aligned16(x) && n % N == 0 && lds) {
      int rep = 4;
      while (rep > 1 && (int64_t)bins * rep > 16384) rep >>= 1;
      const int64_t nvec = n / N;
      int64_t blocks = (int64_t)num_cus() * 2;
      const int64_t min_per_block = (int64_t)kHistDivThreads * 8;
      int64_t vpb = (nvec + blocks - 1) / blocks;
      vpb = vpb < min_per_block ? min_per_block : vpb;
      blocks = (nvec + vpb - 1) / vpb;
      const size_t shr = (size_t)bins * rep * 4;
      switch (rep) {
      case 4:
        hist_div_kernel<T, 4, 4><<<(unsigned)blocks, kHistDivThreads, shr, stream>>>(
            xt, nvec, vpb, hmax, bins, skip_zeros, counts);
        break;
      case 2:
        hist_div_kernel<T, 2, 4><<<(unsigned)blocks, kHistDivThreads, shr, stream>>>(
            xt, nvec, vpb, hmax, bins, skip_zeros, counts);
        break;
      default:
        hist_div_kernel<T, 1, 4><<<(unsigned)blocks, kHistDivThreads, shr, stream>>>(
            xt, nvec, vpb, hmax, bins, skip_zeros, counts);
      }
      return check_launch();
    }
    // unaligned / ragged inputs, or bins past the LDS: one element per lane
    unsigned g = grid_for(n, kThreads * 8);
    hist_kernel<T><<<g, kThreads, shm, stream>>>(xt, n, hmax, bins, skip_zeros, counts, lds ? 1 : 0);
    return check_launch();
  });
}

int64_t mtq_histogram_chunked_scratch_words(int64_t n, int chunks, int bins) {
  if (n < 0 || chunks < 1 || bins < 1) return -1;
  return (int64_t)chunks * hist_chunk_bpc(n, chunks) * bins;
}

int mtq_histogram_abs_chunked(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                              int skip_zeros, const int64_t *bounds, int64_t chunk_elems, int chunks,
                              uint32_t *scratch, int64_t scratch_words, const float *accum, int64_t accum_n,
                              float *hist, hipStream_t stream) {
  if (n < 0 || bins < 1 || bins > 8192 || chunks < 1 || !hmax || !scratch || !hist || (n > 0 && !x))
    return MTQ_ERR_INVALID_ARG;
  if (accum_n < 0 || accum_n > bins || (accum_n > 0 && !accum)) return MTQ_ERR_INVALID_ARG;
  if (!bounds && (chunk_elems < 1 || (chunks - 1) * chunk_elems >= n)) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (n == 0) {  // nothing to count: no launch may read x
    hist_fill_kernel<<<(unsigned)((bins + 255) / 256), 256, 0, stream>>>(accum, accum_n, bins, hist);
    return check_launch();
  }
  if (!aligned16(x) || n % 8 != 0) return MTQ_ERR_INVALID_ARG;
  const int64_t bpc = hist_chunk_bpc(n, chunks);
  if ((int64_t)chunks * bpc > INT32_MAX || scratch_words < (int64_t)chunks * bpc * bins) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    if constexpr (sizeof(T) == 2) {
      const size_t shr = ((size_t)kHistPatterns + (size_t)bins) * 4;
      auto kern = hist_value_kernel<T, 2, kHvChunked>;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      const HistChunks ch{bounds, chunk_elems, n, (int)bpc, chunks, scratch};
      count_dispatch(kDispHistValueChunked);
      kern<<<(unsigned)(chunks * bpc), kHistValThreads, shr, stream>>>(reinterpret_cast<const T *>(x), n / 8, 0,
                                                                      hmax, bins, skip_zeros, nullptr, ch, HistNz{});
      // 64 bins x 16 chunks per 1024-thread workgroup (16 x 16 per 256 threads: 4.99 vs 4.75-4.90 us
      // in the kernel trace, r05)
      constexpr int kFoldBW = 64;
      hist_fold_blocks_kernel<kFoldBW><<<(unsigned)((bins + kFoldBW - 1) / kFoldBW), kFoldBW * 16, 0, stream>>>(scratch, (int)bpc, chunks, bins,
                                                                                 accum, accum_n, hist);
      return check_launch();
    }
    return MTQ_ERR_DTYPE;
  });
}

// kHvNz geometry: ~one 1024-thread workgroup per CU over slab-aligned ranges; more workgroups
// only when a range would hold more slabs than the count kernel's LDS takes (> 1.6 G elements)
struct NzGeom {
  int64_t vpb;
  int G, S;
};
// LDS of the count kernel: 128 KiB pattern table + the bins + 16 words per slab <= 160 KiB
constexpr int64_t kNzLdsWords = 160 * 1024 / 4 - kHistPatterns;

NzGeom nz_geom(int64_t nvec, int bins) {
  int64_t kNzMaxSlabs = (kNzLdsWords - bins) / 16;
  kNzMaxSlabs = kNzMaxSlabs < 64 ? kNzMaxSlabs : 64;  // one slab per lane of the count kernel's VGPR
  NzGeom g;
  int64_t G = num_cus();
  int64_t slabs = (nvec + kNzSlabVec - 1) / kNzSlabVec;
  if (slabs < 1) slabs = 1;
  if (G > slabs) G = slabs;
  int64_t S = (slabs + G - 1) / G;
  if (S > kNzMaxSlabs) {
    S = kNzMaxSlabs;
    G = (slabs + S - 1) / S;
  }
  g.S = (int)S;
  g.vpb = S * kNzSlabVec;
  g.G = (int)((nvec + g.vpb - 1) / g.vpb);
  if (g.G < 1) g.G = 1;
  return g;
}

// the recount and fold kernels keep the workgroup ranks' prefix in LDS (int64 each)
size_t nz_recount_lds(const NzGeom &g, int bins) { return (size_t)(g.G + 1 + g.S + 1 + 18) * 8 + (size_t)bins * 4; }

int64_t mtq_histogram_nonzero_scratch_words(int64_t n, int threads, int bins) {
  if (n < 0 || threads < 1 || threads > 1024 || bins < 1 || bins > kNzLdsWords - 16) return -1;
  const NzGeom g = nz_geom(n / 8, bins);
  if (nz_recount_lds(g, bins) > 64 * 1024) return -1;  // > ~6e10 elements: the caller's per-chunk path
  return (int64_t)g.G * bins + g.G + (int64_t)g.G * g.S + (int64_t)threads * bins;
}

int mtq_histogram_abs_nonzero_chunked(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                                      int threads, int64_t grain, uint32_t *scratch, int64_t scratch_words,
                                      const float *accum, int64_t accum_n, float *hist, hipStream_t stream) {
  if (n < 0 || bins < 1 || bins > kNzLdsWords - 16 || threads < 1 || threads > 1024 || grain < 1 || !hmax || !hist ||
      (n > 0 && (!x || !scratch)))
    return MTQ_ERR_INVALID_ARG;
  if (accum_n < 0 || accum_n > bins || (accum_n > 0 && !accum)) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (n == 0) {  // nothing to count (no launch may read x)
    hist_fill_kernel<<<(unsigned)((bins + 255) / 256), 256, 0, stream>>>(accum, accum_n, bins, hist);
    return check_launch();
  }
  if (!aligned16(x) || n % 8 != 0) return MTQ_ERR_INVALID_ARG;
  if (scratch_words < mtq_histogram_nonzero_scratch_words(n, threads, bins)) return MTQ_ERR_INVALID_ARG;
  const int64_t nvec = n / 8;
  const NzGeom g = nz_geom(nvec, bins);
  HistNz nz;
  nz.vpb = g.vpb;
  nz.S = g.S;
  nz.rows = scratch;
  nz.wg_tot = nz.rows + (int64_t)g.G * bins;
  nz.slab_tot = nz.wg_tot + g.G;
  nz.rec = nz.slab_tot + (int64_t)g.G * g.S;
  nz.rec_words = (int64_t)threads * bins;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    if constexpr (sizeof(T) == 2) {
      const size_t shr = ((size_t)kHistPatterns + (size_t)bins + (size_t)g.S * 16) * 4;
      auto kern = hist_value_kernel<T, 2, kHvNz>;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
      }
      count_dispatch(kDispHistValueNz);
      kern<<<(unsigned)g.G, kHistValThreads, shr, stream>>>(reinterpret_cast<const T *>(x), nvec, g.vpb, hmax, bins,
                                                           1, nullptr, HistChunks{}, nz);
      if (threads > 1) {
        const size_t shr_r = nz_recount_lds(g, bins);
        static bool attr_r = false;
        if (!attr_r) {
          (void)hipFuncSetAttribute(reinterpret_cast<const void *>(hist_nz_recount_kernel<T>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          attr_r = true;
        }
        hist_nz_recount_kernel<T><<<dim3((unsigned)(threads - 1), (unsigned)g.S), kNzThreads, shr_r, stream>>>(
            reinterpret_cast<const u32x4 *>(x), nvec, nz, g.G, threads, grain, hmax, bins);
      }
      constexpr int kFoldBW = 64;
      const size_t shr_f = (size_t)(3 * g.G + 1 + 16) * 8 + (size_t)(16 + kNzFoldMaxRec) * kFoldBW * 4;
      hist_nz_fold_kernel<kFoldBW><<<(unsigned)((bins + kFoldBW - 1) / kFoldBW), kFoldBW * 16, shr_f, stream>>>(
          nz, g.G, threads, grain, bins, accum, accum_n, hist);
      return check_launch();
    }
    return MTQ_ERR_DTYPE;
  });
}

int64_t mtq_mse_workspace_floats(int64_t n, int dtype) {
  if (n < 0 || (dtype != MTQ_F32 && dtype != MTQ_F16 && dtype != MTQ_BF16)) return -1;
  return mse_grid(n, dtype) + 1;
}

int mtq_mse_accumulate(const void *a, const void *b, int64_t n, int dtype, float *loss,
                       float *workspace, int64_t workspace_floats, hipStream_t stream) {
  if (n < 0 || !loss || !workspace || (n > 0 && (!a || !b))) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;  // mean over nothing: the caller's torch path decides NaN
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    const int64_t grid = mse_grid(n, dtype);
    if (workspace_floats < grid + 1) return MTQ_ERR_INVALID_ARG;
    const bool al = aligned16(a) && aligned16(b);
    const int64_t nvec = al ? n / N : 0;
    if (!al && n > (int64_t)kMseThreads * 1024) return MTQ_ERR_INVALID_ARG;  // scalar path is tail-only
    mse_kernel<T><<<(unsigned)grid, kMseThreads, 0, stream>>>(
        reinterpret_cast<const T *>(a), reinterpret_cast<const T *>(b), n, nvec,
        reinterpret_cast<unsigned *>(workspace), workspace + 1, loss);
    return check_launch();
  });
}

int mtq_mul_cols(const void *x, const void *scale, void *y, int64_t rows, int64_t cols, int dtype,
                 hipStream_t stream) {
  if (rows < 0 || cols < 1) return MTQ_ERR_INVALID_ARG;
  if (rows == 0) return MTQ_OK;
  if (!x || !scale || !y) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    if (cols % N != 0 || !aligned16(x) || !aligned16(y) || !aligned16(scale))
      return MTQ_ERR_INVALID_ARG;
    const int64_t nvec = rows * cols / N;
    mul_cols_kernel<T><<<(unsigned)((nvec + kThreads - 1) / kThreads), kThreads, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<const T *>(scale),
        reinterpret_cast<T *>(y), nvec, cols);
    return check_launch();
  });
}

int mtq_nvfp4_fake_quant(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                         const float *global_amax, int block_size, hipStream_t stream) {
  if (rows < 0 || cols < 0 || !global_amax || (rows * cols > 0 && (!x || !y)))
    return MTQ_ERR_INVALID_ARG;
  if (block_size != 8 && block_size != 16 && block_size != 32) return MTQ_ERR_BLOCKSIZE;
  if (rows * cols == 0) return MTQ_OK;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    const T *xt = reinterpret_cast<const T *>(x);
    T *yt = reinterpret_cast<T *>(y);
    switch (block_size) {
    case 8: return launch_nvfp4<T, 8>(xt, yt, rows, cols, global_amax, stream);
    case 16: return launch_nvfp4<T, 16>(xt, yt, rows, cols, global_amax, stream);
    default: return launch_nvfp4<T, 32>(xt, yt, rows, cols, global_amax, stream);
    }
  });
}

int mtq_fp4_block_scale_quant(const void *x, void *y, int64_t nblocks, int block, int dtype,
                              const float *scales, hipStream_t stream) {
  if (nblocks < 0 || block < 1 || (nblocks > 0 && (!x || !y || !scales))) return MTQ_ERR_INVALID_ARG;
  if (nblocks == 0) return MTQ_OK;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    const T *xt = reinterpret_cast<const T *>(x);
    T *yt = reinterpret_cast<T *>(y);
    const int64_t n = nblocks * block;
    if (block % N == 0 && aligned16(x) && aligned16(y)) {
      const int64_t nvec = n / N;
      fp4_scaled_vec_kernel<T><<<(unsigned)((nvec + kThreads - 1) / kThreads), kThreads, 0, stream>>>(
          xt, yt, scales, nvec, block);
    } else {
      fp4_scaled_scalar_kernel<T><<<grid_for(n, kThreads), kThreads, 0, stream>>>(xt, yt, scales, n,
                                                                                  block);
    }
    return check_launch();
  });
}

int mtq_export_fp8(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                   const float *scale, int per_row, int round_to_dtype, hipStream_t stream) {
  if (rows < 0 || cols < 0 || (rows * cols > 0 && (!x || !y || !scale))) return MTQ_ERR_INVALID_ARG;
  if (rows * cols == 0) return MTQ_OK;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    const int64_t n = rows * cols;
    constexpr int N = Vec<T>::N;
    if (cols % N == 0 && aligned16(x) && ((uintptr_t)y % N) == 0) {
      const int64_t nvec = n / N, cv = cols / N;
      const FastDiv fcv = make_fastdiv(cv < (1ll << 31) ? (uint32_t)cv : 1u);
      if (!per_row)
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          if (round_to_dtype)
            export_fp8_pt_kernel<U, T, true><<<export_grid(nvec, U), kThreads, 0, stream>>>(
                reinterpret_cast<const T *>(x), y, nvec, scale);
          else
            export_fp8_pt_kernel<U, T, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(
                reinterpret_cast<const T *>(x), y, nvec, scale);
        });
      else if (nvec < (1ll << 31))
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_fp8_vec_kernel<U, T, true><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, cv, fcv, scale, per_row, round_to_dtype, 1);
        });
      else
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_fp8_vec_kernel<U, T, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, cv, fcv, scale, per_row, round_to_dtype, 1);
        });
    } else {
      export_fp8_kernel<T><<<grid_for(n, kThreads), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, n, cols, scale, per_row, round_to_dtype);
    }
    return check_launch();
  });
}

int mtq_export_fp8_block2d(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype, const float *scale,
                           int64_t block_rows, int64_t block_cols, int round_to_dtype, hipStream_t stream) {
  if (rows < 0 || cols < 0 || block_rows < 1 || block_cols < 1) return MTQ_ERR_INVALID_ARG;
  if (rows * cols == 0) return MTQ_OK;
  if (!x || !y || !scale) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    constexpr int N = Vec<T>::N;
    if (cols % N != 0 || block_cols % N != 0 || !aligned16(x) || ((uintptr_t)y % N) != 0)
      return MTQ_ERR_INVALID_ARG;
    const int64_t nvec = rows * cols / N, cv = cols / N, bcv = block_cols / N;
    const int64_t ncb = (cols + block_cols - 1) / block_cols;
    const bool i32 = nvec < (1ll << 31) && block_rows < (1ll << 31);
    const FastDiv fcv = make_fastdiv(i32 ? (uint32_t)cv : 1u), fbr = make_fastdiv(i32 ? (uint32_t)block_rows : 1u),
                  fbcv = make_fastdiv(i32 ? (uint32_t)bcv : 1u);
    constexpr int U = 2;
    if (i32)
      export_fp8_blk2d_kernel<U, T, true><<<export_grid(nvec, U), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, nvec, cv, fcv, block_rows, fbr, bcv, fbcv, ncb, scale, round_to_dtype, 1);
    else
      export_fp8_blk2d_kernel<U, T, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, nvec, cv, fcv, block_rows, fbr, bcv, fbcv, ncb, scale, round_to_dtype, 1);
    return check_launch();
  });
}

int mtq_export_int4(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                    const float *scale, int block, hipStream_t stream) {
  if (rows < 0 || cols < 0 || rows % 2 || block < 1 || cols % block) return MTQ_ERR_INVALID_ARG;
  if (rows * cols == 0) return MTQ_OK;
  if (!x || !y || !scale) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    const int64_t n = rows / 2 * cols;
    constexpr int N = Vec<T>::N;
    if (cols % N == 0 && block % N == 0 && aligned16(x) && ((uintptr_t)y % N) == 0) {
      const int64_t nvec = n / N;
      const bool i32 = nvec < (1ll << 31) && cols < (1ll << 31);
      const FastDiv fcv = make_fastdiv(i32 ? (uint32_t)(cols / N) : 1u);
      const FastDiv fblk = make_fastdiv((uint32_t)block);
      if (i32)
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_int4_vec_kernel<U, T, true><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, cols, fcv, fblk, scale, cols / block, block);
        });
      else
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_int4_vec_kernel<U, T, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, cols, fcv, fblk, scale, cols / block, block);
        });
    } else {
      export_int4_kernel<T><<<grid_for(n, kThreads), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, rows / 2, cols, scale, cols / block, block);
    }
    return check_launch();
  });
}

int mtq_export_nvfp4(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                     const float *block_scale, const float *scale_2, int block,
                     hipStream_t stream) {
  if (rows < 0 || cols < 0 || cols % 2 || block < 2 || cols % block) return MTQ_ERR_INVALID_ARG;
  if (rows * cols == 0) return MTQ_OK;
  if (!x || !y || !block_scale || !scale_2) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    const int64_t npairs = rows * cols / 2;
    constexpr int N = Vec<T>::N;
    if (block % N == 0 && aligned16(x) && ((uintptr_t)y % (N / 2)) == 0) {
      const int64_t nvec = rows * cols / N, vpb = block / N;
      const FastDiv fvpb = make_fastdiv((uint32_t)vpb);
      if (nvec < (1ll << 31))
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_nvfp4_vec_kernel<U, T, true><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, vpb, fvpb, block_scale, scale_2, 1);
        });
      else
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_nvfp4_vec_kernel<U, T, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(
            reinterpret_cast<const T *>(x), y, nvec, vpb, fvpb, block_scale, scale_2, 1);
        });
    } else {
      export_nvfp4_kernel<T><<<grid_for(npairs, kThreads), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, npairs, cols, block_scale, scale_2, block);
    }
    return check_launch();
  });
}

int mtq_export_mxfp8(const void *x, uint8_t *y, uint8_t *scales, int64_t n, int dtype,
                     hipStream_t stream) {
  if (n < 0 || n % 32) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  if (!x || !y || !scales || !aligned16(x) || ((uintptr_t)y & 7u)) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    if (Vec<T>::N != 8) return MTQ_ERR_DTYPE;  // 16-bit element types
    const int64_t nvec = n / 8;
    export_mxfp8_kernel<T><<<grid_for(nvec, kThreads), kThreads, 0, stream>>>(
        reinterpret_cast<const T *>(x), y, scales, nvec);
    return check_launch();
  });
}

int mtq_export_mxfp4(const void *x, uint8_t *y, uint8_t *scales, int64_t n, int dtype, int block,
                     hipStream_t stream) {
  if (n < 0 || block < 2 || block % 2 || n % block) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  if (!x || !y || !scales) return MTQ_ERR_INVALID_ARG;
  return dispatch_dtype_nof64(dtype, [&](auto t) -> int {
    using T = decltype(t);
    const int64_t nb = n / block;
    constexpr int N = Vec<T>::N;
    if (aligned16(x) && ((uintptr_t)y % (N / 2)) == 0 && (block == 32 || block == 16) && block % N == 0) {
      const int64_t nvec = n / N;
      const bool sc4 = N == 8 && block == 32 && ((uintptr_t)scales % 4) == 0;
      if (block == 32 && sc4) {
        // U = 4 vectors per lane (256 scale bytes per workgroup): 0.69 -> 0.74 of the roofline
        // against U = 2 (profiles/r04/export/export_mxfp4_store_ab_r04w.json)
        if constexpr (N == 8)
          export_mxfp4_vec_kernel<4, T, 32, true><<<export_grid(nvec, 4), kThreads, 0, stream>>>(reinterpret_cast<const T *>(x), y, scales, nvec, 1);
      } else if (block == 32)
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_mxfp4_vec_kernel<U, T, 32, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(reinterpret_cast<const T *>(x), y, scales, nvec, 1);
        });
      else
        with_export_u([&](auto uc) {
          constexpr int U = decltype(uc)::value;
          export_mxfp4_vec_kernel<U, T, 16, false><<<export_grid(nvec, U), kThreads, 0, stream>>>(reinterpret_cast<const T *>(x), y, scales, nvec, 1);
        });
    } else {
      export_mxfp4_kernel<T><<<grid_for(nb, kThreads), kThreads, 0, stream>>>(
          reinterpret_cast<const T *>(x), y, scales, nb, block);
    }
    return check_launch();
  });
}

// Host restatement of convert_to_types (tensor_quant_mx.h:161-188) on the same minifloat
// rounding rule the device uses; E4M3/E5M2 are the satfinite RNE casts.
float mtq_convert_to_exmy(float x, int format) {
  struct F {
    int m, emin;
    float vmax;
    bool away;
  };
  F f;
  switch (format) {
  case MTQ_E4M3: f = {3, -6, 448.f, false}; break;
  case MTQ_E5M2: f = {2, -14, 57344.f, false}; break;
  case MTQ_INT8: {
    float r = rintf(x);
    return r > 127.f ? 127.f : (r < -127.f ? -127.f : r);
  }
  case MTQ_E0M3: f = {3, 3, 7.f, false}; break;
  case MTQ_E1M2: f = {2, 1, 3.5f, false}; break;
  case MTQ_E3M0: f = {0, -2, 16.f, true}; break;
  case MTQ_E2M1: f = {1, 0, 6.f, false}; break;
  case MTQ_E3M2: f = {2, -2, 28.f, false}; break;
  case MTQ_E2M3: f = {3, 0, 7.5f, false}; break;
  default: return 0.f;
  }
  if (x != x) {
    if (format == MTQ_E4M3 || format == MTQ_E5M2) return x;
    return f.vmax;  // table formats saturate NaN (sign of NaN is not negative)
  }
  float sign = x < 0.f ? -1.f : 1.f;
  float v = fabsf(x);
  v = v < f.vmax ? v : f.vmax;
  uint32_t bits;
  memcpy(&bits, &v, 4);
  int e = (int)((bits >> 23) & 0xff) - 127;
  if (e < f.emin) e = f.emin;
  int k = e - f.m;
  float t = ldexpf(v, -k);
  float r = f.away ? floorf(t + 0.5f) : rintf(t);
  r = ldexpf(r, k);
  r = r < f.vmax ? r : f.vmax;
  return sign * r;
}

}  // extern "C"
