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
// mtq_fake_tensor_quant_with_axis / mtq_fake_e4m3fy_with_axis (same make_intq / make_fp8q /
// int_qdq / fp8 qdq helpers), so the dequantised weight values are bit-identical to the unfused
// path; only the GEMM summation order differs (as between any two GEMM libraries).
//
// Tiling: one workgroup per 16 output columns (16 W rows), 8 or 16 waves splitting K; lane l
// owns W row n0 + (l & 15) and the 8 K-elements 8 (l >> 4) .. +7 of each 32-wide K step (the
// bf16 B operand layout of mfma_f32_16x16x32: B[k = 8 (l >> 4) + j][col l & 15]); U = 4 K steps
// of W and of x (M <= 16 rows: one M tile, re-read from L2 by every workgroup) are loaded ahead.
// The waves' partial tiles are summed in LDS in a fixed order (deterministic), then bias is added
// in fp32 and the result rounded once.
//
// Where the time goes (rocprofv3 SQ counters, gate_proj 14336 x 4096, M = 1): the weight
// stream alone runs at 4.7-4.9 TB/s (qdq disabled in a probe variant); the per-element INT /
// FP8 qdq (~12 VALU instructions per element: convert, scale, round, clamp, correctly rounded
// divide, convert back) brings it to 2.8-3.3 TB/s -- still one pass over W instead of the
// reference's three, 1.6-1.8x faster than qdq + hipBLASLt at M <= 16.
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

template <typename T> struct Mfma;
template <> struct Mfma<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <typename T>
__device__ __forceinline__ typename Mfma<T>::v8 as_v8(const Vec<T> &v) {
  typename Mfma<T>::v8 r;
  __builtin_memcpy(&r, &v.raw, 16);
  return r;
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
};

template <typename T, int KIND, int MT, int kQlWaves, int kQlU, int PROBE = 0>
__global__ __launch_bounds__(kQlWaves * 64) void qlinear_small_m_kernel(
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

  // Per-lane pointers advance by one 32-wide K step at a time; the amax index of a W element is
  // row_blk + s / spb (blocks tile whole K steps, so every lane of a step shares the K block and
  // s / spb is wave-uniform -- scalar arithmetic).  A first version divided the 64-bit element
  // index by the block size per step and spent most of its VALU issue on that division.
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
      if (PROBE != 1) qp.template apply<T>(wvec[u]);  // PROBE 1: no qdq (sweep only)
      if (PROBE == 2) {  // loads only: fold the raw bits into the accumulator
        acc[0][0] += __uint_as_float(wvec[u].raw.x ^ wvec[u].raw.y ^ wvec[u].raw.z ^ wvec[u].raw.w);
        continue;
      }
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

template <typename T, int KIND>
int launch_ql(const void *x, const void *w, const void *bias, void *y, int64_t M, int64_t N,
              int64_t K, const QlParams &p, hipStream_t stream) {
  const unsigned g = (unsigned)(N / 16);
  const T *xt = reinterpret_cast<const T *>(x);
  const T *wt = reinterpret_cast<const T *>(w);
  const T *bt = reinterpret_cast<const T *>(bias);
  T *yt = reinterpret_cast<T *>(y);
  static int var = -1;
  if (var < 0) {
    const char *e = getenv("MTQ_AMD_QLINEAR_VARIANT");
    var = e ? atoi(e) : 0;
  }
  switch (var) {
  case 1: qlinear_small_m_kernel<T, KIND, 1, 8, 4><<<g, 8 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 2: qlinear_small_m_kernel<T, KIND, 1, 4, 8><<<g, 4 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 3: qlinear_small_m_kernel<T, KIND, 1, 4, 4><<<g, 4 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 4: qlinear_small_m_kernel<T, KIND, 1, 16, 4><<<g, 16 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 5: qlinear_small_m_kernel<T, KIND, 1, 2, 8><<<g, 2 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 6: qlinear_small_m_kernel<T, KIND, 1, 16, 4, 1><<<g, 16 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 7: qlinear_small_m_kernel<T, KIND, 1, 16, 4, 2><<<g, 16 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  case 8: qlinear_small_m_kernel<T, KIND, 1, 8, 8><<<g, 8 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p); break;
  default:
    // measured (scripts/bench_qlinear.py, variant sweep): 16 waves x U = 4 when there are few
    // 16-row tiles (q/k/v/o, down_proj: 64-256 tiles), 8 waves x U = 4 when there are many
    // (gate/up_proj: 896 tiles)
    if ((int64_t)g >= 2 * (int64_t)mtq::host_num_cus())
      qlinear_small_m_kernel<T, KIND, 1, 8, 4><<<g, 8 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p);
    else
      qlinear_small_m_kernel<T, KIND, 1, 16, 4><<<g, 16 * 64, 0, stream>>>(xt, wt, bt, yt, M, N, K, p);
    break;
  }
  return host_check_launch();
}

bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

extern "C" int mtq_qlinear_small_m(const void *x, const void *w, const void *bias, void *y,
                                   int64_t M, int64_t N, int64_t K, int dtype, const void *amax,
                                   int amax_dtype, int64_t amax_numel, int64_t block, int kind,
                                   int num_bits, int is_unsigned, int narrow_range,
                                   hipStream_t stream) {
  if (M < 1 || M > 16 || N < 16 || N % 16 != 0 || K < 32 || K % 32 != 0) return MTQ_ERR_INVALID_ARG;
  if (!x || !w || !y || !amax || amax_numel < 1) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (amax_dtype < 0 || amax_dtype > 3) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(w)) return MTQ_ERR_INVALID_ARG;
  // per-tensor, or per-(row, block) with blocks that tile the 32-wide K steps
  if (amax_numel > 1 && (block < 32 || block % 32 != 0 || K % block != 0 || amax_numel * block != N * K))
    return MTQ_ERR_INVALID_ARG;
  if (kind != 0 && kind != 1) return MTQ_ERR_FORMAT;
  if (kind == 0 && (num_bits < 1 || num_bits > 31)) return MTQ_ERR_INVALID_ARG;
  QlParams p{amax, amax_dtype, amax_numel, block, 0.f, 0.f};
  if (kind == 0) {
    const float mb = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
    p.max_bound = mb;
    p.min_bound = is_unsigned ? 0.f : (narrow_range ? -mb : -mb - 1.f);
  }
  if (dtype == MTQ_BF16)
    return kind == 0 ? launch_ql<__bf16, 0>(x, w, bias, y, M, N, K, p, stream)
                     : launch_ql<__bf16, 1>(x, w, bias, y, M, N, K, p, stream);
  return kind == 0 ? launch_ql<_Float16, 0>(x, w, bias, y, M, N, K, p, stream)
                   : launch_ql<_Float16, 1>(x, w, bias, y, M, N, K, p, stream);
}
