// mtq_cpu.cpp — host (CPU) kernels of the C1 path: INT-n and FP8 e4m3 fake quant, amax reduction.
//
// The reference registers its ops for ["cpu", "cuda"] (tensor_quant.py:252-256): on a CPU tensor
// it runs the eager ATen sequences `_tensor_quant` (tensor_quant.py:607-645) and `_fp8_eager`
// (:46-59), and `reduce_amax` (utils/core_utils.py:146-183).  These are the product's own CPU
// kernels for the same arithmetic (single pass, multi-threaded), so `mtq.quantize` on a CPU model
// (BASELINE config C1: nn.Linear(1024, 1024), INT8_DEFAULT_CFG) runs without a GPU.  Bit-exact
// with the reference's CPU ops: all math in fp32 with IEEE division (x86 `divss`), rint = ties to
// even (torch.round_), NaN-propagating clamps, fp32 -> e4m3fn RNE by the exact power-of-two
// quantum, fp32 -> f16/bf16 by the compiler's RNE conversions.  Not an oracle: nothing here is
// imported from oracle/, which checks these results in tests/test_cpu_path.py.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "mtq_amd.h"

namespace {

constexpr float kEps = 1.0f / (1 << 24);  // tensor_quant.py: amax <= 2^-24 counts as zero
constexpr float kE4M3Max = 448.0f;

template <typename T> struct H;
template <> struct H<float> {
  static float ld(float v) { return v; }
  static float st(float v) { return v; }
};
template <> struct H<double> {
  static float ld(double v) { return (float)v; }  // inputs.float()
  static double st(float v) { return (double)v; }
};
template <> struct H<_Float16> {
  static float ld(_Float16 v) { return (float)v; }
  static _Float16 st(float v) { return (_Float16)v; }
};
template <> struct H<__bf16> {
  static float ld(__bf16 v) { return (float)v; }
  static __bf16 st(float v) { return (__bf16)v; }
};

// torch.clamp(NaN) is NaN
inline float clamp_nan(float v, float lo, float hi) {
  if (v != v) return v;
  return v < lo ? lo : (v > hi ? hi : v);
}

// fp32 -> e4m3fn (RNE) -> fp32 for |v| <= 448 or NaN: the e4m3 grid in the binade of v has the
// quantum 2^(e-3) (normal, e >= -6) or 2^-9 (subnormal); v / q is exact (power of two), rint
// rounds half to even on the mantissa, and a carry into the next binade lands on its grid.
inline float e4m3_round(float v) {
  if (v != v) return v;
  const float a = fabsf(v);
  if (a == 0.f) return v;
  int e;
  frexpf(a, &e);  // a = m * 2^e, m in [0.5, 1)  ->  binade exponent e - 1
  const int eb = std::max(e - 1, -6);
  const float q = ldexpf(1.0f, eb - 3);
  return rintf(v / q) * q;
}

template <typename Fn> void parallel(int64_t n, int nthreads, Fn fn, int64_t grain = 1 << 16) {
  int t = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  grain = std::max<int64_t>(1, grain);
  t = (int)std::max<int64_t>(1, std::min<int64_t>(t, (n + grain - 1) / grain));
  if (t <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(t);
  const int64_t per = (n + t - 1) / t;
  for (int i = 0; i < t; ++i) {
    const int64_t b = i * per, e = std::min(n, b + per);
    if (b >= e) break;
    th.emplace_back([=] { fn(b, e); });
  }
  for (auto &x : th) x.join();
}

struct IntP {
  float s, d, lo, hi;
};
inline IntP int_param(float amax, float mb, float lo) {
  // scale = max_bound / amax; amax <= eps -> scale 0 for the multiply, 1 for the divide
  if (amax <= kEps) return {0.f, 1.f, lo, mb};
  const float s = mb / amax;
  return {s, s, lo, mb};
}

template <typename T>
void int_qdq(const T *x, T *y, int64_t n, const float *amax, int64_t axis, int64_t inner, float mb,
             float lo, int nthreads) {
  parallel(n, nthreads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e;) {
      const int64_t c = axis == 1 ? 0 : (i / inner) % axis;
      const int64_t run_end = axis == 1 ? e : std::min(e, (i / inner + 1) * inner);
      const IntP p = int_param(amax[c], mb, lo);
      for (; i < run_end; ++i) {
        float v = rintf(H<T>::ld(x[i]) * p.s);
        v = clamp_nan(v, p.lo, p.hi);
        y[i] = H<T>::st(v / p.d);
      }
    }
  });
}

template <typename T>
void fp8_qdq(const T *x, T *y, int64_t n, const float *amax, int64_t axis, int64_t inner,
             int nthreads) {
  parallel(n, nthreads, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e;) {
      const int64_t c = (amax == nullptr || axis == 1) ? 0 : (i / inner) % axis;
      const int64_t run_end =
          (amax == nullptr || axis == 1) ? e : std::min(e, (i / inner + 1) * inner);
      if (amax == nullptr) {  // plain cast round trip (_fp8_eager with amax=None)
        for (; i < run_end; ++i) {
          const float v = H<T>::ld(x[i]);
          // torch's float8_e4m3fn cast: RNE to the grid, (464, inf] -> NaN (464 ties to 448)
          y[i] = H<T>::st(fabsf(v) > 464.0f ? NAN : e4m3_round(v));
        }
        continue;
      }
      const float safe = amax[c] <= kEps ? 1.0f : amax[c];
      // `448.0 / safe` is Tensor.__rtruediv__ = reciprocal(safe) * 448; `1 / scale` likewise
      const float s = (1.0f / safe) * kE4M3Max;
      const float inv = 1.0f / s;
      for (; i < run_end; ++i) {
        const float v = clamp_nan(H<T>::ld(x[i]) * s, -kE4M3Max, kE4M3Max);
        y[i] = H<T>::st(e4m3_round(v) * inv);
      }
    }
  });
}

// out[k] = max(out[k], max_{p,q} |x[p,k,q]|), NaN-propagating (torch.amax semantics).  Each
// thread owns whole output entries (a chunk of k) when there are enough of them, else whole
// entries are split over threads and the partial maxima folded in thread order: no atomics.
inline float fold_abs(float m, float v) {
  const float a = fabsf(v);
  return (a != a || m != m) ? NAN : (a > m ? a : m);
}

template <typename T>
void reduce_amax(const T *x, int64_t P, int64_t K, int64_t Q, float *out, int nthreads) {
  const int64_t KQ = K * Q;
  int t = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  t = std::max(1, t);
  if (K >= t) {
    parallel(K, t, [&](int64_t k0, int64_t k1) {
      std::vector<float> m(out + k0, out + k1);
      for (int64_t p = 0; p < P; ++p) {
        const T *row = x + p * KQ;
        for (int64_t k = k0; k < k1; ++k)
          for (int64_t q = 0; q < Q; ++q) m[k - k0] = fold_abs(m[k - k0], H<T>::ld(row[k * Q + q]));
      }
      std::copy(m.begin(), m.end(), out + k0);
    }, (1 << 16) / std::max<int64_t>(1, P * Q));
    return;
  }
  for (int64_t k = 0; k < K; ++k) {
    const int64_t n = P * Q;
    const int64_t per = (n + t - 1) / t;
    std::vector<float> part(t, 0.f);
    parallel(t, t, [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i) {
        float m = 0.f;
        const int64_t b = i * per, e = std::min(n, b + per);
        for (int64_t j = b; j < e; ++j) m = fold_abs(m, H<T>::ld(x[(j / Q) * KQ + k * Q + j % Q]));
        part[i] = m;
      }
    }, 1);
    float m = out[k];
    for (float v : part) m = (v != v || m != m) ? NAN : (v > m ? v : m);
    out[k] = m;
  }
}

template <template <typename> class F, typename... A> int dispatch(int dtype, A... a) {
  switch (dtype) {
  case MTQ_F32: F<float>::run(a...); return MTQ_OK;
  case MTQ_F16: F<_Float16>::run(a...); return MTQ_OK;
  case MTQ_BF16: F<__bf16>::run(a...); return MTQ_OK;
  case MTQ_F64: F<double>::run(a...); return MTQ_OK;
  default: return MTQ_ERR_DTYPE;
  }
}

template <typename T> struct IntRun {
  static void run(const void *x, void *y, int64_t n, const float *amax, int64_t axis,
                  int64_t inner, float mb, float lo, int nt) {
    int_qdq<T>((const T *)x, (T *)y, n, amax, axis, inner, mb, lo, nt);
  }
};
template <typename T> struct Fp8Run {
  static void run(const void *x, void *y, int64_t n, const float *amax, int64_t axis,
                  int64_t inner, int nt) {
    fp8_qdq<T>((const T *)x, (T *)y, n, amax, axis, inner, nt);
  }
};
template <typename T> struct AmaxRun {
  static void run(const void *x, int64_t P, int64_t K, int64_t Q, float *out, int nt) {
    reduce_amax<T>((const T *)x, P, K, Q, out, nt);
  }
};

}  // namespace

extern "C" int mtq_cpu_fake_tensor_quant(const void *x, void *y, int64_t n, int dtype,
                                         const float *amax, int64_t axis_size, int64_t inner,
                                         int num_bits, int is_unsigned, int narrow_range,
                                         int nthreads) {
  if (n < 0 || (n > 0 && (!x || !y || !amax)) || axis_size < 1 || inner < 1) return MTQ_ERR_INVALID_ARG;
  if (num_bits < 1 || num_bits > 31) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  const float mb = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
  const float lo = is_unsigned ? 0.f : (narrow_range ? -mb : -mb - 1.f);
  return dispatch<IntRun>(dtype, x, y, n, amax, axis_size, inner, mb, lo, nthreads);
}

extern "C" int mtq_cpu_fake_e4m3fy(const void *x, void *y, int64_t n, int dtype, const float *amax,
                                   int64_t axis_size, int64_t inner, int nthreads) {
  if (n < 0 || (n > 0 && (!x || !y)) || axis_size < 1 || inner < 1) return MTQ_ERR_INVALID_ARG;
  if (n == 0) return MTQ_OK;
  return dispatch<Fp8Run>(dtype, x, y, n, amax, axis_size, inner, nthreads);
}

extern "C" int mtq_cpu_reduce_amax(const void *x, int64_t P, int64_t K, int64_t Q, int dtype,
                                   float *out, int nthreads) {
  if (P < 0 || K < 0 || Q < 0 || (P * K * Q > 0 && (!x || !out))) return MTQ_ERR_INVALID_ARG;
  if (P * K * Q == 0) return MTQ_OK;
  return dispatch<AmaxRun>(dtype, x, P, K, Q, out, nthreads);
}
