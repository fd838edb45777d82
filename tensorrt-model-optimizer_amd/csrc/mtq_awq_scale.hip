// mtq_awq_scale.hip — the AWQ-lite scale statistics, bit-identical to the reference's CPU run.
//
// The awq_lite search (modelopt/torch/quantization/model_calib.py:1453-1487) reduces its inputs to
//     act_scale    = mean_rows(|x|)                         get_act_scale    :1471-1472
//     weight_scale = mean_rows(|W| / (block amax + tiny))   get_weight_scale :1453-1469
//     s(alpha)     = clamp(act^a / (w^(1-a) + tiny), 1e-4, 1e4) / sqrt(max * min)   get_scale :1474-1487
// On the GPU, torch's own `mean` sums in a tree order and multiplies by 1/M, and its `pow` is the
// device libm's -- each a few ulps away from what the same expressions give on the CPU, where
// the reference's golden runs (tests/golden/awq_b128.*) were made.  First diverging ops found
// (DESIGN.md §5): `pow` (the CPU's vectorised powf is not correctly rounded on ~1.5 % of the
// elements) and the two means (ATen's CPU cascade-sum order, then a true division by M).  The
// two kernels here restate exactly those CPU operation sequences, so the scale table -- and with
// it best_scale, the folded weights and the block amax -- reproduce the reference run bit for bit
// wherever the inputs to these statistics agree.
//
// 1. mtq_col_mean: ATen's CPU sum over dim 0 of a row-major [M, K] tensor (SumKernel.cpp,
//    vectorized_outer_sum), fp32 accumulation:
//      * columns in whole groups of 32 (two AVX-512 float vectors) -- one cascade per column over
//        the M rows;
//      * the K % 32 remaining columns -- `row_sum`: four interleaved cascades over rows
//        c, c + 4, c + 8, ... (M / 4 rows each), the M % 4 last rows added to the first, then
//        p0 + p1, + p2, + p3.
//    A cascade over S rows with step s = 2^max(4, ceil_log2(S) / 4) keeps four accumulators: rows
//    are summed sequentially from 0 in blocks of s (level 0); every finished block is added to
//    level 1, which is flushed into level 2 every s blocks, which is flushed into level 3 every s
//    level-1 flushes; the S % s last rows go to level 0, and the result is
//    ((l0 + l1) + l2) + l3.  Every level-1 value (s^2 rows) is independent: the first kernel
//    computes them in parallel (one lane per column, one wave per level-1 value), the second
//    replays the level-2 / level-3 / tail combination per column in the CPU's order.  The mean
//    is then T(sum / M) (true division, rounded to the input type, as ATen's CPU mean of a
//    16-bit tensor: fp32 sum, divide, cast).  Pinned against torch's CPU reductions in
//    tests/test_awq_cpu_order.py (host restatement) and tests/test_gpu_awq_b128.py (this kernel).
// 2. mtq_awq_scale_table: all G alphas' get_scale rows in one launch (one workgroup per alpha).
//    `pow` follows ATen's CPU pow(Tensor, Scalar) (Pow.cpp / PowKernel.cpp): exponent 0 -> 1,
//    1 -> copy, 0.5 -> sqrt, 2 / 3 -> products, -1 -> 1 / x, -2 -> 1 / x^2 (-0.5 -> rsqrt, here
//    1 / sqrt: not pinned, the alpha grid never reaches it);
//    any other exponent runs the vectorised powf on the elements the 32-wide vector loop covers
//    (the double-float log / exp evaluation restated below, checked bit for bit against torch's
//    CPU pow on every exponent of the alpha grid, tests/test_awq_cpu_order.py) and the scalar
//    std::pow(float, double) on the K % 32 tail elements (the exponent stays a double there: a
//    double evaluation rounded once to float, restated as exactly that).  Exponents arrive as
//    doubles: the special cases compare the double Scalar as ATen does, the vector loop uses
//    float(e).
//    Division and clamp are IEEE-exact on both sides; sqrt is corrected to the correctly rounded
//    value (sqrt_rn: the device sqrtf / __fsqrt_rn are the hardware approximation -- the first GPU
//    run of the table test found exactly that).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"

// every expression below is a restatement of a fixed CPU operation sequence: no contraction of
// a * b + c into fma unless written as fmaf
#pragma clang fp contract(off)

using namespace mtq;

namespace mtq {
int host_check_launch();
}

namespace {

// ----------------------------------------------------------------------------------------------
// 1. column mean in the CPU cascade order
// ----------------------------------------------------------------------------------------------
constexpr int kColGroup = 32;  // ATen's vectorised outer-sum column group (2 x 16 fp32 lanes)

struct Cascade {
  int64_t S;    // rows in the cascade
  int64_t s;    // level step
  int64_t nb0;  // full level-0 blocks
  int64_t nl1;  // level-1 entries (full + one partial group if any)
  __host__ __device__ int64_t entries() const { return nl1 + 1; }  // + the tail rows' sum
};

__host__ __device__ inline Cascade make_cascade(int64_t S) {
  int cl = 0;  // ceil(log2(S))
  while (cl < 62 && (int64_t(1) << cl) < S) ++cl;
  const int lp = cl / 4 > 4 ? cl / 4 : 4;
  Cascade c;
  c.S = S;
  c.s = int64_t(1) << lp;
  c.nb0 = S / c.s;
  c.nl1 = (c.nb0 + c.s - 1) / c.s;
  return c;
}

template <typename T, bool ABS>
__device__ __forceinline__ float ld_elem(const T *__restrict__ x, int64_t off) {
  float v = Elem<T>::ld(x[off]);
  return ABS ? fabsf(v) : v;
}

// Entry e of cascade (column k, rows r0 + j * rs, j in [0, S)): e < nl1 -> the level-1 value of
// level-0 blocks [e * s, min((e + 1) * s, nb0)); e == nl1 -> the sequential sum of the tail rows.
template <typename T, bool ABS>
__device__ float cascade_entry(const T *__restrict__ x, int64_t ld, int64_t k, int64_t r0, int64_t rs,
                               const Cascade &c, int64_t e) {
  if (e < c.nl1) {
    const int64_t b1 = e * c.s, b2 = (e + 1) * c.s < c.nb0 ? (e + 1) * c.s : c.nb0;
    float acc1 = 0.0f;
    for (int64_t b = b1; b < b2; ++b) {
      float acc0 = 0.0f;
      const int64_t j0 = b * c.s;
      if (c.s == 16) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = ld_elem<T, ABS>(x, (r0 + (j0 + r) * rs) * ld + k);
#pragma unroll
        for (int r = 0; r < 16; ++r) acc0 = acc0 + v[r];
      } else {
        for (int64_t r = 0; r < c.s; ++r) acc0 = acc0 + ld_elem<T, ABS>(x, (r0 + (j0 + r) * rs) * ld + k);
      }
      acc1 = acc1 + acc0;
    }
    return acc1;
  }
  float acc0 = 0.0f;
  for (int64_t j = c.nb0 * c.s; j < c.S; ++j) acc0 = acc0 + ld_elem<T, ABS>(x, (r0 + j * rs) * ld + k);
  return acc0;
}

__device__ float cascade_finish(const float *__restrict__ ent, int64_t stride, const Cascade &c) {
  const int64_t full = c.nb0 / c.s, part = c.nb0 % c.s;
  float acc2 = 0.0f, acc3 = 0.0f;
  for (int64_t g = 0; g < full; ++g) {
    acc2 = acc2 + ent[g * stride];
    if ((g + 1) % c.s == 0) {
      acc3 = acc3 + acc2;
      acc2 = 0.0f;
    }
  }
  const float acc1 = part > 0 ? ent[full * stride] : 0.0f;
  float acc0 = ent[c.nl1 * stride];
  acc0 = acc0 + acc1;
  acc0 = acc0 + acc2;
  acc0 = acc0 + acc3;
  return acc0;
}

constexpr int kColWaves = 4;

// scratch layout: main columns [em, K] (entry-major), tail columns [4, et, K]
template <typename T, bool ABS>
__global__ __launch_bounds__(64 * kColWaves) void colmean_entries_kernel(const T *__restrict__ x, int64_t M,
                                                                          int64_t K, int64_t kmain,
                                                                          float *__restrict__ scratch) {
  const int64_t k = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
  const int64_t u = (int64_t)blockIdx.y * kColWaves + (threadIdx.x >> 6);  // entry unit
  if (k >= K) return;
  if (k < kmain) {
    const Cascade c = make_cascade(M);
    if (u < c.entries()) scratch[u * K + k] = cascade_entry<T, ABS>(x, K, k, 0, 1, c, u);
  } else {
    const Cascade c = make_cascade(M / 4);
    const int64_t et = c.entries();
    if (u < 4 * et) {
      const int64_t ci = u / et, e = u % et;
      float *base = scratch + make_cascade(M).entries() * K;
      base[(ci * et + e) * K + k] = cascade_entry<T, ABS>(x, K, k, ci, 4, c, e);
    }
  }
}

template <typename T, bool ABS>
__global__ __launch_bounds__(256) void colmean_finish_kernel(const T *__restrict__ x, int64_t M, int64_t K,
                                                             int64_t kmain, const float *__restrict__ scratch,
                                                             float *__restrict__ y) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const Cascade cm = make_cascade(M);
  float sum;
  if (k < kmain) {
    sum = cascade_finish(scratch + k, K, cm);
  } else {
    const Cascade c = make_cascade(M / 4);
    const int64_t et = c.entries();
    const float *base = scratch + cm.entries() * K;
    float p[4];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci) p[ci] = cascade_finish(base + ci * et * K + k, K, c);
    for (int64_t i = (M / 4) * 4; i < M; ++i) p[0] = p[0] + ld_elem<T, ABS>(x, i * K + k);
    sum = p[0];
    sum = sum + p[1];
    sum = sum + p[2];
    sum = sum + p[3];
  }
  const float mean = __fdiv_rn(sum, (float)M);
  y[k] = Elem<T>::ld(Elem<T>::st(mean));
}

// ----------------------------------------------------------------------------------------------
// 2. get_scale table with the CPU's pow
// ----------------------------------------------------------------------------------------------
struct F2 {
  float x, y;
};
__device__ __forceinline__ F2 mk(float x, float y) { return F2{x, y}; }
__device__ __forceinline__ float fmapn(float x, float y, float z) { return fmaf(x, y, -z); }
__device__ __forceinline__ float fmanp(float x, float y, float z) { return fmaf(-x, y, z); }
__device__ __forceinline__ F2 df_add2_ff(float x, float y) {
  const float s = x + y, v = s - x;
  return mk(s, (x - (s - v)) + (y - v));
}
__device__ __forceinline__ F2 df_add_f2f2(F2 x, F2 y) {  // |x| >= |y|
  const float s = x.x + y.x;
  return mk(s, (((x.x - s) + y.x) + x.y) + y.y);
}
__device__ __forceinline__ F2 df_add2_f2f(F2 x, float y) {
  const float s = x.x + y, v = s - x.x;
  const float t = (x.x - (s - v)) + (y - v);
  return mk(s, t + x.y);
}
__device__ __forceinline__ F2 df_add_ff2(float x, F2 y) {
  const float s = x + y.x;
  return mk(s, ((x - s) + y.x) + y.y);
}
__device__ __forceinline__ F2 df_add2_f2f2(F2 x, F2 y) {
  const float s = x.x + y.x, v = s - x.x;
  const float t = (x.x - (s - v)) + (y.x - v);
  return mk(s, t + (x.y + y.y));
}
__device__ __forceinline__ F2 df_scale(F2 d, float s) { return mk(d.x * s, d.y * s); }
__device__ __forceinline__ F2 df_normalize(F2 t) {
  const float s = t.x + t.y;
  return mk(s, (t.x - s) + t.y);
}
__device__ __forceinline__ F2 df_mul_f2f(F2 x, float y) {
  const float s = x.x * y;
  return mk(s, fmaf(x.y, y, fmapn(x.x, y, s)));
}
__device__ __forceinline__ F2 df_mul_f2f2(F2 x, F2 y) {
  const float s = x.x * y.x;
  return mk(s, fmaf(x.x, y.y, fmaf(x.y, y.x, fmapn(x.x, y.x, s))));
}
__device__ __forceinline__ F2 df_squ(F2 x) {
  const float s = x.x * x.x;
  return mk(s, fmaf(x.x + x.x, x.y, fmapn(x.x, x.x, s)));
}
__device__ __forceinline__ F2 df_div(F2 n, F2 d) {
  const float t = __fdiv_rn(1.0f, d.x);
  const float s = n.x * t;
  const float u = fmapn(t, n.x, s);
  const float v = fmanp(d.y, t, fmanp(d.x, t, 1.0f));
  return mk(s, fmaf(s, v, fmaf(n.y, t, u)));
}

// log(d) in double-float for d > 0 finite: mantissa in [0.75, 1.5) (the AVX-512 getmant form),
// exponent from d * (1 / 0.75)
__device__ F2 log_df(float d) {
  const float e = (float)ilogbf(d * (1.0f / 0.75f));
  int ex;
  float m = frexpf(d, &ex) * 2.0f;  // [1, 2), exact
  if (m >= 1.5f) m = m * 0.5f;
  const F2 x = df_div(df_add2_ff(-1.0f, m), df_add2_ff(1.0f, m));
  const F2 x2 = df_squ(x);
  float t = 0.240320354700088500976562f;
  t = fmaf(t, x2.x, 0.285112679004669189453125f);
  t = fmaf(t, x2.x, 0.400007992982864379882812f);
  const F2 c = mk(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
  F2 s = df_mul_f2f(mk(0.69314718246459960938f, -1.904654323148236017e-09f), e);
  s = df_add_f2f2(s, df_scale(x, 2.0f));
  s = df_add_f2f2(s, df_mul_f2f2(df_mul_f2f2(x2, x), df_add2_f2f2(df_mul_f2f(x2, t), c)));
  return s;
}

__device__ float exp_df(F2 d) {
  float u = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
  const int q = (int)rintf(u);
  F2 s = df_add2_f2f(d, (float)q * -0.693145751953125f);
  s = df_add2_f2f(s, (float)q * -1.428606765330187045e-06f);
  s = df_normalize(s);
  u = 0.00136324646882712841033936f;
  u = fmaf(u, s.x, 0.00836596917361021041870117f);
  u = fmaf(u, s.x, 0.0416710823774337768554688f);
  u = fmaf(u, s.x, 0.166665524244308471679688f);
  u = fmaf(u, s.x, 0.499999850988388061523438f);
  F2 t = df_add_f2f2(s, df_mul_f2f(df_squ(s), u));
  t = df_add_ff2(1.0f, t);
  u = ldexpf(t.x + t.y, q);
  return d.x < -104.0f ? 0.0f : u;
}

// the CPU's vectorised powf for the finite / positive cases, its IEEE special cases otherwise
__device__ float pow_vec(float x, float y) {
  if (isnan(x) || isnan(y)) return x == 1.0f || y == 0.0f ? 1.0f : __int_as_float(0x7fc00000);
  if (y == 0.0f || x == 1.0f) return 1.0f;
  const float ax = fabsf(x);
  if (x == 0.0f || isinf(x) || isinf(y)) return powf(x, y);  // IEEE special values (exact)
  float r = exp_df(df_mul_f2f(log_df(ax), y));
  if (isnan(r)) r = __int_as_float(0x7f800000);
  if (x < 0.0f) {
    const bool yint = truncf(y) == y || fabsf(y) >= 16777216.0f;
    const bool yodd = yint && fabsf(y) < 16777216.0f && (((int)truncf(y)) & 1);
    r = yint ? (yodd ? -r : r) : __int_as_float(0x7fc00000);
  }
  return r;
}

// correctly rounded fp32 sqrt: the device sqrtf is the hardware approximation (within 1 ulp;
// the first table test on the MI355X differed from the CPU's in the normalisation sqrt(max * min))
// -- corrected against the exact square of the neighbouring midpoint (25 bits, exact in double)
__device__ float sqrt_rn(float x) {
  float r = sqrtf(x);
  if (!(x > 0.0f) || isinf(x) || !(r > 0.0f) || isinf(r)) return r;
  const double xd = (double)x;
  const float lo = __int_as_float(__float_as_int(r) - 1);
  const double ml = 0.5 * ((double)lo + (double)r);
  if (xd < ml * ml) return lo;
  const float hi = __int_as_float(__float_as_int(r) + 1);
  const double mh = 0.5 * ((double)r + (double)hi);
  return xd > mh * mh ? hi : r;
}

// pow(Tensor, Scalar) of ATen's CPU kernel at element index i of a K-long contiguous tensor
__device__ float pow_cpu(float x, double e, int64_t i, int64_t kvec) {
  if (e == 0.0) return 1.0f;
  if (e == 1.0) return x;
  if (e == 0.5) return sqrt_rn(x);
  if (e == 2.0) return x * x;
  if (e == 3.0) return x * x * x;
  if (e == -0.5) return __fdiv_rn(1.0f, sqrt_rn(x));
  if (e == -1.0) return __fdiv_rn(1.0f, x);
  if (e == -2.0) return __fdiv_rn(1.0f, x * x);
  const float ef = (float)e;
  if (i < kvec) return pow_vec(x, ef);
  return (float)pow((double)x, e);  // the tail: std::pow(float, double), double exponent, one rounding
}

__device__ __forceinline__ float clampf_nan(float v, float lo, float hi) {
  if (isnan(v)) return v;
  v = v < lo ? lo : v;
  return v > hi ? hi : v;
}

constexpr int kTabThreads = 1024;

__global__ __launch_bounds__(kTabThreads) void awq_scale_table_kernel(const float *__restrict__ x_max,
                                                                       const float *__restrict__ w_max, int64_t K,
                                                                       const double *__restrict__ e_num,
                                                                       const double *__restrict__ e_den,
                                                                       float *__restrict__ out) {
  const int g = blockIdx.x;
  const double en = e_num[g], ed = e_den[g];
  const int64_t kvec = K / kColGroup * kColGroup;
  float *row = out + (int64_t)g * K;
  float mx = -INFINITY, mn = INFINITY;
  bool nan = false;
  const float tiny = 1.17549435082228750797e-38f;
  for (int64_t k = threadIdx.x; k < K; k += kTabThreads) {
    const float num = pow_cpu(x_max[k], en, k, kvec);
    const float den = pow_cpu(w_max[k], ed, k, kvec) + tiny;
    const float v = clampf_nan(__fdiv_rn(num, den), 9.99999974737875163555e-05f, 10000.0f);
    row[k] = v;
    nan |= isnan(v);
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
  __shared__ float smx[kTabThreads / 64], smn[kTabThreads / 64];
  __shared__ int snan[kTabThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    mn = fminf(mn, __shfl_xor(mn, o, 64));
  }
  const unsigned long long anynan = __ballot(nan);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smx[w] = mx;
    smn[w] = mn;
    snan[w] = anynan != 0ull;
  }
  __syncthreads();
  mx = smx[0];
  mn = smn[0];
  int anyn = snan[0];
  for (int i = 1; i < kTabThreads / 64; ++i) {
    mx = fmaxf(mx, smx[i]);
    mn = fminf(mn, smn[i]);
    anyn |= snan[i];
  }
  // torch.max / min propagate NaN
  const float norm = anyn ? __int_as_float(0x7fc00000) : sqrt_rn(mx * mn);
  for (int64_t k = threadIdx.x; k < K; k += kTabThreads) row[k] = __fdiv_rn(row[k], norm);
}

}  // namespace

extern "C" {

int64_t mtq_col_mean_workspace_floats(int64_t M, int64_t K) {
  if (M < 1 || K < 0) return -1;
  return (make_cascade(M).entries() + 4 * make_cascade(M / 4).entries()) * K;
}

int mtq_col_mean(const void *x, int64_t M, int64_t K, int dtype, int absval, float *workspace,
                 int64_t workspace_floats, float *y, hipStream_t stream) {
  if (M < 1 || K < 0 || (K > 0 && (!x || !y || !workspace))) return MTQ_ERR_INVALID_ARG;
  if (K == 0) return MTQ_OK;
  if (workspace_floats < mtq_col_mean_workspace_floats(M, K)) return MTQ_ERR_INVALID_ARG;
  const int64_t kmain = K / kColGroup * kColGroup;
  const Cascade cm = make_cascade(M), ct = make_cascade(M / 4);
  const int64_t units = kmain > 0 ? cm.entries() : 0;
  const int64_t tunits = kmain < K ? 4 * ct.entries() : 0;
  const int64_t u = units > tunits ? units : tunits;
  const dim3 grid((unsigned)((K + 63) / 64), (unsigned)((u + kColWaves - 1) / kColWaves));
  const unsigned gf = (unsigned)((K + 255) / 256);
  auto run = [&](auto t) -> int {
    using T = decltype(t);
    const T *xt = reinterpret_cast<const T *>(x);
    if (absval) {
      colmean_entries_kernel<T, true><<<grid, 64 * kColWaves, 0, stream>>>(xt, M, K, kmain, workspace);
      colmean_finish_kernel<T, true><<<gf, 256, 0, stream>>>(xt, M, K, kmain, workspace, y);
    } else {
      colmean_entries_kernel<T, false><<<grid, 64 * kColWaves, 0, stream>>>(xt, M, K, kmain, workspace);
      colmean_finish_kernel<T, false><<<gf, 256, 0, stream>>>(xt, M, K, kmain, workspace, y);
    }
    return host_check_launch();
  };
  switch (dtype) {
    case MTQ_F32: return run(float{});
    case MTQ_F16: return run(_Float16{});
    case MTQ_BF16: return run(__bf16{});
    default: return MTQ_ERR_DTYPE;
  }
}

int mtq_awq_scale_table(const float *x_max, const float *w_max, int64_t K, const double *e_num,
                        const double *e_den, int G, float *scales, hipStream_t stream) {
  if (K < 1 || G < 0 || (G > 0 && (!x_max || !w_max || !e_num || !e_den || !scales))) return MTQ_ERR_INVALID_ARG;
  if (G == 0) return MTQ_OK;
  awq_scale_table_kernel<<<(unsigned)G, kTabThreads, 0, stream>>>(x_max, w_max, K, e_num, e_den, scales);
  return host_check_launch();
}

}  // extern "C"
