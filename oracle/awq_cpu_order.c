/* Test infrastructure (oracle): a host restatement of the two CPU operation sequences the AWQ-lite
 * statistics of the reference's CPU run depend on -- NOT product code; only tests/ load it.
 *
 *  - oracle_powf: ATen's vectorised powf (torch CPU pow(Tensor, Scalar) for exponents other than
 *    0, 1, 0.5, 2, 3, -0.5, -1, -2): log in double-float (mantissa in [0.75, 1.5)), product with
 *    the exponent in double-float, exp in double-float, one final rounding.  Used by get_scale
 *    (reference modelopt/torch/quantization/model_calib.py:1474-1487).
 *  - oracle_col_sum: ATen's CPU sum over dim 0 of a row-major fp32 [M, K] array
 *    (SumKernel.cpp vectorized_outer_sum / row_sum cascade order), used by the means of
 *    get_act_scale / get_weight_scale (:1453-1472).
 *
 * tests/test_awq_cpu_order.py pins both against torch's own CPU ops; csrc/mtq_awq_scale.hip is
 * the device restatement of the same sequences.  Build: gcc -O2 -ffp-contract=off -shared -fPIC
 * (no contraction: every fused multiply-add below is written as fmaf). */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct { float x, y; } f2;
static inline f2 mk(float x, float y) { f2 r = {x, y}; return r; }
static inline float fmapn(float x, float y, float z) { return fmaf(x, y, -z); }
static inline float fmanp(float x, float y, float z) { return fmaf(-x, y, z); }
static inline f2 add2_ff(float x, float y) { float s = x + y, v = s - x; return mk(s, (x - (s - v)) + (y - v)); }
static inline f2 add_f2f2(f2 x, f2 y) { float s = x.x + y.x; return mk(s, (((x.x - s) + y.x) + x.y) + y.y); }
static inline f2 add2_f2f(f2 x, float y) { float s = x.x + y, v = s - x.x; return mk(s, ((x.x - (s - v)) + (y - v)) + x.y); }
static inline f2 add_ff2(float x, f2 y) { float s = x + y.x; return mk(s, ((x - s) + y.x) + y.y); }
static inline f2 add2_f2f2(f2 x, f2 y) { float s = x.x + y.x, v = s - x.x; return mk(s, ((x.x - (s - v)) + (y.x - v)) + (x.y + y.y)); }
static inline f2 scale2(f2 d, float s) { return mk(d.x * s, d.y * s); }
static inline f2 normalize2(f2 t) { float s = t.x + t.y; return mk(s, (t.x - s) + t.y); }
static inline f2 mul_f2f(f2 x, float y) { float s = x.x * y; return mk(s, fmaf(x.y, y, fmapn(x.x, y, s))); }
static inline f2 mul_f2f2(f2 x, f2 y) { float s = x.x * y.x; return mk(s, fmaf(x.x, y.y, fmaf(x.y, y.x, fmapn(x.x, y.x, s)))); }
static inline f2 squ2(f2 x) { float s = x.x * x.x; return mk(s, fmaf(x.x + x.x, x.y, fmapn(x.x, x.x, s))); }
static inline f2 div2(f2 n, f2 d) {
  float t = 1.0f / d.x, s = n.x * t, u = fmapn(t, n.x, s);
  float v = fmanp(d.y, t, fmanp(d.x, t, 1.0f));
  return mk(s, fmaf(s, v, fmaf(n.y, t, u)));
}

static f2 log_df(float d) {
  float e = (float)ilogbf(d * (1.0f / 0.75f));
  int ex;
  float m = frexpf(d, &ex) * 2.0f;
  if (m >= 1.5f) m *= 0.5f;
  f2 x = div2(add2_ff(-1.0f, m), add2_ff(1.0f, m)), x2 = squ2(x);
  float t = 0.240320354700088500976562f;
  t = fmaf(t, x2.x, 0.285112679004669189453125f);
  t = fmaf(t, x2.x, 0.400007992982864379882812f);
  f2 c = mk(0.66666662693023681640625f, 3.69183861259614332084311e-09f);
  f2 s = mul_f2f(mk(0.69314718246459960938f, -1.904654323148236017e-09f), e);
  s = add_f2f2(s, scale2(x, 2.0f));
  return add_f2f2(s, mul_f2f2(mul_f2f2(x2, x), add2_f2f2(mul_f2f(x2, t), c)));
}

static float exp_df(f2 d) {
  float u = (d.x + d.y) * 1.442695040888963407359924681001892137426645954152985934135449406931f;
  int q = (int)rintf(u);
  f2 s = add2_f2f(d, (float)q * -0.693145751953125f);
  s = normalize2(add2_f2f(s, (float)q * -1.428606765330187045e-06f));
  u = 0.00136324646882712841033936f;
  u = fmaf(u, s.x, 0.00836596917361021041870117f);
  u = fmaf(u, s.x, 0.0416710823774337768554688f);
  u = fmaf(u, s.x, 0.166665524244308471679688f);
  u = fmaf(u, s.x, 0.499999850988388061523438f);
  f2 t = add_ff2(1.0f, add_f2f2(s, mul_f2f(squ2(s), u)));
  u = ldexpf(t.x + t.y, q);
  return d.x < -104.0f ? 0.0f : u;
}

/* x > 0 finite (the AWQ statistics' domain) */
float oracle_powf(float x, float y) { return exp_df(mul_f2f(log_df(fabsf(x)), y)); }

void oracle_powf_array(const float *x, int64_t n, float y, float *out) {
  for (int64_t i = 0; i < n; ++i) out[i] = oracle_powf(x[i], y);
}

/* one cascade over rows r0 + j * rs (j < S) of column k */
static float cascade(const float *a, int64_t ld, int64_t k, int64_t r0, int64_t rs, int64_t S) {
  int cl = 0;
  while (cl < 62 && ((int64_t)1 << cl) < S) ++cl;
  const int lp = cl / 4 > 4 ? cl / 4 : 4;
  const int64_t step = (int64_t)1 << lp, mask = step - 1;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  int64_t i = 0;
  while (i + step <= S) {
    for (int64_t j = 0; j < step; ++j, ++i) acc[0] = acc[0] + a[(r0 + i * rs) * ld + k];
    for (int j = 1; j < 4; ++j) {
      acc[j] = acc[j] + acc[j - 1];
      acc[j - 1] = 0.0f;
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < S; ++i) acc[0] = acc[0] + a[(r0 + i * rs) * ld + k];
  for (int j = 1; j < 4; ++j) acc[0] = acc[0] + acc[j];
  return acc[0];
}

void oracle_col_sum(const float *a, int64_t M, int64_t K, float *out) {
  const int64_t kmain = K / 32 * 32;
  for (int64_t k = 0; k < K; ++k) {
    if (k < kmain) {
      out[k] = cascade(a, K, k, 0, 1, M);
    } else {
      const int64_t n4 = M / 4;
      float p[4];
      for (int c = 0; c < 4; ++c) p[c] = cascade(a, K, k, c, 4, n4);
      for (int64_t i = n4 * 4; i < M; ++i) p[0] = p[0] + a[i * K + k];
      out[k] = ((p[0] + p[1]) + p[2]) + p[3];
    }
  }
}
