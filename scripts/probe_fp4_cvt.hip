// Probe of the gfx950 OCP FP4 converts against the reference E2M1 rounding
// (modelopt/torch/quantization/src/tensor_quant_mx.h:104-141: table walk, ties to the even
// index == ties-to-even mantissa, saturate at 6, NaN -> 6).
//
// For every bf16 bit pattern (as fp32) and a set of fp32 edge values, times scales 2^k, it runs
//   v_cvt_scalef32_pk_fp4_f32 (down, with the scale operand) and
//   v_cvt_scalef32_pk_f32_fp4 (up, scale 1)
// and compares the decoded value with the host E2M1 rounding of x * scale and of x / scale, to
// establish (1) which way the scale operand applies, (2) the rounding mode, (3) saturation,
// NaN / inf and signed-zero behaviour.
//
//   hipcc --offload-arch=gfx950 -O2 -o scripts/probe_fp4_cvt scripts/probe_fp4_cvt.hip
//   ./scripts/probe_fp4_cvt
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void up_scaled(const uint32_t *codes, int np, float scale, float *out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np) return;
  auto v = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(codes[i], scale, 0);
  out[2 * i] = v[0];
  out[2 * i + 1] = v[1];
}

__global__ void down_up(const float *x, int n, float scale, uint32_t *codes, float *back) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n + 1) return;
  float a = x[2 * i], b = (2 * i + 1 < n) ? x[2 * i + 1] : 0.f;
  uint32_t p = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, a, b, scale, 0);
  codes[i] = p;
  auto v = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(p, 1.0f, 0);
  back[2 * i] = v[0];
  if (2 * i + 1 < n) back[2 * i + 1] = v[1];
}

static float e2m1_round(float v) {  // v >= 0 or NaN
  if (v != v) return 6.f;
  const float grid[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
  if (v >= 6.f) return 6.f;
  for (int k = 0; k < 7; ++k) {
    float lo = grid[k], hi = grid[k + 1], mid = 0.5f * (lo + hi);
    if (v < hi) {
      if (v < mid) return lo;
      if (v > mid) return hi;
      return (k % 2 == 0) ? lo : hi;  // tie: even index
    }
  }
  return 6.f;
}

static float bf2f(uint32_t m) {
  uint32_t u = m << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

int main() {
  std::vector<float> xs;
  for (uint32_t m = 0; m < 65536; ++m) xs.push_back(bf2f(m));
  const float edges[] = {0.25f, 0.75f, 1.25f, 1.75f, 2.5f, 3.5f, 5.f, 6.f, 7.f, 0.5f, 3.f};
  for (float e : edges)
    for (int d = -2; d <= 2; ++d) {
      float v = e;
      for (int k = 0; k < (d < 0 ? -d : d); ++k) v = nextafterf(v, d < 0 ? 0.f : 100.f);
      xs.push_back(v);
      xs.push_back(-v);
    }
  xs.push_back(INFINITY);
  xs.push_back(-INFINITY);
  xs.push_back(NAN);
  xs.push_back(-NAN);
  xs.push_back(1e-40f);  // subnormal fp32
  xs.push_back(-1e-40f);
  const int n = (int)xs.size();
  const int np = (n + 1) / 2;
  float *dx, *dback;
  uint32_t *dcodes;
  hipMalloc(&dx, n * 4);
  hipMalloc(&dback, (size_t)np * 2 * 4);
  hipMalloc(&dcodes, np * 4);
  hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
  const float scales[] = {1.f, 2.f, 0.5f, 0x1p-10f, 0x1p10f, 0x1p-126f, 3.f};
  std::vector<float> back(np * 2);
  std::vector<uint32_t> codes(np);
  for (float s : scales) {
    down_up<<<(np + 255) / 256, 256>>>(dx, n, s, dcodes, dback);
    hipMemcpy(back.data(), dback, np * 2 * 4, hipMemcpyDeviceToHost);
    hipMemcpy(codes.data(), dcodes, np * 4, hipMemcpyDeviceToHost);
    long mul_bad = 0, div_bad = 0, sz_diff = 0, finite = 0;
    long nan_report = 0;
    for (int i = 0; i < n; ++i) {
      float x = xs[i];
      float got = back[i];
      float ax = fabsf(x);
      float want_mul = copysignf(e2m1_round(ax * s), x);
      float want_div = copysignf(e2m1_round(ax / s), x);
      if (x != x || std::isinf(x)) {
        if (i >= 65536 && (s == 1.f || s == 0x1p10f))
          printf("  scale %a special x=%a -> code %x back %a\n", s, x,
                 (codes[i / 2] >> (4 * (i % 2))) & 0xf, got);
        ++nan_report;
        continue;
      }
      ++finite;
      if (fbits(got) != fbits(want_mul)) {
        if (got == want_mul) ++sz_diff;
        else {
          if (mul_bad < 3 && s == 1.f) printf("  mul mismatch x=%a want %a got %a\n", x, want_mul, got);
          ++mul_bad;
        }
      }
      if (got != want_div) ++div_bad;
    }
    {  // up-convert with a scale operand: expected value(code) * scale
      float *dup;
      hipMalloc(&dup, (size_t)np * 2 * 4);
      std::vector<float> up(np * 2);
      long up_bad = 0;
      for (float us : {1.f, 0x1p5f, 0x1p-5f, 0x1p-126f, 0x1p127f, 0x1p-130f, 3.f}) {
        up_scaled<<<(np + 255) / 256, 256>>>(dcodes, np, us, dup);
        hipMemcpy(up.data(), dup, np * 2 * 4, hipMemcpyDeviceToHost);
        long bad = 0;
        for (int i = 0; i < 2 * np && i < n; ++i) {
          float want = back[i] * us;
          if (fbits(want) != fbits(up[i])) {
            if (bad < 2 && s == 1.f) printf("  up(scale %a) code-val %a want %a got %a\n", us, back[i], want, up[i]);
            ++bad;
          }
        }
        if (s == 1.f) printf("  up-convert scale %a: mismatches vs value*scale %ld\n", us, bad);
        up_bad += bad;
      }
      hipFree(dup);
    }
    printf("scale %a: finite %ld, mismatches vs round(x*s) %ld (signed-zero-only %ld), vs round(x/s) %ld\n",
           s, finite, mul_bad, sz_diff, div_bad);
  }
  hipFree(dx);
  hipFree(dback);
  hipFree(dcodes);
  return 0;
}
