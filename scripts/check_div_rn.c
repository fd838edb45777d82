// Host check of the INT-n qdq kernels' division (mtq::div_rn, tensorrt-model-optimizer_amd/csrc/
// mtq_device.hpp): y = copysign(fma(fma(-q*r, s, q), r, q*r), q) with r = RN(1/s) must equal the
// IEEE quotient q / s bit for bit -- the reference divides by the scale
// (modelopt/torch/quantization/tensor_quant.py:643 `outputs = outputs / scale`,
// tensor_quant_gpu.cu:50 `/ scale`).
//
// Cases: every fp32 significand of s (2^23, or every STRIDE-th one) at 7 binades spanning the
// scales INT-n quantisation produces (s = max_bound / amax), times every integer code
// q in [-32768, 32767] that a <= 16-bit quantiser can emit (full sweep: q in [-128, 127] for all
// significands, the 16-bit codes on every 64th significand).
//
//   gcc -O2 -ffp-contract=off -o /tmp/chk scripts/check_div_rn.c && /tmp/chk [STRIDE]
// expected last line: "mismatches 0".  tests/test_div_rn_check.py runs a strided slice.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint32_t bits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}

static float div_rn(float q, float s, float r) {
  float y0 = q * r;
  float e = fmaf(-y0, s, q);
  return copysignf(fmaf(e, r, y0), q);
}

int main(int argc, char **argv) {
  const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 10) : 1u;
  const int exps[7] = {-100, -24, -1, 0, 1, 24, 100};
  long long tot = 0, bad = 0;
  for (int ei = 0; ei < 7; ++ei) {
    for (uint32_t m = 0; m < (1u << 23); m += stride) {
      uint32_t su = ((uint32_t)(exps[ei] + 127) << 23) | m;
      float s;
      memcpy(&s, &su, 4);
      const float r = 1.f / s;
      const int wide = (m / stride) % 64 == 0;
      const int qlo = wide ? -32768 : -128, qhi = wide ? 32767 : 127;
      for (int qi = qlo; qi <= qhi; ++qi) {
        const float q = (float)qi;
        const float want = q / s, got = div_rn(q, s, r);
        ++tot;
        if (bits(want) != bits(got)) {
          if (bad < 10) printf("mismatch s=%a q=%d want=%a got=%a\n", s, qi, want, got);
          ++bad;
        }
      }
    }
  }
  printf("checked %lld cases (stride %u)\nmismatches %lld\n", tot, stride, bad);
  return bad != 0;
}
