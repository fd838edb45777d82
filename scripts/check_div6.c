// Host check of the MXFP4 export's block-scale division (mtq_kernels.hip export_mxfp4_vec_one,
// 16-bit elements): div_rn(a, 6, RN(1/6)) must equal the IEEE quotient a / 6 bit for bit for every
// finite non-negative amax a a bf16 or f16 block can have (the block max of 16-bit magnitudes is
// itself a 16-bit value) -- the reference computes amax / 6.0 (qtensor/mxfp4_tensor.py).
//   gcc -O2 -ffp-contract=off -o /tmp/chk6 scripts/check_div6.c && /tmp/chk6
// expected last line: "mismatches 0".
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float from_bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static float div_rn(float q, float s, float r) {
  float y0 = q * r;
  float e = fmaf(-y0, s, q);
  return copysignf(fmaf(e, r, y0), q);
}
static float half_to_float(uint16_t h) {
  const uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff;
  if (e == 0) return ldexpf((float)m, -24);
  if (e == 31) return m ? NAN : INFINITY;
  return ldexpf((float)(m | 0x400), (int)e - 25);
}

int main(void) {
  const float s = 6.0f, r = 1.0f / 6.0f;
  long long tot = 0, bad = 0;
  for (uint32_t h = 0; h < 0x8000u; ++h) {  // non-negative patterns
    const float a[2] = {from_bits(h << 16), half_to_float((uint16_t)h)};  // bf16, f16
    for (int k = 0; k < 2; ++k) {
      if (!isfinite(a[k])) continue;
      ++tot;
      if (bits(div_rn(a[k], s, r)) != bits(a[k] / s)) {
        if (bad < 10) printf("mismatch %s a=%a\n", k ? "f16" : "bf16", a[k]);
        ++bad;
      }
    }
  }
  printf("checked %lld cases\nmismatches %lld\n", tot, bad);
  return bad != 0;
}
