/* Exhaustive host check of the MX scale-exponent shortcut in csrc/mtq_kernels.hip
 * (mx_e8m0_exponent): for a normal fp32 d = 2^ex * (1 + m / 2^23) with mantissa m > 64,
 * ceil(fp32(log2(d))) == ex + 1, so the kernel skips the double-precision log2 there.  The
 * reference computes torch.ceil(torch.log2(amax / 6)) in fp32 (qtensor/mxfp4_tensor.py:62-66).
 * Also reports the largest m <= 64 where the shortcut would be wrong (the margin).
 * Usage: check_e8m0 [stride]  (stride over m, default 1 = all 254 x 8.4 M normal values) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float ceil_log2(uint32_t bits) {
  float d;
  memcpy(&d, &bits, 4);
  return ceilf((float)log2((double)d));
}

int main(int argc, char **argv) {
  const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u;
  long bad = 0, n = 0;
  uint32_t margin = 0;
  for (uint32_t e = 1; e < 255; ++e) {
    for (uint32_t m = 1; m <= 64; ++m)
      if (ceil_log2((e << 23) | m) != (float)((int)e - 126) && m > margin) margin = m;
    for (uint32_t m = 65; m < (1u << 23); m += stride, ++n)
      if (ceil_log2((e << 23) | m) != (float)((int)e - 126)) ++bad;
  }
  printf("largest m <= 64 needing log2: %u\n", margin);
  printf("checked %ld, mismatches %ld\n", n, bad);
  return bad != 0;
}
