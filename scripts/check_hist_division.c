// Host check that the histogram kernel's Markstein-corrected division (hist_div_kernel,
// mtq_kernels.hip) gives the same bin as the IEEE division of torch.histc's formula for every
// bf16 and f16 |x| at 20 000 random ranges / bin counts.  gcc -O2 -ffp-contract=off -o chk
// scripts/check_hist_division.c -lm && ./chk   (expected: "mismatches 0")
#include <stdio.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
static float bf(uint32_t m){ uint32_t u = m << 16; float f; memcpy(&f,&u,4); return f; }
static float f16(uint32_t h){
  uint32_t e = (h >> 10) & 0x1f, mm = h & 0x3ff; float v;
  if (e == 0) v = ldexpf((float)mm, -24); else if (e == 31) v = mm ? NAN : INFINITY; else v = ldexpf((float)(mm | 0x400), (int)e - 25);
  return (h & 0x8000) ? -v : v; }
static uint32_t rng = 12345; static uint32_t nxt(){ rng = rng*1664525u+1013904223u; return rng; }
int main(){
  long bad = 0, tot = 0;
  int binsl[] = {2048, 3001, 64, 9000, 16384, 2049, 128};
  for (int trial = 0; trial < 20000; ++trial) {
    int bins = binsl[trial % 7];
    // random span: random float in a wide exponent range
    uint32_t su = (nxt() & 0x007fffff) | ((uint32_t)(100 + nxt() % 60) << 23);
    float hi; memcpy(&hi, &su, 4);
    if (trial % 5 == 0) hi = (float)(1 + nxt() % 1000);  // integers
    if (trial % 11 == 0) hi = ldexpf(1.f, (int)(nxt() % 40) - 20);  // powers of two
    volatile float lo = 0.f, fb = (float)bins, span = hi - lo;
    float y = 1.f / span;
    for (uint32_t m = 0; m < 65536; ++m) {
      float a = (m < 32768) ? bf(m) : f16(m - 32768);
      if (!(a <= hi)) continue;
      float t = (a - lo) * fb;
      int b0 = (int)(t / span);
      float q0 = t * y;
      float r = fmaf(-q0, span, t);
      float q1 = fmaf(r, y, q0);
      int b1 = (int)q1;
      tot++;
      if (b0 != b1) { if (bad < 10) printf("mismatch hi=%a bins=%d a=%a t/span=%a mk=%a\n", hi, bins, a, t/span, q1); bad++; }
    }
  }
  printf("checked %ld, mismatches %ld\n", tot, bad);
  return 0;
}
