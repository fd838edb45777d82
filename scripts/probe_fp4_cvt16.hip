// Probe: are the 16-bit-operand gfx950 FP4 converts (v_cvt_scalef32_pk_fp4_{bf16,f16},
// v_cvt_scalef32_pk_{bf16,f16}_fp4) the fp32 ones (probe_fp4_cvt.hip, matched against the
// reference E2M1 rounding there) composed with an exact widening / a RNE narrowing?
// Every 16-bit pattern x, every scale 2^k, k in [-130, 130]:
//   down16(x, s) == down32(float(x), s)        (fp4 codes)
//   up16(c, s)   == RNE16(up32(c, s))          (all 16 codes)
//   hipcc --offload-arch=gfx950 -O2 -o scripts/probe_fp4_cvt16 scripts/probe_fp4_cvt16.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__global__ void down_cmp(int kind, float s, uint32_t *bad, uint32_t *first) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // pair index over 65536 patterns
  if (i >= 32768) return;
  const uint32_t h0 = 2 * i, h1 = 2 * i + 1;
  uint32_t p16, p32;
  float f0, f1;
  if (kind == 0) {
    bf16x2 v = __builtin_bit_cast(bf16x2, h0 | (h1 << 16));
    p16 = __builtin_amdgcn_cvt_scalef32_pk_fp4_bf16(0u, v, s, 0);
    f0 = (float)v[0];
    f1 = (float)v[1];
  } else {
    f16x2 v = __builtin_bit_cast(f16x2, h0 | (h1 << 16));
    p16 = __builtin_amdgcn_cvt_scalef32_pk_fp4_f16(0u, v, s, 0);
    f0 = (float)v[0];
    f1 = (float)v[1];
  }
  p32 = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, f0, f1, s, 0);
  if ((p16 & 0xff) != (p32 & 0xff)) {
    // NaN inputs: only the code matters, both are compared as produced
    if (atomicAdd(bad, 1u) == 0) *first = h0 | ((p16 & 0xff) << 16) | ((p32 & 0xff) << 24);
  }
}

__global__ void up_cmp(int kind, float s, uint32_t *bad, uint32_t *first) {
  const uint32_t c = threadIdx.x;  // 16 codes, as pairs (c, c)
  if (c >= 16) return;
  const uint32_t p = c | (c << 4);
  auto f = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(p, s, 0);
  uint16_t g, w;
  if (kind == 0) {
    bf16x2 v = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(p, s, 0);
    g = (uint16_t)(__builtin_bit_cast(uint32_t, v) & 0xffffu);
    w = __builtin_bit_cast(uint16_t, (__bf16)f[0]);
  } else {
    f16x2 v = __builtin_amdgcn_cvt_scalef32_pk_f16_fp4(p, s, 0);
    g = (uint16_t)(__builtin_bit_cast(uint32_t, v) & 0xffffu);
    w = __builtin_bit_cast(uint16_t, (_Float16)f[0]);
  }
  if (g != w) {
    if (atomicAdd(bad, 1u) == 0) *first = c | ((uint32_t)g << 8) | ((uint32_t)w << 24);
  }
}

int main() {
  uint32_t *d;
  (void)hipMalloc(&d, 8);
  for (int kind = 0; kind < 2; ++kind) {
    long tot_down = 0, tot_up = 0;
    for (int k = -130; k <= 130; ++k) {
      uint32_t sb = k >= -126 ? (uint32_t)(k + 127) << 23 : 1u << (k + 149);
      float s;
      memcpy(&s, &sb, 4);
      uint32_t h[2] = {0, 0};
      (void)hipMemcpy(d, h, 8, hipMemcpyHostToDevice);
      down_cmp<<<128, 256>>>(kind, s, d, d + 1);
      (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
      if (h[0]) printf("%s down scale 2^%d: %u mismatching pairs (first pattern %04x: 16-bit code %02x, fp32 code %02x)\n",
                       kind ? "f16" : "bf16", k, h[0], h[1] & 0xffff, (h[1] >> 16) & 0xff, h[1] >> 24);
      tot_down += h[0];
      h[0] = h[1] = 0;
      (void)hipMemcpy(d, h, 8, hipMemcpyHostToDevice);
      up_cmp<<<1, 64>>>(kind, s, d, d + 1);
      (void)hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
      if (h[0]) printf("%s up scale 2^%d: %u codes differ (first code %u: 16-bit %04x vs RNE(fp32) %04x)\n",
                       kind ? "f16" : "bf16", k, h[0], h[1] & 0xff, (h[1] >> 8) & 0xffff, h[1] >> 24);
      tot_up += h[0];
    }
    printf("%s: down mismatching pairs %ld, up mismatching codes %ld over scales 2^-130..2^130\n",
           kind ? "f16" : "bf16", tot_down, tot_up);
  }
  (void)hipFree(d);
  return 0;
}
