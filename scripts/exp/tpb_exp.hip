// tpb_exp.hip -- measurement-only A/B of workgroup size on the dynamic NVFP4 qdq kernel
// (csrc/mtq_kernels.hip nvfp4_native_u_kernel, block 16, U = 2): var = threads per workgroup
// (256 = the product launch, 512, 1024).  Built by build_exp.sh, timed by bench_tpb_exp.py.
// r05 (profiles/r05/nvfp4_tpb_ab_r05tp1.log): 512 within 0.2-0.5 % of 256, 1024 6 % slower -- the
// launch stays at 256 (unlike the bench primary's group kernel, where 512 gained ~1 %).
#include "../../tensorrt-model-optimizer_amd/csrc/mtq_kernels.hip"

extern "C" int tpb_exp(int var, const void *x, void *y, int64_t n, const float *gamax, hipStream_t stream) {
  using T = __bf16;
  if (n % 16 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return 2;
  const int64_t nvec = n / 8;
  const T *xt = reinterpret_cast<const T *>(x);
  T *yt = reinterpret_cast<T *>(y);
  switch (var) {
  case 256: nvfp4_native_u_kernel<T, 16, 2, 256><<<(unsigned)((nvec + 511) / 512), 256, 0, stream>>>(xt, yt, nvec, gamax); break;
  case 512: nvfp4_native_u_kernel<T, 16, 2, 512><<<(unsigned)((nvec + 1023) / 1024), 512, 0, stream>>>(xt, yt, nvec, gamax); break;
  case 1024: nvfp4_native_u_kernel<T, 16, 2, 1024><<<(unsigned)((nvec + 2047) / 2048), 1024, 0, stream>>>(xt, yt, nvec, gamax); break;
  default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
