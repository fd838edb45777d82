// export_exp.hip -- measurement-only variants of the MXFP4 export packer (csrc/mtq_kernels.hip
// export_mxfp4_vec_kernel), built by scripts/exp/build_exp.sh and timed by
// scripts/exp/bench_export_exp.py against the product op.  Not part of the product library: the
// product translation unit is included so the variant reuses its per-vector conversion.
//
// PF kernel: a persistent grid (WPC waves per CU resident for the whole launch) that walks the
// tensor in 256 x U-vector chunks, loading chunk c+1 (unconditional, clamped) before converting
// chunk c, so every wave keeps a load in flight while it converts (the one-shot product kernel
// has no load in flight during its conversion and store phase).
#include "../../tensorrt-model-optimizer_amd/csrc/mtq_kernels.hip"

namespace {
template <int U, typename T, int BLOCK, bool SC4>
__global__ __launch_bounds__(kThreads) void export_mxfp4_pf_kernel(const T *__restrict__ x, uint8_t *__restrict__ y,
                                                                    uint8_t *__restrict__ sc, int64_t nvec) {
  using V = Vec<T>;
  const int64_t step = (int64_t)gridDim.x * kThreads * U;
  int64_t cb = (int64_t)blockIdx.x * kThreads * U;  // block-uniform chunk base
  V v[U], w[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = cb + threadIdx.x + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * V::N);
  }
  for (; cb < nvec; cb += step) {
    const int64_t nb = cb + step;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = nb + threadIdx.x + u * kThreads;
      w[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * V::N);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      export_mxfp4_vec_one<T, BLOCK, SC4>(cb + threadIdx.x + u * kThreads, v[u], y, sc, nvec, 1);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = w[u];
  }
}
}  // namespace

// bf16 x [n], block 32, 4-byte aligned scales: var 1 = PF U=2 8 blocks/CU, 2 = PF U=2 4 blocks/CU,
// 3 = PF U=1 8 blocks/CU, 4 = PF U=4 4 blocks/CU
extern "C" int export_exp(int var, const void *x, uint8_t *y, uint8_t *scales, int64_t n, hipStream_t stream) {
  if (n % 256 || ((uintptr_t)scales & 3) || ((uintptr_t)x & 15)) return 2;
  const int64_t nvec = n / 8;
  const int cus = num_cus();
  const __bf16 *xt = reinterpret_cast<const __bf16 *>(x);
  switch (var) {
  case 1: export_mxfp4_pf_kernel<2, __bf16, 32, true><<<cus * 8, kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 2: export_mxfp4_pf_kernel<2, __bf16, 32, true><<<cus * 4, kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 3: export_mxfp4_pf_kernel<1, __bf16, 32, true><<<cus * 8, kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 4: export_mxfp4_pf_kernel<4, __bf16, 32, true><<<cus * 4, kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
