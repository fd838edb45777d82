// group_exp.hip -- measurement-only A/B of the FP8 static block-128 group kernel (the bench
// primary, csrc/mtq_kernels.hip ew_group_sk_kernel): var 0 = the product kernel (per-lane guarded
// loads and consumers; the compiler sinks the second load into its guarded consumer and issues the
// amax scalar loads after a vmcnt(0)); var 1 = clamped unconditional loads and an unguarded
// whole-wave path (both loads and the amax loads ahead of every wait in the ISA).  r05
// (profiles/r05/group_ab_r05gx1.log): var 1 0.3 % SLOWER (83.71 / 83.74 vs 83.47 / 83.50 us,
// labelled v0 / v1 the other way round in that log), so the product keeps the guarded form.
// Built by build_exp.sh, timed by bench_group_exp.py.  Not part of the product library.
#include "../../tensorrt-model-optimizer_amd/csrc/mtq_kernels.hip"

namespace {
template <typename T, class Op, int U, int LPB>
__global__ __launch_bounds__(kThreads) void ew_group_sk_clamped_kernel(const T *__restrict__ x, T *__restrict__ y,
                                                                    int64_t nvec, const float *__restrict__ amax,
                                                                    int64_t nchan, Op op) {
  using V = Vec<T>;
  constexpr int CPW = 64 / LPB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wb = ((int64_t)blockIdx.x * kThreads + (int64_t)w * 64) * U;
  const int k = lane / LPB, pos = lane - k * LPB;
  const int64_t v0 = wb + (int64_t)k * LPB * U + pos;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * V::N);
  }
  const int64_t c0 = wb / (LPB * U);
  float am = amax[c0 < nchan ? c0 : nchan - 1];
#pragma unroll
  for (int j = 1; j < CPW; ++j) {
    const float a = amax[c0 + j < nchan ? c0 + j : nchan - 1];
    am = k == j ? a : am;
  }
  const auto q = op.qparam_from(am);
  if (wb + 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      Op::apply(v[u], q);
      stg_vec_nt(y + (v0 + (int64_t)u * LPB) * V::N, v[u]);
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    if (i < nvec) {
      Op::apply(v[u], q);
      stg_vec_nt(y + i * V::N, v[u]);
    }
  }
}
// var 2 / 3: the guarded form with TPB = 512 / 1024 threads per workgroup (fewer, larger
// workgroups: 16 K / 8 K instead of 32 K for the bench input).  r05 (profiles/r05/
// group_tpb_ab_r05gx3.log, measured when the product kernel ran 256 threads): 512 0.5-0.8 %
// faster, 1024 3 % slower; the product kernel now runs 512 (var 0 == var 2), var 1 stays 256.
template <typename T, class Op, int U, int LPB, int TPB>
__global__ __launch_bounds__(TPB) void ew_group_sk_tpb_kernel(const T *__restrict__ x, T *__restrict__ y,
                                                              int64_t nvec, const float *__restrict__ amax,
                                                              int64_t nchan, Op op) {
  using V = Vec<T>;
  constexpr int CPW = 64 / LPB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t wb = ((int64_t)blockIdx.x * TPB + (int64_t)w * 64) * U;
  const int k = lane / LPB, pos = lane - k * LPB;
  const int64_t v0 = wb + (int64_t)k * LPB * U + pos;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    if (i < nvec) v[u] = ldg_vec_nt(x + i * V::N);
  }
  const int64_t c0 = wb / (LPB * U);
  float am = amax[c0 < nchan ? c0 : nchan - 1];
#pragma unroll
  for (int j = 1; j < CPW; ++j) {
    const float a = amax[c0 + j < nchan ? c0 + j : nchan - 1];
    am = k == j ? a : am;
  }
  if (v0 >= nvec) return;
  const auto q = op.qparam_from(am);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = v0 + (int64_t)u * LPB;
    if (i < nvec) {
      Op::apply(v[u], q);
      stg_vec_nt(y + i * V::N, v[u]);
    }
  }
}
}  // namespace

extern "C" int group_exp(int var, const void *x, void *y, int64_t n, const float *amax, hipStream_t stream) {
  using T = __bf16;
  constexpr int N = 8, U = 2, L = 8;
  if (n % 128 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return 2;
  const int64_t nvec = n / N, nchan = n / 128;
  Fp8AxisVecOp<T> op{};
  op.amax = amax;
  op.amax_dtype = MTQ_F32;
  const unsigned g = (unsigned)((nvec + (int64_t)kThreads * U - 1) / ((int64_t)kThreads * U));
  if (var == 0)
    ew_group_sk_kernel<T, Fp8AxisVecOp<T>, U, L><<<(unsigned)((nvec + kGroupSkThreads * U - 1) / (kGroupSkThreads * U)),
                                                   kGroupSkThreads, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, amax, nchan, op);
  else if (var == 1)
    ew_group_sk_clamped_kernel<T, Fp8AxisVecOp<T>, U, L><<<g, kThreads, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, amax, nchan, op);
  else if (var == 2)
    ew_group_sk_tpb_kernel<T, Fp8AxisVecOp<T>, U, L, 512><<<(unsigned)((nvec + 512 * U - 1) / (512 * U)), 512, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, amax, nchan, op);
  else if (var == 4)  // the r05 form before the 512-thread change: guarded, 256 threads
    ew_group_sk_tpb_kernel<T, Fp8AxisVecOp<T>, U, L, 256><<<(unsigned)((nvec + 256 * U - 1) / (256 * U)), 256, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, amax, nchan, op);
  else if (var == 3)
    ew_group_sk_tpb_kernel<T, Fp8AxisVecOp<T>, U, L, 1024><<<(unsigned)((nvec + 1024 * U - 1) / (1024 * U)), 1024, 0, stream>>>(
        reinterpret_cast<const T *>(x), reinterpret_cast<T *>(y), nvec, amax, nchan, op);
  else
    return 3;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
