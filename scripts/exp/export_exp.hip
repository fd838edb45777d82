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

// One-shot product structure (U = 2 vectors per lane, all loads first) with the store kinds as
// parameters: SNT = scale dword stores non-temporal, DNT = code stores non-temporal, LDS = the
// workgroup's 128 scale bytes gathered in LDS and written by 32 lanes as one 128 B line instead of
// 8 waves x 2 x 16 B non-temporal fragments.  bf16, block 32, native path (a lane whose block
// leaves it falls back to the product function).
// MODE 1: the scale exponent branch-free for normal amax / 6 outside 0 < mantissa <= 64 (ex + (m != 0)),
// the product function only for the rare rest; MODE 2: probe -- no conversion (codes = amax bits),
// the structure's memory floor (output wrong)
template <bool SNT, bool DNT, bool LDS, int U = 2, int MODE = 0>
__global__ __launch_bounds__(kThreads) void export_mxfp4_st_kernel(const __bf16 *__restrict__ x, uint8_t *__restrict__ y,
                                                                   uint8_t *__restrict__ sc, int64_t nvec) {
  using T = __bf16;
  using V = Vec<T>;
  constexpr int LPB = 4;
  __shared__ uint8_t sl[U * kThreads / LPB];
  const int64_t wb = (int64_t)blockIdx.x * (kThreads * U);
  const int64_t base = wb + threadIdx.x;
  V v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    v[u] = ldg_vec_nt(x + (i < nvec ? i : nvec - 1) * V::N);
  }
  const bool full = wb + kThreads * U <= nvec;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * kThreads;
    if (!full) {
      export_mxfp4_vec_one<T, 32, true>(i, v[u], y, sc, nvec, 1);
      continue;
    }
    const uint32_t w[4] = {v[u].raw.x, v[u].raw.y, v[u].raw.z, v[u].raw.w};
    const uint32_t m = group_max_u32<LPB>(scan_pairs(w).max_abs);
    const float amax = half_bits_to_float<T>(m);
    constexpr float kInv6 = 1.0f / 6.0f;
    const float d6 = amax <= 3.402823466e38f ? div_rn(amax, 6.0f, kInv6) : amax * kInv6;
    float e;
    if constexpr (MODE == 1) {
      const uint32_t db = __float_as_uint(d6), ef = (db >> 23) & 0xFFu, mm = db & 0x7FFFFFu;
      e = (float)((int)ef - 127 + (mm != 0u ? 1 : 0));
      if (db == 0u) e = -127.f;
      else if (!((ef - 1u) < 0xFEu && (mm == 0u || mm > 64u))) e = mx_e8m0_exponent(d6);
    } else if constexpr (MODE == 2) {
      e = 0.f;
      uint32_t *dy = reinterpret_cast<uint32_t *>(y + i * 4);
      __builtin_nontemporal_store(m, dy);
      if (threadIdx.x % LPB == 0) sl[u * (kThreads / LPB) + threadIdx.x / LPB] = (uint8_t)m;
      continue;
    } else {
      e = mx_e8m0_exponent(d6);
    }
    if (!(e >= -100.f && e <= 127.f)) {  // exact path, product function (writes its own scale)
      export_mxfp4_vec_one<T, 32, true>(i, v[u], y, sc, nvec, 0);
      if constexpr (LDS) {
        if (threadIdx.x % LPB == 0) sl[u * (kThreads / LPB) + threadIdx.x / LPB] = (uint8_t)((uint32_t)(int)(e + 127.f) & 0xFFu);
      }
      continue;
    }
    const uint32_t sbyte = (uint32_t)(int)(e + 127.f) & 0xFFu;
    if constexpr (LDS) {
      if (threadIdx.x % LPB == 0) sl[u * (kThreads / LPB) + threadIdx.x / LPB] = (uint8_t)sbyte;
    } else {
      const uint32_t b1 = (uint32_t)__shfl_down((int)sbyte, 4, 16);
      const uint32_t b2 = (uint32_t)__shfl_down((int)sbyte, 8, 16);
      const uint32_t b3 = (uint32_t)__shfl_down((int)sbyte, 12, 16);
      if ((threadIdx.x & 15) == 0) {
        const uint32_t word = sbyte | (b1 << 8) | (b2 << 16) | (b3 << 24);
        uint32_t *dst = reinterpret_cast<uint32_t *>(sc + i / LPB);
        if constexpr (SNT) __builtin_nontemporal_store(word, dst);
        else *dst = word;
      }
    }
    const int ei = (int)e;
    const float s = __uint_as_float((uint32_t)(ei + 127) << 23);
    const float zthr = __uint_as_float(ei >= 24 ? (uint32_t)(ei - 23) << 23 : (ei >= 1 ? 1u << (ei - 1) : 0u));
    uint32_t o = 0, zero = 0;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const float f0 = Elem<T>::ld(v[u].e[j]), f1 = Elem<T>::ld(v[u].e[j + 1]);
      zero |= (fabsf(f0) <= zthr ? 0xFu : 0u) << (4 * j);
      zero |= (fabsf(f1) <= zthr ? 0xFu : 0u) << (4 * j + 4);
      o |= fp4_pair_hw(__uint_as_float(__float_as_uint(f0) - 1u), __uint_as_float(__float_as_uint(f1) - 1u), s) << (4 * j);
    }
    o = (o & ~zero) | (zero & 0x88888888u);
    uint32_t *dy = reinterpret_cast<uint32_t *>(y + i * 4);
    if constexpr (DNT) __builtin_nontemporal_store(o, dy);
    else *dy = o;
  }
  if constexpr (LDS) {
    if (full) {
      __syncthreads();
      if (threadIdx.x < U * kThreads / LPB / 4) {
        const uint32_t word = reinterpret_cast<const uint32_t *>(sl)[threadIdx.x];
        uint32_t *dst = reinterpret_cast<uint32_t *>(sc + wb / LPB) + threadIdx.x;
        if constexpr (SNT) __builtin_nontemporal_store(word, dst);
        else *dst = word;
      }
    }
  }
}
}  // namespace

// bf16 x [n], block 32, 4-byte aligned scales: var 1 = PF U=2 8 blocks/CU, 2 = PF U=2 4 blocks/CU,
// 3 = PF U=1 8 blocks/CU, 4 = PF U=4 4 blocks/CU; 5..10 = one-shot store kinds (SNT, DNT, LDS):
// 5 = (1,1,0) the product's, 6 = (0,1,0), 7 = (0,0,0), 8 = (1,1,1), 9 = (0,1,1), 10 = (0,0,1);
// 11 / 12 / 13 = 8 with U = 4 / 8 / 1 vectors per lane
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
  case 5: export_mxfp4_st_kernel<true, true, false><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 6: export_mxfp4_st_kernel<false, true, false><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 7: export_mxfp4_st_kernel<false, false, false><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 8: export_mxfp4_st_kernel<true, true, true><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 9: export_mxfp4_st_kernel<false, true, true><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 10: export_mxfp4_st_kernel<false, false, true><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 11: export_mxfp4_st_kernel<true, true, true, 4><<<export_grid(nvec, 4), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 12: export_mxfp4_st_kernel<true, true, true, 8><<<export_grid(nvec, 8), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 13: export_mxfp4_st_kernel<true, true, true, 1><<<export_grid(nvec, 1), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 14: export_mxfp4_st_kernel<true, true, true, 4, 1><<<export_grid(nvec, 4), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 15: export_mxfp4_st_kernel<true, true, true, 4, 2><<<export_grid(nvec, 4), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  case 16: export_mxfp4_st_kernel<true, true, true, 2, 1><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, scales, nvec); break;
  default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// FP8 per-tensor / NVFP4 export packers at U vectors per lane (the product's kernels, other U):
// var 20 / 21 = export_fp8_pt_kernel U = 4 / 2 (round to dtype), 22 / 23 = export_nvfp4_vec_kernel
// U = 4 / 2.  aux0 = the fp8 scale (1 float) or the NVFP4 block scales, aux1 = the NVFP4 scale_2.
extern "C" int export_exp2(int var, const void *x, uint8_t *y, const float *aux0, const float *aux1, int64_t rows,
                           int64_t cols, hipStream_t stream) {
  const int64_t nvec = rows * cols / 8;
  if (cols % 16 || ((uintptr_t)x & 15)) return 2;
  const __bf16 *xt = reinterpret_cast<const __bf16 *>(x);
  const FastDiv fvpb = make_fastdiv(2u);
  switch (var) {
  case 20: export_fp8_pt_kernel<4, __bf16, true><<<export_grid(nvec, 4), kThreads, 0, stream>>>(xt, y, nvec, aux0); break;
  case 21: export_fp8_pt_kernel<2, __bf16, true><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, nvec, aux0); break;
  case 22: export_nvfp4_vec_kernel<4, __bf16, true><<<export_grid(nvec, 4), kThreads, 0, stream>>>(xt, y, nvec, 2, fvpb, aux0, aux1, 1); break;
  case 23: export_nvfp4_vec_kernel<2, __bf16, true><<<export_grid(nvec, 2), kThreads, 0, stream>>>(xt, y, nvec, 2, fvpb, aux0, aux1, 1); break;
  default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
