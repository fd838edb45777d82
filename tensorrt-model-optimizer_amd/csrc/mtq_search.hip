// mtq_search.hip — MI355X (gfx950) calibration *search* kernels: the per-block / per-channel
// amax searches of the MSE calibrators and of AWQ-clip.
//
// Unlike the fake-quant kernels these are VALU-bound: every weight element is quantised once per
// candidate scale (126 FP8 scales, 39 MSE multipliers, 11 clip ratios), so the design goal is
// "read the weight once, keep it in registers, sweep every candidate in-register" instead of the
// reference's one full-tensor pass (or Python loop iteration) per candidate.
//
//  * NVFP4 FP8-scale sweep (nvfp4_fp8_sweep.py:62-160): one thread per 16-element block.  The
//    per-candidate scale and its reciprocal are built once per workgroup in LDS; the loss keeps
//    the reference kernel's fp32 operation order (unfused mul/sub, the Triton interpreter's
//    8-way pairwise row sum), so the chosen candidate is bit-identical to the reference's.
//  * MSE multiplier sweep (calib/mse.py:82-183): all candidates in one pass, per-row losses
//    (per-channel / static-block amax) or per-tensor losses through deterministic partials.
//  * AWQ-clip (model_calib.py:1800-1882): a lane per (output row, clip variant) holds its
//    quantised weight block in VGPRs; the sampled activations are wave-uniform and arrive as
//    scalar loads (SGPR operands of v_pk_mul_f32); bf16/f16 products are rounded to the
//    element type (v_cvt_pk_bf16_f32) and summed with v_dot2c_f32_bf16 against (1, 1), as the
//    reference's ``(inputs * w).sum(-1)`` rounds each product to the dtype.  The original-weight
//    dot product (variant 0) is shared with the clip variants of the same row by ds_bpermute.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"

using namespace mtq;

namespace mtq {
int host_check_launch();  // mtq_kernels.hip
int host_num_cus();
}  // namespace mtq

namespace {

constexpr int kThreads = 256;

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));

template <class F> int dispatch_float_dtype(int dtype, F &&f) {
  switch (dtype) {
  case MTQ_F32: return f(float{});
  case MTQ_F16: return f(_Float16{});
  case MTQ_BF16: return f(__bf16{});
  default: return MTQ_ERR_DTYPE;
  }
}

bool valid_amax_dtype(int d) { return d >= 0 && d <= 3; }

// RN of v to the amax tensor's dtype, back as float (torch: `amax_tensor * python_float`).
__device__ __forceinline__ float round_to_dtype(float v, int dtype) {
  switch (dtype) {
  case MTQ_F16: return Elem<_Float16>::ld(Elem<_Float16>::st(v));
  case MTQ_BF16: return Elem<__bf16>::ld(Elem<__bf16>::st(v));
  default: return v;
  }
}

// numpy's float32 pairwise row sum (the Triton interpreter's tl.sum): n < 8 sequential from 0;
// n <= 128: eight running sums over strides of 8, combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)).
template <int N> __device__ __forceinline__ float pairwise_sum(const float *a) {
#pragma clang fp contract(off)
  if constexpr (N < 8) {
    float r = 0.f;
#pragma unroll
    for (int i = 0; i < N; ++i) r = r + a[i];
    return r;
  } else {
    static_assert(N % 8 == 0 && N <= 128, "block");
    float r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = a[j];
#pragma unroll
    for (int i = 8; i < N; i += 8)
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = r[j] + a[i + j];
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  }
}

template <typename T, int N> __device__ __forceinline__ void load_row(const T *p, float *w) {
  if constexpr ((N * sizeof(T)) % 16 == 0) {
    using V = Vec<T>;
#pragma unroll
    for (int i = 0; i < N / V::N; ++i) {
      V v = ldg_vec(p + i * V::N);
#pragma unroll
      for (int j = 0; j < V::N; ++j) w[i * V::N + j] = Elem<T>::ld(v.e[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) w[j] = Elem<T>::ld(p[j]);
  }
}

// ============================================================================================
// NVFP4 FP8-scale sweep (nvfp4_fp8_sweep.py:62-105 `_fp8_scale_sweep_kernel`)
// ============================================================================================
// scale_k = RN(RN(c_k * g) / 6) (1 when 0); loss_k = sum_j (|w_j| - e2m1(RN(|w_j| / scale_k)) *
// scale_k)^2 with every product / difference rounded separately; first strict minimum wins;
// best = RN(g * c_best).
constexpr int kMaxCand = 128;

template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void nvfp4_sweep_kernel(const T *__restrict__ x,
                                                                float *__restrict__ best,
                                                                int64_t nblocks,
                                                                const float *__restrict__ gamax,
                                                                const float *__restrict__ cands,
                                                                int ncand, int aligned) {
#pragma clang fp contract(off)
  __shared__ float s_scale[kMaxCand], s_rcp[kMaxCand];
  const float g = gamax[0];
  for (int k = threadIdx.x; k < ncand; k += kThreads) {
    float s = (cands[k] * g) / 6.0f;
    s = s == 0.f ? 1.f : s;
    s_scale[k] = s;
    s_rcp[k] = 1.0f / s;
  }
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (b >= nblocks) return;
  float w[BS];
  if (aligned) {
    load_row<T, BS>(x + b * BS, w);
  } else {
#pragma unroll
    for (int j = 0; j < BS; ++j) w[j] = Elem<T>::ld(x[b * BS + j]);
  }
#pragma unroll
  for (int j = 0; j < BS; ++j) w[j] = fabsf(w[j]);
  const TableFmt e2m1{1, 0, 6.0f, false};
  float best_loss = INFINITY;
  int best_k = 0;
  for (int k = 0; k < ncand; ++k) {
    const float s = s_scale[k], r = s_rcp[k];
    float sq[BS];
#pragma unroll
    for (int j = 0; j < BS; ++j) {
      const float q = round_table(div_rn(w[j], s, r), e2m1);
      const float p = q * s;
      const float d = w[j] - p;
      sq[j] = d * d;
    }
    const float loss = pairwise_sum<BS>(sq);
    if (loss < best_loss) {
      best_loss = loss;
      best_k = k;
    }
  }
  best[b] = g * cands[best_k];
}

// ============================================================================================
// MSE multiplier sweep (calib/mse.py:82-125 collect, one tensor, every candidate at once)
// ============================================================================================
// candidate amax = amax * c (rounded to the amax dtype when the amax tensor has dims, fp32 when
// it is 0-dim -- torch's promotion), xq = fake_quant(x_f32, candidate amax) exactly as the
// INT-n / FP8 fake-quant kernels, loss = sum (x - xq)^2 over the row.
struct MseQ {
  int fp8;  // 1: e4m3 (tensor_quant.py:46-59), 0: INT-n (tensor_quant.py:607-645)
  float max_bound, min_bound;
};

struct MseCand {
  IntQ iq;
  Fp8Q fq;
};

__device__ __forceinline__ MseCand make_cand(float a, const MseQ &q) {
  MseCand c;
  if (q.fp8)
    c.fq = make_fp8q(a);
  else
    c.iq = make_intq(a, q.max_bound, q.min_bound);
  return c;
}

__device__ __forceinline__ float mse_term(float x, const MseCand &c, const MseQ &q) {
#pragma clang fp contract(off)
  float xq;
  if (q.fp8) {
    float b = 0.f;
    xq = x;
    fp8_qdq2(xq, b, c.fq);
  } else {
    xq = int_qdq(x, c.iq);
  }
  const float d = x - xq;
  return d * d;
}

__device__ __forceinline__ float cand_amax(float a, float c, int amax_dtype, int round_amax) {
#pragma clang fp contract(off)
  const float v = a * c;
  return round_amax ? round_to_dtype(v, amax_dtype) : v;
}

// One thread per row, the row in VGPRs (rows of <= MAXC elements: static blocks).
template <typename T, int MAXC>
__global__ __launch_bounds__(kThreads) void mse_rows_kernel(const T *__restrict__ x, int64_t rows,
                                                             int cols, const void *__restrict__ amax,
                                                             int amax_dtype, int per_row,
                                                             int round_amax,
                                                             const float *__restrict__ cands,
                                                             int ncand, MseQ q,
                                                             float *__restrict__ loss) {
#pragma clang fp contract(off)
  const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (r >= rows) return;
  float v[MAXC];
#pragma unroll
  for (int j = 0; j < MAXC; ++j) v[j] = j < cols ? Elem<T>::ld(x[r * cols + j]) : 0.f;
  const float a = load_as_float(amax, amax_dtype, per_row ? r : 0);
  for (int k = 0; k < ncand; ++k) {
    const MseCand c = make_cand(cand_amax(a, cands[k], amax_dtype, round_amax), q);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < MAXC; ++j)
      if (j < cols) acc = acc + mse_term(v[j], c, q);
    loss[(int64_t)k * rows + r] = acc;
  }
}

// Long rows (per-channel / per-tensor): a workgroup per (row, chunk of kChunk elements), each
// lane kPer elements in VGPRs; partials[row][chunk][k] reduced in chunk order by mse_finish.
constexpr int kPer = 8;
constexpr int kChunk = kThreads * kPer;

__device__ __forceinline__ float block_sum(float v, float *red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return ((red[0] + red[1]) + (red[2] + red[3]));
}

template <typename T>
__global__ __launch_bounds__(kThreads) void mse_chunk_kernel(const T *__restrict__ x, int64_t rows,
                                                              int64_t cols, int64_t nchunk,
                                                              const void *__restrict__ amax,
                                                              int amax_dtype, int per_row,
                                                              int round_amax,
                                                              const float *__restrict__ cands,
                                                              int ncand, MseQ q,
                                                              float *__restrict__ partials) {
#pragma clang fp contract(off)
  __shared__ float red[kThreads / 64];
  const int64_t chunk = blockIdx.x, r = blockIdx.y;
  const int64_t c0 = chunk * kChunk;
  float v[kPer];
  bool ok[kPer];
#pragma unroll
  for (int j = 0; j < kPer; ++j) {
    const int64_t c = c0 + (int64_t)j * kThreads + threadIdx.x;
    ok[j] = c < cols;
    v[j] = ok[j] ? Elem<T>::ld(x[r * cols + c]) : 0.f;
  }
  const float a = load_as_float(amax, amax_dtype, per_row ? r : 0);
  for (int k = 0; k < ncand; ++k) {
    const MseCand cd = make_cand(cand_amax(a, cands[k], amax_dtype, round_amax), q);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < kPer; ++j)
      if (ok[j]) acc = acc + mse_term(v[j], cd, q);
    const float tot = block_sum(acc, red);
    if (threadIdx.x == 0) partials[(r * nchunk + chunk) * ncand + k] = tot;
  }
}

__global__ __launch_bounds__(kThreads) void mse_finish_kernel(const float *__restrict__ partials,
                                                               int64_t rows, int64_t nchunk,
                                                               int ncand,
                                                               float *__restrict__ loss) {
  const int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (i >= rows * ncand) return;
  const int64_t r = i / ncand;
  const int k = (int)(i - r * ncand);
  float acc = 0.f;
  for (int64_t c = 0; c < nchunk; ++c) acc += partials[(r * nchunk + c) * ncand + k];
  loss[(int64_t)k * rows + r] = acc;
}

// Many chunks per row (per-tensor MSE): a workgroup per (row, candidate); lane t sums chunks
// t, t + 256, ... in order, then a fixed-shape tree -- deterministic for a given shape.
__global__ __launch_bounds__(kThreads) void mse_finish_wide_kernel(const float *__restrict__ partials,
                                                                    int64_t rows, int64_t nchunk,
                                                                    int ncand,
                                                                    float *__restrict__ loss) {
  __shared__ float red[kThreads / 64];
  const int64_t r = blockIdx.x / ncand;
  const int k = (int)(blockIdx.x - r * ncand);
  float acc = 0.f;
  for (int64_t c = threadIdx.x; c < nchunk; c += kThreads) acc += partials[(r * nchunk + c) * ncand + k];
  const float tot = block_sum(acc, red);
  if (threadIdx.x == 0) loss[(int64_t)k * rows + r] = tot;
}

// ============================================================================================
// AWQ-clip block search (model_calib.py:1815-1882, static-block INT-n weights)
// ============================================================================================
// Lane (g, v) of a wave: output row o = tile row g, variant v (0 = the original weight, v >= 1 =
// clip ratio shrinks[v-1]); all lanes of the wave share block column b and walk the tokens
// together, reading the fp32 activations x[t, b*BS + k] as wave-uniform scalar loads.
template <typename T, int BS> struct ClipDot;

template <int BS> struct ClipDot<__bf16, BS> {
  static __device__ __forceinline__ float run(const float *__restrict__ xr, const float *wq) {
    float acc = 0.f;
    const bf16x2_t one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
    for (int k = 0; k < BS; k += 2) {
      const float p0 = xr[k] * wq[k], p1 = xr[k + 1] * wq[k + 1];
      const bf16x2_t pk = {(__bf16)p0, (__bf16)p1};  // v_cvt_pk_bf16_f32: RNE per product
      acc = __builtin_amdgcn_fdot2_f32_bf16(pk, one, acc, false);
    }
    return Elem<__bf16>::ld(Elem<__bf16>::st(acc));
  }
};

template <int BS> struct ClipDot<_Float16, BS> {
  static __device__ __forceinline__ float run(const float *__restrict__ xr, const float *wq) {
    float acc = 0.f;
    const f16x2_t one = {(_Float16)1.0f, (_Float16)1.0f};
#pragma unroll
    for (int k = 0; k < BS; k += 2) {
      const float p0 = xr[k] * wq[k], p1 = xr[k + 1] * wq[k + 1];
      const f16x2_t pk = {Elem<_Float16>::st(p0), Elem<_Float16>::st(p1)};
      acc = __builtin_amdgcn_fdot2(pk, one, acc, false);
    }
    return Elem<_Float16>::ld(Elem<_Float16>::st(acc));
  }
};

template <int BS> struct ClipDot<float, BS> {
  static __device__ __forceinline__ float run(const float *__restrict__ xr, const float *wq) {
#pragma clang fp contract(off)
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < BS; ++k) acc = acc + xr[k] * wq[k];
    return acc;
  }
};

template <typename T, int BS>
__global__ __launch_bounds__(kThreads) void awq_clip_kernel(
    const T *__restrict__ w, const float *__restrict__ xs, int64_t co, int64_t cols, int ntok,
    const void *__restrict__ wamax, int amax_dtype, const float *__restrict__ shrinks, int nvar,
    float max_bound, float min_bound, float *__restrict__ loss, int accumulate) {
#pragma clang fp contract(off)
  const int64_t nb = cols / BS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rpw = 64 / nvar;  // rows per wave
  const int g = lane / nvar, v = lane - g * nvar;
  const int64_t o = ((int64_t)blockIdx.x * (kThreads / 64) + wave) * rpw + g;
  const int64_t b = blockIdx.y;
  const bool active = g < rpw && o < co;
  float wq[BS];
  if (active) {
    load_row<T, BS>(w + o * cols + b * BS, wq);
    if (v > 0) {
      const float a = round_to_dtype(load_as_float(wamax, amax_dtype, o * nb + b) * shrinks[v - 1],
                                     amax_dtype);
      const IntQ q = make_intq(a, max_bound, min_bound);
#pragma unroll
      for (int k = 0; k < BS; ++k) wq[k] = Elem<T>::ld(Elem<T>::st(int_qdq(wq[k], q)));
    }
  } else {
#pragma unroll
    for (int k = 0; k < BS; ++k) wq[k] = 0.f;
  }
  const int src = (g < rpw ? g : 0) * nvar;  // the group's variant-0 lane
  const float *__restrict__ xb = xs + b * BS;
  float lsum = 0.f;
  for (int t = 0; t < ntok; ++t) {
    const float cur = ClipDot<T, BS>::run(xb + (int64_t)t * cols, wq);
    const float org = __shfl(cur, src, 64);
    const float d = Elem<T>::ld(Elem<T>::st(cur - org));
    lsum = lsum + d * d;
  }
  if (active && v > 0) {
    const float m = lsum / (float)ntok;
    const int64_t idx = ((int64_t)(v - 1) * co + o) * nb + b;
    loss[idx] = accumulate ? loss[idx] + m : m;
  }
}

template <typename T>
int launch_awq_clip(const T *w, const float *x, int64_t co, int64_t cols, int ntok,
                    const void *wamax, int amax_dtype, const float *shrinks, int nshrink, int block,
                    float maxb, float minb, float *loss, int accumulate, hipStream_t stream) {
  const int nvar = nshrink + 1;
  const int rpw = 64 / nvar;
  const int64_t rows_per_block = (int64_t)rpw * (kThreads / 64);
  const dim3 grid((unsigned)((co + rows_per_block - 1) / rows_per_block), (unsigned)(cols / block));
  switch (block) {
#define MTQ_CLIP(BS)                                                                              \
  case BS:                                                                                         \
    awq_clip_kernel<T, BS><<<grid, kThreads, 0, stream>>>(w, x, co, cols, ntok, wamax, amax_dtype, \
                                                          shrinks, nvar, maxb, minb, loss,         \
                                                          accumulate);                             \
    break;
    MTQ_CLIP(8)
    MTQ_CLIP(16)
    MTQ_CLIP(32)
    MTQ_CLIP(64)
    MTQ_CLIP(128)
#undef MTQ_CLIP
  default: return MTQ_ERR_BLOCKSIZE;
  }
  return host_check_launch();
}

}  // namespace

// ============================================================================================
// C ABI (include/mtq_amd.h)
// ============================================================================================
extern "C" {

int mtq_nvfp4_fp8_scale_sweep(const void *x, float *best_amax, int64_t n_blocks, int block,
                              int dtype, const float *global_amax, const float *candidates,
                              int n_candidates, hipStream_t stream) {
  if (n_blocks < 0 || (n_blocks > 0 && (!x || !best_amax || !global_amax || !candidates)) ||
      n_candidates < 1 || n_candidates > kMaxCand)
    return MTQ_ERR_INVALID_ARG;
  if (n_blocks == 0) return MTQ_OK;
  const int aligned = ((uintptr_t)x & 15u) == 0;
  const unsigned grid = (unsigned)((n_blocks + kThreads - 1) / kThreads);
  return dispatch_float_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    const T *xt = static_cast<const T *>(x);
    switch (block) {
#define MTQ_SWEEP(BS)                                                                              \
  case BS:                                                                                         \
    nvfp4_sweep_kernel<T, BS><<<grid, kThreads, 0, stream>>>(xt, best_amax, n_blocks, global_amax, \
                                                             candidates, n_candidates, aligned);   \
    break;
      MTQ_SWEEP(8)
      MTQ_SWEEP(16)
      MTQ_SWEEP(32)
#undef MTQ_SWEEP
    default: return (int)MTQ_ERR_BLOCKSIZE;
    }
    return host_check_launch();
  });
}

int64_t mtq_mse_sweep_workspace_floats(int64_t rows, int64_t cols, int n_candidates) {
  if (rows < 0 || cols < 0 || n_candidates < 1) return -1;
  if (cols <= 128) return 0;
  const int64_t nchunk = (cols + kChunk - 1) / kChunk;
  return rows * nchunk * n_candidates;
}

int mtq_mse_sweep(const void *x, int64_t rows, int64_t cols, int dtype, const void *amax,
                  int amax_dtype, int amax_per_row, int round_candidate_amax,
                  const float *candidates, int n_candidates, int num_bits, int is_unsigned,
                  int narrow_range, float *loss, float *workspace, int64_t workspace_floats,
                  hipStream_t stream) {
  if (rows < 0 || cols < 0 || n_candidates < 1 || num_bits < 0 || num_bits > 31)
    return MTQ_ERR_INVALID_ARG;
  if (rows == 0 || cols == 0) return MTQ_OK;
  if (!x || !amax || !candidates || !loss) return MTQ_ERR_INVALID_ARG;
  if (!valid_amax_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  MseQ q;
  q.fp8 = num_bits == 0;
  if (!q.fp8) {
    q.max_bound = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
    q.min_bound = is_unsigned ? 0.f : (narrow_range ? -q.max_bound : -q.max_bound - 1.f);
  } else {
    q.max_bound = 448.f;
    q.min_bound = -448.f;
  }
  return dispatch_float_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    const T *xt = static_cast<const T *>(x);
    if (cols <= 128) {
      const unsigned grid = (unsigned)((rows + kThreads - 1) / kThreads);
#define MTQ_MSE_ROWS(C)                                                                          \
  mse_rows_kernel<T, C><<<grid, kThreads, 0, stream>>>(xt, rows, (int)cols, amax, amax_dtype,      \
                                                       amax_per_row, round_candidate_amax,         \
                                                       candidates, n_candidates, q, loss)
      if (cols <= 16)
        MTQ_MSE_ROWS(16);
      else if (cols <= 32)
        MTQ_MSE_ROWS(32);
      else if (cols <= 64)
        MTQ_MSE_ROWS(64);
      else
        MTQ_MSE_ROWS(128);
#undef MTQ_MSE_ROWS
      return host_check_launch();
    }
    const int64_t nchunk = (cols + kChunk - 1) / kChunk;
    if (!workspace || workspace_floats < rows * nchunk * n_candidates) return (int)MTQ_ERR_INVALID_ARG;
    if (rows > 65535) return (int)MTQ_ERR_INVALID_ARG;
    mse_chunk_kernel<T><<<dim3((unsigned)nchunk, (unsigned)rows), kThreads, 0, stream>>>(
        xt, rows, cols, nchunk, amax, amax_dtype, amax_per_row, round_candidate_amax, candidates,
        n_candidates, q, workspace);
    int st = host_check_launch();
    if (st != MTQ_OK) return st;
    const int64_t n = rows * n_candidates;
    if (nchunk > 64)
      mse_finish_wide_kernel<<<(unsigned)n, kThreads, 0, stream>>>(workspace, rows, nchunk,
                                                                    n_candidates, loss);
    else
      mse_finish_kernel<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, stream>>>(
          workspace, rows, nchunk, n_candidates, loss);
    return host_check_launch();
  });
}

int mtq_awq_clip_search(const void *w, const float *x, int64_t co, int64_t cols, int64_t n_tokens,
                        int dtype, const void *w_amax, int amax_dtype, const float *shrinks,
                        int n_shrinks, int block, int num_bits, int is_unsigned, int narrow_range,
                        float *loss, int accumulate, hipStream_t stream) {
  if (co < 0 || cols < 0 || n_tokens < 0 || n_shrinks < 1 || n_shrinks > 63 || block < 1 ||
      num_bits < 1 || num_bits > 31)
    return MTQ_ERR_INVALID_ARG;
  if (cols % block != 0) return MTQ_ERR_INVALID_ARG;
  if (co == 0 || cols == 0) return MTQ_OK;
  if (n_tokens == 0 || n_tokens > 0x7fffffff || !w || !x || !w_amax || !shrinks || !loss)
    return MTQ_ERR_INVALID_ARG;
  if (cols / block > 65535) return MTQ_ERR_INVALID_ARG;
  if (!valid_amax_dtype(amax_dtype)) return MTQ_ERR_DTYPE;
  const float maxb = (float)((1ll << (num_bits - 1 + (is_unsigned ? 1 : 0))) - 1);
  const float minb = is_unsigned ? 0.f : (narrow_range ? -maxb : -maxb - 1.f);
  return dispatch_float_dtype(dtype, [&](auto t) {
    using T = decltype(t);
    return launch_awq_clip<T>(static_cast<const T *>(w), x, co, cols, (int)n_tokens, w_amax,
                              amax_dtype, shrinks, n_shrinks, block, maxb, minb, loss, accumulate,
                              stream);
  });
}

}  // extern "C"
