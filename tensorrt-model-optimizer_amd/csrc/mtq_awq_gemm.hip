// mtq_awq_gemm.hip — the AWQ-lite alpha-search GEMM on MFMA (gfx950), loss fused in the epilogue.
//
// Reference: awq_lite's search forward (modelopt/torch/quantization/model_calib.py:1513-1560)
// evaluates, for each of the 11 alphas and every calibration batch,
//     out   = F.linear(x * (1/s), qdq_int4_b128(W * s), b)       (quant_module.py:257-278)
//     loss += (out - out_actual).float().pow(2).mean()             (update_loss, :1489-1495)
// i.e. an elementwise pass over x, a GEMM that writes out [M, N] to HBM, and a loss pass that
// reads out and out_actual back.  Here one launch evaluates ALL alphas of a linear:
//
//     loss[g] += mean_{m,n} float(T(T(sum_k T(x[m,k] * sinv[g,k]) * wq[g,n,k] + b[n]) - yref[m,n]))^2
//
// with the x * (1/s) product (rounded to T as the reference's bf16 multiply is) applied while the
// A tile is staged into LDS, bf16/f16 MFMA (v_mfma_f32_32x32x16, fp32 accumulate), and the bias,
// output rounding, difference (rounded to T, as the reference's subtraction) and square-sum done
// on the accumulators -- out never reaches HBM.  wq[g] = qdq_int4_b128(W * s_g) comes from
// mtq_block_quant_dynamic (one HBM pass per alpha).  Grouping the alphas in one grid (tile x g)
// also fills the 256 CUs for the narrow linears (k/v_proj: 4 x 32 tiles per alpha).
//
// Tiling: 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 per
// wave = 4 x 2 tiles of 32 x 32), K step 64, LDS double-buffered (2 x (32 + 32) KiB in one
// __shared__ array).  W tile: global_load_lds (16 B per lane) straight into LDS; x tile: register
// staged (global_load_dwordx4 -> scale by sinv -> ds_write_b128), the next tile's loads issued
// before the current tile's MFMAs.  LDS rows are 128 B; the 16-byte chunk c of row r sits at
// chunk c ^ ((r >> 1) & 7) so the 16-lane groups of every ds_read_b128 hit 16 distinct bank
// slots (cdna_hip_programming.md T2; for the glds-filled W tile the swizzle is applied to the
// global source address, rule 21).  Workgroups are remapped so each XCD runs a contiguous range
// of tiles (T1).  The loss is summed per lane in fp32 in a fixed order, across the workgroup in a
// fixed order, and the per-tile partials are folded in double by a one-block finishing kernel:
// deterministic run to run.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"

using namespace mtq;

namespace mtq {
int host_check_launch();
}

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <typename T> struct Mfma32;
template <> struct Mfma32<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma32<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};

// LDS-DMA (global_load_lds) data is visible to other waves only after the issuing wave's vmcnt
// drain and a barrier (cdna_hip_programming.md §5 'Read a staged buffer one phase AFTER ...')
__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 512;
constexpr int kTileBytes = kBM * kBK * 2;  // 32 KiB per operand tile (bf16/f16)
constexpr int kLdsBytes = 4 * kTileBytes;  // A[2] + B[2]

// byte offset of 16-byte chunk c (0..7) of row r in a [rows][64] 16-bit tile
__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }

struct AwqGemmArgs {
  const void *x;     // [M, K]
  const void *sinv;  // [G, K]
  const void *wq;    // [G, N, K]
  const void *bias;  // [N] or null
  const void *yref;  // [M, N]
  float *partial;    // [G * tiles]
  int64_t M, N, K;
  int tiles_m, tiles_n, G;
};

// PROBE (measurement builds only, MTQ_AMD_AWQ_GEMM_PROBE): 1 = no global loads / LDS staging in
// the K loop (the ds_read + MFMA + barrier structure alone), 2 = no epilogue loads.
// PRE: x holds the pre-scaled activations xs [G, M, K] (mtq_awq_prescale_kernel) and both tiles
// come in by LDS-DMA; otherwise x [M, K] is scaled while being register-staged.
template <typename T, bool PRE, int PROBE = 0>
__global__ __launch_bounds__(kThreads) void awq_search_gemm_kernel(AwqGemmArgs p) {
  typedef typename Mfma32<T>::v8 v8;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLdsBytes];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;

  // XCD-aware remap (bijective for any grid size): blocks that share an XCD get consecutive ids
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tiles = p.tiles_m * p.tiles_n;
  const int g = wgid / tiles;
  const int tile = wgid - g * tiles;
  // grouped order: the ~32 workgroups an XCD runs at once cover 8 row tiles x 4 column tiles,
  // so each K slice of their A and W tiles comes from beyond L2 once per group (12 slices per
  // 32 tiles instead of 33 with a plain row-major walk)
  constexpr int kGroupM = 8;
  const int grp = tile / (kGroupM * p.tiles_n);
  const int first_m = grp * kGroupM;
  const int gsz = p.tiles_m - first_m < kGroupM ? p.tiles_m - first_m : kGroupM;
  const int tin = tile - grp * kGroupM * p.tiles_n;
  const int tm = first_m + tin % gsz, tn = tin / gsz;
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;

  const T *X = reinterpret_cast<const T *>(p.x) + (PRE ? (int64_t)g * p.M * K : 0);
  const T *S = reinterpret_cast<const T *>(p.sinv) + (int64_t)g * K;
  const T *W = reinterpret_cast<const T *>(p.wq) + (int64_t)g * p.N * K;

  // ---- A (x) staging: thread owns chunk c = tid & 7 of rows (tid >> 3) + 64 u, u = 0..3
  // (32-bit element offsets from wave-uniform bases: the launcher checks M*K, N*K < 2^31)
  const int a_c = tid & 7, a_r0 = tid >> 3;
  unsigned a_off[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = a_r0 + 64 * u;
    int64_t row = m0 + r;
    row = row < p.M ? row : p.M - 1;  // clamp: rows past M are computed and masked
    // register staging writes the swizzled position itself; the DMA needs it on the source
    a_off[u] = (unsigned)(row * K + (PRE ? ((a_c ^ ((r >> 1) & 7)) * 8) : a_c * 8));
  }
  // ---- B (wq) staging by global_load_lds: round u writes LDS bytes [u * 8 KiB + tid * 16)
  const int b_row0 = tid >> 3, b_cs = tid & 7;  // LDS row u*64 + b_row0, chunk slot b_cs
  unsigned b_off[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = u * 64 + b_row0;
    int64_t row = n0 + r;
    row = row < p.N ? row : p.N - 1;
    b_off[u] = (unsigned)(row * K + ((b_cs ^ ((r >> 1) & 7)) * 8));
  }

  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  u32x4_t areg[4];
  u32x4_t sreg;
  auto load_a = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) areg[u] = *reinterpret_cast<const u32x4_t *>(X + k0 + a_off[u]);
    sreg = *reinterpret_cast<const u32x4_t *>(S + k0 + a_c * 8);
  };
  auto store_a = [&](unsigned char *abuf) {
    // opaque barrier: keeps the unpacking of the prefetched registers after the MFMAs (hipcc
    // otherwise hoists it next to the loads and waits vmcnt(0) before the tile's compute)
#pragma unroll
    for (int u = 0; u < 4; ++u) asm volatile("" : "+v"(areg[u]));
    asm volatile("" : "+v"(sreg));
    Vec<T> s;
    __builtin_memcpy(&s.raw, &sreg, 16);
    float sf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sf[j] = Elem<T>::ld(s.e[j]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      Vec<T> v;
      __builtin_memcpy(&v.raw, &areg[u], 16);
#pragma unroll
      for (int j = 0; j < 8; ++j) v.e[j] = Elem<T>::st(Elem<T>::ld(v.e[j]) * sf[j]);  // T(x * (1/s))
      *reinterpret_cast<uint4 *>(abuf + swz(a_r0 + 64 * u, a_c)) = v.raw;
    }
  };
  auto load_a_dma = [&](unsigned char *abuf, int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)(X + k0 + a_off[u]),
          (__attribute__((address_space(3))) void *)(abuf + u * 8192 + wave * 1024), 16, 0, 0);
  };
  auto load_b = [&](unsigned char *bbuf, int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)(W + k0 + b_off[u]),
          (__attribute__((address_space(3))) void *)(bbuf + u * 8192 + wave * 1024), 16, 0, 0);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  unsigned char *const A0 = lds, *const B0 = lds + 2 * kTileBytes;
  const int nt = (int)(K / kBK);
  const int fr = lane & 31, fh = lane >> 5;
  auto kclamp = [&](int t) { return (int64_t)(t < nt ? t : nt - 1) * kBK; };
  auto read_frags = [&](const unsigned char *Ac, const unsigned char *Bc, int s, v8 *a, v8 *b) {
    const int ch = 2 * s + fh;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = *reinterpret_cast<const v8 *>(Ac + swz(wm * 128 + i * 32 + fr, ch));
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = *reinterpret_cast<const v8 *>(Bc + swz(wn * 64 + j * 32 + fr, ch));
  };
  auto mfma8 = [&](const v8 *a, const v8 *b) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = Mfma32<T>::mma(a[i], b[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  // Pipeline (per K step t, buffers cur = t & 1):
  //   the x registers hold tile t+1 (loaded during step t-1) -> scaled into A[cur^1] early in
  //   step t, then re-filled with tile t+2; W tile t+1 goes to B[cur^1] by LDS-DMA at the top of
  //   step t.  The step ends with a counted vmcnt that retires only the DMA (the 5 x loads issued
  //   after it stay in flight across the raw barrier) -> every load has a full step to land.
  if (PRE) {
    load_a_dma(A0, 0);
    load_b(B0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    load_a(0);
    load_b(B0, 0);
    store_a(A0);  // waits for the x registers (and, in order, nothing after them)
    load_a(kclamp(1));
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // W tile 0 landed; x tile 1 in flight
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const unsigned char *Ac = A0 + cur * kTileBytes, *Bc = B0 + cur * kTileBytes;
    if (PRE && PROBE != 1) {
      // both tiles of step t+1 by LDS-DMA into the idle buffers (last read in step t-1, before
      // the barrier that ended it): a whole step of MFMAs to land
      load_a_dma(A0 + (cur ^ 1) * kTileBytes, kclamp(t + 1));
      load_b(B0 + (cur ^ 1) * kTileBytes, kclamp(t + 1));
    }
    v8 a0[4], b0[2], a1[4], b1[2];
    read_frags(Ac, Bc, 0, a0, b0);
    read_frags(Ac, Bc, 1, a1, b1);
    mfma8(a0, b0);
    if (!PRE && PROBE != 1) {
      // x tile t+1 -> LDS, its VALU beside the MFMAs.  hipcc waits vmcnt(0) before the first
      // use of the x registers, so the W DMA of tile t+1 is issued after it, not before.
      store_a(A0 + (cur ^ 1) * kTileBytes);
      // keep the ds_writes ahead of the DMA: a ds_write behind an LDS-DMA in flight makes
      // hipcc drain vmcnt(0) first (it cannot tell the two LDS ranges apart)
      __builtin_amdgcn_sched_barrier(0);
      load_b(B0 + (cur ^ 1) * kTileBytes, kclamp(t + 1));
      load_a(kclamp(t + 2));
    }
    read_frags(Ac, Bc, 2, a0, b0);
    mfma8(a1, b1);
    read_frags(Ac, Bc, 3, a1, b1);
    mfma8(a0, b0);
    mfma8(a1, b1);
    if (PRE)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");  // this step's W DMA retired
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- epilogue: bias, round to T, difference vs yref rounded to T, fp32 square-sum.
  // The yref tile [256 x 256] is staged through LDS (all 16 DMA rounds in flight at once, one
  // memory latency) and read back in the accumulator layout; rows past M / chunks past N are
  // clamped on load and masked below (N % 8 == 0).
  const T *Y = reinterpret_cast<const T *>(p.yref);
  const T *Bi = reinterpret_cast<const T *>(p.bias);
  if (PROBE != 2) {
    const int rl = wave * 2 + (lane >> 5), ck = lane & 31;
    int64_t col = n0 + ck * 8;
    col = col < p.N ? col : p.N - 8;
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      int64_t row = m0 + u * 16 + rl;
      row = row < p.M ? row : p.M - 1;
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)(Y + row * p.N + col),
          (__attribute__((address_space(3))) void *)(lds + u * 8192 + wave * 1024), 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = wn * 64 + j * 32 + fr;  // column within the tile
    const bool cok = n0 + cl < p.N;
    const float bj = Bi ? Elem<T>::ld(Bi[cok ? n0 + cl : p.N - 1]) : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int rl = wm * 128 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * fh;
        const T yr = *reinterpret_cast<const T *>(lds + rl * 512 + cl * 2);
        const float y = Elem<T>::ld(Elem<T>::st(acc[i][j][e] + bj));
        const float d = Elem<T>::ld(Elem<T>::st(y - Elem<T>::ld(yr)));
        sum = (cok && m0 + rl < p.M) ? __builtin_fmaf(d, d, sum) : sum;
      }
    }
  }
  __syncthreads();  // the LDS tile is reused for the reduction below
  // fixed-order reduction: wave butterfly, then the 8 waves in order
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) s += red[w];
    p.partial[(int64_t)g * tiles + tile] = s;
  }
}

// xs[g, m, k] = T(x[m, k] * sinv[g, k]) for all g: one read of x, G writes (the reference's
// `inputs * pre_quant_scale` per alpha, tensor_quantizer.py:1143-1144)
template <typename T>
__global__ __launch_bounds__(256) void awq_prescale_kernel(const T *__restrict__ x, const T *__restrict__ sinv,
                                                           T *__restrict__ xs, int64_t chunks, int64_t kchunks,
                                                           int G) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= chunks) return;
  Vec<T> v = ldg_vec(x + c * 8);
  float xf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) xf[j] = Elem<T>::ld(v.e[j]);
  const int64_t kc = c % kchunks;
  for (int g = 0; g < G; ++g) {
    Vec<T> s = ldg_vec(sinv + ((int64_t)g * kchunks + kc) * 8);
    Vec<T> o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o.e[j] = Elem<T>::st(xf[j] * Elem<T>::ld(s.e[j]));
    *reinterpret_cast<uint4 *>(xs + ((int64_t)g * chunks + c) * 8) = o.raw;
  }
}

// The loss of all G alphas from materialised outputs (the wide linears, whose GEMMs stay on
// hipBLASLt): reads the reference output once and each alpha's output once,
// partial[g * grid + block] = sum over the block's elements of float(T(out[g] - ref))^2.
template <typename T>
__global__ __launch_bounds__(256) void awq_mse_multi_kernel(const T *__restrict__ out, const T *__restrict__ ref,
                                                            int64_t chunks, int G, float *__restrict__ partial) {
  __shared__ float red[16][256];
  float acc[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) acc[g] = 0.f;
  for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < chunks; c += (int64_t)gridDim.x * 256) {
    const Vec<T> r = ldg_vec_nt(ref + c * 8);
    float rf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) rf[j] = Elem<T>::ld(r.e[j]);
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      if (g >= G) break;
      const Vec<T> o = ldg_vec_nt(out + ((int64_t)g * chunks + c) * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = Elem<T>::ld(Elem<T>::st(Elem<T>::ld(o.e[j]) - rf[j]));
        acc[g] = __builtin_fmaf(d, d, acc[g]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < 16; ++g) red[g][threadIdx.x] = acc[g];
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o)
      for (int g = 0; g < G; ++g) red[g][threadIdx.x] += red[g][threadIdx.x + o];
    __syncthreads();
  }
  if ((int)threadIdx.x < G) partial[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = red[threadIdx.x][0];
}

// loss[g] += (sum over the group's tiles, in double, fixed order) / (M * N)
__global__ __launch_bounds__(256) void awq_search_finish_kernel(const float *partial, int tiles, int G,
                                                                 double inv_count, float *loss) {
  __shared__ double red[256];
  for (int g = 0; g < G; ++g) {
    double s = 0.0;
    for (int i = threadIdx.x; i < tiles; i += 256) s += (double)partial[(int64_t)g * tiles + i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o >= 1; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) loss[g] += (float)(red[0] * inv_count);
    __syncthreads();
  }
}

bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

// Mode: 1 (default) = x scaled while register-staged; 0 = pre-scaled activations [G, M, K] in the
// workspace (after the per-tile partials) and both tiles by LDS-DMA.  Measured on MI355X
// (scripts/bench_awq_gemm.py, Llama-3-8B shapes, 8192 tokens, 11 alphas; profiles/r02/awq_gemm):
// mode 1 0.94-0.99 PFLOP/s, mode 0 0.79-1.0 including the pre-scale pass -- both at the ceiling
// of a two-buffer, one-barrier-per-K-step pipeline (its ds_read + MFMA + barrier skeleton alone,
// without any global loads, runs 1.2-1.3 PFLOP/s).  MTQ_AMD_AWQ_GEMM_MODE selects.
int awq_mode() {
  static int m = -1;
  if (m < 0) {
    const char *e = getenv("MTQ_AMD_AWQ_GEMM_MODE");
    m = e ? atoi(e) : 1;
  }
  return m;
}

int64_t partial_floats(int64_t M, int64_t N, int G) {
  return ((((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN) * (int64_t)G) + 3) / 4 * 4;  // 16-B aligned
}

}  // namespace

extern "C" int64_t mtq_awq_search_gemm_workspace_floats(int64_t M, int64_t N, int64_t K, int G) {
  if (M < 1 || N < 1 || K < 1 || G < 1) return 0;
  int64_t w = partial_floats(M, N, G);
  if (awq_mode() == 0) w += (G * M * K + 1) / 2;  // xs [G, M, K] in 16-bit elements
  return w;
}

extern "C" int mtq_awq_search_gemm(const void *x, const void *sinv, const void *wq, const void *bias,
                                   const void *yref, int64_t M, int64_t N, int64_t K, int dtype,
                                   int G, float *loss, float *workspace, int64_t workspace_floats,
                                   hipStream_t stream) {
  if (M < 1 || N < 1 || K < kBK || K % kBK != 0 || G < 1 || G > 64) return MTQ_ERR_INVALID_ARG;
  if (!x || !sinv || !wq || !yref || !loss || !workspace) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(sinv) || !al16(wq) || !al16(workspace)) return MTQ_ERR_INVALID_ARG;
  if (M * K >= ((int64_t)1 << 31) || N * K >= ((int64_t)1 << 31) || N % 8 != 0 || !al16(yref))
    return MTQ_ERR_INVALID_ARG;
  const int64_t tiles_m = (M + kBM - 1) / kBM, tiles_n = (N + kBN - 1) / kBN;
  const int64_t tiles = tiles_m * tiles_n;
  if (workspace_floats < mtq_awq_search_gemm_workspace_floats(M, N, K, G) ||
      tiles * G > (int64_t)INT32_MAX)
    return MTQ_ERR_INVALID_ARG;
  const bool pre = awq_mode() == 0;
  const void *xa = x;
  if (pre) {
    void *xs = workspace + partial_floats(M, N, G);
    const int64_t chunks = M * K / 8;
    const unsigned gb = (unsigned)((chunks + 255) / 256);
    if (dtype == MTQ_BF16)
      awq_prescale_kernel<__bf16><<<gb, 256, 0, stream>>>((const __bf16 *)x, (const __bf16 *)sinv,
                                                          (__bf16 *)xs, chunks, K / 8, G);
    else
      awq_prescale_kernel<_Float16><<<gb, 256, 0, stream>>>((const _Float16 *)x, (const _Float16 *)sinv,
                                                            (_Float16 *)xs, chunks, K / 8, G);
    int st = host_check_launch();
    if (st != MTQ_OK) return st;
    xa = xs;
  }
  AwqGemmArgs a{xa, sinv, wq, bias, yref, workspace, M, N, K, (int)tiles_m, (int)tiles_n, G};
  const dim3 grid((unsigned)(tiles * G));
  static int probe = -1;
  if (probe < 0) {
    const char *e = getenv("MTQ_AMD_AWQ_GEMM_PROBE");
    probe = e ? atoi(e) : 0;
  }
#define MTQ_AWQ_LAUNCH(TT, PR)                                                                     \
  do {                                                                                             \
    if (probe == 1)                                                                                \
      awq_search_gemm_kernel<TT, PR, 1><<<grid, kThreads, 0, stream>>>(a);                          \
    else if (probe == 2)                                                                           \
      awq_search_gemm_kernel<TT, PR, 2><<<grid, kThreads, 0, stream>>>(a);                          \
    else                                                                                           \
      awq_search_gemm_kernel<TT, PR, 0><<<grid, kThreads, 0, stream>>>(a);                          \
  } while (0)
  if (dtype == MTQ_BF16) {
    if (pre)
      MTQ_AWQ_LAUNCH(__bf16, true);
    else
      MTQ_AWQ_LAUNCH(__bf16, false);
  } else {
    if (pre)
      awq_search_gemm_kernel<_Float16, true, 0><<<grid, kThreads, 0, stream>>>(a);
    else
      awq_search_gemm_kernel<_Float16, false, 0><<<grid, kThreads, 0, stream>>>(a);
  }
#undef MTQ_AWQ_LAUNCH
  int st = host_check_launch();
  if (st != MTQ_OK) return st;
  awq_search_finish_kernel<<<1, 256, 0, stream>>>(workspace, (int)tiles, G, 1.0 / ((double)M * (double)N),
                                                  loss);
  return host_check_launch();
}

extern "C" int64_t mtq_awq_mse_multi_workspace_floats(int64_t n, int G) {
  if (n < 1 || G < 1) return 0;
  const int64_t chunks = n / 8;
  int64_t grid = (chunks + 255) / 256;
  grid = grid < 2048 ? grid : 2048;
  return grid * G;
}

extern "C" int mtq_awq_mse_multi(const void *out, const void *ref, int64_t n, int dtype, int G, float *loss,
                                 float *workspace, int64_t workspace_floats, hipStream_t stream) {
  if (n < 8 || n % 8 != 0 || G < 1 || G > 16 || !out || !ref || !loss || !workspace) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (!al16(out) || !al16(ref)) return MTQ_ERR_INVALID_ARG;
  const int64_t grid = mtq_awq_mse_multi_workspace_floats(n, G) / G;
  if (workspace_floats < grid * G) return MTQ_ERR_INVALID_ARG;
  if (dtype == MTQ_BF16)
    awq_mse_multi_kernel<__bf16><<<(unsigned)grid, 256, 0, stream>>>((const __bf16 *)out, (const __bf16 *)ref,
                                                                    n / 8, G, workspace);
  else
    awq_mse_multi_kernel<_Float16><<<(unsigned)grid, 256, 0, stream>>>((const _Float16 *)out,
                                                                      (const _Float16 *)ref, n / 8, G, workspace);
  int st = host_check_launch();
  if (st != MTQ_OK) return st;
  awq_search_finish_kernel<<<1, 256, 0, stream>>>(workspace, (int)grid, G, 1.0 / (double)n, loss);
  return host_check_launch();
}

extern "C" int mtq_awq_prescale(const void *x, const void *sinv, void *xs, int64_t M, int64_t K, int dtype, int G,
                                hipStream_t stream) {
  if (M < 1 || K < 8 || K % 8 != 0 || G < 1 || !x || !sinv || !xs) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(sinv) || !al16(xs)) return MTQ_ERR_INVALID_ARG;
  const int64_t chunks = M * K / 8;
  const unsigned gb = (unsigned)((chunks + 255) / 256);
  if (dtype == MTQ_BF16)
    awq_prescale_kernel<__bf16><<<gb, 256, 0, stream>>>((const __bf16 *)x, (const __bf16 *)sinv, (__bf16 *)xs,
                                                        chunks, K / 8, G);
  else
    awq_prescale_kernel<_Float16><<<gb, 256, 0, stream>>>((const _Float16 *)x, (const _Float16 *)sinv,
                                                          (_Float16 *)xs, chunks, K / 8, G);
  return host_check_launch();
}
