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
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// ---------------------------------------------------------------------------------------------
// r03 search kernel: two wave groups in ping-pong, half-tile LDS-DMA ring, counted vmcnt.
//
// 256 x 256 output tile per 512-thread workgroup, 8 waves = 2 groups of 4 (group g = rows
// g*128 .. +128, wave wn of the group = columns wn*64 .. +64), 16x16x32 MFMA (the shape the chip
// clocks higher on random data, MI355X_MICROARCH.md 'DVFS give-back' (7)), K tile 64.
// A K tile is staged as four 16 KiB half-tiles -- A0/A1 = the rows of m-quadrant 0/1 of both
// groups, B0/B1 = the columns of n-quadrant 0/1 of all four waves -- so that each half is
// (re)loaded as soon as its last reader is done with it.  A wave computes its 128 x 64 block in
// four phases, one 64 x 32 quadrant (16 MFMAs over K 64) each, in the order (m0,n0) (m0,n1)
// (m1,n1) (m1,n0): phase q reads the fragments it needs (12, 4, 8, 4 ds_read_b128 -- A or B
// fragments are reused from the previous phase), issues the LDS-DMA of one half of the NEXT K
// tile into the other buffer (A0, B0, B1, A1 for q = 0..3), waits with a counted vmcnt for the
// half the next phase reads (never vmcnt(0) in the loop), then [barrier, MFMAs, barrier].  Group
// 1 starts one barrier late, so on every SIMD one wave runs its MFMA burst while its partner
// issues its reads and loads (cdna_hip_programming.md §5, "The 256² 8-phase template": the
// stagger, the counted waits, setprio around the bursts; "Read a staged buffer one phase AFTER
// the wait that retires it" -- the wait precedes the barrier that each group passes before the
// read, which with the stagger means before the phase's first barrier).
// Operands: xs = T(x * (1/s_g)) pre-scaled for all alphas (awq_prescale_kernel) and wq, both
// [rows][K] with K contiguous, both by LDS-DMA with the 16-byte chunk c of LDS row L stored at
// chunk c ^ ((L >> 1) & 7) (the XOR applied on the global source address, rule 21): conflict-free
// ds_read_b128 fragment reads, whose XOR term is then the lane constant (lane >> 1) & 7.
// Epilogue as the r02 kernel: yref tile through LDS, bias, output and difference rounded to T,
// fp32 square-sum per lane in a fixed order, fixed-order block reduction -> deterministic.
namespace pp {  // tile sizes kBM, kBN, kBK and kThreads as the r02 kernel
constexpr int kHalf = 16384;         // 128 rows x 64 k x 2 B
constexpr int kBuf = 4 * kHalf;      // A0 A1 B0 B1 of one K tile
constexpr int kLds = 2 * kBuf;       // two K tiles in flight (the yref tile reuses it: 256 x 256 x 2)
}  // namespace pp

template <typename T> struct Mfma16;
template <> struct Mfma16<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mfma16<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x4 mma(v8 a, v8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// PROBE (measurement builds only, MTQ_AMD_AWQ_GEMM_PROBE=1): no global loads in the K loop -- the
// ds_read + MFMA + barrier skeleton alone (the loss is then meaningless)
// CLAMP (PH 4): the last K tile re-loads itself (no branch in the loop) instead of skipping its
// loads (PH 5 always clamps).  Variants measured and dropped in r03 (profiles/r03/awq): two phases
// per K tile, the untransposed MFMA orientation, reference rows by direct loads, DMA rounds
// interleaved into the MFMA burst -- none faster than PH 5.
template <typename T, bool HAS_BIAS, int PH, int PROBE = 0, bool CLAMP = true>
__global__ __launch_bounds__(kThreads) void awq_search_pp_kernel(AwqGemmArgs p) {
  using namespace pp;
  typedef typename Mfma16<T>::v8 v8;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wn = wave & 3;

  // XCD-aware remap + grouped tile order, as the r02 kernel
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, rr8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + orig / 8;
  const int tiles = p.tiles_m * p.tiles_n;
  const int g = wgid / tiles;
  const int tile = wgid - g * tiles;
  constexpr int kGroupM = 8;
  const int gm = tile / (kGroupM * p.tiles_n);
  const int first_m = gm * kGroupM;
  const int gsz = p.tiles_m - first_m < kGroupM ? p.tiles_m - first_m : kGroupM;
  const int tin = tile - gm * kGroupM * p.tiles_n;
  const int tm = first_m + tin % gsz, tn = tin / gsz;
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;
  const T *X = reinterpret_cast<const T *>(p.x) + (int64_t)g * p.M * K;
  const T *W = reinterpret_cast<const T *>(p.wq) + (int64_t)g * p.N * K;

  // ---- LDS-DMA sources: half h / round u of a K tile; each lane writes LDS row
  // rr = u*64 + wave*8 + (lane >> 3) of the half, chunk slot lane & 7
  unsigned a_off[2][2], b_off[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = u * 64 + wave * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((rr >> 1) & 7);
      int64_t row = m0 + (rr >> 6) * 128 + h * 64 + (rr & 63);  // group rr>>6, m-quadrant h
      row = row < p.M ? row : p.M - 1;
      a_off[h][u] = (unsigned)(row * K + chunk * 8);
      int64_t col = n0 + (rr >> 5) * 64 + h * 32 + (rr & 31);  // wave rr>>5, n-quadrant h
      col = col < p.N ? col : p.N - 1;
      b_off[h][u] = (unsigned)(col * K + chunk * 8);
    }
  auto dma = [&](const T *base, unsigned off, unsigned char *dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(base + off),
                                     (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
  };
  // half index q of K tile at k0 into buffer buf: q = 0 A0, 1 B0, 2 B1, 3 A1
  auto load_half = [&](int q, unsigned char *buf, int64_t k0) {
    const bool isA = (q == 0 || q == 3);
    const int h = (q == 0 || q == 1) ? 0 : 1;
    unsigned char *dst = buf + (isA ? h : 2 + h) * kHalf + wave * 1024;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (isA)
        dma(X + k0, a_off[h][u], dst + u * 8192);
      else
        dma(W + k0, b_off[h][u], dst + u * 8192);
    }
  };

  // ---- fragment reads: A m-tile i (16 rows) / B n-tile j, k-step s (32 of the tile's 64)
  const int sw = (lane >> 1) & 7, fr = lane & 15, fq = lane >> 4;
  auto read_a = [&](const unsigned char *buf, int i, int s) -> v8 {
    const int L = (i >> 2) * 128 + grp * 64 + (i & 3) * 16 + fr;
    return *reinterpret_cast<const v8 *>(buf + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };
  auto read_b = [&](const unsigned char *buf, int j, int s) -> v8 {
    const int L = (j >> 1) * 128 + wn * 32 + (j & 1) * 16 + fr;
    return *reinterpret_cast<const v8 *>(buf + 2 * kHalf + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (int)(K / kBK);
  // prologue: K tile 0 in full (A0 B0 B1 A1); phase 0 needs A0 and B0
  if constexpr (PH == 5) {
    // stream order B0 A0 B1 A1 of tile 0, then B0 A0 of tile 1 (see the PH 5 loop)
    const int64_t k1 = (int64_t)(nt > 1 ? 1 : 0) * kBK;
    load_half(1, lds, 0);
    load_half(0, lds, 0);
    load_half(2, lds, 0);
    load_half(3, lds, 0);
    load_half(1, lds + kBuf, k1);
    load_half(0, lds + kBuf, k1);
    wait_vm<8>();
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) load_half(q, lds, 0);
    wait_vm<4>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger (wave-uniform: scalar branch)

  if constexpr (PH == 5) {
    // Four phases per K tile as PH 4, but the B0 fragments (n-quadrant 0, used by the first and
    // the last phase) stay in registers from phase 0 to phase 3, so every half-tile's last LDS
    // read is early: A0 phase 1, B0 phase 0, B1 phase 2, A1 phase 3 (phase 3 reads nothing).
    // Each half of tile t+2 / t+1 can then be loaded two phases after the same half of tile t /
    // t-1 was last read (the stagger margin) and still has 4-5 phases to land:
    //   phase 0: B1(t+1) -> buffer t+1     phase 2: B0(t+2) -> buffer t (B0(t) is in registers)
    //   phase 1: A1(t+1) -> buffer t+1     phase 3: A0(t+2) -> buffer t (A0(t) read in phase 1)
    // Waits (before each phase's first barrier, for the next phase's reads): vmcnt(8) -- four
    // halves issued after the one needed may stay in flight -- and vmcnt(10) in phase 2, whose
    // successor reads nothing new.
    v8 af[4][2], b0f[2][2], b1f[2][2];
    for (int t = 0; t < nt; ++t) {
      unsigned char *cur = lds + (t & 1) * kBuf;
      unsigned char *nx1 = lds + ((t + 1) & 1) * kBuf;
      const int64_t k1 = (int64_t)(t + 1 < nt ? t + 1 : nt - 1) * kBK;  // past the end: harmless re-loads
      const int64_t k2 = (int64_t)(t + 2 < nt ? t + 2 : nt - 1) * kBK;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int mq = (q == 0 || q == 1) ? 0 : 1;
        const int nq = (q == 1 || q == 2) ? 1 : 0;
        if (q == 0 || q == 2) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][s2] = read_a(cur, 4 * mq + i, s2);
        }
        if (q == 0) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int j = 0; j < 2; ++j) b0f[j][s2] = read_b(cur, j, s2);
        }
        if (q == 1) {
#pragma unroll
          for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
            for (int j = 0; j < 2; ++j) b1f[j][s2] = read_b(cur, 2 + j, s2);
        }
        // this phase's half: q0 B1(t+1), q1 A1(t+1) -> buffer t+1; q2 B0(t+2), q3 A0(t+2) -> buffer t
        const int hq = q == 0 ? 2 : q == 1 ? 3 : q == 2 ? 1 : 0;
        unsigned char *hb = q < 2 ? nx1 : cur;
        const int64_t hk = q < 2 ? k1 : k2;
        if (PROBE == 0) {
          load_half(hq, hb, hk);
          if (q == 2)
            wait_vm<10>();
          else
            wait_vm<8>();
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) {
          const int s2 = kk >> 3, j = (kk >> 2) & 1, i = kk & 3;
          const v8 bb = nq ? b1f[j][s2] : b0f[j][s2];
          acc[4 * mq + i][2 * nq + j] = Mfma16<T>::mma(bb, af[i][s2], acc[4 * mq + i][2 * nq + j]);
        }
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
      }
    }
  } else {
    static_assert(PH == 4, "PH 4 or 5");
    v8 af[4][2], bf[2][2];
    for (int t = 0; t < nt; ++t) {
      unsigned char *cur = lds + (t & 1) * kBuf;
      unsigned char *nxt = lds + ((t + 1) & 1) * kBuf;
      const int64_t kn = (int64_t)(CLAMP ? (t + 1 < nt ? t + 1 : nt - 1) : t + 1) * kBK;
      const bool more = PROBE == 0 && (CLAMP || t + 1 < nt);  // the last tile loads nothing and drains
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int mq = (q == 0 || q == 1) ? 0 : 1;
        const int nq = (q == 1 || q == 2) ? 1 : 0;
        if (q == 0 || q == 2) {
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i][s] = read_a(cur, 4 * mq + i, s);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j) bf[j][s] = read_b(cur, 2 * nq + j, s);
        if (more) {
          load_half(q, nxt, kn);
          if (q == 2)
            wait_vm<6>();
          else
            wait_vm<4>();
        } else {
          wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j)  // the A operand (W fragment) held for 4 MFMAs
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[4 * mq + i][2 * nq + j] = Mfma16<T>::mma(bf[j][s], af[i][s], acc[4 * mq + i][2 * nq + j]);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // balance the stagger

  float sum = 0.f;
  // ---- epilogue.  The MFMAs computed out^T (W fragment as the A operand), so a lane's four
  // accumulators of tile (i, j) are out[m][n .. n+3] with m = 16 i + (lane & 15), n = 16 j +
  // 4 (lane >> 4): one 8-byte LDS read of the staged reference tile each.  Bias, output and
  // difference rounded to T, fp32 square-sum in a fixed order.
  const T *Y = reinterpret_cast<const T *>(p.yref);
  const T *Bi = reinterpret_cast<const T *>(p.bias);
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  u32x2_t yv[8][4];
  bool rok[8], cok[4];
  int64_t coln[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t c = n0 + wn * 64 + 16 * j + 4 * fq;
    cok[j] = c < p.N;  // N % 8 == 0: the 4 columns are all in or all out
    coln[j] = cok[j] ? c : p.N - 4;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) rok[i] = m0 + grp * 128 + 16 * i + fr < p.M;
  {
    // the yref tile [256 x 256] through LDS: 16 DMA rounds in flight, row r's 16-byte chunk c
    // stored at chunk c ^ (r & 15) (source-side XOR), so the 16 rows of a b64 read hit 16 slots
    wait_vm<0>();
    __syncthreads();
    {
      const int slot = tid & 31;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int rr = u * 16 + (tid >> 5);
        int64_t row = m0 + rr;
        row = row < p.M ? row : p.M - 1;
        int64_t col = n0 + (int64_t)((slot ^ (rr & 15)) * 8);
        col = col < p.N ? col : p.N - 8;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(Y + row * p.N + col),
                                         (__attribute__((address_space(3))) void *)(lds + u * 8192 + wave * 1024),
                                         16, 0, 0);
      }
    }
    wait_vm<0>();
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int rr = grp * 128 + 16 * i + fr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cl = wn * 64 + 16 * j + 4 * fq;
        yv[i][j] = *reinterpret_cast<const u32x2_t *>(lds + rr * 512 + (((cl >> 3) ^ (rr & 15)) << 4) + (cl & 7) * 2);
      }
    }
  }
  float bj[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bj[j][e] = HAS_BIAS ? Elem<T>::ld(Bi[coln[j] + e]) : 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T yr[4];
      __builtin_memcpy(yr, &yv[i][j], 8);
      const bool ok = rok[i] && cok[j];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = Elem<T>::ld(Elem<T>::st(acc[i][j][e] + bj[j][e]));
        const float d = Elem<T>::ld(Elem<T>::st(y - Elem<T>::ld(yr[e])));
        sum = ok ? __builtin_fmaf(d, d, sum) : sum;
      }
    }
  }
  __syncthreads();
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

// ---------------------------------------------------------------------------------------------
// W4 (mode 2, MTQ_AMD_AWQ_PP_PHASES=6): four waves, ONE wave per SIMD, each wave a 128 x 128 block
// of the 256 x 256 tile (8 x 8 tiles of 16x16x32, 256 accumulator registers: VGPR + AGPR file of a
// 512-register wave).  Per K tile (64) a wave reads 32 KiB of fragments (2/3 of the two-group
// layout's LDS traffic per MFMA) and meets ONE barrier:
//   phase A: MFMAs of k-step 0 (64) with the k-step 1 fragments of the same tile read beside them;
//   vmcnt(0) (tile t+1 landed) + lgkmcnt(0), barrier;
//   phase B: MFMAs of k-step 1 (64) with the k-step 0 fragments of tile t+1 read and tile t+2's
//            16 LDS-DMA rounds issued into the buffer tile t just vacated.
// Tile t+2's loads then have phase B of tile t and phase A of tile t+1 (~2k MFMA cycles) to land.
// Fragments are double-buffered in registers (F0 / F1).  Epilogue as the pp kernel (transposed
// accumulators, reference rows by 8-byte loads).
// the accumulators pinned to AGPRs ("+a"): hipcc otherwise shuffles the 256 loop-carried
// accumulators between the two register files every iteration (v_accvgpr_read/write/mov)
template <typename T>
__device__ __forceinline__ void mma_agpr(f32x4 &c, typename Mfma16<T>::v8 a, typename Mfma16<T>::v8 b) {
  if constexpr (__is_same(T, __bf16))
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

template <typename T, bool HAS_BIAS>
__global__ __launch_bounds__(256, 1) void awq_search_w4_kernel(AwqGemmArgs p) {
  typedef typename Mfma16<T>::v8 v8;
  constexpr int kStage = 65536;  // A [256][64] + B [256][64] bf16/f16
  __shared__ __attribute__((aligned(16))) unsigned char lds[2 * kStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg / 8, rr8 = nwg % 8, xcd = orig % 8;
  const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + orig / 8;
  const int tiles = p.tiles_m * p.tiles_n;
  const int g = wgid / tiles;
  const int tile = wgid - g * tiles;
  constexpr int kGroupM = 8;
  const int gm = tile / (kGroupM * p.tiles_n);
  const int first_m = gm * kGroupM;
  const int gsz = p.tiles_m - first_m < kGroupM ? p.tiles_m - first_m : kGroupM;
  const int tin = tile - gm * kGroupM * p.tiles_n;
  const int tm = first_m + tin % gsz, tn = tin / gsz;
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;
  const T *X = reinterpret_cast<const T *>(p.x) + (int64_t)g * p.M * K;
  const T *W = reinterpret_cast<const T *>(p.wq) + (int64_t)g * p.N * K;

  // LDS-DMA: round u (0..7) of an operand writes image bytes [u * 4 KiB + tid * 16): row
  // u * 32 + (tid >> 3), chunk slot tid & 7 holding source chunk slot ^ ((row >> 1) & 7)
  unsigned a_off[8], b_off[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int row = u * 32 + (tid >> 3);
    const int chunk = (tid & 7) ^ ((row >> 1) & 7);
    int64_t ra = m0 + row;
    ra = ra < p.M ? ra : p.M - 1;
    a_off[u] = (unsigned)(ra * K + chunk * 8);
    int64_t rb = n0 + row;
    rb = rb < p.N ? rb : p.N - 1;
    b_off[u] = (unsigned)(rb * K + chunk * 8);
  }
  auto dma = [&](const T *base, unsigned off, unsigned char *dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(base + off),
                                     (__attribute__((address_space(3))) void *)dst, 16, 0, 0);
  };
  auto load_a = [&](unsigned char *stage, int64_t k0, int u) { dma(X + k0, a_off[u], stage + u * 4096 + wave * 1024); };
  auto load_b = [&](unsigned char *stage, int64_t k0, int u) {
    dma(W + k0, b_off[u], stage + 32768 + u * 4096 + wave * 1024);
  };
  const int sw = (lane >> 1) & 7, fr = lane & 15, fq = lane >> 4;
  auto read_a = [&](const unsigned char *stage, int i, int s) -> v8 {
    const int L = wm * 128 + 16 * i + fr;
    return *reinterpret_cast<const v8 *>(stage + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };
  auto read_b = [&](const unsigned char *stage, int j, int s) -> v8 {
    const int L = wn * 128 + 16 * j + fr;
    return *reinterpret_cast<const v8 *>(stage + 32768 + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nt = (int)(K / kBK);
  auto kof = [&](int t) -> int64_t { return (int64_t)(t < nt ? t : nt - 1) * kBK; };
  // prologue: tiles 0 and 1 (a clamped re-load of tile 0 when K = 64), tile 0's k-step 0 fragments
#pragma unroll
  for (int u = 0; u < 8; ++u) { load_a(lds, 0, u); load_b(lds, 0, u); }
#pragma unroll
  for (int u = 0; u < 8; ++u) { load_a(lds + kStage, kof(1), u); load_b(lds + kStage, kof(1), u); }
  wait_vm<16>();
  __syncthreads();
  // registers: A fragments double-buffered (fa0 / fa1, 64 VGPRs), B fragments rotating in place
  // (fb[j] is re-read for the next k-step as soon as its 8 MFMAs are issued, 32 VGPRs)
  v8 fa0[8], fa1[8], fb[8];
  // the asm MFMAs are opaque to hipcc's hazard padding (cdna_hip_programming.md §5.7 item 2):
  // wait states between the compiler's accumulator initialisation and the first MFMA here, and
  // between the last MFMA and the compiler's accumulator reads after the loop
  asm volatile("s_nop 4" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = read_a(lds, i, 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb[j] = read_b(lds, j, 0);
  __builtin_amdgcn_s_waitcnt(0xC07F);  // loop entry with no LDS read pending (as the back-edge)

  for (int t = 0; t < nt; ++t) {
    unsigned char *cur = lds + (t & 1) * kStage;
    unsigned char *nxt = lds + ((t + 1) & 1) * kStage;
    // ---- phase A: k-step 0 of tile t; the k-step 1 fragments of tile t read beside it
#pragma unroll
    for (int i = 0; i < 8; ++i) fa1[i] = read_a(cur, i, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int i = 0; i < 8; ++i) mma_agpr<T>(acc[i][j], fb[j], fa0[i]);
      fb[j] = read_b(cur, j, 1);
    }
    wait_vm<0>();  // tile t+1 (this wave's rounds) landed
    // lgkmcnt(0) through the builtin, which hipcc's wait insertion sees (an asm one it does not,
    // and it would then wait lgkmcnt(0) again before the first MFMA of the next phase)
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    // ---- phase B: k-step 1 of tile t; tile t+1's k-step 0 fragments and tile t+2's DMA
#pragma unroll
    for (int i = 0; i < 8; ++i) fa0[i] = read_a(nxt, i, 0);
    const int64_t k2 = kof(t + 2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      // two of tile t+2's sixteen DMA rounds per 8 MFMAs, spread over the phase (issuing all sixteen
      // up front stalls the wave's MFMA issue behind them: 9.9 vs 8.8 ms on gate_proj,
      // profiles/r03/awq/search_bench_w4_front.json)
      load_a(cur, k2, j);
      load_b(cur, k2, j);
#pragma unroll
      for (int i = 0; i < 8; ++i) mma_agpr<T>(acc[i][j], fb[j], fa1[i]);
      fb[j] = read_b(nxt, j, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // the next phase A then starts without a wait
  }
  wait_vm<0>();
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

  // ---- epilogue: lane holds out[m][n .. n+3], m = wm*128 + 16 i + fr, n = wn*128 + 16 j + 4 fq
  const T *Y = reinterpret_cast<const T *>(p.yref);
  const T *Bi = reinterpret_cast<const T *>(p.bias);
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  float sum = 0.f;
#pragma unroll
  for (int jh = 0; jh < 2; ++jh) {  // two halves of the columns: 32 reference loads in flight each
    u32x2_t yv[8][4];
    bool cok[4];
    int64_t coln[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int64_t c = n0 + wn * 128 + 16 * (4 * jh + jj) + 4 * fq;
      cok[jj] = c < p.N;
      coln[jj] = cok[jj] ? c : p.N - 4;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int64_t r = m0 + wm * 128 + 16 * i + fr;
      r = r < p.M ? r : p.M - 1;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) yv[i][jj] = *reinterpret_cast<const u32x2_t *>(Y + r * p.N + coln[jj]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool rok = m0 + wm * 128 + 16 * i + fr < p.M;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        T yr[4];
        __builtin_memcpy(yr, &yv[i][jj], 8);
        const bool ok = rok && cok[jj];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float bj = HAS_BIAS ? Elem<T>::ld(Bi[coln[jj] + e]) : 0.f;
          const float y = Elem<T>::ld(Elem<T>::st(acc[i][4 * jh + jj][e] + bj));
          const float d = Elem<T>::ld(Elem<T>::st(y - Elem<T>::ld(yr[e])));
          sum = ok ? __builtin_fmaf(d, d, sum) : sum;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  __syncthreads();
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) p.partial[(int64_t)g * tiles + tile] = (red[0] + red[1]) + (red[2] + red[3]);
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

// Mode: 2 (default, r03) = pre-scaled activations [G, M, K] in the workspace + the ping-pong
// kernel (awq_search_pp_kernel); 1 = the r02 kernel with x scaled while register-staged; 0 = the
// r02 kernel on pre-scaled activations.  r02 measurements (scripts/bench_awq_gemm.py, Llama-3-8B
// shapes, 8192 tokens, 11 alphas; profiles/r02/awq): mode 1 0.94-0.99 PFLOP/s, mode 0 0.79-1.0
// including the pre-scale pass -- both at the ceiling of a two-buffer, one-barrier-per-K-step
// pipeline.  MTQ_AMD_AWQ_GEMM_MODE selects.
int awq_mode() {  // read per call: A/B runs switch it inside one process
  const char *e = getenv("MTQ_AMD_AWQ_GEMM_MODE");
  return e ? atoi(e) : 2;
}

int64_t partial_floats(int64_t M, int64_t N, int G) {
  return ((((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN) * (int64_t)G) + 3) / 4 * 4;  // 16-B aligned
}

}  // namespace

extern "C" int64_t mtq_awq_search_gemm_workspace_floats(int64_t M, int64_t N, int64_t K, int G) {
  if (M < 1 || N < 1 || K < 1 || G < 1) return 0;
  int64_t w = partial_floats(M, N, G);
  if (awq_mode() != 1) w += (G * M * K + 1) / 2;  // xs [G, M, K] in 16-bit elements
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
  const int mode = awq_mode();
  const bool pre = mode != 1;
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
  const char *pe_ = getenv("MTQ_AMD_AWQ_GEMM_PROBE");
  const int probe = pe_ ? atoi(pe_) : 0;
#define MTQ_AWQ_LAUNCH(TT, PR)                                                                     \
  do {                                                                                             \
    if (probe == 1)                                                                                \
      awq_search_gemm_kernel<TT, PR, 1><<<grid, kThreads, 0, stream>>>(a);                          \
    else if (probe == 2)                                                                           \
      awq_search_gemm_kernel<TT, PR, 2><<<grid, kThreads, 0, stream>>>(a);                          \
    else                                                                                           \
      awq_search_gemm_kernel<TT, PR, 0><<<grid, kThreads, 0, stream>>>(a);                          \
  } while (0)
  if (mode == 2) {
    // schedule (A/B switch, profiles/r03/awq): 5 = default; 4 = the first r03 schedule (fragments
    // re-read per phase; MTQ_AMD_AWQ_PP_CLAMP=0 skips the last tile's loads behind a branch);
    // 6 = W4, one 128 x 128 wave per SIMD
    const char *pe = getenv("MTQ_AMD_AWQ_PP_PHASES");
    const int phs = pe ? atoi(pe) : 5;
    const char *ce = getenv("MTQ_AMD_AWQ_PP_CLAMP");
    const bool clamp = ce ? atoi(ce) != 0 : true;
#define MTQ_PP(TT, BB)                                                                              \
  do {                                                                                             \
    if (phs == 6)                                                                                  \
      awq_search_w4_kernel<TT, BB><<<grid, 256, 0, stream>>>(a);                                    \
    else if (phs == 4 && probe == 1)                                                               \
      awq_search_pp_kernel<TT, BB, 4, 1><<<grid, kThreads, 0, stream>>>(a);                         \
    else if (phs == 4 && !clamp)                                                                   \
      awq_search_pp_kernel<TT, BB, 4, 0, false><<<grid, kThreads, 0, stream>>>(a);                  \
    else if (phs == 4)                                                                             \
      awq_search_pp_kernel<TT, BB, 4><<<grid, kThreads, 0, stream>>>(a);                            \
    else if (probe == 1)                                                                           \
      awq_search_pp_kernel<TT, BB, 5, 1><<<grid, kThreads, 0, stream>>>(a);                         \
    else                                                                                           \
      awq_search_pp_kernel<TT, BB, 5><<<grid, kThreads, 0, stream>>>(a);                            \
  } while (0)
    if (dtype == MTQ_BF16) {
      if (bias)
        MTQ_PP(__bf16, true);
      else
        MTQ_PP(__bf16, false);
    } else {
      if (bias)
        MTQ_PP(_Float16, true);
      else
        MTQ_PP(_Float16, false);
    }
#undef MTQ_PP
  } else if (dtype == MTQ_BF16) {
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
