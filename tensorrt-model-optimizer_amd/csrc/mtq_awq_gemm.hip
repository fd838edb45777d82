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
// with the x * (1/s) product (rounded to T as the reference's bf16 multiply is) written once for
// all alphas by awq_prescale_kernel, bf16/f16 MFMA (v_mfma_f32_16x16x32, fp32 accumulate), and
// the bias, output rounding, difference (rounded to T, as the reference's subtraction) and
// square-sum done on the accumulators -- out never reaches HBM.  wq[g] = qdq_int4_b128(W * s_g)
// comes from mtq_block_quant_dynamic_multi (one HBM pass for all alphas).  Grouping the alphas in
// one grid (tile x g) also fills the 256 CUs for the narrow linears (k/v_proj: 4 x 32 tiles per
// alpha).  The search kernel (awq_search_pp_kernel below) describes its tiling and schedule; the
// loss is summed per lane in fp32 in a fixed order, across the workgroup in a fixed order, and
// the per-tile partials are folded in double by a one-block-per-alpha finishing kernel:
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

constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 512;
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

// buffer descriptor from wave-uniform inputs (cdna_hip_programming.md T20: no waterfall loops)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// buffer_load_dwordx4 ... lds (16 B per lane).  The builtin exists only in the device pass; named
// in a kernel body seen by the host pass it drops that kernel's host stub, hence the guard.
#if defined(__HIP_DEVICE_COMPILE__)
#define AWQ_DMA(rsrc, lds, voff, soff) \
  __builtin_amdgcn_raw_ptr_buffer_load_lds((rsrc), (__attribute__((address_space(3))) void *)(lds), 16, (voff), (soff), 0, 0)
#else
#define AWQ_DMA(rsrc, lds, voff, soff) ((void)(rsrc), (void)(lds), (void)(voff), (void)(soff))
#endif

// Variants measured and dropped (profiles/r03/awq, profiles/r04/awq): two phases per K tile, the
// untransposed MFMA orientation, reference rows by direct loads, DMA rounds interleaved into the
// MFMA burst, fragments re-read per phase (r03 schedule 4), one 128 x 128 wave per SIMD (W4),
// 4 or 16 row tiles per XCD group, buffer_load ... lds instead of global_load_lds.
template <typename T, bool HAS_BIAS>
__global__ __launch_bounds__(kThreads) void awq_search_pp_kernel(AwqGemmArgs p) {
  using namespace pp;
  typedef typename Mfma16<T>::v8 v8;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wn = wave & 3;

  // Tile order (r04): units of 8 row tiles x 4 column tiles, one per XCD round (32 workgroups =
  // the XCD's 32 CUs; the 8 x 4 shape maximises the K-slice reuse in the XCD's L2: 12 slices per
  // K step for 32 tiles).  Unit u = ((g * NN4) + n4) * MGN + mg runs on XCD u % 8 in local round
  // u / 8 (blocks are dispatched to XCDs round-robin by blockIdx % 8 -- a speed assumption only,
  // any placement is correct), so the eight XCDs work on the SAME alpha and column range at once,
  // on different row groups: every W panel comes from HBM once and is shared through the
  // Infinity Cache, and the alpha's activations stay resident there (r03 gave each XCD a
  // contiguous range of the whole grid, so each W panel was fetched once per row group).
  // Measured (scripts/exp/awq_exp.hip, profiles/r04/awq): gate_proj 7.89 -> 7.77 ms, q_proj 2.30
  // -> 2.20 ms; with the buffer-DMA below 7.70 / 2.17.  Slots past the matrix edge exit at once.
  const int orig = blockIdx.x;
  const int tiles = p.tiles_m * p.tiles_n;
  int g, tm, tn;
  {
    const int xcd = orig % 8, li = orig / 8;
    const int slot = li % 32, u = (li / 32) * 8 + xcd;
    const int mgn = (p.tiles_m + 7) / 8, nn4 = (p.tiles_n + 3) / 4;
    const int mg = u % mgn, n4 = (u / mgn) % nn4;
    g = u / (mgn * nn4);
    tm = mg * 8 + slot % 8;
    tn = n4 * 4 + slot / 8;
    if (g >= p.G || tm >= p.tiles_m || tn >= p.tiles_n) return;  // the whole workgroup, before any barrier
  }
  const int tile = tm * p.tiles_n + tn;
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
  // buffer_load ... lds through one descriptor per operand: the per-lane offset is loop-invariant
  // and the K advance is the scalar offset (global_load_lds needed a 64-bit address per DMA;
  // 1-2 % faster, scripts/exp/awq_exp.hip)
  const __amdgpu_buffer_rsrc_t xr = wave_rsrc(X, (uint32_t)(p.M * K * 2));
  const __amdgpu_buffer_rsrc_t wr = wave_rsrc(W, (uint32_t)(p.N * K * 2));
  // half index q of K tile at k0 into buffer buf: q = 0 A0, 1 B0, 2 B1, 3 A1
  auto load_half = [&](int q, unsigned char *buf, int64_t k0) {
    const bool isA = (q == 0 || q == 3);
    const int h = (q == 0 || q == 1) ? 0 : 1;
    unsigned char *dst = buf + (isA ? h : 2 + h) * kHalf + wave * 1024;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2));
#pragma unroll
    for (int u = 0; u < 2; ++u) AWQ_DMA(isA ? xr : wr, dst + u * 8192, (isA ? a_off[h][u] : b_off[h][u]) * 2u, soff);
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
  // prologue: K tile 0 in full in the stream order B0 A0 B1 A1, then B0 A0 of tile 1 (the loop's
  // phases 2 and 3 of a virtual tile -1); phase 0 needs A0 and B0
  {
    const int64_t k1 = (int64_t)(nt > 1 ? 1 : 0) * kBK;
    load_half(1, lds, 0);
    load_half(0, lds, 0);
    load_half(2, lds, 0);
    load_half(3, lds, 0);
    load_half(1, lds + kBuf, k1);
    load_half(0, lds + kBuf, k1);
    wait_vm<8>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // the stagger (wave-uniform: scalar branch)

  // Four phases per K tile.  The B0 fragments (n-quadrant 0, used by the first and the last
  // phase) stay in registers from phase 0 to phase 3, so every half-tile's last LDS
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
      load_half(hq, hb, hk);
      if (q == 2)
        wait_vm<10>();
      else
        wait_vm<8>();
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
// r06 search kernel: one wave per SIMD, the K loop at the instruction level.  4 waves per 256 x
// 256 tile, a 128 x 128 block per wave (64 accumulators of 4 fp32 = a[0:255]), K tiles of 64 with
// both operands by LDS-DMA in whole 128-byte rows, two 64 KiB LDS slots, one barrier per tile,
// the reference tile carried by the last two tiles' DMAs.  The K loop is ONE inline-asm statement
// generated by scripts/gen_awq_w4.py (mtq_awq_w4.inc; the schedule is described there): hipcc's
// own waits would drain the prefetch (the r04 W4 HIP variants, §4e), so every wait is counted by
// hand and the compiler sees one opaque statement that names the VGPRs v[120:255] and all AGPRs
// it uses.  Same tile order, operands, roundings and loss as awq_search_pp_kernel (a different
// per-tile square-sum order).  Requires K % 64 == 0, K >= 128 and M * N * 2 < 2^32 (32-bit buffer
// offsets of the reference tile); otherwise the launcher runs the pp kernel.  Kernel time at 8192
// tokens x 11 alphas (profiles/r06/awq/): k / q / gate / down 0.61 / 2.10 / 7.28 / 7.42 ms against
// the pp kernel's 0.62 / 2.23 / 8.01 / 7.67 -- the product default where its limits allow.
#include "mtq_awq_w4.inc"

typedef float w4f2 __attribute__((ext_vector_type(2)));
typedef __bf16 w4b2 __attribute__((ext_vector_type(2)));

template <typename T, bool HAS_BIAS>
__global__ __launch_bounds__(256) void awq_search_w4_kernel(AwqGemmArgs p) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[131072];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int g, tm, tn;
  {  // the pp kernel's tile order (8 x 4 units, one per XCD round)
    const int orig = blockIdx.x;
    const int xcd = orig % 8, li = orig / 8;
    const int slot = li % 32, u = (li / 32) * 8 + xcd;
    const int mgn = (p.tiles_m + 7) / 8, nn4 = (p.tiles_n + 3) / 4;
    const int mg = u % mgn, n4 = (u / mgn) % nn4;
    g = u / (mgn * nn4);
    tm = mg * 8 + slot % 8;
    tn = n4 * 4 + slot / 8;
    if (g >= p.G || tm >= p.tiles_m || tn >= p.tiles_n) return;  // the whole workgroup, before any barrier
  }
  const int tile = tm * p.tiles_n + tn;
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;
  const T *X = reinterpret_cast<const T *>(p.x) + (int64_t)g * p.M * K;
  const T *W = reinterpret_cast<const T *>(p.wq) + (int64_t)g * p.N * K;
  const __amdgpu_buffer_rsrc_t xr = wave_rsrc(X, (uint32_t)(p.M * K * 2));
  const __amdgpu_buffer_rsrc_t wr = wave_rsrc(W, (uint32_t)(p.N * K * 2));
  const __amdgpu_buffer_rsrc_t yr = wave_rsrc(p.yref, (uint32_t)(p.M * p.N * 2));

  // K-tile DMA sources: wave w fills 1 KiB blocks w*8 + u of each operand's 32 KiB tile part (8
  // rows of 128 B); lane l writes row 64 w + 8 u + (l >> 3), stored chunk l & 7 = source chunk
  // c ^ ((row >> 1) & 7).  The instruction offset carries the block step (u % 4) KiB: subtracted here.
  unsigned xo[8], wo[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = 64 * wave + 8 * u + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t row = m0 + r < p.M ? m0 + r : p.M - 1;
    const int64_t col = n0 + r < p.N ? n0 + r : p.N - 1;
    xo[u] = (unsigned)((row * K + 8 * c) * 2) - (unsigned)((u % 4) * 1024);
    wo[u] = (unsigned)((col * K + 8 * c) * 2) - (unsigned)((u % 4) * 1024);
  }
  // fragment reads: row 16 i + fr of the wave's block, 16-byte chunk 4 s + fq of k-half s
  const int fr = lane & 15, fq = lane >> 4;
  const unsigned lds0 = (unsigned)(uintptr_t)lds;
  const unsigned lt0 = fr * 128 + ((fq ^ ((fr >> 1) & 7)) << 4);
  const unsigned lt1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) << 4);
  const unsigned xb0 = lds0 + wm * 16384 + lt0, xb1 = lds0 + wm * 16384 + lt1;
  const unsigned wb0 = lds0 + 32768 + wn * 16384 + lt0, wb1 = lds0 + 32768 + wn * 16384 + lt1;
  const unsigned m0b = __builtin_amdgcn_readfirstlane(lds0 + wave * 8192);
  const unsigned klast = __builtin_amdgcn_readfirstlane((unsigned)((K / 64 - 1) * 128));
  unsigned cnt = __builtin_amdgcn_readfirstlane((unsigned)((K / 64 - 2) / 2));  // two tiles per pass
  // reference-tile DMA sources: half h (rows 128 h ..) lands in slot (K / 64 + h) % 2; wave w
  // fills rows 32 w + 2 u + (l >> 5), u = 0..15, row r's 16-byte chunk c at c ^ (r & 15)
  const unsigned yrb = __builtin_amdgcn_readfirstlane((unsigned)(((m0 + 32 * wave) * p.N + n0) * 2));
  const unsigned yh = __builtin_amdgcn_readfirstlane((unsigned)(128 * p.N * 2));
  const unsigned ys2 = __builtin_amdgcn_readfirstlane((unsigned)(2 * p.N * 2));
  const unsigned m0yb = __builtin_amdgcn_readfirstlane(lds0 + wave * 16384);
  unsigned yo[8];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    yo[k] = (unsigned)((lane >> 5) * p.N * 2) + 16u * (unsigned)((lane & 31) ^ ((2 * k + (lane >> 5)) & 15));
  unsigned koff, kc, m0s, sdma, srd, m0y, yso, ybs;
#define MTQ_W4_ASM(BODY)                                                                              \
  asm volatile(BODY                                                                                   \
               : [koff] "=&s"(koff), [kc] "=&s"(kc), [m0s] "=&s"(m0s), [sdma] "=&s"(sdma), [srd] "=&s"(srd), \
                 [cnt] "+s"(cnt), [m0y] "=&s"(m0y), [yso] "=&s"(yso), [ybs] "=&s"(ybs)                 \
               : [xr] "s"(xr), [wr] "s"(wr), [m0b] "s"(m0b), [klast] "s"(klast),                         \
                 [xo0] "v"(xo[0]), [xo1] "v"(xo[1]), [xo2] "v"(xo[2]), [xo3] "v"(xo[3]),                  \
                 [xo4] "v"(xo[4]), [xo5] "v"(xo[5]), [xo6] "v"(xo[6]), [xo7] "v"(xo[7]),                  \
                 [wo0] "v"(wo[0]), [wo1] "v"(wo[1]), [wo2] "v"(wo[2]), [wo3] "v"(wo[3]),                  \
                 [wo4] "v"(wo[4]), [wo5] "v"(wo[5]), [wo6] "v"(wo[6]), [wo7] "v"(wo[7]),                  \
                 [xb0] "v"(xb0), [xb1] "v"(xb1), [wb0] "v"(wb0), [wb1] "v"(wb1),                           \
                 [yr] "s"(yr), [yrb] "s"(yrb), [yh] "s"(yh), [ys2] "s"(ys2), [m0yb] "s"(m0yb),             \
                 [yo0] "v"(yo[0]), [yo1] "v"(yo[1]), [yo2] "v"(yo[2]), [yo3] "v"(yo[3]),                  \
                 [yo4] "v"(yo[4]), [yo5] "v"(yo[5]), [yo6] "v"(yo[6]), [yo7] "v"(yo[7])                   \
               : MTQ_W4_CLOBBERS)
  if constexpr (sizeof(T) == 2 && __is_same(T, __bf16))
    MTQ_W4_ASM(MTQ_W4_BODY_BF16);
  else
    MTQ_W4_ASM(MTQ_W4_BODY_F16);
#undef MTQ_W4_ASM

  // ---- epilogue.  A lane's accumulators of tile (i, j) are out[m][n .. n+3], m = 16 i + fr, n =
  // 16 j + 4 fq of the wave's block (a[32 i + 4 j ..]); bias, output and difference rounded to T,
  // fp32 square-sum in a fixed order; the reference values from the LDS copy.
  const T *Bi = reinterpret_cast<const T *>(p.bias);
  const unsigned yslot = (unsigned)(((K / 64 + wm) & 1) * 65536);
  float bj[8][4];
  bool cok[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t c = n0 + wn * 128 + 16 * j + 4 * fq;
    cok[j] = c < p.N;  // N % 8 == 0: the 4 columns are all in or all out
#pragma unroll
    for (int e = 0; e < 4; ++e) bj[j][e] = HAS_BIAS ? Elem<T>::ld(Bi[cok[j] ? c + e : e]) : 0.f;
  }
  float sum = 0.f;
  float o[32];
  // a whole tile inside the matrix (uniform): no masks; for bf16 the output / difference pairs
  // rounded by one v_cvt_pk_bf16_f32 each and squared-summed by v_dot2c_f32_bf16 (exact
  // products; 4 per element instead of 9 VALU instructions -- the epilogue was ~8 % of a
  // K = 4096 tile, profiles/r06/awq/)
  const bool full = m0 + kBM <= p.M && n0 + kBN <= p.N;
#define MTQ_W4_EPI(I)                                                                                 \
  {                                                                                                   \
    MTQ_W4_STRIP_##I(o);                                                                              \
    const bool rok = m0 + wm * 128 + 16 * (I) + fr < p.M;                                             \
    const int rr = 16 * (I) + fr;                                                                     \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                   \
      const int cl = wn * 128 + 16 * j + 4 * fq;                                                      \
      T yv[4];                                                                                        \
      __builtin_memcpy(yv, lds + yslot + rr * 512 + (((cl >> 3) ^ fr) << 4) + (cl & 7) * 2, 8);       \
      const bool ok = rok && cok[j];                                                                  \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                 \
        const float y = Elem<T>::ld(Elem<T>::st(HAS_BIAS ? o[4 * j + e] + bj[j][e] : o[4 * j + e]));  \
        const float d = Elem<T>::ld(Elem<T>::st(y - Elem<T>::ld(yv[e])));                             \
        sum = ok ? __builtin_fmaf(d, d, sum) : sum;                                                   \
      }                                                                                               \
    }                                                                                                 \
  }
#define MTQ_W4_EPI_BF16(I)                                                                            \
  {                                                                                                   \
    MTQ_W4_STRIP_##I(o);                                                                              \
    const int rr = 16 * (I) + fr;                                                                     \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                   \
      const int cl = wn * 128 + 16 * j + 4 * fq;                                                      \
      uint32_t yr[2];                                                                                 \
      __builtin_memcpy(yr, lds + yslot + rr * 512 + (((cl >> 3) ^ fr) << 4) + (cl & 7) * 2, 8);       \
      _Pragma("unroll") for (int h = 0; h < 2; ++h) {                                                 \
        w4f2 y = {o[4 * j + 2 * h], o[4 * j + 2 * h + 1]};                                            \
        if (HAS_BIAS) y += w4f2{bj[j][2 * h], bj[j][2 * h + 1]};                                     \
        const uint32_t yu = __builtin_bit_cast(uint32_t, __builtin_convertvector(y, w4b2));           \
        const w4f2 yf = {__builtin_bit_cast(float, yu << 16), __builtin_bit_cast(float, yu & 0xffff0000u)}; \
        const w4f2 rf = {__builtin_bit_cast(float, yr[h] << 16),                                      \
                         __builtin_bit_cast(float, yr[h] & 0xffff0000u)};                             \
        const w4b2 d = __builtin_convertvector(yf - rf, w4b2);                                        \
        s4[(2 * j + h) & 3] = __builtin_amdgcn_fdot2_f32_bf16(d, d, s4[(2 * j + h) & 3], false);      \
      }                                                                                               \
    }                                                                                                 \
  }
  if constexpr (__is_same(T, __bf16)) {
    if (full) {
      float s4[4] = {0.f, 0.f, 0.f, 0.f};
      MTQ_W4_EPI_BF16(0) MTQ_W4_EPI_BF16(1) MTQ_W4_EPI_BF16(2) MTQ_W4_EPI_BF16(3)
      MTQ_W4_EPI_BF16(4) MTQ_W4_EPI_BF16(5) MTQ_W4_EPI_BF16(6) MTQ_W4_EPI_BF16(7)
      sum = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    } else {
      MTQ_W4_EPI(0) MTQ_W4_EPI(1) MTQ_W4_EPI(2) MTQ_W4_EPI(3) MTQ_W4_EPI(4) MTQ_W4_EPI(5) MTQ_W4_EPI(6) MTQ_W4_EPI(7)
    }
  } else {
    MTQ_W4_EPI(0) MTQ_W4_EPI(1) MTQ_W4_EPI(2) MTQ_W4_EPI(3) MTQ_W4_EPI(4) MTQ_W4_EPI(5) MTQ_W4_EPI(6) MTQ_W4_EPI(7)
  }
#undef MTQ_W4_EPI
#undef MTQ_W4_EPI_BF16
  __syncthreads();
#pragma unroll
  for (int o2 = 32; o2 >= 1; o2 >>= 1) sum += __shfl_xor(sum, o2);
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) p.partial[(int64_t)g * p.tiles_m * p.tiles_n + tile] = red[0] + red[1] + red[2] + red[3];
}

// xs[g, m, k] = T(x[m, k] * sinv[g, k]) for all g: one read of x, G writes (the reference's
// `inputs * pre_quant_scale` per alpha, tensor_quantizer.py:1143-1144).  GT > 0: the alpha count
// as a compile-time constant, so every sinv load of the thread is issued before the first product
// (the runtime-G loop waited for each L2 round trip in turn: 197 us = 4.1 TB/s at [8192, 4096] x
// 11 in the r04 C3 profile); the G output planes stream out with non-temporal stores (written
// once, read once by the next GEMM, 11x larger than the Infinity Cache).
template <typename T, int GT>
__global__ __launch_bounds__(256) void awq_prescale_kernel(const T *__restrict__ x, const T *__restrict__ sinv,
                                                           T *__restrict__ xs, int64_t chunks, int64_t kchunks,
                                                           int G) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= chunks) return;
  const int64_t kc = c % kchunks;
  Vec<T> v = ldg_vec_nt(x + c * 8);
  if constexpr (GT > 0) {
    Vec<T> s[GT];
#pragma unroll
    for (int g = 0; g < GT; ++g) s[g] = ldg_vec(sinv + ((int64_t)g * kchunks + kc) * 8);
    float xf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xf[j] = Elem<T>::ld(v.e[j]);
#pragma unroll
    for (int g = 0; g < GT; ++g) {
      Vec<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.e[j] = Elem<T>::st(xf[j] * Elem<T>::ld(s[g].e[j]));
      stg_vec_nt(xs + ((int64_t)g * chunks + c) * 8, o);
    }
  } else {
    float xf[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xf[j] = Elem<T>::ld(v.e[j]);
    for (int g = 0; g < G; ++g) {
      Vec<T> sv = ldg_vec(sinv + ((int64_t)g * kchunks + kc) * 8);
      Vec<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.e[j] = Elem<T>::st(xf[j] * Elem<T>::ld(sv.e[j]));
      stg_vec_nt(xs + ((int64_t)g * chunks + c) * 8, o);
    }
  }
}

template <typename T>
void launch_prescale(const void *x, const void *sinv, void *xs, int64_t M, int64_t K, int G, hipStream_t stream) {
  const int64_t chunks = M * K / 8;
  const unsigned gb = (unsigned)((chunks + 255) / 256);
  const T *xt = reinterpret_cast<const T *>(x);
  const T *st = reinterpret_cast<const T *>(sinv);
  T *ot = reinterpret_cast<T *>(xs);
  count_dispatch(kDispAwqPrescale);
  if (G == 11)  // alpha_step 0.1, the awq_lite default
    awq_prescale_kernel<T, 11><<<gb, 256, 0, stream>>>(xt, st, ot, chunks, K / 8, G);
  else
    awq_prescale_kernel<T, 0><<<gb, 256, 0, stream>>>(xt, st, ot, chunks, K / 8, G);
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

// loss[g] += (sum over the tiles of alpha g, in double, fixed order) / (M * N): one block per
// alpha (the r03 single block walked the alphas one after another: 28 us per call in the r04 C3
// profile); per alpha the same summation order as before (per thread strided, then the tree).
__global__ __launch_bounds__(256) void awq_search_finish_kernel(const float *partial, int tiles, int G,
                                                                 double inv_count, float *loss) {
  __shared__ double red[256];
  const int g = blockIdx.x;
  if (g >= G) return;
  double s = 0.0;
  for (int i = threadIdx.x; i < tiles; i += 256) s += (double)partial[(int64_t)g * tiles + i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o >= 1; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[g] += (float)(red[0] * inv_count);
}

bool al16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

int64_t partial_floats(int64_t M, int64_t N, int G) {
  return ((((M + kBM - 1) / kBM) * ((N + kBN - 1) / kBN) * (int64_t)G) + 3) / 4 * 4;  // 16-B aligned
}

}  // namespace

extern "C" int64_t mtq_awq_search_gemm_workspace_floats(int64_t M, int64_t N, int64_t K, int G) {
  if (M < 1 || N < 1 || K < 1 || G < 1) return 0;
  return partial_floats(M, N, G) + (G * M * K + 1) / 2;  // + xs [G, M, K] in 16-bit elements
}

extern "C" int mtq_awq_search_gemm_kernel(const void *x, const void *sinv, const void *wq, const void *bias,
                                          const void *yref, int64_t M, int64_t N, int64_t K, int dtype,
                                          int G, float *loss, float *workspace, int64_t workspace_floats,
                                          int kernel, hipStream_t stream) {
  if (kernel < MTQ_AWQ_SEARCH_AUTO || kernel > MTQ_AWQ_SEARCH_W4) return MTQ_ERR_INVALID_ARG;
  if (M < 1 || N < 1 || K < kBK || K % kBK != 0 || G < 1 || G > 64) return MTQ_ERR_INVALID_ARG;
  if (!x || !sinv || !wq || !yref || !loss || !workspace) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(sinv) || !al16(wq) || !al16(workspace)) return MTQ_ERR_INVALID_ARG;
  if (M * K >= ((int64_t)1 << 31) || N * K >= ((int64_t)1 << 31) || N % 8 != 0 || !al16(yref))
    return MTQ_ERR_INVALID_ARG;
  const int64_t tiles_m = (M + kBM - 1) / kBM, tiles_n = (N + kBN - 1) / kBN;
  const int64_t tiles = tiles_m * tiles_n;
  if (workspace_floats < mtq_awq_search_gemm_workspace_floats(M, N, K, G) ||
      tiles * G > (int64_t)INT32_MAX / 4)
    return MTQ_ERR_INVALID_ARG;
  // x * (1/s_g) for every alpha into the workspace (the reference's bf16 multiply, one read of x)
  void *xs = workspace + partial_floats(M, N, G);
  if (dtype == MTQ_BF16)
    launch_prescale<__bf16>(x, sinv, xs, M, K, G, stream);
  else
    launch_prescale<_Float16>(x, sinv, xs, M, K, G, stream);
  int st0 = host_check_launch();
  if (st0 != MTQ_OK) return st0;
  AwqGemmArgs a{xs, sinv, wq, bias, yref, workspace, M, N, K, (int)tiles_m, (int)tiles_n, G};
  // 32 slots per 8 x 4 tile unit, units padded to a multiple of the 8 XCDs (see the kernel)
  const int64_t units = (int64_t)G * ((tiles_m + 7) / 8) * ((tiles_n + 3) / 4);
  const dim3 grid((unsigned)((units + 7) / 8 * 8 * 32));
  const bool w4_ok = K >= 128 && K % 128 == 0 && M * N * 2 < ((int64_t)1 << 32);
  if (kernel == MTQ_AWQ_SEARCH_W4 && !w4_ok) return MTQ_ERR_INVALID_ARG;
  if (kernel == MTQ_AWQ_SEARCH_W4 || (kernel == MTQ_AWQ_SEARCH_AUTO && w4_ok)) {
    count_dispatch(kDispAwqSearchW4);
    if (dtype == MTQ_BF16) {
      if (bias)
        awq_search_w4_kernel<__bf16, true><<<grid, 256, 0, stream>>>(a);
      else
        awq_search_w4_kernel<__bf16, false><<<grid, 256, 0, stream>>>(a);
    } else {
      if (bias)
        awq_search_w4_kernel<_Float16, true><<<grid, 256, 0, stream>>>(a);
      else
        awq_search_w4_kernel<_Float16, false><<<grid, 256, 0, stream>>>(a);
    }
  } else {
  count_dispatch(kDispAwqSearchPp);
  if (dtype == MTQ_BF16) {
    if (bias)
      awq_search_pp_kernel<__bf16, true><<<grid, kThreads, 0, stream>>>(a);
    else
      awq_search_pp_kernel<__bf16, false><<<grid, kThreads, 0, stream>>>(a);
  } else {
    if (bias)
      awq_search_pp_kernel<_Float16, true><<<grid, kThreads, 0, stream>>>(a);
    else
      awq_search_pp_kernel<_Float16, false><<<grid, kThreads, 0, stream>>>(a);
  }
  }
  int st = host_check_launch();
  if (st != MTQ_OK) return st;
  awq_search_finish_kernel<<<(unsigned)G, 256, 0, stream>>>(workspace, (int)tiles, G, 1.0 / ((double)M * (double)N),
                                                  loss);
  return host_check_launch();
}

extern "C" int mtq_awq_search_gemm(const void *x, const void *sinv, const void *wq, const void *bias,
                                   const void *yref, int64_t M, int64_t N, int64_t K, int dtype,
                                   int G, float *loss, float *workspace, int64_t workspace_floats,
                                   hipStream_t stream) {
  return mtq_awq_search_gemm_kernel(x, sinv, wq, bias, yref, M, N, K, dtype, G, loss, workspace, workspace_floats,
                                    MTQ_AWQ_SEARCH_AUTO, stream);
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
  count_dispatch(kDispAwqMseMulti);
  if (dtype == MTQ_BF16)
    awq_mse_multi_kernel<__bf16><<<(unsigned)grid, 256, 0, stream>>>((const __bf16 *)out, (const __bf16 *)ref,
                                                                    n / 8, G, workspace);
  else
    awq_mse_multi_kernel<_Float16><<<(unsigned)grid, 256, 0, stream>>>((const _Float16 *)out,
                                                                      (const _Float16 *)ref, n / 8, G, workspace);
  int st = host_check_launch();
  if (st != MTQ_OK) return st;
  awq_search_finish_kernel<<<(unsigned)G, 256, 0, stream>>>(workspace, (int)grid, G, 1.0 / (double)n, loss);
  return host_check_launch();
}

extern "C" int mtq_awq_prescale(const void *x, const void *sinv, void *xs, int64_t M, int64_t K, int dtype, int G,
                                hipStream_t stream) {
  if (M < 1 || K < 8 || K % 8 != 0 || G < 1 || !x || !sinv || !xs) return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16) return MTQ_ERR_DTYPE;
  if (!al16(x) || !al16(sinv) || !al16(xs)) return MTQ_ERR_INVALID_ARG;
  if (dtype == MTQ_BF16)
    launch_prescale<__bf16>(x, sinv, xs, M, K, G, stream);
  else
    launch_prescale<_Float16>(x, sinv, xs, M, K, G, stream);
  return host_check_launch();
}
