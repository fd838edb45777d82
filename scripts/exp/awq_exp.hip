// awq_exp.hip -- measurement-only variants of the AWQ search kernel (csrc/mtq_awq_gemm.hip
// awq_search_pp_kernel, schedule 5), built by scripts/exp/build_exp.sh and timed by
// scripts/exp/bench_awq_exp.py against the product kernel.  Not part of the product library.
//
// Knobs: PROBE 0 = as the product; 1 = no global loads in the K loop; 3 = every K tile loads the
// FIRST K tile (same instructions, always L2 hits: isolates the L2-miss latency from the issue
// cost).  GM = row tiles per XCD tile group (product 8).  BUF = 1: buffer_load ... lds with the K
// advance in the scalar offset (no 64-bit address per DMA) instead of global_load_lds.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"

using namespace mtq;

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 512;
constexpr int kHalf = 16384, kBuf = 4 * kHalf, kLds = 2 * kBuf;

struct Args {
  const void *x, *wq, *yref;
  float *partial;
  int64_t M, N, K;
  int tiles_m, tiles_n, G;
};

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// MAP 1: units of 8 m-tiles x 4 n-tiles (32 slots, one per CU of an XCD); unit u = ((g * NN4) +
// n4) * MGN + mg runs on XCD u % 8 in local round u / 8, so at any time the 8 XCDs work on the
// SAME alpha and n-range, different m-groups: every W panel is fetched from HBM once and shared
// through the Infinity Cache, the alpha's activations stay resident there.  Slots past the
// matrix edge exit at once.
// YPF 1: the reference (yref) tile of the epilogue rides in the K loop's past-the-end half-loads
// (tile nt-2 phases 2-3 and tile nt-1 phases 0-3 re-load clamped K tiles nobody reads): each such
// half writes the same 16 KiB of LDS the yref rounds 2 b + {0, 1} (b = its 8 KiB index) occupy in
// the epilogue layout, at the same time as the re-load would have -- same WAR margins, same DMA
// count for the counted waits -- so 12 of the tile's 16 rounds are in flight before the loop ends
// and only the last buffer's A1 / B1 slots (4 rounds) load after it.  YPF 2: no yref load at all
// (probe: the epilogue's load cost; loss wrong).
template <int PROBE, int GM, int BUF, int MAP = 0, int YPF = 0>
__global__ __launch_bounds__(kThreads) void pp_exp_kernel(Args p) {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wn = wave & 3;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int tiles = p.tiles_m * p.tiles_n;
  int g, tile, tm, tn;
  if constexpr (MAP == 1) {
    const int xcd = orig % 8, li = orig / 8;
    const int slot = li % 32, u = (li / 32) * 8 + xcd;
    const int mgn = (p.tiles_m + 7) / 8, nn4 = (p.tiles_n + 3) / 4;
    const int mg = u % mgn, n4 = (u / mgn) % nn4;
    g = u / (mgn * nn4);
    tm = mg * 8 + slot % 8;
    tn = n4 * 4 + slot / 8;
    if (g >= p.G || tm >= p.tiles_m || tn >= p.tiles_n) return;  // whole workgroup: no barrier reached
    tile = tm * p.tiles_n + tn;
  } else {
    const int q8 = nwg / 8, rr8 = nwg % 8, xcd = orig % 8;
    const int wgid = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + orig / 8;
    g = wgid / tiles;
    tile = wgid - g * tiles;
    const int gm = tile / (GM * p.tiles_n);
    const int first_m = gm * GM;
    const int gsz = p.tiles_m - first_m < GM ? p.tiles_m - first_m : GM;
    const int tin = tile - gm * GM * p.tiles_n;
    tm = first_m + tin % gsz;
    tn = tin / gsz;
  }
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;
  const __bf16 *X = reinterpret_cast<const __bf16 *>(p.x) + (int64_t)g * p.M * K;
  const __bf16 *W = reinterpret_cast<const __bf16 *>(p.wq) + (int64_t)g * p.N * K;
  unsigned a_off[2][2], b_off[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = u * 64 + wave * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((rr >> 1) & 7);
      int64_t row = m0 + (rr >> 6) * 128 + h * 64 + (rr & 63);
      row = row < p.M ? row : p.M - 1;
      a_off[h][u] = (unsigned)(row * K + chunk * 8);
      int64_t col = n0 + (rr >> 5) * 64 + h * 32 + (rr & 31);
      col = col < p.N ? col : p.N - 1;
      b_off[h][u] = (unsigned)(col * K + chunk * 8);
    }
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(X, (uint32_t)(p.M * K * 2));
  const __amdgpu_buffer_rsrc_t wr = rsrc_of(W, (uint32_t)(p.N * K * 2));
  auto load_half = [&](int q, unsigned char *buf, int64_t k0) {
    const bool isA = (q == 0 || q == 3);
    const int h = (q == 0 || q == 1) ? 0 : 1;
    unsigned char *dst = buf + (isA ? h : 2 + h) * kHalf + wave * 1024;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if constexpr (BUF) {
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? xr : wr, (__attribute__((address_space(3))) void *)(dst + u * 8192),
                                                 16, (isA ? a_off[h][u] : b_off[h][u]) * 2,
                                                 __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2)), 0, 0);
#endif
      } else {
        const __bf16 *src = (isA ? X : W) + k0 + (isA ? a_off[h][u] : b_off[h][u]);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)src,
                                         (__attribute__((address_space(3))) void *)(dst + u * 8192), 16, 0, 0);
      }
    }
  };
  const __bf16 *Y = reinterpret_cast<const __bf16 *>(p.yref);
  auto yref_round = [&](int r) {  // 16 rows x 256 columns of yref -> LDS bytes [r * 8 KiB, +8 KiB)
    const int rr = r * 16 + (tid >> 5);
    int64_t row = m0 + rr;
    row = row < p.M ? row : p.M - 1;
    int64_t col = n0 + (int64_t)(((tid & 31) ^ (rr & 15)) * 8);
    col = col < p.N ? col : p.N - 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(Y + row * p.N + col),
                                     (__attribute__((address_space(3))) void *)(lds + r * 8192 + wave * 1024), 16, 0, 0);
  };
  auto load_yref_half = [&](int q, unsigned char *buf) {
    const bool isA = (q == 0 || q == 3);
    const int h = (q == 0 || q == 1) ? 0 : 1;
    const int r0 = (int)((buf - lds) / 8192) + (isA ? h : 2 + h) * 2;
    yref_round(r0);
    yref_round(r0 + 1);
  };
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
  auto kt = [&](int t) -> int64_t { return PROBE == 3 ? 0 : (int64_t)(t < nt ? t : nt - 1) * kBK; };
  {
    load_half(1, lds, 0);
    load_half(0, lds, 0);
    load_half(2, lds, 0);
    load_half(3, lds, 0);
    load_half(1, lds + kBuf, kt(1));
    load_half(0, lds + kBuf, kt(1));
    wait_vm<8>();
  }
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  v8 af[4][2], b0f[2][2], b1f[2][2];
  for (int t = 0; t < nt; ++t) {
    unsigned char *cur = lds + (t & 1) * kBuf;
    unsigned char *nx1 = lds + ((t + 1) & 1) * kBuf;
    const int64_t k1 = kt(t + 1);
    const int64_t k2 = kt(t + 2);
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
      const int hq = q == 0 ? 2 : q == 1 ? 3 : q == 2 ? 1 : 0;
      unsigned char *hb = q < 2 ? nx1 : cur;
      const int64_t hk = q < 2 ? k1 : k2;
      if (PROBE != 1) {
        if (YPF == 1 && nt >= 2 && (q < 2 ? t + 1 >= nt : t + 2 >= nt))
          load_yref_half(hq, hb);
        else
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
        acc[4 * mq + i][2 * nq + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb, af[i][s2], acc[4 * mq + i][2 * nq + j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  // epilogue as the product kernel (no bias): the loss partial
  float sum = 0.f;
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  u32x2_t yv[8][4];
  wait_vm<0>();
  __syncthreads();
  if (YPF == 1 && nt >= 2) {
    const int b = ((nt - 1) & 1) * 8;  // the last K tile's A1 / B1 slots
    yref_round(b + 2);
    yref_round(b + 3);
    yref_round(b + 6);
    yref_round(b + 7);
  } else if (YPF != 2) {
#pragma unroll
    for (int u = 0; u < 16; ++u) yref_round(u);
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
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __bf16 yr[4];
      __builtin_memcpy(yr, &yv[i][j], 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (float)(__bf16)acc[i][j][e];
        const float d = (float)(__bf16)(y - (float)yr[e]);
        sum = __builtin_fmaf(d, d, sum);
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
    for (int w = 0; w < 8; ++w) s += red[w];
    p.partial[(int64_t)g * tiles + tile] = s;
  }
}

template <int PROBE, int GM, int BUF, int MAP = 0, int YPF = 0>
int go(const Args &a, hipStream_t stream) {
  unsigned grid = (unsigned)(a.tiles_m * a.tiles_n * a.G);
  if (MAP == 1) {
    const int units = a.G * ((a.tiles_m + 7) / 8) * ((a.tiles_n + 3) / 4);
    grid = (unsigned)((units + 7) / 8 * 8 * 32);
  }
  pp_exp_kernel<PROBE, GM, BUF, MAP, YPF><<<grid, kThreads, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// RING: ten 16 KiB half-tile slots (all 160 KiB of LDS) instead of two 64 KiB tile buffers, so
// every half of tile t+2 is issued during tile t (four halves per tile, one per phase, in the
// order B0 A0 B1 A1): 7-8 phases between issue and first read instead of 5-6.  Half (tau, k)
// lives in slot (4 tau + k) % 10; a slot is re-filled 2-3 phases after its last read (the stagger
// margin).  Waits before each phase's first barrier, for the next phase's reads: six halves (12
// DMAs) issued after the one needed may stay in flight (14 in phase 2, whose successor reads
// nothing new).  MAP 1 tile order, buffer DMA.
template <int PROBE>
__global__ __launch_bounds__(kThreads) void pp_ring_kernel(Args p) {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  constexpr int kSlots = 10;
  __shared__ __attribute__((aligned(16))) unsigned char lds[kSlots * kHalf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, wn = wave & 3;
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
    if (g >= p.G || tm >= p.tiles_m || tn >= p.tiles_n) return;
  }
  const int tile = tm * p.tiles_n + tn;
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN;
  const int64_t K = p.K;
  const __bf16 *X = reinterpret_cast<const __bf16 *>(p.x) + (int64_t)g * p.M * K;
  const __bf16 *W = reinterpret_cast<const __bf16 *>(p.wq) + (int64_t)g * p.N * K;
  unsigned a_off[2][2], b_off[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int rr = u * 64 + wave * 8 + (lane >> 3);
      const int chunk = (lane & 7) ^ ((rr >> 1) & 7);
      int64_t row = m0 + (rr >> 6) * 128 + h * 64 + (rr & 63);
      row = row < p.M ? row : p.M - 1;
      a_off[h][u] = (unsigned)(row * K + chunk * 8) * 2u;
      int64_t col = n0 + (rr >> 5) * 64 + h * 32 + (rr & 31);
      col = col < p.N ? col : p.N - 1;
      b_off[h][u] = (unsigned)(col * K + chunk * 8) * 2u;
    }
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(X, (uint32_t)(p.M * K * 2));
  const __amdgpu_buffer_rsrc_t wr = rsrc_of(W, (uint32_t)(p.N * K * 2));
  const int nt = (int)(K / kBK);
  auto kt = [&](int t) -> int64_t { return PROBE == 3 ? 0 : (int64_t)(t < nt ? t : nt - 1) * kBK; };
  // half k of tile tau (k: 0 B0, 1 A0, 2 B1, 3 A1) into its ring slot
  auto issue = [&](int tau, int k) {
    const bool isA = (k & 1) != 0;
    const int h = k >> 1;
    unsigned char *dst = lds + ((4 * tau + k) % kSlots) * kHalf + wave * 1024;
    const uint32_t soff = __builtin_amdgcn_readfirstlane((uint32_t)(kt(tau) * 2));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(isA ? xr : wr, (__attribute__((address_space(3))) void *)(dst + u * 8192),
                                               16, isA ? a_off[h][u] : b_off[h][u], soff, 0, 0);
#endif
    }
  };
  const int sw = (lane >> 1) & 7, fr = lane & 15, fq = lane >> 4;
  auto read_a = [&](const unsigned char *half, int i, int s) -> v8 {  // i: 0..3 within the half
    const int L = grp * 64 + i * 16 + fr;
    return *reinterpret_cast<const v8 *>(half + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };
  auto read_b = [&](const unsigned char *half, int j, int s) -> v8 {  // j: 0..1 within the half
    const int L = wn * 32 + j * 16 + fr;
    return *reinterpret_cast<const v8 *>(half + L * 128 + (((4 * s + fq) ^ sw) << 4));
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tau = 0; tau < 2; ++tau)
#pragma unroll
    for (int k = 0; k < 4; ++k) issue(tau, k);
  wait_vm<12>();
  __builtin_amdgcn_s_barrier();
  if (grp == 1) __builtin_amdgcn_s_barrier();
  v8 af[4][2], b0f[2][2], b1f[2][2];
  for (int t = 0; t < nt; ++t) {
    const int s0 = (4 * t) % kSlots;
    const unsigned char *hB0 = lds + s0 * kHalf;
    const unsigned char *hA0 = lds + ((s0 + 1) % kSlots) * kHalf;
    const unsigned char *hB1 = lds + ((s0 + 2) % kSlots) * kHalf;
    const unsigned char *hA1 = lds + ((s0 + 3) % kSlots) * kHalf;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int mq = (q == 0 || q == 1) ? 0 : 1;
      const int nq = (q == 1 || q == 2) ? 1 : 0;
      if (q == 0 || q == 2) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i][s2] = read_a(q == 0 ? hA0 : hA1, i, s2);
      }
      if (q == 0) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 2; ++j) b0f[j][s2] = read_b(hB0, j, s2);
      }
      if (q == 1) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
          for (int j = 0; j < 2; ++j) b1f[j][s2] = read_b(hB1, j, s2);
      }
      if (PROBE != 1) {
        issue(t + 2, q);
        if (q == 2)
          wait_vm<14>();
        else
          wait_vm<12>();
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const int s2 = kk >> 3, j = (kk >> 2) & 1, i = kk & 3;
        const v8 bb = nq ? b1f[j][s2] : b0f[j][s2];
        acc[4 * mq + i][2 * nq + j] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb, af[i][s2], acc[4 * mq + i][2 * nq + j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_s_barrier();
    }
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();
  float sum = 0.f;
  const __bf16 *Y = reinterpret_cast<const __bf16 *>(p.yref);
  typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
  u32x2_t yv[8][4];
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
                                       (__attribute__((address_space(3))) void *)(lds + u * 8192 + wave * 1024), 16, 0, 0);
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
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      __bf16 yr[4];
      __builtin_memcpy(yr, &yv[i][j], 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (float)(__bf16)acc[i][j][e];
        const float d = (float)(__bf16)(y - (float)yr[e]);
        sum = __builtin_fmaf(d, d, sum);
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
    for (int w = 0; w < 8; ++w) s += red[w];
    p.partial[(int64_t)g * tiles + tile] = s;
  }
}

template <int PROBE>
int go_ring(const Args &a, hipStream_t stream) {
  const int units = a.G * ((a.tiles_m + 7) / 8) * ((a.tiles_n + 3) / 4);
  pp_ring_kernel<PROBE><<<(unsigned)((units + 7) / 8 * 8 * 32), kThreads, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}  // namespace

// xs [G, M, K] pre-scaled activations, wq [G, N, K], yref [M, N]; partial [G * tiles]
extern "C" int awq_exp(int var, const void *xs, const void *wq, const void *yref, float *partial, int64_t M, int64_t N,
                       int64_t K, int G, hipStream_t stream) {
  if (M % 256 || N % 256 || K % 64) return 2;
  Args a{xs, wq, yref, partial, M, N, K, (int)(M / 256), (int)(N / 256), G};
  switch (var) {
  case 0: return go<0, 8, 0>(a, stream);
  case 1: return go<1, 8, 0>(a, stream);
  case 3: return go<3, 8, 0>(a, stream);
  case 10: return go<0, 8, 1>(a, stream);
  case 13: return go<3, 8, 1>(a, stream);
  case 20: return go<0, 4, 0>(a, stream);
  case 21: return go<0, 16, 0>(a, stream);
  case 22: return go<0, 2, 0>(a, stream);
  case 30: return go<0, 8, 0, 1>(a, stream);
  case 31: return go<0, 8, 1, 1>(a, stream);
  case 33: return go<3, 8, 0, 1>(a, stream);
  case 34: return go<0, 8, 1, 1, 1>(a, stream);
  case 35: return go<0, 8, 1, 1, 2>(a, stream);
  case 50: return go_ring<0>(a, stream);
  case 53: return go_ring<3>(a, stream);
  default: return 3;
  }
}
