// awq_w4r.hip -- measurement-only AWQ search kernel in the library GEMM's shape: 4 waves per
// 256 x 256 tile (one 128 x 128 block per wave = one wave per SIMD), 256 accumulators per lane,
// K tile 64, both operands REGISTER-staged (global_load_dwordx4 -> ds_write_b128, no LDS-DMA:
// with one wave per SIMD the DMA issue cost stalled the MFMA issue, r03 schedule 6), two LDS
// stages, the next tile's writes and the tile after's loads issued inside the current tile's
// MFMA stream.  Loss epilogue as the product kernel.  Built by scripts/exp/build_exp.sh, timed by
// scripts/exp/bench_awq_w4r.py against the product kernel.  Not part of the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 v8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr int kBM = 256, kBN = 256, kBK = 64, kThreads = 256;
constexpr int kTile = 256 * 128;   // one operand's K tile: 256 rows x 64 k x 2 B
constexpr int kStage = 2 * kTile;  // X then W
constexpr int kLds = 2 * kStage;   // two stages: 128 KiB

struct Args {
  const __bf16 *x, *wq, *yref;
  float *partial;
  int64_t M, N, K;
  int tiles_m, tiles_n, G;
};

__device__ __forceinline__ unsigned swz(int row, int chunk) {  // byte offset of (row, 16-B chunk)
  return (unsigned)(row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4));
}

// SCHED: 0 = compiler's order; 1 = sched_group_barrier interleave of the next tile's LDS writes,
// the tile after's global loads and the fragment reads into the MFMA stream
template <int SCHED>
__global__ __launch_bounds__(kThreads, 1) void w4r_kernel(Args p) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[kLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int orig = blockIdx.x, tiles = p.tiles_m * p.tiles_n;
  int g, tm, tn;
  {  // the product's unit order: 8 row tiles x 4 column tiles per XCD round, XCDs on one alpha
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
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN, K = p.K;
  const __bf16 *X = p.x + (int64_t)g * p.M * K;
  const __bf16 *W = p.wq + (int64_t)g * p.N * K;
  // staging: thread t moves chunk q = t + 256 u (u < 8) of each operand tile: row q >> 3, chunk q & 7
  // (M, N multiples of 256 in this experiment: no edge clamps; 32-bit element offsets, the u
  // stride 32 K wave-uniform)
  const int srow = tid >> 3, schunk = tid & 7;
  const uint32_t xo = (uint32_t)((m0 + srow) * K + schunk * 8), wo = (uint32_t)((n0 + srow) * K + schunk * 8);
  const uint32_t ustride = (uint32_t)(32 * K);
  const unsigned so = swz(srow, schunk);  // + u * 32 rows * 128 B (the XOR term is u-invariant)
  u32x4 sx[8], sw[8];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sx[u] = *reinterpret_cast<const u32x4 *>(X + xo + u * ustride + k0);
      sw[u] = *reinterpret_cast<const u32x4 *>(W + wo + u * ustride + k0);
    }
  };
  auto lwrite = [&](unsigned char *st) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      *reinterpret_cast<u32x4 *>(st + so + u * 4096) = sx[u];
      *reinterpret_cast<u32x4 *>(st + kTile + so + u * 4096) = sw[u];
    }
  };
  const int fr = lane & 15, fq = lane >> 4;
  auto rd = [&](const unsigned char *base, int row0, int s) -> v8 {
    const int row = row0 + fr;
    return *reinterpret_cast<const v8 *>(base + swz(row, 4 * s + fq));
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (int)(K / kBK);
  gload(0);
  lwrite(lds);
  gload((int64_t)(nt > 1 ? 1 : 0) * kBK);
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const unsigned char *cur = lds + (t & 1) * kStage;
    unsigned char *nxt = lds + ((t + 1) & 1) * kStage;
    const int64_t k2 = (int64_t)(t + 2 < nt ? t + 2 : nt - 1) * kBK;
    // k-step 0's fragments, then tile t+1 into the other stage, tile t+2's loads and k-step 1's
    // fragments issued beside k-step 0's MFMAs, then k-step 1's MFMAs
    v8 x0[8], w0[8], x1[8], w1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x0[i] = rd(cur, wm * 128 + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) w0[j] = rd(cur + kTile, wn * 128 + 16 * j, 0);
    lwrite(nxt);
    gload(k2);
#pragma unroll
    for (int i = 0; i < 8; ++i) x1[i] = rd(cur, wm * 128 + 16 * i, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) w1[j] = rd(cur + kTile, wn * 128 + 16 * j, 1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[i], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[i][j], 0, 0, 0);
    if constexpr (SCHED == 1) {
      __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // k-step 0 fragment reads
      for (int r = 0; r < 16; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMAs of k-step 0
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);  // 1 LDS write (tile t+1)
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // 1 global load (tile t+2)
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 fragment read (k-step 1)
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);  // k-step 1
    }
    __syncthreads();
  }
  // epilogue: lane holds out[m0 + wm*128 + 16 i + (lane & 15)][n0 + wn*128 + 16 j + 4 (lane >> 4) + e]
  float sum = 0.f;
  const __bf16 *Y = p.yref;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t m = m0 + wm * 128 + 16 * i + fr;
    const bool mok = m < p.M;
    const int64_t mm = mok ? m : p.M - 1;
    u32x2 yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t n = n0 + wn * 128 + 16 * j + 4 * fq;
      n = n < p.N ? n : p.N - 4;
      yv[j] = *reinterpret_cast<const u32x2 *>(Y + mm * p.N + n);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 yr[4];
      __builtin_memcpy(yr, &yv[j], 8);
      const bool ok = mok && (n0 + wn * 128 + 16 * j + 4 * fq < p.N);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (float)(__bf16)acc[i][j][e];
        const float d = (float)(__bf16)(y - (float)yr[e]);
        sum = ok ? __builtin_fmaf(d, d, sum) : sum;
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  __syncthreads();
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) p.partial[(int64_t)g * tiles + tile] = red[0] + red[1] + red[2] + red[3];
}

// v2: X tile by LDS-DMA into three stages (issued two tiles ahead, no registers), W tile register
// staged into two stages (one tile ahead); raw barriers with counted waits: per tile the W loads
// of tile t+2 go out before the X DMA of tile t+2, so the W registers' wait leaves the 8 DMA in
// flight and the end-of-tile vmcnt(16) retires only tile t+1's X.  LDS: 3 x 32 + 2 x 32 = 160 KiB.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

__global__ __launch_bounds__(kThreads, 1) void w4r2_kernel(Args p) {
  constexpr int kX = 0, kW = 3 * kTile;  // X stages at 0, 32K, 64K; W stages at 96K, 128K
  __shared__ __attribute__((aligned(16))) unsigned char lds[5 * kTile];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int orig = blockIdx.x, tiles = p.tiles_m * p.tiles_n;
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
  const int64_t m0 = (int64_t)tm * kBM, n0 = (int64_t)tn * kBN, K = p.K;
  const __bf16 *X = p.x + (int64_t)g * p.M * K;
  const __bf16 *W = p.wq + (int64_t)g * p.N * K;
  // X by DMA: wave instruction u (< 8) fills LDS rows (wave * 8 + u) * 8 + (lane >> 3), slot lane & 7
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(X, (uint32_t)(p.M * K * 2));
  uint32_t xv[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int r = (wave * 8 + u) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ ((r >> 1) & 7);
    xv[u] = (uint32_t)(((m0 + r) * K + chunk * 8) * 2);
  }
  auto xdma = [&](int stage, int64_t k0) {
    unsigned char *dst = lds + kX + stage * kTile + wave * 8192;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2));
#pragma unroll
    for (int u = 0; u < 8; ++u) {
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void *)(dst + u * 1024), 16, xv[u], so, 0, 0);
#endif
    }
  };
  // W by registers, as the v1 kernel
  const int srow = tid >> 3, schunk = tid & 7;
  const uint32_t wo = (uint32_t)((n0 + srow) * K + schunk * 8);
  const uint32_t ustride = (uint32_t)(32 * K);
  const unsigned sof = swz(srow, schunk);
  u32x4 sw[8];
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) sw[u] = *reinterpret_cast<const u32x4 *>(W + wo + u * ustride + k0);
  };
  auto lwrite = [&](int stage) {
#pragma unroll
    for (int u = 0; u < 8; ++u) *reinterpret_cast<u32x4 *>(lds + kW + stage * kTile + sof + u * 4096) = sw[u];
  };
  const int fr = lane & 15, fq = lane >> 4;
  auto rd = [&](const unsigned char *base, int row0, int s) -> v8 {
    const int row = row0 + fr;
    return *reinterpret_cast<const v8 *>(base + swz(row, 4 * s + fq));
  };
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nt = (int)(K / kBK);
  auto kt = [&](int t) -> int64_t { return (int64_t)(t < nt ? t : nt - 1) * kBK; };
  gload(kt(0));
  xdma(0, kt(0));
  xdma(1, kt(1));
  lwrite(0);  // waits for W(0) (and the X DMAs issued before it)
  gload(kt(1));
  wait_vm<8>();  // X(0), X(1) landed; W(1) may be in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int t = 0; t < nt; ++t) {
    const unsigned char *xc = lds + kX + (t % 3) * kTile;
    const unsigned char *wc = lds + kW + (t & 1) * kTile;
    v8 x0[8], w0[8], x1[8], w1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x0[i] = rd(xc, wm * 128 + 16 * i, 0);
#pragma unroll
    for (int j = 0; j < 8; ++j) w0[j] = rd(wc, wn * 128 + 16 * j, 0);
    lwrite((t + 1) & 1);  // W(t+1): its loads are followed by X(t+1)'s 8 DMA
    gload(kt(t + 2));
    xdma((t + 2) % 3, kt(t + 2));
#pragma unroll
    for (int i = 0; i < 8; ++i) x1[i] = rd(xc, wm * 128 + 16 * i, 1);
#pragma unroll
    for (int j = 0; j < 8; ++j) w1[j] = rd(wc, wn * 128 + 16 * j, 1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0[j], x0[i], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[j], x1[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);
    for (int r = 0; r < 8; ++r) {
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    wait_vm<16>();  // X(t+1) landed (W(t+2) and X(t+2) may stay in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  wait_vm<0>();
  __syncthreads();
  float sum = 0.f;
  const __bf16 *Y = p.yref;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t m = m0 + wm * 128 + 16 * i + fr;
    u32x2 yv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) yv[j] = *reinterpret_cast<const u32x2 *>(Y + m * p.N + n0 + wn * 128 + 16 * j + 4 * fq);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 yr[4];
      __builtin_memcpy(yr, &yv[j], 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y = (float)(__bf16)acc[i][j][e];
        const float d = (float)(__bf16)(y - (float)yr[e]);
        sum = __builtin_fmaf(d, d, sum);
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) p.partial[(int64_t)g * tiles + tile] = red[0] + red[1] + red[2] + red[3];
}
}  // namespace

// xs [G, M, K] pre-scaled activations, wq [G, N, K], yref [M, N]; partial [G * tiles]
extern "C" int awq_w4r(int var, const void *xs, const void *wq, const void *yref, float *partial, int64_t M, int64_t N,
                       int64_t K, int G, hipStream_t stream) {
  if (M % 256 || N % 256 || K % 64) return 2;
  Args a{(const __bf16 *)xs, (const __bf16 *)wq, (const __bf16 *)yref, partial, M, N, K, (int)(M / 256), (int)(N / 256), G};
  const int units = G * ((a.tiles_m + 7) / 8) * ((a.tiles_n + 3) / 4);
  const unsigned grid = (unsigned)((units + 7) / 8 * 8 * 32);
  switch (var) {
  case 0: w4r_kernel<0><<<grid, kThreads, 0, stream>>>(a); break;
  case 1: w4r_kernel<1><<<grid, kThreads, 0, stream>>>(a); break;
  case 2: w4r2_kernel<<<grid, kThreads, 0, stream>>>(a); break;
  default: return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
