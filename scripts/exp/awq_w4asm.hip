// awq_w4asm.hip -- measurement-only: the AWQ search GEMM + loss (the product's awq_search_pp_kernel
// arithmetic) on the one-wave-per-SIMD 256 x 256 tile, K loop written at the instruction level
// (scripts/exp/gen_w4asm.py describes the schedule; w4asm_body.inc is its output).  Built by
// scripts/exp/build_exp.sh, timed by scripts/exp/bench_awq_exp.py (variant 70) against the
// product kernel and hipBLASLt.  Not part of the product library.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtq_amd.h"
#include "mtq_device.hpp"
#include "w4asm_body.inc"

using namespace mtq;

namespace {
struct Args {
  const void *x, *wq, *yref;
  float *partial;
  int64_t M, N, K;
  int tiles_m, tiles_n, G;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void *base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

template <int V>
__global__ __launch_bounds__(256) void w4asm_kernel(Args p) {
  constexpr int S = kW4Slots[V], EPI = kW4Epi[V], GM = kW4Gm[V] < 0 ? -kW4Gm[V] : kW4Gm[V];
  constexpr bool XN = kW4Gm[V] < 0;
  __shared__ __attribute__((aligned(16))) unsigned char lds[S == 2 ? 131072 : S * 32768];  // S 2: the T64 schedule, two 64 KiB tile slots
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int orig = blockIdx.x;
  int g, tm, tn;
  {  // the product's tile order: 8 x 4 tile units, one per XCD round, XCDs on the same alpha / column range
    const int xcd = orig % 8, li = orig / 8;
    constexpr int GN = 32 / GM;
    const int slot = li % 32, u = (li / 32) * 8 + xcd;
    const int mgn = (p.tiles_m + GM - 1) / GM, nn4 = (p.tiles_n + GN - 1) / GN;
    // GM < 0 encodes the N-synchronised order: the 8 XCDs of a round share the X panels (same
    // row group) and take consecutive column groups (different W panels)
    const int mg = XN ? (u / nn4) % mgn : u % mgn, n4 = XN ? u % nn4 : (u / mgn) % nn4;
    g = u / (mgn * nn4);
    tm = mg * GM + slot % GM;
    tn = n4 * GN + slot / GM;
    if (g >= p.G || tm >= p.tiles_m || tn >= p.tiles_n) return;
  }
  const int tiles = p.tiles_m * p.tiles_n;
  const int tile = tm * p.tiles_n + tn;
  const int64_t m0 = (int64_t)tm * 256, n0 = (int64_t)tn * 256;
  const int64_t K = p.K;
  const __bf16 *X = reinterpret_cast<const __bf16 *>(p.x) + (int64_t)g * p.M * K;
  const __bf16 *W = reinterpret_cast<const __bf16 *>(p.wq) + (int64_t)g * p.N * K;
  const __amdgpu_buffer_rsrc_t xr = rsrc_of(X, (uint32_t)(p.M * K * 2));
  const __amdgpu_buffer_rsrc_t wr = rsrc_of(W, (uint32_t)(p.N * K * 2));

  static_assert(S == 2, "T64 only");
  {
    // T64 (gen_w4asm.py body_t64): K tiles of 64, 128-byte LDS rows, chunk c of row r stored at
    // c ^ ((r >> 1) & 7).  DMA: wave w fills 1 KiB blocks w*8 + u of each operand's tile part (8
    // rows of 128 B); lane l writes row 64 w + 8 u + (l >> 3), stored chunk l & 7.
    unsigned xo[8], wo[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = 64 * wave + 8 * u + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int64_t row = m0 + r < p.M ? m0 + r : p.M - 1;
      const int64_t col = n0 + r < p.N ? n0 + r : p.N - 1;
      xo[u] = (unsigned)((row * K + 8 * c) * 2) - (unsigned)((u % 4) * 1024);  // the instruction offset adds it back
      wo[u] = (unsigned)((col * K + 8 * c) * 2) - (unsigned)((u % 4) * 1024);
    }
    const int fr = lane & 15, fq = lane >> 4;
    const unsigned lds0 = (unsigned)(uintptr_t)lds;
    const unsigned lt0 = fr * 128 + (((0 + fq) ^ ((fr >> 1) & 7)) << 4);
    const unsigned lt1 = fr * 128 + (((4 + fq) ^ ((fr >> 1) & 7)) << 4);
    const unsigned xb0 = lds0 + wm * 16384 + lt0, xb1 = lds0 + wm * 16384 + lt1;
    const unsigned wb0 = lds0 + 32768 + wn * 16384 + lt0, wb1 = lds0 + 32768 + wn * 16384 + lt1;
    const unsigned m0b = __builtin_amdgcn_readfirstlane(lds0 + wave * 8192);
    unsigned koff, kc, m0s, sdma, srd;
    unsigned cnt = __builtin_amdgcn_readfirstlane((unsigned)(K / 64));
    const unsigned klast = __builtin_amdgcn_readfirstlane((unsigned)((K / 64 - 1) * 128));
    if constexpr (EPI >= 2) {
      // the reference tile rides in the last two K tiles' DMAs (gen_w4asm.py body_t64y): half h
      // (rows 128 h ..) lands in slot (K / 64 + h) % 2, row r's 16-byte chunk c at c ^ (r & 15)
      const __amdgpu_buffer_rsrc_t yr = rsrc_of(p.yref, (uint32_t)(p.M * p.N * 2));
      const unsigned yrb = __builtin_amdgcn_readfirstlane((unsigned)(((m0 + 32 * wave) * p.N + n0) * 2));
      const unsigned yh = __builtin_amdgcn_readfirstlane((unsigned)(128 * p.N * 2));
      const unsigned ys2 = __builtin_amdgcn_readfirstlane((unsigned)(2 * p.N * 2));
      const unsigned m0yb = __builtin_amdgcn_readfirstlane(lds0 + wave * 16384);
      unsigned yo[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        yo[k] = (unsigned)((lane >> 5) * p.N * 2) + 16u * (unsigned)((lane & 31) ^ ((2 * k + (lane >> 5)) & 15));
      unsigned m0y, yso, ybs;
      // EPI 3 (T64B): the loop runs two tiles per pass (K % 128 == 0)
      unsigned cnt2 = __builtin_amdgcn_readfirstlane((unsigned)(EPI == 3 ? (K / 64 - 2) / 2 : K / 64 - 2));
#define W4_ASMY(BODY) \
      asm volatile(BODY \
                   : [koff] "=&s"(koff), [kc] "=&s"(kc), [m0s] "=&s"(m0s), [sdma] "=&s"(sdma), [srd] "=&s"(srd), \
                     [cnt] "+s"(cnt2), [m0y] "=&s"(m0y), [yso] "=&s"(yso), [ybs] "=&s"(ybs) \
                   : [xr] "s"(xr), [wr] "s"(wr), [m0b] "s"(m0b), [klast] "s"(klast), \
                     [xo0] "v"(xo[0]), [xo1] "v"(xo[1]), [xo2] "v"(xo[2]), [xo3] "v"(xo[3]), \
                     [xo4] "v"(xo[4]), [xo5] "v"(xo[5]), [xo6] "v"(xo[6]), [xo7] "v"(xo[7]), \
                     [wo0] "v"(wo[0]), [wo1] "v"(wo[1]), [wo2] "v"(wo[2]), [wo3] "v"(wo[3]), \
                     [wo4] "v"(wo[4]), [wo5] "v"(wo[5]), [wo6] "v"(wo[6]), [wo7] "v"(wo[7]), \
                     [xb0] "v"(xb0), [xb1] "v"(xb1), [wb0] "v"(wb0), [wb1] "v"(wb1), \
                     [yr] "s"(yr), [yrb] "s"(yrb), [yh] "s"(yh), [ys2] "s"(ys2), [m0yb] "s"(m0yb), \
                     [yo0] "v"(yo[0]), [yo1] "v"(yo[1]), [yo2] "v"(yo[2]), [yo3] "v"(yo[3]), \
                     [yo4] "v"(yo[4]), [yo5] "v"(yo[5]), [yo6] "v"(yo[6]), [yo7] "v"(yo[7]) \
                   : W4ASM_CLOBBERS)
      if constexpr (V == 0) W4_ASMY(W4ASM_BODY_Y_0);
      if constexpr (V == 1) W4_ASMY(W4ASM_BODY_Y_1);
      if constexpr (V == 2) W4_ASMY(W4ASM_BODY_Y_2);




#undef W4_ASMY
    }
#define W4_ASM64(BODY)                                                                               \
  asm volatile(BODY                                                                                  \
               : [koff] "=&s"(koff), [kc] "=&s"(kc), [m0s] "=&s"(m0s), [sdma] "=&s"(sdma),             \
                 [srd] "=&s"(srd), [cnt] "+s"(cnt)                                                       \
               : [xr] "s"(xr), [wr] "s"(wr), [m0b] "s"(m0b), [klast] "s"(klast),                         \
                 [xo0] "v"(xo[0]), [xo1] "v"(xo[1]), [xo2] "v"(xo[2]), [xo3] "v"(xo[3]),                  \
                 [xo4] "v"(xo[4]), [xo5] "v"(xo[5]), [xo6] "v"(xo[6]), [xo7] "v"(xo[7]),                  \
                 [wo0] "v"(wo[0]), [wo1] "v"(wo[1]), [wo2] "v"(wo[2]), [wo3] "v"(wo[3]),                  \
                 [wo4] "v"(wo[4]), [wo5] "v"(wo[5]), [wo6] "v"(wo[6]), [wo7] "v"(wo[7]),                  \
                 [xb0] "v"(xb0), [xb1] "v"(xb1), [wb0] "v"(wb0), [wb1] "v"(wb1)                           \
               : W4ASM_CLOBBERS)
    static_assert(EPI >= 2, "the reference-prefetch epilogue only");
#undef W4_ASM64
  }
  const int fr = lane & 15, fq = lane >> 4;
  // epilogue: a lane's accumulators of tile (i, j) are out[m][n .. n+3], m = 16 i + fr, n = 16 j + 4 fq
  // (the W fragment is the MFMA's A operand); output and difference rounded to bf16, fp32 square-sum
  const __bf16 *Y = reinterpret_cast<const __bf16 *>(p.yref);
  float sum = 0.f;
  float o[32];
  const unsigned yslot = (unsigned)(((K / 64 + wm) & 1) * 65536);
#define W4_STRIP(I)                                                                                  \
  {                                                                                                  \
    W4ASM_STRIP_##I(o);                                                                              \
    const int64_t m = m0 + wm * 128 + 16 * (I) + fr;                                                 \
    const bool rok = m < p.M;                                                                        \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                                  \
      const int64_t n = n0 + wn * 128 + 16 * j + 4 * fq;                                             \
      const bool ok = rok && n < p.N;                                                                \
      __bf16 yr[4];                                                                                  \
      const int64_t off = (ok ? m : 0) * p.N + (ok ? n : 0);                                         \
      if constexpr (EPI == 1) {                                                                      \
        __builtin_memset(yr, 0, 8);                                                                  \
      } else if constexpr (EPI >= 2) {                                                               \
        const int rr = 16 * (I) + fr, cl = wn * 128 + 16 * j + 4 * fq;                               \
        __builtin_memcpy(yr, lds + yslot + rr * 512 + (((cl >> 3) ^ fr) << 4) + (cl & 7) * 2, 8);    \
      } else {                                                                                       \
        __builtin_memcpy(yr, Y + off, 8);                                                            \
      }                                                                                              \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                                \
        const float y = Elem<__bf16>::ld(Elem<__bf16>::st(o[j * 4 + e]));                            \
        const float d = Elem<__bf16>::ld(Elem<__bf16>::st(y - Elem<__bf16>::ld(yr[e])));             \
        sum = ok ? __builtin_fmaf(d, d, sum) : sum;                                                  \
      }                                                                                              \
    }                                                                                                \
  }
  W4_STRIP(0) W4_STRIP(1) W4_STRIP(2) W4_STRIP(3) W4_STRIP(4) W4_STRIP(5) W4_STRIP(6) W4_STRIP(7)
#undef W4_STRIP
  __syncthreads();
#pragma unroll
  for (int o2 = 32; o2 >= 1; o2 >>= 1) sum += __shfl_xor(sum, o2);
  float *red = reinterpret_cast<float *>(lds);
  if (lane == 0) red[wave] = sum;
  __syncthreads();
  if (tid == 0) p.partial[(int64_t)g * tiles + tile] = red[0] + red[1] + red[2] + red[3];
}
}  // namespace

// xs [G, M, K] pre-scaled activations, wq [G, N, K], yref [M, N] (bf16); partial [G * tiles]
template <int V> int go(const Args &a, hipStream_t stream) {
  constexpr int GM = kW4Gm[V] < 0 ? -kW4Gm[V] : kW4Gm[V], GN = 32 / GM;
  const int units = a.G * ((a.tiles_m + GM - 1) / GM) * ((a.tiles_n + GN - 1) / GN);
  w4asm_kernel<V><<<(unsigned)((units + 7) / 8 * 8 * 32), 256, 0, stream>>>(a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// var: gen_w4asm.py VARIANTS index
extern "C" int awq_w4asm(int var, const void *xs, const void *wq, const void *yref, float *partial, int64_t M, int64_t N,
                         int64_t K, int G, hipStream_t stream) {
  if (K % 128 || K < 128 || N % 8) return 2;
  Args a{xs, wq, yref, partial, M, N, K, (int)((M + 255) / 256), (int)((N + 255) / 256), G};
  switch (var) {
  case 0: return go<0>(a, stream);
  case 1: return go<1>(a, stream);
  case 2: return go<2>(a, stream);
  default: return 3;
  }
}
