// hist_exp.hip -- measurement-only variants of the 16-bit pattern histogram (csrc/mtq_kernels.hip
// hist_value_kernel), built into scripts/exp/libhist_exp.so by scripts/exp/build_exp.sh and timed
// against the product kernel by scripts/exp/bench_hist_exp.py.  Not part of the product library.
//
// VAR bits: 1 = final bin atomics in a per-workgroup rotated order (concurrent workgroups hit
// different addresses); 2 = two named register batches (A/B) with unconditional, clamped loads --
// no register copy of an in-flight load and no branch around a load, so the compiler can count
// vmcnt; 4 = probe: no main loop (zero + fold + flush only); 8 = U * 2 vectors per batch;
// 64 = stream probe: the A/B loop with the LDS atomics replaced by a register xor (the loop's
// memory floor; counts wrong); 128 = three named batches (A/B/C, two batches in flight while one
// is counted), clamped loads; 256 = fold fast path: a wave whose 256 patterns all land in one bin
// (monotone bins: first == last) sums its counts by a wave reduction and adds once (the bin-0
// region below hi / bins holds ~90 % of the patterns <= phi); 512 = the first batch's loads
// issued before the hmax load and the LDS zeroing (VAR 2 loop only); 1024 = flush into the
// workgroup's chunk row (counts + (block / bpc) * bins, atomics: the product's chunked form);
// 2048 = plain stores of every bin into the workgroup's own row (counts + block * bins, no
// atomics, no zeroing needed), folded by hist_fold_blocks_kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kThreads = 1024;
constexpr int kPatterns = 32768;
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_bits_to_float(uint32_t b) { return __uint_as_float(b << 16); }

template <int U, int VAR>
__global__ __launch_bounds__(kThreads) void hist_exp_kernel(const uint16_t *__restrict__ x, int64_t nvec,
                                                            int64_t vec_per_block, const float *hmax, int bins,
                                                            uint32_t *counts, int bpc) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t *vh = sh;
  uint32_t *bh = sh + kPatterns;
  u32x4 a[U];
  {
    const int64_t v0 = (int64_t)blockIdx.x * vec_per_block;
    int64_t v1 = v0 + vec_per_block;
    v1 = v1 < nvec ? v1 : nvec;
    if constexpr ((VAR & 512) != 0) {
      const int64_t last = v1 - 1, i = v0 + threadIdx.x;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t k = i + (int64_t)u * kThreads;
        a[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(x + (k < last ? k : last) * 8));
      }
    }
  }
  float lo = 0.f, hi = *hmax;
  if (hi == lo) {
    lo -= 1.f;
    hi += 1.f;
  }
  // VAR & 16: only the patterns whose value can be <= hi are zeroed and folded (the largest bf16
  // pattern p with value(p) <= hi; NaN hi -> nothing counts); the main loop still increments every
  // pattern, the entries past phi are never read
  int phi = kPatterns - 1;
  if constexpr ((VAR & 16) != 0) {
    if (!(hi >= 0.f)) {
      phi = -1;
    } else {
      uint32_t b = __float_as_uint(hi) >> 16;  // truncation: value(b) <= hi
      b = b < 0x7F80u ? b : 0x7F80u;
      phi = (int)b;
    }
  }
  const float fb = (float)bins;
  const float span = hi - lo;
  const float y = 1.f / span;
  const uint32_t lastb = (uint32_t)bins - 1u;
  auto bin_of = [&](uint32_t p) -> uint32_t {
    const float a = bf16_bits_to_float(p);
    const float t = (a - lo) * fb;
    const float q0 = t * y;
    const float q = __builtin_fmaf(__builtin_fmaf(-q0, span, t), y, q0);
    const uint32_t b = (uint32_t)(int)q;
    return b < lastb ? b : lastb;
  };
  // VAR & 4096: compact table (r05: no faster on the bench input, 6 % slower on the 117 M tensor,
  // profiles/r05/hist/hist_compact_table_ab_*_r05hx9.log -- the extra VALU per element outweighs
  // the smaller zero / fold) -- every pattern below p0 (the first pattern whose bin is >= 1; the
  // bins are monotone in the pattern) shares slot 0 (bin 0), pattern p >= p0 takes slot p - d
  // (d = p0 - 1), every pattern past phi the dump slot cap; zeroing and folding cover cap + 1
  // slots instead of phi + 1 patterns (bf16, 2048 bins, hmax 96: ~1.4 K vs ~17 K)
  int d = -1, cap = phi + 1;
  if constexpr ((VAR & 4096) != 0) {
    if (phi >= 0) {
      int lo_p = 0, hi_p = phi + 1;  // first p in [0, phi + 1) with bin_of(p) >= 1, else phi + 1
      while (lo_p < hi_p) {
        const int mid = (lo_p + hi_p) >> 1;
        if (bin_of((uint32_t)mid) >= 1u) hi_p = mid; else lo_p = mid + 1;
      }
      d = lo_p - 1;
      cap = phi - d + 1;
    }
  }
  const int nz4 = (VAR & 4096) ? (cap + 4) / 4 : (phi + 4) / 4;  // uint4 words to zero / fold
  for (int i = threadIdx.x; i < nz4; i += kThreads) reinterpret_cast<uint4 *>(vh)[i] = make_uint4(0u, 0u, 0u, 0u);
  for (int b = threadIdx.x; b < bins; b += kThreads) bh[b] = 0;
  const int64_t v0 = (int64_t)blockIdx.x * vec_per_block;
  int64_t v1 = v0 + vec_per_block;
  v1 = v1 < nvec ? v1 : nvec;
  constexpr int64_t kStep = (int64_t)kThreads * U;
  uint32_t sink = 0;
  auto count1 = [&](u32x4 v, bool ok) {
    if constexpr ((VAR & 64) != 0) {
      sink ^= ok ? (v.x ^ v.y ^ v.z ^ v.w) : 0u;
      return;
    }
    const uint32_t w[4] = {ok ? v.x : 0x7FFF7FFFu, ok ? v.y : 0x7FFF7FFFu, ok ? v.z : 0x7FFF7FFFu,
                           ok ? v.w : 0x7FFF7FFFu};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr ((VAR & 4096) != 0) {
        const int a0 = (int)(w[j] & 0x7FFFu) - d, a1 = (int)((w[j] >> 16) & 0x7FFFu) - d;
        atomicAdd(vh + min(max(a0, 0), cap), 1u);
        atomicAdd(vh + min(max(a1, 0), cap), 1u);
      } else {
        atomicAdd(vh + (w[j] & 0x7FFFu), 1u);
        atomicAdd(vh + ((w[j] >> 16) & 0x7FFFu), 1u);
      }
    }
  };
  int64_t i = v0 + threadIdx.x;
  if constexpr ((VAR & 4) == 0) {
    if constexpr (VAR & 128) {
      const int64_t last = v1 - 1;
      auto ld = [&](int64_t k) -> u32x4 {
        const int64_t kc = k < last ? k : last;
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(x + kc * 8));
      };
      u32x4 b[U], c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] = ld(i + (int64_t)u * kThreads);
#pragma unroll
      for (int u = 0; u < U; ++u) b[u] = ld(i + kStep + (int64_t)u * kThreads);
      __syncthreads();
      for (; i < v1; i += 3 * kStep) {
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = ld(i + 2 * kStep + (int64_t)u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(a[u], i + (int64_t)u * kThreads < v1);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(i + 3 * kStep + (int64_t)u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(b[u], i + kStep + (int64_t)u * kThreads < v1);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(i + 4 * kStep + (int64_t)u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(c[u], i + 2 * kStep + (int64_t)u * kThreads < v1);
      }
    } else if constexpr (VAR & 2) {
      const int64_t last = v1 - 1;
      auto ld = [&](int64_t k) -> u32x4 {
        const int64_t kc = k < last ? k : last;
        return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(x + kc * 8));
      };
      u32x4 b[U];
      if constexpr ((VAR & 512) == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(i + (int64_t)u * kThreads);
      }
      __syncthreads();
      for (; i < v1; i += 2 * kStep) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(i + kStep + (int64_t)u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(a[u], i + (int64_t)u * kThreads < v1);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(i + 2 * kStep + (int64_t)u * kThreads);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(b[u], i + kStep + (int64_t)u * kThreads < v1);
      }
    } else {
      auto load = [&](int64_t ii, u32x4 (&v)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t k = ii + (int64_t)u * kThreads;
          if (k < v1)
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(x + k * 8));
          else
            v[u] = u32x4{0x7FFF7FFFu, 0x7FFF7FFFu, 0x7FFF7FFFu, 0x7FFF7FFFu};
        }
      };
      u32x4 cur[U];
      load(i, cur);
      __syncthreads();
      for (; i < v1; i += kStep) {
        u32x4 nxt[U];
        if (i + kStep < v1) load(i + kStep, nxt);
#pragma unroll
        for (int u = 0; u < U; ++u) count1(cur[u], true);
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
      }
    }
  } else {
    __syncthreads();
  }
  if constexpr ((VAR & 64) != 0)
    if (sink == 0x12345678u) atomicAdd(vh, 1u);  // keeps the loads alive
  __syncthreads();
  if constexpr ((VAR & 256) != 0) {
    // wave-uniform iteration: wave w0 .. w0 + 63 words; uniform-bin waves reduce and add once
    const int lane = threadIdx.x & 63;
    for (int wb = threadIdx.x & ~63; wb < nz4; wb += kThreads) {
      const int w = wb + lane;
      const uint4 c4 = w < nz4 ? reinterpret_cast<const uint4 *>(vh)[w] : make_uint4(0u, 0u, 0u, 0u);
      const int plast = 4 * (wb + 63) + 3 < phi ? 4 * (wb + 63) + 3 : phi;
      const uint32_t bfirst = bin_of((uint32_t)(4 * wb)), blast = bin_of((uint32_t)plast);
      if (bfirst == blast) {
        // every pattern <= phi of this wave is in bin bfirst (patterns past phi are dropped)
        uint32_t sum = 0;
        const uint32_t cs[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) sum += (4 * w + j <= phi) ? cs[j] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) sum += (uint32_t)__shfl_xor((int)sum, o, 64);
        if (lane == 0 && sum) atomicAdd(bh + bfirst, sum);
        continue;
      }
      if (w >= nz4) continue;
      const uint32_t cs[4] = {c4.x, c4.y, c4.z, c4.w};
      uint32_t run_b = 0xFFFFFFFFu, run_c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t pp = (uint32_t)(4 * w + j);
        if (cs[j] == 0u || (int)pp > phi) continue;
        const float av = bf16_bits_to_float(pp);
        if (!(av <= hi)) continue;
        const uint32_t b = bin_of(pp);
        if (b != run_b) {
          if (run_c) atomicAdd(bh + run_b, run_c);
          run_b = b;
          run_c = 0;
        }
        run_c += cs[j];
      }
      if (run_c) atomicAdd(bh + run_b, run_c);
    }
  } else if constexpr ((VAR & 4096) != 0) {
    // slots: 0 = every pattern below p0 (bin 0, when d >= 0), 1 .. cap - 1 = patterns d + 1 ..
    // phi, cap = past phi (dropped); four slots per lane, equal-bin runs merged
    for (int w = threadIdx.x; w < nz4; w += kThreads) {
      const uint4 c4 = reinterpret_cast<const uint4 *>(vh)[w];
      const uint32_t cs[4] = {c4.x, c4.y, c4.z, c4.w};
      uint32_t run_b = 0xFFFFFFFFu, run_c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int sl = 4 * w + j;
        if (cs[j] == 0u || sl >= cap) continue;
        const uint32_t b = sl == 0 ? 0u : bin_of((uint32_t)(sl + d));
        if (b != run_b) {
          if (run_c) atomicAdd(bh + run_b, run_c);
          run_b = b;
          run_c = 0;
        }
        run_c += cs[j];
      }
      if (run_c) atomicAdd(bh + run_b, run_c);
    }
  } else if constexpr ((VAR & 32) != 0) {
    // 4 consecutive patterns per lane (one ds_read_b128; a wave reads 1 KB contiguous), the
    // counts of equal bins merged in registers before one LDS atomic per run
    for (int w = threadIdx.x; w < nz4; w += kThreads) {
      const uint4 c4 = reinterpret_cast<const uint4 *>(vh)[w];
      const uint32_t cs[4] = {c4.x, c4.y, c4.z, c4.w};
      uint32_t run_b = 0xFFFFFFFFu, run_c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t p = (uint32_t)(4 * w + j);
        if (cs[j] == 0u || (int)p > phi) continue;
        const float a = bf16_bits_to_float(p);
        if (!(a <= hi)) continue;
        const uint32_t b = bin_of(p);
        if (b != run_b) {
          if (run_c) atomicAdd(bh + run_b, run_c);
          run_b = b;
          run_c = 0;
        }
        run_c += cs[j];
      }
      if (run_c) atomicAdd(bh + run_b, run_c);
    }
  } else {
    for (int p = threadIdx.x; p <= phi; p += kThreads) {
      const uint32_t c = vh[p];
      if (c == 0u) continue;
      const float a = bf16_bits_to_float((uint32_t)p);
      if (a <= hi) atomicAdd(bh + bin_of((uint32_t)p), c);
    }
  }
  __syncthreads();
  if constexpr ((VAR & 2048) != 0) {
    uint32_t *row = counts + (int64_t)blockIdx.x * bins;
    for (int b = threadIdx.x; b < bins; b += kThreads) __builtin_nontemporal_store(bh[b], row + b);
    return;
  }
  if constexpr ((VAR & 1024) != 0) counts += (int64_t)(blockIdx.x / bpc) * bins;
  const int rot = (VAR & 1) ? (int)((blockIdx.x * 64u) % (unsigned)bins) : 0;
  for (int bb = threadIdx.x; bb < bins; bb += kThreads) {
    int b = bb + rot;
    b = b >= bins ? b - bins : b;
    if (bh[b]) atomicAdd(counts + b, bh[b]);
  }
}

// the product's fold (hist_fold_rows_kernel): 16 chunk rows, clamp, chunk-order fp32 sum, rows zeroed
__global__ __launch_bounds__(256) void fold_rows_kernel(uint32_t *__restrict__ rows, int chunks, int bins,
                                                        float *hist) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= bins) return;
  float h = 0.f;
  for (int c0 = 0; c0 < chunks; c0 += 16) {
    uint32_t v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = c0 + j < chunks ? rows[(int64_t)(c0 + j) * bins + b] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      h += fminf((float)v[j], 16777216.f);
      if (c0 + j < chunks) rows[(int64_t)(c0 + j) * bins + b] = 0u;
    }
  }
  hist[b] = h;
}
// per-workgroup rows: 1024 threads = 64 bins x 16 chunks; a thread sums its chunk's bpc rows
// (exact, uint32), clamps, and lane (bin, chunk 0) adds the 16 clamped chunk counts in order
__global__ __launch_bounds__(1024) void fold_blocks_kernel(const uint32_t *__restrict__ rows, int bpc, int chunks,
                                                           int bins, float *hist) {
  __shared__ float sc[16][64];
  const int bl = threadIdx.x & 63, c = threadIdx.x >> 6, b = blockIdx.x * 64 + bl;
  if (c < chunks && b < bins) {
    uint32_t s = 0;
    for (int k0 = 0; k0 < bpc; k0 += 8) {
      uint32_t v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[k] = k0 + k < bpc ? __builtin_nontemporal_load(rows + ((int64_t)c * bpc + k0 + k) * bins + b) : 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    sc[c][bl] = fminf((float)s, 16777216.f);
  }
  __syncthreads();
  if (c == 0 && b < bins) {
    float h = 0.f;
    for (int k = 0; k < chunks; ++k) h += sc[k][bl];
    hist[b] = h;
  }
}

template <int U, int VAR>
int launch(const void *x, int64_t n, const float *hmax, int bins, uint32_t *counts, hipStream_t stream) {
  const int64_t nvec = n / 8;
  int cu = 256;
  int dev = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev);
  int64_t blocks = cu;
  const int64_t min_per_block = (int64_t)kThreads * 8;
  int64_t vpb = (nvec + blocks - 1) / blocks;
  vpb = vpb < min_per_block ? min_per_block : vpb;
  blocks = (nvec + vpb - 1) / vpb;
  const size_t shr = ((size_t)kPatterns + (size_t)bins) * 4;
  auto kern = hist_exp_kernel<U, VAR>;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  kern<<<(unsigned)blocks, kThreads, shr, stream>>>(reinterpret_cast<const uint16_t *>(x), nvec, vpb, hmax, bins,
                                                    counts, 1);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
}  // namespace

// chunked pairs (16 chunks of 16 workgroups, uniform per-workgroup ranges -- the timing shape of
// the product's chunked call, not its chunk edges): 0 = VAR 562|1024 + fold_rows_kernel (the
// product's structure on the A/B loop); 1 = VAR 562|2048 + fold_blocks_kernel
extern "C" int hist_exp_chunked(int var, const void *x, int64_t n, const float *hmax, int bins, uint32_t *scratch,
                                float *hist, hipStream_t stream) {
  if (n % 8 || bins < 1 || bins > 8192 || ((uintptr_t)x & 15)) return 2;
  const int64_t nvec = n / 8;
  const int chunks = 16, bpc = 16, blocks = chunks * bpc;
  const int64_t vpb = (nvec + blocks - 1) / blocks;
  const size_t shr = ((size_t)kPatterns + (size_t)bins) * 4;
  if (var == 0) {
    auto kern = hist_exp_kernel<2, 562 | 1024>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    kern<<<blocks, kThreads, shr, stream>>>(reinterpret_cast<const uint16_t *>(x), nvec, vpb, hmax, bins, scratch, bpc);
    fold_rows_kernel<<<(bins + 255) / 256, 256, 0, stream>>>(scratch, chunks, bins, hist);
  } else if (var == 1) {
    auto kern = hist_exp_kernel<2, 562 | 2048>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    kern<<<blocks, kThreads, shr, stream>>>(reinterpret_cast<const uint16_t *>(x), nvec, vpb, hmax, bins, scratch, bpc);
    fold_blocks_kernel<<<(bins + 63) / 64, 1024, 0, stream>>>(scratch, bpc, chunks, bins, hist);
  } else {
    return 3;
  }
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int hist_exp(int var, const void *x, int64_t n, const float *hmax, int bins, uint32_t *counts,
                        hipStream_t stream) {
  if (n % 8 || bins < 1 || bins > 8192 || ((uintptr_t)x & 15)) return 2;
  switch (var) {
  case 0: return launch<2, 0>(x, n, hmax, bins, counts, stream);
  case 1: return launch<2, 1>(x, n, hmax, bins, counts, stream);
  case 2: return launch<2, 2>(x, n, hmax, bins, counts, stream);
  case 3: return launch<2, 3>(x, n, hmax, bins, counts, stream);
  case 4: return launch<2, 4>(x, n, hmax, bins, counts, stream);
  case 11: return launch<4, 1>(x, n, hmax, bins, counts, stream);
  case 13: return launch<4, 3>(x, n, hmax, bins, counts, stream);
  case 17: return launch<1, 3>(x, n, hmax, bins, counts, stream);
  case 40: return launch<2, 16>(x, n, hmax, bins, counts, stream);
  case 41: return launch<2, 48>(x, n, hmax, bins, counts, stream);
  case 44: return launch<2, 20>(x, n, hmax, bins, counts, stream);
  case 45: return launch<2, 52>(x, n, hmax, bins, counts, stream);
  case 50: return launch<2, 50>(x, n, hmax, bins, counts, stream);
  case 51: return launch<4, 50>(x, n, hmax, bins, counts, stream);
  case 114: return launch<2, 114>(x, n, hmax, bins, counts, stream);
  case 115: return launch<4, 114>(x, n, hmax, bins, counts, stream);
  case 176: return launch<2, 176>(x, n, hmax, bins, counts, stream);
  case 177: return launch<1, 176>(x, n, hmax, bins, counts, stream);
  case 48: return launch<2, 48>(x, n, hmax, bins, counts, stream);
  case 304: return launch<2, 304>(x, n, hmax, bins, counts, stream);    // 48 | 256
  case 306: return launch<2, 306>(x, n, hmax, bins, counts, stream);    // 50 | 256
  case 562: return launch<2, 562>(x, n, hmax, bins, counts, stream);    // 50 | 512
  case 818: return launch<2, 818>(x, n, hmax, bins, counts, stream);    // 50 | 256 | 512
  case 4658: return launch<2, 4658>(x, n, hmax, bins, counts, stream);  // 562 | 4096 (compact table)
  default: return 3;
  }
}
