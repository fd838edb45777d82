// mtq_attention.hip — fused flash attention with softmax-P fake quant-dequant (gfx950).
//
// Reference: modelopt/torch/kernels/common/attention/triton_fa.py `_attn_fwd` (:255-516) as
// dispatched by `attention()` (:1221-1390) from the quantization plugin's `_triton_qdq_attention`
// (plugins/huggingface.py:145-195) when `p_bmm_quantizer` is per-tensor FP8 or dynamic NVFP4
// block 16 on causal attention.  Per query row and per 32-key tile (the kernel's BLOCK_N):
//
//     s   = (q . k) * sm_scale * log2(e);  masked keys -> -inf           (:395-403, :194-217)
//     m'  = max(m, max_tile s);  p = exp2(s - m');  c = exp2(m - m')      (:426-430)
//     l   = l * c + sum(p);  acc = acc * c                                (:431-432)
//     p   = qdq(p)            FP8:   e4m3(clamp(p / S, +-448)) * S,  S = amax / 448
//                             NVFP4: p -> V dtype, per 16 keys e2m1 with an e4m3 block scale,
//                                    global scale S = amax / (6 * 448)     (:436-451, bmm2_qdq.py)
//     acc += p . v            FP8/none: p rounded to the V dtype, bf16/f16 MMA, fp32 accumulate
//                             NVFP4:    fp32 MMA ("ieee" dot, :489)
//     o   = acc / max(l, 1e-6)                                            (:495)
// fp32 q/k/v (the reference's Q_IS_FP32 path, :392-393) run both products on
// v_mfma_f32_32x32x2_f32.
//
// The denominator l sums the UNQUANTISED p; the quantised p is relative to the running max of
// the tiles seen so far, so the result depends on the 32-key tiling -- kept here exactly.
//
// Layout (CDNA4-first): a 256-thread workgroup = 4 waves = 128 query rows of one (batch, head);
// each wave owns 32 rows.  Scores are computed transposed, S^T = K . Q^T with
// v_mfma_f32_32x32x16_{bf16,f16}, so lane l holds the 16 scores of query (l & 31) for keys
// crow(j, l >> 5) = (j & 3) + 8 (j >> 2) + 4 (l >> 5): the row max / row sum are 15 in-lane ops
// and one lane^32 exchange, and the P fragments of P . V come straight out of the score registers
// (the MMA's k index is permuted to the keys a lane already holds; V is read in the same order).
// The output is accumulated transposed, O^T = V^T . P^T, so the online-softmax correction is one
// per-lane scalar.  K and V [64 keys x D] (two softmax tiles) are register-staged into LDS per
// barrier pair (one copy per workgroup; K rows padded so ds_read_b128 of the K fragment hits
// distinct banks, V rows padded for conflict-free ds_read_b64_tr_b16, which delivers the V^T
// fragments transposed), the next stage's global loads issued before the current stage's math.  Workgroups of one KV head are
// consecutive on one XCD (shared K/V in its L2), the longest causal tiles first.
#include <hip/hip_runtime.h>
#include <math.h>
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

template <typename T> struct AMma;
template <> struct AMma<__bf16> {
  typedef __bf16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct AMma<_Float16> {
  typedef _Float16 v8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ f32x16 mma(v8 a, v8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
// fp32 q/k/v (the reference's Q_IS_FP32 path, "ieee" dots): both products on v_mfma_f32_32x32x2_f32
template <> struct AMma<float> {
  typedef float v8 __attribute__((ext_vector_type(8)));  // unused placeholder
};

struct AttnArgs {
  const void *q, *k, *v;
  void *o;
  const int32_t *start_q, *len_q, *start_k, *len_k;
  int64_t qb, qt, qh, kb, kt, kh, vb, vt, vh, ob, ot, oh;  // element strides (batch, token, head)
  int hkv, group, tiles_q, causal, ppw;  // ppw: query-tile pairs per workgroup
  float qk_scale, p_scale;
};

constexpr int kThreads = 256, kRowsPerBlock = 128, kKv = 32;
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
constexpr float kNegInf = -__builtin_inff();

// key (within the 32-key tile) of score register j of a lane in half hi (C layout of 32x32 MFMA)
__device__ __forceinline__ int crow(int j, int hi) { return (j & 3) + 8 * (j >> 2) + 4 * hi; }

__device__ __forceinline__ float fp8_rt(float v) {  // e4m3 round trip, RNE (v already clamped)
  const int p = __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
  return __builtin_amdgcn_cvt_f32_fp8(p, 0);
}

// fp4_round_magnitude (kernels/quantization/common/nvfp4_quant.py): nearest E2M1 magnitude,
// ties to even
__device__ __forceinline__ float e2m1_mag(float a) {
  return a <= 0.25f ? 0.f
       : a < 0.75f  ? 0.5f
       : a <= 1.25f ? 1.f
       : a < 1.75f  ? 1.5f
       : a <= 2.5f  ? 2.f
       : a < 3.5f   ? 3.f
       : a <= 5.f   ? 4.f
                    : 6.f;
}

typedef float f2v __attribute__((ext_vector_type(2)));

// v < 448 ? v : 448 for v >= +0 or a quiet NaN in ONE v_min_f32 (IEEE minNum returns the non-NaN
// operand: NaN -> 448, as the compare form; -0 stays -0); the compiler's form was v_cmp +
// v_cndmask
__device__ __forceinline__ float min448(float v) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(kE4M3Max));
  return r;
}

// RN(a / s) for a pair of a >= +0 (or NaN) on the packed fp32 ALU: div_rn (mtq_device.hpp) without
// its copysign -- p never is -0 -- two quotients per v_pk_mul / v_pk_fma
__device__ __forceinline__ f2v div_rn_pos2(f2v q, float s, float r) {
  const f2v sv = {s, s}, rv = {r, r};
  const f2v y0 = q * rv;
  const f2v e = __builtin_elementwise_fma(-y0, sv, q);
  return __builtin_elementwise_fma(e, rv, y0);
}

// two fp32 -> two packed T (one v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32, RNE); the asm pins the fp32
// pair so no mixed-precision fma folds the rounding (as Elem<T>::st)
template <typename T> __device__ __forceinline__ uint32_t pack2(float a, float b) {
  f2v v = {a, b};
  asm("" : "+v"(v));
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, t2));
}
template <typename T> __device__ __forceinline__ f2v unpack2(uint32_t w) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  return __builtin_convertvector(__builtin_bit_cast(t2, w), f2v);
}

// buffer descriptor of one K/V stage: wave-uniform base and size (readfirstlane: no waterfall)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stage_rsrc(const void *base, uint32_t bytes) {
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), 0, nb, 0x00020000);
}

// v op partner(v) for a symmetric op, partner = the lane^32 value: one v_permlane32_swap of v with
// itself gives each lane its own value in one result and its partner's in the other (lanes 0-31:
// r[0] own, r[1] partner; lanes 32-63: r[0] partner, r[1] own), so op(r[0], r[1]) needs no select
// -- replaces __shfl_xor(v, 32) (a ds_bpermute round trip through the LDS and its address math)
__device__ __forceinline__ float xmax32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xadd32(float v) {  // own + partner (commutative: same bits)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// LDS image sizes of one workgroup (K rows padded, V rows at the tr-read pitch)
// DBUF (16-bit q/k/v): two K/V stages, stage t+1 written while stage t is read -- one barrier per
// stage instead of two (2 x 37.9 KiB at D 128: two workgroups still fit a CU's 160 KiB)
template <typename T, int D, int PQ, int kStage> struct AttnLds {
  static constexpr bool F32 = sizeof(T) == 4;
  static constexpr int ES = sizeof(T), DP = D < 32 ? 32 : D;
  static constexpr int PITCH = DP * ES + 16;
  static constexpr int VPITCH = F32 ? PITCH : DP * 2 + 4 * ((16 - (DP / 2) % 32 + 32) % 32);
  static constexpr bool DBUF = !F32;
  static constexpr int NBUF = DBUF ? 2 : 1;
  static constexpr int KIMG = kStage * PITCH, VIMG = kStage * VPITCH;
};

// One 128-row query tile `tile` of (batch b, query head h, KV head kvh).
template <typename T, int D, int PQ, int kStage>  // kStage: keys staged in LDS per barrier pair
__device__ __forceinline__ void attn_tile(const AttnArgs &a, int b, int h, int kvh, int tile,
                                          unsigned char *__restrict__ Ks, unsigned char *__restrict__ Vs) {
  typedef typename AMma<T>::v8 v8;
  constexpr bool F32 = sizeof(T) == 4;
  // P . V of NVFP4 is an fp32 ("ieee") dot in the reference.  Its P is c * s_b: an E2M1 value c
  // (exact in bf16 / f16) times the fp32 scale s_b of the 16-key block b, and a 16-key block is
  // exactly the k extent of one v_mfma_f32_32x32x16 step, so (FACT) each step multiplies V by the
  // codes on the 16-bit MFMA (exact products, fp32 sums) into a zero accumulator and adds that
  // partial times the lane's s_b into O^T with one fma per element (a query's scale is a per-lane
  // scalar of the O^T layout).  Products c * v are exact either way; the rounding moves from the
  // reference's RN(c * s_b) per element to one RN per block partial -- fp32-level, far inside the
  // output dtype's ulp.  (r02 split P into three exact bf16 terms: 3 MFMAs per step.)  fp32 q/k/v
  // keep the fp32 MFMA.
  constexpr bool FACT = PQ == 2 && !F32;
  constexpr bool F32PV = F32;
  constexpr int ES = sizeof(T);
  constexpr int DP = D < 32 ? 32 : D;  // head_dim 16: one 32-wide d block, columns >= D zero
  constexpr int PITCH = DP * ES + 16;  // K row bytes (16-byte pad: conflict-free b128 reads)
  // V rows for ds_read_b64_tr_b16: a 32-lane half reads 4 rows x 16 dwords, conflict-free when
  // the row stride is 16 or 48 dwords mod 64
  // (the fp32 P . V path reads V per element instead and keeps the K pitch: its two lane halves
  // read rows 4 apart, which the tr pitch would put on the same banks)
  constexpr int VPITCH = F32PV ? PITCH : DP * 2 + 4 * ((16 - (DP / 2) % 32 + 32) % 32);
  constexpr int CR = D * ES / 16;     // 16-byte chunks per row
  constexpr int EC = 16 / ES;         // elements per chunk
  constexpr int NCH = kStage * CR;   // chunks per stage
  constexpr int NU = (NCH + kThreads - 1) / kThreads;
  constexpr int DB = DP / 32;  // 32-wide d blocks of O^T
  constexpr int QS = D / 16;  // k steps of S^T
  static_assert(AttnLds<T, D, PQ, kStage>::VPITCH == VPITCH && AttnLds<T, D, PQ, kStage>::PITCH == PITCH,
                "LDS layout");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, fr = lane & 31, hi = lane >> 5;

  const int lq = a.len_q[b], lk = a.len_k[b];
  const int r0 = tile * kRowsPerBlock;
  if (r0 >= lq) return;  // uniform over the workgroup
  const int off = lk - lq;  // causal: queries are the last lq positions of the key span
  const T *Q = reinterpret_cast<const T *>(a.q) + b * a.qb + (int64_t)a.start_q[b] * a.qt + h * a.qh;
  const T *K = reinterpret_cast<const T *>(a.k) + b * a.kb + (int64_t)a.start_k[b] * a.kt + kvh * a.kh;
  const T *V = reinterpret_cast<const T *>(a.v) + b * a.vb + (int64_t)a.start_k[b] * a.vt + kvh * a.vh;
  T *O = reinterpret_cast<T *>(a.o) + b * a.ob + (int64_t)a.start_q[b] * a.ot + h * a.oh;

  const int last = r0 + kRowsPerBlock < lq ? r0 + kRowsPerBlock : lq;
  int kv_end = a.causal ? off + last : lk;
  kv_end = kv_end < lk ? kv_end : lk;
  const int nstages = kv_end > 0 ? (kv_end + kStage - 1) / kStage : 0;

  const int q0 = r0 + 32 * wave;
  const bool active = q0 < lq;
  int w_end = a.causal ? off + (q0 + 32 < lq ? q0 + 32 : lq) : lk;
  w_end = w_end < lk ? w_end : lk;
  const int qrow = q0 + fr;

  v8 qf[F32 ? 1 : QS];
  float qf32[F32 ? D / 2 : 1];
  if constexpr (F32) {
#pragma unroll
    for (int s = 0; s < D / 2; ++s)
      qf32[s] = qrow < lq ? reinterpret_cast<const float *>(Q)[(int64_t)qrow * a.qt + 2 * s + hi] : 0.f;
  } else {
#pragma unroll
    for (int s = 0; s < QS; ++s) {
      if (qrow < lq) {
        qf[s] = *reinterpret_cast<const v8 *>(Q + (int64_t)qrow * a.qt + 16 * s + 8 * hi);
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) qf[s][i] = (T)0.f;
      }
    }
  }

  f32x16 acc[DB];
#pragma unroll
  for (int d = 0; d < DB; ++d)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[d][e] = 0.f;
  float m = kNegInf, l = 0.f;

  // K/V stage loads by raw buffer loads: the wave-uniform base of stage t (key t * kStage) in the
  // descriptor, the per-lane row/column offset in ONE loop-invariant VGPR per operand and the
  // u-th row group in the SGPR soffset.  Keys past the sequence fall outside the descriptor's
  // num_records (rows_valid * kt * ES bytes; kt >= D is a launch precondition) and read as zero
  // (0 * garbage could be NaN) without a per-row compare.  Replaces 64-bit global addresses
  // recomputed per stage (address math and VGPRs: 208 vs 226 at D 128, no spills).
  constexpr bool ROWSPLIT = (kThreads % CR) == 0;  // a lane's chunks share its column
  constexpr int RPU = kThreads / CR;               // rows per u (ROWSPLIT)
  uint32_t koff[ROWSPLIT ? 1 : NU], voff[ROWSPLIT ? 1 : NU];
  if constexpr (ROWSPLIT) {
    koff[0] = (uint32_t)((tid / CR) * a.kt * ES + (tid % CR) * 16);
    voff[0] = (uint32_t)((tid / CR) * a.vt * ES + (tid % CR) * 16);
  } else {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c = tid + kThreads * u, row = c / CR, col = c - (c / CR) * CR;
      koff[u] = (uint32_t)(row * a.kt * ES + col * 16);
      voff[u] = (uint32_t)(row * a.vt * ES + col * 16);
    }
  }
  const int kt_b = (int)(a.kt * ES), vt_b = (int)(a.vt * ES);
  uint4 kst[NU], vst[NU];
  auto gload = [&](int t) {
    int rows = lk - t * kStage;
    rows = rows < kStage ? rows : kStage;
    const __amdgpu_buffer_rsrc_t kr = stage_rsrc(K + (int64_t)t * kStage * a.kt, (uint32_t)(rows * kt_b));
    const __amdgpu_buffer_rsrc_t vr = stage_rsrc(V + (int64_t)t * kStage * a.vt, (uint32_t)(rows * vt_b));
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c = tid + kThreads * u;
      if (NCH % kThreads == 0 || c < NCH) {
        const uint32_t ko = ROWSPLIT ? koff[0] : koff[u], vo = ROWSPLIT ? voff[0] : voff[u];
        const int ks = ROWSPLIT ? u * RPU * kt_b : 0, vs = ROWSPLIT ? u * RPU * vt_b : 0;
        kst[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(kr, ko, ks, 0));
        vst[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vr, vo, vs, 0));
      }
    }
  };
  using LD = AttnLds<T, D, PQ, kStage>;
  auto swrite = [&](int buf) {
    unsigned char *const kb = Ks + buf * LD::KIMG;
    unsigned char *const vb = Vs + buf * LD::VIMG;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int c = tid + kThreads * u;
      if (NCH % kThreads == 0 || c < NCH) {
        const int row = c / CR, col = c - row * CR;
        *reinterpret_cast<uint4 *>(kb + row * PITCH + col * 16) = kst[u];
        *reinterpret_cast<uint4 *>(vb + row * VPITCH + col * 16) = vst[u];
      }
    }
  };

  float rs_p = 0.f, six_gs = 0.f, rs_six = 0.f;
  if (PQ == 1) rs_p = 1.0f / a.p_scale;
  if (PQ == 2) {
    six_gs = 6.0f * a.p_scale;
    rs_six = 1.0f / six_gs;
  }

  if constexpr (DP != D) {  // V columns D..31 are read by the d block and must be zero
    for (int i = tid; i < LD::NBUF * kStage * (DP - D); i += kThreads) {
      const int bi = i / (kStage * (DP - D)), r = i % (kStage * (DP - D));
      const int row = r / (DP - D), col = D + r % (DP - D);
      *reinterpret_cast<T *>(Vs + bi * LD::VIMG + row * VPITCH + col * ES) = (T)0.f;
    }
  }
  // ds_read_b64_tr_b16 address of this lane (T10): lane 4q+p of 16-lane group G supplies row
  // 4 (G >> 1) + q, columns 16 (G & 1) + 4p .. +3 of a [keys][d] block; lane (G, i) receives
  // column 16 (G & 1) + i = fr of those 4 rows = the V^T fragment elements of its half
  const int trq = (lane & 15) >> 2, trp = lane & 3, trg = lane >> 4;
  const int tr_off = (4 * (trg >> 1) + trq) * VPITCH + (16 * (trg & 1) + 4 * trp) * 2;

  if (nstages > 0) {
    gload(0);
    swrite(0);
  }
  // vmcnt(0) on EVERY path here: the Q fragment loads above are otherwise waited for only inside
  // the branch, the compiler's (path-insensitive) wait analysis then keeps them pending at the
  // loop head, and the first score MFMA of every stage (it reads qf) waited with vmcnt(0) -- for
  // the stage's own K/V prefetch too, so the prefetch never overlapped the math (ISA-verified)
  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15
  __syncthreads();
  constexpr int NSUB = kStage / kKv;
  const unsigned char *Kb = Ks, *Vb = Vs;  // the stage being read
  // ---- S^T = K . Q^T of one 32-key tile of the staged keys (lane: query fr, keys crow(j, hi))
  auto score = [&](int sub) -> f32x16 {
    const unsigned char *const Kt = Kb + sub * kKv * PITCH;
    f32x16 s;
#pragma unroll
    for (int e = 0; e < 16; ++e) s[e] = 0.f;
    if constexpr (F32) {
#pragma unroll
      for (int st = 0; st < D / 2; ++st) {
        const float kv = *reinterpret_cast<const float *>(Kt + fr * PITCH + (2 * st + hi) * 4);
        s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv, qf32[st], s, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int st = 0; st < QS; ++st) {
        const v8 kf = *reinterpret_cast<const v8 *>(Kt + fr * PITCH + (16 * st + 8 * hi) * 2);
        s = AMma<T>::mma(kf, qf[st], s);
      }
    }
    return s;
  };
  for (int t = 0; t < nstages; ++t) {
    if constexpr (LD::DBUF) {
      Kb = Ks + (t & 1) * LD::KIMG;
      Vb = Vs + (t & 1) * LD::VIMG;
    }
    if (t + 1 < nstages) gload(t + 1);  // in flight across this stage's math
    // the scores of tile sub + 1 are issued before the softmax of tile sub (they do not depend on
    // it): the matrix core works on them while the VALU runs the softmax and the P qdq
    // (not for NVFP4, whose per-block P . V partial needs those 16 registers at D 128, nor fp32)
    constexpr bool AHEAD = !FACT && !F32;
    // ---- pieces of one 32-key softmax tile (the reference's per-BLOCK_N step)
    // x = s * qk_scale (masked keys -inf); returns the lane's max of x
    auto scale_x = [&](const f32x16 &s, bool need_mask, int kv0, float (&x)[16]) -> float {
      float mloc = kNegInf;
      if (need_mask) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const int key = kv0 + crow(j, hi);
          const bool ok = key < lk && (!a.causal || qrow + off >= key);
          x[j] = ok ? s[j] * a.qk_scale : kNegInf;
          mloc = fmaxf(mloc, x[j]);
        }
      } else {
        const f2v qs2 = {a.qk_scale, a.qk_scale};  // two scores per v_pk_mul_f32 (same products)
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          const f2v xv = f2v{s[j], s[j + 1]} * qs2;
          x[j] = xv.x;
          x[j + 1] = xv.y;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) mloc = fmaxf(mloc, x[j]);
      }
      return mloc;
    };
    // p = exp2(x - mu) and the lane pair's sum of p (keys in j order, then the partner)
    auto expsum = [&](const float (&x)[16], float mu, float (&p)[16]) -> float {
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        p[j] = __builtin_amdgcn_exp2f(x[j] - mu);
        ls += p[j];
      }
      return xadd32(ls);
    };
    // acc * 1 == acc (NaN included): the rescale runs only when some row of the wave moved its
    // running max (wave-uniform branch), on packed pairs
    auto rescale = [&](float corr, bool moved) {
      if (__builtin_amdgcn_ballot_w64(moved)) {
        const f2v c2 = {corr, corr};
#pragma unroll
        for (int d = 0; d < DB; ++d)
#pragma unroll
          for (int e = 0; e < 16; e += 2) {
            const f2v r = f2v{acc[d][e], acc[d][e + 1]} * c2;
            acc[d][e] = r.x;
            acc[d][e + 1] = r.y;
          }
      }
    };
    // P fake quant in place (sblk: NVFP4's two 16-key block scales for FACT)
    auto qdq = [&](float (&p)[16], float (&sblk)[2]) {
      if (PQ == 1) {
        // ---- FP8 P qdq: e4m3(clamp(p / S, +-448)) * S  (p >= +0 or NaN), two keys per packed
        // divide, per v_cvt_pk_fp8_f32 and per v_cvt_pk_f32_fp8
        const f2v sp2 = {a.p_scale, a.p_scale};
#pragma unroll
        for (int j = 0; j < 16; j += 2) {
          f2v v = div_rn_pos2(f2v{p[j], p[j + 1]}, a.p_scale, rs_p);
          v.x = min448(v.x);  // NaN -> 448, as the scalar form
          v.y = min448(v.y);
          const int c8 = __builtin_amdgcn_cvt_pk_fp8_f32(v.x, v.y, 0, false);
          const f2v r = __builtin_amdgcn_cvt_pk_f32_fp8(c8, false) * sp2;
          p[j] = r.x;
          p[j + 1] = r.y;
        }
      } else if (PQ == 2) {
        // ---- NVFP4 P qdq: p -> V dtype -> fp32; per 16 keys (j = 8g..8g+7 of both halves)
        if constexpr (!F32) {
#pragma unroll
          for (int j = 0; j < 16; j += 2) {
            const f2v r = unpack2<T>(pack2<T>(p[j], p[j + 1]));
            p[j] = r.x;
            p[j + 1] = r.y;
          }
        }
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          float bmax = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) bmax = fmaxf(bmax, p[8 * g + i]);
          bmax = xmax32(bmax);
          float s8 = div_rn(bmax, six_gs, rs_six);
          s8 = s8 < kE4M3Max ? s8 : kE4M3Max;
          const float sc = fp8_rt(s8) * a.p_scale;
          const bool zero = sc == 0.f;
          const float safe = (zero || !(fabsf(sc) < __builtin_inff())) ? 1.f : sc;
          const float rsafe = 1.0f / safe;
          bool nan = false;
#pragma unroll
          for (int i = 0; i < 8; ++i) nan |= p[8 * g + i] != p[8 * g + i];
          // FACT: p[] gets the E2M1 values c and sblk[g] the block scale (0 for a zero scale);
          // otherwise p[] gets c * safe as the reference
          sblk[g] = zero ? 0.f : safe;
          const float cs = FACT ? 1.f : safe;
          if (!nan) {
            // p >= +0: |p| / safe rounded to E2M1 by the converter (round half to even on the
            // E2M1 grid with saturation at 6 = e2m1_mag's thresholds), two keys per convert
            const f2v sf2 = {cs, cs};
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
              const f2v q = div_rn_pos2(f2v{p[8 * g + i], p[8 * g + i + 1]}, safe, rsafe);
              const uint32_t c4 = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, q.x, q.y, 1.0f, 0);
              const auto w = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(c4, 1.0f, 0);
              const f2v r = f2v{w[0], w[1]} * sf2;
              p[8 * g + i] = zero ? 0.f : r.x;
              p[8 * g + i + 1] = zero ? 0.f : r.y;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float v = p[8 * g + i];
              const float qv = e2m1_mag(div_rn(fabsf(v), safe, rsafe)) * cs;
              p[8 * g + i] = zero ? 0.f : (v >= 0.f ? qv : -qv);
            }
          }
        }
      }
    };
    // O^T += V^T . P^T over the 32 keys of Vt
    auto pv = [&](const float (&p)[16], const float (&sblk)[2], const unsigned char *Vt) {
      if constexpr (F32PV) {
        // ---- O^T += V^T . P^T in fp32 (v_mfma_f32_32x32x2_f32): step tt pairs key crow(tt, 0)
        // (lanes 0-31) with crow(tt, 1) (lanes 32-63)
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
          const unsigned char *vrow = Vt + crow(tt, hi) * VPITCH;
#pragma unroll
          for (int d = 0; d < DB; ++d) {
            const float vv = Elem<T>::ld(*reinterpret_cast<const T *>(vrow + (32 * d + fr) * ES));
            acc[d] = __builtin_amdgcn_mfma_f32_32x32x2f32(vv, p[tt], acc[d], 0, 0, 0);
          }
        }
      } else {
        // ---- O^T += V^T . P^T with P rounded to the V dtype; k index i of half hi in k-block g
        // is key crow(8g + i, hi)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
          typedef uint32_t u4v __attribute__((ext_vector_type(4)));
          u4v w1;
#pragma unroll
          for (int i = 0; i < 8; i += 2) w1[i / 2] = pack2<T>(p[8 * g + i], p[8 * g + i + 1]);
          const v8 pb = __builtin_bit_cast(v8, w1);
#pragma unroll
          for (int d = 0; d < DB; ++d) {
            // elements 0-3: keys 16g + 4hi + 0..3, elements 4-7: keys 16g + 8 + 4hi + 0..3
            const unsigned char *base = Vt + tr_off + 16 * g * VPITCH + 64 * d;
            const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s *)(base));
            const v4s up = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) v4s *)(base + 8 * VPITCH));
            typedef uint32_t u2v __attribute__((ext_vector_type(2)));
            const u2v l2 = __builtin_bit_cast(u2v, lo), u2 = __builtin_bit_cast(u2v, up);
            const v8 vf = __builtin_bit_cast(v8, u4v{l2.x, l2.y, u2.x, u2.y});
            if constexpr (FACT) {
              f32x16 z;
#pragma unroll
              for (int e = 0; e < 16; ++e) z[e] = 0.f;
              const f32x16 part = AMma<T>::mma(vf, pb, z);
#pragma unroll
              for (int e = 0; e < 16; ++e) acc[d][e] = __builtin_fmaf(part[e], sblk[g], acc[d][e]);
              // one 16-register partial live at a time (hoisting the four MFMAs spills at D 128)
              __builtin_amdgcn_sched_barrier(0);
            } else {
              acc[d] = AMma<T>::mma(vf, pb, acc[d]);
            }
          }
        }
      }
    };
    const int kvs = t * kStage;
    f32x16 s_a, s_b;  // scores of the stage's two 32-key tiles (fixed registers, no copies)
    if (AHEAD && active && kvs < w_end) s_a = score(0);
    {
#pragma unroll
    for (int sub = 0; sub < NSUB; ++sub) {
    const int kv0 = kvs + sub * kKv;
    const unsigned char *const Vt = Vb + sub * kKv * VPITCH;
    // wave-uniform: a tile with no masked (row, key) pair skips the mask arithmetic
    const bool need_mask = kv0 + kKv > lk || (a.causal && kv0 + kKv - 1 > q0 + off);
    if (active && kv0 < w_end) {
      // tile 1's scores are issued unconditionally (keys past w_end are in LDS: zero or real
      // data, their scores unused) so no register copy or phi joins the two paths
      if (AHEAD && NSUB > 1 && sub == 0) s_b = score(1);
      const f32x16 s = !AHEAD ? score(sub) : (sub == 0 ? s_a : s_b);
      float x[16], p[16];
      const float mloc = xmax32(scale_x(s, need_mask, kv0, x));
      const float mn = fmaxf(m, mloc);
      const float mu = mn == kNegInf ? 0.f : mn;  // rows with no key yet: p = 0, not NaN
      const float ls = expsum(x, mu, p);
      const float corr = m == mn ? 1.f : __builtin_amdgcn_exp2f(m - mu);
      l = l * corr + ls;
      rescale(corr, m != mn);
      m = mn;
      float sblk[2] = {1.f, 1.f};  // NVFP4 (FACT): the two 16-key blocks' scales
      qdq(p, sblk);
      pv(p, sblk, Vt);
    }
    }
    }
    if constexpr (LD::DBUF) {
      // stage t+1 into the other buffer (last read in stage t-1, before the previous barrier),
      // then one barrier: stage t+1 visible, stage t's reads done before stage t+2 overwrites it
      if (t + 1 < nstages) swrite((t + 1) & 1);
      __syncthreads();
    } else {
      __syncthreads();
      if (t + 1 < nstages) {
        swrite(0);
        __syncthreads();
      }
    }
  }

  // ---- o = acc / max(l, 1e-6); lane holds d = 32 d + crow(e, hi) of query row qrow
  if constexpr (!F32 && DP == D && !FACT) {
    // 16-bit output, d blocks of 32, staged through the K image (free: every wave passed the
    // last stage's barrier) so it leaves as whole rows.  Lane hi = 0 holds columns 8k .. 8k+3 of
    // its row and its partner (hi = 1) 8k+4 .. 8k+7, k = 4 d + e4; one v_permlane32_swap per
    // dword of the groups (k, k+1) gives the low half columns 8k .. 8k+7 and the high half
    // 8k+8 .. 8k+15 (guide T21), written as ds_write_b128 into this wave's 32 rows at the K pitch
    // (conflict-free); read back 16 B per lane, CR chunks of a row on consecutive lanes, and
    // stored with 64 / CR whole rows per instruction.  Per-lane row stores at the row stride
    // (16 dwordx2, 32-64 rows each) made the epilogue ~4.5 k cycles per pass (r06 stamps,
    // scripts/exp/bench_attn_exp.py): store-issue bound.
    if (!active) return;  // wave-uniform
    unsigned char *const ob = Ks + wave * 32 * PITCH;
    if (qrow < lq) {
      const float den = l > 1e-6f ? l : 1e-6f;
      const float rden = 1.0f / den;
      const f2v sv = {den, den}, rv = {rden, rden};
#pragma unroll
      for (int k = 0; k < 4 * DB; k += 2) {  // 8-column groups k, k + 1 (one pair live at a time)
        uint32_t w[2][2];
#pragma unroll
        for (int g = 0; g < 2; ++g)
#pragma unroll
          for (int i = 0; i < 4; i += 2) {  // div_rn on packed pairs (same ops, same copysign)
            const int d = (k + g) >> 2, e = 4 * ((k + g) & 3) + i;
            const f2v qv = {acc[d][e], acc[d][e + 1]};
            const f2v y0 = qv * rv;
            const f2v y = __builtin_elementwise_fma(__builtin_elementwise_fma(-y0, sv, qv), rv, y0);
            // both halves in one v_cvt_pk (RNE, as Elem<T>::st twice; no shift / or)
            w[g][i / 2] = pack2<T>(__builtin_copysignf(y.x, qv.x), __builtin_copysignf(y.y, qv.y));
          }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const auto r = __builtin_amdgcn_permlane32_swap(w[0][j], w[1][j], false, false);
          w[0][j] = r[0];
          w[1][j] = r[1];
        }
        *reinterpret_cast<uint4 *>(ob + fr * PITCH + 16 * k + 16 * hi) = make_uint4(w[0][0], w[0][1], w[1][0], w[1][1]);
      }
    }
#pragma unroll
    for (int c = lane; c < 32 * CR; c += 64) {  // 32 * CR is a multiple of 64 (D % 16 == 0)
      const int row = c / CR, ch = c - row * CR;
      const uint4 v = *reinterpret_cast<const uint4 *>(ob + row * PITCH + ch * 16);
      if (q0 + row < lq) *reinterpret_cast<uint4 *>(O + (int64_t)(q0 + row) * a.ot + ch * EC) = v;
    }
    return;
  }
  if (active && qrow < lq) {
    const float den = l > 1e-6f ? l : 1e-6f;
    const float rden = 1.0f / den;
    T *orow = O + (int64_t)qrow * a.ot;
#pragma unroll
    for (int d = 0; d < DB; ++d)
#pragma unroll
      for (int e4 = 0; e4 < 4; ++e4) {
        if (DP != D && 32 * d + 8 * e4 + 4 * hi >= D) continue;
        struct alignas(4 * sizeof(T)) Pack {
          T h[4];
        } pk;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {  // div_rn on packed pairs (same ops, same copysign)
          const f2v sv = {den, den}, rv = {rden, rden};
          const f2v qv = {acc[d][4 * e4 + i], acc[d][4 * e4 + i + 1]};
          const f2v y0 = qv * rv;
          const f2v y = __builtin_elementwise_fma(__builtin_elementwise_fma(-y0, sv, qv), rv, y0);
          pk.h[i] = Elem<T>::st(__builtin_copysignf(y.x, qv.x));
          pk.h[i + 1] = Elem<T>::st(__builtin_copysignf(y.y, qv.y));
        }
        *reinterpret_cast<Pack *>(orow + 32 * d + 8 * e4 + 4 * hi) = pk;
      }
  }
}

// A workgroup runs ppw pairs of query tiles of one (batch, head), each the longest and the
// shortest causal tile of a pair (tiles_q - 1 - p, then p), so every workgroup does the same work
// and the grid has no long-tile tail (r02 ran one tile per workgroup, longest first: 1:tiles_q
// work spread).  ppw = 1 (two pairs per workgroup measured no faster, profiles/r03/attention/ppw_ab).
template <typename T, int D, int PQ, int kStage>
__global__ __launch_bounds__(kThreads, 2) void attn_fwd_kernel(AttnArgs a) {  // >= 2 waves / SIMD
  using L = AttnLds<T, D, PQ, kStage>;
  __shared__ __attribute__((aligned(16))) unsigned char Ks[L::NBUF * L::KIMG];
  __shared__ __attribute__((aligned(16))) unsigned char Vs[L::NBUF * L::VIMG];
  // XCD-contiguous remap (bijective): consecutive ids share an XCD, hence its L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int qn = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  int rem = (xcd < rr ? xcd * (qn + 1) : rr * (qn + 1) + (xcd - rr) * qn) + orig / 8;
  const int npair = (a.tiles_q + 1) / 2;
  const int ngrp = (npair + a.ppw - 1) / a.ppw;  // pair groups of a (batch, head)
  const int pg = rem % ngrp;
  rem /= ngrp;
  const int hg = rem % a.group;
  rem /= a.group;
  const int kvh = rem % a.hkv;
  const int b = rem / a.hkv;
  const int h = kvh * a.group + hg;
  const int p_end = (pg + 1) * a.ppw < npair ? (pg + 1) * a.ppw : npair;
  for (int pr = pg * a.ppw; pr < p_end; ++pr) {
    const int t_long = a.tiles_q - 1 - pr;
    if (pr > pg * a.ppw) __syncthreads();  // the LDS images are re-staged
    attn_tile<T, D, PQ, kStage>(a, b, h, kvh, t_long, Ks, Vs);
    if (pr < t_long) {  // odd tiles_q: the middle tile runs once
      __syncthreads();
      attn_tile<T, D, PQ, kStage>(a, b, h, kvh, pr, Ks, Vs);
    }
  }
}

template <typename T, int D, int ST>
void launch_st(const AttnArgs &a, unsigned grid, int mode, hipStream_t stream) {
  if (mode == 0)
    attn_fwd_kernel<T, D, 0, ST><<<grid, kThreads, 0, stream>>>(a);
  else if (mode == 1)
    attn_fwd_kernel<T, D, 1, ST><<<grid, kThreads, 0, stream>>>(a);
  else
    attn_fwd_kernel<T, D, 2, ST><<<grid, kThreads, 0, stream>>>(a);
}

// 64 keys per LDS stage (32-key stages at 3 waves / SIMD measured slower: 0.104 vs 0.090 ms,
// profiles/r03/attention/stage_ab)
template <typename T, int D>
int launch_d(const AttnArgs &a, unsigned grid, int mode, hipStream_t stream) {
  launch_st<T, D, 64>(a, grid, mode, stream);
  return host_check_launch();
}

template <typename T>
int launch_t(const AttnArgs &a, unsigned grid, int d, int mode, hipStream_t stream) {
  switch (d) {
  case 16: return launch_d<T, 16>(a, grid, mode, stream);
  case 32: return launch_d<T, 32>(a, grid, mode, stream);
  case 64: return launch_d<T, 64>(a, grid, mode, stream);
  case 96: return launch_d<T, 96>(a, grid, mode, stream);
  case 128: return launch_d<T, 128>(a, grid, mode, stream);
  default: return MTQ_ERR_INVALID_ARG;
  }
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int mtq_attention_fwd(const void *q, const void *k, const void *v, void *o,
                                 const int32_t *b_start_loc, const int32_t *b_seq_len,
                                 const int32_t *b_start_loc_k, const int32_t *b_seq_len_k, int batch,
                                 int max_len_q, int num_q_heads, int num_kv_heads, int head_dim,
                                 const int64_t *strides, int is_causal, double softmax_scale,
                                 int p_qdq_mode, double p_qdq_scale, int dtype, hipStream_t stream) {
  if (!q || !k || !v || !o || !b_start_loc || !b_seq_len || !b_start_loc_k || !b_seq_len_k || !strides)
    return MTQ_ERR_INVALID_ARG;
  if (dtype != MTQ_BF16 && dtype != MTQ_F16 && dtype != MTQ_F32) return MTQ_ERR_DTYPE;
  if (batch < 1 || max_len_q < 0 || num_q_heads < 1 || num_kv_heads < 1 || num_q_heads % num_kv_heads)
    return MTQ_ERR_INVALID_ARG;
  if (head_dim != 16 && head_dim != 32 && head_dim != 64 && head_dim != 96 && head_dim != 128)
    return MTQ_ERR_INVALID_ARG;
  if (p_qdq_mode < 0 || p_qdq_mode > 2) return MTQ_ERR_FORMAT;
  if (p_qdq_mode && !(p_qdq_scale > 0.0 && p_qdq_scale < 3.4e38)) return MTQ_ERR_INVALID_ARG;
  if (!al16(q) || !al16(k) || !al16(v) || !al16(o)) return MTQ_ERR_INVALID_ARG;
  const int64_t ec = dtype == MTQ_F32 ? 4 : 8;  // elements per 16 bytes
  for (int i = 0; i < 12; ++i)  // 16-byte aligned rows: every stride a multiple of 16 bytes
    if (strides[i] < 0 || strides[i] % ec) return MTQ_ERR_INVALID_ARG;
  // K/V rows are staged by buffer loads bounded per 64-key stage: token rows must not overlap
  // (token stride >= head_dim) and a stage's span must fit a 31-bit buffer offset
  const int64_t esz = dtype == MTQ_F32 ? 4 : 2;
  if (strides[4] < head_dim || strides[7] < head_dim) return MTQ_ERR_INVALID_ARG;
  if (strides[4] * esz * 64 >= (1ll << 31) || strides[7] * esz * 64 >= (1ll << 31)) return MTQ_ERR_INVALID_ARG;
  if (max_len_q == 0) return MTQ_OK;
  const int64_t tiles_q = (max_len_q + kRowsPerBlock - 1) / kRowsPerBlock;
  // one pair of query tiles (the longest and the shortest causal tile) per workgroup
  const int64_t npair = (tiles_q + 1) / 2;
  const int ppw = 1;
  const int64_t blocks = (npair + ppw - 1) / ppw * num_q_heads * (int64_t)batch;
  if (blocks > (int64_t)INT32_MAX) return MTQ_ERR_INVALID_ARG;
  AttnArgs a;
  a.q = q, a.k = k, a.v = v, a.o = o;
  a.start_q = b_start_loc, a.len_q = b_seq_len, a.start_k = b_start_loc_k, a.len_k = b_seq_len_k;
  a.qb = strides[0], a.qt = strides[1], a.qh = strides[2];
  a.kb = strides[3], a.kt = strides[4], a.kh = strides[5];
  a.vb = strides[6], a.vt = strides[7], a.vh = strides[8];
  a.ob = strides[9], a.ot = strides[10], a.oh = strides[11];
  a.hkv = num_kv_heads;
  a.group = num_q_heads / num_kv_heads;
  a.tiles_q = (int)tiles_q;
  a.causal = is_causal ? 1 : 0;
  a.ppw = ppw;
  // triton_fa.py:922 `qk_scale = sm_scale * LOG2E` in Python (double), passed as an fp32 scalar
  a.qk_scale = (float)(softmax_scale * 1.44269504088896);
  a.p_scale = (float)p_qdq_scale;
  if (dtype == MTQ_BF16) return launch_t<__bf16>(a, (unsigned)blocks, head_dim, p_qdq_mode, stream);
  if (dtype == MTQ_F16) return launch_t<_Float16>(a, (unsigned)blocks, head_dim, p_qdq_mode, stream);
  return launch_t<float>(a, (unsigned)blocks, head_dim, p_qdq_mode, stream);
}
