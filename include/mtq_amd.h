/*
 * mtq_amd.h — C ABI of the MI355X-native (gfx950 / CDNA4) fake-quantization and
 * calibration kernels (libmtq_amd.so).
 *
 * This is the drop-in boundary for the hot path of ModelOpt's PTQ fake quantization
 * (`modelopt.torch.quantization`).  Every entry point here replaces one function of the
 * reference's native extension ABI (pybind modules modelopt_cuda_ext / _fp8 / _mx built by
 * modelopt/torch/quantization/extensions.py:28-72) or one ATen reduction the reference's
 * Python layer issues on the hot path.  Reference citations are relative to the reference
 * repository root.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch types.  All tensors are dense, contiguous and
 *     device-resident (HBM).  `x` and `y` may alias (in-place, as fake_tensor_quant_).
 *   - Element dtype codes: MTQ_F32, MTQ_F16, MTQ_BF16, MTQ_F64.  All arithmetic is fp32
 *     (the reference casts to float in every kernel and in its ATen fallback).
 *   - `amax` pointers may be any of the dtype codes (`amax_dtype`), converted to fp32 on
 *     load (reference: `amax.to(at::ScalarType::Float)`, tensor_quant_gpu.cu:84).
 *   - Every launcher takes an explicit hipStream_t (reference kernels use
 *     c10::cuda::getCurrentCUDAStream(), tensor_quant_gpu.cu:79).  Launchers never
 *     synchronise, never allocate, and are safe to capture in a hipGraph.
 *   - Return value: MTQ_OK (0) or a negative MTQ_ERR_* code; nothing throws across the ABI
 *     (the reference raises TORCH_CHECK / std::invalid_argument, tensor_quant_mx.cu:337).
 */
#ifndef MTQ_AMD_H_
#define MTQ_AMD_H_

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- dtype / format / status codes -------------------------------------------------- */
enum mtq_dtype { MTQ_F32 = 0, MTQ_F16 = 1, MTQ_BF16 = 2, MTQ_F64 = 3 };

/* Element / scale formats.  Same order and names as the reference's `enum class Types`
 * (modelopt/torch/kernels/quantization/gemm/tensor_quant_mx.h:38). */
enum mtq_format {
  MTQ_E4M3 = 0, MTQ_E5M2 = 1, MTQ_INT8 = 2, MTQ_E0M3 = 3, MTQ_E1M2 = 4,
  MTQ_E3M0 = 5, MTQ_E2M1 = 6, MTQ_E3M2 = 7, MTQ_E2M3 = 8, MTQ_E8M0 = 9
};

enum mtq_status {
  MTQ_OK = 0,
  MTQ_ERR_INVALID_ARG = -1,
  MTQ_ERR_DTYPE = -2,
  MTQ_ERR_BLOCKSIZE = -3, /* reference: "Blocksize for fused call must be one of {8, 16, 32}" */
  MTQ_ERR_FORMAT = -4,
  MTQ_ERR_LAUNCH = -5,    /* hipGetLastError() after launch; see mtq_last_hip_error() */
  MTQ_ERR_NO_DEVICE = -6
};

/* Human-readable message for a status code (static storage). */
const char *mtq_status_string(int status);
/* hipError_t of the most recent failing launch on this thread (0 if none). */
int mtq_last_hip_error(void);
/* Library version: major*10000 + minor*100 + patch. */
int mtq_version(void);

/* ---- INT-n fake quant ----------------------------------------------------------------
 * y = clamp(rint(x * s), min_bound, max_bound) / s,  s = max_bound / amax (fp32),
 * max_bound = 2^(num_bits-1+unsigned) - 1, min_bound = 0 | -max_bound | -max_bound-1
 * (unsigned | narrow_range | full); amax <= 2^-24 quantizes to (signed) zero.
 * Bit-exact with the reference's ATen path `_tensor_quant`
 * (modelopt/torch/quantization/tensor_quant.py:607-645).
 *
 * mtq_fake_tensor_quant replaces `fake_tensor_quant` / `fake_tensor_quant_`
 * (tensor_quant.cpp:39-56 -> tensor_quant_gpu.cu:59-98): per-tensor, amax has 1 element. */
int mtq_fake_tensor_quant(const void *x, void *y, int64_t n, int dtype, const void *amax,
                          int amax_dtype, int num_bits, int is_unsigned, int narrow_range,
                          hipStream_t stream);

/* Replaces `fake_tensor_quant_with_axis` (tensor_quant.cpp:58-64 ->
 * tensor_quant_gpu.cu:100-140): channel of element i is (i / inner) % axis_size where
 * inner = stride(axis) of the contiguous input; amax has axis_size elements.  Also the
 * static block-quant path (input reshaped to (-1, block) with axis 0,
 * tensor_quantizer.py:975-1061). */
int mtq_fake_tensor_quant_with_axis(const void *x, void *y, int64_t n, int dtype,
                                    const void *amax, int amax_dtype, int64_t axis_size,
                                    int64_t inner, int num_bits, int is_unsigned,
                                    int narrow_range, hipStream_t stream);

/* ---- FP8 E4M3 fake quant ---------------------------------------------------------------
 * safe = amax <= 2^-24 ? 1 : amax; s = RN(RN(1/safe) * 448) (Python `448.0 / t` is
 * t.reciprocal() * 448); inv = 1/s;
 * y = fp32(e4m3_rne(clamp(x*s, -448, 448))) * inv   (gfx950 v_cvt_pk_fp8_f32, OCP e4m3fn).
 * Bit-exact with `_fp8_eager` (tensor_quant.py:46-59).
 * Replaces `fake_e4m3fy` (tensor_quant_gpu_fp8.cu:90-107). */
int mtq_fake_e4m3fy(const void *x, void *y, int64_t n, int dtype, const void *amax,
                    int amax_dtype, hipStream_t stream);
/* Replaces `fake_e4m3fy_with_axis` (tensor_quant_gpu_fp8.cu:66-88); also the FP8 static
 * block path (amax [rows*K/block, 1] on the (-1, block) view). */
int mtq_fake_e4m3fy_with_axis(const void *x, void *y, int64_t n, int dtype, const void *amax,
                              int amax_dtype, int64_t axis_size, int64_t inner,
                              hipStream_t stream);

/* Unscaled e4m3 round trip, `_fp8_eager(x, amax=None)` (tensor_quant.py:55-59): torch's
 * float8_e4m3fn cast, RNE, |x| > 464 (incl. inf) -> NaN (no saturation). */
int mtq_e4m3_cast(const void *x, void *y, int64_t n, int dtype, hipStream_t stream);

/* ---- dynamic block (MX) fake quant -------------------------------------------------------
 * Replaces `fused_amax_convert` (tensor_quant_mx.cu:316-352 -> amax_and_convert_kernel
 * :239-294).  Input viewed as [rows, cols] (cols = last dim); blocks of block_size along
 * cols (a partial last block is zero-padded); per block amax = max|x| (inf clamps to
 * FLT_MAX), scale from `scale_format` (E8M0 = the reference's NV rounding, :104-137;
 * otherwise :139-183 in double), y = sign * convert(|x| * scale, format) * unscale.
 * global_amax may be NULL; with per_channel != 0 it holds one fp32 value per row. */
int mtq_fused_amax_convert(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                           int block_size, int format, int scale_format,
                           const float *global_amax, int per_channel, hipStream_t stream);

/* Host-side scalar conversion (reference `convert_to_exmy`, tensor_quant_mx.cu:399 ->
 * convert_to_types, tensor_quant_mx.h:161-188). */
float mtq_convert_to_exmy(float x, int format);

/* ---- amax reductions ---------------------------------------------------------------------
 * Accumulating max|x| reduction: out[k] = max(out[k], max_{p,q} |x[p, k, q]|) for x viewed
 * as [P, K, Q] (dense).  NaN anywhere in a reduced set makes out[k] NaN (torch.max
 * semantics).  `out` is fp32 and must be initialised by the caller (0 for a fresh
 * reduction); accumulation across calls implements MaxCalibrator.collect's running max
 * (calib/max.py:53-86 over reduce_amax, utils/core_utils.py:146-183) in one launch,
 * without the reference's two passes (max, min) and host-syncing asserts. */
int mtq_reduce_amax(const void *x, int64_t P, int64_t K, int64_t Q, int dtype, float *out,
                    hipStream_t stream);

/* Calibration bookkeeping on the running-max buffers, in this library so that a calibration
 * pass launches no kernel the model's own forward has not already loaded (the first launch of a
 * kernel from another code object stalls the host for tens to hundreds of ms on the GPU box,
 * DESIGN §4 "First-use stalls"):
 *  mtq_amax_fill:  out[i] = value for i < n (0 starts a running max).
 *  mtq_amax_fold:  dst[i] = max(dst[i], src[i]) for fp32 running maxima of |x| (NaN propagates,
 *                  as torch.maximum); the shared-collect fold of MaxCalibrator (calib/max.py).
 *  mtq_amax_check: flags[0] = any NaN, flags[1] = any +-inf, flags[2] = any value < 0 over the
 *                  n elements of x (fp32 / bf16 / f16), written by one workgroup (no prior
 *                  zeroing): the reference's per-collect asserts (calib/max.py:69-77) and
 *                  validate_attr checks (tensor_quantizer.py:757-773) batched over many
 *                  quantizers; flags is int32[3] device memory. */
int mtq_amax_fill(float *out, int64_t n, float value, hipStream_t stream);
int mtq_amax_fold(float *dst, const float *src, int64_t n, hipStream_t stream);
int mtq_amax_check(const void *x, int64_t n, int dtype, int32_t *flags, hipStream_t stream);

/* MoE shared input quantizer (huggingface.py _QuantFusedExperts, the once-per-layer form of the
 * reference's per-expert input quantizer calls, plugins/huggingface.py:976-1115): y[r, :] = x[r, :]
 * when any of row r's k expert indices (idx int64 [rows, k]) lies in [0, num_experts), else +0
 * (rows routed to no local expert, e.g. expert-parallel sentinels).  x, y [rows, cols] of dtype. */
int mtq_mask_unrouted_rows(const void *x, void *y, const int64_t *idx, int64_t rows, int64_t cols, int k,
                           int64_t num_experts, int dtype, hipStream_t stream);

/* Fused dynamic INT-n block quant with in-kernel block amax and an optional per-column
 * pre-quant scale:  t = T(x * pqs[col]) (rounded to the input dtype, as the reference's
 * `inputs * pre_quant_scale`, tensor_quantizer.py:1143-1144), per block of `block` along
 * cols amax = max|t|, y = INT-n qdq(t, amax).  One HBM pass; this is the weight side of the
 * AWQ-lite alpha search (model_calib.py:1540-1553) where the reference issues a multiply,
 * two reductions and the qdq per alpha.  pqs may be NULL (no scaling); pqs_dtype as dtype. */
int mtq_block_quant_dynamic(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                            const void *pqs, int pqs_dtype, int block, int num_bits,
                            int is_unsigned, int narrow_range, hipStream_t stream);

/* ---- histogram ---------------------------------------------------------------------------
 * torch.histc(|x|, bins, min=0, max=*hmax) semantics (as used by HistogramCalibrator.collect,
 * calib/histogram.py:108-130): bin = (int)((|x| * bins) / max) in fp32 (multiply, then
 * divide), |x| == max -> last bin, |x| > max or NaN dropped; max == 0 widens the range to
 * [-1, 1] like histc; skip_zeros drops exact zeros (calib/histogram.py:105-106).  Counts are
 * accumulated into
 * `counts` (uint32, caller-initialised) so repeated calls sum.  `hmax` is a device fp32
 * scalar (no host sync). */
int mtq_histogram_abs(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                      int skip_zeros, uint32_t *counts, hipStream_t stream);

/* torch.histc's CPU accumulation for calls above 2^24 elements (calib/histogram.py:116-130 ->
 * torch.histc -> at::parallel_for): element chunk c is [bounds[c], bounds[c+1]) (device int64
 * [chunks + 1], e.g. the skip_zeros boundaries mapped back to the input), or, with bounds null,
 * [c * chunk_elems, min((c + 1) * chunk_elems, n)).  Two launches: the chunks are counted exactly
 * by a fixed number of workgroups each, every workgroup storing its bin row into `scratch` (uint32
 * [scratch_words >= mtq_histogram_chunked_scratch_words(n, chunks, bins)], contents irrelevant,
 * overwritten), then hist[b] = sum_c min(fp32(count_c[b]), 2^24) in chunk order, + accum[b] for
 * b < accum_n (the calibrator's running histogram, calib/histogram.py:127; accum may alias hist;
 * accum_n 0 = none) (fp32 [bins], overwritten).
 * bf16 / f16 only, x 16-byte aligned, n % 8 == 0, bins <= 8192 (MTQ_ERR_DTYPE /
 * MTQ_ERR_INVALID_ARG otherwise: the caller counts chunk by chunk with mtq_histogram_abs). */
int64_t mtq_histogram_chunked_scratch_words(int64_t n, int chunks, int bins);
int mtq_histogram_abs_chunked(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                              int skip_zeros, const int64_t *bounds, int64_t chunk_elems, int chunks,
                              uint32_t *scratch, int64_t scratch_words, const float *accum, int64_t accum_n,
                              float *hist, hipStream_t stream);

/* torch.histc of the non-zero |x| with skip_zeros (calib/histogram.py:105-130: `x[x != 0]`, then
 * torch.histc's per-thread fp32 chunk counts), in ONE read of x and no host sync: the N non-zero
 * elements form at::parallel_for chunks -- T' = min(threads, ceil(N / grain)), chunk = ceil(N / T'),
 * chunk t = non-zero ranks [t * chunk, (t + 1) * chunk) (grain = at::internal::GRAIN_SIZE =
 * 32768) -- each counted exactly, clamped at 2^24 and added in chunk order in fp32, + accum[b]
 * for b < accum_n; hist fp32 [bins].  Zero = |x| bit pattern 0 (+0 and -0); NaN is non-zero (it
 * takes a rank, no bin).  bf16 / f16, x 16-byte aligned, n % 8 == 0, threads <= 1024, bins <=
 * 8176 (MTQ_ERR_INVALID_ARG otherwise; n == 0 writes accum / zeros without reading x).  scratch:
 * uint32 [mtq_histogram_nonzero_scratch_words(n, threads, bins)], contents irrelevant.
 * Replaces the r05 mtq_histogram_nonzero_bounds (boundaries by a second read of x). */
int64_t mtq_histogram_nonzero_scratch_words(int64_t n, int threads, int bins);
int mtq_histogram_abs_nonzero_chunked(const void *x, int64_t n, int dtype, const float *hmax, int bins,
                                      int threads, int64_t grain, uint32_t *scratch, int64_t scratch_words,
                                      const float *accum, int64_t accum_n, float *hist, hipStream_t stream);

/* ---- NVFP4 --------------------------------------------------------------------------------
 * Two-level dynamic NVFP4 fake quant of x [rows, cols] (blocks of block_size along cols, zero
 * padded): the reference's primary NVFP4 kernel, fp4_fake_quant_block
 * (kernels/quantization/gemm/fp4_kernel_hopper.py:102-160, dispatched from
 * tensor_quant.py:173-181 for num_bits (2,1) / scale_bits (4,3)).  global_amax is a device fp32
 * scalar; per block the FP8-E4M3-quantised scale q = e4m3(min(bmax / (6 gs), 448)) * gs with
 * gs = global_amax / 2688, then y = sign(x) * e2m1(|x| / q) * q.  block_size in {8, 16, 32}
 * (the reference always passes its default, 16). */
int mtq_nvfp4_fake_quant(const void *x, void *y, int64_t rows, int64_t cols, int dtype,
                         const float *global_amax, int block_size, hipStream_t stream);

/* Static NVFP4 element pass: x viewed as [nblocks, block] with one precomputed fp32 scale per
 * block (already FP8-quantised by the caller): y = sign(x) * e2m1(|x| / s) * s, a zero scale gives
 * a block of +0, a NaN/inf scale acts as 1 -- static_blockwise_fp4_fake_quant's kernel
 * (kernels/quantization/gemm/fp4_kernel.py:193-214, nvfp4_scalar_quant in
 * common/nvfp4_quant.py).  The per-block scale math (compute_fp4_scales, fp4_kernel.py:217-251)
 * is a few small device ops on the host side. */
int mtq_fp4_block_scale_quant(const void *x, void *y, int64_t nblocks, int block, int dtype,
                              const float *scales, hipStream_t stream);

/* ---- QuantLinear simulated GEMM, short inputs (MFMA) ---------------------------------------
 * Replaces, for M <= 16 input rows, the fake-quantised linear of the reference
 * (nn/modules/quant_module.py:257-278 QuantLinearConvBase.forward + quant_linear.py:38-53:
 * F.linear(x, weight_quantizer(W), b)) with one kernel that applies the weight fake quant to the
 * MFMA operands in registers: y[M, N] = x[M, K] . qdq(W)[N, K]^T (+ bias[N]), dtype bf16 or f16
 * (x, W, bias, y alike), fp32 accumulation (v_mfma_f32_16x16x32), one rounding of y.
 * qdq(W): kind 0 = INT-n (num_bits, is_unsigned, narrow_range; as mtq_fake_tensor_quant_with_axis),
 * kind 1 = FP8 e4m3 (as mtq_fake_e4m3fy_with_axis); amax_numel == 1 per tensor, else one amax per
 * `block` consecutive elements of row-major W (block == K: per output channel; block % 32 == 0).
 * Requires N % 16 == 0, K % 32 == 0, 16-byte aligned x and W; bias may be NULL. */
int mtq_qlinear_small_m(const void *x, const void *w, const void *bias, void *y, int64_t M,
                        int64_t N, int64_t K, int dtype, const void *amax, int amax_dtype,
                        int64_t amax_numel, int64_t block, int kind, int num_bits,
                        int is_unsigned, int narrow_range, hipStream_t stream);
/* The same with a caller-owned workspace for split-K: `ws` (16-byte aligned, at least
 * mtq_qlinear_small_m_workspace_bytes(M, N, K) bytes, 0 when the shape does not split) holds fp32
 * partial tiles; the chunks are summed in a fixed order, so results are deterministic.  With
 * ws == NULL (or mtq_qlinear_small_m) K is not split: a launch has N/16 waves.  The streaming
 * kernel takes fp32 amax; other amax dtypes and blocks that do not line up with its 128-column
 * batches (e.g. block 96) run the workgroup-per-tile kernel. */
size_t mtq_qlinear_small_m_workspace_bytes(int64_t M, int64_t N, int64_t K);
int mtq_qlinear_small_m_ws(const void *x, const void *w, const void *bias, void *y, int64_t M,
                           int64_t N, int64_t K, int dtype, const void *amax, int amax_dtype,
                           int64_t amax_numel, int64_t block, int kind, int num_bits,
                           int is_unsigned, int narrow_range, void *ws, size_t ws_bytes,
                           hipStream_t stream);

/* Up to 4 short-input linears of the same M and K in ONE launch (the q/k/v projections of a decode
 * step, each reading the same hidden state through its own input quantizer): problem i computes
 * y_i[M, N_i] = x_i . qdq_i(W_i)^T (+ bias_i) exactly as mtq_qlinear_small_m_ws would (same qdq,
 * same per-linear split-K chunk order for a given split), the units of all linears sharing one
 * grid.  Linears that cannot share a launch (different `kind` or amax class, non-fp32 amax, blocks
 * not aligned to the stream kernel's batches) run one after another.  Reference: the separate
 * k_proj / v_proj (q_proj) forwards of an HF attention module, each the QuantLinear forward of
 * nn/modules/quant_module.py:257-278.  `ws`: mtq_qlinear_small_m_group_workspace_bytes bytes. */
typedef struct {
  const void *x;
  const void *w;
  const void *bias;
  void *y;
  int64_t N;
  const void *amax;
  int amax_dtype;
  int64_t amax_numel;
  int64_t block;
  int kind;
  int num_bits;
  int is_unsigned;
  int narrow_range;
} mtq_qlinear_problem;
size_t mtq_qlinear_small_m_group_workspace_bytes(int64_t M, const int64_t *N, int n, int64_t K);
int mtq_qlinear_small_m_group(const mtq_qlinear_problem *problems, int n, int64_t M, int64_t K,
                              int dtype, void *ws, size_t ws_bytes, hipStream_t stream);

/* FP8 (E4M3) bytes of a [rows, cols] weight with 2D block scales: y = e4m3(x / scale[r / block_rows,
 * c / block_cols]) (FP8QTensor.quantize(w, s, block_sizes={-1: bc, -2: br}),
 * qtensor/fp8_tensor.py:40-117; the FP8_PB_WO export, export/quant_utils.py:874-877): the fp32
 * quotient, or with round_to_dtype the quotient rounded to the weight's 16-bit dtype first (a
 * scale tensor in the weight's own dtype: torch divides in that dtype).  scale: fp32 values
 * [ceil(rows / block_rows), ceil(cols / block_cols)] contiguous; cols and block_cols multiples of
 * the 16-byte vector (8 bf16 / f16, 4 fp32), x 16-byte aligned (MTQ_ERR_INVALID_ARG otherwise). */
int mtq_export_fp8_block2d(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype, const float *scale,
                           int64_t block_rows, int64_t block_cols, int round_to_dtype, hipStream_t stream);

/* ---- checkpoint export (real-quant packing) ----------------------------------------------
 * export/quant_utils.py:836-938 to_quantized_weight and the qtensor quantize() routines; weights
 * [rows, cols] row-major of dtype, outputs raw bytes.
 *  mtq_export_fp8:   y = e4m3(w / scale) as torch's float8_e4m3fn cast (RNE, |v| > 464 -> NaN);
 *                    per_row: scale[rows] (fp32 quotient), else scale[0] with the quotient first
 *                    rounded to dtype when round_to_dtype (bf16 / 0-dim fp32 stays bf16 in torch).
 *  mtq_export_int4:  pack_int4_in_uint8 (:792-833): q = clamp(rint(w / scale[r, c/block]), -8, 7),
 *                    rows 2i and 2i+1 share byte y[i, c] (low nibble = even row); rows even.
 *  mtq_export_nvfp4: NVFP4QTensor.quantize (qtensor/nvfp4_tensor.py:253-342): code of
 *                    w / (block_scale[r, c/block] * scale_2[0]) (E2M1 RNE, sign bit), columns 2j
 *                    and 2j+1 share y[r, j] (low = even); block_scale holds the fp8 scales as fp32.
 *  mtq_export_mxfp4: MXFP4QTensor.quantize (qtensor/mxfp4_tensor.py:38-81): per `block` elements
 *                    an E8M0 exponent byte in scales[n/block] and packed codes in y[n/2]. */
int mtq_export_fp8(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                   const float *scale, int per_row, int round_to_dtype, hipStream_t stream);
int mtq_export_int4(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                    const float *scale, int block, hipStream_t stream);
int mtq_export_nvfp4(const void *x, uint8_t *y, int64_t rows, int64_t cols, int dtype,
                     const float *block_scale, const float *scale_2, int block,
                     hipStream_t stream);
int mtq_export_mxfp4(const void *x, uint8_t *y, uint8_t *scales, int64_t n, int dtype, int block,
                     hipStream_t stream);
/* MXFP8QTensor.quantize (qtensor/mxfp8_tensor.py:163-187; the MXFP8 branch of the unified export,
 * export/unified_export_hf.py:671-680 + quant_utils.py:309-310, 871-872): x bf16/f16 with
 * n % 32 == 0, blocks of 32 consecutive elements; y n e4m3 bytes, scales n/32 E8M0 bytes. */
int mtq_export_mxfp8(const void *x, uint8_t *y, uint8_t *scales, int64_t n, int dtype,
                     hipStream_t stream);

/* ---- AWQ-lite search helpers ---------------------------------------------------------------
 * loss[0] += mean(float(T(a - b))^2) over n elements of dtype T: the per-alpha search loss
 * `(out - out_act).float().pow(2).mean()` (model_calib.py:1494) in one read of a and b
 * (reference: 4 ATen passes with an fp32 intermediate).  The difference is rounded to T before
 * squaring as the reference's T-typed subtraction does; the sum is fp32 per lane, double across
 * blocks, and deterministic for a given n on a given device (fixed grid, fixed final order).
 * `workspace` holds mtq_mse_workspace_floats(n, dtype) floats (word 0 a completion counter, then
 * one partial per block), zero-filled once before first
 * use (the kernel leaves it reusable); one workspace per concurrently used stream. */
int64_t mtq_mse_workspace_floats(int64_t n, int dtype);
int mtq_mse_accumulate(const void *a, const void *b, int64_t n, int dtype, float *loss,
                       float *workspace, int64_t workspace_floats, hipStream_t stream);

/* y[r, c] = T(x[r, c] * scale[c]) -- the input side of the AWQ-lite search, `inputs *
 * pre_quant_scale` (tensor_quantizer.py:1143-1144 via model_calib.py:1547); x, y [rows, cols]
 * contiguous, scale [cols], all of dtype T; cols a multiple of 16 B / sizeof(T). */
int mtq_mul_cols(const void *x, const void *scale, void *y, int64_t rows, int64_t cols, int dtype,
                 hipStream_t stream);

/* ---- calibration searches (csrc/mtq_search.hip) ---------------------------------------------
 *  mtq_nvfp4_fp8_scale_sweep: NVFP4MSECalibrator's fused FP8-scale sweep
 *    (kernels/quantization/gemm/nvfp4_fp8_sweep.py:62-160 `nvfp4_fp8_scale_sweep`, called from
 *    calib/mse.py:267-287): x [n_blocks, block] (block 8/16/32), per block the candidate c of
 *    `candidates` (the 126 E4M3 values / 448) minimising sum(|w| - e2m1(|w|/s)*s)^2 with
 *    s = RN(RN(c*g)/6); best_amax[b] = RN(g * c_best) (fp32), g = *global_amax.
 *  mtq_mse_sweep: MseCalibrator.collect (calib/mse.py:82-125) of one tensor with every candidate
 *    at once: x [rows, cols] (the calibrator's fp32 view; any float dtype, read exactly),
 *    amax [rows] (amax_per_row) or [1]; candidate amax = amax * c, rounded to amax_dtype when
 *    round_candidate_amax (torch promotion of a dimensioned amax), quantised as the INT-n
 *    (num_bits >= 1) or E4M3 (num_bits == 0) fake-quant kernels do;
 *    loss[k, r] = sum_c (x - xq)^2.  Rows longer than 128 need a workspace of
 *    mtq_mse_sweep_workspace_floats(rows, cols, n_candidates) floats (no zero-fill needed).
 *  mtq_awq_clip_search: the block branch of awq_clip's `_clip_search` (model_calib.py:1815-1882)
 *    for static-block INT-n weights: w [co, cols] (zero-padded to a multiple of block),
 *    x [n_tokens, cols] fp32 (the stride-sampled, padded activations), w_amax [co * cols/block];
 *    for clip ratio i and block (o, b):
 *      loss[i, o, b] (+)= mean_t float(T(dot_T(x_t, qdq(w, T(amax*shrink_i))) - dot_T(x_t, w)))^2
 *    where dot_T rounds every product and the sum to T (the reference's (inputs * w).sum(-1)). */
int mtq_nvfp4_fp8_scale_sweep(const void *x, float *best_amax, int64_t n_blocks, int block,
                              int dtype, const float *global_amax, const float *candidates,
                              int n_candidates, hipStream_t stream);
int64_t mtq_mse_sweep_workspace_floats(int64_t rows, int64_t cols, int n_candidates);
int mtq_mse_sweep(const void *x, int64_t rows, int64_t cols, int dtype, const void *amax,
                  int amax_dtype, int amax_per_row, int round_candidate_amax,
                  const float *candidates, int n_candidates, int num_bits, int is_unsigned,
                  int narrow_range, float *loss, float *workspace, int64_t workspace_floats,
                  hipStream_t stream);
int mtq_awq_clip_search(const void *w, const float *x, int64_t co, int64_t cols, int64_t n_tokens,
                        int dtype, const void *w_amax, int amax_dtype, const float *shrinks,
                        int n_shrinks, int block, int num_bits, int is_unsigned, int narrow_range,
                        float *loss, int accumulate, hipStream_t stream);

/* ---- AWQ-lite alpha search GEMM (MFMA) ---------------------------------------------------
 * Replaces, for all G alphas of one linear and one calibration batch, the reference's search
 * forward + update_loss (model_calib.py:1513-1560, :1489-1495):
 *   loss[g] += mean_{m,n} float(T(T(sum_k T(x[m,k]*sinv[g,k]) * wq[g,n,k] + bias[n]) - yref[m,n]))^2
 * x [M, K], sinv [G, K] (= (1/s_g).to(T)), wq [G, N, K] (= qdq(W * s_g), mtq_block_quant_dynamic),
 * bias [N] or NULL, yref [M, N] (the unquantized output), all dtype T (bf16 / f16), 16-byte
 * aligned, K % 64 == 0, N % 8 == 0, M*K and N*K < 2^31; fp32 accumulation on v_mfma_f32_16x16x32; the output is never stored.
 * workspace: mtq_awq_search_gemm_workspace_floats(M, N, K, G) floats, 16-byte aligned, no
 * initialisation needed (per-tile partial sums + the pre-scaled activations [G, M, K]).
 * Deterministic (fixed-order sums).  G <= 64. */
int64_t mtq_awq_search_gemm_workspace_floats(int64_t M, int64_t N, int64_t K, int G);
int mtq_awq_search_gemm(const void *x, const void *sinv, const void *wq, const void *bias,
                        const void *yref, int64_t M, int64_t N, int64_t K, int dtype, int G,
                        float *loss, float *workspace, int64_t workspace_floats,
                        hipStream_t stream);
/* The same with the search kernel named (for A/B and tests; same arguments and results up to the
 * per-tile square-sum order): MTQ_AWQ_SEARCH_AUTO = what mtq_awq_search_gemm runs (W4 where its
 * limits allow, else PP); PP = the r03 two-group ping-pong kernel (8 waves, 128 x 64 per wave);
 * W4 = the r06 one-wave-per-SIMD kernel (4 waves, 128 x 128 per wave, K loop in generated inline
 * asm; needs K % 128 == 0 and M * N * 2 < 2^32, MTQ_ERR_INVALID_ARG otherwise). */
enum { MTQ_AWQ_SEARCH_AUTO = 0, MTQ_AWQ_SEARCH_PP = 1, MTQ_AWQ_SEARCH_W4 = 2 };
int mtq_awq_search_gemm_kernel(const void *x, const void *sinv, const void *wq, const void *bias,
                               const void *yref, int64_t M, int64_t N, int64_t K, int dtype, int G,
                               float *loss, float *workspace, int64_t workspace_floats, int kernel,
                               hipStream_t stream);
/* The same search with the GEMMs elsewhere (wide linears keep hipBLASLt):
 *  mtq_awq_prescale: xs[g, m, k] = T(x[m, k] * sinv[g, k]), one read of x for all G alphas
 *    (the reference's `inputs * pre_quant_scale` per alpha, tensor_quantizer.py:1143-1144).
 *  mtq_awq_mse_multi: loss[g] += mean(float(T(out[g] - ref))^2) over n elements for all G <= 16
 *    outputs [G, n] (update_loss, model_calib.py:1489-1495), reading ref once; workspace of
 *    mtq_awq_mse_multi_workspace_floats(n, G) floats; deterministic. */
int mtq_awq_prescale(const void *x, const void *sinv, void *xs, int64_t M, int64_t K, int dtype, int G,
                     hipStream_t stream);
/* AWQ-lite scale statistics, bit-identical to the reference's CPU run (csrc/mtq_awq_scale.hip):
 *  mtq_col_mean: y[k] = float(T(sum_m v[m, k] / M)), v = |x| (absval) or x, row-major [M, K] of
 *    dtype T (bf16 / f16 / fp32), summed in ATen's CPU order (SumKernel.cpp cascade) -- replaces
 *    get_act_scale `x.abs().view(-1, K).mean(0).float()` (model_calib.py:1471-1472) and the mean of
 *    get_weight_scale (:1453-1469).  workspace: mtq_col_mean_workspace_floats(M, K) floats.
 *  mtq_awq_scale_table: scales[g, :] = get_scale(x_max, w_max, alpha_g) (:1474-1487) for G
 *    alphas, e_num[g] = alpha_g and e_den[g] = 1 - alpha_g as doubles (device), pow as ATen's CPU
 *    pow(Tensor, Scalar) computes it. */
int64_t mtq_col_mean_workspace_floats(int64_t M, int64_t K);
int mtq_col_mean(const void *x, int64_t M, int64_t K, int dtype, int absval, float *workspace,
                 int64_t workspace_floats, float *y, hipStream_t stream);
int mtq_awq_scale_table(const float *x_max, const float *w_max, int64_t K, const double *e_num,
                        const double *e_den, int G, float *scales, hipStream_t stream);
int64_t mtq_awq_mse_multi_workspace_floats(int64_t n, int G);
int mtq_awq_mse_multi(const void *out, const void *ref, int64_t n, int dtype, int G, float *loss,
                      float *workspace, int64_t workspace_floats, hipStream_t stream);

/* ---- host (CPU) kernels: the reference's "cpu" op registration ---------------------------
 * The reference registers tensorrt::quantize_op for ["cpu", "cuda"] (tensor_quant.py:252-256)
 * and runs `_tensor_quant` (:607-645), `_fp8_eager` (:46-59) and `reduce_amax`
 * (utils/core_utils.py:146-183) as eager ATen on CPU tensors.  These are the same arithmetic
 * on host memory (x, y, amax, out are host pointers; amax is fp32 with axis_size elements,
 * channel of element i = (i / inner) % axis_size, axis_size 1 = per tensor), multi-threaded
 * with `nthreads` std::threads (0 = all hardware threads), bit-exact with the ATen sequences.
 *  mtq_cpu_fake_tensor_quant: INT-n qdq, as mtq_fake_tensor_quant(_with_axis).
 *  mtq_cpu_fake_e4m3fy:       FP8 qdq, as mtq_fake_e4m3fy(_with_axis); amax NULL = the plain
 *                             e4m3 cast round trip (mtq_e4m3_cast).
 *  mtq_cpu_reduce_amax:       as mtq_reduce_amax (accumulating, NaN-propagating). */
int mtq_cpu_fake_tensor_quant(const void *x, void *y, int64_t n, int dtype, const float *amax,
                              int64_t axis_size, int64_t inner, int num_bits, int is_unsigned,
                              int narrow_range, int nthreads);
int mtq_cpu_fake_e4m3fy(const void *x, void *y, int64_t n, int dtype, const float *amax,
                        int64_t axis_size, int64_t inner, int nthreads);
int mtq_cpu_reduce_amax(const void *x, int64_t P, int64_t K, int64_t Q, int dtype, float *out,
                        int nthreads);

/* ---- Fused flash attention with softmax-P quant-dequant (MFMA) ----------------------------
 * Replaces the reference's Triton `_attn_fwd` / `attention()` forward
 * (modelopt/torch/kernels/common/attention/triton_fa.py:255-516, :1221-1390) as the quantization
 * plugin dispatches it for `p_bmm_quantizer` (plugins/huggingface.py:125-195): GQA, causal or
 * not, online softmax over 32-key tiles, P fake-quantised before P.V:
 *   p_qdq_mode 0: none; 1: FP8 e4m3 per tensor, scale = p_qdq_scale (= amax / 448);
 *   2: NVFP4 (e2m1, e4m3 scale per 16 keys, global scale p_qdq_scale = amax / (6 * 448)).
 * Varlen layout of the reference: sequence b's query rows are [b_start_loc[b], + b_seq_len[b])
 * and its keys [b_start_loc_k[b], + b_seq_len_k[b]) (device int32 arrays of `batch` entries);
 * element (b, position t, head h, d) of q/k/v/o lives at
 *   base + b * strides[0|3|6|9] + t * strides[1|4|7|10] + h * strides[2|5|8|11] + d
 * (element strides, multiples of 16 bytes; d contiguous) -- the reference's flat [tokens, heads, D]
 * tensors use a zero batch stride, HF's [B, H, S, D] states a non-zero one (no copies).
 * Causal queries are the last b_seq_len[b] positions of the key span.  Rows past b_seq_len[b]
 * are not written.  q/k/v/o bf16, f16 or f32 (dtype), 16-byte aligned, head_dim in {16, 32, 64, 96, 128},
 * num_q_heads % num_kv_heads == 0.  softmax_scale / p_qdq_scale are the Python doubles the
 * reference passes (its fp32 kernel scalars are derived from them the same way).
 * K/V token strides (strides[4], strides[7]) must be >= head_dim (token rows do not overlap) and
 * span < 2^31 bytes over 64 tokens: the kernel stages keys by buffer loads bounded per 64-key
 * stage (MTQ_ERR_INVALID_ARG otherwise; every dense [B, S, H, D] / [B, H, S, D] layout passes). */
int mtq_attention_fwd(const void *q, const void *k, const void *v, void *o,
                      const int32_t *b_start_loc, const int32_t *b_seq_len,
                      const int32_t *b_start_loc_k, const int32_t *b_seq_len_k, int batch,
                      int max_len_q, int num_q_heads, int num_kv_heads, int head_dim,
                      const int64_t *strides, int is_causal, double softmax_scale,
                      int p_qdq_mode, double p_qdq_scale, int dtype, hipStream_t stream);

/* ---- dispatch registry (tracing) ----------------------------------------------------------
 * The launchers choose among kernel forms by shape, dtype and alignment (vector / block-group /
 * row-wave fake quant, persistent / row / column amax, ...); each launch of the families below
 * bumps a process-wide counter (one relaxed atomic add on the host).  mtq_dispatch_counts copies
 * min(n, count) counters into `counts` and returns the number of families; mtq_dispatch_name(i)
 * is family i's name (NULL out of range).  Used by the production-shape parity tests to prove
 * which kernels a Llama-shaped mtq.quantize reaches; no reference counterpart (tracing aux). */
int mtq_dispatch_counts(int64_t *counts, int n);
const char *mtq_dispatch_name(int id);

#ifdef __cplusplus
}
#endif
#endif /* MTQ_AMD_H_ */
