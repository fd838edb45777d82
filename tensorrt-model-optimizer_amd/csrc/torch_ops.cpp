// torch_ops.cpp — PyTorch-ROCm custom ops over the C ABI of libmtq_amd.so.
//
// Registers, under the `modelopt_amd` namespace, the op schemas of the reference's
// torch.library ops (tensorrt::quantize_op / tensorrt::dynamic_block_quantize_op,
// modelopt/torch/quantization/tensor_quant.py:222-276) and of its pybind extension modules
// (modelopt_cuda_ext, tensor_quant.cpp:63-76; modelopt_cuda_ext_fp8,
// tensor_quant_gpu_fp8.cu:109-114; modelopt_cuda_ext_mx, tensor_quant_mx.cu:393-411), plus
// the calibration reductions, on the device ("CUDA" dispatch key = HIP on ROCm) and Meta keys.
// The reference also registers "cpu" (tensor_quant.py:252-256): the INT / FP8 qdq ops and the
// amax reduction have CPU implementations here too, on the product's own host kernels
// (mtq_cpu_*, csrc/mtq_cpu.cpp); every other op raises on a CPU tensor.
// Every device kernel runs on the caller's current HIP stream; nothing here synchronises.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/Parallel.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <utility>
#include <tuple>
#include <vector>

#include "mtq_amd.h"

namespace {

hipStream_t cur_stream(const at::Tensor &t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

int dtype_code(at::ScalarType s) {
  switch (s) {
  case at::kFloat: return MTQ_F32;
  case at::kHalf: return MTQ_F16;
  case at::kBFloat16: return MTQ_BF16;
  case at::kDouble: return MTQ_F64;
  default: return -1;
  }
}

void check_status(int st, const char *what) {
  if (st == MTQ_ERR_BLOCKSIZE) TORCH_CHECK_VALUE(false, what, ": ", mtq_status_string(st));
  TORCH_CHECK(st == MTQ_OK, what, ": ", mtq_status_string(st),
              st == MTQ_ERR_LAUNCH ? " (hipError " : "",
              st == MTQ_ERR_LAUNCH ? std::to_string(mtq_last_hip_error()) : std::string(),
              st == MTQ_ERR_LAUNCH ? ")" : "");
}

void check_device(const at::Tensor &t, const char *name) {
  TORCH_CHECK(t.is_cuda(), "modelopt_amd: ", name,
              " must be on a ROCm (HIP) device; the MI355X-native path has no CPU kernels");
}

int cpu_threads() { return std::max(1, (int)at::get_num_threads()); }

// fp32 amax on the host for the CPU kernels (reference: amax.float())
at::Tensor cpu_amax(const at::Tensor &amax) {
  return amax.to(at::kCPU).to(at::kFloat).contiguous();
}

int checked_dtype(const at::Tensor &t, const char *name) {
  int d = dtype_code(t.scalar_type());
  TORCH_CHECK(d >= 0, "modelopt_amd: unsupported dtype ", t.scalar_type(), " for ", name);
  return d;
}

// amax -> (axis_size, inner) on the contiguous input, numpy-broadcast aligned to the input's
// trailing dims.  The non-singleton dims of amax must form one contiguous run of input dims
// (the reference's single-axis ext path, tensor_quant.py:85-91 / :103-108, is the one-dim case;
// a run such as amax [B, T, 1] on input [B, T, H] merges into one axis).
struct AxisMap {
  bool per_tensor;
  bool adjacent;  // false: the quantized axes are not one contiguous run (see permuted())
  int64_t axis_size, inner;
};

AxisMap axis_map(const at::Tensor &x, const at::Tensor &amax) {
  if (amax.numel() == 1) return {true, true, 1, 1};
  const int64_t xd = x.dim(), ad = amax.dim();
  TORCH_CHECK(ad <= xd, "modelopt_amd: amax of rank ", ad, " does not broadcast to input of rank ",
              xd);
  int first = -1, last = -1;
  bool adjacent = true;
  for (int64_t i = 0; i < ad; ++i) {
    const int64_t xi = xd - ad + i;
    if (amax.size(i) != 1) {
      TORCH_CHECK(amax.size(i) == x.size(xi), "modelopt_amd: amax shape ", amax.sizes(),
                  " does not broadcast to input shape ", x.sizes());
      if (first < 0) first = (int)xi;
      if (last >= 0 && last != xi - 1) adjacent = false;
      last = (int)xi;
    }
  }
  if (!adjacent) return {false, false, 0, 0};
  int64_t axis_size = 1, inner = 1;
  for (int i = first; i <= last; ++i) axis_size *= x.size(i);
  for (int64_t i = last + 1; i < xd; ++i) inner *= x.size(i);
  return {false, true, axis_size, inner};
}

// Non-adjacent quantization axes (e.g. the 2-D block view [2, 2, 3, 2, 2] with amax
// [2, 2, 1, 2, 1], tensor_quantizer_common.py:501-516): move the quantized axes to the front
// (device permute copies), quantize with one merged axis, and permute back.
template <class Fn>
at::Tensor permuted(const at::Tensor &x, const at::Tensor &amax, Fn fn) {
  const int64_t xd = x.dim();
  at::Tensor a = amax.reshape([&] {
    std::vector<int64_t> s(xd - amax.dim(), 1);
    for (auto v : amax.sizes()) s.push_back(v);
    return s;
  }());
  std::vector<int64_t> perm, rest;
  for (int64_t i = 0; i < xd; ++i) (a.size(i) != 1 ? perm : rest).push_back(i);
  perm.insert(perm.end(), rest.begin(), rest.end());
  std::vector<int64_t> inv(xd);
  for (int64_t i = 0; i < xd; ++i) inv[perm[i]] = i;
  at::Tensor xp = x.permute(perm).contiguous();
  at::Tensor ap = a.permute(perm).contiguous();
  at::Tensor yp = fn(xp, ap);
  return yp.permute(inv).contiguous();
}

at::Tensor amax_operand(const at::Tensor &amax, const at::Tensor &x) {
  at::Tensor a = amax;
  if (a.device() != x.device()) a = a.to(x.device());
  if (!a.is_contiguous()) a = a.contiguous();
  if (dtype_code(a.scalar_type()) < 0) a = a.to(at::kFloat);
  return a;
}

// ---- INT ---------------------------------------------------------------------------------------
void int_qdq_into(const at::Tensor &x, at::Tensor &y, const at::Tensor &amax_in, int64_t num_bits,
                  bool is_unsigned, bool narrow_range);
void int_qdq_into(const at::Tensor &x, at::Tensor &y, const at::Tensor &amax_in, int64_t num_bits,
                  bool is_unsigned, bool narrow_range) {
  if (x.is_cpu()) {
    at::Tensor xc = x.contiguous();
    at::Tensor amax = cpu_amax(amax_in);
    AxisMap m = axis_map(xc, amax);
    if (!m.adjacent) {
      y.copy_(permuted(xc, amax, [&](const at::Tensor &xp, const at::Tensor &ap) {
        at::Tensor yp = at::empty_like(xp);
        int_qdq_into(xp, yp, ap, num_bits, is_unsigned, narrow_range);
        return yp;
      }));
      return;
    }
    at::Tensor yc = y.is_contiguous() ? y : at::empty_like(xc);
    check_status(mtq_cpu_fake_tensor_quant(xc.data_ptr(), yc.data_ptr(), xc.numel(),
                                           checked_dtype(xc, "inputs"), amax.data_ptr<float>(),
                                           m.per_tensor ? 1 : m.axis_size,
                                           m.per_tensor ? 1 : m.inner, (int)num_bits, is_unsigned,
                                           narrow_range, cpu_threads()),
                 "fake_tensor_quant (cpu)");
    if (!yc.is_same(y)) y.copy_(yc);
    return;
  }
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  at::Tensor amax = amax_operand(amax_in, x);
  AxisMap m = axis_map(x, amax);
  if (!m.adjacent) {
    y.copy_(permuted(x, amax, [&](const at::Tensor &xp, const at::Tensor &ap) {
      at::Tensor yp = at::empty_like(xp);
      int_qdq_into(xp, yp, ap, num_bits, is_unsigned, narrow_range);
      return yp;
    }));
    return;
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st;
  if (m.per_tensor)
    st = mtq_fake_tensor_quant(x.data_ptr(), y.data_ptr(), x.numel(), dt, amax.data_ptr(),
                               dtype_code(amax.scalar_type()), (int)num_bits, is_unsigned,
                               narrow_range, cur_stream(x));
  else
    st = mtq_fake_tensor_quant_with_axis(x.data_ptr(), y.data_ptr(), x.numel(), dt,
                                         amax.data_ptr(), dtype_code(amax.scalar_type()),
                                         m.axis_size, m.inner, (int)num_bits, is_unsigned,
                                         narrow_range, cur_stream(x));
  check_status(st, "fake_tensor_quant");
}

at::Tensor fake_tensor_quant(const at::Tensor &inputs, const at::Tensor &amax, int64_t num_bits,
                             bool is_unsigned, bool narrow_range) {
  TORCH_CHECK(amax.numel() == 1, "fake_tensor_quant expects a per-tensor amax");
  at::Tensor x = inputs.contiguous();
  at::Tensor y = at::empty_like(x);
  int_qdq_into(x, y, amax, num_bits, is_unsigned, narrow_range);
  return y;
}

void fake_tensor_quant_(at::Tensor inputs, const at::Tensor &amax, int64_t num_bits,
                        bool is_unsigned, bool narrow_range) {
  TORCH_CHECK(inputs.is_contiguous(), "fake_tensor_quant_ requires a contiguous tensor");
  TORCH_CHECK(amax.numel() == 1, "fake_tensor_quant_ expects a per-tensor amax");
  int_qdq_into(inputs, inputs, amax, num_bits, is_unsigned, narrow_range);
}

at::Tensor fake_tensor_quant_with_axis(const at::Tensor &inputs, const at::Tensor &amax,
                                       int64_t axis, int64_t num_bits, bool is_unsigned,
                                       bool narrow_range) {
  at::Tensor x = inputs.contiguous();
  const int64_t ax = axis < 0 ? axis + x.dim() : axis;
  TORCH_CHECK(ax >= 0 && ax < x.dim(), "axis out of range");
  TORCH_CHECK(amax.numel() == x.size(ax), "amax must have size(axis) elements");
  if (x.is_cpu()) {
    at::Tensor a = cpu_amax(amax);
    at::Tensor y = at::empty_like(x);
    check_status(mtq_cpu_fake_tensor_quant(x.data_ptr(), y.data_ptr(), x.numel(),
                                           checked_dtype(x, "inputs"), a.data_ptr<float>(),
                                           x.size(ax), x.stride(ax), (int)num_bits, is_unsigned,
                                           narrow_range, cpu_threads()),
                 "fake_tensor_quant_with_axis (cpu)");
    return y;
  }
  check_device(x, "inputs");
  at::Tensor a = amax_operand(amax, x);
  at::Tensor y = at::empty_like(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_fake_tensor_quant_with_axis(
      x.data_ptr(), y.data_ptr(), x.numel(), checked_dtype(x, "inputs"), a.data_ptr(),
      dtype_code(a.scalar_type()), x.size(ax), x.stride(ax), (int)num_bits, is_unsigned,
      narrow_range, cur_stream(x));
  check_status(st, "fake_tensor_quant_with_axis");
  return y;
}

// ---- FP8 -----------------------------------------------------------------------------------
at::Tensor fp8_qdq(const at::Tensor &inputs, const at::Tensor &amax_in);
// Per-tensor element-wise qdq is layout-free: a dense, non-overlapping strided input (e.g. the
// transposed [B, H, S, D] K/V states of HF attention) is processed in its storage order and the
// output gets the same strides (empty_like preserves them), instead of a .contiguous() copy.
bool storage_order_ok(const at::Tensor &t, const at::Tensor &amax) {
  return amax.numel() == 1 && !t.is_contiguous() && t.is_non_overlapping_and_dense();
}

at::Tensor fp8_qdq(const at::Tensor &inputs, const at::Tensor &amax_in) {
  if (inputs.is_cpu()) {
    at::Tensor x = inputs.contiguous();
    at::Tensor amax = cpu_amax(amax_in);
    AxisMap m = axis_map(x, amax);
    if (!m.adjacent) return permuted(x, amax, [](const at::Tensor &xp, const at::Tensor &ap) {
      return fp8_qdq(xp, ap);
    });
    at::Tensor y = at::empty_like(x);
    check_status(mtq_cpu_fake_e4m3fy(x.data_ptr(), y.data_ptr(), x.numel(),
                                     checked_dtype(x, "inputs"), amax.data_ptr<float>(),
                                     m.per_tensor ? 1 : m.axis_size, m.per_tensor ? 1 : m.inner,
                                     cpu_threads()),
                 "fake_e4m3fy (cpu)");
    return y;
  }
  at::Tensor x = storage_order_ok(inputs, amax_in) ? inputs : inputs.contiguous();
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  at::Tensor amax = amax_operand(amax_in, x);
  AxisMap m = axis_map(x, amax);
  if (!m.adjacent) return permuted(x, amax, [](const at::Tensor &xp, const at::Tensor &ap) {
    return fp8_qdq(xp, ap);
  });
  at::Tensor y = at::empty_like(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st;
  if (m.per_tensor)
    st = mtq_fake_e4m3fy(x.data_ptr(), y.data_ptr(), x.numel(), dt, amax.data_ptr(),
                         dtype_code(amax.scalar_type()), cur_stream(x));
  else
    st = mtq_fake_e4m3fy_with_axis(x.data_ptr(), y.data_ptr(), x.numel(), dt, amax.data_ptr(),
                                   dtype_code(amax.scalar_type()), m.axis_size, m.inner,
                                   cur_stream(x));
  check_status(st, "fake_e4m3fy");
  return y;
}

at::Tensor fake_e4m3fy(const at::Tensor &inputs, const at::Tensor &amax) {
  TORCH_CHECK(amax.numel() == 1, "fake_e4m3fy expects a per-tensor amax");
  return fp8_qdq(inputs, amax);
}

at::Tensor fake_e4m3fy_with_axis(const at::Tensor &inputs, const at::Tensor &amax, int64_t axis) {
  at::Tensor x = inputs.contiguous();
  const int64_t ax = axis < 0 ? axis + x.dim() : axis;
  TORCH_CHECK(ax >= 0 && ax < x.dim(), "axis out of range");
  TORCH_CHECK(amax.numel() == x.size(ax), "amax must have size(axis) elements");
  if (x.is_cpu()) {
    at::Tensor a = cpu_amax(amax);
    at::Tensor y = at::empty_like(x);
    check_status(mtq_cpu_fake_e4m3fy(x.data_ptr(), y.data_ptr(), x.numel(),
                                     checked_dtype(x, "inputs"), a.data_ptr<float>(), x.size(ax),
                                     x.stride(ax), cpu_threads()),
                 "fake_e4m3fy_with_axis (cpu)");
    return y;
  }
  check_device(x, "inputs");
  at::Tensor a = amax_operand(amax, x);
  at::Tensor y = at::empty_like(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_fake_e4m3fy_with_axis(x.data_ptr(), y.data_ptr(), x.numel(),
                                     checked_dtype(x, "inputs"), a.data_ptr(),
                                     dtype_code(a.scalar_type()), x.size(ax), x.stride(ax),
                                     cur_stream(x));
  check_status(st, "fake_e4m3fy_with_axis");
  return y;
}

// plain e4m3 cast round trip (`_fp8_eager` with amax=None, tensor_quant.py:55-59).
at::Tensor e4m3_cast(const at::Tensor &inputs) {
  at::Tensor x = inputs.contiguous();
  if (x.is_cpu()) {
    at::Tensor y = at::empty_like(x);
    check_status(mtq_cpu_fake_e4m3fy(x.data_ptr(), y.data_ptr(), x.numel(),
                                     checked_dtype(x, "inputs"), nullptr, 1, 1, cpu_threads()),
                 "e4m3_cast (cpu)");
    return y;
  }
  check_device(x, "inputs");
  at::Tensor y = at::empty_like(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_e4m3_cast(x.data_ptr(), y.data_ptr(), x.numel(), checked_dtype(x, "inputs"),
                             cur_stream(x)),
               "e4m3_cast");
  return y;
}

// ---- dynamic block (MX) ----------------------------------------------------------------------
at::Tensor fused_amax_convert(const at::Tensor &inputs, int64_t block_size, int64_t format,
                              int64_t scale_format, const c10::optional<at::Tensor> &global_amax) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  TORCH_CHECK(dt != MTQ_F64, "fused_amax_convert: float64 not implemented");
  at::Tensor y = at::empty_like(x);
  if (x.numel() == 0) return y;
  const int64_t cols = x.dim() == 0 ? 1 : x.size(-1);
  const int64_t rows = x.numel() / cols;
  at::Tensor g;
  bool per_channel = false;
  if (global_amax.has_value() && global_amax->defined()) {
    g = global_amax->to(x.device(), at::kFloat).contiguous();
    // get_global_scaling, tensor_quant_mx.cu:296-312
    per_channel = x.dim() == 2 && g.numel() == x.size(0);
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_fused_amax_convert(x.data_ptr(), y.data_ptr(), rows, cols, dt, (int)block_size,
                                  (int)format, (int)scale_format,
                                  g.defined() ? g.data_ptr<float>() : nullptr, per_channel ? 1 : 0,
                                  cur_stream(x));
  check_status(st, "fused_amax_convert");
  return y;
}

// ---- reductions ---------------------------------------------------------------------------------
// out (fp32, contiguous, K elements) = max(out, max_{p,q} |x[p,k,q]|)
void amax_accumulate(const at::Tensor &inputs, at::Tensor out, int64_t P, int64_t K, int64_t Q) {
  at::Tensor x = inputs.contiguous();
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == K,
              "amax_accumulate: out must be a contiguous fp32 tensor with K elements");
  TORCH_CHECK(P * K * Q == x.numel(), "amax_accumulate: view [P,K,Q] does not match numel");
  if (x.is_cpu()) {
    TORCH_CHECK(out.is_cpu(), "amax_accumulate: out must be on the input's device");
    check_status(mtq_cpu_reduce_amax(x.data_ptr(), P, K, Q, checked_dtype(x, "inputs"),
                                     out.data_ptr<float>(), cpu_threads()),
                 "reduce_amax (cpu)");
    return;
  }
  check_device(x, "inputs");
  int dt = checked_dtype(x, "inputs");
  at::Tensor xx = x;
  if (dt == MTQ_F64) {  // exactness for doubles is lost in fp32; upcast path not provided
    TORCH_CHECK(false, "amax_accumulate: float64 inputs are not supported by the HIP reduction");
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_reduce_amax(xx.data_ptr(), P, K, Q, dt, out.data_ptr<float>(), cur_stream(x));
  check_status(st, "reduce_amax");
}

// Calibration bookkeeping on fp32 running-max buffers (mtq_amax_fill / _fold / _check): kept in
// the kernel library so a calibration pass loads no code object the model's forward has not.
void amax_fill_(at::Tensor out, double value) {
  check_device(out, "out");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous(), "amax_fill_: contiguous fp32 tensor");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(out.device());
  check_status(mtq_amax_fill(out.data_ptr<float>(), out.numel(), (float)value, cur_stream(out)), "amax_fill_");
}

void amax_fold_(at::Tensor dst, const at::Tensor &src) {
  check_device(dst, "dst");
  check_device(src, "src");
  TORCH_CHECK(dst.scalar_type() == at::kFloat && src.scalar_type() == at::kFloat && dst.is_contiguous() &&
                  src.is_contiguous() && dst.numel() == src.numel() && dst.device() == src.device(),
              "amax_fold_: contiguous fp32 tensors of equal size on one device");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dst.device());
  check_status(mtq_amax_fold(dst.data_ptr<float>(), src.data_ptr<float>(), dst.numel(), cur_stream(dst)),
               "amax_fold_");
}

// int32 [3] on x's device: any NaN, any +-inf, any negative value
at::Tensor amax_check(const at::Tensor &x) {
  check_device(x, "x");
  at::Tensor xc = x.contiguous();
  const int dt = checked_dtype(xc, "x");
  TORCH_CHECK(dt != MTQ_F64, "amax_check: float64 is not supported");
  at::Tensor flags = at::empty({3}, xc.options().dtype(at::kInt));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(xc.device());
  check_status(mtq_amax_check(xc.data_ptr(), xc.numel(), dt, flags.data_ptr<int32_t>(), cur_stream(xc)),
               "amax_check");
  return flags;
}

// hidden_states with the rows routed to no local expert zeroed (mtq_mask_unrouted_rows)
at::Tensor mask_unrouted_rows(const at::Tensor &x, const at::Tensor &idx, int64_t num_experts) {
  check_device(x, "hidden_states");
  check_device(idx, "top_k_index");
  TORCH_CHECK(x.dim() == 2 && idx.dim() == 2 && idx.size(0) == x.size(0) && idx.size(1) >= 1 &&
                  idx.scalar_type() == at::kLong && idx.device() == x.device(),
              "mask_unrouted_rows: hidden_states [T, H] and int64 top_k_index [T, k] on one device");
  at::Tensor xc = x.contiguous(), ic = idx.contiguous();
  at::Tensor y = at::empty_like(xc);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(xc.device());
  check_status(mtq_mask_unrouted_rows(xc.data_ptr(), y.data_ptr(), ic.data_ptr<int64_t>(), xc.size(0), xc.size(1),
                                      (int)ic.size(1), num_experts, checked_dtype(xc, "hidden_states"),
                                      cur_stream(xc)),
               "mask_unrouted_rows");
  return y;
}

// Persistent zero-initialised workspace per (device, stream) for the deterministic MSE
// reduction; the kernel restores its counter, so the buffer is filled once.
at::Tensor mse_workspace(const at::Tensor &like, int64_t floats) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, at::Tensor> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto key = std::make_pair((int)like.device().index(), cur_stream(like));
  auto it = cache.find(key);
  if (it == cache.end() || it->second.numel() < floats) {
    at::Tensor w = at::zeros({std::max<int64_t>(floats, 4096)}, like.options().dtype(at::kFloat));
    cache[key] = w;
    return w;
  }
  return it->second;
}

void mse_accumulate(const at::Tensor &a, const at::Tensor &b, at::Tensor loss, int64_t index) {
  check_device(a, "a");
  check_device(b, "b");
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.sizes() == b.sizes(),
              "mse_accumulate: a and b must have the same dtype and shape");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() && index >= 0 &&
                  index < loss.numel(),
              "mse_accumulate: loss must be a contiguous fp32 tensor and index in range");
  const int dt = checked_dtype(a, "a");
  TORCH_CHECK(dt != MTQ_F64, "mse_accumulate: float64 is not supported");
  at::Tensor ac = a.contiguous(), bc = b.contiguous();
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  const int64_t n = ac.numel();
  const int64_t wf = mtq_mse_workspace_floats(n, dt);
  at::Tensor ws = mse_workspace(ac, wf);
  int st = mtq_mse_accumulate(ac.data_ptr(), bc.data_ptr(), n, dt, loss.data_ptr<float>() + index,
                              ws.data_ptr<float>(), ws.numel(), cur_stream(ac));
  check_status(st, "mse_accumulate");
}

// AWQ-lite alpha search, all alphas of one linear in one MFMA launch (mtq_awq_search_gemm):
// loss[g] += mean((T(T(x * sinv[g]) @ wq[g]^T + bias) - yref)^2), the GEMM output never stored.
void awq_search_gemm(const at::Tensor &x, const at::Tensor &sinv, const at::Tensor &wq,
                     const c10::optional<at::Tensor> &bias, const at::Tensor &yref, at::Tensor loss,
                     int64_t kernel) {
  check_device(x, "x");
  check_device(wq, "wq");
  check_device(yref, "yref");
  const int dt = checked_dtype(x, "x");
  TORCH_CHECK(dt == MTQ_BF16 || dt == MTQ_F16, "awq_search_gemm: bf16 / f16 only");
  TORCH_CHECK(sinv.scalar_type() == x.scalar_type() && wq.scalar_type() == x.scalar_type() &&
                  yref.scalar_type() == x.scalar_type(),
              "awq_search_gemm: x, sinv, wq and yref must share the dtype");
  TORCH_CHECK(wq.dim() == 3 && sinv.dim() == 2, "awq_search_gemm: wq [G, N, K], sinv [G, K]");
  const int64_t G = wq.size(0), N = wq.size(1), K = wq.size(2);
  TORCH_CHECK(x.size(-1) == K && sinv.size(0) == G && sinv.size(1) == K,
              "awq_search_gemm: shape mismatch");
  at::Tensor xc = x.contiguous().view({-1, K});
  const int64_t M = xc.size(0);
  TORCH_CHECK(yref.numel() == M * N && yref.size(-1) == N, "awq_search_gemm: yref must be [..., N]");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() && loss.numel() == G,
              "awq_search_gemm: loss must be a contiguous fp32 tensor with G elements");
  at::Tensor sc = sinv.contiguous(), wc = wq.contiguous(), yc = yref.contiguous();
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->contiguous();
    TORCH_CHECK(b.scalar_type() == x.scalar_type() && b.numel() == N, "awq_search_gemm: bias");
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t wf = mtq_awq_search_gemm_workspace_floats(M, N, K, (int)G);
  at::Tensor ws = at::empty({std::max<int64_t>(wf, 1)}, x.options().dtype(at::kFloat));
  int st = mtq_awq_search_gemm_kernel(xc.data_ptr(), sc.data_ptr(), wc.data_ptr(),
                                      b.defined() ? b.data_ptr() : nullptr, yc.data_ptr(), M, N, K, dt,
                                      (int)G, loss.data_ptr<float>(), ws.data_ptr<float>(), ws.numel(),
                                      (int)kernel, cur_stream(xc));
  check_status(st, "awq_search_gemm");
}

// xs [G, M, K] = T(x * sinv[g]) for every alpha (mtq_awq_prescale)
at::Tensor awq_prescale(const at::Tensor &x, const at::Tensor &sinv) {
  check_device(x, "x");
  const int dt = checked_dtype(x, "x");
  TORCH_CHECK(dt == MTQ_BF16 || dt == MTQ_F16, "awq_prescale: bf16 / f16 only");
  const int64_t K = x.size(-1);
  at::Tensor xc = x.contiguous().view({-1, K});
  at::Tensor sc = sinv.to(x.device(), x.scalar_type()).contiguous();
  TORCH_CHECK(sc.dim() == 2 && sc.size(1) == K, "awq_prescale: sinv must be [G, K]");
  at::Tensor y = at::empty({sc.size(0), xc.size(0), K}, x.options());
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_awq_prescale(xc.data_ptr(), sc.data_ptr(), y.data_ptr(), xc.size(0), K, dt,
                                (int)sc.size(0), cur_stream(xc)),
               "awq_prescale");
  return y;
}

// y[k] = float(T(sum_m x[m, k] / M)) in ATen's CPU summation order (mtq_col_mean): awq_lite's
// get_act_scale (absval) and get_weight_scale means, reference model_calib.py:1453-1472
at::Tensor col_mean(const at::Tensor &x, bool absval) {
  check_device(x, "x");
  const int dt = checked_dtype(x, "x");
  TORCH_CHECK(dt == MTQ_BF16 || dt == MTQ_F16 || dt == MTQ_F32, "col_mean: bf16 / f16 / fp32 only");
  TORCH_CHECK(x.dim() >= 1, "col_mean: x must have a last dimension");
  const int64_t K = x.size(-1);
  at::Tensor xc = x.contiguous().view({-1, K});
  const int64_t M = xc.size(0);
  TORCH_CHECK(M >= 1, "col_mean: no rows");
  at::Tensor y = at::empty({K}, x.options().dtype(at::kFloat));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t wf = mtq_col_mean_workspace_floats(M, K);
  at::Tensor ws = at::empty({std::max<int64_t>(wf, 1)}, x.options().dtype(at::kFloat));
  check_status(mtq_col_mean(xc.data_ptr(), M, K, dt, absval ? 1 : 0, ws.data_ptr<float>(), ws.numel(),
                            y.data_ptr<float>(), cur_stream(xc)),
               "col_mean");
  return y;
}

// the AWQ get_scale rows of G alphas with the CPU's pow (mtq_awq_scale_table); e_num / e_den are
// the fp64 exponents alpha and 1 - alpha (reference model_calib.py:1474-1487)
at::Tensor awq_scale_table(const at::Tensor &x_max, const at::Tensor &w_max, const at::Tensor &e_num,
                           const at::Tensor &e_den) {
  check_device(x_max, "x_max");
  TORCH_CHECK(x_max.scalar_type() == at::kFloat && w_max.scalar_type() == at::kFloat,
              "awq_scale_table: fp32 act / weight scales");
  const int64_t K = x_max.numel();
  TORCH_CHECK(K >= 1 && w_max.numel() == K, "awq_scale_table: act / weight scale sizes differ");
  TORCH_CHECK(e_num.scalar_type() == at::kDouble && e_den.scalar_type() == at::kDouble &&
                  e_num.numel() == e_den.numel(),
              "awq_scale_table: fp64 exponent vectors of equal length");
  const int64_t G = e_num.numel();
  at::Tensor xc = x_max.contiguous().view({-1}), wc = w_max.to(x_max.device()).contiguous().view({-1});
  at::Tensor en = e_num.to(x_max.device()).contiguous(), ed = e_den.to(x_max.device()).contiguous();
  at::Tensor out = at::empty({G, K}, x_max.options());
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x_max.device());
  check_status(mtq_awq_scale_table(xc.data_ptr<float>(), wc.data_ptr<float>(), K, en.data_ptr<double>(),
                                   ed.data_ptr<double>(), (int)G, out.data_ptr<float>(), cur_stream(xc)),
               "awq_scale_table");
  return out;
}

// loss[g] += mean((out[g] - ref)^2) for all g at once (mtq_awq_mse_multi)
void awq_mse_multi(const at::Tensor &out, const at::Tensor &ref, at::Tensor loss) {
  check_device(out, "out");
  check_device(ref, "ref");
  const int dt = checked_dtype(out, "out");
  TORCH_CHECK(ref.scalar_type() == out.scalar_type(), "awq_mse_multi: dtype mismatch");
  const int64_t G = out.size(0), n = ref.numel();
  TORCH_CHECK(out.numel() == G * n, "awq_mse_multi: out must be [G, *ref.shape]");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() && loss.numel() == G,
              "awq_mse_multi: loss must be a contiguous fp32 tensor with G elements");
  at::Tensor oc = out.contiguous(), rc = ref.contiguous();
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(out.device());
  const int64_t wf = mtq_awq_mse_multi_workspace_floats(n, (int)G);
  at::Tensor ws = at::empty({std::max<int64_t>(wf, 1)}, out.options().dtype(at::kFloat));
  check_status(mtq_awq_mse_multi(oc.data_ptr(), rc.data_ptr(), n, dt, (int)G, loss.data_ptr<float>(),
                                 ws.data_ptr<float>(), ws.numel(), cur_stream(oc)),
               "awq_mse_multi");
}

at::Tensor mul_cols(const at::Tensor &x, const at::Tensor &scale) {
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  TORCH_CHECK(dt != MTQ_F64, "mul_cols: float64 is not supported");
  at::Tensor xc = x.contiguous();
  const int64_t cols = xc.size(-1);
  at::Tensor s = scale.to(x.device(), x.scalar_type()).contiguous();
  TORCH_CHECK(s.numel() == cols, "mul_cols: scale must have size(-1) elements");
  at::Tensor y = at::empty_like(xc);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_mul_cols(xc.data_ptr(), s.data_ptr(), y.data_ptr(), xc.numel() / cols, cols, dt,
                        cur_stream(xc));
  check_status(st, "mul_cols");
  return y;
}

at::Tensor nvfp4_fake_quant_block(const at::Tensor &inputs, const at::Tensor &global_amax,
                                  int64_t block_size) {
  check_device(inputs, "inputs");
  const int dt = checked_dtype(inputs, "inputs");
  TORCH_CHECK(dt != MTQ_F64, "nvfp4_fake_quant_block: float64 is not supported");
  at::Tensor x = inputs.contiguous();
  at::Tensor y = at::empty_like(x);
  if (x.numel() == 0) return y;
  at::Tensor g = global_amax.to(x.device(), at::kFloat).contiguous();
  TORCH_CHECK(g.numel() == 1, "nvfp4_fake_quant_block: global_amax must be a scalar");
  const int64_t cols = x.dim() == 0 ? 1 : x.size(-1);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_nvfp4_fake_quant(x.data_ptr(), y.data_ptr(), x.numel() / cols, cols, dt,
                                g.data_ptr<float>(), (int)block_size, cur_stream(x));
  check_status(st, "nvfp4_fake_quant_block");
  return y;
}

at::Tensor fp4_block_scale_quant(const at::Tensor &inputs, const at::Tensor &scales) {
  check_device(inputs, "inputs");
  const int dt = checked_dtype(inputs, "inputs");
  TORCH_CHECK(dt != MTQ_F64, "fp4_block_scale_quant: float64 is not supported");
  at::Tensor x = inputs.contiguous();
  at::Tensor y = at::empty_like(x);
  const int64_t nb = scales.numel();
  if (x.numel() == 0) return y;
  TORCH_CHECK(nb > 0 && x.numel() % nb == 0,
              "fp4_block_scale_quant: x.numel() must be a multiple of scales.numel()");
  at::Tensor s = scales.to(x.device(), at::kFloat).contiguous();
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_fp4_block_scale_quant(x.data_ptr(), y.data_ptr(), nb, (int)(x.numel() / nb), dt,
                                     s.data_ptr<float>(), cur_stream(x));
  check_status(st, "fp4_block_scale_quant");
  return y;
}

// ---- checkpoint export packing ---------------------------------------------------------------
at::Tensor export_fp8(const at::Tensor &weight, const at::Tensor &scale, bool per_row,
                      bool round_to_dtype) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt != MTQ_F64, "export_fp8: float64 is not supported");
  at::Tensor x = weight.contiguous();
  const int64_t cols = x.dim() == 0 ? 1 : x.size(-1);
  const int64_t rows = cols ? x.numel() / cols : 0;
  at::Tensor s = scale.to(x.device(), at::kFloat).contiguous();
  TORCH_CHECK(per_row ? s.numel() == rows : s.numel() == 1, "export_fp8: scale shape");
  at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_fp8(x.data_ptr(), y.data_ptr<uint8_t>(), rows, cols, dt,
                              s.data_ptr<float>(), per_row, round_to_dtype, cur_stream(x)),
               "export_fp8");
  return y.view(at::kFloat8_e4m3fn);
}

// FP8 with 2D block scales (FP8QTensor.quantize with {-1: bc, -2: br}): scale [R, C] block grid of
// a 2-D weight (any shape with that many elements); the quotient in the scale's dtype when it is
// the weight's 16-bit dtype (torch's bf16 / bf16 division), fp32 otherwise
at::Tensor export_fp8_block2d(const at::Tensor &weight, const at::Tensor &scale, int64_t block_rows,
                              int64_t block_cols) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt != MTQ_F64 && weight.dim() == 2, "export_fp8_block2d: 2-D f32/f16/bf16 weight expected");
  at::Tensor x = weight.contiguous();
  const int64_t rows = x.size(0), cols = x.size(1);
  TORCH_CHECK(block_rows >= 1 && block_cols >= 1, "export_fp8_block2d: block sizes");
  const int64_t nrb = (rows + block_rows - 1) / block_rows, ncb = (cols + block_cols - 1) / block_cols;
  TORCH_CHECK(scale.numel() == nrb * ncb, "export_fp8_block2d: scale must hold one value per block");
  const bool round = scale.scalar_type() == weight.scalar_type() && dt != MTQ_F32;
  at::Tensor s = scale.to(x.device(), at::kFloat).contiguous();
  at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_fp8_block2d(x.data_ptr(), y.data_ptr<uint8_t>(), rows, cols, dt, s.data_ptr<float>(),
                                      block_rows, block_cols, round ? 1 : 0, cur_stream(x)),
               "export_fp8_block2d");
  return y.view(at::kFloat8_e4m3fn);
}

at::Tensor export_int4(const at::Tensor &weight, const at::Tensor &scale) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt != MTQ_F64 && weight.dim() == 2, "export_int4: 2-D f32/f16/bf16 weight expected");
  at::Tensor x = weight.contiguous();
  at::Tensor s = scale.to(x.device(), at::kFloat).contiguous();
  const int64_t rows = x.size(0), cols = x.size(1);
  TORCH_CHECK(s.dim() == 2 && s.size(0) == rows && cols % s.size(1) == 0, "export_int4: scale shape");
  at::Tensor y = at::empty({rows / 2, cols}, x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_int4(x.data_ptr(), y.data_ptr<uint8_t>(), rows, cols, dt,
                               s.data_ptr<float>(), (int)(cols / s.size(1)), cur_stream(x)),
               "export_int4");
  return y;
}

at::Tensor export_nvfp4(const at::Tensor &weight, const at::Tensor &block_scale,
                        const at::Tensor &scale_2) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt != MTQ_F64, "export_nvfp4: float64 is not supported");
  at::Tensor x = weight.contiguous();
  const int64_t cols = x.size(-1), rows = x.numel() / cols;
  at::Tensor bs = block_scale.to(x.device(), at::kFloat).contiguous();
  at::Tensor s2 = scale_2.to(x.device(), at::kFloat).contiguous();
  TORCH_CHECK(bs.numel() > 0 && x.numel() % bs.numel() == 0 && s2.numel() == 1,
              "export_nvfp4: scale shapes");
  const int block = (int)(x.numel() / bs.numel());
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = cols / 2;
  at::Tensor y = at::empty(shape, x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_nvfp4(x.data_ptr(), y.data_ptr<uint8_t>(), rows, cols, dt,
                                bs.data_ptr<float>(), s2.data_ptr<float>(), block, cur_stream(x)),
               "export_nvfp4");
  return y;
}

std::tuple<at::Tensor, at::Tensor> export_mxfp4(const at::Tensor &weight, int64_t block) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt != MTQ_F64, "export_mxfp4: float64 is not supported");
  at::Tensor x = weight.contiguous();
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = shape.back() / 2;
  at::Tensor y = at::empty(shape, x.options().dtype(at::kByte));
  at::Tensor sc = at::empty({x.numel() / block, 1}, x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_mxfp4(x.data_ptr(), y.data_ptr<uint8_t>(), sc.data_ptr<uint8_t>(),
                                x.numel(), dt, (int)block, cur_stream(x)),
               "export_mxfp4");
  return {y, sc};
}

// MXFP8: (e4m3 codes as float8_e4m3fn, same shape; E8M0 scale bytes [..., K/32])
std::tuple<at::Tensor, at::Tensor> export_mxfp8(const at::Tensor &weight) {
  check_device(weight, "weight");
  const int dt = checked_dtype(weight, "weight");
  TORCH_CHECK(dt == MTQ_BF16 || dt == MTQ_F16, "export_mxfp8: bf16 / f16 weights only");
  TORCH_CHECK(weight.dim() >= 1 && weight.size(-1) % 32 == 0, "export_mxfp8: last dim % 32 != 0");
  at::Tensor x = weight.contiguous();
  at::Tensor y = at::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  std::vector<int64_t> sshape(x.sizes().begin(), x.sizes().end());
  sshape.back() = sshape.back() / 32;
  at::Tensor sc = at::empty(sshape, x.options().dtype(at::kByte));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_export_mxfp8(x.data_ptr(), reinterpret_cast<uint8_t *>(y.data_ptr()),
                                sc.data_ptr<uint8_t>(), x.numel(), dt, cur_stream(x)),
               "export_mxfp8");
  return {y, sc};
}

// ---- calibration searches (mtq_search.hip) ------------------------------------------------
// nvfp4_fp8_scale_sweep(x [n_blocks, block], global_amax, candidates [126] fp32) -> best amax
// [n_blocks] fp32 (kernels/quantization/gemm/nvfp4_fp8_sweep.py:108-160).
at::Tensor nvfp4_fp8_scale_sweep(const at::Tensor &inputs, const at::Tensor &global_amax,
                                 const at::Tensor &candidates, int64_t block_size) {
  check_device(inputs, "x");
  TORCH_CHECK_VALUE(block_size > 0 && inputs.numel() % block_size == 0, "x.numel() (",
                    inputs.numel(), ") is not divisible by block_size (", block_size, ").");
  at::Tensor x = inputs.contiguous();
  const int dt = checked_dtype(x, "x");
  TORCH_CHECK(dt != MTQ_F64, "nvfp4_fp8_scale_sweep: float64 is not supported");
  at::Tensor g = global_amax.to(x.device(), at::kFloat).reshape({1}).contiguous();
  at::Tensor c = candidates.to(x.device(), at::kFloat).contiguous();
  const int64_t nb = x.numel() / block_size;
  at::Tensor best = at::empty({nb}, x.options().dtype(at::kFloat));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_nvfp4_fp8_scale_sweep(x.data_ptr(), best.data_ptr<float>(), nb, (int)block_size,
                                         dt, g.data_ptr<float>(), c.data_ptr<float>(),
                                         (int)c.numel(), cur_stream(x)),
               "nvfp4_fp8_scale_sweep");
  return best;
}

// mse_sweep(x [rows, cols], amax [rows] or [1], candidates [K], num_bits (0 = e4m3), unsigned,
// narrow_range, round_candidate_amax) -> loss [K, rows] fp32 (calib/mse.py:82-125).
at::Tensor mse_sweep(const at::Tensor &inputs, const at::Tensor &amax, const at::Tensor &candidates,
                     int64_t num_bits, bool is_unsigned, bool narrow_range,
                     bool round_candidate_amax) {
  check_device(inputs, "x");
  TORCH_CHECK(inputs.dim() == 2, "mse_sweep: x must be 2-D [rows, cols]");
  at::Tensor x = inputs.contiguous();
  const int dt = checked_dtype(x, "x");
  TORCH_CHECK(dt != MTQ_F64, "mse_sweep: float64 is not supported");
  const int64_t rows = x.size(0), cols = x.size(1);
  at::Tensor a = amax.to(x.device()).contiguous();
  const int adt = checked_dtype(a, "amax");
  TORCH_CHECK(a.numel() == 1 || a.numel() == rows, "mse_sweep: amax must have 1 or rows elements");
  at::Tensor c = candidates.to(x.device(), at::kFloat).contiguous();
  const int k = (int)c.numel();
  at::Tensor loss = at::empty({k, rows}, x.options().dtype(at::kFloat));
  const int64_t wsn = mtq_mse_sweep_workspace_floats(rows, cols, k);
  TORCH_CHECK(wsn >= 0, "mse_sweep: invalid shape");
  at::Tensor ws = at::empty({std::max<int64_t>(wsn, 1)}, x.options().dtype(at::kFloat));
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_status(mtq_mse_sweep(x.data_ptr(), rows, cols, dt, a.data_ptr(), adt,
                             a.numel() != 1 || rows == 1 ? 1 : 0, round_candidate_amax ? 1 : 0,
                             c.data_ptr<float>(), k, (int)num_bits, is_unsigned, narrow_range,
                             loss.data_ptr<float>(), ws.data_ptr<float>(), wsn, cur_stream(x)),
               "mse_sweep");
  return loss;
}

// awq_clip_search(w [co, cols], x [tokens, cols] fp32, w_amax [co * cols/block], shrinks [S],
// loss [S, co, cols/block] fp32 (in/out), block, num_bits, unsigned, narrow_range, accumulate)
// (model_calib.py:1815-1882).
void awq_clip_search(const at::Tensor &weight, const at::Tensor &x, const at::Tensor &w_amax,
                     const at::Tensor &shrinks, at::Tensor loss, int64_t block, int64_t num_bits,
                     bool is_unsigned, bool narrow_range, bool accumulate) {
  check_device(weight, "weight");
  TORCH_CHECK(weight.dim() == 2 && x.dim() == 2 && x.size(1) == weight.size(1),
              "awq_clip_search: weight [co, cols] and x [tokens, cols] expected");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous(), "awq_clip_search: x must be fp32 contiguous");
  at::Tensor w = weight.contiguous();
  const int dt = checked_dtype(w, "weight");
  TORCH_CHECK(dt != MTQ_F64, "awq_clip_search: float64 is not supported");
  at::Tensor a = w_amax.contiguous();
  const int adt = checked_dtype(a, "w_amax");
  const int64_t co = w.size(0), cols = w.size(1);
  TORCH_CHECK(block > 0 && cols % block == 0, "awq_clip_search: cols must be a multiple of block");
  TORCH_CHECK(a.numel() == co * (cols / block), "awq_clip_search: w_amax must have co*cols/block elements");
  at::Tensor s = shrinks.to(w.device(), at::kFloat).contiguous();
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() &&
                  loss.numel() == s.numel() * co * (cols / block),
              "awq_clip_search: loss must be fp32 contiguous [S, co, cols/block]");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(w.device());
  check_status(mtq_awq_clip_search(w.data_ptr(), x.data_ptr<float>(), co, cols, x.size(0), dt,
                                   a.data_ptr(), adt, s.data_ptr<float>(), (int)s.numel(), (int)block,
                                   (int)num_bits, is_unsigned, narrow_range, loss.data_ptr<float>(),
                                   accumulate ? 1 : 0, cur_stream(w)),
               "awq_clip_search");
}

at::Tensor block_quant_dynamic(const at::Tensor &inputs, const c10::optional<at::Tensor> &pqs,
                               int64_t block, int64_t num_bits, bool is_unsigned,
                               bool narrow_range) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  at::Tensor y = at::empty_like(x);
  const int64_t cols = x.size(-1), rows = x.numel() / cols;
  at::Tensor s;
  if (pqs.has_value() && pqs->defined()) {
    s = pqs->to(x.device(), x.scalar_type()).contiguous();
    TORCH_CHECK(s.numel() == cols, "block_quant_dynamic: pre_quant_scale must have cols elements");
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_block_quant_dynamic(x.data_ptr(), y.data_ptr(), rows, cols, dt,
                                   s.defined() ? s.data_ptr() : nullptr, dt, (int)block,
                                   (int)num_bits, is_unsigned, narrow_range, cur_stream(x));
  check_status(st, "block_quant_dynamic");
  return y;
}

// The weight side of every AWQ alpha at once: out[g] = qdq_block(T(W * pqs[g])), out [G, N, K]
// (G launches of mtq_block_quant_dynamic writing straight into the stacked output).
at::Tensor block_quant_dynamic_multi(const at::Tensor &inputs, const at::Tensor &pqs, int64_t block,
                                     int64_t num_bits, bool is_unsigned, bool narrow_range) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  const int dt = checked_dtype(x, "inputs");
  const int64_t cols = x.size(-1), rows = x.numel() / cols;
  at::Tensor s = pqs.to(x.device(), x.scalar_type()).contiguous();
  TORCH_CHECK(s.dim() == 2 && s.size(1) == cols, "block_quant_dynamic_multi: pqs must be [G, cols]");
  const int64_t G = s.size(0);
  at::Tensor y = at::empty({G, rows, cols}, x.options());
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const size_t esz = x.element_size();
  for (int64_t g = 0; g < G; ++g) {
    int st = mtq_block_quant_dynamic(
        x.data_ptr(), static_cast<char *>(y.data_ptr()) + g * rows * cols * esz, rows, cols, dt,
        static_cast<const char *>(s.data_ptr()) + g * cols * esz, dt, (int)block, (int)num_bits,
        is_unsigned, narrow_range, cur_stream(x));
    check_status(st, "block_quant_dynamic_multi");
  }
  return y;
}

// QuantLinear simulated GEMM for short inputs: y = x . qdq(W)^T (+ bias), weight fake quant fused
// into the MFMA operand loads (mtq_qlinear_small_m).  kind 0 = INT-n, 1 = FP8 e4m3.
at::Tensor qlinear_small_m(const at::Tensor &input, const at::Tensor &weight,
                           const c10::optional<at::Tensor> &bias, const at::Tensor &amax,
                           int64_t block, int64_t kind, int64_t num_bits, bool is_unsigned,
                           bool narrow_range) {
  check_device(input, "input");
  check_device(weight, "weight");
  TORCH_CHECK(weight.dim() == 2, "qlinear_small_m: 2-D weight expected");
  TORCH_CHECK(input.scalar_type() == weight.scalar_type(), "qlinear_small_m: input/weight dtype mismatch");
  const int dt = checked_dtype(input, "input");
  const int64_t N = weight.size(0), K = weight.size(1);
  TORCH_CHECK(input.size(-1) == K, "qlinear_small_m: input last dim must equal weight.size(1)");
  at::Tensor x = input.contiguous();
  at::Tensor w = weight.contiguous();
  const int64_t M = K ? x.numel() / K : 0;
  // fp32 amax: the streaming kernel's layout (a no-op for the calibrators' fp32 amax)
  at::Tensor a = amax.to(at::kFloat).contiguous();
  TORCH_CHECK(a.device() == x.device(), "qlinear_small_m: amax must be on the input device");
  at::Tensor b;
  if (bias.has_value() && bias->defined()) {
    b = bias->contiguous();
    TORCH_CHECK(b.scalar_type() == x.scalar_type() && b.numel() == N, "qlinear_small_m: bias");
  }
  std::vector<int64_t> shape(input.sizes().begin(), input.sizes().end());
  shape.back() = N;
  at::Tensor y = at::empty(shape, x.options());
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  // split-K partial tiles (fp32) from the caching allocator
  const size_t wsb = M >= 1 && M <= 16 ? mtq_qlinear_small_m_workspace_bytes(M, N, K) : 0;
  at::Tensor ws = at::empty({(int64_t)(wsb / sizeof(float))}, x.options().dtype(at::kFloat));
  int st = mtq_qlinear_small_m_ws(x.data_ptr(), w.data_ptr(), b.defined() ? b.data_ptr() : nullptr,
                                  y.data_ptr(), M, N, K, dt, a.data_ptr(), checked_dtype(a, "amax"),
                                  a.numel(), block, (int)kind, (int)num_bits, is_unsigned,
                                  narrow_range, wsb ? ws.data_ptr() : nullptr, wsb, cur_stream(x));
  check_status(st, "qlinear_small_m");
  return y;
}

// Up to 4 short-input linears of one M and K in one launch (mtq_qlinear_small_m_group): the
// q/k/v projections of a decode step.  Per linear as qlinear_small_m; flags as 0/1 ints.
std::vector<at::Tensor> qlinear_small_m_group(at::TensorList inputs, at::TensorList weights,
                                              const c10::List<c10::optional<at::Tensor>> &biases,
                                              at::TensorList amaxs, at::IntArrayRef blocks, int64_t kind,
                                              at::IntArrayRef num_bits, at::IntArrayRef is_unsigned,
                                              at::IntArrayRef narrow_range) {
  const size_t n = inputs.size();
  TORCH_CHECK(n >= 1 && n <= 4, "qlinear_small_m_group: 1 to 4 linears");
  TORCH_CHECK(weights.size() == n && biases.size() == n && amaxs.size() == n && blocks.size() == n &&
                  num_bits.size() == n && is_unsigned.size() == n && narrow_range.size() == n,
              "qlinear_small_m_group: one entry per linear in every list");
  check_device(inputs[0], "input");
  const int dt = checked_dtype(inputs[0], "input");
  const int64_t K = inputs[0].size(-1);
  const int64_t M = K ? inputs[0].numel() / K : 0;
  std::vector<at::Tensor> xs, ws, as, bs, ys;
  std::vector<mtq_qlinear_problem> pr(n);
  std::vector<int64_t> Ns(n);
  for (size_t i = 0; i < n; ++i) {
    check_device(inputs[i], "input");
    check_device(weights[i], "weight");
    TORCH_CHECK(weights[i].dim() == 2 && weights[i].size(1) == K && inputs[i].size(-1) == K &&
                    inputs[i].numel() == M * K,
                "qlinear_small_m_group: every linear needs the same input rows and K");
    TORCH_CHECK(inputs[i].scalar_type() == inputs[0].scalar_type() &&
                    weights[i].scalar_type() == inputs[0].scalar_type(),
                "qlinear_small_m_group: one dtype for all inputs and weights");
    xs.push_back(inputs[i].contiguous());
    ws.push_back(weights[i].contiguous());
    as.push_back(amaxs[i].to(at::kFloat).contiguous());
    TORCH_CHECK(as.back().device() == xs.back().device(), "qlinear_small_m_group: amax device");
    at::Tensor b;
    const c10::optional<at::Tensor> bo = biases.get(i);
    if (bo.has_value() && bo->defined()) {
      b = bo->contiguous();
      TORCH_CHECK(b.scalar_type() == xs.back().scalar_type() && b.numel() == weights[i].size(0),
                  "qlinear_small_m_group: bias");
    }
    bs.push_back(b);
    std::vector<int64_t> shape(inputs[i].sizes().begin(), inputs[i].sizes().end());
    shape.back() = weights[i].size(0);
    ys.push_back(at::empty(shape, xs.back().options()));
    Ns[i] = weights[i].size(0);
    pr[i] = mtq_qlinear_problem{xs[i].data_ptr(), ws[i].data_ptr(), b.defined() ? b.data_ptr() : nullptr,
                                ys[i].data_ptr(), Ns[i], as[i].data_ptr(), checked_dtype(as[i], "amax"),
                                as[i].numel(), blocks[i], (int)kind, (int)num_bits[i], (int)is_unsigned[i],
                                (int)narrow_range[i]};
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(xs[0].device());
  const size_t wsb = M >= 1 && M <= 16 ? mtq_qlinear_small_m_group_workspace_bytes(M, Ns.data(), (int)n, K) : 0;
  at::Tensor wsp = at::empty({(int64_t)(wsb / sizeof(float))}, xs[0].options().dtype(at::kFloat));
  check_status(mtq_qlinear_small_m_group(pr.data(), (int)n, M, K, dt, wsb ? wsp.data_ptr() : nullptr, wsb,
                                         cur_stream(xs[0])),
               "qlinear_small_m_group");
  return ys;
}

void histogram_abs_accumulate(const at::Tensor &inputs, const at::Tensor &hmax, at::Tensor counts,
                              int64_t bins, bool skip_zeros) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  TORCH_CHECK(counts.scalar_type() == at::kInt && counts.is_contiguous() && counts.numel() >= bins,
              "histogram: counts must be a contiguous int32 tensor with >= bins elements");
  TORCH_CHECK(hmax.scalar_type() == at::kFloat && hmax.numel() == 1, "histogram: hmax fp32 scalar");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  int st = mtq_histogram_abs(x.data_ptr(), x.numel(), checked_dtype(x, "inputs"),
                             hmax.data_ptr<float>(), (int)bins, skip_zeros ? 1 : 0,
                             reinterpret_cast<uint32_t *>(counts.data_ptr<int32_t>()),
                             cur_stream(x));
  check_status(st, "histogram_abs");
}

at::Tensor histogram_abs_chunked(const at::Tensor &inputs, const at::Tensor &hmax, int64_t bins,
                                 bool skip_zeros, const c10::optional<at::Tensor> &bounds,
                                 int64_t chunk_elems, int64_t chunks,
                                 const c10::optional<at::Tensor> &scratch_in,
                                 const c10::optional<at::Tensor> &accum_in) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  TORCH_CHECK(hmax.scalar_type() == at::kFloat && hmax.numel() == 1, "histogram: hmax fp32 scalar");
  TORCH_CHECK(chunks >= 1 && chunks <= (1 << 20), "histogram_abs_chunked: bad chunk count");
  const int64_t *bp = nullptr;
  at::Tensor b;
  if (bounds.has_value() && bounds->defined()) {
    b = bounds->contiguous();
    TORCH_CHECK(b.scalar_type() == at::kLong && b.numel() == chunks + 1 && b.device() == x.device(),
                "histogram_abs_chunked: bounds must be int64 [chunks + 1] on the input's device");
    bp = b.data_ptr<int64_t>();
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  // the per-workgroup count rows (any contents, overwritten): the caller's buffer when it is large
  // enough, else a fresh one from the caching allocator
  const int64_t words = mtq_histogram_chunked_scratch_words(x.numel(), (int)chunks, (int)bins);
  TORCH_CHECK(words >= 0, "histogram_abs_chunked: bad size");
  at::Tensor scratch;
  if (scratch_in.has_value() && scratch_in->defined()) {
    scratch = *scratch_in;
    TORCH_CHECK(scratch.scalar_type() == at::kInt && scratch.is_contiguous() && scratch.device() == x.device(),
                "histogram_abs_chunked: scratch must be contiguous int32 on the input's device");
  }
  if (!scratch.defined() || scratch.numel() < words) scratch = at::empty({words > 0 ? words : 1}, x.options().dtype(at::kInt));
  // accum: a running fp32 histogram added into the result (its first accum.numel() bins)
  at::Tensor accum;
  if (accum_in.has_value() && accum_in->defined()) {
    accum = accum_in->contiguous();
    TORCH_CHECK(accum.scalar_type() == at::kFloat && accum.dim() == 1 && accum.numel() <= bins &&
                    accum.device() == x.device(),
                "histogram_abs_chunked: accum must be fp32 [<= bins] on the input's device");
  }
  at::Tensor hist = at::empty({bins}, x.options().dtype(at::kFloat));
  int st = mtq_histogram_abs_chunked(x.data_ptr(), x.numel(), checked_dtype(x, "inputs"),
                                     hmax.data_ptr<float>(), (int)bins, skip_zeros ? 1 : 0, bp,
                                     chunk_elems, (int)chunks,
                                     reinterpret_cast<uint32_t *>(scratch.data_ptr<int32_t>()), scratch.numel(),
                                     accum.defined() ? accum.data_ptr<float>() : nullptr,
                                     accum.defined() ? accum.numel() : 0, hist.data_ptr<float>(),
                                     cur_stream(x));
  check_status(st, "histogram_abs_chunked");
  return hist;
}

// torch.histc's chunking with skip_zeros, all on the device and in one read of the input
// (mtq_histogram_abs_nonzero_chunked)
at::Tensor histogram_abs_chunked_nonzero(const at::Tensor &inputs, const at::Tensor &hmax, int64_t bins,
                                         int64_t threads, const c10::optional<at::Tensor> &scratch_in,
                                         const c10::optional<at::Tensor> &accum_in) {
  at::Tensor x = inputs.contiguous();
  check_device(x, "inputs");
  TORCH_CHECK(hmax.scalar_type() == at::kFloat && hmax.numel() == 1, "histogram: hmax fp32 scalar");
  TORCH_CHECK(threads >= 1 && threads <= 1024, "histogram_abs_chunked_nonzero: threads must be 1..1024");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const int64_t words = mtq_histogram_nonzero_scratch_words(x.numel(), (int)threads, (int)bins);
  TORCH_CHECK(words >= 0, "histogram_abs_chunked_nonzero: bad size (bins <= 8176)");
  at::Tensor scratch;
  if (scratch_in.has_value() && scratch_in->defined()) {
    scratch = *scratch_in;
    TORCH_CHECK(scratch.scalar_type() == at::kInt && scratch.is_contiguous() && scratch.device() == x.device(),
                "histogram_abs_chunked_nonzero: scratch must be contiguous int32 on the input's device");
  }
  if (!scratch.defined() || scratch.numel() < words) scratch = at::empty({words > 0 ? words : 1}, x.options().dtype(at::kInt));
  at::Tensor accum;
  if (accum_in.has_value() && accum_in->defined()) {
    accum = accum_in->contiguous();
    TORCH_CHECK(accum.scalar_type() == at::kFloat && accum.dim() == 1 && accum.numel() <= bins &&
                    accum.device() == x.device(),
                "histogram_abs_chunked_nonzero: accum must be fp32 [<= bins] on the input's device");
  }
  at::Tensor hist = at::empty({bins}, x.options().dtype(at::kFloat));
  int st = mtq_histogram_abs_nonzero_chunked(
      x.data_ptr(), x.numel(), checked_dtype(x, "inputs"), hmax.data_ptr<float>(), (int)bins, (int)threads, 32768,
      reinterpret_cast<uint32_t *>(scratch.data_ptr<int32_t>()), scratch.numel(),
      accum.defined() ? accum.data_ptr<float>() : nullptr, accum.defined() ? accum.numel() : 0,
      hist.data_ptr<float>(), cur_stream(x));
  check_status(st, "histogram_abs_chunked_nonzero");
  return hist;
}

// ---- reference torch.library ops (tensor_quant.py:115-195) -------------------------------------
at::Tensor quantize_op(const at::Tensor &input, const at::Tensor &amax, int64_t num_bits,
                       int64_t exponent_bits, bool is_unsigned, bool narrow_range) {
  if (num_bits == 8 && exponent_bits == 4) return fp8_qdq(input, amax);
  TORCH_CHECK_VALUE(exponent_bits == 0, "Invalid combination of (num_bits, exponent_bits): (",
                    num_bits, ", ", exponent_bits, ").");
  at::Tensor x = storage_order_ok(input, amax) ? input : input.contiguous();
  at::Tensor y = at::empty_like(x);
  int_qdq_into(x, y, amax, num_bits, is_unsigned, narrow_range);
  return y;
}

int format_code(int64_t e, int64_t m, bool is_int) {
  if (is_int) return e == 8 ? MTQ_INT8 : -1;  // mx_format_map key 8
  if (e == 4 && m == 3) return MTQ_E4M3;
  if (e == 5 && m == 2) return MTQ_E5M2;
  if (e == 3 && m == 2) return MTQ_E3M2;
  if (e == 2 && m == 3) return MTQ_E2M3;
  if (e == 8 && m == 0) return MTQ_E8M0;
  if (e == 2 && m == 1) return MTQ_E2M1;
  if (e == 1 && m == 2) return MTQ_E1M2;
  if (e == 0 && m == 3) return MTQ_E0M3;
  if (e == 3 && m == 0) return MTQ_E3M0;
  return -1;
}

// mirrors tensor_quant.DISABLE_TRITON_KERNEL (tensor_quant.py:43)
std::atomic<bool> g_disable_nvfp4_kernel{false};

at::Tensor dynamic_block_quantize_op(const at::Tensor &input, int64_t block_size,
                                     const c10::optional<at::Tensor> &amax, int64_t num_bits,
                                     int64_t exponent_bits, int64_t scale_num_bits,
                                     int64_t scale_exponent_bits) {
  // _dynamic_block_quantize_impl, tensor_quant.py:157-195
  const int64_t se = scale_exponent_bits, sm = scale_num_bits - scale_exponent_bits - 1;
  int fmt;
  if (exponent_bits != 0)
    fmt = format_code(exponent_bits, num_bits - exponent_bits - 1, false);
  else
    fmt = format_code(num_bits, 0, true);
  TORCH_CHECK(fmt >= 0, "Unsupported num_bits: ", num_bits, ", exponent_bits: ", exponent_bits,
              " for dynamic block quantization.");
  const int sfmt = format_code(se, sm, false);
  TORCH_CHECK(sfmt >= 0, "Scale bits (", se, ", ", sm, ") are not a supported format");
  c10::optional<at::Tensor> g;
  if (sfmt != MTQ_E8M0) {
    TORCH_CHECK(amax.has_value() && amax->defined() && amax->is_cuda(),
                "amax must be a CUDA tensor for dynamic block quantization.");
    g = amax->numel() != 1 ? amax->amax() : *amax;
  }
  // NVFP4 goes to the reference's primary kernel (fp4_fake_quant_block, default block 16,
  // tensor_quant.py:173-181) unless DISABLE_TRITON_KERNEL routes it to fused_amax_convert
  if (fmt == MTQ_E2M1 && sfmt == MTQ_E4M3 && !g_disable_nvfp4_kernel.load())
    return nvfp4_fake_quant_block(input, *g, 16);
  return fused_amax_convert(input, block_size, fmt, sfmt, g);
}

void set_disable_triton_kernel(bool v) { g_disable_nvfp4_kernel.store(v); }

at::Tensor meta_like(const at::Tensor &x) { return at::empty_like(x); }

}  // namespace

// attention_fwd(q, k, v, o (out), b_start_loc, b_seq_len, b_start_loc_k, b_seq_len_k, max_len_q,
// is_causal, softmax_scale, p_qdq_mode, p_qdq_scale): the reference's Triton flash attention with
// softmax-P qdq (triton_fa.py:255-516).  q/k/v/o are either the reference's flat [tokens, heads, D]
// tensors or [B, S, H, D] strided views (e.g. HF's [B, H, S, D] states transposed, no copy); the
// last dim must be contiguous.  Rows past b_seq_len are left untouched in o.
void attention_fwd(const at::Tensor &q, const at::Tensor &k, const at::Tensor &v, at::Tensor o,
                   const at::Tensor &b_start_loc, const at::Tensor &b_seq_len,
                   const at::Tensor &b_start_loc_k, const at::Tensor &b_seq_len_k, int64_t max_len_q,
                   bool is_causal, double softmax_scale, int64_t p_qdq_mode, double p_qdq_scale) {
  check_device(q, "q");
  const int dt = dtype_code(q.scalar_type());
  TORCH_CHECK(dt == MTQ_BF16 || dt == MTQ_F16 || dt == MTQ_F32, "attention_fwd: q/k/v must be bf16, fp16 or fp32");
  TORCH_CHECK(k.scalar_type() == q.scalar_type() && v.scalar_type() == q.scalar_type() &&
                  o.scalar_type() == q.scalar_type(),
              "attention_fwd: q, k, v and o must share the dtype");
  const int64_t nd = q.dim();
  TORCH_CHECK((nd == 3 || nd == 4) && k.dim() == nd && v.dim() == nd && o.dim() == nd,
              "attention_fwd: q/k/v/o must all be [tokens, heads, D] or all [B, S, heads, D]");
  for (const at::Tensor *t : {&q, &k, &v, static_cast<const at::Tensor *>(&o)})
    TORCH_CHECK(t->is_cuda() && t->device() == q.device() && t->stride(-1) == 1,
                "attention_fwd: tensors on q's device with a contiguous last dim expected");
  TORCH_CHECK(o.sizes() == q.sizes() && v.sizes() == k.sizes() && k.size(-1) == q.size(-1),
              "attention_fwd: shape mismatch");
  int64_t st[12];
  const at::Tensor *ts[4] = {&q, &k, &v, &o};
  for (int i = 0; i < 4; ++i) {
    st[3 * i] = nd == 4 ? ts[i]->stride(0) : 0;
    st[3 * i + 1] = ts[i]->stride(nd - 3);
    st[3 * i + 2] = ts[i]->stride(nd - 2);
  }
  const int64_t batch = b_seq_len.numel();
  auto meta = [&](const at::Tensor &t, const char *name) {
    TORCH_CHECK(t.numel() == batch, "attention_fwd: ", name, " must have one entry per sequence");
    return t.to(q.device(), at::kInt).contiguous();
  };
  at::Tensor sl = meta(b_start_loc, "b_start_loc"), ln = meta(b_seq_len, "b_seq_len");
  at::Tensor slk = meta(b_start_loc_k, "b_start_loc_k"), lnk = meta(b_seq_len_k, "b_seq_len_k");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(q.device());
  check_status(mtq_attention_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                 sl.data_ptr<int32_t>(), ln.data_ptr<int32_t>(), slk.data_ptr<int32_t>(),
                                 lnk.data_ptr<int32_t>(), (int)batch, (int)max_len_q, (int)q.size(-2),
                                 (int)k.size(-2), (int)q.size(-1), st, is_causal ? 1 : 0, softmax_scale,
                                 (int)p_qdq_mode, p_qdq_scale, dt, cur_stream(q)),
               "attention_fwd");
}

TORCH_LIBRARY(modelopt_amd, m) {
  m.def("quantize_op(Tensor input, Tensor amax, int num_bits, int exponent_bits, bool unsigned, "
        "bool narrow_range) -> Tensor");
  m.def("dynamic_block_quantize_op(Tensor input, int block_size, Tensor? amax, int num_bits, "
        "int exponent_bits, int scale_num_bits, int scale_exponent_bits) -> Tensor");
  m.def("fake_tensor_quant(Tensor inputs, Tensor amax, int num_bits=8, bool unsigned=False, "
        "bool narrow_range=True) -> Tensor");
  m.def("fake_tensor_quant_(Tensor(a!) inputs, Tensor amax, int num_bits=8, bool unsigned=False, "
        "bool narrow_range=True) -> ()");
  m.def("fake_tensor_quant_with_axis(Tensor inputs, Tensor amax, int axis, int num_bits=8, "
        "bool unsigned=False, bool narrow_range=True) -> Tensor");
  m.def("fake_e4m3fy(Tensor inputs, Tensor amax) -> Tensor");
  m.def("fake_e4m3fy_with_axis(Tensor inputs, Tensor amax, int axis) -> Tensor");
  m.def("e4m3_cast(Tensor inputs) -> Tensor");
  m.def("fused_amax_convert(Tensor inputs, int block_size, int format, int scale_format, "
        "Tensor? global_amax=None) -> Tensor");
  m.def("amax_accumulate(Tensor inputs, Tensor(a!) out, int P, int K, int Q) -> ()");
  m.def("amax_fill_(Tensor(a!) out, float value) -> ()");
  m.def("amax_fold_(Tensor(a!) dst, Tensor src) -> ()");
  m.def("amax_check(Tensor x) -> Tensor");
  m.def("mask_unrouted_rows(Tensor hidden_states, Tensor top_k_index, int num_experts) -> Tensor");
  m.def("block_quant_dynamic(Tensor inputs, Tensor? pre_quant_scale, int block, int num_bits, "
        "bool unsigned, bool narrow_range) -> Tensor");
  m.def("histogram_abs_accumulate(Tensor inputs, Tensor hmax, Tensor(a!) counts, int bins, "
        "bool skip_zeros) -> ()");
  m.def("histogram_abs_chunked(Tensor inputs, Tensor hmax, int bins, bool skip_zeros, Tensor? bounds, "
        "int chunk_elems, int chunks, Tensor(a!)? scratch=None, Tensor? accum=None) -> Tensor");
  m.def("histogram_abs_chunked_nonzero(Tensor inputs, Tensor hmax, int bins, int threads, "
        "Tensor(a!)? scratch=None, Tensor? accum=None) -> Tensor");
  m.def("qlinear_small_m_group(Tensor[] inputs, Tensor[] weights, Tensor?[] biases, Tensor[] amaxs, int[] blocks, "
        "int kind, int[] num_bits, int[] is_unsigned, int[] narrow_range) -> Tensor[]");
  m.def("qlinear_small_m(Tensor input, Tensor weight, Tensor? bias, Tensor amax, int block, int kind, "
        "int num_bits, bool unsigned, bool narrow_range) -> Tensor");
  m.def("mse_accumulate(Tensor a, Tensor b, Tensor(a!) loss, int index) -> ()");
  m.def("mul_cols(Tensor inputs, Tensor scale) -> Tensor");
  m.def("block_quant_dynamic_multi(Tensor inputs, Tensor pqs, int block, int num_bits, bool unsigned, "
        "bool narrow_range) -> Tensor");
  m.def("awq_prescale(Tensor x, Tensor sinv) -> Tensor");
  m.def("col_mean(Tensor x, bool absval) -> Tensor");
  m.def("awq_scale_table(Tensor x_max, Tensor w_max, Tensor e_num, Tensor e_den) -> Tensor");
  m.def("awq_mse_multi(Tensor out, Tensor ref, Tensor(a!) loss) -> ()");
  m.def("awq_search_gemm(Tensor x, Tensor sinv, Tensor wq, Tensor? bias, Tensor yref, Tensor(a!) loss, "
        "int kernel=0) -> ()");
  m.def("nvfp4_fake_quant_block(Tensor inputs, Tensor global_amax, int block_size=16) -> Tensor");
  m.def("set_disable_triton_kernel(bool disable) -> ()", &set_disable_triton_kernel);
  m.def("fp4_block_scale_quant(Tensor inputs, Tensor scales) -> Tensor");
  m.def("export_fp8(Tensor weight, Tensor scale, bool per_row, bool round_to_dtype) -> Tensor");
  m.def("export_fp8_block2d(Tensor weight, Tensor scale, int block_rows, int block_cols) -> Tensor");
  m.def("export_int4(Tensor weight, Tensor scale) -> Tensor");
  m.def("export_nvfp4(Tensor weight, Tensor block_scale, Tensor scale_2) -> Tensor");
  m.def("export_mxfp4(Tensor weight, int block) -> (Tensor, Tensor)");
  m.def("export_mxfp8(Tensor weight) -> (Tensor, Tensor)");
  m.def("nvfp4_fp8_scale_sweep(Tensor x, Tensor global_amax, Tensor candidates, int block_size=16) -> Tensor");
  m.def("mse_sweep(Tensor x, Tensor amax, Tensor candidates, int num_bits, bool unsigned, "
        "bool narrow_range, bool round_candidate_amax) -> Tensor");
  m.def("awq_clip_search(Tensor weight, Tensor x, Tensor w_amax, Tensor shrinks, Tensor(a!) loss, "
        "int block, int num_bits, bool unsigned, bool narrow_range, bool accumulate) -> ()");
  m.def("attention_fwd(Tensor q, Tensor k, Tensor v, Tensor(a!) o, Tensor b_start_loc, Tensor b_seq_len, "
        "Tensor b_start_loc_k, Tensor b_seq_len_k, int max_len_q, bool is_causal, float softmax_scale, "
        "int p_qdq_mode, float p_qdq_scale) -> ()");
}

TORCH_LIBRARY_IMPL(modelopt_amd, CUDA, m) {
  m.impl("quantize_op", &quantize_op);
  m.impl("qlinear_small_m", &qlinear_small_m);
  m.impl("qlinear_small_m_group", &qlinear_small_m_group);
  m.impl("dynamic_block_quantize_op", &dynamic_block_quantize_op);
  m.impl("fake_tensor_quant", &fake_tensor_quant);
  m.impl("fake_tensor_quant_", &fake_tensor_quant_);
  m.impl("fake_tensor_quant_with_axis", &fake_tensor_quant_with_axis);
  m.impl("fake_e4m3fy", &fake_e4m3fy);
  m.impl("fake_e4m3fy_with_axis", &fake_e4m3fy_with_axis);
  m.impl("e4m3_cast", &e4m3_cast);
  m.impl("fused_amax_convert", &fused_amax_convert);
  m.impl("amax_fill_", &amax_fill_);
  m.impl("amax_fold_", &amax_fold_);
  m.impl("amax_check", &amax_check);
  m.impl("mask_unrouted_rows", &mask_unrouted_rows);
  m.impl("amax_accumulate", &amax_accumulate);
  m.impl("block_quant_dynamic", &block_quant_dynamic);
  m.impl("histogram_abs_accumulate", &histogram_abs_accumulate);
  m.impl("histogram_abs_chunked", &histogram_abs_chunked);
  m.impl("histogram_abs_chunked_nonzero", &histogram_abs_chunked_nonzero);
  m.impl("mse_accumulate", &mse_accumulate);
  m.impl("mul_cols", &mul_cols);
  m.impl("awq_search_gemm", &awq_search_gemm);
  m.impl("awq_prescale", &awq_prescale);
  m.impl("col_mean", &col_mean);
  m.impl("awq_scale_table", &awq_scale_table);
  m.impl("awq_mse_multi", &awq_mse_multi);
  m.impl("block_quant_dynamic_multi", &block_quant_dynamic_multi);
  m.impl("nvfp4_fake_quant_block", &nvfp4_fake_quant_block);
  m.impl("fp4_block_scale_quant", &fp4_block_scale_quant);
  m.impl("export_fp8", &export_fp8);
  m.impl("export_fp8_block2d", &export_fp8_block2d);
  m.impl("export_int4", &export_int4);
  m.impl("export_nvfp4", &export_nvfp4);
  m.impl("export_mxfp4", &export_mxfp4);
  m.impl("export_mxfp8", &export_mxfp8);
  m.impl("nvfp4_fp8_scale_sweep", &nvfp4_fp8_scale_sweep);
  m.impl("mse_sweep", &mse_sweep);
  m.impl("awq_clip_search", &awq_clip_search);
  m.impl("attention_fwd", &attention_fwd);
}

// the reference's "cpu" registration (tensor_quant.py:252-256), on the host kernels
TORCH_LIBRARY_IMPL(modelopt_amd, CPU, m) {
  m.impl("quantize_op", &quantize_op);
  m.impl("fake_tensor_quant", &fake_tensor_quant);
  m.impl("fake_tensor_quant_", &fake_tensor_quant_);
  m.impl("fake_tensor_quant_with_axis", &fake_tensor_quant_with_axis);
  m.impl("fake_e4m3fy", &fake_e4m3fy);
  m.impl("fake_e4m3fy_with_axis", &fake_e4m3fy_with_axis);
  m.impl("e4m3_cast", &e4m3_cast);
  m.impl("amax_accumulate", &amax_accumulate);
}

TORCH_LIBRARY_IMPL(modelopt_amd, Meta, m) {
  m.impl("qlinear_small_m", [](const at::Tensor &x, const at::Tensor &w, const c10::optional<at::Tensor> &,
                               const at::Tensor &, int64_t, int64_t, int64_t, bool, bool) {
    std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
    shape.back() = w.size(0);
    return at::empty(shape, x.options().device(at::kMeta));
  });
  m.impl("quantize_op", [](const at::Tensor &x, const at::Tensor &, int64_t, int64_t, bool, bool) {
    return meta_like(x);
  });
  m.impl("dynamic_block_quantize_op",
         [](const at::Tensor &x, int64_t, const c10::optional<at::Tensor> &, int64_t, int64_t,
            int64_t, int64_t) { return meta_like(x); });
  m.impl("fake_tensor_quant",
         [](const at::Tensor &x, const at::Tensor &, int64_t, bool, bool) { return meta_like(x); });
  m.impl("fake_tensor_quant_with_axis",
         [](const at::Tensor &x, const at::Tensor &, int64_t, int64_t, bool, bool) {
           return meta_like(x);
         });
  m.impl("fake_e4m3fy", [](const at::Tensor &x, const at::Tensor &) { return meta_like(x); });
  m.impl("fake_e4m3fy_with_axis",
         [](const at::Tensor &x, const at::Tensor &, int64_t) { return meta_like(x); });
  m.impl("e4m3_cast", [](const at::Tensor &x) { return meta_like(x); });
  m.impl("fused_amax_convert",
         [](const at::Tensor &x, int64_t, int64_t, int64_t, const c10::optional<at::Tensor> &) {
           return meta_like(x);
         });
  m.impl("block_quant_dynamic",
         [](const at::Tensor &x, const c10::optional<at::Tensor> &, int64_t, int64_t, bool, bool) {
           return meta_like(x);
         });
  m.impl("mul_cols", [](const at::Tensor &x, const at::Tensor &) { return meta_like(x); });
  m.impl("nvfp4_fake_quant_block",
         [](const at::Tensor &x, const at::Tensor &, int64_t) { return meta_like(x); });
  m.impl("fp4_block_scale_quant", [](const at::Tensor &x, const at::Tensor &) { return meta_like(x); });
  m.impl("mse_accumulate", [](const at::Tensor &, const at::Tensor &, at::Tensor, int64_t) {});
}
