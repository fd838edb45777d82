"""The drop-in boundary exercised the way a reference maintainer would bind it, on device tensors.

* The ctypes stub printed in INTEGRATION.md (``_mtq_amd_ctypes.py``: fake_e4m3fy,
  fake_tensor_quant, nvfp4_pack) is extracted from the document verbatim, pointed at the in-tree
  libmtq_amd.so and run on HIP tensors; results equal the oracle bit for bit.
* ``torch.ops.tensorrt.quantize_op`` / ``dynamic_block_quantize_op`` (the reference's own op
  names, tensor_quant.py:222-276) resolve to the HIP kernels.
"""

import re
from pathlib import Path

import pytest
import torch

from modelopt_amd import _ext
from oracle import ref_ops as R

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _same(a, b):
    iv = {torch.bfloat16: torch.int16, torch.float16: torch.int16, torch.float32: torch.int32,
          torch.uint8: torch.uint8}[a.dtype]
    if a.dtype == torch.uint8:
        return torch.equal(a, b)
    nan = torch.isnan(a) & torch.isnan(b)
    return bool(((a.view(iv) == b.view(iv)) | nan).all())


def _integration_stub():
    """The python blocks of INTEGRATION.md that make up ``_mtq_amd_ctypes.py``, executed."""
    text = (REPO / "INTEGRATION.md").read_text()
    blocks = re.findall(r"```python\n(.*?)```", text, flags=re.S)
    code = "\n".join(b for b in blocks if "_mtq_amd_ctypes.py" in b)
    assert "def fake_e4m3fy" in code and "def nvfp4_pack" in code
    code = code.replace('ctypes.CDLL("libmtq_amd.so")', f'ctypes.CDLL("{_ext.KERNEL_LIB}")')
    ns: dict = {}
    exec(compile(code, "INTEGRATION.md:_mtq_amd_ctypes.py", "exec"), ns)
    return ns


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_integration_ctypes_stub_on_device(gpu, dtype):
    stub = _integration_stub()
    g = torch.Generator().manual_seed(7)
    x = (torch.randn(129, 256, generator=g) * 4).to(dtype)
    amax = x.float().abs().amax() * 0.6
    y = stub["fake_e4m3fy"](x.to(gpu), amax.to(gpu))
    assert _same(y.cpu(), R.fp8_eager(x, amax))
    for bits, unsigned, narrow in ((8, False, True), (4, False, False)):
        y = stub["fake_tensor_quant"](x.to(gpu), amax.to(gpu), bits, unsigned, narrow)
        assert _same(y.cpu(), R.tensor_quant(x, amax, bits, unsigned, narrow))
    # the export packing step bound through the same stub
    w = (torch.randn(64, 256, generator=g) * 0.05).to(dtype)
    s2 = w.float().abs().amax() / 2688
    bs = (w.float().reshape(64, -1, 16).abs().amax(-1) / (6 * s2)).clamp(2**-9, 448)
    bs = bs.to(torch.float8_e4m3fn).float()
    q = stub["nvfp4_pack"](w.to(gpu), bs.to(gpu), s2.to(gpu))
    torch.cuda.synchronize()
    assert torch.equal(q.cpu(), R.export_nvfp4(w, bs, s2))


@pytest.mark.parametrize("p_qdq", [None, "fp8", "nvfp4"])
def test_integration_attention_stub_on_device(gpu, p_qdq):
    """The attention binding of INTEGRATION.md §2c on device tensors == the torch op path and
    the oracle (oracle/attention_ref.py) within the fused-attention tolerance."""
    from modelopt_amd.torch.kernels.common.attention import attention
    from oracle import attention_ref as A

    stub = _integration_stub()
    g = torch.Generator().manual_seed(17)
    q = torch.randn(2 * 70, 4, 64, generator=g).bfloat16()
    k = torch.randn(2 * 70, 2, 64, generator=g).bfloat16()
    v = torch.randn(2 * 70, 2, 64, generator=g).bfloat16()
    st, ln = torch.tensor([0, 70]).int(), torch.tensor([70, 41]).int()
    o = stub["attention_fwd"](q.to(gpu), k.to(gpu), v.to(gpu), st.to(gpu), ln.to(gpu), 70, p_qdq=p_qdq)
    ref = attention(q.to(gpu), k.to(gpu), v.to(gpu), st.to(gpu), ln.to(gpu), 70, p_qdq=p_qdq)
    valid = torch.cat([torch.ones(70), torch.ones(41), torch.zeros(29)]).bool()
    assert torch.equal(o[valid.to(gpu)], ref[valid.to(gpu)])
    want = A.attention_fwd(q, k, v, st, ln, p_qdq=p_qdq)
    torch.testing.assert_close(o.cpu()[valid].float(), want[valid].float(), rtol=2e-2, atol=2e-2)


def test_integration_qlinear_group_stub_on_device(gpu):
    """The grouped decode-projection binding of INTEGRATION.md §2d == the torch op's grouped launch
    (same kernel, same split) bit for bit, for q/k/v-shaped FP8 and INT4-block linears."""
    from modelopt_amd import _ext

    stub = _integration_stub()
    g = torch.Generator().manual_seed(23)
    x = torch.randn(3, 512, generator=g).bfloat16().to(gpu)
    ws = [(torch.randn(n, 512, generator=g) * 0.05).bfloat16().to(gpu) for n in (512, 128, 128)]
    for kind, nb, blk in ((1, 8, None), (0, 4, 128)):
        if blk is None:
            am = [w.float().abs().amax().reshape(()) for w in ws]
            blocks = [512] * 3
        else:
            am = [w.float().reshape(-1, blk).abs().amax(1, keepdim=True) for w in ws]
            blocks = [blk] * 3
        ys = stub["qlinear_group"](x, ws, am, blocks, kind, nb)
        want = _ext.ops().qlinear_small_m_group([x] * 3, ws, [None] * 3, am, blocks, kind, [nb] * 3, [0] * 3, [0] * 3)
        for y, w in zip(ys, want):
            assert torch.equal(y, w)


def test_integration_stub_reports_errors(gpu):
    stub = _integration_stub()
    x = torch.randn(8, device=gpu, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        stub["fake_tensor_quant"](x, torch.tensor(1.0, device=gpu), 40)  # num_bits out of range


def test_reference_op_names_on_device(gpu):
    from modelopt_amd.torch.quantization import tensor_quant as tq

    assert tq.register_reference_op_names()  # opt-in
    assert tq.REFERENCE_OP_NAMES_REGISTERED
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(64, 256, generator=g) * 2).to(torch.bfloat16)
    ab = x.float().view(-1, 128).abs().amax(dim=1, keepdim=True)
    y = torch.ops.tensorrt.quantize_op(x.view(-1, 128).to(gpu), ab.to(gpu), 8, 4, False, False)
    assert _same(y.cpu(), R.fp8_eager(x.view(-1, 128), ab))
    a = x.float().abs().amax()
    y = torch.ops.tensorrt.quantize_op(x.to(gpu), a.to(gpu), 4, 0, False, False)
    assert _same(y.cpu(), R.tensor_quant(x, a, 4, False, False))
    # MXFP4 (E2M1, E8M0 scales): the None-amax overload
    y = torch.ops.tensorrt.dynamic_block_quantize_op(x.to(gpu), 32, None, 4, 2, 9, 8)
    assert _same(y.cpu(), R.fused_amax_convert(x, 32, "E2M1"))
    y = torch.ops.tensorrt.dynamic_block_quantize_op.overload(x.to(gpu), 32, None, 4, 2, 9, 8)
    assert _same(y.cpu(), R.fused_amax_convert(x, 32, "E2M1"))
    # meta (torch.export / fake tensors)
    m = torch.ops.tensorrt.quantize_op(x.to("meta"), a.to("meta"), 8, 4, False, False)
    assert m.shape == x.shape and m.device.type == "meta"
