"""AWQ-lite scale statistics on the GPU, bit-identical to the reference's CPU run.

The first ops where the GPU's awq_lite used to leave the reference's CPU run (tests/golden/
awq_b128.*, made by running the reference on the CPU) -- found by feeding each stage the
reference's own inputs:
* ``pow`` in get_scale (model_calib.py:1474-1487): ATen's CPU pow is a vectorised double-float
  powf that is not correctly rounded on ~1.5 % of the elements; the device libm's is another;
* the two means, get_act_scale / get_weight_scale (:1453-1472): ATen's CPU sum order (a four-level
  cascade) and a true division by the row count, vs the device's tree sum times 1/M;
* ``act_scale / num_cache_steps``: a division by a Python int, which torch on the GPU performs as
  a multiplication by the reciprocal.
``mtq_awq_scale_table`` / ``mtq_col_mean`` (csrc/mtq_awq_scale.hip) restate the CPU sequences and
the division goes through a device tensor; every one is pinned here against torch's own CPU ops
(the reference's ATen sequence) and against the golden run.  What remains: (1) the CPU's sqrt
(MKL VML: not correctly rounded on ~0.6 % of the inputs, host-dependent) in the normalisation
sqrt(max * min) and in pow(x, 0.5) -- the kernel takes the IEEE sqrt; (2) the calibration forward
itself: a linear's input after the first one is a bf16 GEMM output, whose fp32 summation order
differs between the CPU and the GPU -- measured below.
"""

from pathlib import Path

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu
G = Path(__file__).resolve().parent / "golden"


def _bits(t):
    t = t.detach().cpu().contiguous()
    return t.view({torch.float32: torch.int32, torch.bfloat16: torch.int16, torch.float16: torch.int16}[t.dtype])


def _ieee_sqrt(t):
    return torch.from_numpy(np.sqrt(t.reshape(-1).numpy())).reshape(t.shape)


def _ref_scale_row(x, w, a):
    """Reference get_scale on the CPU, with every sqrt -- the normalisation ``sqrt(max * min)`` and
    ATen's exponent-0.5 special case of pow -- taken as the IEEE (correctly rounded) sqrt: torch's
    CPU ``sqrt`` runs MKL's VML, which is not correctly rounded on ~0.6 % of the inputs and gives
    different results on the Intel host that made the goldens and the AMD host of the GPU box
    (found by this test's first runs on the box).  That sqrt is the one op of the
    reference's CPU sequence the kernel does not restate (it has no public definition)."""
    def pw(v, e):
        return _ieee_sqrt(v) if float(e) == 0.5 else v.pow(e)

    s = (pw(x, a) / (pw(w, 1 - a) + torch.finfo(torch.float32).tiny)).clamp(min=1e-4, max=1e4).view(-1)
    n = _ieee_sqrt((s.max() * s.min()).reshape(1))[0]
    return (s / n).view(-1)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("M,K", [(1, 64), (3, 40), (17, 33), (192, 256), (255, 100), (256, 2304), (1000, 48),
                                 (4097, 96), (8192, 1024), (14336, 72), (5000, 4101)])
def test_col_mean_matches_cpu_mean_bitwise(gpu, dtype, M, K):
    from modelopt_amd import _ext

    g = torch.Generator().manual_seed(M * 131 + K)
    x = (torch.randn(M, K, generator=g) * torch.exp2(torch.rand(K, generator=g) * 10 - 5)).to(dtype)
    want = x.abs().contiguous().view(-1, K).mean(0).to(torch.float32)  # get_act_scale on the CPU
    got = _ext.ops().col_mean(x.to(gpu), True)
    assert torch.equal(_bits(got), _bits(want))
    # without |.|: the weight-scale mean of a non-negative tensor, and signed data
    want2 = x.mean(0).to(torch.float32)
    assert torch.equal(_bits(_ext.ops().col_mean(x.to(gpu), False)), _bits(want2))


@pytest.mark.parametrize("K", [33, 256, 1000, 2304, 4096, 14336, 28672])
def test_scale_table_matches_cpu_get_scale_bitwise(gpu, K):
    from modelopt_amd.torch.quantization import model_calib as MC

    g = torch.Generator().manual_seed(K)
    x = (torch.rand(K, generator=g) * 12 - 6).exp2()
    w = torch.rand(K, generator=g) * 0.9 + 0.05
    x[::97] = 0.0  # zero act scale channels
    for step in (0.1, 0.05):
        alphas = [k.item() for k in torch.arange(0, 1.0 + step, step)]
        want = torch.stack([_ref_scale_row(x, w, a) for a in alphas])
        got = MC._scale_table(x.to(gpu), w.to(gpu), alphas)
        assert torch.equal(_bits(got), _bits(want)), step
        got1 = MC.get_scale(x.to(gpu), w.to(gpu), alphas[3])
        assert torch.equal(_bits(got1), _bits(want[3]))


class _WideMLP(torch.nn.Module):  # the golden's model (tests/golden/make_golden.py awq_b128_inputs)
    def __init__(self):
        super().__init__()
        nn = torch.nn
        self.net = nn.Sequential(
            nn.Linear(256, 2304), nn.ReLU(), nn.Linear(2304, 256), nn.ReLU(),
            nn.Linear(256, 1024, bias=False), nn.ReLU(), nn.Linear(1024, 256),
        )

    def forward(self, x):
        return self.net(x)


def _golden_run(gpu, inject_act_scale):
    import modelopt_amd.torch.quantization as mtq
    from modelopt_amd.torch.quantization import model_calib as MC

    t = load_file(str(G / "awq_b128.safetensors"))
    model = _WideMLP().to(torch.bfloat16)
    model.load_state_dict({k[3:]: v for k, v in t.items() if k.startswith("sd.")})
    model.to(gpu)
    data = [t[f"data{i}"].to(gpu) for i in range(3)]
    cfg = dict(mtq.INT4_AWQ_CFG)
    cfg["algorithm"] = {"method": "awq_lite", "alpha_step": 0.1, "debug": True}
    got = {}
    orig = MC._awq_sync_act_scale

    def sync(mods):
        orig(mods)
        for name, m in mods:
            got[name] = m.awq_lite.act_scale.clone()
            if inject_act_scale:
                m.awq_lite.act_scale = t[f"act_scale.{name}"].to(gpu)

    MC._awq_sync_act_scale = sync
    try:
        mtq.quantize(model, cfg, lambda mm: [mm(d) for d in data])
    finally:
        MC._awq_sync_act_scale = orig
    return model, t, got


def _check_downstream(model, t, names):
    for n, m in model.named_modules():
        if n not in names:
            continue
        h = m.awq_lite
        assert torch.equal(_bits(h.weight_scale), _bits(t[f"weight_scale.{n}"])), n
        assert torch.equal(_bits(h.best_scale), _bits(t[f"best_scale.{n}"])), n
        assert torch.equal(_bits(m.weight), _bits(t[f"weight.{n}"])), n
        assert torch.equal(_bits(m.weight_quantizer.amax), _bits(t[f"wamax.{n}"])), n
        assert torch.equal(_bits(m.input_quantizer.pre_quant_scale), _bits(t[f"pqs.{n}"])), n


def test_awq_b128_bit_exact_given_the_reference_act_scale(gpu):
    """With the reference's act_scale in place after the caching pass (the only input of the
    statistics that passes through a GEMM), weight_scale, best_scale, the folded weights, the INT4
    block amax and pre_quant_scale of every linear are bit-identical to the reference run (the
    alpha choice agrees on the golden's losses, which are >= 1.3 % apart)."""
    model, t, _ = _golden_run(gpu, inject_act_scale=True)
    names = [n for n, m in model.named_modules() if hasattr(m, "awq_lite")]
    assert len(names) == 4
    _check_downstream(model, t, set(names))


def test_awq_b128_first_linear_bit_exact_end_to_end(gpu):
    """net.0 reads the calibration batches themselves (no GEMM before it): its whole AWQ state --
    act_scale included -- equals the reference run bit for bit with nothing injected.  The later
    linears' act_scale differ only through the bf16 GEMM outputs that feed them (summation order);
    the differing fraction and size are bounded here and recorded in DESIGN.md §5."""
    model, t, got = _golden_run(gpu, inject_act_scale=False)
    assert torch.equal(_bits(got["net.0"]), _bits(t["act_scale.net.0"]))
    _check_downstream(model, t, {"net.0"})
    for n in ("net.2", "net.4", "net.6"):
        a, r = got[n].float().cpu(), t[f"act_scale.{n}"].float()
        frac = (a != r).float().mean().item()
        rel = ((a - r).abs() / r.abs().clamp_min(1e-30)).max().item()
        print(f"{n}: act_scale differs on {frac:.4f} of the channels, max relative {rel:.3g}")
        assert rel <= 2**-6, (n, rel)
