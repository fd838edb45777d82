"""AWQ-lite caching pass: linears that read the same input tensor (q/k/v_proj, gate/up_proj) share
one act-scale computation (model_calib._act_scale_shared); a new tensor, or the same tensor after
an in-place change, is computed again.  Values are the reference's get_act_scale
(model_calib.py:1471-1472)."""
import torch

from modelopt_amd.torch.quantization import model_calib


def test_act_scale_shared_per_tensor(monkeypatch):
    calls = []
    real = model_calib.get_act_scale

    def counting(x):
        calls.append(x)
        return real(x)

    monkeypatch.setattr(model_calib, "get_act_scale", counting)
    x = torch.randn(2, 5, 8).to(torch.bfloat16)
    a = model_calib._act_scale_shared(x)
    b = model_calib._act_scale_shared(x)
    assert len(calls) == 1 and a is b
    assert torch.equal(a, x.abs().contiguous().view(-1, 8).mean(0).to(torch.float32))
    x.mul_(2)  # same object, new version: recomputed
    c = model_calib._act_scale_shared(x)
    assert len(calls) == 2 and torch.equal(c, real(x))
    y = x.clone()  # equal values, another tensor: recomputed
    model_calib._act_scale_shared(y)
    assert len(calls) == 3


def test_act_scale_shared_inference_tensor():
    """Inference tensors have no version counter: the memo is bypassed."""
    with torch.inference_mode():
        x = torch.randn(3, 8)
        a = model_calib._act_scale_shared(x)
    assert torch.equal(a, x.abs().view(-1, 8).mean(0))


def test_awq_lite_forward_loop_under_inference_mode():
    """awq_lite with a forward_loop under torch.inference_mode() (CPU), equal to the same
    calibration under no_grad; the act-scale memo is empty after the caching pass."""
    import torch.nn as nn

    import modelopt_amd.torch.quantization as mtq

    cfg = {
        "quant_cfg": [
            {"quantizer_name": "*", "enable": False},
            {"quantizer_name": "*weight_quantizer", "cfg": {"num_bits": 4, "block_sizes": {-1: 8, "type": "static"}}},
        ],
        "algorithm": {"method": "awq_lite", "alpha_step": 0.25},
    }
    g = torch.Generator().manual_seed(3)
    data = [torch.randn(8, 16, generator=g) for _ in range(2)]

    def build():
        torch.manual_seed(1)
        return nn.Sequential(nn.Linear(16, 32), nn.ReLU(), nn.Linear(32, 16))

    def loop_inf(m):
        with torch.inference_mode():
            for d in data:
                m(d)

    def loop_ng(m):
        with torch.no_grad():
            for d in data:
                m(d)

    a = mtq.quantize(build(), cfg, loop_inf)
    assert model_calib._act_scale_memo == [None, None, None]
    b = mtq.quantize(build(), cfg, loop_ng)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb and torch.equal(pa, pb), na
