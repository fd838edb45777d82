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
