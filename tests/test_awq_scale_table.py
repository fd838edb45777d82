"""AWQ-lite search tables: model_calib._scale_table (the [G, K] stack built with batched ops) is
bit-identical to stacking the reference's per-alpha get_scale (model_calib.py:1474-1487) --
including zero and tiny activation / weight scales and the special-cased exponents 0, 0.5, 1."""
import torch

from modelopt_amd.torch.quantization import model_calib as MC


def test_scale_table_bit_identical_to_per_alpha():
    g = torch.Generator().manual_seed(0)
    alphas = [k.item() for k in torch.arange(0, 1.0 + 0.1, 0.1)]
    for K in (1, 7, 4096):
        x = torch.rand(K, generator=g) * 3
        w = torch.rand(K, generator=g)
        if K > 4:
            x[0], w[1], x[2], w[3] = 0.0, 0.0, 1e-30, 1e-38
        want = torch.stack([MC.get_scale(x, w, a, None) for a in alphas])
        got = MC._scale_table(x, w, alphas)
        assert torch.equal(got.view(torch.int32), want.view(torch.int32)), K
    fine = [k.item() for k in torch.arange(0, 1.0 + 0.01, 0.01)]
    x, w = torch.rand(64, generator=g), torch.rand(64, generator=g)
    want = torch.stack([MC.get_scale(x, w, a, None) for a in fine])
    assert torch.equal(MC._scale_table(x, w, fine).view(torch.int32), want.view(torch.int32))


import pytest  # noqa: E402


@pytest.mark.gpu
def test_scale_table_bit_identical_on_gpu(gpu):
    g = torch.Generator(device=gpu).manual_seed(1)
    alphas = [k.item() for k in torch.arange(0, 1.0 + 0.1, 0.1)]
    for K in (4096, 14336):
        x = torch.rand(K, device=gpu, generator=g) * 3
        w = torch.rand(K, device=gpu, generator=g)
        x[0], w[1] = 0.0, 0.0
        want = torch.stack([MC.get_scale(x, w, a, None) for a in alphas])
        got = MC._scale_table(x, w, alphas)
        assert torch.equal(got.view(torch.int32), want.view(torch.int32)), K
