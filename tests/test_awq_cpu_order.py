"""The host restatement (oracle/awq_cpu_order.c) of the two CPU operation sequences behind the
reference's AWQ-lite statistics, pinned against torch's own CPU ops -- the understanding the
device kernels (csrc/mtq_awq_scale.hip) are written from:

* ATen's vectorised powf (torch CPU ``pow(Tensor, Scalar)``, get_scale model_calib.py:1474-1487)
  -- bit-identical on every exponent of the alpha grids awq_lite builds (step 0.1 and 0.05);
  the elements past the 32-wide vector loop and the special exponents (0, 1, 0.5) take other
  paths, as the kernel does;
* ATen's CPU column sum (the means of get_act_scale / get_weight_scale, :1453-1472): the
  four-level cascade per column in groups of 32 columns, ``row_sum`` for the K % 32 rest.

Runs on the CPU of whichever host runs the suite; it needs the same vector ISA family as the
container that made the goldens (AVX-512) for the vector-loop width, and skips otherwise."""

import numpy as np
import pytest
import torch

from oracle import cpu_order

pytestmark = pytest.mark.skipif(torch.backends.cpu.get_cpu_capability() != "AVX512",
                                reason="the golden runs' ATen vector width (AVX-512) is what is restated")


def _alphas(step):
    return [k.item() for k in torch.arange(0, 1.0 + step, step)]


@pytest.mark.parametrize("step", [0.1, 0.05])
def test_powf_restatement_matches_torch_cpu_pow(step):
    g = torch.Generator().manual_seed(11)
    x = ((torch.rand(1 << 18, generator=g) * 40 - 20).exp2()).contiguous()
    for a in _alphas(step):
        for e in (a, 1 - a):
            if float(np.float32(e)) in (0.0, 1.0, 0.5):
                continue  # ATen's special exponents (fill / copy / sqrt)
            want = x.pow(e).numpy()
            got = cpu_order.powf(x.numpy(), float(np.float32(e)))
            assert np.array_equal(got.view(np.int32), want.view(np.int32)), e


def test_powf_tail_elements_take_the_scalar_libm_path():
    """Elements past the last whole 32-element vector step: the scalar ``std::pow(float, double)``
    with the exponent kept in double (the vector loop casts it to float), a double evaluation
    rounded once to float -- what the device kernel restates it as."""
    g = torch.Generator().manual_seed(12)
    x = ((torch.rand(20000, generator=g) * 40 - 20).exp2())
    for e in (0.1, 0.30000001192092896, 0.8999999985098839):
        tail = torch.stack([x[i:i + 1].pow(e)[0] for i in range(2000)])  # 1-element tensors: all tail
        dbl = torch.from_numpy(np.power(x[:2000].double().numpy(), e).astype(np.float32))
        assert torch.equal(tail, dbl), e


@pytest.mark.parametrize("M,K", [(1, 64), (3, 40), (192, 256), (255, 100), (1000, 48), (4097, 96), (8192, 64),
                                 (14336, 40), (300, 4101)])
def test_col_sum_restatement_matches_torch_cpu_sum(M, K):
    g = torch.Generator().manual_seed(M + K)
    x = (torch.randn(M, K, generator=g) * torch.exp2(torch.rand(K, generator=g) * 10 - 5)).abs()
    want = x.sum(0).numpy()
    got = cpu_order.col_sum(x.numpy())
    assert np.array_equal(got.view(np.int32), want.view(np.int32))
    # the mean of a bf16 tensor: fp32 sum of the upcast values, true division, cast back
    xb = x.to(torch.bfloat16)
    m = torch.from_numpy(cpu_order.col_sum(xb.float().numpy()) / np.float32(M)).to(torch.bfloat16)
    assert torch.equal(m.view(torch.int16), xb.mean(0).view(torch.int16))
