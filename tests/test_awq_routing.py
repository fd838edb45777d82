"""AWQ-lite search routing (model_calib._awq_use_fused): which linears take the fused MFMA search
kernel and which the batched hipBLASLt path, per the r06 measurements."""
from modelopt_amd.torch.quantization.model_calib import _awq_use_fused


def test_llama3_8b_shapes_auto():
    M, G = 8192, 11
    # (N, K): k/v, q/o, gate/up fused; down_proj (K > N) on the library path
    assert _awq_use_fused(M, 1024, 4096, G, "auto")
    assert _awq_use_fused(M, 4096, 4096, G, "auto")
    assert _awq_use_fused(M, 14336, 4096, G, "auto")
    assert not _awq_use_fused(M, 4096, 14336, G, "auto")
    # narrow linears stay fused whatever K
    assert _awq_use_fused(M, 2048, 8192, G, "auto")


def test_modes_and_limits():
    M = 8192
    assert _awq_use_fused(M, 4096, 14336, 11, "always")
    assert not _awq_use_fused(M, 1024, 4096, 11, "library")
    assert not _awq_use_fused(M, 1024, 4096, 11, "never")
    assert not _awq_use_fused(M, 1024, 4096, 65, "always")   # > 64 alphas
    assert not _awq_use_fused(2**20, 1024, 4096, 11, "auto")  # 32-bit element offsets of x
