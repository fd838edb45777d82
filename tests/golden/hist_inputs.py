"""Deterministic inputs of the histogram goldens (``calib_ref.*``), shared by the generator
(``make_golden.py gen_calib_ref``, run against the reference) and the tests: integer arithmetic
only, no RNG, so both sides build the very same tensors."""

import torch


def peaked(n: int = 40_000_000, scale: float = 1.0, zeros_every: int = 0) -> torch.Tensor:
    """bf16 [n // 4000, 4000]: 80 % of the elements share one value (one histogram bin holds
    ~32 M > 2^24 counts), the rest spread over [0, 3 * scale) by a multiplicative hash, every
    second element negative; optionally every ``zeros_every``-th element zero."""
    i = torch.arange(n, dtype=torch.int64)
    spread = ((i * 2654435761) % 4093).to(torch.float32) * (3.0 * scale / 4093)
    x = torch.where(i % 5 != 0, torch.full_like(spread, 0.01 * scale), spread)
    x = torch.where(i % 2 == 1, -x, x)
    if zeros_every:
        x = torch.where(i % zeros_every == 0, torch.zeros_like(x), x)
    return x.to(torch.bfloat16).reshape(-1, 4000)
