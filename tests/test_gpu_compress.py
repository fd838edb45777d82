"""mtq.compress on the GPU for every format the reference compresses (FP8, INT8, INT4, NVFP4, MXFP4,
MXFP8): packed bytes, scale buffers and dequantised weights bit-exact vs the reference's own
compress (tests/golden/compress.*), logits within bf16 GEMM-order tolerance; and the MXFP8 branch of
the unified HF export bit-exact vs the reference's export."""

import json

import pytest
import torch
from safetensors.torch import load_file

from compress_cases import CASES, META, build, check_compressed

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", CASES)
def test_compress_matches_reference(gpu, case):
    import modelopt_amd.torch.quantization as mtq

    m, t = build(case, gpu)
    mtq.compress(m)
    bad = check_compressed(case, m, t)
    assert not bad, bad[:6]
    with torch.no_grad():
        logits = m(t["test_ids"].to(gpu)).logits.float().cpu()
    torch.testing.assert_close(logits, t[f"{case}.logits"], rtol=2e-2, atol=2e-2)


def test_mxfp8_kernel_vs_oracle(gpu):
    from modelopt_amd import _ext
    from oracle import ref_ops as R

    g = torch.Generator().manual_seed(3)
    for dt in (torch.bfloat16, torch.float16):
        w = (torch.randn(48, 256, generator=g) * torch.logspace(-4, 2, 256)).to(dt)
        w[0, :32] = 0
        w[1, 5] = float("nan")
        w[2, 7] = float("inf")
        w[3, :32] = 2.0 ** -20  # tiny block
        q, s = _ext.ops().export_mxfp8(w.to(gpu))
        rq, rs = R.mxfp8_quantize(w)
        assert torch.equal(s.cpu(), rs), (s.cpu() != rs).nonzero()[:5]
        a, b = q.cpu().view(torch.uint8), rq.view(torch.uint8)
        assert torch.equal(a, b), (a != b).nonzero()[:5]


def test_mxfp8_export_matches_reference(gpu, tmp_path):
    from modelopt_amd.torch.export import export_hf_checkpoint

    m, t = build("mxfp8_export", gpu, prefix="mxfp8_export")
    export_hf_checkpoint(m, export_dir=str(tmp_path))
    got = load_file(str(tmp_path / "model.safetensors"))
    want = {k[len("mxfp8_export.export."):]: v for k, v in t.items() if k.startswith("mxfp8_export.export.")}
    assert set(got) == set(want), sorted(set(got) ^ set(want))[:10]
    bad = [k for k, v in want.items()
           if not torch.equal(got[k].view(torch.uint8) if got[k].element_size() == 1 else got[k], v)]
    assert not bad, bad[:8]
    hq = json.loads((tmp_path / "hf_quant_config.json").read_text())
    hq["producer"]["version"] = None
    assert hq == META["mxfp8_export"]["hf_quant_config"]
