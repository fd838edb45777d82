"""MTQ_AMD_REGISTER_TENSORRT_OPS=1 at import registers the reference's own op names
(tensorrt::quantize_op, tensor_quant.py:222-237) on the product kernels (here: the CPU dispatch key,
the C1 host path); without it the namespace stays untouched."""

import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
PROBE = """
import sys, torch
sys.path[:0] = [{pkg!r}]
import modelopt_amd.torch.quantization as mtq
from modelopt_amd.torch.quantization import tensor_quant as tq
print(tq.REFERENCE_OP_NAMES_REGISTERED)
if tq.REFERENCE_OP_NAMES_REGISTERED:
    x = torch.randn(64, 256).to(torch.bfloat16)
    a = x.view(-1, 128).float().abs().amax(dim=1, keepdim=True)
    y = torch.ops.tensorrt.quantize_op(x.view(-1, 128), a, 8, 4, False, False)
    z = torch.ops.modelopt_amd.quantize_op(x.view(-1, 128), a, 8, 4, False, False)
    print(bool(torch.equal(y.view(torch.int16), z.view(torch.int16))))
"""


def _run(flag):
    env = dict(os.environ)
    env.pop("MTQ_AMD_REGISTER_TENSORRT_OPS", None)
    if flag:
        env["MTQ_AMD_REGISTER_TENSORRT_OPS"] = "1"
    code = PROBE.format(pkg=str(REPO / "tensorrt-model-optimizer_amd"))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout.split()


def test_env_switch_registers_reference_op_names():
    assert _run(True) == ["True", "True"]


def test_default_leaves_tensorrt_namespace_alone():
    assert _run(False) == ["False"]
