"""Framework plugins: on-the-fly registration of model-specific quantized modules.

Reference: modelopt/torch/quantization/plugins/custom.py (register_custom_model_plugins_on_the_fly)
and plugins/huggingface.py.  Only the HF MoE paths on the PTQ hot path are provided
(``huggingface.py``: fused experts, sparse sequential MoE).
"""

from __future__ import annotations

_ON_THE_FLY = []


def register_on_the_fly(fn):
    _ON_THE_FLY.append(fn)
    return fn


def register_custom_model_plugins_on_the_fly(model):
    for fn in _ON_THE_FLY:
        fn(model)


try:  # transformers is optional
    from . import huggingface  # noqa: F401
except ImportError:  # pragma: no cover
    pass
