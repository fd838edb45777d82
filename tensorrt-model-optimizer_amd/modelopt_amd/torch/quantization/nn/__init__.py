"""Quantization nn modules (reference: modelopt/torch/quantization/nn)."""

from .modules.quant_embedding import *  # noqa: F403
from .modules.quant_linear import *  # noqa: F403
from .modules.quant_module import *  # noqa: F403
from .modules.tensor_quantizer import *  # noqa: F403
