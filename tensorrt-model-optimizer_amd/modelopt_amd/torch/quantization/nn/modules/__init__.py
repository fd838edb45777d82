"""Quantized module wrappers."""

from .quant_linear import *  # noqa: F403
from .quant_module import *  # noqa: F403
from .tensor_quantizer import *  # noqa: F403
