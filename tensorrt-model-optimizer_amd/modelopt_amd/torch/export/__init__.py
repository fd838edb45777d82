"""Checkpoint export of fake-quant models (reference: modelopt/torch/export)."""

from .convert_hf_config import convert_hf_quant_config_format  # noqa: F401
from .model_config import *  # noqa: F401,F403
from .quant_utils import *  # noqa: F401,F403
from .unified_export_hf import export_hf_checkpoint, requantize_resmooth_fused_llm_layers  # noqa: F401
