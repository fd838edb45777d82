"""MI355X-native ``modelopt.torch.quantization`` (PTQ fake-quant + calibration hot path).

``import modelopt_amd.torch.quantization as mtq`` gives the reference's API for this path:
``mtq.quantize / calibrate``, the preset configs (``mtq.FP8_DEFAULT_CFG`` ...), ``TensorQuantizer``,
``QuantModuleRegistry``, calibrators, and the functional ops -- backed by the HIP kernels of
``csrc/`` behind ``include/mtq_amd.h``.
"""

from . import calib, nn, plugins, tensor_quant, utils
from .config import *  # noqa: F403
from .conversion import *  # noqa: F403
from .extensions import get_cuda_ext, get_cuda_ext_fp8, get_cuda_ext_mx
from .model_calib import (
    apply_pre_quant_scale_and_smooth,
    awq,
    awq_lite,
    enable_stats_collection,
    finish_stats_collection,
    max_calibrate,
)
from .model_quant import *  # noqa: F403
from .nn.modules.quant_module import QuantModuleRegistry
from .nn.modules.tensor_quantizer import (
    SequentialQuantizer,
    StaticBlockScaleQuantizer,
    TensorQuantizer,
    register_quant_backend,
    unregister_quant_backend,
)
from . import qtensor
from .compress import CompressConfig, RealQuantLinear, compress, is_real_quantized
from .utils.core_utils import update_quant_cfg_with_kv_cache_quant
