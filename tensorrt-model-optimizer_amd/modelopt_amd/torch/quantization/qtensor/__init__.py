"""Real-quantized (packed) weight tensors for ``mtq.compress`` (reference: quantization/qtensor/).

Packing runs on the MI355X kernels where the product has one (FP8 per-tensor / per-channel,
NVFP4, MXFP4, MXFP8: the export packers of csrc/mtq_kernels.hip); INT4 / INT8 packing and every
dequantisation are the reference's own tensor expressions evaluated on the device.
"""

from .base_qtensor import BaseQuantizedTensor, QTensorWrapper, pack_real_quantize_weight
from .fp8_tensor import FP8QTensor
from .int4_tensor import INT4QTensor
from .int8_tensor import INT8QTensor
from .mxfp4_tensor import MXFP4QTensor
from .mxfp8_tensor import MXFP8QTensor
from .nvfp4_tensor import NVFP4QTensor

__all__ = [
    "BaseQuantizedTensor",
    "FP8QTensor",
    "INT4QTensor",
    "INT8QTensor",
    "MXFP4QTensor",
    "MXFP8QTensor",
    "NVFP4QTensor",
    "QTensorWrapper",
    "pack_real_quantize_weight",
]
