"""MI355X-native (gfx950 / CDNA4) PTQ fake-quantization and calibration.

Drop-in for the hot path of ``modelopt.torch.quantization``: ``import modelopt_amd.torch.quantization
as mtq`` exposes ``mtq.quantize`` / ``TensorQuantizer`` / ``QuantModule`` with the reference's
names and semantics, backed by hand-written HIP kernels (``csrc/``) behind the C ABI of
``include/mtq_amd.h``.
"""

__version__ = "0.1.0"
