"""Calibrators (reference: modelopt/torch/quantization/calib)."""

from .calibrator import _Calibrator
from .histogram import HistogramCalibrator
from .max import MaxCalibrator
from .mse import MseCalibrator, NVFP4MSECalibrator

__all__ = ["HistogramCalibrator", "MaxCalibrator", "MseCalibrator", "NVFP4MSECalibrator", "_Calibrator"]
