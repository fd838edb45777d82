"""Calibrators (reference: modelopt/torch/quantization/calib)."""

from .calibrator import _Calibrator
from .histogram import HistogramCalibrator
from .max import MaxCalibrator

__all__ = ["HistogramCalibrator", "MaxCalibrator", "_Calibrator"]
