"""MI355X-native counterpart of ``modelopt.torch`` (quantization hot path only)."""
