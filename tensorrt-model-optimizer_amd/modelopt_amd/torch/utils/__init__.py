"""Distributed helpers (reference: modelopt/torch/utils)."""
