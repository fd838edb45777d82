"""Kernels shared by quantization and sparsity (reference ``modelopt/torch/kernels/common``)."""
