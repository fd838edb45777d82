"""MI355X-native kernels behind the reference's ``modelopt.torch.kernels`` interfaces."""
