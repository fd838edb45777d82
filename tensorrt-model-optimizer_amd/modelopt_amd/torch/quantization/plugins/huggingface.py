"""HuggingFace plugins (filled in with the MoE fused-experts path)."""
