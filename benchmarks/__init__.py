"""Workload drivers that ``bench.py`` runs (PTQ wall-clock C2-C5, the fused-attention bench); also
runnable on their own (``python benchmarks/ptq_llama.py ...``).  Measurement code, not product."""
