#!/usr/bin/env python3
"""C3 alone (Llama-3-8B dims, INT4_AWQ_CFG, 512 x 512 tokens, batch 16): one JSON line with the
PTQ wall-clock; for rocprofv3 kernel traces of the AWQ-lite path without the rest of bench.py.
    python scripts/run_c3.py"""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "tensorrt-model-optimizer_amd"), str(REPO)]
from benchmarks import ptq_llama  # noqa: E402

r = ptq_llama.run(samples=512, seq=512, rank=0, world=1, baseline=False, config="INT4_AWQ_CFG")
print(json.dumps({k: v for k, v in r.items() if not isinstance(v, (dict, list))}))
