#!/usr/bin/env python3
"""Turn rocprofv3 PMC passes into the bench's `roofline.traffic` figure and archive the summaries.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports
exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane stores.  The two counters are collected in separate passes
(FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2).  Traffic per launch = median over the dispatches of
the named kernel.

    python scripts/pmc_traffic.py TAG [--kernel Fp8AxisVecOp]
reads gpurun_out/{pmc_fetch_TAG,pmc_write_TAG,prof_TAG}/ and writes profiles/traffic_TAG.json and
profiles/TAG/*.csv.
"""

import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def per_dispatch(path: Path, kernel: str, counter: str):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1]
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "Fp8AxisVecOp"
    out = REPO / "gpurun_out"
    fetch = per_dispatch(out / f"pmc_fetch_{tag}" / "pmc_counter_collection.csv", kernel, "FETCH_SIZE")
    write = per_dispatch(out / f"pmc_write_{tag}" / "pmc_counter_collection.csv", kernel, "WRITE_SIZE")
    f_med, w_med = statistics.median(fetch), statistics.median(write)
    read_bytes = f_med * 1024 * 2  # gfx950 FETCH_SIZE = half the bytes of a 16 B/lane stream
    write_bytes = w_med * 1024
    res = {
        "kernel_config": "fp8_block128_bf16_32768x4096",
        "kernel_match": kernel,
        "dispatches": [len(fetch), len(write)],
        "fetch_size_kib_median": f_med,
        "write_size_kib_median": w_med,
        "read_bytes_corrected": read_bytes,
        "write_bytes": write_bytes,
        "hbm_bytes_per_launch": int(read_bytes + write_bytes),
        "algorithmic_bytes_per_launch": 32768 * 4096 * 4 + (32768 * 4096 // 128) * 4,
        "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), KiB x1024",
    }
    res["traffic_over_algorithmic"] = round(res["hbm_bytes_per_launch"] / res["algorithmic_bytes_per_launch"], 4)
    (REPO / "profiles").mkdir(exist_ok=True)
    (REPO / "profiles" / f"traffic_{tag}.json").write_text(json.dumps(res, indent=1))
    dst = REPO / "profiles" / tag
    dst.mkdir(parents=True, exist_ok=True)
    for src in [out / f"prof_{tag}" / "trace_kernel_stats.csv", out / f"prof_{tag}" / "trace_domain_stats.csv"]:
        if src.exists():
            shutil.copy(src, dst / src.name)
    for d in (f"pmc_fetch_{tag}", f"pmc_write_{tag}"):
        src = out / d / "pmc_counter_collection.csv"
        if src.exists():
            rows = [r for r in csv.DictReader(open(src)) if kernel in r["Kernel_Name"]]
            with open(dst / f"{d}_dominant_kernel.csv", "w", newline="") as f:
                if rows:
                    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
                    w.writeheader()
                    w.writerows(rows)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
