#!/usr/bin/env python3
"""Summarise scripts/gpu_export_pmc.sh TAG (MXFP4 export packer, bench input [32768, 4096] bf16):
per-launch duration (kernel trace), effective clock GRBM_GUI_ACTIVE / 8 XCDs / dispatch time
(MI355X_MICROARCH.md: reads high on dispatches under ~0.3 ms), and HBM bytes per launch from
FETCH_SIZE (x2, gfx950 wide-stream correction) and WRITE_SIZE against the algorithmic bytes.

    python scripts/export_pmc_summary.py TAG   ->   profiles/r04/export/export_mxfp4_pmc_TAG.json
"""
import csv
import json
import statistics
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
KERNEL = "export_mxfp4_vec_kernel"
N = 32768 * 4096


def rows(d: Path, name: str):
    f = next(d.rglob(name))
    return [r for r in csv.DictReader(open(f)) if KERNEL in r["Kernel_Name"]]


def main():
    tag = sys.argv[1]
    out = REPO / "gpurun_out"
    tr = rows(out / f"{tag}_trace", "*kernel_trace.csv")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr]
    res = {"kernel": KERNEL, "launches": len(dur), "duration_us": {
        "mean": round(statistics.mean(dur), 2), "min": round(min(dur), 2), "max": round(max(dur), 2),
        "stddev": round(statistics.pstdev(dur), 2)}}
    g = {}
    for r in rows(out / f"{tag}_grbm", "*counter_collection.csv"):
        e = g.setdefault(r["Dispatch_Id"], {"t": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        e[r["Counter_Name"]] = float(r["Counter_Value"])
    clk = [e["GRBM_GUI_ACTIVE"] / 8 / e["t"] / 1e9 for e in g.values() if "GRBM_GUI_ACTIVE" in e and e["t"] > 0]
    res["effective_clock_ghz"] = {"median": round(statistics.median(clk), 3), "min": round(min(clk), 3),
                                  "max": round(max(clk), 3), "note": "GRBM_GUI_ACTIVE / 8 / dispatch time; "
                                  "reads high on dispatches shorter than ~0.3 ms"}
    fetch = statistics.median(float(r["Counter_Value"]) for r in rows(out / f"{tag}_fetch", "*counter_collection.csv"))
    write = statistics.median(float(r["Counter_Value"]) for r in rows(out / f"{tag}_write", "*counter_collection.csv"))
    alg = N * 2 + N // 2 + N // 32
    hbm = fetch * 1024 * 2 + write * 1024
    res["traffic"] = {"read_bytes_corrected": fetch * 1024 * 2, "write_bytes": write * 1024,
                      "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": alg,
                      "traffic_over_algorithmic": round(hbm / alg, 4)}
    res["achieved_frac_of_8tbs_at_mean"] = round(alg / (res["duration_us"]["mean"] * 1e-6) / 8e12, 4)
    dst = REPO / "profiles" / "r04" / "export" / f"export_mxfp4_pmc_{tag}.json"
    dst.write_text(json.dumps(res, indent=1))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
