#!/usr/bin/env python3
"""Summarise a rocprofv3 run database (rocpd SQLite, ROCm 7 default output) as JSON.

    python scripts/pmc_summary.py DB [--kernel SUBSTR] [--out FILE]

PMC runs: per kernel and counter, the mean / min / max over dispatches (SQ_* cycle counters
as rocprofv3 reports them: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles on
gfx950, MI355X_MICROARCH.md).  Kernel-trace runs: per kernel the dispatch count and the
mean / median duration in microseconds.
"""

import argparse
import json
import sqlite3
import statistics
import sys


def summarise(db: str, kernel: str | None) -> dict:
    c = sqlite3.connect(db)
    out: dict = {"db": db, "pmc": {}, "trace": {}}
    tabs = {r[0] for r in c.execute("select name from sqlite_master")}
    if "counters_collection" in tabs:
        q = "select kernel_name, counter_name, value from counters_collection"
        acc: dict = {}
        for name, ctr, val in c.execute(q):
            if kernel and kernel not in name:
                continue
            acc.setdefault(name, {}).setdefault(ctr, []).append(float(val))
        for name, ctrs in acc.items():
            out["pmc"][name] = {
                k: {"mean": statistics.fmean(v), "min": min(v), "max": max(v), "n": len(v)}
                for k, v in sorted(ctrs.items())
            }
    if "kernels" in tabs:
        cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
        name_col = "name" if "name" in cols else "kernel_name"
        acc = {}
        for name, s, e in c.execute(f"select {name_col}, start, end from kernels"):
            if kernel and kernel not in name:
                continue
            acc.setdefault(name, []).append((e - s) / 1e3)
        for name, d in acc.items():
            out["trace"][name] = {
                "dispatches": len(d),
                "mean_us": round(statistics.fmean(d), 3),
                "median_us": round(statistics.median(d), 3),
                "min_us": round(min(d), 3),
            }
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernel")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = summarise(a.db, a.kernel)
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    else:
        sys.stdout.write(txt + "\n")


if __name__ == "__main__":
    main()
