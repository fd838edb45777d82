#!/usr/bin/env python3
"""Kernel durations from a rocprofv3 SQLite output (rocpd `kernels` view), grouped by kernel name
and grid size:  python scripts/rocpd_kernels.py <results.db> [name-substring]"""
import collections
import json
import sqlite3
import sys


def main():
    db, sub = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    c = sqlite3.connect(db)
    agg = collections.defaultdict(list)
    order = []
    for n, g, wg, d in c.execute("select name, grid_x, workgroup_x, duration from kernels order by start"):
        if sub not in n:
            continue
        key = f"{n.split('(')[0][-70:]} grid={g} wg={wg}"
        if key not in agg:
            order.append(key)
        agg[key].append(d / 1e3)
    out = {}
    for k in order:
        ds = sorted(agg[k])
        out[k] = {"n": len(ds), "median_us": round(ds[len(ds) // 2], 2), "min_us": round(ds[0], 2),
                  "mean_us": round(sum(ds) / len(ds), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
