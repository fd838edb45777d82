#!/usr/bin/env python3
"""GPU busy time vs span from a rocprofv3 kernel-trace CSV: the union of kernel intervals, the idle
gaps between them (histogram), and the busy time per 1-second window -- where a PTQ run's wall
clock goes beyond its kernels.  python scripts/trace_gaps.py <kernel_trace.csv> [out.json]"""
import csv
import json
import sys


def main():
    path = sys.argv[1]
    iv = []
    names = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            iv.append((s, e, row["Kernel_Name"]))
    iv.sort()
    busy = 0
    gaps = []
    cur_s, cur_e = iv[0][0], iv[0][1]
    for s, e, n in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    edges = [1e3, 1e4, 1e5, 1e6, 1e7, 1e12]
    hist = {}
    lo = 0
    for hi in edges:
        sel = [g for g, _, _ in gaps if lo <= g < hi]
        hist[f"{lo / 1e3:g}-{hi / 1e3:g}us"] = {"n": len(sel), "total_ms": round(sum(sel) / 1e6, 2)}
        lo = hi
    big = sorted(gaps, reverse=True)[:15]
    out = {
        "kernels": len(iv),
        "span_s": round(span / 1e9, 3),
        "busy_s": round(busy / 1e9, 3),
        "idle_s": round((span - busy) / 1e9, 3),
        "gap_hist": hist,
        "largest_gaps": [{"ms": round(g / 1e6, 2), "at_s": round((t - iv[0][0]) / 1e9, 3), "next": n[:90]}
                         for g, t, n in big],
    }
    for s, e, n in iv:
        names[n] = names.get(n, 0) + (e - s)
    out["top_kernels_s"] = {k[:110]: round(v / 1e9, 3) for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:25]}
    txt = json.dumps(out, indent=1)
    print(txt)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)


if __name__ == "__main__":
    main()
