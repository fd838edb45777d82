#!/usr/bin/env python3
"""Mean per dispatch of every PMC counter for kernels matching SUBSTR, over rocprofv3 CSV runs.

    python scripts/pmc_csv_summary.py DIR SUBSTR   (reads DIR/**/*counter_collection.csv)"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

root, sub = Path(sys.argv[1]), sys.argv[2]
acc = defaultdict(list)
for f in root.rglob("*counter_collection.csv"):
    per = defaultdict(float)  # (dispatch, counter) -> summed over dimensions
    for r in csv.DictReader(open(f)):
        if sub not in r.get("Kernel_Name", ""):
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        acc[c].append(v)
print(json.dumps({c: {"mean": sum(v) / len(v), "n": len(v)} for c, v in sorted(acc.items())}, indent=1))
