#!/usr/bin/env python3
"""Per-launch kernel durations (us) from a rocprofv3 --kernel-trace directory, in launch order,
grouped by kernel: python3 tools/ktrace.py DIR [name-substring ...]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

f = next(Path(sys.argv[1]).rglob("*kernel_trace.csv"))
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
by = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("pbrt_amd::", "").split("(")[0]
    if "rocclr" in name:
        continue
    by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
keys = sys.argv[2:]
for name, d in by.items():
    if keys and not any(k in name for k in keys):
        continue
    print(f"{name[-34:]:34s} n={len(d):3d} sum={sum(d):9.1f}  " + " ".join(f"{x:.0f}" for x in d[:12]))
