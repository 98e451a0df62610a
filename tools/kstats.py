#!/usr/bin/env python3
"""Compact per-kernel summary of a rocprofv3 --stats directory: calls, mean us, total share."""
import csv
import sys
from pathlib import Path

f = next(Path(sys.argv[1]).rglob("*kernel_stats.csv"))
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:14]:
    name = r["Name"].replace("pbrt_amd::", "").split("(")[0][:40]
    print(f"   {name:40s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.1f} us {100*float(r['TotalDurationNs'])/tot:6.1f}%")
