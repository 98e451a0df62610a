#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc passes (tools/pmc.sh) per kernel: mean counter value per dispatch.
Usage: python tools/pmc_summary.py [gpurun_out/pmc] [--json out.json]"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "gpurun_out/pmc")
per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
for f in sorted(root.glob("*/run_counter_collection.csv")):
    acc = defaultdict(float)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("pbrt_amd::", "")
        acc[(k, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in acc.items():
        per[k][c].append(v)
out = {}
for k, cs in per.items():
    out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    out[k]["dispatches"] = max(len(v) for v in cs.values())
for k, cs in sorted(out.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {v:16.1f}")
if "--json" in sys.argv:
    Path(sys.argv[sys.argv.index("--json") + 1]).write_text(json.dumps(out, indent=1))
