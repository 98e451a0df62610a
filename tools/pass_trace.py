#!/usr/bin/env python3
"""Per-launch kernel durations of one render pass from a rocprofv3 kernel trace."""
import csv
import sys

f = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("pbrt_amd::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
       for r in rows]
cams = [i for i, x in enumerate(seq) if x[0] == "k_camera"]
i0, i1 = cams[-2], cams[-1]
prev = None
tot = 0
for name, s, e in seq[i0:i1]:
    print(f"  {name:32s} {(e - s) / 1000:8.1f} us   gap {(s - prev) / 1000 if prev else 0:6.1f}")
    tot += (e - s) / 1000
    prev = e
print(f"  pass: {(seq[i1][1] - seq[i0][1]) / 1000:.1f} us wall, {tot:.1f} us in kernels")
