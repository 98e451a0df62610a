#!/usr/bin/env python3
"""C4 k_closest HBM traffic record (round 3): rocprofv3 PMC passes FETCH_SIZE, WRITE_SIZE and
TCC_HIT/TCC_MISS (each its own run, tools/pmc.sh) -> per-launch bytes and bytes
per ray next to the algorithmic bytes of the bench line.  FETCH_SIZE is doubled (gfx950
correction, MI355X_MICROARCH.md HBM section); values are KB per dispatch.
Usage: python tools/c4_pmc_json.py gpurun_out/pmc BENCH_LINE.json profiles/r03_c4_closest_pmc.json HEAD
(gpurun_out/pmc as tools/pmc.sh writes it: fetch/, write/, tcc/ passes)"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_dispatch(csv_path, counter, kernel="k_closest"):
    acc = defaultdict(float)
    for r in csv.DictReader(open(csv_path)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0]
        if name.endswith(kernel) and r["Counter_Name"] == counter:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = list(acc.values())
    return sum(v) / len(v), len(v)


src, bench_path, dst = Path(sys.argv[1]), Path(sys.argv[2]), Path(sys.argv[3])
head = sys.argv[4] if len(sys.argv) > 4 else "unknown"
label = sys.argv[5] if len(sys.argv) > 5 else "C4: 9,994,244 triangles"
fetch, n = per_dispatch(src / "fetch" / "run_counter_collection.csv", "FETCH_SIZE")
write, _ = per_dispatch(src / "write" / "run_counter_collection.csv", "WRITE_SIZE")
hit, _ = per_dispatch(src / "tcc" / "run_counter_collection.csv", "TCC_HIT_sum")
miss, _ = per_dispatch(src / "tcc" / "run_counter_collection.csv", "TCC_MISS_sum")
bench = json.loads(bench_path.read_text().strip().splitlines()[-1])
rays = bench["roofline"]["rays_per_launch"]
fetch_b, write_b = 2 * 1024 * fetch, 1024 * write
rec = {
    "kernel": f"k_closest ({label}, quantised BVH8 nodes, 6 waves/SIMD, rays binned at depth >= 1)",
    "head": head,
    "dispatches": n,
    "fetch_size_kb_mean": fetch,
    "write_size_kb_mean": write,
    "hbm_bytes_per_launch": round(fetch_b + write_b),
    "rays_per_launch": rays,
    "hbm_bytes_per_ray": round((fetch_b + write_b) / rays, 2),
    "fetched_bytes_per_ray": round(fetch_b / rays, 2),
    "algorithmic_bytes_per_ray": bench["roofline"]["bytes_per_ray"],
    # SURVEY 8(d)'s BVH term (round 4): HBM-resident nodes + triangles touched once per launch
    "bvh_bytes_per_launch": bench["roofline"].get("bvh_bytes_per_launch"),
    "algorithmic_bytes_per_launch": bench["roofline"].get("algorithmic_bytes_per_launch"),
    "tcc_hit_per_launch": hit,
    "tcc_miss_per_launch": miss,
    "l2_hit_rate": round(hit / (hit + miss), 4),
    "mean_launch_us": bench["roofline"]["mean_launch_us"],
    "bench_value_msamples_s": bench["value"],
    "note": ("PMC dispatches average all depths of one bench step's render; rays_per_launch and the launch time "
             "are the bench line's event-timed launches"),
}
dst.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps(rec, indent=1))
