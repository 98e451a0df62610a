#!/usr/bin/env python3
"""Write the k_closest HBM-traffic record that bench.py reports as roofline.traffic.

Input: the rocprofv3 PMC passes of tools/pmc.sh (FETCH_SIZE and WRITE_SIZE each in its own
pass, values in KB per dispatch) plus the bench JSON line those runs printed (rays/launch).
gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a
wide coalesced read, so it is doubled; WRITE_SIZE is used as is.
With the sq1 / sq2 passes present it adds the kernel's compute roof: VALU issue = 2 cycles x
SQ_INSTS_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) -- a wave64 fp32 VALU instruction
occupies its SIMD for 2 cycles at full rate (MI355X_MICROARCH.md, v_fma_f32 throughput; 8 for
transcendentals, so this is a lower bound) -- and, per wave, SQ_ACTIVE_INST_VALU /
SQ_WAVE_CYCLES and SQ_WAIT_ANY / SQ_WAVE_CYCLES.
Usage: python tools/closest_pmc_json.py gpurun_out/pmc profiles/r05_c2_closest_pmc.json [kernel] [--head SHA]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def per_dispatch(csv_path, kernel, counter):
    acc = defaultdict(float)
    for r in csv.DictReader(open(csv_path)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0]
        if name.endswith(kernel) and r["Counter_Name"] == counter:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(acc.values())


def bench_line(log):
    for line in open(log):
        if line.startswith('{"metric"'):
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


args = [a for a in sys.argv[1:]]
head = None
if "--head" in args:
    i = args.index("--head")
    head = args[i + 1]
    del args[i:i + 2]
src, dst = Path(args[0]), Path(args[1])
kernel = args[2] if len(args) > 2 else "k_closest"
fetch = per_dispatch(src / "fetch" / "run_counter_collection.csv", kernel, "FETCH_SIZE")
write = per_dispatch(src / "write" / "run_counter_collection.csv", kernel, "WRITE_SIZE")
b = bench_line(src / "fetch.log")
fetch_b = 2 * 1024 * sum(fetch) / len(fetch)
write_b = 1024 * sum(write) / len(write)
rays = b["roofline"]["rays_per_launch"]
rec = {
    "kernel": kernel,
    "dispatches": len(fetch),
    "fetch_size_kb_mean": sum(fetch) / len(fetch),
    "write_size_kb_mean": sum(write) / len(write),
    "fetch_bytes_corrected": fetch_b,
    "write_bytes": write_b,
    "hbm_bytes_per_launch": round(fetch_b + write_b),
    "rays_per_launch": rays,
    "hbm_bytes_per_ray": round((fetch_b + write_b) / rays, 2),
    "algorithmic_bytes_per_ray": b["roofline"]["bytes_per_ray"],
    "bench_config": b["config"]["workload"],
    "note": "FETCH_SIZE x2 per the gfx950 correction; 4-byte-per-lane SoA accesses are not calibrated "
            "by the guide, so the corrected read figure is an upper estimate",
}
def mean(pass_, counter):
    f = src / pass_ / "run_counter_collection.csv"
    if not f.exists():
        return None
    v = per_dispatch(f, kernel, counter)
    return sum(v) / len(v) if v else None


valu, wave, wait, grbm = (mean("sq2", "SQ_ACTIVE_INST_VALU"), mean("sq1", "SQ_WAVE_CYCLES"),
                          mean("sq2", "SQ_WAIT_ANY"), mean("sq2", "GRBM_GUI_ACTIVE"))
insts = mean("sq1", "SQ_INSTS_VALU")
if insts is not None and grbm:
    rec["valu_busy"] = round(2 * insts / (1024 * grbm / 8), 4)
    rec["valu_insts_per_launch"] = round(insts)
    rec["grbm_gui_active_per_xcd"] = round(grbm / 8)
if valu is not None and wave:
    rec["valu_active_per_wave"] = round(valu / wave, 4)
if wait is not None and wave:
    rec["wait_any_per_wave"] = round(wait / wave, 4)
if head:
    rec["head"] = head
dst.write_text(json.dumps(rec, indent=1) + "\n")
print(json.dumps(rec, indent=1))
