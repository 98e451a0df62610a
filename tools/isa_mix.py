#!/usr/bin/env python3
"""Instruction mix per kernel of the gfx950 assembly (hipcc --cuda-device-only -S)."""
import re
import subprocess
import sys

src = "/root/repo/pbrt-v4_amd/csrc/kernels/wavefront.hip"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                       "-I/root/repo/pbrt-v4_amd/csrc", "--cuda-device-only", "-S", src, "-o", "/tmp/wf.s"],
                      stderr=subprocess.DEVNULL)
s = open("/tmp/wf.s").read()
names = sys.argv[1:] or ["k_camera", "k_closest", "k_shade_diffuse", "k_shadow", "k_film"]
pats = ["ds_read", "ds_write", "flat_load", "global_load", "global_store", "global_atomic", "scratch_", "s_waitcnt",
        "v_div_scale", "v_sqrt", "v_rcp", "s_cbranch"]
for k in names:
    m = re.search(r"^(_ZN8pbrt_amd\d+" + k + r"E\S*):.*?\n(.*?)\.Lfunc_end", s, re.S | re.M)
    if not m:
        print(k, "not found")
        continue
    body = m.group(2)
    lines = [l for l in body.split("\n") if l.startswith("\t") and not l.startswith("\t.") and not l.startswith("\t;")]
    cnt = {p: sum(1 for l in lines if l.split()[0].startswith(p)) for p in pats}
    print(f"{k}: {len(lines)} instrs", " ".join(f"{p}={v}" for p, v in cnt.items() if v))
