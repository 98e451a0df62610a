#!/usr/bin/env python3
"""Traversal work per ray on the bench workload (profiling build: PBRT_AMD_TRAV_STATS).
Run on the GPU box: make -C pbrt-v4_amd prof && python tools/trav_stats.py [c2|c3|c4]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("PBRT_AMD_LIB", str(ROOT / "pbrt-v4_amd" / "lib" / "libpbrt_amd_prof.so"))
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401
import bench

import json

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
sys.argv = ["bench.py", "--workload", wl, "--spp", "4"]
a = bench.parse()
import pbrt_amd as pa
sc = bench.load(a)
integ = pa.WavefrontPathIntegrator(sc, device=0)
integ.render(n_samples=1)
integ.synchronize()
integ.reset_stats()
integ.render()
integ.synchronize()
c = integ.kernel_sections(32)
rec = {"workload": wl, "spp": 4, "note": "BVH8 group traversal work per ray (PBRT_AMD_TRAV_STATS build); "
       "wave figures are the per-wave maxima over lanes, averaged over waves"}
for name, b in (("closest", 8), ("shadow", 16)):
    rays, waves = max(c[b + 4], 1), max(c[b + 5], 1)
    rec[name] = {"rays": c[b + 4], "nodes_per_ray": c[b] / rays, "tris_per_ray": c[b + 1] / rays,
                 "wave_max_nodes": c[b + 2] / waves, "wave_max_tris": c[b + 3] / waves}
    print(f"{name:8s} rays {c[b+4]:>11d}  per ray: nodes {c[b]/rays:6.2f} tris {c[b+1]/rays:6.2f}  "
          f"per wave (max lane): nodes {c[b+2]/waves:6.2f} tris {c[b+3]/waves:6.2f}  lanes/wave {rays/waves:5.1f}")
if out_json:
    Path(out_json).write_text(json.dumps(rec, indent=1) + "\n")
