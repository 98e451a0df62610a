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

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
args = bench.parse.__wrapped__(wl) if hasattr(bench.parse, "__wrapped__") else None
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
for name, b in (("closest", 8), ("shadow", 16)):
    rays, waves = max(c[b + 4], 1), max(c[b + 5], 1)
    print(f"{name:8s} rays {c[b+4]:>11d}  per ray: nodes {c[b]/rays:6.2f} tris {c[b+1]/rays:6.2f}  "
          f"per wave (max lane): nodes {c[b+2]/waves:6.2f} tris {c[b+3]/waves:6.2f}  lanes/wave {rays/waves:5.1f}")
