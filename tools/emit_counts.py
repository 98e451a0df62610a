#!/usr/bin/env python3
"""Per-depth queue counts of one C2 pass (tools only): rays, diffuse, shadow, escaped, emissive
per depth, to size the emission stage (python tools/emit_counts.py)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
import torch  # noqa: F401
import pbrt_amd as pa

sc = pa.load_scene(ROOT / "scenes" / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64)
integ = pa.WavefrontPathIntegrator(sc, device=0)
integ.render(first_sample=0, n_samples=1)
integ.synchronize()
print("depth rays diffuse shadow escaped emissive dielectric conductor")
for d, row in enumerate(integ.queue_counts()):
    print(d, *[int(x) for x in row])
