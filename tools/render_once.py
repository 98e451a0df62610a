#!/usr/bin/env python3
"""One C2-scene render (default 1280x720, 8 spp) for profilers: python tools/render_once.py [spp] [scene]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
import torch  # noqa: F401  (same HIP runtime as bench.py)
import pbrt_amd as pa

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 8
scene = sys.argv[2] if len(sys.argv) > 2 else str(ROOT / "scenes" / "cornell-box.pbrt")
sc = pa.load_scene(scene, xresolution=1280, yresolution=720, spp=spp)
integ = pa.WavefrontPathIntegrator(sc, device=0)
integ.render()
integ.synchronize()
print("rendered", spp, "spp")
