#!/usr/bin/env python3
"""Per-section wave cycles of k_shade_diffuse on the bench workload (profiling build).
Run on the GPU box: make -C pbrt-v4_amd prof && python tools/sections.py"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("PBRT_AMD_LIB", str(ROOT / "pbrt-v4_amd" / "lib" / "libpbrt_amd_prof.so"))
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
import torch  # noqa: F401  (same HIP runtime as bench.py)
import pbrt_amd as pa

NAMES = ["loads+surface", "halton", "R != 0 + frame", "light sample geometry", "BSDF sample geometry",
         "wavelength pass", "RR + decisions", "queue push + writes"]
if len(sys.argv) > 1 and sys.argv[1] == "c3":  # C3 at reduced size (ZSobol: the full kernel)
    sys.path.insert(0, str(ROOT / "scenes"))
    import gen_c3
    sc = pa.Scene.from_string(gen_c3.scene_text(960, 540, 16), ROOT / "scenes")
else:
    sc = pa.load_scene(ROOT / "scenes" / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64)
integ = pa.WavefrontPathIntegrator(sc, device=0)
integ.render(n_samples=4)
integ.synchronize()
integ.reset_stats()
integ.render()
integ.synchronize()
cyc = integ.kernel_sections(16)
tot = sum(cyc[:8]) or 1
for i, n in enumerate(NAMES):
    print(f"{i} {n:28s} {cyc[i] / 1e9:10.3f} Gcyc  {100 * cyc[i] / tot:5.1f}%")
print("queue counts of the last pass (rays, material, shadow, escaped, emissive):")
print(integ.queue_counts())
