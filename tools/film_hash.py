#!/usr/bin/env python3
"""Renders a scene with the library PBRT_AMD_LIB selects and prints a hash of the raw fp64 film,
so build variants can be compared bit for bit: python tools/film_hash.py [scene] [xres yres spp]"""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
sys.path.insert(0, str(ROOT / "scenes"))
import torch  # noqa: F401  (same HIP runtime as bench.py)
import pbrt_amd as pa

scene = sys.argv[1] if len(sys.argv) > 1 else "cornell"
x, y, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (320, 180, 16)
if scene in ("cornell", "c2"):
    sc = pa.load_scene(ROOT / "scenes" / "cornell-box.pbrt", xresolution=x, yresolution=y, spp=spp)
elif scene == "c3":
    import gen_c3
    sc = pa.Scene.from_string(gen_c3.scene_text(x, y, spp), ROOT / "scenes")
elif scene == "c5":
    import gen_c5
    sc = pa.Scene.from_string(gen_c5.scene_text(x, y, spp, grid=64), ROOT / "scenes")
elif scene == "c4":
    import tempfile
    import gen_c4
    path, _ = gen_c4.generate(Path(tempfile.mkdtemp(prefix="pbrt_c4_")), xres=x, yres=y, spp=spp, textured=True)
    sc = pa.load_scene(path)
else:
    sc = pa.load_scene(scene, xresolution=x, yresolution=y, spp=spp)
integ = pa.WavefrontPathIntegrator(sc, device=0)
integ.render()
integ.synchronize()
f = integ.film_raw()
print(scene, x, y, spp, hashlib.sha256(f.tobytes()).hexdigest()[:16], f"mean {f[..., 0].mean():.9g}")
