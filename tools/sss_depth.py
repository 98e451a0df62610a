#!/usr/bin/env python3
"""At which path depth does one subsurface sample diverge between GPU and oracle (tools only):
python tools/sss_depth.py FORM ROW COL SAMPLE"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "pbrt-v4_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
import numpy as np
import torch  # noqa: F401
import pbrt_amd as pa
import pyoracle as oracle
from conftest import SCENES
import test_subsurface as T

oracle.set_math_mode(oracle.MATH_DEVICE)
form, row, col, s = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
for md in range(1, 7):
    src = T.scene(T.FORMS[form], T.BLOB + T.BOX).replace('"integer maxdepth" 6', f'"integer maxdepth" {md}')
    sc = pa.Scene.from_string(src, SCENES)
    i2 = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
    i2.render(rows=[row], first_sample=s, n_samples=1)
    i2.synchronize()
    g = np.asarray(i2.film_raw())[:3, row, col]
    o = np.asarray(oracle.render(sc, rows=np.array([row], np.int32), first_sample=s, n_samples=1, threads=1))[:3, row, col]
    print(f"maxdepth {md}: gpu {g} oracle {o} {'OK' if np.allclose(g, o, rtol=1e-4, atol=1e-7) else 'DIFF'}", flush=True)
print("done")
