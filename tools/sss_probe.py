#!/usr/bin/env python3
"""Per-sample GPU vs oracle film values of one row of a subsurface parity scene (tools only):
python tools/sss_probe.py FORM ROW X0 X1"""
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
form, row, x0, x1 = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
sc = pa.Scene.from_string(T.scene(T.FORMS[form], T.BLOB + T.BOX), SCENES)
for s in range(sc.info.spp):
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
    integ.render(rows=[row], first_sample=s, n_samples=1)
    integ.synchronize()
    g = integ.film_raw()
    o = oracle.render(sc, rows=np.array([row], np.int32), first_sample=s, n_samples=1, threads=4)
    g = np.asarray(g).reshape(4, sc.info.yres, sc.info.xres) if np.asarray(g).ndim != 3 else np.asarray(g)
    for x in range(x0, x1):
        a, b = g[:3, row, x], o[:3, row, x]
        if not np.allclose(a, b, rtol=1e-3, atol=1e-5):
            print(f"s={s} x={x} gpu={a} oracle={b}")
print("done")
