#!/usr/bin/env python3
"""Which rows / samples of a subsurface parity scene differ between GPU and oracle (tools only):
python tools/sss_rows.py FORM"""
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
form = sys.argv[1]
sc = pa.Scene.from_string(T.scene(T.FORMS[form], T.BLOB + T.BOX), SCENES)
ref = np.asarray(oracle.render(sc, threads=16))
integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 20)
integ.render()
integ.synchronize()
g = np.asarray(integ.film_raw())
bad = ~np.isclose(g[:3], ref[:3], rtol=1e-3, atol=1e-5).all(axis=0)
rows = np.nonzero(bad.any(axis=1))[0]
print("bad pixels", int(bad.sum()), "rows", rows.tolist(), flush=True)
for r in rows[:3]:
    xs = np.nonzero(bad[r])[0]
    print(f"row {r}: cols {xs.tolist()}", flush=True)
    for s in range(sc.info.spp):
        i2 = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
        i2.render(rows=[int(r)], first_sample=s, n_samples=1)
        i2.synchronize()
        gs = np.asarray(i2.film_raw())
        os_ = np.asarray(oracle.render(sc, rows=np.array([r], np.int32), first_sample=s, n_samples=1, threads=4))
        for x in xs:
            a, b = gs[:3, r, x], os_[:3, r, x]
            if not np.allclose(a, b, rtol=1e-3, atol=1e-6):
                print(f"  s={s} x={x} gpu={a} oracle={b}", flush=True)
print("done")
