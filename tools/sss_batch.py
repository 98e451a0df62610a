#!/usr/bin/env python3
"""Does the subsurface GPU/oracle film difference depend on the batch (paths in flight)?  Full
frame at several max_paths, and the worst rows rendered on their own (tools only):
python tools/sss_batch.py FORM"""
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


def gpu(max_paths, **kw):
    integ = pa.WavefrontPathIntegrator(sc, max_paths=max_paths)
    integ.render(**kw)
    integ.synchronize()
    return np.asarray(integ.film_raw())


def bad(a, b):
    return ~np.isclose(a[:3], b[:3], rtol=1e-3, atol=1e-5).all(axis=0)


for mp in (1 << 20, 1 << 16, 1 << 12):
    g = gpu(mp)
    m = bad(g, ref)
    rows = np.nonzero(m.any(axis=1))[0]
    print(f"max_paths {mp}: {m.sum()} bad pixels, rows {rows[:12].tolist()} sum gpu {g[:3].sum():.4f} oracle {ref[:3].sum():.4f}",
          flush=True)
g = gpu(1 << 20)
m = bad(g, ref)
worst = np.argsort(-m.sum(axis=1))[:4]
for r in worst:
    gr = gpu(1 << 20, rows=[int(r)])
    print(f"row {r}: full-frame bad {m[r].sum()}, row-only bad {bad(gr, ref)[r].sum()}", flush=True)
    for s in range(sc.info.spp):
        gs = gpu(1 << 16, rows=[int(r)], first_sample=s, n_samples=1)
        os_ = np.asarray(oracle.render(sc, rows=np.array([r], np.int32), first_sample=s, n_samples=1, threads=4))
        nb = bad(gs, os_)[r]
        if nb.any():
            x = int(np.nonzero(nb)[0][0])
            print(f"  sample {s}: {nb.sum()} bad, x={x} gpu={gs[:3, r, x]} oracle={os_[:3, r, x]}", flush=True)
print("done")
