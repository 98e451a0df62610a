#!/usr/bin/env python3
"""Subsurface batch dependence, second cut (tools only): GPU run-to-run determinism, one row
with all samples at several max_paths, oracle thread-count independence.
python tools/sss_batch2.py FORM ROW"""
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
form, row = sys.argv[1], int(sys.argv[2])
sc = pa.Scene.from_string(T.scene(T.FORMS[form], T.BLOB + T.BOX), SCENES)
rows = np.array([row], np.int32)


def gpu(max_paths, **kw):
    integ = pa.WavefrontPathIntegrator(sc, max_paths=max_paths)
    integ.render(**kw)
    integ.synchronize()
    return np.asarray(integ.film_raw())


def nbad(a, b):
    return int((~np.isclose(a[:3, row], b[:3, row], rtol=1e-3, atol=1e-5).all(axis=0)).sum())


o16 = np.asarray(oracle.render(sc, rows=rows, threads=16))
o1 = np.asarray(oracle.render(sc, rows=rows, threads=1))
print("oracle threads 16 vs 1 identical:", np.array_equal(o16[:, row], o1[:, row]), flush=True)
osum = np.zeros_like(o1)
for s in range(sc.info.spp):
    osum += np.asarray(oracle.render(sc, rows=rows, first_sample=s, n_samples=1, threads=1))
print("oracle per-sample sum vs all-sample bad:", nbad(osum, o1), flush=True)
a = gpu(1 << 20, rows=[row])
b = gpu(1 << 20, rows=[row])
print("gpu run-to-run identical:", np.array_equal(a[:, row], b[:, row]), "bad vs oracle:", nbad(a, o1), flush=True)
for mp in (64, 128, 256, 512, 1024):
    print(f"gpu max_paths {mp}: bad vs oracle {nbad(gpu(mp, rows=[row]), o1)}", flush=True)
gsum = np.zeros_like(a)
for s in range(sc.info.spp):
    gsum += gpu(1 << 16, rows=[row], first_sample=s, n_samples=1)
print("gpu per-sample sum bad vs oracle:", nbad(gsum, o1), " vs gpu all-sample:", nbad(gsum, a), flush=True)
print("done")
