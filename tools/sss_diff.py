#!/usr/bin/env python3
"""Renders the subsurface parity scenes (tests/test_subsurface.py FORMS) on the GPU and with the
oracle (device-math mode) and saves both images to gpurun_out/sss_<form>.npz (tools only)."""
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
from test_gpu_media import gpu_rgb, oracle_rgb

oracle.set_math_mode(oracle.MATH_DEVICE)
for form in sys.argv[1:] or list(T.FORMS):
    sc = pa.Scene.from_string(T.scene(T.FORMS[form], T.BLOB + T.BOX), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    b = oracle_rgb(oracle, sc)
    np.savez(ROOT / "gpurun_out" / f"sss_{form}.npz", gpu=a, oracle=b)
    ok = np.abs(a - b) <= np.maximum(1e-3 * np.abs(b), 1e-4)
    print(form, "frac", ok.all(axis=-1).mean(), "bad px", (~ok.all(axis=-1)).sum())
