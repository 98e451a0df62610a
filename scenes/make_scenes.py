#!/usr/bin/env python3
"""Generate the synthetic test/benchmark scenes that stand in for pbrt-v4-scenes
(not available offline).  Deterministic (fixed seeds)."""
import math
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent


def sphere_mesh(radius, n_theta, n_phi):
    verts, idx = [], []
    for i in range(n_theta + 1):
        th = math.pi * i / n_theta
        for j in range(n_phi):
            ph = 2 * math.pi * j / n_phi
            verts.append((radius * math.sin(th) * math.cos(ph), radius * math.sin(th) * math.sin(ph), radius * math.cos(th)))
    for i in range(n_theta):
        for j in range(n_phi):
            a = i * n_phi + j
            b = i * n_phi + (j + 1) % n_phi
            c = (i + 1) * n_phi + j
            d = (i + 1) * n_phi + (j + 1) % n_phi
            if i != 0:
                idx += [a, c, b]
            if i != n_theta - 1:
                idx += [b, c, d]
    return verts, idx


def fmt_mesh(verts, idx):
    p = " ".join(f"{x:.7g} {y:.7g} {z:.7g}" for x, y, z in verts)
    i = " ".join(str(k) for k in idx)
    return f'Shape "trianglemesh" "integer indices" [ {i} ]\n    "point3 P" [ {p} ]\n'


def furnace():
    """RenderTest.RadianceMatches scene 'Sphere, Kd = 0.5, Le = 0.5' (cpu/integrators_test.cpp:
    128-155): camera at the centre of a unit sphere (reverse orientation), diffuse 0.5,
    constant Le scaled to 0.5 nit -> image average 1.0 +- 0.025 (integrators_test.cpp:51-64)."""
    v, i = sphere_mesh(1.0, 48, 96)
    return ("# Furnace known-answer scene (see scenes/make_scenes.py)\n"
            'Camera "perspective" "float fov" [ 45 ]\n'
            'Film "rgb" "integer xresolution" [ 10 ] "integer yresolution" [ 10 ]\n'
            'Sampler "halton" "integer pixelsamples" [ 256 ]\n'
            'Integrator "volpath" "integer maxdepth" [ 8 ]\n'
            'PixelFilter "box"\n'
            "WorldBegin\n"
            'Material "diffuse" "float reflectance" [ 0.5 ]\n'
            "ReverseOrientation\n"
            'AreaLightSource "diffuse" "spectrum L" [ 300 1 800 1 ] "float scale" [ 0.5 ]\n'
            + fmt_mesh(v, i))


def main():
    (HERE / "furnace.pbrt").write_text(furnace())
    print("wrote furnace.pbrt")


if __name__ == "__main__":
    sys.exit(main())
