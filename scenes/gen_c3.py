#!/usr/bin/env python3
"""C3 scene (killeroo stand-in): a seeded, displaced icosphere of 20,480
triangles with a dielectric (eta 1.5) shell, a rough conductor floor (constant eta, k;
roughness 0.1) of 9,800 triangles, a diffuse backdrop, a quad area light and a uniform
infinite light -- 30,284 triangles in all, every material type of the hot path.

The text is a pure function of its arguments (numpy seeded with `seed`), so tests and
bench.py generate it on the fly instead of committing half a megabyte of vertices.

    python scenes/gen_c3.py > c3.pbrt                  # 1920x1080, 256 spp (config C3)
    python scenes/gen_c3.py --xres 192 --yres 108 --spp 16
"""
import argparse

import numpy as np


def icosphere(level):
    t = (1 + 5 ** 0.5) / 2
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    verts = [np.array(p, float) / np.linalg.norm(p) for p in v]
    for _ in range(level):
        cache, nf = {}, []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                cache[key] = len(verts) - 1
            return cache[key]

        for a, b, c in f:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        f = nf
    return np.array(verts), np.array(f, dtype=np.int64)


def outward(P, F, center):
    """reorder faces so Cross(p0 - p2, p1 - p2) (pbrt's triangle normal) points away from center"""
    p0, p1, p2 = P[F[:, 0]], P[F[:, 1]], P[F[:, 2]]
    n = np.cross(p0 - p2, p1 - p2)
    flip = np.einsum("ij,ij->i", n, (p0 + p1 + p2) / 3 - center) < 0
    F = F.copy()
    F[flip, 1], F[flip, 2] = F[flip, 2], F[flip, 1].copy()
    return F


def fmt(a):
    return " ".join(f"{x:.6f}" for x in np.asarray(a, float).ravel())


def scene_text(xres=1920, yres=1080, spp=256, seed=0, maxdepth=5, sampler="zsobol"):
    rng = np.random.default_rng(seed)
    P, F = icosphere(5)
    # seeded displacement: a few random-direction sinusoids on the unit sphere
    r = np.ones(len(P))
    for amp, freq in ((0.09, 5.0), (0.05, 11.0), (0.025, 23.0)):
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        r += amp * np.sin(freq * P @ d + rng.uniform(0, 2 * np.pi))
    center = np.array([0.0, 1.15, 0.0])
    P = P * r[:, None] + center
    F = outward(P, F, center)

    n = 70  # floor grid: n x n quads, 2 triangles each
    g = np.linspace(-4.0, 4.0, n + 1)
    fx, fz = np.meshgrid(g, g, indexing="xy")
    FP = np.stack([fx.ravel(), np.zeros(fx.size), fz.ravel()], 1)
    idx = []
    for j in range(n):
        for i in range(n):
            a, b, c, d = j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i + 1, (j + 1) * (n + 1) + i
            idx += [a, c, b, a, d, c]  # normals +y
    FI = np.array(idx).reshape(-1, 3)
    FI = outward(FP, FI, np.array([0.0, -1.0, 0.0]))

    spl = {"zsobol": f'Sampler "zsobol" "integer pixelsamples" [ {spp} ]',
           "halton": f'Sampler "halton" "integer pixelsamples" [ {spp} ]'}[sampler]
    return f"""# C3: displaced dielectric icosphere + rough conductor floor (scenes/gen_c3.py, seed {seed})
LookAt 0 1.7 -5.2  0 1.0 0  0 1 0
Camera "perspective" "float fov" [ 38 ]
Film "rgb" "integer xresolution" [ {xres} ] "integer yresolution" [ {yres} ]
    "string filename" [ "c3.exr" ]
{spl}
Integrator "volpath" "integer maxdepth" [ {maxdepth} ]
PixelFilter "box"

WorldBegin

LightSource "infinite" "rgb L" [ 0.12 0.14 0.18 ]

MakeNamedMaterial "glass" "string type" [ "dielectric" ] "float eta" [ 1.5 ]
MakeNamedMaterial "metal" "string type" [ "conductor" ]
    "spectrum eta" [ 300 0.2 800 0.2 ] "spectrum k" [ 300 3.9 800 3.9 ] "float roughness" [ 0.1 ]
MakeNamedMaterial "backdrop" "string type" [ "diffuse" ] "rgb reflectance" [ 0.6 0.5 0.4 ]

NamedMaterial "glass"
Shape "trianglemesh" "integer indices" [ {" ".join(map(str, F.ravel()))} ]
    "point3 P" [ {fmt(P)} ]

NamedMaterial "metal"
Shape "trianglemesh" "integer indices" [ {" ".join(map(str, FI.ravel()))} ]
    "point3 P" [ {fmt(FP)} ]

NamedMaterial "backdrop"
Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
    "point3 P" [ -4 0 4  4 0 4  4 4 4  -4 4 4 ]

AttributeBegin
  NamedMaterial "backdrop"
  AreaLightSource "diffuse" "rgb L" [ 9 8.5 8 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
      "point3 P" [ -0.8 4.2 -0.8  0.8 4.2 -0.8  0.8 4.2 0.8  -0.8 4.2 0.8 ]
AttributeEnd
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--xres", type=int, default=1920)
    ap.add_argument("--yres", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--sampler", default="zsobol")
    a = ap.parse_args()
    print(scene_text(a.xres, a.yres, a.spp, a.seed, sampler=a.sampler), end="")


if __name__ == "__main__":
    main()
