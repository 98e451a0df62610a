#!/usr/bin/env python3
"""C4 scene (San-Miguel stand-in): a seeded field of copied (not instanced)
displaced icospheres packed for depth complexity, diffuse and conductor materials, on a
rough conductor ground, lit by a large quad light and a uniform sky.  The default is 122
copies of a 81,920-triangle sphere + a 2-triangle ground + the light = 9,994,244 triangles,
written as binary little-endian PLY files (one per copy) next to the .pbrt file.

    python scenes/gen_c4.py OUTDIR                       # full C4: 1920x1080, 128 spp
    python scenes/gen_c4.py OUTDIR --copies 6 --level 3  # small variant for tests
"""
import argparse
from pathlib import Path

import numpy as np

from gen_c3 import icosphere, outward


def write_ply(path, P, F):
    """binary_little_endian PLY: float x y z, faces as uchar-count int indices"""
    P = np.ascontiguousarray(P, dtype="<f4")
    faces = np.zeros(len(F), dtype=[("n", "u1"), ("i", "<i4", (3,))])
    faces["n"] = 3
    faces["i"] = F
    head = (f"ply\nformat binary_little_endian 1.0\nelement vertex {len(P)}\n"
            "property float x\nproperty float y\nproperty float z\n"
            f"element face {len(F)}\nproperty list uchar int vertex_indices\nend_header\n")
    with open(path, "wb") as f:
        f.write(head.encode())
        f.write(P.tobytes())
        f.write(faces.tobytes())


def generate(outdir, copies=122, level=6, xres=1920, yres=1080, spp=128, seed=0, maxdepth=5):
    out = Path(outdir)
    out.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(seed)
    P0, F0 = icosphere(level)
    F0 = outward(P0, F0, np.zeros(3))
    # a jittered 3D grid of copies in front of the camera (rows recede into the distance)
    nx = int(np.ceil(np.sqrt(copies / 2)))
    rows = int(np.ceil(copies / (2 * nx)))
    cells = [(i, j, k) for k in range(2) for j in range(rows) for i in range(nx)][:copies]
    lines = []
    n_tris = 0
    for c, (i, j, k) in enumerate(cells):
        r = np.ones(len(P0))
        for amp, freq in ((0.12, 4.0), (0.06, 9.0), (0.03, 19.0)):
            d = rng.normal(size=3)
            d /= np.linalg.norm(d)
            r += amp * np.sin(freq * P0 @ d + rng.uniform(0, 2 * np.pi))
        scale = rng.uniform(0.35, 0.7)
        center = np.array([(i - (nx - 1) / 2) * 1.3 + rng.uniform(-0.2, 0.2),
                           0.55 + k * 1.25 + rng.uniform(-0.1, 0.1),
                           j * 1.4 + rng.uniform(-0.2, 0.2)])
        P = P0 * (r * scale)[:, None] + center
        name = f"c4_{c:04d}.ply"
        write_ply(out / name, P, F0)
        n_tris += len(F0)
        if c % 3 == 2:
            metal = ["metal-Au", "metal-Cu", "metal-Al"][c % 9 // 3]
            mat = (f'Material "conductor" "spectrum eta" "{metal}-eta" "spectrum k" "{metal}-k" '
                   f'"float roughness" [ {rng.uniform(0.01, 0.3):.4f} ]')
        else:
            rgb = rng.uniform(0.15, 0.85, 3)
            mat = f'Material "diffuse" "rgb reflectance" [ {rgb[0]:.4f} {rgb[1]:.4f} {rgb[2]:.4f} ]'
        lines.append(f'{mat}\nShape "plymesh" "string filename" "{name}"')
    n_tris += 2 + 2
    depth = max(cells, key=lambda c: c[1])[1] * 1.4 + 4
    text = f"""# C4: {len(cells)} copied displaced icospheres, {n_tris} triangles (scenes/gen_c4.py, seed {seed})
LookAt 0 3.2 -6  0 1.0 {depth / 3:.3f}  0 1 0
Camera "perspective" "float fov" [ 50 ]
Film "rgb" "integer xresolution" [ {xres} ] "integer yresolution" [ {yres} ]
    "string filename" [ "c4.exr" ]
Sampler "zsobol" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ {maxdepth} ]
PixelFilter "box"

WorldBegin

LightSource "infinite" "rgb L" [ 0.15 0.17 0.2 ]

AttributeBegin
  AreaLightSource "diffuse" "rgb L" [ 4 3.8 3.5 ]
  Material "diffuse" "rgb reflectance" [ 0.5 0.5 0.5 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
      "point3 P" [ -6 9 -2  6 9 -2  6 9 {depth:.2f}  -6 9 {depth:.2f} ]
AttributeEnd

Material "conductor" "spectrum eta" [ 300 0.3 800 0.3 ] "spectrum k" [ 300 3.5 800 3.5 ] "float roughness" [ 0.2 ]
Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
    "point3 P" [ -40 0 -10  -40 0 {depth + 40:.2f}  40 0 {depth + 40:.2f}  40 0 -10 ]

""" + "\n".join(lines) + "\n"
    (out / "c4.pbrt").write_text(text)
    return out / "c4.pbrt", n_tris


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--copies", type=int, default=122)
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--xres", type=int, default=1920)
    ap.add_argument("--yres", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=128)
    a = ap.parse_args()
    path, n = generate(a.outdir, a.copies, a.level, a.xres, a.yres, a.spp)
    print(path, n, "triangles")


if __name__ == "__main__":
    main()
