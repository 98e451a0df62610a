#!/usr/bin/env python3
"""C5 scene (cloud stand-in): a seeded fBm density grid as
MakeNamedMedium "uniformgrid" (pbrt's GridMedium, sigma_a 0.5, sigma_s 5, g 0.3) inside an
"interface" box, over a diffuse ground, lit by a quad area light and a uniform sky.  pbrt's
distant light is not in the hot path's light set, so the quad light stands in for it.
Optionally the camera sits in a thin homogeneous haze (camera medium + a second medium).

    python scenes/gen_c5.py > c5.pbrt                    # 1280x720, 1024 spp, 256^3 grid
    python scenes/gen_c5.py --grid 32 --spp 16 --xres 160 --yres 90
"""
import argparse

import numpy as np


def fbm(n, seed=0, octaves=5):
    """Value-noise fBm on an n^3 grid in [0, 1], shaped into a soft-edged cloud."""
    rng = np.random.default_rng(seed)
    x = (np.arange(n) + 0.5) / n
    total = np.zeros((n, n, n), np.float64)
    amp, freq = 1.0, 4
    for _ in range(octaves):
        lattice = rng.uniform(0, 1, (freq + 1,) * 3)
        f = x * freq
        i = np.minimum(f.astype(int), freq - 1)
        t = f - i
        t = t * t * (3 - 2 * t)
        # separable trilinear upsampling of the lattice
        a = lattice[i] * (1 - t)[:, None, None] + lattice[i + 1] * t[:, None, None]
        a = a[:, i] * (1 - t)[None, :, None] + a[:, i + 1] * t[None, :, None]
        a = a[:, :, i] * (1 - t)[None, None, :] + a[:, :, i + 1] * t[None, None, :]
        total += amp * a
        amp *= 0.5
        freq *= 2
    total /= total.max()
    zz, yy, xx = np.meshgrid(x, x, x, indexing="ij")
    r = np.sqrt((xx - 0.5) ** 2 + (yy - 0.45) ** 2 * 1.6 + (zz - 0.5) ** 2)
    shape = np.clip(1.0 - 2.2 * r, 0, 1)
    return np.clip(total * shape * 2.0 - 0.15, 0, None).astype(np.float32)  # [z][y][x]


def box(x0, x1, y0, y1, z0, z1):
    idx = "0 2 1 0 3 2  4 5 6 4 6 7  0 1 5 0 5 4  3 7 6 3 6 2  0 4 7 0 7 3  1 2 6 1 6 5"
    P = (f"{x0} {y0} {z0}  {x1} {y0} {z0}  {x1} {y1} {z0}  {x0} {y1} {z0}  "
         f"{x0} {y0} {z1}  {x1} {y0} {z1}  {x1} {y1} {z1}  {x0} {y1} {z1}")
    return f'Shape "trianglemesh" "integer indices" [ {idx} ] "point3 P" [ {P} ]'


def scene_text(xres=1280, yres=720, spp=1024, grid=256, seed=0, maxdepth=5, sampler="zsobol", haze=False):
    d = fbm(grid, seed)
    dens = " ".join(f"{v:.4g}" for v in d.ravel())
    haze_media = ('MakeNamedMedium "haze" "string type" "homogeneous" "rgb sigma_a" [0.01 0.01 0.01] '
                  '"rgb sigma_s" [0.04 0.04 0.04] "float g" 0.6\n') if haze else ""
    cam_medium = 'MediumInterface "" "haze"\n' if haze else ""
    outside = "haze" if haze else ""
    return f"""# C5: fBm uniformgrid cloud {grid}^3 (scenes/gen_c5.py, seed {seed})
{haze_media}{cam_medium}LookAt 0 1.2 -4.5  0 1.0 0  0 1 0
Camera "perspective" "float fov" [ 40 ]
Film "rgb" "integer xresolution" [ {xres} ] "integer yresolution" [ {yres} ]
    "string filename" [ "c5.exr" ]
Sampler "{sampler}" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ {maxdepth} ]
PixelFilter "box"

WorldBegin

LightSource "infinite" "rgb L" [ 0.25 0.3 0.4 ]
MakeNamedMedium "cloud" "string type" "uniformgrid"
    "rgb sigma_a" [ 0.5 0.5 0.5 ] "rgb sigma_s" [ 5 5 5 ] "float g" 0.3
    "integer nx" {grid} "integer ny" {grid} "integer nz" {grid}
    "point3 p0" [ -1.2 0.1 -1.2 ] "point3 p1" [ 1.2 2.5 1.2 ]
    "float density" [ {dens} ]

AttributeBegin
  MediumInterface "cloud" "{outside}"
  Material "interface"
  {box(-1.2, 1.2, 0.1, 2.5, -1.2, 1.2)}
AttributeEnd

AttributeBegin
  MediumInterface "" "{outside}"
  AreaLightSource "diffuse" "rgb L" [ 14 13 11 ]
  Material "diffuse" "rgb reflectance" [ 0.5 0.5 0.5 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
      "point3 P" [ 1.5 4.5 -1.5  3.5 4.5 -1.5  3.5 4.5 0.5  1.5 4.5 0.5 ]
AttributeEnd

AttributeBegin
  MediumInterface "" "{outside}"
  Material "diffuse" "rgb reflectance" [ 0.4 0.4 0.35 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
      "point3 P" [ -10 0 -10  -10 0 10  10 0 10  10 0 -10 ]
AttributeEnd
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--xres", type=int, default=1280)
    ap.add_argument("--yres", type=int, default=720)
    ap.add_argument("--spp", type=int, default=1024)
    ap.add_argument("--grid", type=int, default=256)
    ap.add_argument("--haze", action="store_true")
    a = ap.parse_args()
    print(scene_text(a.xres, a.yres, a.spp, a.grid, haze=a.haze), end="")


if __name__ == "__main__":
    main()
