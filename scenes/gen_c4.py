#!/usr/bin/env python3
"""C4 scene (San-Miguel stand-in): a seeded field of copied (not instanced)
displaced icospheres packed for depth complexity, diffuse and conductor materials, on a
rough conductor ground, lit by a large quad light and a uniform sky.  The default is 122
copies of a 81,920-triangle sphere + a 2-triangle ground + the light = 9,994,244 triangles,
written as binary little-endian PLY files (one per copy) next to the .pbrt file.

Textured (the default, as BASELINE configs[3] "San-Miguel (~10M tris, textured)"): every mesh
carries per-vertex uv, the diffuse copies read their reflectance from one of eight 8-bit sRGB
PNG image textures (256^2 .. 1024^2, written next to the scene, bilinear or trilinear MIP
filtering, random uv scales), the metals and the ground their roughness from float image
textures.  --untextured writes round 2's constant-material scene.

    python scenes/gen_c4.py OUTDIR                       # full C4: 1920x1080, 128 spp
    python scenes/gen_c4.py OUTDIR --copies 6 --level 3  # small variant for tests
"""
import argparse
import struct
import zlib
from pathlib import Path

import numpy as np

from gen_c3 import icosphere, outward


def write_ply(path, P, F, UV=None):
    """binary_little_endian PLY: float x y z (u v), faces as uchar-count int indices"""
    V = P if UV is None else np.concatenate([P, UV], axis=1)
    V = np.ascontiguousarray(V, dtype="<f4")
    faces = np.zeros(len(F), dtype=[("n", "u1"), ("i", "<i4", (3,))])
    faces["n"] = 3
    faces["i"] = F
    head = (f"ply\nformat binary_little_endian 1.0\nelement vertex {len(P)}\n"
            "property float x\nproperty float y\nproperty float z\n"
            + ("" if UV is None else "property float u\nproperty float v\n") +
            f"element face {len(F)}\nproperty list uchar int vertex_indices\nend_header\n")
    with open(path, "wb") as f:
        f.write(head.encode())
        f.write(V.tobytes())
        f.write(faces.tobytes())


def write_png(path, img):
    """8-bit RGB (or grey) PNG, filter type 0 rows (numpy + zlib)"""
    img = np.ascontiguousarray(np.clip(img, 0, 255).astype(np.uint8))
    h, w = img.shape[:2]
    ct = 2 if img.ndim == 3 else 0
    raw = np.concatenate([np.zeros((h, 1), np.uint8), img.reshape(h, -1)], axis=1).tobytes()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    path.write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ct, 0, 0, 0)) +
                     chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def texture_images(out, rng):
    """eight albedo images (bricks, stripes, tiles, wood, noise, checks, rings, plaster) and two
    grey roughness maps; sizes 256^2 .. 1024^2"""
    names = []
    for t in range(8):
        n = [256, 512, 1024, 512, 256, 1024, 512, 256][t]
        y, x = np.mgrid[0:n, 0:n].astype(np.float32) / n
        base = rng.uniform(40, 200, 3)
        if t % 4 == 0:
            pat = ((np.floor(x * 8 + (np.floor(y * 16) % 2) * 0.5) + np.floor(y * 16)) % 2)[..., None]
        elif t % 4 == 1:
            pat = (0.5 + 0.5 * np.sin(2 * np.pi * (x * 6 + 2 * np.sin(2 * np.pi * y * 3))))[..., None]
        elif t % 4 == 2:
            pat = (((np.floor(x * 12) + np.floor(y * 12)) % 3) / 2.0)[..., None]
        else:
            r = np.sqrt((x - .5) ** 2 + (y - .5) ** 2)
            pat = (0.5 + 0.5 * np.sin(60 * r))[..., None]
        noise = rng.uniform(-25, 25, (n, n, 1))
        img = base[None, None, :] * (0.45 + 0.55 * pat) + noise
        name = f"c4_tex{t}.png"
        write_png(out / name, img)
        names.append(name)
    for t in range(2):
        n = 512
        y, x = np.mgrid[0:n, 0:n].astype(np.float32) / n
        g = 40 + 160 * (0.5 + 0.5 * np.sin(2 * np.pi * (x * (4 + 3 * t) + y * 2))) + rng.uniform(-20, 20, (n, n))
        name = f"c4_gloss{t}.png"
        write_png(out / name, g)
        names.append(name)
    return names


def leaf_mask(out, n=256):
    """grey 8-bit PNG of a leaf cut-out (1 inside an elliptic blade with a notched tip and a
    stem, 0 outside, a one-texel ramp at the edge): the alpha texture of the leaf canopy"""
    y, x = (np.mgrid[0:n, 0:n].astype(np.float32) + 0.5) / n
    u, v = x - 0.5, y - 0.5
    blade = (u / 0.32) ** 2 + (v / 0.46) ** 2 - 0.08 * np.cos(18 * np.arctan2(v, u))
    stem = (np.abs(u) < 0.02) & (v > 0.3)
    a = np.clip((1 - blade) * n / 8, 0, 1)
    a = np.maximum(a, stem.astype(np.float32))
    write_png(out / "c4_leaf.png", 255 * a)
    return "c4_leaf.png"


def leaf_canopy(rng, n_leaves, lo, hi):
    """n_leaves randomly oriented unit-ish quads (2 triangles each, uv over the leaf image) in the
    box [lo, hi]: one trianglemesh whose "texture alpha" cuts the leaf shape out of each quad"""
    c = rng.uniform(lo, hi, (n_leaves, 3))
    a = rng.normal(size=(n_leaves, 3))
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    b = np.cross(a, rng.normal(size=(n_leaves, 3)))
    b /= np.linalg.norm(b, axis=1, keepdims=True)
    s = rng.uniform(0.15, 0.35, (n_leaves, 1))
    P = np.stack([c - s * a - s * b, c + s * a - s * b, c + s * a + s * b, c - s * a + s * b], axis=1)
    F = (np.arange(n_leaves)[:, None, None] * 4 + np.array([[0, 1, 2], [0, 2, 3]])[None]).reshape(-1, 3)
    UV = np.tile(np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float32), (n_leaves, 1))
    return P.reshape(-1, 3), F, UV


def generate(outdir, copies=122, level=6, xres=1920, yres=1080, spp=128, seed=0, maxdepth=5, textured=True,
             leaves=0):
    """leaves > 0 adds an alpha-tested leaf canopy (that many cut-out quads, one PLY mesh with
    per-vertex uv and a "texture alpha" leaf image) above the field of copies, as San Miguel's
    foliage: every candidate hit on it runs the stochastic alpha test (gpu/optix.cu:197-243)"""
    out = Path(outdir)
    out.mkdir(parents=True, exist_ok=True)
    rng = np.random.default_rng(seed)
    P0, F0 = icosphere(level)
    F0 = outward(P0, F0, np.zeros(3))
    # spherical uv of the unit sphere (u around y, v from the pole)
    UV0 = np.stack([np.arctan2(P0[:, 2], P0[:, 0]) / (2 * np.pi) + 0.5,
                    np.arccos(np.clip(P0[:, 1] / np.linalg.norm(P0, axis=1), -1, 1)) / np.pi], axis=1)
    tex_lines = []
    if textured:
        names = texture_images(out, np.random.default_rng(seed + 1))
        for t in range(8):
            filt = "trilinear" if t % 2 else "bilinear"
            tex_lines.append(f'Texture "albedo{t}" "spectrum" "imagemap" "string filename" "{names[t]}" '
                             f'"string filter" "{filt}"')
        for t in range(2):
            tex_lines.append(f'Texture "gloss{t}" "float" "imagemap" "string filename" "{names[8 + t]}" '
                             f'"float scale" 0.35')
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
        write_ply(out / name, P, F0, UV0 if textured else None)
        n_tris += len(F0)
        if c % 3 == 2:
            metal = ["metal-Au", "metal-Cu", "metal-Al"][c % 9 // 3]
            rough = (f'"texture roughness" "gloss{c % 2}"' if textured
                     else f'"float roughness" [ {rng.uniform(0.01, 0.3):.4f} ]')
            mat = f'Material "conductor" "spectrum eta" "{metal}-eta" "spectrum k" "{metal}-k" {rough}'
        elif textured:
            # a per-copy scaled view of one of the eight images (the scale folds into the image)
            tex = f"albedo{c % 8}"
            mat = (f'Texture "a{c}" "spectrum" "scale" "texture tex" "{tex}" '
                   f'"float scale" {rng.uniform(0.6, 1.0):.4f}\n'
                   f'Material "diffuse" "texture reflectance" "a{c}"')
        else:
            rgb = rng.uniform(0.15, 0.85, 3)
            mat = f'Material "diffuse" "rgb reflectance" [ {rgb[0]:.4f} {rgb[1]:.4f} {rgb[2]:.4f} ]'
        lines.append(f'{mat}\nShape "plymesh" "string filename" "{name}"')
    n_tris += 2 + 2
    depth = max(cells, key=lambda c: c[1])[1] * 1.4 + 4
    if leaves:
        mask = leaf_mask(out)
        P, F, UV = leaf_canopy(np.random.default_rng(seed + 2), leaves, [-(nx / 2) * 1.3, 1.8, -0.5],
                               [(nx / 2) * 1.3, 3.4, depth - 2])
        write_ply(out / "c4_leaves.ply", P, F, UV)
        n_tris += len(F)
        lines.append(f'Texture "leafmask" "float" "imagemap" "string filename" "{mask}" "string encoding" "linear"\n'
                     'Material "diffuse" "rgb reflectance" [ 0.12 0.35 0.08 ]\n'
                     'Shape "plymesh" "string filename" "c4_leaves.ply" "texture alpha" "leafmask"')
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

""" + "\n".join(tex_lines) + ("\n" if tex_lines else "") + f"""
Material "conductor" "spectrum eta" [ 300 0.3 800 0.3 ] "spectrum k" [ 300 3.5 800 3.5 ] {'"texture roughness" "gloss0"' if textured else '"float roughness" [ 0.2 ]'}
Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
    "point3 P" [ -40 0 -10  -40 0 {depth + 40:.2f}  40 0 {depth + 40:.2f}  40 0 -10 ]
    "point2 uv" [ 0 0  0 20  20 20  20 0 ]

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
    ap.add_argument("--untextured", action="store_true")
    ap.add_argument("--leaves", type=int, default=0, help="alpha-tested leaf quads above the copies")
    a = ap.parse_args()
    path, n = generate(a.outdir, a.copies, a.level, a.xres, a.yres, a.spp, textured=not a.untextured,
                       leaves=a.leaves)
    print(path, n, "triangles")


if __name__ == "__main__":
    main()
