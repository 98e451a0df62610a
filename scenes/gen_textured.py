#!/usr/bin/env python3
"""Writes the textured test scenes' image fixtures (deterministic, numpy + zlib only):

  scenes/textures/bricks_rgb8.png    48x40 8-bit sRGB RGB  (non power of two: pyramid resize)
  scenes/textures/marble_rgba8.png   32x32 8-bit RGBA, alpha 1 everywhere (drops to RGB)
  scenes/textures/bumps_grey16.png   20x12 16-bit grey     (Half pyramid)
  scenes/textures/tiles_pal.png      16x16 8-bit palette   (decoded to RGB)
  scenes/textures/gloss.pfm          24x24 float grey      (roughness texture)
  scenes/textures/sky.pfm            16x8  float RGB

scenes/textured.pbrt uses them with imagemap, checkerboard, mix, scale, bilerp, directionmix
textures on diffuse, conductor and dielectric materials."""
import struct
import zlib
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent / "textures"


def png(path, img, color_type, bit_depth=8, palette=None):
    h, w = img.shape[:2]
    raw = b""
    rows = img.reshape(h, -1)
    for y in range(h):
        row = rows[y]
        if bit_depth == 16:
            row = row.astype(">u2").tobytes()
        else:
            row = row.astype(np.uint8).tobytes()
        raw += bytes([y % 5]) + _filter(row, y % 5, raw, w, img, bit_depth, color_type)
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, bit_depth, color_type, 0, 0, 0))
    if palette is not None:
        data += chunk(b"PLTE", palette.astype(np.uint8).tobytes())
    data += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    path.write_bytes(data)


_prev = {}


def _filter(row, ft, raw, w, img, bit_depth, color_type):
    """PNG filter types 0-4 over bytes (the reader must undo every one of them)"""
    samples = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[color_type]
    bpp = max(1, samples * bit_depth // 8)
    cur = np.frombuffer(row, dtype=np.uint8).astype(np.int32)
    prev = _prev.get(id(img), np.zeros_like(cur))
    out = np.zeros_like(cur)
    for i in range(len(cur)):
        a = cur[i - bpp] if i >= bpp else 0
        b = prev[i]
        c = prev[i - bpp] if i >= bpp else 0
        if ft == 0: p = 0
        elif ft == 1: p = a
        elif ft == 2: p = b
        elif ft == 3: p = (a + b) >> 1
        else:
            pp = a + b - c
            pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
            p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (cur[i] - p) & 255
    _prev[id(img)] = cur
    return out.astype(np.uint8).tobytes()


def pfm(path, img):
    h, w = img.shape[:2]
    nc = 1 if img.ndim == 2 else img.shape[2]
    hdr = ("Pf" if nc == 1 else "PF") + f"\n{w} {h}\n-1.0\n"
    path.write_bytes(hdr.encode() + np.ascontiguousarray(img[::-1].astype("<f4")).tobytes())


def main():
    OUT.mkdir(exist_ok=True)
    rng = np.random.default_rng(7)
    y, x = np.mgrid[0:40, 0:48]
    bricks = np.stack([(150 + 80 * ((x // 8 + (y // 6) % 2) % 2)) * (y % 6 != 0),
                       60 + (x * 3) % 90, 40 + (y * 5) % 120], axis=-1)
    bricks = np.clip(bricks + rng.integers(0, 25, bricks.shape), 0, 255)
    png(OUT / "bricks_rgb8.png", bricks, 2)
    y, x = np.mgrid[0:32, 0:32]
    v = 128 + 100 * np.sin(x / 3.0 + 2 * np.sin(y / 5.0))
    marble = np.stack([v, v * 0.9, v * 0.7, np.full_like(v, 255)], axis=-1)
    png(OUT / "marble_rgba8.png", np.clip(marble, 0, 255), 6)
    y, x = np.mgrid[0:12, 0:20]
    bumps = 32768 + 30000 * np.sin(x * 0.9) * np.cos(y * 1.3)
    png(OUT / "bumps_grey16.png", bumps.astype(np.int64), 0, 16)
    pal = np.array([[230, 230, 220], [40, 60, 160], [200, 40, 40], [30, 140, 60]])
    y, x = np.mgrid[0:16, 0:16]
    png(OUT / "tiles_pal.png", ((x // 4 + y // 4) % 4), 3, 8, palette=pal)
    y, x = np.mgrid[0:24, 0:24]
    pfm(OUT / "gloss.pfm", (0.05 + 0.4 * ((x // 6 + y // 6) % 2) + 0.01 * x).astype(np.float32))
    y, x = np.mgrid[0:8, 0:16]
    pfm(OUT / "sky.pfm", np.stack([0.2 + 0.1 * x, 0.3 + 0.05 * y, 0.9 - 0.02 * x], axis=-1).astype(np.float32))


if __name__ == "__main__":
    main()
