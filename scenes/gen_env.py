#!/usr/bin/env python3
"""Environment-map fixtures for ImageInfiniteLight (deterministic, numpy + zlib only).

  scenes/textures/env_sky.pfm        64x64 float RGB  sky gradient + a small bright sun
  scenes/textures/env_sky_zip.exr    same pixels, HALF channels, ZIP (16-line blocks)
  scenes/textures/env_sky_rle.exr    same pixels, HALF, RLE
  scenes/textures/env_sky_zips.exr   same pixels, FLOAT, ZIPS
  scenes/textures/env_sky_none.exr   same pixels, FLOAT, uncompressed
  scenes/textures/env_sky.png        32x32 8-bit sRGB of a dimmer sky (LDR)
  scenes/textures/env_const.pfm      8x8 constant 0.5 grey (furnace known answer)

The EXR writer here follows the published OpenEXR file layout (header attributes, scanline
offset table, the RLE / zlib codecs with their byte predictor and half-stream interleave);
it is independent of the C++ reader it checks."""
import struct
import zlib
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent / "textures"


def equal_area_dir(u, v):
    """EqualAreaSquareToSphere (util/math.cpp:292-314), numpy float64"""
    uu, vv = 2 * u - 1, 2 * v - 1
    up, vp = np.abs(uu), np.abs(vv)
    sd = 1 - (up + vp)
    r = 1 - np.abs(sd)
    phi = np.where(r == 0, 1, (vp - up) / np.where(r == 0, 1, r) + 1) * np.pi / 4
    z = np.copysign(1 - r * r, sd)
    s = r * np.sqrt(np.maximum(0, 2 - r * r))
    return np.stack([np.copysign(np.cos(phi), uu) * s, np.copysign(np.sin(phi), vv) * s, z], axis=-1)


def sky(n, sun=(0.3, 0.5, 0.81), sun_power=400.0):
    """a blue-to-white gradient over z with a small bright warm sun around direction `sun`"""
    c = (np.arange(n) + 0.5) / n
    u, v = np.meshgrid(c, c)  # row y = v
    d = equal_area_dir(u, v)
    z = d[..., 2]
    base = np.stack([0.25 + 0.35 * (1 - z), 0.35 + 0.3 * (1 - z), 0.9 - 0.2 * (1 - z)], axis=-1)
    base = np.where(z[..., None] < 0, np.array([0.08, 0.07, 0.05]), base)
    s = np.array(sun) / np.linalg.norm(sun)
    cosang = d @ s
    spot = (cosang > 0.995)[..., None] * np.array([1.0, 0.85, 0.6]) * sun_power
    return (base + spot).astype(np.float32)


def write_pfm(path, img):
    h, w = img.shape[:2]
    data = b"PF\n%d %d\n-1\n" % (w, h) + np.ascontiguousarray(img[::-1]).astype("<f4").tobytes()
    path.write_bytes(data)


def _attr(name, typ, payload):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(payload)) + payload


def _predict_interleave(raw):
    """inverse of the reader's un-predict: split even / odd bytes, then byte deltas + 128"""
    b = np.frombuffer(raw, dtype=np.uint8)
    t = np.concatenate([b[0::2], b[1::2]]).astype(np.int32)
    d = t.copy()
    d[1:] = (t[1:] - t[:-1] + 128) & 0xFF
    return d.astype(np.uint8).tobytes()


def _rle(data):
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        j = i + 1
        while j < n and data[j] == data[i] and j - i < 128:
            j += 1
        if j - i >= 3:
            out += bytes([j - i - 1, data[i]])
            i = j
            continue
        j = i
        while j < n and j - i < 127 and not (j + 2 < n and data[j] == data[j + 1] == data[j + 2]):
            j += 1
        out += bytes([(256 - (j - i)) & 0xFF]) + data[i:j]
        i = j
    return bytes(out)


def write_exr(path, img, half=True, compression=3):
    """scanline OpenEXR, channels B G R (sorted), compression 0 NONE 1 RLE 2 ZIPS 3 ZIP"""
    h, w = img.shape[:2]
    ptype, dt = (1, "<f2") if half else (2, "<f4")
    ch = b"".join(c.encode() + b"\0" + struct.pack("<iBBBBii", ptype, 0, 0, 0, 0, 1, 1) for c in "BGR") + b"\0"
    hdr = struct.pack("<ii", 20000630, 2)
    hdr += _attr("channels", "chlist", ch)
    hdr += _attr("compression", "compression", bytes([compression]))
    hdr += _attr("dataWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += _attr("displayWindow", "box2i", struct.pack("<iiii", 0, 0, w - 1, h - 1))
    hdr += _attr("lineOrder", "lineOrder", b"\0")
    hdr += _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    hdr += _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0))
    hdr += _attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    hdr += _attr("chromaticities", "chromaticities", struct.pack("<8f", .64, .33, .3, .6, .15, .06, .3127, .329))
    hdr += b"\0"
    lpb = 16 if compression == 3 else 1
    blocks = []
    for y0 in range(0, h, lpb):
        raw = b""
        for y in range(y0, min(h, y0 + lpb)):
            for c in (2, 1, 0):
                raw += img[y, :, c].astype(dt).tobytes()
        if compression == 1:
            data = _rle(_predict_interleave(raw))
        elif compression in (2, 3):
            data = zlib.compress(_predict_interleave(raw), 9)
        else:
            data = raw
        if len(data) >= len(raw):
            data = raw
        blocks.append(struct.pack("<ii", y0, len(data)) + data)
    off = len(hdr) + 8 * len(blocks)
    table = b""
    for b in blocks:
        table += struct.pack("<Q", off)
        off += len(b)
    path.write_bytes(hdr + table + b"".join(blocks))


def srgb8(lin):
    lin = np.clip(lin, 0, 1)
    s = np.where(lin <= 0.0031308, 12.92 * lin, 1.055 * lin ** (1 / 2.4) - 0.055)
    return np.round(s * 255).astype(np.uint8)


def write_png_rgb8(path, img8):
    h, w = img8.shape[:2]
    raw = b"".join(b"\0" + img8[y].tobytes() for y in range(h))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)

    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    data += chunk(b"IDAT", zlib.compress(raw, 9)) + chunk(b"IEND", b"")
    path.write_bytes(data)


def main():
    OUT.mkdir(exist_ok=True)
    img = sky(64)
    write_pfm(OUT / "env_sky.pfm", img)
    write_exr(OUT / "env_sky_zip.exr", img, half=True, compression=3)
    write_exr(OUT / "env_sky_rle.exr", img, half=True, compression=1)
    write_exr(OUT / "env_sky_zips.exr", img, half=False, compression=2)
    write_exr(OUT / "env_sky_none.exr", img, half=False, compression=0)
    write_png_rgb8(OUT / "env_sky.png", srgb8(sky(32, sun_power=0.0) * 0.9))
    write_pfm(OUT / "env_const.pfm", np.full((8, 8, 3), 0.5, np.float32))


if __name__ == "__main__":
    main()
