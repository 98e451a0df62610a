"""Image output and imgtool metrics (csrc/host/image.cpp): PFM / EXR
round trips, the EXR half encoding, PNG container validity, and Image::MAE / MSE / MRSE
(util/image.cpp:543-639) against their numpy statement.  Host only (no GPU)."""
import struct
import zlib

import numpy as np
import pytest


@pytest.fixture()
def img():
    rng = np.random.default_rng(7)
    a = rng.uniform(0, 4, (17, 23, 3)).astype(np.float32)
    a[0, 0] = [0, 1e-6, 65504]
    return a


def test_pfm_round_trip_exact(pa, img, tmp_path):
    p = tmp_path / "x.pfm"
    pa.write_image(p, img)
    raw = p.read_bytes()
    assert raw.startswith(b"PF\n23 17\n-1.000000\n")  # Image::WritePFM header, little endian
    np.testing.assert_array_equal(pa.read_image(p), img)
    # rows are stored bottom to top
    first_row = np.frombuffer(raw[len(b"PF\n23 17\n-1.000000\n"):][:23 * 12], np.float32).reshape(23, 3)
    np.testing.assert_array_equal(first_row, img[-1])


def test_exr_float_round_trip_exact(pa, img, tmp_path):
    p = tmp_path / "x.exr"
    pa.write_image(p, img, write_fp16=False)
    assert p.read_bytes()[:4] == struct.pack("<I", 20000630)
    np.testing.assert_array_equal(pa.read_image(p), img)


def test_exr_half_round_trip(pa, img, tmp_path):
    p = tmp_path / "h.exr"
    pa.write_image(p, img)
    back = pa.read_image(p)
    np.testing.assert_array_equal(back, img.astype(np.float16).astype(np.float32))  # IEEE half, RNE


def test_png_is_valid(pa, img, tmp_path):
    p = tmp_path / "x.png"
    pa.write_image(p, img)
    b = p.read_bytes()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    while pos < len(b):
        n, t = struct.unpack(">I4s", b[pos:pos + 8])
        data = b[pos + 8:pos + 8 + n]
        assert zlib.crc32(t + data) == struct.unpack(">I", b[pos + 8 + n:pos + 12 + n])[0]
        if t == b"IDAT":
            idat += data
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(17, 1 + 23 * 3)
    assert (raw[:, 0] == 0).all()
    px = raw[:, 1:].reshape(17, 23, 3).astype(np.float64) / 255
    lin = np.clip(img.astype(np.float64), 0, None)
    srgb = np.where(lin <= 0.0031308, 12.92 * lin, 1.055 * lin ** (1 / 2.4) - 0.055)
    assert np.abs(px - np.clip(srgb, 0, 1)).max() <= 0.5 / 255 + 1e-6


@pytest.mark.parametrize("metric", ["MAE", "MSE", "MRSE"])
def test_error_metrics_match_definition(pa, img, metric):
    ref = img * np.float32(0.9) + np.float32(0.05)
    got = pa.image_error(img, ref, metric)
    a, r = img.astype(np.float64), ref.astype(np.float64)
    if metric == "MAE":
        want = (a - r).mean(axis=(0, 1))  # pbrt's MAE is the signed mean difference
    elif metric == "MSE":
        want = ((a - r) ** 2).mean(axis=(0, 1))
    else:
        want = ((a - r) ** 2 / (r + 0.01) ** 2).mean(axis=(0, 1))
    np.testing.assert_allclose(got, want, rtol=1e-6)


def test_imgtool_diff_and_errors(pa, img, tmp_path):
    pa.write_image(tmp_path / "a.exr", img, write_fp16=False)
    pa.write_image(tmp_path / "b.pfm", img * np.float32(1.01))
    d = pa.imgtool_diff(tmp_path / "a.exr", tmp_path / "b.pfm", "MSE")
    assert d["delta_percent"] == pytest.approx(100 * (1 / 1.01 - 1), rel=1e-4)
    assert np.isclose(pa.image_error(img, img, "MSE"), 0).all()
    assert (pa.image_error(img, img, "FLIP") == 0).all()
    with pytest.raises(pa.PbrtError, match="FLIP"):
        pa.image_error(img, img, "PSNR")
    with pytest.raises(pa.PbrtError, match="unsupported"):
        pa.write_image(tmp_path / "x.tga", img)


@pytest.mark.gpu
def test_film_write_image_gpu(pa, tmp_path):
    """RGBFilm::WriteImage of a rendered film: the EXR / PFM contents are the film's RGB."""
    from conftest import SCENES
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=64, yresolution=48, spp=4)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
    integ.render()
    integ.synchronize()
    rgb = integ.film_rgb()
    integ.write_image(tmp_path / "c.exr", write_fp16=False)
    integ.write_image(tmp_path / "c.pfm")
    integ.write_image(tmp_path / "h.exr")
    np.testing.assert_array_equal(pa.read_image(tmp_path / "c.exr"), rgb)
    np.testing.assert_array_equal(pa.read_image(tmp_path / "c.pfm"), rgb)
    np.testing.assert_array_equal(pa.read_image(tmp_path / "h.exr"), rgb.astype(np.float16).astype(np.float32))


def _exr_attr(name, typ, payload):
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<I", len(payload)) + payload


def test_exr_header_bytes_match_openexr_layout(pa, tmp_path):
    """Byte-level check of a 2x2 float EXR against the OpenEXR file layout (single-part
    scanline, version 2): magic, version, attributes in the library's name order (Header keeps
    them in a std::map), chlist = per channel name\\0 + int32 pixel type + uint8 pLinear + 3
    reserved + int32 x/y sampling, closed by \\0; then the end-of-header \\0, one uint64 offset
    per scanline and scanlines of int32 y, int32 byte count and the channel planes in chlist
    order.  No OpenEXR library or reference EXR fixture exists here, so this pins the layout to
    the specification, not to bytes the reference wrote (parity of the byte stream unpinned)."""
    img = np.array([[[1, 2, 3], [4, 5, 6]], [[7, 8, 9], [10, 11, 12]]], np.float32)
    p = tmp_path / "t.exr"
    pa.write_image(p, img, write_fp16=False)
    b = p.read_bytes()
    chl = b"".join(c + b"\0" + struct.pack("<iB3xii", 2, 0, 1, 1) for c in (b"B", b"G", b"R")) + b"\0"
    box = struct.pack("<iiii", 0, 0, 1, 1)
    hdr = (struct.pack("<II", 20000630, 2) + _exr_attr("channels", "chlist", chl)
           + _exr_attr("compression", "compression", b"\0") + _exr_attr("dataWindow", "box2i", box)
           + _exr_attr("displayWindow", "box2i", box) + _exr_attr("lineOrder", "lineOrder", b"\0")
           + _exr_attr("pixelAspectRatio", "float", struct.pack("<f", 1))
           + _exr_attr("screenWindowCenter", "v2f", struct.pack("<ff", 0, 0))
           + _exr_attr("screenWindowWidth", "float", struct.pack("<f", 1)) + b"\0")
    line = 3 * 2 * 4
    table = struct.pack("<QQ", len(hdr) + 16, len(hdr) + 16 + 8 + line)
    lines = b"".join(struct.pack("<ii", y, line) + img[y][:, ::-1].T.astype("<f4").tobytes() for y in range(2))
    assert b == hdr + table + lines


@pytest.mark.gpu
def test_film_write_image_crop_window(pa, tmp_path):
    """--pixelbounds / cropwindow: RGBFilm::GetImage covers pixelBounds only and Image::WriteEXR
    records it as the dataWindow inside the full-resolution displayWindow (util/image.cpp:
    1179-1200); PFM holds the cropped pixels."""
    from conftest import SCENES
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=64, yresolution=48, spp=4,
                       pixelbounds="8,40,4,30")
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
    integ.render()
    integ.synchronize()
    rgb = integ.film_rgb()[4:30, 8:40]
    integ.write_image(tmp_path / "c.exr", write_fp16=False)
    integ.write_image(tmp_path / "c.pfm")
    np.testing.assert_array_equal(pa.read_image(tmp_path / "c.exr"), rgb)
    np.testing.assert_array_equal(pa.read_image(tmp_path / "c.pfm"), rgb)
    b = (tmp_path / "c.exr").read_bytes()
    i = b.index(b"dataWindow\0box2i\0")
    assert struct.unpack("<Iiiii", b[i + 17:i + 37]) == (16, 8, 4, 39, 29)
    i = b.index(b"displayWindow\0box2i\0")
    assert struct.unpack("<Iiiii", b[i + 20:i + 40]) == (16, 0, 0, 63, 47)


def test_flip_matches_reference_flip(pa, golden):
    """imgtool --metric FLIP: the product's FLIP (csrc/host/image.cpp FlipErrorMap) against
    ComputeFLIPError of the reference's vendored src/ext/flip/flip.cpp (oracle/ref/refgold.cpp)
    on three image pairs; the error maps agree to float rounding."""
    from conftest import fl
    for c in golden["flip"]:
        w, h = c["w"], c["h"]
        t = np.array(fl(c["test"]), np.float32).reshape(h, w, 3)
        r = np.array(fl(c["reference"]), np.float32).reshape(h, w, 3)
        e = np.array(fl(c["error"]), np.float32).reshape(h, w)
        m = pa.flip_error_map(t, r)
        np.testing.assert_allclose(m, e, rtol=1e-5, atol=1e-6)
        err = pa.image_error(t, r, "FLIP")
        assert err[0] == err[1] == err[2]
        np.testing.assert_allclose(err[0], e.mean(), rtol=1e-5)


def test_flip_identical_images_and_clamping(pa):
    rng = np.random.default_rng(1)
    a = rng.uniform(0, 1, (20, 24, 3)).astype(np.float32)
    assert pa.flip_error_map(a, a).max() == 0
    # values outside [0, 1] are clamped first (imgtool.cpp:1236-1243)
    np.testing.assert_array_equal(pa.flip_error_map(a * 3 - 1, a), pa.flip_error_map(np.clip(a * 3 - 1, 0, 1), a))
