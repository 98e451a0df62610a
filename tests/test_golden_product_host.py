"""Host-side product components (scene loader tables the kernels consume) against the
reference's own outputs in tests/golden/reference_components.json.  No GPU needed."""
import ctypes

import numpy as np
import pytest

from conftest import SCENES, fl


def f32(v):
    return np.asarray(fl(v), dtype=np.float32)


@pytest.mark.parametrize("cfg_index", [0, 1, 2])
def test_halton_tables_bit_exact(pa, golden, cfg_index):
    cfg = golden["halton"][cfg_index]
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=cfg["xres"], yresolution=cfg["yres"], seed=cfg["seed"])
    f = sc.flat()
    assert list(f.halton_base_scales) == cfg["baseScales"]
    assert list(f.halton_mult_inverse) == cfg["multInverse"]
    for px, py, si, dim, p0, p1, vals in cfg["samples"]:
        got = [sc.halton(px, py, si, dim + j) for j in range(7)]
        np.testing.assert_array_equal(np.float32(got), f32(vals))
        assert sc.halton(px, py, si, -1) == np.float32(p0)
        assert sc.halton(px, py, si, -2) == np.float32(p1)


def test_rgb2spec_columns_bit_exact(pa, golden):
    lib = pa._lib()
    for col in golden["rgb2spec_columns"]:
        out = (ctypes.c_float * 192)()
        assert lib.pbrt_debug_rgb2spec_column(col["maxc"], col["j"], col["i"], out) == 0
        np.testing.assert_array_equal(np.array(out, np.float32), f32(col["values"]))


def test_rgb_to_sigmoid_coeffs_bit_exact(pa, golden):
    lib = pa._lib()
    for e in golden["rgb_to_spectrum"]:
        c = (ctypes.c_float * 3)()
        assert lib.pbrt_debug_rgb_coeffs(*[ctypes.c_float(v) for v in e["rgb"]], c) == 0
        np.testing.assert_array_equal(np.array(c, np.float32), f32(e["coeffs"]))


def test_sensor_cie_tables_bit_exact(pa, golden):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    f = sc.flat()
    xyz = np.ctypeslib.as_array(f.sensor_xyz, shape=(3 * 311,)).reshape(3, 311)
    np.testing.assert_array_equal(xyz[0], f32(golden["cie_x_dense"]))
    np.testing.assert_array_equal(xyz[1], f32(golden["cie_y_dense"]))
    np.testing.assert_array_equal(xyz[2], f32(golden["cie_z_dense"]))


def test_area_light_emission_matches_reference(pa, golden):
    """DiffuseAreaLight: Lemit = DenselySampled(RGBIlluminantSpectrum(sRGB, L)) and
    scale = 1 / SpectrumToPhotometric(illuminant) (lights.cpp:941)."""
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    f = sc.flat()
    ref = next(e for e in golden["rgb_illuminant"] if e["L"] == [17, 12, 4])
    dense = np.ctypeslib.as_array(f.dense_spectra, shape=(f.n_spectra * 311,)).reshape(f.n_spectra, 311)
    li = f.light_spectrum[0]
    np.testing.assert_array_equal(dense[li], f32(ref["dense"]))
    assert np.float32(f.light_scale[0]) == np.float32(1.0) / np.float32(fl(ref["photometric"]))
    assert np.float32(fl(ref["photometric"])) == np.float32(fl(golden["photometric_srgb_illuminant"]))


def test_output_colour_space_matrix(pa, golden):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    f = sc.flat()
    m = np.array(list(f.output_rgb_from_sensor_rgb), np.float64)
    np.testing.assert_allclose(m, np.float64(f32(golden["srgb_rgb_from_xyz"])), rtol=2e-6, atol=1e-7)


@pytest.mark.parametrize("i", [0, 1])
def test_camera_rays_match_reference(pa, golden, i):
    cam = golden["camera"][i]
    xres, yres = cam["res"]
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=xres, yresolution=yres)
    f = sc.flat()
    cfr = np.array(list(f.camera_from_raster), np.float32).reshape(4, 4)
    rfc = np.array(list(f.render_from_camera), np.float32).reshape(4, 4)
    np.testing.assert_allclose(cfr, f32(cam["camera_from_raster"]).reshape(4, 4), rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(rfc, f32(cam["render_from_camera"]).reshape(4, 4), rtol=1e-6, atol=1e-7)
    for px, py, dx, dy, dz in cam["dirs"]:
        p = cfr @ np.array([px, py, 0, 1], np.float32)
        d = p[:3] / p[3]
        d = d / np.linalg.norm(d)
        d = rfc[:3, :3] @ d
        np.testing.assert_allclose(d, [dx, dy, dz], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cfg_index", range(6))
def test_zsobol_bit_exact(pa, golden, cfg_index):
    """ZSobolSampler (samplers.h:225-370): the product's sampler evaluation against the
    reference's ZSobolSampler for the wavefront's call pattern (1D, 2D, 1D, 2D, 1D)."""
    from conftest import cornell_with_sampler
    cfg = golden["zsobol"][cfg_index]
    line = (f'Sampler "zsobol" "integer pixelsamples" [ {cfg["spp"]} ] "integer seed" [ {cfg["seed"]} ] '
            f'"string randomization" "{cfg["randomization"]}"')
    sc = cornell_with_sampler(pa, line, xresolution=cfg["xres"], yresolution=cfg["yres"])
    assert sc.flat().sampler_type == 1
    for px, py, si, dim, vals in cfg["samples"]:
        np.testing.assert_array_equal(sc.zsobol(px, py, si, dim), f32(vals), err_msg=f"{px} {py} {si} {dim}")


def test_halton_fastpath_matches_64bit_restatement(pa):
    """The kernels' Halton digits for indices < 2^24 (float-reciprocal quotient with one
    correction, reversedDigits accumulated exactly in double: core.h ScrambledRadicalInverse24)
    and its six-digit branch-free form for bases >= 17 (ScrambledRadicalInverse24x6)
    equal the 64-bit restatement of ScrambledRadicalInverse (util/lowdiscrepancy.h:115-134), bit
    for bit: every dimension the wavefront uses at maxdepth 5 (0..40), a strided sweep of the
    whole 2^24 range plus the top 2^16 indices and the first 2^16 exhaustively.  For dimensions
    >= 6 the same calls also check the Lean shade stage's digit-major form (HaltonDepthSamples)
    with the digit count of the sweep's bound, here also at the bounds spp * 128 * 243 of
    C2-like renders (fewer digits: 4 for 64 spp at depth 1)."""
    from conftest import SCENES
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64)
    top = 1 << 24
    # 0..40: maxdepth 5; beyond: bases whose digit count leaves a longer or no six-digit tail
    # (ScrambledRadicalInverse24x6)
    for dim in range(0, 41):
        assert sc.halton_fastpath_mismatches(dim, 0, top, 61) == 0, dim
        assert sc.halton_fastpath_mismatches(dim, top - (1 << 16), top) == 0, dim
        assert sc.halton_fastpath_mismatches(dim, 0, 1 << 16) == 0, dim
    for bound in (31104 * 64, 31104 * 16, 31104):
        for dim in range(6, 41):
            assert sc.halton_fastpath_mismatches(dim, 0, bound, 7) == 0, (dim, bound)
            assert sc.halton_fastpath_mismatches(dim, bound - min(bound, 1 << 14), bound) == 0, (dim, bound)
    deep = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64, maxdepth=60)
    for dim in (55, 97, 146, 300, 426):
        assert deep.halton_fastpath_mismatches(dim, 0, top, 61) == 0, dim
        assert deep.halton_fastpath_mismatches(dim, top - (1 << 16), top) == 0, dim
    assert sc.halton_fastpath_mismatches(0, 0, top + 1) == -1


def test_dense_offset_32bit_form_is_lround():
    """core.h DenseOffset: floor(lambda + 0.5f) - 395 on [394.5, 705.5), else -1, equals the
    reference's lround(lambda) - 395 with its range check (util/spectrum.h:420) for every float
    in [256, 1024) (float32 arithmetic, as on the host and the device)."""
    lam = np.arange(np.float32(256).view(np.uint32), np.float32(1024).view(np.uint32), dtype=np.uint32).view(np.float32)
    fast = np.where((lam >= np.float32(394.5)) & (lam < np.float32(705.5)),
                    np.floor(lam + np.float32(0.5)).astype(np.int64) - 395, -1)
    # lround: round half away from zero, in exact (float64) arithmetic
    o = np.floor(lam.astype(np.float64) + 0.5).astype(np.int64) - 395
    ref = np.where((o < 0) | (o > 310), -1, o)
    assert np.array_equal(fast, ref)
