"""RGB colour spaces: sRGB, DCI-P3, Rec2020 and ACES2065-1 (util/colorspace.cpp:23-112), the
ColorSpace directive (scene.cpp:108-115) and where the graphics state's colour space reaches the
scene (ParameterDictionary / ParsedParameter::colorSpace, paramdict.cpp:380-400; lights.cpp,
film.cpp:493-505, media.cpp:382-452), and the film's output (util/image.cpp:989-1005, 1231-1242).

Pinned against tests/golden "color_spaces" and "named_illuminants", written by
oracle/ref/refgold.cpp from the reference's own RGBColorSpace objects and the four
RGBToSpectrumTables that cmd/rgb2spec_opt.cpp generates (oracle/ref/Makefile TABLES):
* the illuminant (stdillum-D65, illum-acesD60) densely sampled, its photometric integral, the
  white point, the table columns, the coefficients of 48 RGB values and the albedo / unbounded /
  illuminant spectra they make: bit for bit;
* XYZFromRGB / RGBFromXYZ and the luminance vector: restated in pbrt's float arithmetic
  (compensated products, DifferenceOfProducts cofactors), bit for bit;
* the film sensor with each space as its output space (cie1931 plain and white-balanced, a
  fitted camera) as tests/test_sensors.py holds sRGB's (the plain cie1931 output matrix is
  RGBFromXYZ itself, bit for bit; white-balanced and fitted matrices within 2e-5).
The device kernels see only the converted spectra and the film matrix, so the GPU test is film
parity of a scene authored in ACES2065-1 against the oracle on the same flat scene."""
import struct

import numpy as np
import pytest

from conftest import SCENES, fl

CORNELL = (SCENES / "cornell-box.pbrt").read_text()
NAMES = ("srgb", "dci-p3", "rec2020", "aces2065-1")
LAMS = [395.0, 400.5, 455.25, 550.0, 600.125, 704.9]


def f32(v):
    return np.array(fl(v), np.float32)


def cs_golden(golden, k):
    g = golden["color_spaces"][k]
    assert g["name"] == NAMES[k]
    return g


@pytest.mark.parametrize("k", range(4))
def test_color_space_constants(pa, golden, k):
    g = cs_golden(golden, k)
    c = pa.debug_color_space(k)
    np.testing.assert_array_equal(c["prim"], f32(g["rgbw"])[:6])
    np.testing.assert_array_equal(c["w"], f32(g["rgbw"])[6:])
    np.testing.assert_array_equal(c["illuminant"], f32(g["illuminant"]))
    assert c["photometric"] == np.float32(fl(g["photometric"]))
    np.testing.assert_array_equal(c["xyz_from_rgb"].ravel(), f32(g["xyz_from_rgb"]))
    np.testing.assert_array_equal(c["rgb_from_xyz"].ravel(), f32(g["rgb_from_xyz"]))
    # the luminance vector is XYZFromRGB's middle row (colorspace.h:51-53)
    np.testing.assert_array_equal(c["xyz_from_rgb"][1], f32(g["luminance"]))


@pytest.mark.parametrize("k", range(4))
def test_table_columns_match_rgb2spec_opt(pa, golden, k):
    for col in cs_golden(golden, k)["columns"]:
        v = f32(col)
        maxc, j, i = (int(x) for x in v[:3])
        np.testing.assert_array_equal(pa.debug_rgb2spec_column(k, maxc, j, i).ravel(), v[3:])


@pytest.mark.parametrize("k", range(4))
def test_rgb_to_spectrum_matches_reference(pa, golden, k):
    rows = np.array([fl(r) for r in cs_golden(golden, k)["rgb_rows"]], np.float32)
    out = pa.debug_rgb_spectrum(k, rows[:, :3], LAMS, unbounded_scale=3.0)
    np.testing.assert_array_equal(out, rows[:, 3:])


@pytest.mark.parametrize("k", range(4))
def test_rgb_illuminant_dense_and_photometric(pa, golden, k):
    """DiffuseAreaLight's Lemit = DenselySampled(RGBIlluminantSpectrum(cs, L)) and its scale
    1 / SpectrumToPhotometric (the colour space illuminant's integral), through the loader."""
    name = NAMES[k]
    for row in cs_golden(golden, k)["rgb_illuminant"]:
        v = f32(row)
        L = [float(x) for x in v[:3]]
        text = CORNELL.replace("WorldBegin", f'WorldBegin\nColorSpace "{name}"').replace(
            'AreaLightSource "diffuse" "rgb L" [ 17 12 4 ]', f'AreaLightSource "diffuse" "rgb L" [ {L[0]!r} {L[1]!r} {L[2]!r} ]')
        assert f'"rgb L" [ {L[0]!r}' in text
        sc = pa.Scene.from_string(text, SCENES)
        f = sc.flat()
        dense = np.ctypeslib.as_array(f.dense_spectra, shape=(f.n_spectra * 311,)).reshape(f.n_spectra, 311)
        np.testing.assert_array_equal(dense[f.light_spectrum[0]], v[4:])
        assert np.float32(f.light_scale[0]) == np.float32(1.0) / v[3]


@pytest.mark.parametrize("k", range(4))
@pytest.mark.parametrize("si", range(3))
def test_sensor_with_output_color_space(pa, golden, k, si):
    cfg = cs_golden(golden, k)["sensors"][si]
    p = f'"string sensor" "{cfg["sensor"]}"'
    if float(cfg["whitebalance"]) != 0:
        p += f' "float whitebalance" {float(cfg["whitebalance"])!r}'
    lines = [ln + " " + p if ln.startswith("Film ") else ln for ln in CORNELL.splitlines()]
    text = f'ColorSpace "{NAMES[k]}"\n' + "\n".join(lines) + "\n"
    sc = pa.Scene.from_string(text, SCENES, xresolution=16, yresolution=16)
    f = sc.flat()
    m = np.array(list(f.xyz_from_sensor_rgb), np.float32).reshape(3, 3)
    np.testing.assert_allclose(m, np.array(fl(cfg["xyz_from_sensor_rgb"])).reshape(3, 3), rtol=2e-5, atol=2e-6)
    om = np.array([f.output_rgb_from_sensor_rgb[i] for i in range(9)]).reshape(3, 3)
    np.testing.assert_allclose(om, np.array(fl(cfg["output_rgb_from_sensor_rgb"])).reshape(3, 3), rtol=2e-5,
                               atol=2e-6)
    if cfg["sensor"] == "cie1931" and float(cfg["whitebalance"]) == 0:
        np.testing.assert_array_equal(om.astype(np.float32).ravel(), f32(cfg["output_rgb_from_sensor_rgb"]))


@pytest.mark.parametrize("name", ["stdillum-A", "stdillum-D50", "stdillum-D65", "stdillum-F1", "stdillum-F4",
                                  "stdillum-F9", "stdillum-F12", "illum-acesD60"])
def test_named_illuminants(pa, golden, name):
    """GetNamedSpectrum of the normalised standard illuminants (luminance-1 PiecewiseLinear)."""
    lam = np.arange(395, 706, dtype=np.float32)
    np.testing.assert_array_equal(pa.named_spectrum(name, lam), f32(golden["named_illuminants"][name]))


def test_color_space_names(pa):
    assert [pa.color_space_index(n) for n in NAMES] == [0, 1, 2, 3]
    assert pa.color_space_index("ACES2065-1") == 3 and pa.color_space_index("Rec2020") == 2
    with pytest.raises(pa.PbrtError, match="color space unknown"):
        pa.color_space_index("adobergb")


def test_unknown_color_space_directive_is_an_error(pa):
    with pytest.raises(pa.PbrtError, match="prophoto: color space unknown"):
        pa.Scene.from_string('ColorSpace "prophoto"\n' + CORNELL, SCENES)


def _material_coeffs(sc):
    f = sc.flat()
    return np.array([f.material_coeffs[i] for i in range(4 * f.n_materials)], np.float32).reshape(-1, 4)


def test_colour_space_reaches_material_rgb(pa):
    """RGB parameters convert through the colour space in force when their directive is parsed;
    AttributeEnd restores the previous one."""
    text = CORNELL.replace(
        'MakeNamedMaterial "red"', 'AttributeBegin\nColorSpace "rec2020"\nMakeNamedMaterial "red"').replace(
        'MakeNamedMaterial "green"', 'AttributeEnd\nMakeNamedMaterial "green"')
    sc = pa.Scene.from_string(text, SCENES)
    co = _material_coeffs(sc)
    red = pa.debug_rgb_spectrum(2, [0.65, 0.05, 0.05], LAMS)[0, :3]
    green = pa.debug_rgb_spectrum(0, [0.12, 0.45, 0.15], LAMS)[0, :3]
    rows = [tuple(r[:3]) for r in co]
    assert tuple(red) in rows and tuple(green) in rows
    assert tuple(pa.debug_rgb_spectrum(0, [0.65, 0.05, 0.05], LAMS)[0, :3]) not in rows


def test_default_light_is_the_colour_space_illuminant(pa):
    """With no "L", a DiffuseAreaLight emits the colour space's illuminant scaled by
    1 / SpectrumToPhotometric of it (lights.cpp:936-941): ACES2065-1's D60."""
    text = CORNELL.replace('AreaLightSource "diffuse" "rgb L" [ 17 12 4 ]',
                           'ColorSpace "aces2065-1"\nAreaLightSource "diffuse"')
    assert "ColorSpace" in text
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    c = pa.debug_color_space(3)
    dense = np.ctypeslib.as_array(f.dense_spectra, shape=(f.n_spectra * 311,)).reshape(f.n_spectra, 311)
    np.testing.assert_array_equal(dense[f.light_spectrum[0]], c["illuminant"])
    assert np.float32(f.light_scale[0]) == np.float32(1.0) / c["photometric"]


def _exr_chromaticities(path):
    b = path.read_bytes()
    key = b"chromaticities\x00chromaticities\x00"
    at = b.find(key)
    if at < 0:
        return None
    size = struct.unpack_from("<i", b, at + len(key))[0]
    assert size == 32
    return np.frombuffer(b, np.float32, 8, at + len(key) + 4)


def test_film_output_matrix(pa):
    """A Film authored in Rec2020 with the cie1931 sensor: outputRGBFromSensorRGB is Rec2020's
    RGBFromXYZ (film.cpp:505)."""
    sc = pa.Scene.from_string('ColorSpace "rec2020"\n' + CORNELL, SCENES, xresolution=8, yresolution=8)
    f = sc.flat()
    om = np.array([f.output_rgb_from_sensor_rgb[i] for i in range(9)]).reshape(3, 3)
    np.testing.assert_array_equal(om.astype(np.float32), pa.debug_color_space(2)["rgb_from_xyz"])


@pytest.mark.gpu
def test_film_write_color_space_gpu(pa, golden, tmp_path):
    """Writing a Rec2020 film: EXR keeps the film's values and records Rec2020's chromaticities
    (util/image.cpp:1231-1242); PFM is converted to sRGB by ConvertRGBColorSpace (:989-1005);
    an sRGB film's EXR has no chromaticities."""
    g = cs_golden(golden, 2)
    sc = pa.Scene.from_string('ColorSpace "rec2020"\n' + CORNELL, SCENES, xresolution=32, yresolution=32, spp=4)
    integ = pa.WavefrontPathIntegrator(sc)
    integ.render()
    integ.synchronize()
    rgb = integ.film_rgb()
    integ.write_image(tmp_path / "a.exr", write_fp16=False)
    integ.write_image(tmp_path / "a.pfm")
    np.testing.assert_array_equal(_exr_chromaticities(tmp_path / "a.exr"), f32(g["rgbw"]))
    m = f32(g["to_srgb"]).reshape(3, 3)
    want = np.einsum("ij,hwj->hwi", m.astype(np.float64), rgb.astype(np.float64))
    got = pa.read_image(tmp_path / "a.pfm")
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)
    base = pa.Scene.from_string(CORNELL, SCENES, xresolution=16, yresolution=16, spp=1)
    bi = pa.WavefrontPathIntegrator(base)
    bi.render()
    bi.synchronize()
    bi.write_image(tmp_path / "b.exr")
    assert _exr_chromaticities(tmp_path / "b.exr") is None


@pytest.mark.gpu
def test_aces_scene_matches_oracle_gpu(pa, oracle):
    """A Cornell box authored in ACES2065-1 (materials, emitter and film): GPU film parity with
    the oracle on the same flat scene."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb

    sc = pa.Scene.from_string('ColorSpace "aces2065-1"\n' + CORNELL, SCENES, xresolution=64, yresolution=64, spp=8)
    a, _ = gpu_rgb(pa, oracle, sc)
    check(a, oracle_rgb(oracle, sc))


@pytest.mark.parametrize("k", range(4))
def test_convert_to_srgb_matrix(pa, golden, k):
    g = cs_golden(golden, k)
    c, srgb = pa.debug_color_space(k), pa.debug_color_space(0)
    m = srgb["rgb_from_xyz"].astype(np.float64) @ c["xyz_from_rgb"].astype(np.float64)
    np.testing.assert_allclose(m.ravel(), f32(g["to_srgb"]), rtol=1e-6, atol=1e-7)
