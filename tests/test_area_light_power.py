"""AreaLightSource "diffuse" "float power" (DiffuseAreaLight::Create, lights.cpp:905-968): each
triangle of the shape is its own light, its scale multiplied by phi_v / k_e with
k_e = (twoSided ? 2 : 1) * Area * Pi, after the 1 / SpectrumToPhotometric(L) normalisation."""
import numpy as np
import pytest

from conftest import SCENES

SCENE = """LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" [ 30 ]
Film "rgb" "integer xresolution" [ 16 ] "integer yresolution" [ 16 ]
Sampler "zsobol" "integer pixelsamples" [ 4 ]
WorldBegin
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [ 2 3 4 ] {extra}
  Shape "trianglemesh" "integer indices" [ 0 1 2  0 2 3 ]
      "point3 P" [ -1 -1 0  1 -1 0  1 1 0  -3 1 0 ]
AttributeEnd
"""


def _lights(pa, extra):
    f = pa.Scene.from_string(SCENE.format(extra=extra), SCENES).flat()
    return np.array([f.light_scale[i] for i in range(2)], np.float64)


def test_power_scales_each_triangle(pa):
    base = _lights(pa, "")
    areas = np.array([2.0, 4.0])  # 0.5 |(p1-p0) x (p2-p0)| of the two triangles
    for extra, sides in (('"float power" 10', 1), ('"float power" 10 "bool twosided" true', 2)):
        got = _lights(pa, extra)
        want = base * 10 / (sides * areas * np.pi)
        np.testing.assert_allclose(got, want, rtol=1e-6)
    # no power (or a non-positive one): the scale is untouched
    np.testing.assert_array_equal(_lights(pa, '"float power" -1'), base)


def test_blackbody_emitter_matches_reference(pa, golden):
    """ "blackbody L" [T]: BlackbodySpectrum (util/spectrum.h) densely sampled, and the
    1 / SpectrumToPhotometric scale, against the reference's own outputs
    (tests/golden/reference_components.json "blackbody", oracle/ref/refgold.cpp)."""
    cases = golden["blackbody"]
    assert len(cases) == 7
    for e in cases:
        T = float(e["T"][0])
        f = pa.Scene.from_string(SCENE.replace('"rgb L" [ 2 3 4 ]', f'"blackbody L" [ {T} ]').format(extra=""),
                                 SCENES).flat()
        spec = f.light_spectrum[0]
        dense = np.array([f.dense_spectra[311 * spec + i] for i in range(311)], np.float32)
        want = np.asarray(e["values"], np.float32)
        np.testing.assert_allclose(dense, want, rtol=2e-6, atol=0)
        assert f.light_scale[0] == pytest.approx(1 / float(e["photometric"][0]), rel=1e-5)


def test_image_area_light_errors(pa):
    """An image emitter ("string filename", lights.cpp:909-939; tests/test_area_image_lights.py):
    "L" together with "filename" is the reference's own error, and a missing file is a located
    error rather than a silent default illuminant."""
    with pytest.raises(pa.PbrtError, match="Both \"L\" and \"filename\""):
        pa.Scene.from_string(SCENE.format(extra='"string filename" "emit.exr"'), SCENES)
    no_l = SCENE.replace('"rgb L" [ 2 3 4 ]', '"string filename" "emit.exr"')
    with pytest.raises(pa.PbrtError, match="emit.exr: unable to open"):
        pa.Scene.from_string(no_l.format(extra=""), SCENES)