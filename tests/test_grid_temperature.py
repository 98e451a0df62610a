"""GridMedium "temperature" (media.h:254-318, media.cpp:253-330): a temperature grid beside the
density grid makes the medium emissive with Le(p) = LeScale(p) * BlackbodySpectrum(T'(p)),
T' = (T(p) - temperatureoffset) * temperaturescale, and no emission where T' <= 100 K.

* the loader: the flat layout ({offset, scale, T[nz][ny][nx]} at medium_info[15]), the
  "temperaturecutoff" default of "temperatureoffset", pbrt's errors;
* the oracle: a constant-temperature absorbing grid against the same grid with "blackbody Le"
  of that temperature (DenselySampled at integer wavelengths, scaled by 1 / photometric), whose
  image is the same up to the dense table's rounding of lambda; a cold grid emits nothing;
* GPU parity: test_gpu_media.py::test_medium_box_matches_oracle[grid_temperature].

The blackbody itself (util/spectrum.h Blackbody / BlackbodySpectrum) is pinned by the
reference goldens of tests/golden "blackbody" (test_area_light_power.py)."""
import numpy as np
import pytest

from conftest import SCENES
from test_media import medium_scene, render

N = 4


def grid(extra, density=None, p0="-1 -1 0", p1="1 1 1"):
    d = density if density is not None else np.full(N ** 3, 1.0)
    return ('MakeNamedMedium "m" "string type" "uniformgrid" "rgb sigma_a" [0.8 0.8 0.8] "rgb sigma_s" [0 0 0] '
            f'"integer nx" {N} "integer ny" {N} "integer nz" {N} "point3 p0" [{p0}] "point3 p1" [{p1}] '
            f'"float density" [ {" ".join(f"{v:.4f}" for v in d)} ] {extra}')


def temps(t):
    return f'"float temperature" [ {" ".join(f"{v:.2f}" for v in t)} ]'


def flat_medium(pa, line):
    sc = pa.Scene.from_string(medium_scene(line, res=8, spp=1), SCENES)
    f = sc.flat()
    info = np.ctypeslib.as_array(f.medium_info, shape=(f.n_media * 16,)).reshape(-1, 16)
    return sc, f, info[0]


def test_temperature_layout(pa):
    t = np.round(np.linspace(50, 3000, N ** 3), 2)
    _, f, info = flat_medium(pa, grid(temps(t) + ' "float temperaturecutoff" 150 "float temperaturescale" 2'))
    assert info[0] == 1 and info[4] == 1 and info[14] == 0  # grid, emissive, not grey
    off = info[15]
    vals = np.ctypeslib.as_array(f.medium_values, shape=(off + 2 + N ** 3,))
    assert (vals[off], vals[off + 1]) == (150, 2)  # temperatureoffset defaults to the cutoff
    np.testing.assert_array_equal(vals[off + 2:], t.astype(np.float32))
    _, f2, info2 = flat_medium(pa, grid(temps(t) + ' "float temperatureoffset" 10 "float temperaturecutoff" 150'))
    vals2 = np.ctypeslib.as_array(f2.medium_values, shape=(info2[15] + 2,))
    assert vals2[info2[15]] == 10
    _, _, plain = flat_medium(pa, grid(""))
    assert plain[15] == -1 and plain[4] == 0


@pytest.mark.parametrize("extra, msg", [
    ('"float temperature" [1 2 3]', "Different number of samples"),
    (temps(np.full(N ** 3, 1000.0)) + ' "rgb Le" [1 1 1]', "Both \"Le\" and \"temperature\""),
])
def test_temperature_errors(pa, extra, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(medium_scene(grid(extra), res=8, spp=1), SCENES)


def test_constant_temperature_equals_blackbody_le(pa, oracle):
    """The grids extend past the interface box by a voxel, so the trilinear temperature lookup
    is constant inside it (a lookup lerps to 0 outside the grid, and the blackbody is not linear
    in T)."""
    T = 2500.0
    big = dict(p0="-2 -2 -1", p1="2 2 2")
    hot = grid(temps(np.full(N ** 3, T + 300)) + ' "float temperatureoffset" 300', **big)
    a, _ = render(pa, oracle, medium_scene(hot, res=16, spp=16, sky="0 0 0"))
    bb = grid(f'"blackbody Le" [ {T} ]', **big)
    b, sc = render(pa, oracle, medium_scene(bb, res=16, spp=16, sky="0 0 0"))
    # LeScale of the "Le" grid is 1 / SpectrumToPhotometric(BlackbodySpectrum(T)); the
    # temperature grid's is 1
    f = sc.flat()
    info = np.ctypeslib.as_array(f.medium_info, shape=(16,))
    inv_photometric = np.ctypeslib.as_array(f.medium_values, shape=(info[12] + 1,))[info[12]]
    assert a.mean() > 1e-3
    np.testing.assert_allclose(a.mean(axis=(0, 1)) * inv_photometric, b.mean(axis=(0, 1)), rtol=1e-2)
    lit = a.max(axis=-1) > 0
    np.testing.assert_allclose(a[lit] * inv_photometric, b[lit], rtol=2e-2, atol=1e-6)


def test_cold_grid_emits_nothing(pa, oracle):
    cold = grid(temps(np.full(N ** 3, 350.0)) + ' "float temperatureoffset" 300')  # T' = 50 K
    a, _ = render(pa, oracle, medium_scene(cold, res=8, spp=4, sky="0 0 0"))
    assert a.max() == 0
