"""Participating media: MakeNamedMedium "homogeneous" / "uniformgrid",
MediumInterface, Material "interface", the camera medium.  The oracle restates the wavefront's
medium stages (wavefront/media.cpp, intersect.h TraceTransmittance, media.h SampleT_maj); these
CPU tests pin it with known answers of the radiative transfer equation.  GPU parity against
the oracle lives in test_gpu_parity.py.

No reference fixture covers media (media.cpp / media.h need NanoVDB, absent here): the media
path's parity is pinned by these known answers plus the component goldens it shares with the
surface path -- "parity unpinned" at the component level for SampleT_maj itself."""
import numpy as np
import pytest

from conftest import SCENES

BOX = """Shape "trianglemesh" "integer indices" [ 0 2 1 0 3 2  4 5 6 4 6 7  0 1 5 0 5 4  3 7 6 3 6 2  0 4 7 0 7 3  1 2 6 1 6 5 ]
  "point3 P" [ {x0} {y0} {z0}  {x1} {y0} {z0}  {x1} {y1} {z0}  {x0} {y1} {z0}
               {x0} {y0} {z1}  {x1} {y0} {z1}  {x1} {y1} {z1}  {x0} {y1} {z1} ]"""


def box(x0, x1, y0, y1, z0, z1):
    return BOX.format(x0=x0, x1=x1, y0=y0, y1=y1, z0=z0, z1=z1)


def medium_scene(medium_line, res=32, spp=32, maxdepth=5, sky="1 1 1", extra="", fov=20, sampler="zsobol"):
    """Camera looking down +z at a 2x2x1 interface box (z in [0, 1]) filled with medium "m"."""
    return f"""LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" [ {fov} ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "{sampler}" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ {maxdepth} ]
WorldBegin
LightSource "infinite" "rgb L" [ {sky} ]
{medium_line}
{extra}
AttributeBegin
  MediumInterface "m" ""
  Material "interface"
  {box(-1, 1, -1, 1, 0, 1)}
AttributeEnd
"""


def render(pa, oracle, text, threads=8):
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    film = oracle.render(sc, threads=threads)
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)]), sc


def test_loader_media_tables(pa):
    text = medium_scene('MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.5 0.25 0.1] '
                        '"rgb sigma_s" [1 1 1] "float scale" 2 "float g" 0.3')
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    assert f.n_media == 1 and f.camera_medium == -1
    info = [f.medium_info[i] for i in range(16)]
    assert info[0] == 0 and info[4] == 0  # homogeneous, not emissive
    assert f.medium_params[0] == pytest.approx(0.3)
    tm = np.ctypeslib.as_array(f.tri_medium, shape=(sc.info.n_triangles * 2,)).reshape(-1, 2)
    assert (tm == [0, -1]).all()


@pytest.mark.parametrize("bad,msg", [
    ('MakeNamedMedium "m" "string type" "nanovdb"', "not supported"),
    ('MakeNamedMedium "m" "string type" "uniformgrid" "integer nx" 2', "density"),
    ('MakeNamedMedium "q" "string type" "homogeneous"', "undefined"),
])
def test_media_errors_are_loud(pa, bad, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(medium_scene(bad), SCENES)


def test_absorbing_slab_transmittance(pa, oracle):
    """Pure absorber, thickness 1: every pixel through the slab sees sky * exp(-sigma_a)."""
    sa = 0.7
    img, _ = render(pa, oracle, medium_scene(
        f'MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [{sa} {sa} {sa}] '
        '"rgb sigma_s" [0 0 0]', spp=64, fov=10))
    sky, _ = render(pa, oracle, medium_scene('MakeNamedMedium "m" "string type" "homogeneous" '
                                             '"rgb sigma_a" [0 0 0] "rgb sigma_s" [0 0 0]', spp=4, fov=10))
    ratio = img.mean() / sky.mean()
    # oblique rays travel slightly farther than 1 (fov 10 => < 0.4 %)
    assert ratio == pytest.approx(np.exp(-sa), rel=0.03), ratio


def test_emissive_absorbing_slab(pa, oracle):
    """Le (1 - exp(-sigma_a d)) from an emitting absorber under a black sky."""
    sa = 0.8
    text = medium_scene(f'MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [{sa} {sa} {sa}] '
                        '"rgb sigma_s" [0 0 0] "rgb Le" [1 1 1]', spp=64, fov=10, sky="0 0 0")
    img, _ = render(pa, oracle, text)
    ref, _ = render(pa, oracle, text.replace('"rgb sigma_a" [0.8 0.8 0.8]', '"rgb sigma_a" [1000 1000 1000]'))
    assert img.mean() / ref.mean() == pytest.approx(1 - np.exp(-sa), rel=0.03)


@pytest.mark.parametrize("kind", ["homogeneous", "grid"])
def test_scattering_furnace(pa, oracle, kind):
    """Albedo-1 medium under a uniform white sky: radiance stays 1 (energy conservation)."""
    if kind == "homogeneous":
        m = 'MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0 0 0] "rgb sigma_s" [1.5 1.5 1.5] "float g" 0.4'
    else:
        rng = np.random.default_rng(3)
        d = rng.uniform(0, 1, 8 * 8 * 8)
        m = ('MakeNamedMedium "m" "string type" "uniformgrid" "rgb sigma_a" [0 0 0] "rgb sigma_s" [3 3 3] '
             '"float g" -0.3 "integer nx" 8 "integer ny" 8 "integer nz" 8 "point3 p0" [-1 -1 0] "point3 p1" [1 1 1] '
             f'"float density" [ {" ".join(f"{v:.5f}" for v in d)} ]')
    img, _ = render(pa, oracle, medium_scene(m, spp=32, maxdepth=60, fov=30))
    assert img.mean() == pytest.approx(1.0, rel=0.02), img.mean()


def c5_small_text(res=48, spp=8, maxdepth=8, sampler="zsobol"):
    """A C5-like scene at test size: an fBm-density uniformgrid cloud inside an interface box,
    an area light and a sky, a diffuse floor, and the camera inside a thin homogeneous haze."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c5
    return gen_c5.scene_text(res, res, spp, grid=12, maxdepth=maxdepth, sampler=sampler, haze=True)


def test_oracle_c5_small_plausible(pa, oracle):
    img, sc = render(pa, oracle, c5_small_text())
    assert sc.flat().camera_medium >= 0
    assert np.isfinite(img).all() and img.min() >= 0 and img.mean() > 0.01


def test_medium_preset_equals_its_rgb(pa):
    """HomogeneousMedium "preset" (media.cpp:170-186): GetMediumScatteringProperties' measured
    sigma_a / sigma'_s (mm^-1, media.cpp:74-151) as RGBUnboundedSpectrum -- the same dense
    spectra as writing them as "rgb sigma_a" / "rgb sigma_s"; "scale" applies to both."""
    def dense(line):
        sc = pa.Scene.from_string(medium_scene(line, res=8, spp=1), SCENES)
        f = sc.flat()
        info = np.ctypeslib.as_array(f.medium_info, shape=(f.n_media * 16,)).reshape(-1, 16)
        d = np.ctypeslib.as_array(f.dense_spectra, shape=(f.n_spectra * 311,)).reshape(-1, 311)
        return d[info[0, 1]].copy(), d[info[0, 2]].copy()
    a = dense('MakeNamedMedium "m" "string type" "homogeneous" "string preset" "Skin1" "float scale" 2')
    b = dense('MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.032 0.17 0.48] '
              '"rgb sigma_s" [0.74 0.88 1.01] "float scale" 2')
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    c = dense('MakeNamedMedium "m" "string type" "homogeneous" "string preset" "Regular Milk"')
    assert c[1].mean() > 4 and c[0].max() < 0.05
    # an unknown preset warns and keeps the parameters (pbrt's Warning, not an error)
    u = dense('MakeNamedMedium "m" "string type" "homogeneous" "string preset" "Nope" "rgb sigma_a" [0.032 0.17 0.48] '
              '"rgb sigma_s" [0.74 0.88 1.01] "float scale" 2')
    np.testing.assert_array_equal(u[0], b[0])


def test_medium_preset_only_on_homogeneous(pa):
    with pytest.raises(pa.PbrtError, match="preset"):
        pa.Scene.from_string(medium_scene('MakeNamedMedium "m" "string type" "uniformgrid" "string preset" "Skin1" '
                                          '"float density" [1]', res=8, spp=1), SCENES)
