"""RGBGridMedium (MakeNamedMedium "rgbgrid": media.h:355-428, media.cpp:338-452): sigma_a,
sigma_s and Le as trilinear SampledGrid lookups of per-voxel RGBUnboundedSpectrum /
RGBIlluminantSpectrum values, scaled by "scale" / "Lescale"; a DDA majorant over the 16^3
grid of sigmaScale * (max sigma_a + max sigma_s).

* Pinned against the reference (oracle/ref/refgold.cpp "rgb_grid"): the oracle's
  Medium::SamplePoint at seeded points and wavelengths, bit for bit, and the loader's
  majorant grid, bit for bit, against SampledGrid::Lookup / MaxValue over the same voxels.
* Loader: RGBGridMedium::Create's errors.
* Known answer on the oracle: a grey RGB grid renders the same image as the uniform grid of
  density 1 with the same grey coefficients (equal in expectation, equal but for ulps here).
* GPU film parity on an emitting, coloured RGB grid (libm oracle, as the media kernels)."""
import numpy as np
import pytest

from conftest import SCENES
from test_media import medium_scene

GOLD_KEY = "rgb_grid"


def rgb_list(v):
    return " ".join(f"{float(x):.9g}" for x in v)


def gold_medium(g, extra=""):
    return ('MakeNamedMedium "m" "string type" "rgbgrid" "integer nx" 3 "integer ny" 2 "integer nz" 4 '
            f'"rgb sigma_a" [{rgb_list(g["sigma_a"])}] "rgb sigma_s" [{rgb_list(g["sigma_s"])}] '
            f'"rgb Le" [{rgb_list(g["Le"])}] {extra}')


def gold_scene(pa, g, extra=""):
    # camera at the origin: render space is world space, and the medium's space too
    text = ('LookAt 0 0 0  0 0 1  0 1 0\nCamera "perspective"\nFilm "rgb" "integer xresolution" 8 '
            '"integer yresolution" 8\nWorldBegin\nLightSource "infinite" "rgb L" [1 1 1]\n' + gold_medium(g, extra) +
            '\n')
    return pa.Scene.from_string(text, SCENES)


def test_sample_point_matches_reference(pa, oracle, golden):
    g = golden[GOLD_KEY]
    sc = gold_scene(pa, g)
    pts = np.array([e["p"] for e in g["points"]], np.float32)
    lam = np.array([e["lambda"] for e in g["points"]], np.float32)
    got = oracle.medium_point(sc, 0, pts, lam)
    for k, name in enumerate(("sigma_a", "sigma_s", "Le")):
        want = np.array([e[name] for e in g["points"]], np.float32)
        np.testing.assert_array_equal(got[:, k], want, err_msg=name)
    assert (got[:, 2] > 0).any() and np.ptp(got[:, 0]) > 0.5  # emitting points, varying sigma_a


def test_majorant_grid_matches_reference(pa, golden):
    g = golden[GOLD_KEY]
    sc = gold_scene(pa, g, '"float scale" 2.5')
    f = sc.flat()
    info = [f.medium_info[i] for i in range(16)]
    assert info[0] == 3 and info[15] == 7 and info[14] == 0  # all three grids, not grey
    vals = np.ctypeslib.as_array(f.medium_values, shape=(info[13] + 4096,))
    want = np.float32(2.5) * (np.array(g["max_a"], np.float32) + np.array(g["max_s"], np.float32))
    np.testing.assert_array_equal(vals[info[13]:], want)
    assert f.medium_params[7] == np.float32(2.5)


@pytest.mark.parametrize("params, msg", [
    ('"integer nx" 2 "rgb Le" [1 1 1 1 1 1]', 'requires "sigma_a" and/or "sigma_s"'),
    ('"integer nx" 2 "rgb sigma_s" [1 1 1 1 1 1] "rgb Le" [1 1 1 1 1 1]', 'requires "sigma_a" if "Le"'),
    ('"integer nx" 2 "rgb sigma_a" [1 1 1 1 1 1] "rgb sigma_s" [1 1 1]', "Different number of samples"),
    ('"integer nx" 2 "rgb sigma_a" [1 1 1 1 1 1] "rgb Le" [1 1 1]', 'values for "Le"'),
    ('"integer nx" 3 "rgb sigma_a" [1 1 1 1 1 1]', "expected nx\\*ny\\*nz = 3"),
    ('"integer nx" 1 "rgb sigma_a" [1 -1 1]', "negative"),
])
def test_loader_errors(pa, params, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(medium_scene('MakeNamedMedium "m" "string type" "rgbgrid" ' + params), SCENES)


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_grey_rgb_grid_equals_uniform_grid(pa, oracle):
    """Grey voxels (v, v, v): RGBUnboundedSpectrum samples v at every wavelength (sigmoid 1/2
    times scale 2v), so the RGB grid is the uniform grid of density 1 with sigma = v; both
    fade to zero over the outer half voxel alike.  The two renders agree to float rounding."""
    n = 4
    a, s = 0.7, 2.5
    bounds = '"point3 p0" [-1 -1 0] "point3 p1" [1 1 1] "float g" 0.3'
    rgbg = ('MakeNamedMedium "m" "string type" "rgbgrid" "integer nx" 4 "integer ny" 4 "integer nz" 4 '
            f'"rgb sigma_a" [{" ".join([f"{a} {a} {a}"] * n ** 3)}] "rgb sigma_s" [{" ".join([f"{s} {s} {s}"] * n ** 3)}] '
            + bounds)
    unif = ('MakeNamedMedium "m" "string type" "uniformgrid" "integer nx" 4 "integer ny" 4 "integer nz" 4 '
            f'"float density" [{" ".join(["1"] * n ** 3)}] "rgb sigma_a" [{a} {a} {a}] "rgb sigma_s" [{s} {s} {s}] '
            + bounds)
    imgs = []
    for med in (rgbg, unif):
        sc = pa.Scene.from_string(medium_scene(med, res=24, spp=16), SCENES)
        imgs.append(_rgb(oracle, sc, oracle.render(sc, threads=8)))
    assert imgs[1].mean() > 0
    close = np.isclose(imgs[0], imgs[1], rtol=1e-4, atol=1e-5).all(axis=-1).mean()
    assert close > 0.97, close
    assert abs(imgs[0].mean() / imgs[1].mean() - 1) < 2e-3


def colour_grid(seed=5, n=6, scale=1.5, le_scale=0.8):
    rng = np.random.default_rng(seed)
    sa = rng.uniform(0, 1.5, (n ** 3, 3))
    ss = rng.uniform(0, 4, (n ** 3, 3))
    le = rng.uniform(0, 1, (n ** 3, 3)) * (rng.uniform(0, 1, (n ** 3, 1)) > 0.7)
    return ('MakeNamedMedium "m" "string type" "rgbgrid" '
            f'"integer nx" {n} "integer ny" {n} "integer nz" {n} "rgb sigma_a" [{rgb_list(sa.ravel())}] '
            f'"rgb sigma_s" [{rgb_list(ss.ravel())}] "rgb Le" [{rgb_list(le.ravel())}] "float scale" {scale} '
            f'"float Lescale" {le_scale} "float g" -0.2 "point3 p0" [-1 -1 0] "point3 p1" [1 1 1]')


def test_colour_grid_renders(pa, oracle):
    sc = pa.Scene.from_string(medium_scene(colour_grid(), res=16, spp=4), SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    assert np.isfinite(img).all() and img.mean() > 0


@pytest.mark.gpu
def test_rgb_grid_gpu_matches_oracle(pa, oracle):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(medium_scene(colour_grid(), res=48, spp=16, sky="0.6 0.7 1"), SCENES)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mean_rel = check(gpu, oracle_rgb(oracle, sc))
    print(f"rgb grid medium parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
