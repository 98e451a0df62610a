"""CloudMedium (MakeNamedMedium "cloud": media.h:430-525, media.cpp:462-484): a procedural
Perlin-noise density over [p0, p1] with a homogeneous majorant.

* Pinned against the reference: util/noise.cpp's Noise / DNoise on seeded points (small, large
  and negative coordinates) and CloudMedium::Density over the reference's own Noise / DNoise
  (oracle/ref/refgold.cpp "noise", "cloud_density") -- the product's host evaluation
  (pbrt_debug_cloud_density, the same core.h code the media kernels run) and the oracle's
  restatement, bit for bit.
* Loader: parameters, defaults, the permutation table travelling with the medium.
* Known answers on the oracle: with density 0 the cloud is empty above p.y = 0.5 (Density's
  altitude term is zero there), so a cloud box spanning y in [0.5, 1] is transparent in
  expectation; a cloud box dims what lies behind it.
* GPU film parity on a cloud scene (the media kernels' transcendentals are glibc's, as the oracle's libm mode:
  bit-level agreement expected)."""
import json

import numpy as np
import pytest

from conftest import SCENES
from test_media import box

GOLD = json.loads((SCENES.parent / "tests" / "golden" / "reference_components.json").read_text())


def test_noise_matches_reference(pa, oracle):
    rows = np.array(GOLD["noise"], np.float32)
    prod = pa.cloud_density([1, 1, 5], rows[:, :3])
    orc = oracle.cloud_density([1, 1, 5], rows[:, :3])
    np.testing.assert_array_equal(prod[:, :4], rows[:, 3:7])
    np.testing.assert_array_equal(orc[:, :4], rows[:, 3:7])


@pytest.mark.parametrize("k", range(4))
def test_cloud_density_matches_reference(pa, oracle, k):
    g = GOLD["cloud_density"][k]
    rows = np.array(g["rows"], np.float32)
    prod = pa.cloud_density(g["params"], rows[:, :3])[:, 4]
    orc = oracle.cloud_density(g["params"], rows[:, :3])[:, 4]
    np.testing.assert_array_equal(prod, rows[:, 3])
    np.testing.assert_array_equal(orc, rows[:, 3])
    assert 0 < (rows[:, 3] > 0).mean() < 1  # a mix of empty and dense points


def cloud_scene(cloud, res=32, spp=16, depth=5, sky="1 1 1"):
    return f"""LookAt 0.5 0.5 -3  0.5 0.5 0.5  0 1 0
Camera "perspective" "float fov" [ 30 ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "zsobol" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ {depth} ]
WorldBegin
LightSource "infinite" "rgb L" [ {sky} ]
MakeNamedMedium "c" "string type" "cloud" {cloud}
AttributeBegin
  MediumInterface "c" ""
  Material "interface"
  {box(0, 1, 0, 1, 0, 1)}
AttributeEnd
"""


def test_cloud_loader(pa):
    sc = pa.Scene.from_string(cloud_scene('"float density" 2 "float g" 0.3 "point3 p1" [1 1 1]'), SCENES)
    f = sc.flat()
    info = [f.medium_info[i] for i in range(16)]
    assert f.n_media == 1 and info[0] == 2
    vals = np.ctypeslib.as_array(f.medium_values, shape=(info[11] + 3 + 512,))
    np.testing.assert_array_equal(vals[info[11]:info[11] + 3], [2, 1, 5])  # density, default wispiness, frequency
    assert vals[info[11] + 3] == 151 and f.medium_params[0] == pytest.approx(0.3)


def test_cloud_rejects_unknown_parameters(pa):
    with pytest.raises(pa.PbrtError, match="Lescale|unused"):
        pa.Scene.from_string(cloud_scene('"float Lescale" 2'), SCENES)


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_empty_cloud_is_transparent(pa, oracle):
    """density 0 and the box above y = 0.5: Density = 0 everywhere inside, so the sky seen
    through the box keeps its radiance (null collisions only) -- the mean within 1 %."""
    sc = pa.Scene.from_string(cloud_scene('"float density" 0 "point3 p0" [0 0.5 0] "point3 p1" [1 1 1]'), SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    sky = pa.Scene.from_string(cloud_scene('"float density" 0 "point3 p0" [0 0.5 0] "point3 p1" [1 1 1]')
                               .replace('MakeNamedMedium "c"', '# no medium\nMakeNamedMedium "c"')
                               .replace('MediumInterface "c" ""', 'MediumInterface "" ""'), SCENES)
    ref = _rgb(oracle, sky, oracle.render(sky, threads=8))
    assert abs(img.mean() / ref.mean() - 1) < 0.01, (img.mean(), ref.mean())


def test_dense_cloud_dims_the_sky(pa, oracle):
    thin = pa.Scene.from_string(cloud_scene('"float density" 0.2 "rgb sigma_a" [2 2 2] "rgb sigma_s" [1 1 1]'), SCENES)
    thick = pa.Scene.from_string(cloud_scene('"float density" 3 "rgb sigma_a" [2 2 2] "rgb sigma_s" [1 1 1]'), SCENES)
    a = _rgb(oracle, thin, oracle.render(thin, threads=8)).mean()
    b = _rgb(oracle, thick, oracle.render(thick, threads=8)).mean()
    assert 0 < b < a < 1.0


@pytest.mark.gpu
def test_cloud_gpu_matches_oracle(pa, oracle):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(cloud_scene('"float density" 1.5 "rgb sigma_a" [0.5 0.8 1] "rgb sigma_s" [4 4 4] '
                                          '"float g" 0.4 "float frequency" 4', res=64, spp=32), SCENES)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mean_rel = check(gpu, oracle_rgb(oracle, sc))
    print(f"cloud medium parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
