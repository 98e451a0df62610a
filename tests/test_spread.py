"""This fork's area-light "spread" (scienstanford pbrt-v4: DiffuseAreaLight, lights.cpp:715-717,
743-775, lights.h:443-470): an emitter radiates only within `spread` degrees of its normal --
DiffuseAreaLight::L is zero where AbsDot(w, n) < cos(spread) -- and a light sample toward wi is
attenuated by max((1 - tan(Pi/2 - spread) tan(theta)) normalize, 0).  90 degrees (the default)
changes nothing (cos(Radians(90)) < 0 in float).

* Loader: the three float terms as the constructor computes them.
* Known answers (oracle): spread 90 renders the same bits as no spread; seen from outside its
  cone an emitter is black (its emission term vanishes), from inside it is unchanged; direct
  light under a narrow spread vanishes on the floor far off the light's axis and stays on
  near it.
* GPU film parity with a spread emitter, surfaces and a medium."""
import math

import numpy as np
import pytest

from conftest import SCENES

LIGHT = """AttributeBegin
AreaLightSource "diffuse" "rgb L" [4 4 4] {spread}
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.3 2 -0.3 0.3 2 -0.3 0.3 2 0.3 -0.3 2 0.3]
AttributeEnd
"""


def scene(pa, spread="", eye="0 3 -4", look="0 0.5 0", depth=1, res=48, spp=4, extra=""):
    text = (f'LookAt {eye}  {look}  0 1 0\nCamera "perspective" "float fov" 60\n'
            f'Film "rgb" "integer xresolution" {res} "integer yresolution" {res}\n'
            f'Sampler "halton" "integer pixelsamples" {spp}\nIntegrator "volpath" "integer maxdepth" {depth}\n'
            'PixelFilter "box"\nWorldBegin\nMaterial "diffuse" "rgb reflectance" [0.5 0.5 0.5]\n'
            'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-6 0 -6 6 0 -6 6 0 6 -6 0 6]\n'
            + extra + LIGHT.format(spread=spread))
    return pa.Scene.from_string(text, SCENES)


def rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_spread_loader(pa):
    for deg in (90, 30, 5):
        f = scene(pa, f'"float spread" {deg}').flat()
        sp = np.ctypeslib.as_array(f.light_spread, shape=(f.n_area_lights * 3,)).reshape(-1, 3)[0]
        rad = np.float32(np.float32(math.pi / 180) * np.float32(deg))
        assert sp[0] == np.float32(math.cos(rad)) or abs(sp[0] - math.cos(rad)) < 1e-7
        if deg == 90:
            assert sp[0] < 0
        else:
            tan_e = math.tan(math.pi / 2 - rad)
            assert abs(sp[1] - tan_e) <= 1e-6 * max(1, tan_e)
            norm = 2 / (2 + (2 * (math.pi / 2 - rad) - math.pi) * tan_e)
            assert abs(sp[2] - norm) <= 1e-5 * abs(norm)


def test_spread_90_is_default(pa, oracle):
    a = oracle.render(scene(pa), threads=8)
    b = oracle.render(scene(pa, '"float spread" 90'), threads=8)
    np.testing.assert_array_equal(a, b)


def test_emitter_black_outside_its_spread(pa, oracle):
    """The camera sees the light's underside at about 50 degrees off its normal: visible with
    a 70 degree spread, black (its own emission) with 30 degrees; depth 0 = emission only."""
    kw = dict(eye="0 0.2 -1.8", look="0 2 0", depth=0, res=32, spp=4)
    wide = rgb(oracle, sc := scene(pa, '"float spread" 70', **kw), oracle.render(sc, threads=8))
    narrow = rgb(oracle, sc2 := scene(pa, '"float spread" 30', **kw), oracle.render(sc2, threads=8))
    none = rgb(oracle, sc3 := scene(pa, **kw), oracle.render(sc3, threads=8))
    assert wide.max() > 0
    np.testing.assert_array_equal(wide, none)
    assert narrow.max() == 0


def test_direct_light_vanishes_far_off_axis(pa, oracle):
    """maxdepth 1 (direct light only), spread 20: floor points 2 below the light and more than
    2 tan(20 deg) + the light's half size away from its axis get no direct light."""
    sc = scene(pa, '"float spread" 20', eye="0 6 -0.01", look="0 0 0", res=64, spp=4)
    im = rgb(oracle, sc, oracle.render(sc, threads=8)).sum(axis=-1)
    ref = rgb(oracle, sc0 := scene(pa, eye="0 6 -0.01", look="0 0 0", res=64, spp=4),
              oracle.render(sc0, threads=8)).sum(axis=-1)
    # the camera looks straight down from 6 above: pixel -> floor point via the fov
    n = 64
    t = np.tan(np.radians(30))
    c = (np.arange(n) + 0.5) / n * 2 - 1
    x, z = np.meshgrid(c * 6 * t, -c * 6 * t)
    r = np.hypot(x, z)
    far = r > 2 * np.tan(np.radians(20)) + 0.45
    # the ring just outside the light's own shadow (the quad hides r < 0.45 from the camera)
    ring = (r > 0.5) & (r < 0.8)
    assert ref[far].min() > 0 and im[far].max() == 0
    assert im[ring].mean() > 0.1 * ref[ring].mean()


@pytest.mark.gpu
@pytest.mark.parametrize("medium", [False, True])
def test_spread_gpu_matches_oracle(pa, oracle, medium):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    extra = ('Material "conductor" "float roughness" 0.3\nShape "trianglemesh" "integer indices" [0 1 2] '
             '"point3 P" [-1 0 1 1 0 1 0 1.3 1.2]\n')
    if medium:  # a fog-filled interface box between the light and the floor (the volumetric kernels)
        from test_media import box
        extra += ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.05 0.05 0.05] '
                  '"rgb sigma_s" [0.4 0.4 0.4]\nAttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\n'
                  + box(-1.5, 1.5, 0.05, 1.5, -1.5, 0.8) + '\nAttributeEnd\n')
    sc = scene(pa, '"float spread" 35', depth=5, res=80, spp=16, extra=extra)
    if medium:  # the media kernels round transcendentals once from double: the oracle's CR mode
        from test_gpu_media import check, gpu_rgb, oracle_rgb
        frac, mean_rel = check(gpu_rgb(pa, oracle, sc)[0], oracle_rgb(oracle, sc))
    else:
        film, _ = gpu_film(pa, sc)
        frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"spread (medium={medium}) parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
