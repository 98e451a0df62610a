"""Point, spot and distant lights (PointLight, SpotLight, DistantLight: lights.h:200-300, 740-800,
lights.cpp:168-276, 1376-1495) on the surface wavefront: SampleLi with pdf 1, no BSDF MIS weight
(IsDeltaLight), point and spot lights in the light BVH after the area lights (their
LightBounds), distant lights in the infinite-light list with the uniform infinite lights, in the
order the LightSource directives are written.

Known answers (oracle here; the GPU repeats them in the gpu tests below): a diffuse plane
(reflectance 0.5) under a point or spot light of I = rgb(1 1 1) with "scale" pi h^2 at height h,
or under a distant light of L = rgb(1 1 1) with "scale" pi, reflects radiance 0.5 where the light
falls perpendicularly (the photometric normalisation makes rgb(1 1 1) unit RGB); outside a spot
light's cone the plane is black.  GPU parity: the Cornell box with point, spot and distant lights
added beside its area light, BVH and uniform light samplers."""
import numpy as np
import pytest

from conftest import SCENES

H = 2.0


def plane_scene(light, res=33, spp=16, fov=10, maxdepth=1, extra=""):
    return f"""
LookAt 0 10 0  0 0 0  0 0 1
Camera "perspective" "float fov" [ {fov} ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "halton" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ {maxdepth} ] {extra}
PixelFilter "box"
WorldBegin
{light}
Material "diffuse" "rgb reflectance" [ 0.5 0.5 0.5 ]
Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ]
    "point3 P" [ -100 0 -100  100 0 -100  100 0 100  -100 0 100 ]
"""


POINT = f'LightSource "point" "rgb I" [ 1 1 1 ] "float scale" {np.pi * H * H} "point3 from" [ 0 {H} 0 ]'
SPOT = (f'LightSource "spot" "rgb I" [ 1 1 1 ] "float scale" {np.pi * H * H} "point3 from" [ 0 {H} 0 ] '
        '"point3 to" [ 0 0 0 ] "float coneangle" 30 "float conedeltaangle" 5')
DISTANT = f'LightSource "distant" "rgb L" [ 1 1 1 ] "float scale" {np.pi} "point3 from" [ 0 1 0 ] "point3 to" [ 0 0 0 ]'


def _oracle_rgb(pa, oracle, text):
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    film = oracle.render(sc, threads=8)
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_loader(pa):
    sc = pa.Scene.from_string(plane_scene(POINT + "\n" + DISTANT + "\n" + SPOT), SCENES)
    f = sc.flat()
    assert f.n_area_lights == 0 and f.n_delta_lights == 3 and f.n_point_spot == 2 and f.n_infinite_lights == 1
    d = np.ctypeslib.as_array(f.delta_lights, shape=(3, 24))
    assert d[0, 0] == 0 and d[1, 0] == 1 and d[2, 0] == 2  # point, spot, then the distant light
    np.testing.assert_allclose(d[0, 5:8], [0, H - 10, 0], atol=1e-5)  # render space: camera at the origin
    assert f.inf_distant[0] == 2
    # pbrt's light order: point, distant, spot -> global indices 0, 2 (infinite list), 1
    assert [f.uniform_order[i] for i in range(3)] == [0, 2, 1]
    # cos(30 deg), cos(25 deg)
    assert d[1, 4] == pytest.approx(np.cos(np.radians(30)), rel=1e-6)
    assert d[1, 3] == pytest.approx(np.cos(np.radians(25)), rel=1e-6)
    assert f.n_light_nodes == 3  # the point and the spot light in the light BVH
    with pytest.raises(RuntimeError, match="not supported"):
        pa.Scene.from_string(plane_scene('LightSource "goniometric"'), SCENES)


@pytest.mark.parametrize("light", [POINT, SPOT, DISTANT], ids=["point", "spot", "distant"])
def test_plane_known_answer(pa, oracle, light):
    img = _oracle_rgb(pa, oracle, plane_scene(light))
    c = img[16, 16]
    np.testing.assert_allclose(c, [0.5, 0.5, 0.5], rtol=2e-3)
    if light is DISTANT:  # uniform irradiance: the whole plane
        np.testing.assert_allclose(img, 0.5, rtol=2e-3)


def test_spot_cone(pa, oracle):
    """Wide view: beyond the 30-degree cone (radius h tan 30 on the plane) nothing is lit; inside
    the 25-degree inner cone the plane matches the point light."""
    spot = _oracle_rgb(pa, oracle, plane_scene(SPOT, res=41, fov=40, spp=4))
    point = _oracle_rgb(pa, oracle, plane_scene(POINT, res=41, fov=40, spp=4))
    half = 10 * np.tan(np.radians(20))  # half width of the visible plane
    x = (np.arange(41) + 0.5) / 41 * 2 * half - half
    r = np.hypot(*np.meshgrid(x, x))
    pix = 2 * half / 41 * 0.75  # a pixel's samples reach this far from its centre
    outside, inside = r > H * np.tan(np.radians(30)) + pix, r < H * np.tan(np.radians(25)) - pix
    assert outside.sum() > 100 and inside.sum() > 40
    assert np.abs(spot[outside]).max() == 0
    np.testing.assert_allclose(spot[inside], point[inside], rtol=1e-6)


def cornell_with_delta(extra=""):
    text = (SCENES / "cornell-box.pbrt").read_text()
    lights = ('LightSource "point" "rgb I" [ 0.9 0.8 0.6 ] "float power" 4e5 "point3 from" [ 150 450 250 ]\n'
              'LightSource "distant" "blackbody L" [ 5500 ] "float scale" 0.3 "point3 from" [ 278 600 -400 ] '
              '"point3 to" [ 278 273 280 ]\n'
              'LightSource "spot" "spectrum I" [ 400 1 550 3 700 2 ] "float power" 3e5 "point3 from" [ 400 500 100 ] '
              '"point3 to" [ 250 0 300 ] "float coneangle" 35 "float conedeltaangle" 10\n')
    text = text.replace("WorldBegin", "WorldBegin\n" + lights)
    if extra:
        text = text.replace('"integer maxdepth" [ 5 ]', '"integer maxdepth" [ 5 ] ' + extra)
    return text


def test_cornell_with_delta_lights_renders(pa, oracle):
    sc = pa.Scene.from_string(cornell_with_delta(), SCENES, xresolution=32, yresolution=32, spp=4)
    f = sc.flat()
    assert f.n_area_lights == 2 and f.n_point_spot == 2 and f.n_infinite_lights == 1
    img = _oracle_rgb(pa, oracle, cornell_with_delta().replace('[ 256 ]', '[ 32 ]').replace('[ 16 ]', '[ 4 ]'))
    assert np.isfinite(img).all() and img.mean() > 0


# ---------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("light", [POINT, SPOT, DISTANT], ids=["point", "spot", "distant"])
def test_plane_known_answer_gpu(pa, oracle, light):
    from test_gpu_media import gpu_rgb
    sc = pa.Scene.from_string(plane_scene(light), SCENES)
    img, _ = gpu_rgb(pa, oracle, sc)
    np.testing.assert_allclose(img[16, 16], [0.5, 0.5, 0.5], rtol=2e-3)
    ref = _oracle_rgb(pa, oracle, plane_scene(light))
    np.testing.assert_allclose(img, ref, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("sampler", ["", '"string lightsampler" "uniform"'], ids=["bvh", "uniform"])
def test_cornell_with_delta_lights_matches_oracle(pa, oracle, sampler):
    from test_gpu_media import check, gpu_rgb
    sc = pa.Scene.from_string(cornell_with_delta(sampler), SCENES, xresolution=64, yresolution=64, spp=8)
    a, _ = gpu_rgb(pa, oracle, sc)
    f = sc.flat()
    b = oracle.film_to_rgb(oracle.render(sc, threads=16), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    frac, mr = check(a, b)
    print(f"cornell + delta lights ({sampler or 'bvh'}): {frac*100:.2f}% within 1e-3, mean rel {mr:.2e}")


DELTA3 = ('LightSource "point" "rgb I" [ 0.9 0.8 0.6 ] "float power" 40 "point3 from" [ 0.3 2.2 0.6 ]\n'
          'LightSource "distant" "rgb L" [ 1 0.9 0.8 ] "float scale" 0.5 "point3 from" [ 1 3 -1 ] "point3 to" [ 0 0 0.5 ]\n'
          'LightSource "spot" "rgb I" [ 0.5 0.7 1 ] "float power" 30 "point3 from" [ -0.8 2 0.2 ] '
          '"point3 to" [ 0 0 0.5 ] "float coneangle" 40 "float conedeltaangle" 8\n')


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["homogeneous", "grid"])
def test_media_with_delta_lights_matches_oracle(pa, oracle, kind):
    """The volumetric kernels: medium scattering and surface vertices sample point, spot and
    distant lights beside the area light (phase-function / BSDF MIS weight 0 for them)."""
    from test_gpu_media import HOMOG, LIGHT, check, gpu_rgb, grid_medium, medium_scene, oracle_rgb
    m = HOMOG if kind == "homogeneous" else grid_medium()
    sc = pa.Scene.from_string(medium_scene(m, res=40, spp=16, maxdepth=6, sky="0.3 0.4 0.5", extra=LIGHT + DELTA3,
                                           fov=35), SCENES)
    assert sc.flat().n_delta_lights == 3
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"media {kind} + delta lights: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_layered_plane_under_point_light_matches_oracle(pa, oracle):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    text = plane_scene(POINT + "\n" + SPOT, fov=40, spp=16, maxdepth=3).replace(
        'Material "diffuse" "rgb reflectance" [ 0.5 0.5 0.5 ]',
        'Material "coateddiffuse" "rgb reflectance" [ 0.6 0.4 0.2 ] "float roughness" 0.2')
    sc = pa.Scene.from_string(text, SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    check(a, oracle_rgb(oracle, sc))


@pytest.mark.gpu
def test_c3_with_delta_lights_matches_oracle(pa, oracle):
    """Rough conductor and dielectric shading (k_shade_microfacet) under a point, a spot and a
    distant light beside C3's area and infinite lights."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c3
    from test_gpu_media import check, gpu_rgb
    lights = ('LightSource "point" "rgb I" [ 1 0.9 0.8 ] "float power" 2000 "point3 from" [ 3 6 -4 ]\n'
              'LightSource "spot" "rgb I" [ 0.6 0.8 1 ] "float power" 3000 "point3 from" [ -4 5 -3 ] '
              '"point3 to" [ 0 0 0 ] "float coneangle" 25\n'
              'LightSource "distant" "rgb L" [ 1 1 1 ] "float scale" 0.8 "point3 from" [ 1 2 -1 ] "point3 to" [ 0 0 0 ]\n')
    text = gen_c3.scene_text(96, 54, 8).replace("WorldBegin", "WorldBegin\n" + lights, 1)
    sc = pa.Scene.from_string(text, SCENES)
    assert sc.flat().n_delta_lights == 3
    a, _ = gpu_rgb(pa, oracle, sc)
    f = sc.flat()
    b = oracle.film_to_rgb(oracle.render(sc, threads=16), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    frac, mr = check(a, b)
    print(f"C3 + delta lights: {frac*100:.2f}% within 1e-3, mean rel {mr:.2e}")
