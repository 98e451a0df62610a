"""ImageInfiniteLight (lights.h:557-641, lights.cpp:1038-1083, 1558-1694): environment image
readers, the equal-area mapping / compensated distribution / per-pixel spectra against the
oracle's independent restatement (bit-exact, both on the host), a furnace known answer, and
GPU film parity.

Fixtures come from scenes/gen_env.py (its own EXR encoder for the NONE / RLE / ZIPS / ZIP
codecs).  pbrt's own EXR path goes through the OpenEXR library, which is absent here: the
decoded pixels are checked against the arrays the generator encoded."""
import importlib.util

import numpy as np
import pytest

from conftest import SCENES

TEX = SCENES / "textures"


def _gen():
    spec = importlib.util.spec_from_file_location("gen_env", SCENES / "gen_env.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


SCENE = """LookAt 0 0.5 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 48 "integer yresolution" 32
Sampler "halton" "integer pixelsamples" 8
Integrator "volpath" "integer maxdepth" 5
WorldBegin
AttributeBegin
Rotate -90 1 0 0
LightSource "infinite" "string filename" "textures/{fn}" "float scale" 0.7
AttributeEnd
Material "diffuse" "rgb reflectance" [0.6 0.5 0.4]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 -1 -3 3 -1 -3 3 -1 3 -3 -1 3]
Material "conductor" "float roughness" 0.15
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 1 1 -1 1 1 1 1 -1 1 1]
Material "dielectric" "float roughness" 0.05
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [1.2 -1 0 2.2 -1 0 2.2 0.5 -0.5 1.2 0.5 -0.5]
"""


def _env_rgb(sc):
    f = sc.flat()
    n = f.env_info[0]
    return np.ctypeslib.as_array(f.env_rgb, shape=(n * n * 3,)).reshape(n, n, 3).copy()


@pytest.mark.parametrize("fn, half", [("env_sky_zip.exr", True), ("env_sky_rle.exr", True),
                                      ("env_sky_zips.exr", False), ("env_sky_none.exr", False),
                                      ("env_sky.pfm", False)])
def test_environment_readers_decode_the_encoded_pixels(pa, fn, half):
    want = _gen().sky(64)
    if half:
        want = want.astype(np.float16).astype(np.float32)
    got = _env_rgb(pa.Scene.from_string(SCENE.format(fn=fn), SCENES))
    assert np.array_equal(got, want)


def test_png_environment_is_srgb_decoded(pa):
    from PIL import Image
    b = np.asarray(Image.open(TEX / "env_sky.png").convert("RGB")).astype(np.float64) / 255
    lin = np.where(b <= 0.04045, b / 12.92, ((b + 0.055) / 1.055) ** 2.4)
    got = _env_rgb(pa.Scene.from_string(SCENE.format(fn="env_sky.png"), SCENES))
    assert np.abs(got - lin).max() < 1e-6


@pytest.mark.parametrize("fn", ["env_sky.pfm", "env_sky_zip.exr", "env_sky.png", "env_const.pfm"])
def test_env_lookups_match_oracle_bitwise(pa, oracle, fn):
    """Le's (u, v), PDF_Li, the pixel spectra, the compensated distribution's samples and the
    sampled directions: the product's shared host/device code vs the oracle, bit for bit."""
    sc = pa.Scene.from_string(SCENE.format(fn=fn), SCENES)
    rng = np.random.default_rng(7)
    d = rng.normal(size=(4000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d[:8] = [[0, 0, 1], [0, 0, -1], [1, 0, 0], [0, 1, 0], [-1, 0, 0], [0, -1, 0], [1, 1, 0], [0, 1, 1]]
    u = rng.random((4000, 2), dtype=np.float32)
    u[:4] = [[0, 0], [0.99999994, 0.99999994], [0.5, 0.5], [0, 0.99999994]]
    a = sc.env_eval(0, d, u)
    b = oracle.env_eval(sc, 0, d, u)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert (a[:, 9] > 0).all()  # every pixel of these maps has mass (compensation leaves some)


def test_compensated_distribution_follows_the_sun(pa):
    """Sampling concentrates where the map is brightest above its mean (lights.cpp:1064-1070):
    most samples land within the sun's cone."""
    sc = pa.Scene.from_string(SCENE.format(fn="env_sky.pfm"), SCENES)
    u = np.random.default_rng(3).random((20000, 2), dtype=np.float32)
    out = sc.env_eval(0, np.tile([0, 0, 1.0], (20000, 1)), u)
    # light space: the sun direction of gen_env.sky; render space = Rotate(-90, x) of it
    s = np.array([0.3, 0.5, 0.81]) / np.linalg.norm([0.3, 0.5, 0.81])
    s_render = np.array([s[0], s[2], -s[1]])
    wi = out[:, 10:13] / np.linalg.norm(out[:, 10:13], axis=1, keepdims=True)
    assert (wi @ s_render > 0.99).mean() > 0.5


def test_constant_environment_furnace(pa, oracle):
    """A constant 0.5 grey map over a white Lambertian quad seen head on, one bounce: every
    pixel reflects 0.5 (a furnace known answer, as for the uniform light of the same radiance)."""
    text = """LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 20
Film "rgb" "integer xresolution" 16 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 64
Integrator "volpath" "integer maxdepth" 1
WorldBegin
LightSource "infinite" "string filename" "textures/env_const.pfm"
Material "diffuse" "rgb reflectance" [1 1 1]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0 1 -1 0 1 1 0 -1 1 0]
"""
    for t in (text, text.replace('"string filename" "textures/env_const.pfm"', '"rgb L" [0.5 0.5 0.5]')):
        sc = pa.Scene.from_string(t, SCENES)
        f = sc.flat()
        img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
        assert img[2:14, 2:14].mean() == pytest.approx(0.5, abs=0.01)


def _write_pfm(path, img):
    h, w = img.shape[:2]
    path.write_bytes(b"PF\n%d %d\n-1\n" % (w, h) + np.ascontiguousarray(img[::-1]).astype("<f4").tobytes())


def test_env_loader_errors(pa, tmp_path):
    _write_pfm(tmp_path / "rect.pfm", np.ones((4, 8, 3), np.float32))
    nan = np.ones((4, 4, 3), np.float32)
    nan[1, 2, 0] = np.nan
    _write_pfm(tmp_path / "nan.pfm", nan)
    inf = np.ones((4, 4, 3), np.float32)
    inf[0, 0, 1] = np.inf
    _write_pfm(tmp_path / "inf.pfm", inf)
    _write_pfm(tmp_path / "ok.pfm", np.ones((4, 4, 3), np.float32))
    piz = bytearray((TEX / "env_sky_none.exr").read_bytes())
    k = piz.index(b"compression\0compression\0") + len(b"compression\0compression\0") + 4
    piz[k] = 4
    (tmp_path / "piz.exr").write_bytes(bytes(piz))
    (tmp_path / "grey.png").write_bytes((TEX / "bumps_grey16.png").read_bytes())
    cases = [
        ('"string filename" "rect.pfm"', "non-square"),
        ('"string filename" "nan.pfm"', "not-a-number"),
        ('"string filename" "inf.pfm"', "infinite pixel values"),
        ('"string filename" "piz.exr"', "PIZ is not supported"),
        ('"string filename" "grey.png"', "must have R, G, and B channels"),
        ('"string filename" "missing.exr"', "unable to open|No such file|cannot open"),
        ('"string filename" "rect.pfm" "rgb L" [1 1 1]', "Can't specify both"),
        ('"point3 portal" [0 0 0 1 0 0 1 1 0 0 1 0]', "portal"),
    ]
    for params, msg in cases:
        text = SCENE.replace('"string filename" "textures/{fn}" "float scale" 0.7', params)
        with pytest.raises(pa.PbrtError, match=msg):
            pa.Scene.from_string(text, tmp_path)


def test_uniform_infinite_light_illuminance(pa):
    """UniformInfiniteLight "illuminance" E_v: scale *= E_v / pi (lights.cpp:1581-1597)"""
    base = 'LightSource "infinite" "rgb L" [0.2 0.3 0.4]'
    a = pa.Scene.from_string(SCENE.replace('LightSource "infinite" "string filename" "textures/{fn}" "float scale" 0.7',
                                           base), SCENES).flat()
    b = pa.Scene.from_string(SCENE.replace('LightSource "infinite" "string filename" "textures/{fn}" "float scale" 0.7',
                                           base + ' "float illuminance" 2.5'), SCENES).flat()
    assert b.inf_scale[0] == np.float32(np.float32(a.inf_scale[0]) * np.float32(np.float32(2.5) / np.float32(np.pi)))


def test_image_infinite_light_illuminance(pa, tmp_path):
    """ImageInfiniteLight "illuminance" (lights.cpp:1651-1679): scale *= E_v / (the map's
    upper-hemisphere illuminance).  The reference sums the equal-area pixels above the horizon
    with the weight 2 pi / (w h) rather than the pixel solid angle 4 pi / (w h), so a constant map
    c measures c pi / 2 (half the cosine integral pi c) and its scale is 2 E_v / pi / c to the
    discretisation -- the reference's own normalisation, kept; the sky map's scale follows the
    same formula restated here in float64."""
    _write_pfm(tmp_path / "c.pfm", np.full((64, 64, 3), 0.5, np.float32))
    line = 'LightSource "infinite" "string filename" "textures/{fn}" "float scale" 0.7'
    plain = pa.Scene.from_string(SCENE.replace(line, 'LightSource "infinite" "string filename" "c.pfm"'), tmp_path).flat()
    lit = pa.Scene.from_string(SCENE.replace(line, 'LightSource "infinite" "string filename" "c.pfm" '
                                                   '"float illuminance" 3'), tmp_path).flat()
    ratio = lit.inf_scale[0] / plain.inf_scale[0]
    assert ratio == pytest.approx(2 * 3 / np.pi / 0.5, rel=2e-3)
    # the sky map: the formula in float64 over the loader's own pixels, with the sRGB luminance
    # vector (XYZFromRGB row 1) and EqualAreaSquareToSphere's z (1 - r^2, r = 1 - |1 - |2u - 1| - |2v - 1||
    # at the pixel centre, signed by the inner square: util/math.cpp:292-330)
    sky = pa.Scene.from_string(SCENE.format(fn="env_sky.pfm"), SCENES)
    sky_lit = pa.Scene.from_string(SCENE.format(fn="env_sky.pfm").replace('"float scale" 0.7',
                                                                           '"float scale" 0.7 "float illuminance" 2'), SCENES)
    f = sky.flat()
    res = f.env_info[0]
    rgb = np.ctypeslib.as_array(f.env_rgb, shape=(res * res * 3,)).reshape(res, res, 3).astype(np.float64)
    c = (np.arange(res) + 0.5) / res
    u, v = np.meshgrid(c, c)
    r = 1 - np.abs(np.abs(2 * u - 1) + np.abs(2 * v - 1) - 1)
    z = np.where(np.abs(2 * u - 1) + np.abs(2 * v - 1) <= 1, 1 - r * r, -(1 - r * r))
    lum = np.array([0.212639, 0.715169, 0.072192])
    ill = (rgb @ lum * np.where(z > 0, z, 0)).sum() * 2 * np.pi / (res * res)
    assert sky_lit.flat().inf_scale[0] / f.inf_scale[0] == pytest.approx(2.0 / ill, rel=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("fn", ["env_sky.pfm", "env_sky_zip.exr"])
def test_env_scene_matches_oracle_gpu(pa, oracle, fn):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.Scene.from_string(SCENE.format(fn=fn).replace('"integer pixelsamples" 8', '"integer pixelsamples" 16'),
                              SCENES, xresolution=96, yresolution=64)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"env light ({fn}) parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_env_scene_zsobol_bvh_sampler_gpu(pa, oracle):
    """The env light beside an area light: the BVH light sampler's infinite-light branch and the
    escaped-ray MIS PMF (BVHLightSampler::PMF of an infinite light)."""
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    text = SCENE.format(fn="env_sky.pfm").replace(
        'Sampler "halton" "integer pixelsamples" 8', 'Sampler "zsobol" "integer pixelsamples" 16').replace(
        "AttributeEnd\n", 'AttributeEnd\nAttributeBegin\nAreaLightSource "diffuse" "rgb L" [4 4 4]\n'
        'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.5 2 -0.5 0.5 2 -0.5 0.5 2 0.5 -0.5 2 0.5]\n'
        'AttributeEnd\n', 1)
    sc = pa.Scene.from_string(text, SCENES, xresolution=96, yresolution=64)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"env + area light parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def _env_volumetric_scenes():
    from test_media import box
    coated = SCENE.format(fn="env_sky.pfm").replace('Material "diffuse" "rgb reflectance" [0.6 0.5 0.4]',
                                                    'Material "coateddiffuse" "rgb reflectance" [0.6 0.5 0.4] '
                                                    '"float roughness" 0.2')
    coated += ('MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.3 0.5 0.2] '
               '"rgb sigma_s" [1.2 0.8 1.5] "float g" 0.4\n'
               'AttributeBegin\nMediumInterface "m" ""\nMaterial "interface"\n' + box(-2.6, -1.6, -0.9, 0.1, -0.5, 0.5) +
               '\nAttributeEnd\n')
    iface = SCENE.format(fn="env_sky.pfm") + ('AttributeBegin\nMaterial "interface"\n' +
                                              box(-2.6, -1.6, -0.9, 0.1, -0.5, 0.5) + '\nAttributeEnd\n')
    return {"coated+medium": coated, "interface": iface}


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["coated+medium", "interface"])
def test_env_volumetric_queues_have_no_holes_gpu(pa, oracle, name):
    """Regression test for the round-3 volumetric-kernel defect: the image-light
    volumetric kernels (k_vsurface<..., Ext>) counted shadow-queue slots they never wrote, which
    left a NaN at pixel 0 and then faulted.  With the queue-integrity check on, every counted
    slot of the surface, layered and scattering stages must be written, and the film must be
    the same bits as with the check off."""
    from test_gpu_media import gpu_rgb
    sc = pa.Scene.from_string(_env_volumetric_scenes()[name], SCENES, xresolution=96, yresolution=64)
    pa.queue_holes()
    pa.set_queue_check(True)
    try:
        a, _ = gpu_rgb(pa, oracle, sc)
        holes = pa.queue_holes()
    finally:
        pa.set_queue_check(False)
    b, _ = gpu_rgb(pa, oracle, sc)
    assert holes == 0
    assert np.isfinite(b).all()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
def test_env_coated_and_medium_match_oracle_gpu(pa, oracle):
    """The volumetric kernels with an image light: a coated-diffuse floor (layered BSDF) and a
    homogeneous-medium box, NEE from surface and medium points and escaped-ray MIS.  The
    oracle runs in its libm mode (conftest), as for the other media tests."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    from test_media import box
    text = SCENE.format(fn="env_sky.pfm").replace('Material "diffuse" "rgb reflectance" [0.6 0.5 0.4]',
                                                  'Material "coateddiffuse" "rgb reflectance" [0.6 0.5 0.4] '
                                                  '"float roughness" 0.2')
    text += ('MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.3 0.5 0.2] '
             '"rgb sigma_s" [1.2 0.8 1.5] "float g" 0.4\n'
             'AttributeBegin\nMediumInterface "m" ""\nMaterial "interface"\n' + box(-2.6, -1.6, -0.9, 0.1, -0.5, 0.5) +
             '\nAttributeEnd\n')
    sc = pa.Scene.from_string(text, SCENES, xresolution=96, yresolution=64)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"env + coated + medium parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")


def test_interface_surfaces_pass_shadow_rays(pa, oracle):
    """An "interface" material makes pbrt trace shadow rays with IntersectShadowTr, which passes
    interface surfaces (wavefront/integrator.cpp:49-110 haveMedia): a distant light behind an
    interface quad lights the floor exactly as without the quad."""
    text = """LookAt 0 3 -6  0 0 0  0 1 0
Camera "perspective" "float fov" 30
Film "rgb" "integer xresolution" 24 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 4
Integrator "volpath" "integer maxdepth" 1
WorldBegin
LightSource "distant" "point3 from" [0 10 0] "point3 to" [0 0 0] "rgb L" [2 2 2]
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3]
"""
    quad = ('AttributeBegin\nMaterial "interface"\nShape "trianglemesh" "integer indices" [0 1 2 0 2 3] '
            '"point3 P" [-9 6 -9 9 6 -9 9 6 9 -9 6 9]\nAttributeEnd\n')
    a = oracle.render(pa.Scene.from_string(text, SCENES), threads=4)
    b = oracle.render(pa.Scene.from_string(text + quad, SCENES), threads=4)
    assert a[0].sum() > 0
    np.testing.assert_allclose(b, a, rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_env_through_interface_surfaces_gpu(pa, oracle):
    """Image-light NEE shadow rays crossing an interface-only box (no media)."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    from test_media import box
    text = SCENE.format(fn="env_sky.pfm") + ('AttributeBegin\nMaterial "interface"\n' +
                                             box(-2.6, -1.6, -0.9, 0.1, -0.5, 0.5) + '\nAttributeEnd\n')
    sc = pa.Scene.from_string(text, SCENES, xresolution=96, yresolution=64)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"env through interfaces parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")


# ---------------------------------------------------------------- reference goldens
# tests/golden/reference_components.json "equal_area" / "env_distribution": the reference's own
# EqualAreaSquareToSphere / EqualAreaSphereToSquare (util/math.cpp) and PiecewiseConstant2D
# (util/sampling.h) over the compensated distribution of a seeded RGB map (oracle/ref/refgold.cpp
# EnvGoldens; the per-pixel average and compensation loops of image.cpp / lights.cpp are restated
# there because those files do not compile here).
def test_equal_area_mapping_matches_reference_goldens(pa, oracle, golden):
    from conftest import fl
    rows = golden["equal_area"]
    p = np.array([fl(r["p"]) for r in rows], np.float32)
    d = np.array([fl(r["d"]) for r in rows], np.float32)
    sphere = np.array([fl(r["sphere"]) for r in rows], np.float32)
    square = np.array([fl(r["square"]) for r in rows], np.float32)
    for impl in (pa, oracle):
        assert np.array_equal(impl.equal_area(p, True).view(np.uint32), sphere.view(np.uint32))
        assert np.array_equal(impl.equal_area(d, False).view(np.uint32), square.view(np.uint32))


@pytest.mark.parametrize("ci", range(3))
def test_env_distribution_matches_reference_goldens(pa, oracle, golden, tmp_path, ci):
    """The image infinite light's compensated PiecewiseConstant2D: Sample(u) -> (u, v) and its
    pdf, PDF at the sample and PDF at arbitrary points, against the reference, bit for bit."""
    from conftest import fl
    g = golden["env_distribution"][ci]
    n = g["res"]
    _write_pfm(tmp_path / "env.pfm", np.array(fl(g["rgb"]), np.float32).reshape(n, n, 3))
    text = ('LookAt 0 0 0  0 0 1  0 1 0\nCamera "perspective"\nWorldBegin\n'
            'LightSource "infinite" "string filename" "env.pfm"\n')
    sc = pa.Scene.from_string(text, tmp_path)
    s = np.array([fl(r) for r in g["samples"]], np.float32)  # u, p, pdf, PDF(p), pq, PDF(pq)
    dirs = np.tile(np.float32([0, 0, 1]), (len(s), 1))
    for name, impl in (("product", lambda u: sc.env_eval(0, dirs, u)),
                       ("oracle", lambda u: oracle.env_eval(sc, 0, dirs, u))):
        a = impl(s[:, 0:2])
        got = np.stack([a[:, 7], a[:, 8], a[:, 9], a[:, 13]], 1)
        assert np.array_equal(got.view(np.uint32), s[:, 2:6].view(np.uint32)), name
        b = impl(s[:, 6:8])
        assert np.array_equal(b[:, 14].view(np.uint32), s[:, 8].view(np.uint32)), name
