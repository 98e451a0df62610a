"""Goniometric and projection lights (GoniometricLight / ProjectionLight: lights.h:300-404,
lights.cpp:281-680): point lights whose intensity is an image lookup -- the goniometric light's
Y image at EqualAreaSphereToSquare of the light-space direction, the projection light's RGB
pixel through a perspective screen window, as an RGBIlluminantSpectrum.

* Loader: the images, their errors (non-square goniometric images, a projection light without
  "filename" or with a grey image, NaN / Inf pixels).
* Known answers on the oracle: a goniometric light with an all-white image renders the same
  bits as a point light at its position; a projection light with a white image renders, pixel
  for pixel at one sample per pixel and direct lighting only, either the bits of a point light
  with "rgb I [1 1 1]" (RGBIlluminantSpectrum(1, 1, 1) is the illuminant itself) or zero
  (outside its frustum), with large areas of both and the footprint's centre lit; a half-black
  goniometric image darkens the floor on one side only; a red / blue projection image splits
  its footprint into the two colours.
* GPU film parity on scenes with both lights."""
import numpy as np
import pytest

from conftest import SCENES


def png(path, img):
    from PIL import Image
    img = np.asarray(img)
    Image.fromarray(img.astype(np.uint8), mode="L" if img.ndim == 2 else "RGB").save(path)


HEAD = """LookAt 0 4 -4  0 0 0  0 1 0
Camera "perspective" "float fov" 50
Film "rgb" "integer xresolution" {res} "integer yresolution" {res}
Sampler "halton" "integer pixelsamples" {spp}
Integrator "volpath" "integer maxdepth" {depth}
PixelFilter "box"
WorldBegin
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-5 0 -5 5 0 -5 5 0 5 -5 0 5]
"""


def scene(pa, tmp_path, light, res=48, spp=1, depth=1, extra=""):
    text = HEAD.format(res=res, spp=spp, depth=depth) + extra + light
    return pa.Scene.from_string(text, tmp_path)


def rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_goniometric_loader(pa, tmp_path):
    png(tmp_path / "g.png", np.full((8, 8), 255))
    sc = scene(pa, tmp_path, 'AttributeBegin\nTranslate 0 2 0\nLightSource "goniometric" "string filename" "g.png"\nAttributeEnd\n')
    f = sc.flat()
    d = np.ctypeslib.as_array(f.delta_lights, shape=(f.n_delta_lights * 24,)).reshape(-1, 24)
    assert d[0, 0] == 3 and f.n_point_spot == 1
    np.testing.assert_array_equal(d[0, 5:8], [0, 2 - 4, 0 + 4])  # render space: world - camera position
    assert d[0, 22] == 8 and d[0, 23] == 8 and d[0, 20] > 0


@pytest.mark.parametrize("light, msg", [
    ('LightSource "goniometric" "string filename" "rect.png"\n', "non-square"),
    ('LightSource "projection" "float fov" 40\n', "Must provide \"filename\""),
    ('LightSource "projection" "string filename" "grey.png"\n', "must have R, G, and B"),
])
def test_image_light_errors(pa, tmp_path, light, msg):
    png(tmp_path / "rect.png", np.full((4, 8), 200))
    png(tmp_path / "grey.png", np.full((8, 8), 200))
    png(tmp_path / "rgb.png", np.full((8, 8, 3), 200))
    with pytest.raises(pa.PbrtError, match=msg):
        scene(pa, tmp_path, light)


def test_goniometric_white_equals_point(pa, oracle, tmp_path):
    png(tmp_path / "g.png", np.full((16, 16), 255))
    xf = "AttributeBegin\nTranslate 0.3 2 -0.2\nRotate 30 1 0 0\n"
    I = '"spectrum I" [300 1 800 1] "float scale" 3'
    g = scene(pa, tmp_path, xf + f'LightSource "goniometric" "string filename" "g.png" {I}\nAttributeEnd\n', spp=4, depth=3)
    p = scene(pa, tmp_path, xf + f'LightSource "point" {I}\nAttributeEnd\n', spp=4, depth=3)
    a, b = oracle.render(g, threads=8), oracle.render(p, threads=8)
    assert a[:3].sum() > 0
    np.testing.assert_array_equal(a, b)


def test_goniometric_half_image(pa, oracle, tmp_path):
    """Y = 1 where the equal-area square's u < 1/2, 0 elsewhere: the light shines only into
    directions whose light-space x is negative (EqualAreaSphereToSquare keeps the sign of x)."""
    img = np.zeros((16, 16))
    img[:, :8] = 255
    png(tmp_path / "half.png", img)
    # light space after Create's swapYZ: x = render x; the camera looks down at the floor
    sc = scene(pa, tmp_path, 'AttributeBegin\nTranslate 0 2 0\nLightSource "goniometric" "string filename" "half.png"\nAttributeEnd\n',
               res=64, spp=4)
    im = rgb(oracle, sc, oracle.render(sc, threads=8)).sum(axis=-1)
    # the camera's image x runs along render -x... compare the two halves: one lit, one dark
    left, right = im[:, :28].mean(), im[:, 36:].mean()
    assert max(left, right) > 0 and min(left, right) < 1e-3 * max(left, right), (left, right)


def test_projection_white_equals_point_inside_frustum(pa, oracle, tmp_path):
    png(tmp_path / "w.png", np.full((12, 16, 3), 255))
    xf = "AttributeBegin\nTranslate 0 2 0\nRotate 90 1 0 0\n"  # light z axis points down (-y)
    proj = scene(pa, tmp_path, xf + 'LightSource "projection" "string filename" "w.png" "float fov" 50 "float scale" 2\nAttributeEnd\n',
                 res=64)
    pt = scene(pa, tmp_path, xf + 'LightSource "point" "rgb I" [1 1 1] "float scale" 2\nAttributeEnd\n', res=64)
    a, b = oracle.render(proj, threads=8), oracle.render(pt, threads=8)
    same = (a[:3] == b[:3]).all(axis=0)
    zero = (a[:3] == 0).all(axis=0)
    lit_pt = (b[:3] > 0).any(axis=0)
    assert (same | zero).all()
    inside = same & lit_pt
    assert inside.sum() > 200 and (zero & lit_pt).sum() > 200
    # the lit footprint: |x| <= 2 tan(25 deg) * aspect(4/3), |z| <= 2 tan(25 deg) on the floor;
    # at the image centre the projection light is on
    assert inside[32, 32]


def test_projection_pattern_oracle(pa, oracle, tmp_path):
    """A red / blue split image: the two halves of the footprint take the two colours."""
    img = np.zeros((16, 16, 3))
    img[:, :8, 0] = 255
    img[:, 8:, 2] = 255
    png(tmp_path / "rb.png", img)
    sc = scene(pa, tmp_path, 'AttributeBegin\nTranslate 0 2 0\nRotate 90 1 0 0\n'
               'LightSource "projection" "string filename" "rb.png" "float fov" 60\nAttributeEnd\n', res=64, spp=4)
    im = rgb(oracle, sc, oracle.render(sc, threads=8))
    red = im[..., 0] > 4 * im[..., 2]
    blue = im[..., 2] > 4 * im[..., 0]
    assert red.sum() > 100 and blue.sum() > 100


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["goniometric", "projection"])
def test_image_light_gpu_matches_oracle(pa, oracle, tmp_path, kind):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    y, x = np.mgrid[0:32, 0:32]
    png(tmp_path / "g.png", 128 + 120 * np.sin(x / 5.0) * np.cos(y / 7.0))
    png(tmp_path / "p.png", np.stack([128 + 120 * np.sin(x / 4.0), 128 + 100 * np.cos(y / 6.0), np.full_like(x, 90)], -1))
    light = ('AttributeBegin\nTranslate 0.2 2 0.1\nRotate 80 1 0 0\n' +
             ('LightSource "goniometric" "string filename" "g.png" "float scale" 4\n' if kind == "goniometric" else
              'LightSource "projection" "string filename" "p.png" "float fov" 70 "float scale" 4\n') + 'AttributeEnd\n')
    extra = ('Material "conductor" "float roughness" 0.2\nShape "trianglemesh" "integer indices" [0 1 2] '
             '"point3 P" [-1 0.01 1 1 0.01 1 0 1.2 1.5]\n')
    sc = scene(pa, tmp_path, light, res=96, spp=16, depth=5, extra=extra)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"{kind} light parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_projection_power_known_answer(pa, oracle, tmp_path):
    """ProjectionLight "power" (lights.cpp:479-511): scale = power / (A * the image's mean
    luminance weighted by dw/dA = cos^3): for a white image the light emits its power into the
    frustum, so doubling "power" doubles the scale, and the scale matches that integral
    evaluated here in float64 (sRGB luminance vector; 8-bit 255 = 1 after the sRGB decode)."""
    png(tmp_path / "w.png", np.full((6, 8, 3), 255))
    base = 'LightSource "projection" "string filename" "w.png" "float fov" 50'

    def scale(extra):
        sc = scene(pa, tmp_path, base + extra + "\n")
        f = sc.flat()
        return np.ctypeslib.as_array(f.delta_lights, shape=(f.n_delta_lights * 24,)).reshape(-1, 24)[0, 2]

    s0, s1, s2 = scale(""), scale(' "float power" 10'), scale(' "float power" 20')
    assert s2 / s1 == pytest.approx(2, rel=1e-6)
    w, h, fov = 8, 6, 50.0
    aspect = w / h
    inv_tan = 1 / np.tan(np.radians(fov) / 2)
    xs = -aspect + 2 * aspect * (np.arange(w) + 0.5) / w
    ys = -1 + 2 * (np.arange(h) + 0.5) / h
    X, Y = np.meshgrid(xs / inv_tan, ys / inv_tan)
    dwdA = (1 / np.sqrt(X * X + Y * Y + 1)) ** 3
    A = 4 * np.tan(np.radians(fov) / 2) ** 2 * aspect
    k_e = A * dwdA.mean() * 1.0  # luminance of white = 1
    assert s1 / s0 == pytest.approx(10 / k_e, rel=1e-4)
