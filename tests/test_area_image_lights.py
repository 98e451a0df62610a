"""Image area lights (DiffuseAreaLight with "filename": lights.cpp:898-972, lights.h:443-470):
an emitter's radiance is scale * RGBIlluminantSpectrum(ClampZero(image.Bilerp((u, 1 - v)))),
at the hit's uv for emission and at the light sample's uv (Triangle::Sample's barycentric uv)
for light sampling; the light BVH's phi is the image's mean channel value.

* Loader: the image, its errors (with "L", a grey image); "power" normalises by the image's mean luminance (lights.cpp:943-965).
* Known answers on the oracle: an all-white image emits "rgb L [1 1 1]" (the grey
  RGBIlluminantSpectrum is the illuminant itself) to the bilerp's last-bit rounding; a camera looking at a red-over-blue emitter
  sees red in the image's top half and blue in its bottom half (the v flip); a floor under a
  left-red / right-blue emitter is tinted accordingly on each side.
* Emitters on spheres, disks, cylinders and bilinear patches (the uv of their hits and of their
  shape samples): white image == "rgb L" [1 1 1] on the oracle; GPU film parity.
* GPU film parity on an image emitter scene, on the surface and the volumetric path."""
import numpy as np
import pytest

from conftest import SCENES


def png(path, img):
    from PIL import Image
    img = np.asarray(img)
    Image.fromarray(img.astype(np.uint8), mode="L" if img.ndim == 2 else "RGB").save(path)


def scene(pa, tmp_path, emitter, eye="0 3 -4", look="0 0.5 0", depth=3, res=48, spp=8, extra="", single=False):
    text = (f'LookAt {eye}  {look}  0 1 0\nCamera "perspective" "float fov" 60\n'
            f'Film "rgb" "integer xresolution" {res} "integer yresolution" {res}\n'
            f'Sampler "halton" "integer pixelsamples" {spp}\nIntegrator "volpath" "integer maxdepth" {depth}\n'
            'PixelFilter "box"\nWorldBegin\n' + extra +
            'Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]\n'
            'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-6 0 -6 6 0 -6 6 0 6 -6 0 6]\n'
            'AttributeBegin\n' + emitter + '\n'
            f'Shape "trianglemesh" "integer indices" [{"0 1 2" if single else "0 1 2 0 2 3"}] '
            '"point3 P" [-1 2 -1 1 2 -1 1 2 1 -1 2 1]\n'
            '  "point2 uv" [0 0 1 0 1 1 0 1]\nAttributeEnd\n')
    return pa.Scene.from_string(text, tmp_path)


def rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_image_emitter_loader(pa, tmp_path):
    png(tmp_path / "e.png", np.full((4, 6, 3), 255))
    sc = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "e.png" "float scale" 2')
    f = sc.flat()
    li = np.ctypeslib.as_array(f.light_image, shape=(f.n_area_lights,))
    assert f.n_area_lights == 2 and (li >= 0).all()
    img = np.ctypeslib.as_array(f.area_images, shape=(2 + 4 * 6 * 3,))
    assert img[0] == 6 and img[1] == 4 and (img[2:] == 1).all()


@pytest.mark.parametrize("emitter, msg", [
    ('AreaLightSource "diffuse" "string filename" "e.png" "rgb L" [1 1 1]', "Both"),
    ('AreaLightSource "diffuse" "string filename" "g.png"', "must have R, G, and B"),
])
def test_image_emitter_errors(pa, tmp_path, emitter, msg):
    png(tmp_path / "e.png", np.full((4, 4, 3), 200))
    png(tmp_path / "g.png", np.full((4, 4), 200))
    with pytest.raises(pa.PbrtError, match=msg):
        scene(pa, tmp_path, emitter)


SHAPES = {
    "sphere": 'Translate 0 2 0\nShape "sphere" "float radius" 0.6',
    "disk": 'Translate 0 2 0\nRotate 90 1 0 0\nShape "disk" "float radius" 0.9 "float innerradius" 0.2',
    "cylinder": 'Translate 0 1.6 0\nRotate 90 1 0 0\nShape "cylinder" "float radius" 0.4 "float zmin" -0.5 "float zmax" 0.5',
    "patch": 'Shape "bilinearmesh" "point3 P" [-1 2 -1  1 2 -1  -1 2 1  1 2 1] "point2 uv" [0 0 1 0 0 1 1 1]',
}


def shape_scene(pa, tmp_path, shape, emitter, extra="", spp=8, res=40):
    text = (f'LookAt 0 3 -4  0 0.5 0  0 1 0\nCamera "perspective" "float fov" 60\n'
            f'Film "rgb" "integer xresolution" {res} "integer yresolution" {res}\n'
            f'Sampler "halton" "integer pixelsamples" {spp}\nIntegrator "volpath" "integer maxdepth" 3\n'
            'WorldBegin\n' + extra +
            'Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]\n'
            'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-6 0 -6 6 0 -6 6 0 6 -6 0 6]\n'
            f'AttributeBegin\n{emitter}\n{SHAPES[shape]}\nAttributeEnd\n')
    return pa.Scene.from_string(text, tmp_path)


@pytest.mark.parametrize("shape", list(SHAPES))
def test_white_image_on_shape_equals_rgb_emitter(pa, oracle, tmp_path, shape):
    """an image emitter on a sphere, disk, cylinder or patch: the (u, v) of its hits and of its
    light samples look the image up; an all-white image emits "rgb L" [1 1 1]"""
    png(tmp_path / "w.png", np.full((8, 8, 3), 255))
    a = shape_scene(pa, tmp_path, shape, 'AreaLightSource "diffuse" "string filename" "w.png" "float scale" 2')
    b = shape_scene(pa, tmp_path, shape, 'AreaLightSource "diffuse" "rgb L" [1 1 1] "float scale" 2')
    fa, fb = oracle.render(a, threads=8), oracle.render(b, threads=8)
    assert fa[:3].sum() > 0
    np.testing.assert_allclose(fa, fb, rtol=3e-6, atol=0)


IMG_EXTRA = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.1 0.1 0.1] "rgb sigma_s" [0.6 0.6 0.6]\n'
             'AttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\nTranslate 1.6 0.6 0\n'
             'Shape "sphere" "float radius" 0.5\nAttributeEnd\n')


@pytest.mark.gpu
@pytest.mark.parametrize("shape", list(SHAPES))
@pytest.mark.parametrize("medium", [False, True])
def test_image_on_shape_matches_oracle_gpu(pa, oracle, tmp_path, shape, medium):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    img = np.zeros((8, 8, 3))
    img[:, :4, 0] = 255
    img[:, 4:, 2] = 255
    img[2:6, 2:6, 1] = 200
    png(tmp_path / "e.png", img)
    sc = shape_scene(pa, tmp_path, shape, 'AreaLightSource "diffuse" "string filename" "e.png" "float power" 30 '
                                          '"bool twosided" true', extra=IMG_EXTRA if medium else "", spp=16)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"image emitter on {shape} (medium={medium}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_image_emitter_with_media_matches_oracle_gpu(pa, oracle, tmp_path):
    """an image emitter on the volumetric path (a fog ball puts the scene there): emission at the
    hit's uv in k_vsurface, light samples at the sample's uv through SampleLiSurface"""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    img = np.zeros((8, 8, 3))
    img[:, :4, 0] = 255
    img[:, 4:, 2] = 255
    img[2:6, 2:6, 1] = 200
    png(tmp_path / "e.png", img)
    extra = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.1 0.1 0.1] "rgb sigma_s" [0.6 0.6 0.6]\n'
             'AttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\nTranslate 0.4 0.6 0\n'
             'Shape "sphere" "float radius" 0.5\nAttributeEnd\n')
    sc = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "e.png" "float scale" 3 "float power" 40',
               extra=extra, spp=16)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"image emitter with media: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


def test_white_image_equals_rgb_emitter(pa, oracle, tmp_path):
    png(tmp_path / "w.png", np.full((8, 8, 3), 255))
    # one emitting triangle: the light BVH's phi (the image's mean vs the spectrum's maximum)
    # would otherwise move the two triangles' light-choice pmf by ulps
    a = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "w.png" "float scale" 3', single=True)
    b = scene(pa, tmp_path, 'AreaLightSource "diffuse" "rgb L" [1 1 1] "float scale" 3', single=True)
    fa, fb = oracle.render(a, threads=8), oracle.render(b, threads=8)
    assert fa[:3].sum() > 0
    # equal up to the bilerp's own rounding: its four weights sum to 1 within an ulp, so the
    # bilerped white is 1 +- 1 ulp where pbrt's would be too
    np.testing.assert_allclose(fa, fb, rtol=3e-7, atol=0)


def test_image_emitter_power(pa, oracle, tmp_path):
    """power: k_e = mean luminance x (twoSided ? 2 : 1) x area x pi, so a uniform image of any
    level emits what "rgb L" [1 1 1] with the same power does (white: luminance 1)"""
    png(tmp_path / "w.png", np.full((8, 8, 3), 255))
    png(tmp_path / "h.png", np.full((8, 8, 3), 128))
    films = [oracle.render(scene(pa, tmp_path, f'AreaLightSource "diffuse" {src} "float power" 20', single=True),
                           threads=8) for src in ('"string filename" "w.png"', '"string filename" "h.png"', '"rgb L" [1 1 1]')]
    assert films[0][:3].sum() > 0
    # the luminance vector sums to 1 within a few ulp, and the bilerp rounds by an ulp
    np.testing.assert_allclose(films[0], films[2], rtol=1e-5, atol=0)
    np.testing.assert_allclose(films[1], films[2], rtol=1e-5, atol=0)


def test_image_emitter_seen_directly(pa, oracle, tmp_path):
    """Looking up at the emitter: its uv (0,0)-(1,1) spans the quad; image row 0 (top) is v = 1."""
    img = np.zeros((16, 16, 3))
    img[:8, :, 0] = 255   # top half red -> v > 1/2
    img[8:, :, 2] = 255   # bottom half blue -> v < 1/2
    png(tmp_path / "rb.png", img)
    sc = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "rb.png" "bool twosided" true',
               eye="0 0.5 0", look="0 2 0.001", depth=0, res=32, spp=4)
    im = rgb(oracle, sc, oracle.render(sc, threads=8))
    # camera up vector +y, looking at +y: image rows follow render z; compare the two halves
    top, bottom = im[:14].mean(axis=(0, 1)), im[18:].mean(axis=(0, 1))
    halves = [top, bottom]
    red = [h[0] > 4 * h[2] for h in halves]
    blue = [h[2] > 4 * h[0] for h in halves]
    assert sorted(red) == [False, True] and sorted(blue) == [False, True] and red != blue


def test_image_emitter_tints_the_floor(pa, oracle, tmp_path):
    img = np.zeros((8, 16, 3))
    img[:, :8, 0] = 255   # u < 1/2 red (render x < 0)
    img[:, 8:, 2] = 255   # u > 1/2 blue
    png(tmp_path / "lr.png", img)
    sc = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "lr.png"', eye="0 6 -0.01", look="0 0 0",
               depth=1, res=48, spp=16)
    im = rgb(oracle, sc, oracle.render(sc, threads=8))
    # the floor left and right of the emitter's footprint, outside its shadow
    a, b = im[20:28, 2:10].mean(axis=(0, 1)), im[20:28, -10:-2].mean(axis=(0, 1))
    assert (a[0] > a[2]) != (b[0] > b[2]), (a, b)


@pytest.mark.gpu
def test_image_emitter_gpu_matches_oracle(pa, oracle, tmp_path):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    y, x = np.mgrid[0:24, 0:32]
    png(tmp_path / "e.png", np.stack([128 + 120 * np.sin(x / 4.0), 128 + 100 * np.cos(y / 5.0), np.full_like(x, 60)], -1))
    extra = ('Material "conductor" "float roughness" 0.2\nShape "trianglemesh" "integer indices" [0 1 2] '
             '"point3 P" [-1 0 1 1 0 1 0 1.3 1.2]\n')
    sc = scene(pa, tmp_path, 'AreaLightSource "diffuse" "string filename" "e.png" "float scale" 2', depth=5, res=96,
               spp=16, extra=extra)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"image emitter parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
