"""Bump and normal mapping (surfscatter.cpp:109-127; NormalMap / BumpMap materials.h:86-140;
the shading frame and dndu / dndv of Triangle::InteractionFromIntersection shapes.h:961-1006):
the loader's "displacement" / "normalmap" on diffuse, dielectric and conductor materials, the
oracle's restatement against known answers, and GPU parity of films (k_texture evaluates the
perturbed shading normal and dpdu per record; the shade kernels, light sampling and the next
vertex's emission MIS use them)."""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 2.2 -4.5  0 0.3 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.2 0.2 0.25]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [5 5 5]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.6 3 -0.6 0.6 3 -0.6 0.6 3 0.6 -0.6 3 0.6]
AttributeEnd
"""

BODY = """Texture "bumps" "float" "imagemap" "string filename" "bumps.png" "string encoding" "linear" "float scale" 0.05
Material "diffuse" "rgb reflectance" [0.6 0.55 0.5] "texture displacement" "bumps"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3]
    "point2 uv" [0 0 3 0 3 3 0 3]
Material "conductor" "float roughness" 0.05 "string normalmap" "normals.png"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1.6 0 1 -0.2 0 1 -0.2 1.4 1.2 -1.6 1.4 1.2]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "diffuse" "rgb reflectance" [0.3 0.5 0.7] "float displacement" 0.02
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [0.2 0 0.8 1.6 0 0.6 1.6 1.4 0.9 0.2 1.4 1.1]
    "normal N" [0.2 0.1 -1 -0.2 0.1 -1 -0.1 -0.2 -1 0.1 0.2 -1] "point2 uv" [0 0 1 0 1 1 0 1]
Material "dielectric" "float roughness" 0.1 "texture displacement" "bumps"
Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [-0.5 0.05 -1 0.5 0.05 -1 0 0.9 -0.8]
    "point2 uv" [0 0 1 0 0.5 1]
"""


def write_maps(d, n=64):
    from PIL import Image
    y, x = np.mgrid[0:n, 0:n]
    h = 0.5 + 0.5 * np.sin(x / n * 6 * np.pi) * np.cos(y / n * 4 * np.pi)
    Image.fromarray((h * 255).astype(np.uint8), mode="L").save(d / "bumps.png")
    # a tangent-space normal map: tilted normals in a ring pattern
    r = np.hypot(x - n / 2, y - n / 2) / (n / 2)
    nx, ny = 0.4 * np.sin(r * 5 * np.pi), 0.3 * np.cos(x / n * 4 * np.pi)
    nz = np.sqrt(np.clip(1 - nx * nx - ny * ny, 0, 1))
    rgb = np.stack([nx, ny, nz], -1) * 0.5 + 0.5
    Image.fromarray((rgb * 255).astype(np.uint8), mode="RGB").save(d / "normals.png")


def _scene(pa, tmp_path, body=BODY, **kw):
    write_maps(tmp_path)
    return pa.Scene.from_string(HEAD + body, tmp_path, **kw)


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_bump_loader(pa, tmp_path):
    sc = _scene(pa, tmp_path)
    f = sc.flat()
    mb = np.ctypeslib.as_array(f.material_bump, shape=(f.n_materials * 2,)).reshape(-1, 2)
    # light's default material, diffuse bump, conductor normal map, constant displacement, dielectric
    bumped = [(d >= 0, m >= 0) for d, m in mb]
    assert bumped.count((True, False)) == 3 and bumped.count((False, True)) == 1


@pytest.mark.parametrize("body, msg", [
    ('Material "diffuse" "float displacement" 0.1\nShape "sphere"\n', "bump and normal mapping on spheres"),
    ('Material "diffuse" "string normalmap" "bumps.png"\nShape "trianglemesh" "integer indices" [0 1 2] '
     '"point3 P" [0 0 0 1 0 0 0 1 0]\n', "must contain R, G, and B"),
])
def test_bump_loader_errors(pa, tmp_path, body, msg):
    write_maps(tmp_path)
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(HEAD + body, tmp_path)


def test_zero_displacement_known_answer(pa, oracle, tmp_path):
    """A zero (or constant, on flat triangles without vertex normals) displacement leaves the
    shading frame's direction unchanged: BumpMap gives dpdu, dpdv = the shading ones, so the
    image equals the unbumped one up to the last-bit rounding of the renormalised normal."""
    plain = ('Material "diffuse" "rgb reflectance" [0.6 0.55 0.5]\nShape "trianglemesh" "integer indices" '
             '[0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3] "point2 uv" [0 0 3 0 3 3 0 3]\n')
    kw = dict(xresolution=48, yresolution=32, spp=16)
    a = _rgb(oracle, sc0 := pa.Scene.from_string(HEAD + plain, SCENES, **kw), oracle.render(sc0, threads=8))
    for disp in ("0", "0.37"):
        text = HEAD + plain.replace('[0.6 0.55 0.5]', f'[0.6 0.55 0.5] "float displacement" {disp}')
        sc = pa.Scene.from_string(text, SCENES, **kw)
        b = _rgb(oracle, sc, oracle.render(sc, threads=8))
        close = (np.abs(a - b) <= np.maximum(1e-3 * np.abs(a), 1e-4)).all(axis=-1).mean()
        assert close >= 0.99, (disp, close)
        assert abs(b.mean() / a.mean() - 1) < 1e-3


def test_bumps_change_the_image(pa, oracle, tmp_path):
    sc = _scene(pa, tmp_path, xresolution=48, yresolution=32, spp=8)
    flat = _scene(pa, tmp_path, body=BODY.replace(' "texture displacement" "bumps"', '')
                  .replace(' "string normalmap" "normals.png"', ''), xresolution=48, yresolution=32, spp=8)
    a = _rgb(oracle, sc, oracle.render(sc, threads=8))
    b = _rgb(oracle, flat, oracle.render(flat, threads=8))
    assert np.isfinite(a).all()
    assert np.abs(a - b).mean() > 1e-3


@pytest.mark.gpu
def test_bump_scene_matches_oracle_gpu(pa, oracle, tmp_path):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = _scene(pa, tmp_path)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"bump parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
