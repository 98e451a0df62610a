"""C3 (dielectric + conductor BxDFs on a ~30k-triangle mesh) on the CPU side:
the scene generator, the loader's material parameters (materials.cpp:51-74, :217-251,
paramdict.cpp:384-450, 817-875) and known answers of the oracle.  GPU parity for C3 lives
in test_gpu_parity.py."""
import sys

import numpy as np
import pytest

from conftest import SCENES

sys.path.insert(0, str(SCENES))
import gen_c3  # noqa: E402


def _flat_materials(sc):
    f = sc.flat()
    n = sc.info.n_materials
    types = [f.material_type[i] for i in range(n)]
    params = np.array([f.material_params[i] for i in range(4 * n)], np.float32).reshape(n, 4)
    spectra = [(f.material_spectra[2 * i], f.material_spectra[2 * i + 1]) for i in range(n)]
    return f, types, params, spectra


def test_c3_scene_shape(pa):
    sc = pa.Scene.from_string(gen_c3.scene_text(64, 36, 4), SCENES)
    assert sc.info.n_triangles == 30284
    f, types, params, spectra = _flat_materials(sc)
    assert sorted(types) == [0, 1, 2]
    glass, metal = types.index(1), types.index(2)
    assert params[glass][2] == np.float32(1.5) and params[glass][0] == 0  # smooth: alpha 0
    # roughness 0.1 remapped: RoughnessToAlpha = sqrt (util/scattering.h:192)
    assert params[metal][0] == np.float32(np.sqrt(np.float32(0.1)))
    e, k = spectra[metal]
    assert f.n_pl_spectra == 2 and e >= 0 and k >= 0
    assert [f.pl_lambda[i] for i in range(4)] == [300, 800, 300, 800]  # inline: not extended


def test_conductor_defaults_and_named_spectra(pa):
    base = 'WorldBegin\nLightSource "infinite"\n{}\nShape "trianglemesh" "point3 P" [0 0 0 1 0 0 0 1 0]\n'
    sc = pa.Scene.from_string(base.format('Material "conductor"'), SCENES)
    f, types, params, spectra = _flat_materials(sc)
    assert types == [2] and params[0][0] == 0 and params[0][1] == 0
    # default metal-Cu-eta / -k (materials.cpp:230-236), FromInterleaved-extended to 394 / 706
    lam = [f.pl_lambda[i] for i in range(f.pl_offsets[0], f.pl_offsets[1])]
    assert lam[0] < 395 and lam[-1] > 705
    cu = pa.named_spectrum("metal-Cu-eta", [500.0])
    assert 0.5 < cu[0] < 1.5
    sc = pa.Scene.from_string(base.format(
        'Material "conductor" "spectrum eta" "metal-Au-eta" "spectrum k" "metal-Au-k" '
        '"float uroughness" 0.04 "float vroughness" 0.09 "bool remaproughness" false'), SCENES)
    f, types, params, spectra = _flat_materials(sc)
    assert params[0][0] == np.float32(0.04) and params[0][1] == np.float32(0.09)
    sc = pa.Scene.from_string(base.format('Material "conductor" "rgb reflectance" [0.9 0.6 0.3]'), SCENES)
    f, types, params, spectra = _flat_materials(sc)
    assert spectra[0] == (-1, -1)


@pytest.mark.parametrize("mat,msg", [
    ('Material "conductor" "rgb reflectance" [0.9 0.6 0.3] "spectrum eta" "metal-Au-eta"', "can't be provided"),
    ('Material "conductor" "spectrum eta" "metal-Xx-eta"', "unknown named spectrum"),
    ('Material "conductor" "spectrum eta" [400 1 500]', "odd number"),
    ('Material "dielectric" "texture roughness" "foo"', "Couldn't find float texture"),
])
def test_material_errors_are_loud(pa, mat, msg):
    text = 'WorldBegin\nLightSource "infinite"\n' + mat + '\nShape "trianglemesh" "point3 P" [0 0 0 1 0 0 0 1 0]\n'
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(text, SCENES)


def furnace_glass_text(eta, roughness, spp=8, res=32, sphere=True):
    """An index-matched (eta = 1) glass sphere under a uniform sky is invisible: every pixel
    equals the sky seen through the same wavelengths (DielectricBxDF with eta 1 transmits
    straight through with f / pdf = 1/|cos|).  sphere=False: only a triangle behind the camera."""
    P, F = gen_c3.icosphere(2)
    if not sphere:
        P, F = np.array([[0, 0, -10], [1, 0, -10], [0, 1, -10]], float), np.array([[0, 1, 2]])
    return f"""LookAt 0 0 -4  0 0 0  0 1 0
Camera "perspective" "float fov" [ 30 ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "zsobol" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ 8 ]
WorldBegin
LightSource "infinite" "rgb L" [ 1 1 1 ]
Material "dielectric" "float eta" [ {eta} ] "float roughness" [ {roughness} ]
Shape "trianglemesh" "integer indices" [ {" ".join(map(str, F.ravel()))} ] "point3 P" [ {gen_c3.fmt(P)} ]
"""


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


@pytest.mark.parametrize("roughness", [0.0, 0.2])
def test_oracle_index_matched_glass_is_invisible(pa, oracle, roughness):
    sc = pa.Scene.from_string(furnace_glass_text(1.0, roughness), SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    empty = pa.Scene.from_string(furnace_glass_text(1.0, roughness, sphere=False), SCENES)
    sky = _rgb(oracle, empty, oracle.render(empty, threads=8))
    # eta == 1 takes the specular branch whatever the roughness (bxdfs.cpp:80): R ~ 0, T ~ 1
    # up to the rounding of FrDielectric / Refract at eta 1
    np.testing.assert_allclose(img, sky, rtol=1e-5)


def test_oracle_c3_plausible(pa, oracle):
    sc = pa.Scene.from_string(gen_c3.scene_text(64, 36, 8), SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    assert np.isfinite(img).all() and img.min() >= 0
    assert 0.05 < img.mean() < 1.0


def test_c4_generator_small_variant_loads(pa, oracle, tmp_path):
    """scenes/gen_c4.py (PLY copies, diffuse + named-metal conductors) at a small size."""
    import gen_c4
    path, n = gen_c4.generate(tmp_path, copies=6, level=2, xres=48, yres=27, spp=4)
    sc = pa.load_scene(path)
    assert sc.info.n_triangles == n == 6 * 320 + 4
    f, types, params, spectra = _flat_materials(sc)
    assert types.count(2) >= 3 and types.count(0) >= 4
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    assert np.isfinite(img).all() and img.mean() > 0.01
