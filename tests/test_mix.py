"""MixMaterial (materials.h:272-330, materials.cpp:105-125): loader, oracle and GPU parity.

pbrt picks one of the two materials per hit in the closest-hit stage
(wavefront/intersect.h:90-97): amount <= 0 -> materials[0], amount >= 1 -> materials[1],
otherwise HashFloat(p, wo, material0, material1) < amount picks materials[1]. pbrt hashes the
two material *pointers*; this framework and its oracle hash the material indices instead, so
for an interior amount the per-hit choice is comparable between them but not with pbrt itself
(parity unpinned against pbrt for interior amounts; amounts 0 and 1 and the expected mixture
are pinned by the known answers below).
"""
import numpy as np
import pytest

from conftest import SCENES

BASE = """LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 22
Film "rgb" "integer xresolution" 32 "integer yresolution" 32
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 1
WorldBegin
LightSource "infinite" "rgb L" [1 1 1]
MakeNamedMaterial "white" "string type" "diffuse" "rgb reflectance" [1 1 1]
MakeNamedMaterial "black" "string type" "diffuse" "rgb reflectance" [0 0 0]
MakeNamedMaterial "red" "string type" "diffuse" "rgb reflectance" [0.8 0.1 0.1]
MakeNamedMaterial "gold" "string type" "conductor" "spectrum eta" "metal-Au-eta" "spectrum k" "metal-Au-k" "float roughness" 0.2
"""
QUAD = ('Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0 1 -1 0 1 1 0 -1 1 0] '
        '"point2 uv" [0 0 1 0 1 1 0 1]\n')


def _mix(amount, a="white", b="black"):
    amt = "" if amount is None else f'"float amount" {amount} '
    return f'Material "mix" "string materials" ["{a}" "{b}"] {amt}\n'


def _scene(pa, body):
    return pa.Scene.from_string(BASE + body + QUAD, SCENES)


@pytest.mark.parametrize("body, msg", [
    ('Material "mix" "string materials" ["white"]\n', "two values"),
    ('Material "mix" "string materials" ["white" "nope"]\n', "named material not found"),
    ('Texture "c" "float" "checkerboard"\nMaterial "mix" "string materials" ["white" "black"] '
     '"texture amount" "c"\n', "basic textures"),
    ('Material "mix" "string materials" ["white" "black"] "texture amount" "nope"\n',
     "Couldn't find float texture"),
])
def test_mix_loader_errors(pa, body, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        _scene(pa, body)


def test_mix_flat_records_materials_and_amount(pa):
    sc = _scene(pa, 'MakeNamedMaterial "m" "string type" "mix" "string materials" ["red" "gold"] '
                    '"float amount" 0.25\nNamedMaterial "m"\n')
    f = sc.flat()
    types = [f.material_type[i] for i in range(f.n_materials)]
    mix = np.ctypeslib.as_array(f.material_mix, shape=(f.n_materials * 4,)).reshape(-1, 4)
    m = types.index(8)
    assert [types[mix[m][0]], types[mix[m][1]]] == [0, 2]  # diffuse, conductor
    assert mix[m][2] >= 0  # the compiled constant amount program


@pytest.mark.parametrize("amount, plain", [(0, "white"), (-1, "white"), (1, "black"), (3, "black")])
def test_mix_extreme_amounts_render_like_the_chosen_material(pa, oracle, amount, plain):
    """amount <= 0 is materials[0] and amount >= 1 is materials[1] without hashing
    (MixMaterial::ChooseMaterial, materials.h:285-294): bit-identical oracle films."""
    a = _scene(pa, _mix(amount))
    b = _scene(pa, f'NamedMaterial "{plain}"\n')
    assert np.array_equal(oracle.render(a, threads=4), oracle.render(b, threads=4))


def test_mix_interior_amount_is_a_stochastic_blend(pa, oracle):
    """White/black diffuse mix under a uniform unit sky, one bounce: a pixel reflects about the
    share of its hits that chose white, i.e. 1 - amount on average (a furnace known answer)."""
    for amount in (0.25, 0.5, 0.8):
        sc = _scene(pa, _mix(amount))
        f = sc.flat()
        img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
        inner = img[6:26, 6:26].mean()
        assert inner == pytest.approx(1 - amount, abs=0.03), amount


def test_mix_default_amount_is_one_half(pa, oracle):
    a = _scene(pa, _mix(None))
    b = _scene(pa, _mix(0.5))
    assert np.array_equal(oracle.render(a, threads=4), oracle.render(b, threads=4))


MIXED = """LookAt 0 0.6 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 30
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.4 0.45 0.5]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [6 6 6]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.5 2 -0.5 0.5 2 -0.5 0.5 2 0.5 -0.5 2 0.5]
AttributeEnd
MakeNamedMaterial "red" "string type" "diffuse" "rgb reflectance" [0.8 0.1 0.1]
MakeNamedMaterial "gold" "string type" "conductor" "spectrum eta" "metal-Au-eta" "spectrum k" "metal-Au-k" "float roughness" 0.2
MakeNamedMaterial "glass" "string type" "dielectric" "float eta" 1.5 "float roughness" 0.1
MakeNamedMaterial "rg" "string type" "mix" "string materials" ["red" "gold"] "float amount" 0.35
Texture "marble" "float" "imagemap" "string filename" "textures/bumps_grey16.png"
MakeNamedMaterial "tex" "string type" "mix" "string materials" ["rg" "glass"] "texture amount" "marble"
NamedMaterial "tex"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 -1 -3 3 -1 -3 3 -1 3 -3 -1 3] "point2 uv" [0 0 2 0 2 2 0 2]
NamedMaterial "rg"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 1 1 -1 1 1 1 1 -1 1 1] "point2 uv" [0 0 1 0 1 1 0 1]
"""


def test_mix_scene_loads_nested_mix(pa):
    sc = pa.Scene.from_string(MIXED, SCENES)
    f = sc.flat()
    assert sum(f.material_type[i] == 8 for i in range(f.n_materials)) == 2


@pytest.mark.gpu
def test_mix_first_hit_choice_matches_oracle_gpu(pa, oracle):
    """maxdepth 1: only camera-ray hits resolve a mix; camera rays are bit-identical between the
    device and the oracle, so the per-hit hash picks the same material on both sides."""
    from test_gpu_parity import check_parity, gpu_film, oracle_film, to_rgb
    text = MIXED.replace('"integer maxdepth" 5', '"integer maxdepth" 1').replace(
        "WorldBegin", 'PixelFilter "box"\nWorldBegin')
    sc = pa.Scene.from_string(text, SCENES)
    film, integ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle_film(oracle, sc, integ)))
    print(f"mix first-hit parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_mix_scene_matches_oracle_gpu(pa, oracle):
    """Nested mix (constant amount inside an image-textured amount) across diffuse, conductor
    and dielectric components, 5 bounces.  Each bounce's mix choice hashes the hit point and
    wo, so a bounce direction one ulp off the oracle's would re-roll it; the device's portable
    transcendentals (core/detmath.h) are the oracle's, so the standard per-pixel bar applies."""
    from test_gpu_parity import check_parity, gpu_film, oracle_film, to_rgb
    text = MIXED.replace('"integer pixelsamples" 16', '"integer pixelsamples" 64')
    sc = pa.Scene.from_string(text, SCENES)
    film, integ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle_film(oracle, sc, integ)))
    print(f"mix 5-bounce: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_mix_extreme_amount_film_bit_identical_gpu(pa):
    """The mix-resolving closest-hit kernel with amount 0 gives the plain material's film bits."""
    from test_gpu_parity import gpu_film
    fa, _ = gpu_film(pa, _scene(pa, _mix(0, "red", "gold")))
    fb, _ = gpu_film(pa, _scene(pa, 'NamedMaterial "red"\n'))
    assert np.array_equal(fa, fb)
