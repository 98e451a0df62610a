"""Bump and normal mapping on the materials the volumetric kernels shade (round 6): coated
diffuse / coated conductor, diffuse transmission, measured, retroreflective (k_vlayered) and thin
dielectric (k_vsurface).  pbrt reads "displacement" / "normalmap" in every material's Create but
hair's, interface's and mix's (materials.cpp:51-664) and applies NormalMap / BumpMap before
GetBxDF (surfscatter.cpp:109-127); k_vtexture leaves the perturbed shading normal and dpdu per
record, which k_vlayered and k_vsurface now shade with.  The oracle applies the same perturbation
to every material (oracle.cpp MakeBSDF).  CPU: the loader accepts the parameters and the bumps
change the oracle's image; GPU: film parity with the oracle per material."""
import numpy as np
import pytest

from measured_bsdf import make_bsdf
from test_bump import HEAD, write_maps

GROUND = ('Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3] '
          '"point2 uv" [0 0 3 0 3 3 0 3]\n')
PANEL = ('Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1.2 0 0.6 1.2 0 0.6 1.2 1.6 0.9 '
         '-1.2 1.6 0.9] "point2 uv" [0 0 1 0 1 1 0 1]\n')
BUMPS = 'Texture "bumps" "float" "imagemap" "string filename" "bumps.png" "string encoding" "linear" "float scale" 0.05\n'

MATERIALS = {
    "coateddiffuse": '"coateddiffuse" "rgb reflectance" [0.6 0.4 0.3] "float roughness" 0.05',
    "coatedconductor": '"coatedconductor" "float interface.roughness" 0.02 "float conductor.roughness" 0.1',
    "diffusetransmission": '"diffusetransmission" "rgb reflectance" [0.5 0.5 0.45] "rgb transmittance" [0.3 0.3 0.3]',
    "measured": '"measured" "string filename" "m.bsdf"',
    "retroreflective": '"retroreflective" "float roughness" 0.1',
    "thindielectric": '"thindielectric" "float eta" 1.5',
}


def body(kind, bump=True, normal=True):
    m = MATERIALS[kind]
    d = ' "texture displacement" "bumps"' if bump else ""
    n = ' "string normalmap" "normals.png"' if normal else ""
    return (BUMPS + f'Material {m}{d}\n' + GROUND + f'Material {m}{n}\n' + PANEL)


def scene(pa, tmp_path, kind, res=(64, 48), spp=8, **kw):
    write_maps(tmp_path)
    make_bsdf(tmp_path / "m.bsdf")
    return pa.Scene.from_string(HEAD + body(kind, **kw), tmp_path, xresolution=res[0], yresolution=res[1], spp=spp)


def rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


@pytest.mark.parametrize("kind", sorted(MATERIALS))
def test_loader_accepts_bump_maps(pa, tmp_path, kind):
    f = scene(pa, tmp_path, kind).flat()
    mb = np.ctypeslib.as_array(f.material_bump, shape=(f.n_materials * 2,)).reshape(-1, 2)
    bumped = [(d >= 0, m >= 0) for d, m in mb]
    assert bumped.count((True, False)) == 1 and bumped.count((False, True)) == 1


def test_hair_takes_no_bump_map(pa, tmp_path):
    """HairMaterial::Create reads no displacement (materials.cpp:135-184): an unused parameter."""
    write_maps(tmp_path)
    with pytest.raises(pa.PbrtError, match="displacement"):
        pa.Scene.from_string(HEAD + BUMPS + 'Material "hair" "texture displacement" "bumps"\n' + GROUND, tmp_path)


@pytest.mark.parametrize("kind", ["coateddiffuse", "diffusetransmission", "retroreflective"])
def test_bumps_change_the_image(pa, oracle, tmp_path, kind):
    a = scene(pa, tmp_path, kind, res=(40, 30), spp=8)
    b = scene(pa, tmp_path, kind, res=(40, 30), spp=8, bump=False, normal=False)
    ia, ib = rgb(oracle, a, oracle.render(a, threads=8)), rgb(oracle, b, oracle.render(b, threads=8))
    assert np.isfinite(ia).all()
    assert np.abs(ia - ib).mean() > 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("kind", sorted(MATERIALS))
def test_bumped_volumetric_materials_match_oracle_gpu(pa, oracle, tmp_path, kind):
    from test_gpu_media import check, gpu_rgb, oracle_rgb

    sc = scene(pa, tmp_path, kind)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"{kind} bump parity: {frac * 100:.3f}% pixels, mean rel {mr:.2e}")
