"""Textures and bump mapping on the volumetric path (a scene with media): the volumetric
surface stage evaluates the same texEval calls and bump / normal mapping as the surface path
(EvaluateMaterialAndBSDF, surfscatter.cpp:57-137).  k_vtexture evaluates them over the
iteration's surface queue; k_vsurface<..., Tex> reads the results.  The oracle's volumetric
integrator shares MakeBSDF and the mix resolution with its surface integrator, so the GPU film
is checked against it (libm oracle, as the media kernels).  Mix materials resolve at the
closest hit (k_vclosest<TM, true>) there too."""
import numpy as np
import pytest

from conftest import SCENES
from test_bump import BODY, HEAD, write_maps
from test_media import box

TEX = """Texture "checks" "spectrum" "checkerboard" "float uscale" 4 "float vscale" 4
    "rgb tex1" [0.8 0.25 0.1] "rgb tex2" [0.1 0.3 0.8]
Texture "rough" "float" "checkerboard" "float uscale" 3 "float vscale" 3 "float tex1" 0.05 "float tex2" 0.4
Texture "img" "spectrum" "imagemap" "string filename" "normals.png"
MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.05 0.08 0.1] "rgb sigma_s" [0.4 0.35 0.3]
    "float g" 0.3
AttributeBegin
  MediumInterface "fog" ""
  Material "interface"
  {box}
AttributeEnd
Material "diffuse" "texture reflectance" "checks"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 2 3 0 2 3 3 2 -3 3 2]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "conductor" "texture roughness" "rough" "spectrum eta" "metal-Cu-eta" "spectrum k" "metal-Cu-k"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [1.8 0 -1 2.8 0 0 2.8 1.5 0 1.8 1.5 -1]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "conductor" "texture reflectance" "img" "float roughness" 0.2
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-2.8 0 0 -1.8 0 -1 -1.8 1.5 -1 -2.8 1.5 0]
    "point2 uv" [0 0 1 0 1 1 0 1]
"""


def vol_scene(pa, tmp_path, res=None):
    write_maps(tmp_path)
    text = HEAD + BODY + TEX.replace("{box}", box(-1.2, 1.2, 0.02, 1.6, -1.5, 0.6))
    if res:
        text = text.replace('"integer xresolution" 96 "integer yresolution" 64',
                            f'"integer xresolution" {res[0]} "integer yresolution" {res[1]}')
    return pa.Scene.from_string(text, tmp_path)


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_textured_media_scene_renders_on_the_oracle(pa, oracle, tmp_path):
    """The loader takes textures together with media, and the oracle's volumetric integrator
    evaluates them (the checkerboard wall differs from a constant one)."""
    sc = vol_scene(pa, tmp_path, res=(32, 24))
    assert sc.flat().n_media == 1
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    text = (HEAD + BODY + TEX.replace("{box}", box(-1.2, 1.2, 0.02, 1.6, -1.5, 0.6))).replace(
        '"texture reflectance" "checks"', '"rgb reflectance" [0.45 0.28 0.45]').replace(
        '"integer xresolution" 96 "integer yresolution" 64', '"integer xresolution" 32 "integer yresolution" 24')
    flat = pa.Scene.from_string(text, tmp_path)
    ref = _rgb(oracle, flat, oracle.render(flat, threads=8))
    assert np.isfinite(img).all() and np.abs(img - ref).mean() > 1e-3


MIX = """MakeNamedMaterial "a" "string type" "diffuse" "rgb reflectance" [0.7 0.3 0.2]
MakeNamedMaterial "b" "string type" "conductor" "float roughness" 0.15
Texture "amt" "float" "imagemap" "string filename" "normals.png"
Material "mix" "string materials" ["a" "b"] "texture amount" "amt"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 0.01 -2.5 1 0.01 -2.5 1 0.01 -1.6 -1 0.01 -1.6]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "mix" "string materials" ["a" "b"] "float amount" 0.4
Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [-0.4 0.2 0.9 0.4 0.2 0.9 0 1.0 1.0]
"""


@pytest.mark.gpu
def test_mix_with_media_matches_oracle_gpu(pa, oracle, tmp_path):
    """Mix materials on the volumetric path: MixMaterial::ChooseMaterial at the closest hit
    (k_vclosest<TM, true>), the chosen material shaded by k_vsurface / k_vlayered."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    write_maps(tmp_path)
    text = HEAD + TEX.replace("{box}", box(-1.2, 1.2, 0.02, 1.6, -1.5, 0.6)) + MIX
    sc = pa.Scene.from_string(text, tmp_path)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mean_rel = check(gpu, oracle_rgb(oracle, sc))
    print(f"volumetric mix parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_textured_media_scene_matches_oracle_gpu(pa, oracle, tmp_path):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = vol_scene(pa, tmp_path)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mean_rel = check(gpu, oracle_rgb(oracle, sc))
    print(f"volumetric textures parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
