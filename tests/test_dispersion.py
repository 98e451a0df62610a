"""Dispersion: a dielectric with a spectral eta ("spectrum eta" named glass or inline pairs).
DielectricMaterial::GetBxDF (materials.cpp:25-49) takes eta(lambda_0) and, for a non-constant
eta, calls SampledWavelengths::TerminateSecondary; the wavefront writes the terminated
wavelengths back to the pixel state (surfscatter.cpp:139-141) and the film divides the whole
path's L by them (film.cpp:28, film.h:95-100).  The GPU keeps a lambda_0-only sensor-RGB sum
next to the full one per slot and the film takes it for terminated paths.  Scenes with
dispersion render through the volumetric kernels.  GPU parity: test_gpu_layered.py."""
import numpy as np
import pytest

from conftest import SCENES
from test_layered import LIGHT, layered_scene
from test_media import box


def glass_scene(eta='"spectrum eta" "glass-BK7"', res=24, spp=16, sky="0.9 0.5 0.2"):
    extra = (f'{LIGHT}\nAttributeBegin\n  Material "diffuse" "rgb reflectance" [0.2 0.6 0.3]\n'
             f'  {box(-2, 2, -2, 2, 1.5, 1.6)}\nAttributeEnd')
    return layered_scene(f'Material "dielectric" {eta}', res=res, spp=spp, maxdepth=6, sky=sky, extra=extra)


def _render(pa, oracle, text):
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    film = oracle.render(sc, threads=8)
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_loader_spectral_eta(pa):
    sc = pa.Scene.from_string(glass_scene(), SCENES)
    f = sc.flat()
    mats = [i for i in range(sc.info.n_materials) if f.material_type[i] == 1]
    assert len(mats) == 1 and f.material_spectra[2 * mats[0]] >= 0
    sc = pa.Scene.from_string(glass_scene('"spectrum eta" [300 1.6 800 1.4]'), SCENES)
    f = sc.flat()
    es = f.material_spectra[2 * [i for i in range(sc.info.n_materials) if f.material_type[i] == 1][0]]
    assert [f.pl_value[f.pl_offsets[es] + k] for k in range(2)] == [np.float32(1.6), np.float32(1.4)]


def dispersive_medium_scene():
    from test_media import medium_scene
    text = medium_scene('MakeNamedMedium "m" "string type" "homogeneous"',
                        extra='AttributeBegin\n Material "dielectric" "spectrum eta" "glass-BK7"\n'
                              f' {box(-0.2, 0.2, -0.2, 0.2, -2, -1.5)}\nAttributeEnd')
    return text


def test_dispersion_with_media_loads(pa):
    """The loader accepts it; the renderer refuses it at context creation (GPU test)."""
    sc = pa.Scene.from_string(dispersive_medium_scene(), SCENES)
    assert any(sc.flat().material_spectra[2 * i] >= 0 for i in range(sc.info.n_materials))


def test_termination_is_unbiased(pa, oracle):
    """A constant-valued spectral eta follows the same paths as "float eta" 1.5 but terminates
    the secondary wavelengths: the image means agree within the noise, the images do not."""
    a = _render(pa, oracle, glass_scene('"spectrum eta" [300 1.5 800 1.5]', spp=64))
    b = _render(pa, oracle, glass_scene('"float eta" 1.5', spp=64))
    assert not np.array_equal(a, b)
    np.testing.assert_allclose(a.mean(axis=(0, 1)), b.mean(axis=(0, 1)), rtol=0.03)


def test_bk7_renders(pa, oracle):
    img = _render(pa, oracle, glass_scene())
    assert np.isfinite(img).all() and img.mean() > 0.05
