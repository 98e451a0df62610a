"""GPU parity of the layered materials and of dispersion (spectral dielectric eta) (k_vlayered in pbrt-v4_amd/csrc/kernels/volpath.hip over
core.h's LayeredBxDF) against the oracle's independent restatement (oracle/oracle.cpp
LayeredBxDF).  The walks' RNGs hash direction bits, so, as for media, both sides evaluate
transcendentals, glibc's bit for bit as the oracle's libm mode computes them (core/detmath.h).  Known answers of test_layered.py are
repeated on the GPU image.  Tolerances as test_gpu_media.py."""
import numpy as np
import pytest

from conftest import SCENES
from test_gpu_media import check, gpu_rgb, oracle_rgb
from test_layered import layered_scene, showcase_scene

pytestmark = pytest.mark.gpu


def test_showcase_matches_oracle(pa, oracle):
    sc = pa.Scene.from_string(showcase_scene(res=48, spp=8), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"layered showcase: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.parametrize("material", [
    'Material "coateddiffuse" "rgb reflectance" [0.6 0.4 0.2] "float roughness" 0.3 "integer nsamples" 2',
    'Material "coatedconductor" "float interface.roughness" 0.2 "float conductor.roughness" 0.1 '
    '"rgb albedo" [0.5 0.5 0.5] "float thickness" 0.1',
])
def test_quad_matches_oracle(pa, oracle, material):
    from test_layered import LIGHT
    sc = pa.Scene.from_string(layered_scene(material, res=32, spp=16, sky="0.4 0.5 0.6", extra=LIGHT), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    check(a, oracle_rgb(oracle, sc))


def test_known_answers_gpu(pa, oracle):
    black = pa.Scene.from_string(layered_scene('Material "coateddiffuse" "float reflectance" 0', spp=64), SCENES)
    img, _ = gpu_rgb(pa, oracle, black)
    assert img.mean() == pytest.approx(0.0401, rel=0.06), img.mean()
    white = pa.Scene.from_string(layered_scene(
        'Material "coateddiffuse" "float reflectance" 1 "float thickness" 0.0001 "integer maxdepth" 100', spp=32),
        SCENES)
    img, _ = gpu_rgb(pa, oracle, white)
    assert img.mean() == pytest.approx(1.0, rel=0.01), img.mean()


@pytest.mark.parametrize("eta", ['"spectrum eta" "glass-BK7"', '"spectrum eta" [300 1.7 800 1.4] "float roughness" 0.2',
                                 'coated'])
def test_dispersion_matches_oracle(pa, oracle, eta):
    from test_dispersion import glass_scene
    text = glass_scene(eta, res=32, spp=16) if eta != 'coated' else glass_scene(res=32, spp=16).replace(
        'Material "dielectric" "spectrum eta" "glass-BK7"',
        'Material "coateddiffuse" "spectrum eta" "glass-F11" "rgb reflectance" [0.3 0.5 0.7] "float roughness" 0.1')
    sc = pa.Scene.from_string(text, SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"dispersion {eta}: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


def test_dispersion_with_media_refused(pa):
    from test_dispersion import dispersive_medium_scene
    sc = pa.Scene.from_string(dispersive_medium_scene(), SCENES)
    with pytest.raises(RuntimeError, match="dispersion"):
        pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)


@pytest.mark.parametrize("eta", ['"float eta" 1.6', '"spectrum eta" "glass-BAF10"'])
def test_thin_dielectric_matches_oracle(pa, oracle, eta):
    from test_dispersion import glass_scene
    sc = pa.Scene.from_string(glass_scene(eta, res=32, spp=16).replace('"dielectric"', '"thindielectric"'), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"thin dielectric {eta}: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.parametrize("mat", ['"diffusetransmission" "rgb reflectance" [0.6 0.3 0.2] "rgb transmittance" [0.2 0.4 0.5]',
                                 '"diffusetransmission" "float scale" 2'])
def test_diffuse_transmission_matches_oracle(pa, oracle, mat):
    from test_dispersion import glass_scene
    sc = pa.Scene.from_string(glass_scene(res=32, spp=16).replace('"dielectric" "spectrum eta" "glass-BK7"', mat), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"diffuse transmission {mat}: {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")
