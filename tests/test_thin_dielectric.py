"""Material "thindielectric" (ThinDielectricMaterial, materials.cpp:83-97; ThinDielectricBxDF,
bxdfs.h:342-404): specular reflection or straight-through transmission, the slab's
inter-reflections folded into R and T.  Rendered by the volumetric kernels.  Known answer: in a
white furnace a thin pane is invisible (R + T = 1 on every sample).  GPU parity:
test_gpu_layered.py."""
import numpy as np
import pytest

from conftest import SCENES
from test_dispersion import glass_scene
from test_layered import layered_scene


def _render(pa, oracle, text):
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    film = oracle.render(sc, threads=8)
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_loader(pa):
    sc = pa.Scene.from_string(layered_scene('Material "thindielectric"'), SCENES)
    f = sc.flat()
    assert f.material_type[0] == 6 and f.material_params[2] == np.float32(1.5)
    sc = pa.Scene.from_string(layered_scene('Material "thindielectric" "spectrum eta" "glass-F5"'), SCENES)
    assert sc.flat().material_spectra[0] >= 0
    with pytest.raises(RuntimeError, match="roughness"):
        pa.Scene.from_string(layered_scene('Material "thindielectric" "float roughness" 0.1'), SCENES)


def test_thin_pane_vanishes_in_furnace(pa, oracle):
    """Every sample's throughput is (R + T) = 1 to rounding, whichever lobe it takes, so the
    image equals the sky seen through a null ("interface") quad, pixel by pixel."""
    img = _render(pa, oracle, layered_scene('Material "thindielectric" "float eta" 1.7', spp=8, maxdepth=3))
    sky = _render(pa, oracle, layered_scene('Material "interface"', spp=8, maxdepth=3))
    np.testing.assert_allclose(img, sky, rtol=1e-5)
    assert img.mean() == pytest.approx(1.0, rel=0.01)


def test_thin_pane_renders(pa, oracle):
    img = _render(pa, oracle, glass_scene('"float eta" 1.5').replace('"dielectric"', '"thindielectric"'))
    assert np.isfinite(img).all() and img.mean() > 0.05


# ---- Material "diffusetransmission" (DiffuseTransmissionMaterial, materials.cpp:620-645;
# DiffuseTransmissionBxDF, bxdfs.h:218-296), shaded by k_vlayered

def test_diffuse_transmission_loader(pa):
    sc = pa.Scene.from_string(layered_scene('Material "diffusetransmission"'), SCENES)
    f = sc.flat()
    assert f.material_type[0] == 7 and f.material_coeffs[3] == np.float32(0.25)
    assert f.material_layer[7] == np.float32(0.25) and f.material_layer[8] == 1 and f.material_params[3] == 1
    sc = pa.Scene.from_string(layered_scene(
        'Material "diffusetransmission" "rgb reflectance" [0.2 0.3 0.4] "rgb transmittance" [0.5 0.4 0.3] '
        '"float scale" 1.5'), SCENES)
    f = sc.flat()
    assert f.material_constant[0] == 0 and f.material_layer[8] == 0 and f.material_params[3] == np.float32(1.5)


def test_diffuse_transmission_furnace(pa, oracle):
    """R + T = 1 (grey): each sample's throughput is pr + pt = 1, so the quad shows the sky."""
    mat = 'Material "diffusetransmission" "float reflectance" 0.3 "float transmittance" 0.7'
    img = _render(pa, oracle, layered_scene(mat, spp=8, maxdepth=3))
    sky = _render(pa, oracle, layered_scene('Material "interface"', spp=8, maxdepth=3))
    np.testing.assert_allclose(img, sky, rtol=1e-5)
