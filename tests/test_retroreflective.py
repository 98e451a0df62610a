"""Material "retroreflective" -- this fork's RetroreflectiveMaterial (materials.h:553-627, created by
materials.cpp:263-297 from the conductor's parameters) and its RetroreflectiveBxDF (bxdfs.h:102-215),
shaded by the volumetric kernels' k_vlayered stage.

The BxDF is kept with the reference's quirks, bit for bit:
* Sample_f, smooth: wi = wo (the light goes back where it came from), f = FrComplex(|cos wi|) / |cos wi|,
  pdf 1, specular;
* Sample_f, rough: the conductor's microfacet reflection sample and the conductor's f (no retro lobe);
* f: (1 - (R_i - R_o)) [D(wo) F(|wi.wo|) G / 4cc + D(wm) F(|wo.wm|) G / 4cc] with R = FrDielectric(., 1.59);
* PDF: the conductor's (the retro lobe is not sampled).

bxdfs.h does not compile here (media.h -> NanoVDB), so the pin is two independent restatements (the
product's core.h and the oracle's BxDF) agreeing bit for bit, plus the known answers below; GPU
film parity against the oracle is in the gpu tests at the end."""
import numpy as np
import pytest

from conftest import SCENES
from test_bxdf import _cases, _conductor_spectra, same
from test_layered import layered_scene


@pytest.mark.parametrize("params,metal", [((0.0, 0.0, 0.0), "Cu"), ((0.3162278, 0.3162278, 0.0), "Au"),
                                          ((0.1, 0.02, 0.0), "Al"), ((0.6, 0.6, 0.0), "Ag")])
def test_retroreflective_bxdf_product_matches_oracle(pa, oracle, params, metal):
    """Sample_f / f / PDF (pbrt_debug_bxdf type 11) against the oracle's restatement, bit for bit."""
    wo, wi, u = _cases(3, 1000)
    eta, k = _conductor_spectra(pa, metal, 431.7)
    n_ok = n_f = 0
    for j in range(len(wo)):
        a = pa.debug_bxdf(11, params, wo[j], wi[j], u[j], eta, k)
        b = oracle.bxdf(11, params, wo[j], wi[j], u[j], eta, k)
        assert same(a, b), (params, j, a[:8], b[:8])
        n_ok += a[0] == 1
        n_f += np.any(a[38:69] != 0)
    assert n_ok > 300
    if params[0] > 0:
        assert n_f > 300


def test_smooth_sample_goes_back_along_wo(pa):
    eta, k = _conductor_spectra(pa, "Cu", 500.0)
    wo = np.array([0.3, -0.2, 0.9327379], np.float32)
    out = pa.debug_bxdf(11, (0, 0, 0), wo, wo, (0.5, 0.5, 0.5), eta, k)
    assert out[0] == 1 and np.array_equal(out[1:4], wo) and out[4] == 1
    assert int(out[5]) == 17  # BxDFFlags::SpecularReflection
    assert not np.any(out[38:70])  # smooth: f = 0, PDF = 0
    # f = FrComplex(|cos|) / |cos| for every wavelength
    cond = pa.debug_bxdf(2, (0, 0, 0), np.array([-0.3, 0.2, 0.9327379], np.float32), wo, (0.5, 0.5, 0.5), eta, k)
    np.testing.assert_array_equal(out[7:38], cond[7:38])


def test_rough_f_is_conductor_plus_retro_lobe(pa):
    """Where wi = wo the retro and conductor lobes coincide (wm = wo) and R_i = R_o, so f is twice
    the conductor's f; PDF equals the conductor's everywhere."""
    eta, k = _conductor_spectra(pa, "Au", 420.0)
    w = np.array([0.2, 0.1, 0.9746794], np.float32)
    w = (w / np.linalg.norm(w)).astype(np.float32)
    r = pa.debug_bxdf(11, (0.3, 0.3, 0), w, w, (0.5, 0.5, 0.5), eta, k)
    c = pa.debug_bxdf(2, (0.3, 0.3, 0), w, w, (0.5, 0.5, 0.5), eta, k)
    np.testing.assert_allclose(r[38:69], 2 * c[38:69], rtol=2e-6)
    assert r[69] == c[69]
    wo, wi, u = _cases(5, 200)
    for j in range(len(wo)):
        a = pa.debug_bxdf(11, (0.2, 0.2, 0), wo[j], wi[j], u[j], eta, k)
        b = pa.debug_bxdf(2, (0.2, 0.2, 0), wo[j], wi[j], u[j], eta, k)
        assert a[69] == b[69]
        assert np.array_equal(a[:38], b[:38])  # the rough sample is the conductor's


def test_loader(pa):
    sc = pa.Scene.from_string(layered_scene('Material "retroreflective" "float roughness" 0.1'), SCENES)
    f = sc.flat()
    assert f.material_type[0] == 11 and f.material_spectra[0] >= 0 and f.material_spectra[1] >= 0
    assert f.material_params[0] == np.float32(np.sqrt(np.float32(0.1)))  # remaproughness
    sc = pa.Scene.from_string(layered_scene('Material "retroreflective" "rgb reflectance" [0.8 0.7 0.2]'), SCENES)
    assert sc.flat().material_spectra[0] == -1
    with pytest.raises(RuntimeError, match="both"):
        pa.Scene.from_string(layered_scene('Material "retroreflective" "rgb reflectance" [0.8 0.7 0.2] '
                                           '"spectrum eta" "metal-Au-eta"'), SCENES)
    with pytest.raises(RuntimeError, match="textured"):
        pa.Scene.from_string(layered_scene('Texture "r" "float" "constant" "float value" 0.2\n'
                                           'Material "retroreflective" "texture roughness" "r"'), SCENES)


def retro_scene(res=48, spp=16, roughness=0.15, medium=False):
    """A retroreflective sphere and floor beside a conductor, lit by an area light near the camera
    (where a retroreflector sends the light back) and a dim sky."""
    med = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.02 0.02 0.02] '
           '"rgb sigma_s" [0.05 0.05 0.05]\nMediumInterface "" "fog"\n') if medium else ""
    cam_medium = 'MediumInterface "" "fog"\n' if medium else ""
    head = (f'LookAt 0 1 -4  0 0.3 0  0 1 0\n{med if medium else ""}Camera "perspective" "float fov" 40\n'
            f'Film "rgb" "integer xresolution" {res} "integer yresolution" {res}\n'
            f'Sampler "halton" "integer pixelsamples" {spp}\nIntegrator "volpath" "integer maxdepth" 5\n')
    return head + f"""WorldBegin
{cam_medium}LightSource "infinite" "rgb L" [0.05 0.05 0.06]
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [8 8 8]
  Material "diffuse"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3]
    "point3 P" [-0.3 1.3 -3.6  0.3 1.3 -3.6  0.3 0.9 -3.8  -0.3 0.9 -3.8]
AttributeEnd
AttributeBegin
  Material "retroreflective" "float roughness" {roughness}
  Translate -0.6 0.4 0
  Shape "sphere" "float radius" 0.4
AttributeEnd
AttributeBegin
  Material "retroreflective" "rgb reflectance" [0.9 0.8 0.3] "float roughness" 0
  Translate 0.6 0.4 0
  Shape "sphere" "float radius" 0.4
AttributeEnd
AttributeBegin
  Material "retroreflective" "float roughness" 0.3 "spectrum eta" "metal-Ag-eta" "spectrum k" "metal-Ag-k"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3]
    "point3 P" [-3 0 -3  3 0 -3  3 0 3  -3 0 3]
AttributeEnd
"""


def test_retroreflector_returns_light_to_the_source(pa, oracle):
    """Known answer of the smooth case: a quad turned 30 degrees from the view, lit only by a large
    emitter behind the camera.  The smooth retroreflector sends every camera path straight back
    (wi = wo), onto the emitter: the image is Fr(cos) L.  A smooth conductor in the same place
    mirrors the paths 60 degrees sideways, past the emitter: black."""
    head = ('LookAt 0 0 -3  0 0 0  0 1 0\nCamera "perspective" "float fov" 20\n'
            'Film "rgb" "integer xresolution" 16 "integer yresolution" 16\n'
            'Sampler "halton" "integer pixelsamples" 4\nIntegrator "volpath" "integer maxdepth" 3\nWorldBegin\n'
            'AttributeBegin\n  AreaLightSource "diffuse" "rgb L" [1 1 1] "bool twosided" true\n'
            '  Material "diffuse" "float reflectance" 0\n'
            '  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 -3 -4  3 -3 -4  3 3 -4  -3 3 -4]\n'
            'AttributeEnd\n')
    quad = ('Rotate 30 0 1 0\nShape "trianglemesh" "integer indices" [0 1 2 0 2 3] '
            '"point3 P" [-2 -2 0  2 -2 0  2 2 0  -2 2 0]\n')
    imgs = {}
    for name in ("retroreflective", "conductor"):
        sc = pa.Scene.from_string(head + f'Material "{name}" "float roughness" 0\n' + quad, SCENES)
        f = sc.flat()
        imgs[name] = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert imgs["conductor"].max() == 0
    # copper's Fresnel at 20-40 degrees, every pixel (the emitter is black, so nothing else adds)
    assert imgs["retroreflective"].min() > 0.2 and imgs["retroreflective"].max() < 1


@pytest.mark.gpu
@pytest.mark.parametrize("medium", [False, True])
def test_retroreflective_gpu_matches_oracle(pa, oracle, medium):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(retro_scene(medium=medium), SCENES)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    ref = oracle_rgb(oracle, sc)
    assert ref.mean() > 0.01
    frac, mr = check(gpu, ref)
    print(f"retroreflective (medium={medium}): {frac * 100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")
