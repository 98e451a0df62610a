"""Procedural textures: FloatDots/SpectrumDots, FBm, Wrinkled, Windy and Marble (textures.h:
427-505, 813-841, 1117-1160; textures.cpp:287-353, 524-563, 1008-1032; FBm / Turbulence
util/noise.cpp:114-152), as the wavefront's UniversalTextureEvaluator runs them.

* the product's code (core/texture_eval.h, through pbrt_debug_procedural on the host) and the
  oracle's restatement against the reference's FBm / Turbulence and refgold's restatement of
  InsidePolkaDot / MarbleTexture over the reference's Noise, FBm, EvaluateCubicBezier and sRGB
  RGBToSpectrumTable (tests/golden, "procedural_textures"), bit for bit;
* the loader (Create defaults, float / spectrum availability);
* texture programs in a scene: product texture evaluation against the oracle's tree walk;
* GPU film parity on a scene with every procedural texture in reflectance, roughness and bump.

The wavefront's texture contexts carry no dpdx / dpdy (workitems.h:288-304), so in a render
every FBm evaluates all its octaves; the goldens also cover nonzero differentials.
"""
import numpy as np
import pytest

from conftest import SCENES

KINDS = {0: "fbm", 1: "turbulence", 2: "windy", 3: "dots", 4: "marble"}


def _rows(cfg):
    x = np.array([r[0] for r in cfg["rows"]], np.float32)
    y = np.array([r[1] for r in cfg["rows"]], np.float32)
    return x, y


def _perm(sc):
    f = sc.flat()
    return np.ctypeslib.as_array(f.noise_perm, shape=(512,)).copy()


def test_procedural_goldens_present(golden):
    kinds = {c["kind"] for c in golden["procedural_textures"]}
    assert kinds == set(KINDS)


@pytest.mark.parametrize("cfg_index", range(8))
def test_procedural_product_bit_exact(pa, golden, cfg_index):
    cfg = golden["procedural_textures"][cfg_index]
    x, y = _rows(cfg)
    got = pa.procedural(cfg["kind"], cfg["params"], x)
    cols = 6 if cfg["kind"] == 4 else 1
    np.testing.assert_array_equal(got[:, :cols], y[:, :cols], err_msg=KINDS[cfg["kind"]])


@pytest.mark.parametrize("cfg_index", range(8))
def test_procedural_oracle_bit_exact(pa, oracle, golden, cfg_index):
    cfg = golden["procedural_textures"][cfg_index]
    x, y = _rows(cfg)
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    got = oracle.procedural(cfg["kind"], _perm(sc), cfg["params"], x)
    cols = 6 if cfg["kind"] == 4 else 1
    np.testing.assert_array_equal(got[:, :cols], y[:, :cols], err_msg=KINDS[cfg["kind"]])


HEAD = """LookAt 0 1.2 -4  0 0.4 0  0 1 0
Camera "perspective" "float fov" 38
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 4
WorldBegin
LightSource "infinite" "rgb L" [0.35 0.38 0.42]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [5 5 5]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.6 2.6 -0.6 0.6 2.6 -0.6 0.6 2.6 0.6 -0.6 2.6 0.6]
AttributeEnd
"""
PROC = """Texture "dotsf" "float" "dots" "float uscale" 6 "float vscale" 6 "float inside" 0.02 "float outside" 0.3
Texture "dotss" "spectrum" "dots" "float uscale" 5 "float vscale" 5 "rgb inside" [0.8 0.2 0.1] "rgb outside" [0.2 0.5 0.7]
Texture "fbm" "float" "fbm" "integer octaves" 6 "float roughness" 0.6
Texture "wrink" "float" "wrinkled" "integer octaves" 5
Texture "windy" "float" "windy"
Texture "marble" "spectrum" "marble" "float scale" 2.5 "float variation" 0.4
Texture "fbmscaled" "float" "scale" "texture tex" "fbm" "float scale" 0.05
Material "diffuse" "texture reflectance" "dotss" "texture displacement" "fbmscaled"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-4 0 -4 4 0 -4 4 0 4 -4 0 4]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "diffuse" "texture reflectance" "marble"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1.6 0 1 -0.2 0 1 -0.2 1.4 1 -1.6 1.4 1]
    "point2 uv" [0 0 1 0 1 1 0 1]
Material "conductor" "texture roughness" "dotsf" "spectrum eta" "metal-Cu-eta" "spectrum k" "metal-Cu-k"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [0.2 0 1 1.6 0 1 1.6 1.4 1 0.2 1.4 1]
    "point2 uv" [0 0 1 0 1 1 0 1]
Texture "wmix" "float" "mix" "texture tex1" "wrink" "texture tex2" "windy" "float amount" 0.5
Material "dielectric" "float eta" 1.5 "texture roughness" "wmix" "bool remaproughness" true
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.5 0.2 -0.5 0.5 0.2 -0.5 0.5 1.0 -0.2 -0.5 1.0 -0.2]
    "point2 uv" [0 0 1 0 1 1 0 1]
"""


def test_procedural_loader(pa):
    sc = pa.Scene.from_string(HEAD + PROC, SCENES)
    f = sc.flat()
    info = np.ctypeslib.as_array(f.tex_node_info, shape=(f.n_tex_nodes * 8,)).reshape(-1, 8)
    par = np.ctypeslib.as_array(f.tex_node_params, shape=(f.n_tex_nodes * 28,)).reshape(-1, 28)
    kinds = set(info[:, 0].tolist())
    assert {7, 8, 9, 10, 11} <= kinds
    fbm = par[info[:, 0] == 8][0]
    assert (fbm[22], np.float32(fbm[23])) == (6, np.float32(0.6))
    wr = par[info[:, 0] == 9][0]
    assert (wr[22], wr[23]) == (5, 0.5)  # roughness default .5
    mb = par[info[:, 0] == 11][0]
    assert (mb[22], mb[23], np.float32(mb[24]), np.float32(mb[26])) == (8, 0.5, np.float32(0.4), np.float32(2.5))


@pytest.mark.parametrize("text, msg", [
    ('Texture "m" "float" "marble"\nMaterial "diffuse" "texture roughness" "m"\n', "not supported"),
    ('Texture "f" "spectrum" "fbm"\nMaterial "diffuse" "texture reflectance" "f"\n', "not supported"),
])
def test_procedural_loader_float_spectrum_classes(pa, text, msg):
    """pbrt's FloatTexture::Create knows fbm / wrinkled / windy but not marble, its
    SpectrumTexture::Create marble but not the others (textures.cpp:1606-1707)."""
    shape = 'Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [0 0 0 1 0 0 0 1 0]\n'
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(HEAD + text + shape, SCENES)


def test_procedural_texture_eval_matches_oracle(pa, oracle):
    """Every textured material slot of the scene (dots as reflectance and roughness, marble,
    a mix of wrinkled and windy roughness) at 300 seeded hits: the product's compiled programs
    (TexPhase1 / TexPhase2, run on the host) against the oracle's tree walk, bit for bit."""
    sc = pa.Scene.from_string(HEAD + PROC, SCENES)
    f = sc.flat()
    mt = np.ctypeslib.as_array(f.material_tex, shape=(f.n_materials * 4,)).reshape(-1, 4)
    rng = np.random.default_rng(5)
    lam = np.linspace(395, 705, 31).astype(np.float32)
    checked = 0
    for m in range(f.n_materials):
        for slot in range(3):
            if mt[m][slot] < 0:
                continue
            for _ in range(300):
                p = rng.uniform(-3, 3, 3)
                nrm = rng.normal(size=3)
                nrm /= np.linalg.norm(nrm)
                hit = np.concatenate([p, nrm, rng.normal(size=3), rng.normal(size=3),
                                      rng.uniform(-0.5, 1.5, 2)]).astype(np.float32)
                d1, v1 = sc.texture_eval(m, slot, hit, lam)
                d2, v2 = oracle.texture_eval(sc, m, slot, hit, lam)
                assert np.array_equal(d1, d2)
                assert np.array_equal(np.atleast_1d(v1), np.atleast_1d(v2)), (m, slot, hit)
                checked += 1
    assert checked >= 4 * 300


@pytest.mark.gpu
def test_procedural_scene_matches_oracle_gpu(pa, oracle):
    """The textured material stage (k_texture<..., Full>) with dots, fbm (bump), wrinkled and
    windy (roughness) and marble (reflectance) on the GPU against the oracle."""
    from test_gpu_parity import check_parity, gpu_film, oracle_film, to_rgb
    sc = pa.Scene.from_string(HEAD + PROC, SCENES)
    film, integ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle_film(oracle, sc, integ)))
    print(f"procedural textures: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_procedural_volumetric_matches_oracle_gpu(pa, oracle):
    """The same textures on the volumetric kernels (k_vtexture) beside a fog box."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    from test_media import box
    fog = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.05 0.08 0.1] '
           '"rgb sigma_s" [0.4 0.35 0.3] "float g" 0.3\nAttributeBegin\nMediumInterface "fog" ""\n'
           'Material "interface"\n' + box(-1.2, 1.2, 0.02, 1.6, -1.5, 0.6) + '\nAttributeEnd\n')
    sc = pa.Scene.from_string(HEAD + fog + PROC.replace(' "texture displacement" "fbmscaled"', ''), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"procedural textures (volumetric): {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")
