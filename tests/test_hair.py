"""Hair: HairMaterial (materials.h:353-427, materials.cpp:135-184) and its HairBxDF (bxdfs.h:
1054-1152, bxdfs.cpp:279-573), shaded by the volumetric path's k_vlayered on any surface (the
curves pbrt's wavefront aggregate dices to bilinear patches, h = -1 + 2 v across the width).

* BxDF level: the product's core/hair.h through pbrt_debug_hair against the oracle's ohair
  restatement -- host build (libm) == oracle libm mode bit for bit (CPU), GPU == oracle
  libm mode bit for bit (gpu);
* the reference's own HairBxDF tests (bsdfs_test.cpp:673-820): WhiteFurnace, WhiteFurnaceSampled,
  SamplingWeights, SamplingConsistency, HOnTheEdge -- on the product's host build and on the
  oracle (their thresholds; y(lambda) replaced by the wavelength average, sigma_a = 0 gives a
  constant spectrum);
* the loader's parameter forms (sigma_a, reflectance / color, eumelanin / pheomelanin, the
  default) and refusals, and GPU film parity against the oracle on a curve scene.
"""
import numpy as np
import pytest

from conftest import SCENES

NS = 31


def sphere(u0, u1):
    """SampleUniformSphere (sampling.h)"""
    z = 1 - 2 * u0
    r = np.sqrt(np.maximum(0, 1 - z * z))
    phi = 2 * np.pi * u1
    return np.stack([r * np.cos(phi), r * np.sin(phi), z], -1)


def queries(n, seed, h=None, eta=1.55, bm=None, bn=None, alpha=None, sa=None, slope=0.0):
    rng = np.random.default_rng(seed)
    q = np.zeros((n, 16), np.float32)
    q[:, 0] = rng.uniform(-1, 1, n) if h is None else h
    q[:, 1] = eta
    q[:, 2] = rng.uniform(0.05, 1, n) if bm is None else bm
    q[:, 3] = rng.uniform(0.05, 1, n) if bn is None else bn
    q[:, 4] = rng.uniform(0, 4, n) if alpha is None else alpha
    q[:, 5] = rng.uniform(0, 3, n) if sa is None else sa
    q[:, 6:9] = sphere(rng.uniform(size=n), rng.uniform(size=n))
    q[:, 9:12] = sphere(rng.uniform(size=n), rng.uniform(size=n))
    q[:, 12:15] = rng.uniform(size=(n, 3))
    q[:, 15] = slope
    return q


def test_hair_host_matches_oracle_bitwise(pa, oracle):
    """core/hair.h compiled for the host (libm) == the oracle's restatement in libm mode"""
    q = np.concatenate([queries(20000, 1, slope=0.05), queries(2000, 2, bm=0.08, bn=0.3),  # v <= .1: LogI0 form
                        queries(2000, 3, h=0.0), queries(2000, 4, sa=0.0, alpha=0.0)])
    got = pa.hair_eval(q)
    with oracle.math_mode(oracle.MATH_LIBM):
        ref = oracle.hair_eval(q)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.isfinite(got).all()
    assert got[:, NS + 1].mean() > 0.9  # Sample_f succeeds almost always


def _impls(pa, oracle):
    return {"product": pa.hair_eval, "oracle": oracle.hair_eval}


@pytest.mark.parametrize("impl", ["product", "oracle"])
def test_hair_white_furnace(pa, oracle, impl):
    """bsdfs_test.cpp:673-705: with sigma_a = 0 the BxDF scatters all incident energy"""
    ev = _impls(pa, oracle)[impl]
    rng = np.random.default_rng(5)
    wo = sphere(*rng.uniform(size=2))
    for bm in (0.1, 0.5, 0.9):
        for bn in (0.1, 0.5, 0.9):
            count = 100000 if (bm < .5 or bn < .5) else 20000
            # scrambled low-discrepancy points as the reference's RadicalInverse sequence
            from scipy.stats import qmc
            u = qmc.Halton(d=3, seed=7).random(count)
            q = np.zeros((count, 16), np.float32)
            q[:, 0] = np.clip(-1 + 2 * u[:, 0], -.999999, .999999)
            q[:, 1], q[:, 2], q[:, 3] = 1.55, bm, bn
            q[:, 6:9] = wo
            q[:, 9:12] = sphere(u[:, 1], u[:, 2])
            out = ev(q)
            f = out[:, :NS].mean(axis=1) * np.abs(q[:, 11])
            avg = f.sum() / (count * (1 / (4 * np.pi)))
            assert 0.95 <= avg <= 1.05, (bm, bn, avg)


@pytest.mark.parametrize("impl", ["product", "oracle"])
def test_hair_white_furnace_sampled(pa, oracle, impl):
    """bsdfs_test.cpp:717-748 and :750-784 (SamplingWeights): importance-sampled weights f cos / pdf
    average to 1 (within 1%), and each sample's weight is 1 for beta_n >= 0.4"""
    ev = _impls(pa, oracle)[impl]
    rng = np.random.default_rng(6)
    wo = sphere(*rng.uniform(size=2))
    from scipy.stats import qmc
    for bm in (0.1, 0.3, 0.5, 0.7, 0.9):
        for bn in (0.1, 0.3, 0.5, 0.7, 0.9):
            count = 10000
            u = qmc.Halton(d=4, seed=11).random(count)
            q = np.zeros((count, 16), np.float32)
            q[:, 0] = np.clip(-1 + 2 * u[:, 0], -.999999, .999999)
            q[:, 1], q[:, 2], q[:, 3] = 1.55, bm, bn
            q[:, 6:9] = wo
            q[:, 12:15] = u[:, 1:4]
            out = ev(q)
            ok = out[:, NS + 1] == 1
            w = np.zeros(count)
            w[ok] = out[ok, NS + 6:].mean(axis=1) * np.abs(out[ok, NS + 4]) / out[ok, NS + 5]
            assert 0.99 <= w.sum() / count <= 1.01, (bm, bn, w.sum() / count)
            if bn >= 0.4:
                assert (np.abs(w[ok] - 1) < 0.01).all(), (bm, bn, np.abs(w[ok] - 1).max())


@pytest.mark.parametrize("impl", ["product", "oracle"])
def test_hair_sampling_consistency(pa, oracle, impl):
    """bsdfs_test.cpp:786-820: importance-sampled and uniformly sampled estimates of the light
    scattered from L(w) = w.z^2 agree within 5% (sigma_a = 0.25)"""
    ev = _impls(pa, oracle)[impl]
    rng = np.random.default_rng(8)
    for bm in (0.2, 0.6):
        for bn in (0.4, 0.8):
            count = 64 * 1024
            wo = sphere(*rng.uniform(size=2))
            q = np.zeros((count, 16), np.float32)
            q[:, 0] = rng.uniform(-1, 1, count)
            q[:, 1], q[:, 2], q[:, 3], q[:, 5] = 1.55, bm, bn, 0.25
            q[:, 6:9] = wo
            q[:, 12:15] = rng.uniform(size=(count, 3))
            q[:, 9:12] = sphere(q[:, 13], q[:, 14])
            out = ev(q)
            ok = out[:, NS + 1] == 1
            wi_s = out[:, NS + 2:NS + 5]
            imp = np.where(ok, out[:, NS + 6:].mean(axis=1) * wi_s[:, 2] ** 2 * np.abs(wi_s[:, 2]) /
                           np.where(ok, out[:, NS + 5], 1), 0).sum() / count
            uni = (out[:, :NS].mean(axis=1) * q[:, 11] ** 2 * np.abs(q[:, 11])).sum() / (count / (4 * np.pi))
            assert abs(imp - uni) / uni < 0.05, (bm, bn, imp, uni)


def test_hair_h_on_the_edge(pa, oracle):
    """bsdfs_test.cpp:707-715: h = -1 with beta .1 evaluates without NaN"""
    q = np.zeros((1, 16), np.float32)
    q[0, :6] = [-1, 1.55, .1, .1, 0, 0]
    q[0, 6:12] = [0.54986966, 0.03359017, 0.83457476, -0.37383357, -0.91920084, 0.12376696]
    q[0, 12:15] = 0.5
    for out in (pa.hair_eval(q), oracle.hair_eval(q)):
        assert np.isfinite(out).all()


@pytest.mark.gpu
def test_hair_gpu_matches_oracle_bitwise(pa, oracle):
    """the BxDF compiled for gfx950 (detmath transcendentals, glibc's bit for bit) == the oracle in
    its libm mode"""
    q = np.concatenate([queries(1 << 16, 21, slope=0.05), queries(8192, 22, bm=0.08, bn=0.3), queries(4096, 23, h=0.0)])
    got = pa.hair_eval(q, device=0)
    with oracle.math_mode(oracle.MATH_LIBM):
        ref = oracle.hair_eval(q)
    bad = (got.view(np.uint32) != ref.view(np.uint32)).any(axis=1)
    assert not bad.any(), (bad.sum(), q[bad][:3], got[bad][:3, :8], ref[bad][:3, :8])


# ---------------------------------------------------------------------------------- scenes
HEAD = """LookAt 0 0.55 -1.6  0 0.35 0  0 1 0
Camera "perspective" "float fov" 38
Film "rgb" "integer xresolution" 64 "integer yresolution" 48
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.3 0.32 0.35]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [9 9 9]
Shape "bilinearmesh" "point3 P" [-0.6 2.2 -0.9  0.6 2.2 -0.9  -0.6 2.2 0.3  0.6 2.2 0.3]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.4 0.4 0.4]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3]
"""


def strands(n=48, seed=4, width=0.03):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        x, z = rng.uniform(-0.45, 0.45), rng.uniform(-0.25, 0.25)
        top = rng.uniform(0.5, 0.8)
        bend = rng.uniform(-0.25, 0.25, 2)
        P = [x, 0, z, x + bend[0] * 0.3, top * 0.35, z + bend[1] * 0.3, x + bend[0] * 0.8, top * 0.7, z + bend[1] * 0.8,
             x + bend[0], top, z + bend[1]]
        out.append(f'Shape "curve" "point3 P" [{" ".join(f"{v:.6g}" for v in P)}] "string type" "cylinder" '
                   f'"float width0" {width} "float width1" {width * 0.5}')
    return "\n".join(out) + "\n"


def scene(material, shapes=None):
    return HEAD + f"AttributeBegin\n{material}\n{shapes or strands()}AttributeEnd\n"


def layer(pa, material):
    sc = pa.Scene.from_string(scene(material, 'Shape "sphere" "float radius" 0.2\n'), SCENES)
    f = sc.flat()
    mt = np.ctypeslib.as_array(f.material_type, shape=(f.n_materials,)).copy()
    ml = np.ctypeslib.as_array(f.material_layer, shape=(f.n_materials * 12,)).reshape(-1, 12).copy()
    return ml[mt == 9]


def test_hair_loader_forms(pa):
    # sigma_a given (RGBUnbounded: scale 2 max), eta / betas / alpha
    (ml,) = layer(pa, 'Material "hair" "rgb sigma_a" [0.2 0.4 1.0] "float eta" 1.5 "float beta_m" 0.2 '
                      '"float beta_n" 0.6 "float alpha" 3')
    assert (ml[0], ml[1], ml[6]) == (0, 1, 2.0) and (ml[8], ml[9], ml[10], ml[11]) == (1.5, np.float32(0.2), np.float32(0.6), 3)
    # reflectance (and its alias color): mode 1, an albedo (scale 1)
    for nm in ("reflectance", "color"):
        (ml,) = layer(pa, f'Material "hair" "rgb {nm}" [0.3 0.2 0.1]')
        assert (ml[0], ml[1], ml[6]) == (1, 1, 1) and ml[8] == np.float32(1.55)
    # eumelanin / pheomelanin: SigmaAFromConcentration's RGB
    (ml,) = layer(pa, 'Material "hair" "float eumelanin" 2 "float pheomelanin" 0.5')
    assert ml[0] == 0 and ml[6] == np.float32(2 * (np.float32(1.37) * 2 + np.float32(1.05) * np.float32(0.5)))
    # the default: eumelanin 1.3, beta .3 .3, alpha 2
    (ml,) = layer(pa, 'Material "hair"')
    assert ml[6] == np.float32(2 * np.float32(np.float32(1.3) * np.float32(1.37)))
    assert (ml[9], ml[10], ml[11]) == (np.float32(0.3), np.float32(0.3), 2)


@pytest.mark.parametrize("material, msg", [
    ('Material "hair" "rgb reflectance" [1.2 0.5 0.5]', "albedo"),
    ('Material "hair" "rgb sigma_a" [-1 0.5 0.5]', "negative"),
    ('Material "hair" "rgb beta_m" [0.1 0.2 0.3]', "not a float parameter"),
    ('Material "hair" "texture beta_m" "nope"', "nope"),
])
def test_hair_loader_errors(pa, material, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(scene(material), SCENES)


def test_hair_oracle_renders(pa, oracle):
    sc = pa.Scene.from_string(scene('Material "hair" "float eumelanin" 0.8'), SCENES, xresolution=24, yresolution=18, spp=8)
    f = sc.flat()
    img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert np.isfinite(img).all() and img.mean() > 0.01


# textured sigma_a (Unbounded) and reflectance (Albedo): GetSpectrumTexture per hit
# (materials.cpp:135-160, materials.h:380-404), evaluated by k_vtexture for k_vlayered
TEX_REFL = ('Texture "c" "spectrum" "checkerboard" "float uscale" 6 "float vscale" 6 "rgb tex1" [0.8 0.5 0.3] '
            '"rgb tex2" [0.25 0.2 0.1]\nMaterial "hair" "texture reflectance" "c" "float beta_n" 0.4')
TEX_SIGMA = ('Texture "s" "spectrum" "checkerboard" "float uscale" 6 "float vscale" 6 "rgb tex1" [0.2 0.4 1.0] '
             '"rgb tex2" [1.5 1.0 0.6]\nMaterial "hair" "texture sigma_a" "s"')

# textured floats (GetFloatTexture, materials.cpp:135-184): beta_m / beta_n / alpha / eta per
# hit, and the eumelanin / pheomelanin pair forming sigma_a per hit (SigmaAFromConcentration)
TEX_FLOATS = ('Texture "bm" "float" "checkerboard" "float uscale" 6 "float vscale" 6 "float tex1" 0.15 "float tex2" 0.6\n'
              'Texture "al" "float" "scale" "float tex" 3 "float scale" 0.5\n'
              'Material "hair" "rgb sigma_a" [0.2 0.4 1.0] "texture beta_m" "bm" "texture beta_n" "bm" '
              '"texture alpha" "al" "float eta" 1.5')
TEX_MELANIN = ('Texture "eu" "float" "checkerboard" "float uscale" 6 "float vscale" 6 "float tex1" 0.3 "float tex2" 2.5\n'
               'Material "hair" "texture eumelanin" "eu" "float pheomelanin" 0.4')
TEX_ETA = ('Texture "e" "float" "checkerboard" "float uscale" 6 "float vscale" 6 "float tex1" 1.3 "float tex2" 1.9\n'
           'Material "hair" "rgb reflectance" [0.8 0.55 0.3] "texture eta" "e"')

FORMS = {
    "melanin": 'Material "hair" "float eumelanin" 0.8 "float pheomelanin" 0.3',
    "reflectance": 'Material "hair" "rgb reflectance" [0.8 0.55 0.3] "float beta_m" 0.25 "float beta_n" 0.4',
    "sigma_rough": 'Material "hair" "rgb sigma_a" [0.06 0.1 0.2] "float beta_m" 0.6 "float beta_n" 0.8 "float alpha" 0',
    "tex_reflectance": TEX_REFL,
    "tex_sigma_a": TEX_SIGMA,
    "tex_floats": TEX_FLOATS,
    "tex_melanin": TEX_MELANIN,
    "tex_eta": TEX_ETA,
}


@pytest.mark.parametrize("material, const", [
    (TEX_REFL, 'Material "hair" "rgb reflectance" [0.8 0.5 0.3] "float beta_n" 0.4'),
    (TEX_SIGMA, 'Material "hair" "rgb sigma_a" [0.2 0.4 1.0]'),
])
def test_textured_hair_oracle(pa, oracle, material, const):
    """The textured forms load (the program in the material's texture slot), render finite,
    and differ from the constant form that equals one of the checks."""
    kw = dict(xresolution=24, yresolution=18, spp=8)
    sc, sc0 = pa.Scene.from_string(scene(material), SCENES, **kw), pa.Scene.from_string(scene(const), SCENES, **kw)
    f = sc.flat()
    assert any(f.material_tex[4 * k] >= 0 for k in range(f.n_materials))
    m = [f.output_rgb_from_sensor_rgb[i] for i in range(9)]
    a = oracle.film_to_rgb(oracle.render(sc, threads=8), m)
    b = oracle.film_to_rgb(oracle.render(sc0, threads=8), m)
    assert np.isfinite(a).all() and a.mean() > 0.005
    assert np.abs(a - b).mean() > 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("form", list(FORMS))
def test_hair_matches_oracle_gpu(pa, oracle, form):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(scene(FORMS[form]), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"hair ({form}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.parametrize("material, const, slots", [
    (TEX_FLOATS, 'Material "hair" "rgb sigma_a" [0.2 0.4 1.0] "float beta_m" 0.15 "float beta_n" 0.15 "float alpha" 1.5 '
                 '"float eta" 1.5', (1, 2, 3)),
    (TEX_MELANIN, 'Material "hair" "float eumelanin" 0.3 "float pheomelanin" 0.4', (4, 5)),
    (TEX_ETA, 'Material "hair" "rgb reflectance" [0.8 0.55 0.3] "float eta" 1.3', (0,)),
])
def test_textured_hair_floats_oracle(pa, oracle, material, const, slots):
    """Textured hair floats load into material_hair_tex (the other slots stay constants), render
    finite, and differ from the constant form that equals one of the checks."""
    kw = dict(xresolution=24, yresolution=18, spp=8)
    sc, sc0 = pa.Scene.from_string(scene(material), SCENES, **kw), pa.Scene.from_string(scene(const), SCENES, **kw)
    f = sc.flat()
    mt = np.ctypeslib.as_array(f.material_type, shape=(f.n_materials,))
    hair = int(np.flatnonzero(mt == 9)[0])
    ht = np.ctypeslib.as_array(f.material_hair_tex, shape=(f.n_materials * 6,)).reshape(-1, 6)[hair]
    assert [k for k in range(6) if ht[k] >= 0] == list(slots)
    assert not sc0.flat().material_hair_tex
    m = [f.output_rgb_from_sensor_rgb[i] for i in range(9)]
    a = oracle.film_to_rgb(oracle.render(sc, threads=8), m)
    b = oracle.film_to_rgb(oracle.render(sc0, threads=8), m)
    assert np.isfinite(a).all() and a.mean() > 0.005
    assert np.abs(a - b).mean() > 1e-4
