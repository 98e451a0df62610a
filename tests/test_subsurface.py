"""Subsurface scattering: SubsurfaceMaterial (materials.h:772-866, materials.cpp:544-613), its
TabulatedBSSRDF (bssrdf.h, bssrdf.cpp) and the wavefront's SampleSubsurface stages
(wavefront/subsurface.cpp:18-206) with the aggregate's IntersectOneRandom probe
(optix.cu:478-518).  The product renders subsurface scenes on the volumetric kernels
(k_vsurface diverts transmitted samples to k_vsss_probe / k_vsss_scatter).

* the Catmull-Rom spline utilities the BSSRDF runs on (CatmullRomWeights, InvertCatmullRom,
  SampleCatmullRom2D) -- product (core/bssrdf.h through pbrt_debug_catmull_rom) and oracle --
  bit for bit against the reference's own functions (tests/golden "catmull_rom");
* the BSSRDF table (ComputeBeamDiffusionBSSRDF): bssrdf.cpp includes media.h -> NanoVDB, which
  this image lacks, so the table is restated twice (host/bssrdf.cpp for the product, the
  oracle's osss::Table) and the two are held equal bit for bit -- parity unpinned against the
  reference itself for the beam-diffusion integrals;
* the loader's four parameter forms and pbrt's errors; the sampler's 10 dimensions per depth;
* GPU film parity against the oracle for the forms, rough and smooth interfaces.
"""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 1.4 -3.2  0 0.45 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 64 "integer yresolution" 48
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 6
WorldBegin
LightSource "infinite" "rgb L" [0.25 0.27 0.3]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [7 7 7]
Shape "bilinearmesh" "point3 P" [-0.7 2.6 -0.7  0.7 2.6 -0.7  -0.7 2.6 0.7  0.7 2.6 0.7]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.45 0.45 0.45]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3]
"""
# a closed smooth blob (loop-subdivided octahedron) and a box
BLOB = ('Shape "loopsubdiv" "integer levels" 3 "integer indices" [0 2 4 2 1 4 1 3 4 3 0 4 2 0 5 1 2 5 3 1 5 0 3 5] '
        '"point3 P" [0.5 0.5 0  -0.5 0.5 0  0 1.0 0  0 0.02 0  0 0.5 0.5  0 0.5 -0.5]\n')
BOX = ('Shape "trianglemesh" "integer indices" [0 2 1 0 3 2  4 5 6 4 6 7  0 1 5 0 5 4  3 7 6 3 6 2  0 4 7 0 7 3  1 2 6 1 6 5] '
       '"point3 P" [0.45 0.01 -0.3  1.05 0.01 -0.3  1.05 0.61 -0.3  0.45 0.61 -0.3  '
       '0.45 0.01 0.3  1.05 0.01 0.3  1.05 0.61 0.3  0.45 0.61 0.3]\n')


def scene(material, shape=BLOB):
    return HEAD + f"AttributeBegin\n{material}\n{shape}AttributeEnd\n"


def flat_sss(pa, material):
    sc = pa.Scene.from_string(scene(material), SCENES)
    f = sc.flat()
    # copies: the views die with the scene
    ms = np.ctypeslib.as_array(f.material_sss, shape=(f.n_materials,)).copy()
    par = np.ctypeslib.as_array(f.sss_params, shape=(f.n_sss * 20,)).reshape(-1, 20).copy()
    tab = np.ctypeslib.as_array(f.sss_tables, shape=(f.n_sss * 13064,)).reshape(-1, 13064).copy()
    return sc, f, ms, par, tab


def test_catmull_rom_matches_reference(pa, oracle, golden):
    c = golden["catmull_rom"]
    n1, n2, f1 = (np.array(c[k], np.float32) for k in ("nodes1", "nodes2", "f1"))
    vals, cdf = np.array(c["values"], np.float32), np.array(c["cdf"], np.float32)
    w = np.array(c["weights"], np.float32)
    inv = np.array(c["invert"], np.float32)
    smp = np.array(c["sample2d"], np.float32)
    for impl in (pa.catmull_rom, oracle.catmull_rom):
        got = impl(0, n1, n2, vals, cdf, w[:, 0])
        ok = w[:, 1] == 1
        np.testing.assert_array_equal(got[:, 0], w[:, 1])
        np.testing.assert_array_equal(got[ok, 1:], w[ok, 2:])
        np.testing.assert_array_equal(impl(1, n1, n2, f1, cdf, inv[:, 0]), inv[:, 1])
        np.testing.assert_array_equal(impl(3, n1, n2, vals, cdf, smp[:, :2].ravel()), smp[:, 2])


@pytest.mark.parametrize("g, eta", [(0.0, 1.33), (0.3, 1.5), (-0.2, 1.2)])
def test_bssrdf_table_product_equals_oracle(pa, oracle, g, eta):
    sc, f, ms, par, tab = flat_sss(pa, f'Material "subsurface" "float g" {g} "float eta" {eta} '
                                      '"rgb sigma_a" [0.2 0.3 0.4] "rgb sigma_s" [2 3 4]')
    ref = oracle.sss_table(g, eta)
    np.testing.assert_array_equal(tab[0], ref)
    rho, rad, prof, rhoEff = ref[:100], ref[100:164], ref[164:164 + 6400].reshape(100, 64), ref[6564:6664]
    cdf = ref[6664:].reshape(100, 64)
    assert rho[0] == 0 and rho[-1] == 1 and (np.diff(rho) > 0).all()
    assert rad[0] == 0 and rad[1] == np.float32(2.5e-3)
    assert (np.diff(rhoEff) > 0).all() and rhoEff[-1] < 1.2 and rhoEff[0] == 0
    assert (np.diff(cdf, axis=1) >= -1e-7).all()
    np.testing.assert_array_equal(cdf[:, -1], rhoEff)
    assert f.dims_per_depth == 10


def test_subsurface_loader_forms(pa):
    # sigma_a / sigma_s given (RGBUnbounded: scale 2 max)
    sc, f, ms, par, _ = flat_sss(pa, 'Material "subsurface" "rgb sigma_a" [0.2 0.3 0.4] "rgb sigma_s" [2 3 4] '
                                     '"float scale" 3 "float eta" 1.4 "float roughness" 0.2')
    assert (ms >= 0).sum() == 1
    p = par[0]
    assert (p[0], p[1], np.float32(p[2])) == (0, 3, np.float32(1.4))
    assert p[4] == 1 and p[9] == np.float32(0.8) and p[11] == 1 and p[16] == 8
    mt = np.ctypeslib.as_array(f.material_type, shape=(f.n_materials,))
    assert mt[ms >= 0][0] == 1  # a dielectric at the surface
    # reflectance / mfp (mode 1), mfp default ConstantSpectrum(1)
    _, _, _, par, _ = flat_sss(pa, 'Material "subsurface" "rgb reflectance" [0.8 0.5 0.3]')
    assert par[0][0] == 1 and par[0][4] == 1 and par[0][9] == 1 and (par[0][11], par[0][12]) == (0, 1)
    # a named medium: g forced to 0 (with a warning), Skin1's measured coefficients
    _, _, _, par, _ = flat_sss(pa, 'Material "subsurface" "string name" "Skin1" "float g" 0.5')
    assert par[0][18] == 0 and par[0][9] == np.float32(2 * 0.48) and par[0][16] == np.float32(2 * 1.01)
    # nothing given: the defaults RGB(.0011, .0024, .014) / RGB(2.55, 3.21, 3.77)
    _, _, _, par, _ = flat_sss(pa, 'Material "subsurface"')
    assert par[0][9] == np.float32(2 * 0.014) and par[0][16] == np.float32(2 * 3.77)
    assert par[0][2] == np.float32(1.33)


@pytest.mark.parametrize("material, msg", [
    ('Material "subsurface" "rgb sigma_a" [1 1 1]', 'without "sigma_s"'),
    ('Material "subsurface" "rgb sigma_s" [1 1 1]', 'without "sigma_a"'),
    ('Material "subsurface" "string name" "Nope"', "named medium not found"),
    ('Material "subsurface" "rgb reflectance" [1.2 0.5 0.5]', "albedo"),
    ('Material "subsurface" "rgb reflectance" [0.5 0.5 0.5] "texture mfp" "nope"', "nope"),
])
def test_subsurface_loader_errors(pa, material, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(scene(material), SCENES)


def test_subsurface_oracle_renders(pa, oracle):
    sss = pa.Scene.from_string(scene('Material "subsurface" "rgb reflectance" [0.8 0.6 0.4] "rgb mfp" [0.05 0.05 0.05]'),
                               SCENES, xresolution=24, yresolution=18, spp=8)
    f = sss.flat()
    img = oracle.film_to_rgb(oracle.render(sss, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert np.isfinite(img).all() and img.mean() > 0.01


# a textured reflectance (GetBSSRDF's texEval(reflectance), materials.h:823-841): the texture stage
# evaluates it at the entry hit and k_vsss_probe / k_vsss_scatter read it there
TEX_REFL = ('Texture "t" "spectrum" "checkerboard" "float uscale" 4 "float vscale" 4 "rgb tex1" [0.9 0.6 0.4] '
            '"rgb tex2" [0.3 0.5 0.8]\nMaterial "subsurface" "texture reflectance" "t" "rgb mfp" [0.08 0.06 0.05]')


def test_textured_reflectance_oracle(pa, oracle):
    kw = dict(xresolution=32, yresolution=24, spp=8)
    a_sc = pa.Scene.from_string(scene(TEX_REFL, BLOB + BOX), SCENES, **kw)
    b_sc = pa.Scene.from_string(scene('Material "subsurface" "rgb reflectance" [0.9 0.6 0.4] "rgb mfp" [0.08 0.06 0.05]',
                                      BLOB + BOX), SCENES, **kw)
    f = a_sc.flat()
    assert any(f.material_tex[4 * k] >= 0 for k in range(f.n_materials))
    m = [f.output_rgb_from_sensor_rgb[i] for i in range(9)]
    a = oracle.film_to_rgb(oracle.render(a_sc, threads=8), m)
    b = oracle.film_to_rgb(oracle.render(b_sc, threads=8), m)
    assert np.isfinite(a).all() and a.mean() > 0.01
    assert np.abs(a - b).mean() > 1e-4


# textured mfp (with a constant or a textured reflectance) and textured sigma_a / sigma_s
# (GetSpectrumTextureOrNull, Unbounded; texEval per hit at the entry, materials.h:823-841)
TEX_MFP = ('Texture "m" "spectrum" "checkerboard" "float uscale" 4 "float vscale" 4 "rgb tex1" [0.03 0.03 0.02] '
           '"rgb tex2" [0.2 0.15 0.1]\nMaterial "subsurface" "rgb reflectance" [0.9 0.6 0.4] "texture mfp" "m"')
TEX_BOTH = ('Texture "t" "spectrum" "checkerboard" "float uscale" 4 "float vscale" 4 "rgb tex1" [0.9 0.6 0.4] '
            '"rgb tex2" [0.3 0.5 0.8]\nTexture "m" "spectrum" "scale" "rgb tex" [0.08 0.06 0.05] "float scale" 1.5\n'
            'Material "subsurface" "texture reflectance" "t" "texture mfp" "m"')
TEX_SIGMA = ('Texture "sa" "spectrum" "checkerboard" "float uscale" 4 "float vscale" 4 "rgb tex1" [0.8 1.2 2.0] '
             '"rgb tex2" [3 2 1]\nMaterial "subsurface" "texture sigma_a" "sa" "rgb sigma_s" [20 16 10] "float scale" 3')


@pytest.mark.parametrize("material, const, slots", [
    (TEX_MFP, 'Material "subsurface" "rgb reflectance" [0.9 0.6 0.4] "rgb mfp" [0.03 0.03 0.02]', (1,)),
    (TEX_SIGMA, 'Material "subsurface" "rgb sigma_a" [0.8 1.2 2.0] "rgb sigma_s" [20 16 10] "float scale" 3', (0,)),
])
def test_textured_sss_spectra_oracle(pa, oracle, material, const, slots):
    """Textured sigma_a / sigma_s / mfp load into material_sss_tex, render finite, and differ
    from the constant form that equals one of the checks."""
    kw = dict(xresolution=32, yresolution=24, spp=8)
    a_sc = pa.Scene.from_string(scene(material, BLOB + BOX), SCENES, **kw)
    b_sc = pa.Scene.from_string(scene(const, BLOB + BOX), SCENES, **kw)
    f = a_sc.flat()
    st = np.ctypeslib.as_array(f.material_sss_tex, shape=(f.n_materials * 2,)).reshape(-1, 2)
    assert sorted({k for row in st for k in range(2) if row[k] >= 0}) == list(slots)
    assert not b_sc.flat().material_sss_tex
    m = [f.output_rgb_from_sensor_rgb[i] for i in range(9)]
    a = oracle.film_to_rgb(oracle.render(a_sc, threads=8), m)
    b = oracle.film_to_rgb(oracle.render(b_sc, threads=8), m)
    assert np.isfinite(a).all() and a.mean() > 0.01
    assert np.abs(a - b).mean() > 1e-4


FORMS = {
    "tex_reflectance": TEX_REFL,
    "tex_mfp": TEX_MFP,
    "tex_both": TEX_BOTH,
    "tex_sigma": TEX_SIGMA,
    "sigma": 'Material "subsurface" "rgb sigma_a" [0.8 1.2 2.0] "rgb sigma_s" [20 16 10] "float scale" 3',
    "reflectance": 'Material "subsurface" "rgb reflectance" [0.85 0.55 0.35] "rgb mfp" [0.08 0.06 0.05] "float eta" 1.45',
    "named_rough": 'Material "subsurface" "string name" "Ketchup" "float scale" 40 "float roughness" 0.25',
}


@pytest.mark.gpu
@pytest.mark.parametrize("form", list(FORMS))
def test_subsurface_matches_oracle_gpu(pa, oracle, form):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(scene(FORMS[form], BLOB + BOX), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"subsurface ({form}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_catmull_rom_gpu_equals_host(pa):
    """the spline utilities compiled for gfx950 give the host build's bits on a real BSSRDF table
    (weights over the albedos, InvertCatmullRom of rhoEff, SampleCatmullRom2D of the profile)"""
    _, _, _, _, tab = flat_sss(pa, FORMS["reflectance"])
    t = tab[0]
    rho, rad, prof = t[:100], t[100:164], t[164:164 + 6400]
    rhoEff, cdf = t[6564:6664], t[6664:6664 + 6400]
    rng = np.random.default_rng(4)
    n = 1 << 16
    x = np.concatenate([rng.uniform(0, 1, n), rng.uniform(0.3, 0.99, n)]).astype(np.float32)
    for op, args in ((0, (rho, rad, prof, cdf, x)), (1, (rho, rad, rhoEff, cdf, x)),
                     (3, (rho, rad, prof, cdf, np.stack([rng.uniform(0, 1, n), rng.uniform(0, 1, n)], 1).ravel()))):
        host = pa.catmull_rom(op, *args)
        dev = pa.catmull_rom(op, *args, device=0)
        bad = host.view(np.uint32) != dev.view(np.uint32)
        assert not bad.any(), (op, int(bad.sum()), np.nonzero(bad.reshape(len(host), -1).any(axis=1))[0][:5])


def probe_segments(n=6000, seed=12):
    """Probe-like segments: axis-aligned (the BSSRDF frames of the box's faces) and random ones
    through the blob and the box"""
    rng = np.random.default_rng(seed)
    c = rng.uniform([-0.6, -0.1, -0.6], [1.2, 1.1, 0.6], (n, 3))
    d = rng.normal(size=(n, 3))
    ax = rng.integers(0, 3, n)
    axis = np.zeros((n, 3))
    axis[np.arange(n), ax] = rng.choice([-1, 1], n)
    d[: n // 2] = axis[: n // 2]
    d /= np.linalg.norm(d, axis=1)[:, None]
    half = rng.uniform(0.05, 1.2, n)[:, None]
    c = c - EYE  # render space: world minus the eye (cameraworld)
    return np.concatenate([(c - d * half).T, (c + d * half).T]).astype(np.float32)


EYE = np.array([0, 1.4, -3.2])


def test_intersect_one_random_oracle_plausible(pa, oracle):
    sc = pa.Scene.from_string(scene(FORMS["sigma"], BLOB + BOX), SCENES)
    f = sc.flat()
    ms = np.ctypeslib.as_array(f.material_sss, shape=(f.n_materials,))
    mat = int(np.nonzero(ms >= 0)[0][0])
    segs = probe_segments(2000)
    prim, hit, pdf = oracle.intersect_one_random(sc, segs, np.full(segs.shape[1], mat, np.int32))
    assert (prim >= 0).mean() > 0.15
    assert set(np.unique(pdf[prim >= 0])) <= {1.0, 0.5, np.float32(1 / 3), 0.25, 0.2, np.float32(1 / 6)}
    assert (pdf[prim < 0] == 0).all()


@pytest.mark.gpu
def test_intersect_one_random_matches_oracle_gpu(pa, oracle):
    """pbrt_intersect_one_random (HIPAggregate::IntersectOneRandom) against the oracle's probe,
    bit for bit: the chosen primitive, its hit coordinates and the reservoir probability."""
    import torch
    sc = pa.Scene.from_string(scene(FORMS["sigma"], BLOB + BOX), SCENES)
    f = sc.flat()
    ms = np.ctypeslib.as_array(f.material_sss, shape=(f.n_materials,))
    mat = int(np.nonzero(ms >= 0)[0][0])
    segs = probe_segments()
    mats = np.full(segs.shape[1], mat, np.int32)
    mats[::7] = 0  # the ground's material: its hits are the ones sampled
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    p, h, q = agg.IntersectOneRandom(torch.from_numpy(segs).cuda(), torch.from_numpy(mats).cuda())
    p, h, q = p.cpu().numpy(), h.cpu().numpy(), q.cpu().numpy()
    po, ho, qo = oracle.intersect_one_random(sc, segs, mats)
    same = (p == po)
    print(f"IntersectOneRandom: {same.mean()*100:.3f}% same primitive, {(po >= 0).mean()*100:.1f}% with a hit")
    assert same.mean() >= 0.999
    np.testing.assert_array_equal(q[same], qo[same])
    np.testing.assert_array_equal(h[:, same & (p >= 0)], ho[:, same & (po >= 0)])
