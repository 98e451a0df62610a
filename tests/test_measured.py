"""MeasuredMaterial / MeasuredBxDF (materials.h:925-967, bxdfs.h:1154-1204, bxdfs.cpp:690-1124)
over PiecewiseLinear2D (util/sampling.h:1264-1749).  No measured data ships with the reference
or this image: the RGL tensor files are synthesised by tests/measured_bsdf.py (GGX-derived
tables, isotropic and anisotropic), so parity here is product-vs-oracle on those files,
pinned to pbrt's own invariants (Sample_f's pdf equals PDF of the sampled direction; Sample_f's
f equals f) rather than to a pbrt render ("parity unpinned" against pbrt itself).

* Loader: the material, the file cache, pbrt's errors (no filename, a bad file, phi reduction).
* Host (core/measured.h via pbrt_debug_measured) vs the oracle's own reader and restatement,
  bit for bit in libm mode: f, PDF, Sample_f.
* The invariants above; an oracle render is finite and lit.
* GPU film parity on the volumetric kernels (k_vlayered), with and without a medium."""
import numpy as np
import pytest

from measured_bsdf import make_bsdf, write_tensor


def scene_text(fn="m.bsdf", extra="", spp=8, res=32):
    return (f'LookAt 0 2 -4  0 0.6 0  0 1 0\nCamera "perspective" "float fov" 50\n'
            f'Film "rgb" "integer xresolution" {res} "integer yresolution" {res}\n'
            f'Sampler "halton" "integer pixelsamples" {spp}\nIntegrator "volpath" "integer maxdepth" 4\n'
            'WorldBegin\nLightSource "distant" "point3 from" [1 4 -2] "point3 to" [0 0 0] "blackbody L" 5500 "float scale" 3\n'
            'AttributeBegin\nAreaLightSource "diffuse" "rgb L" [2 2 2]\nTranslate 0 3 0\nShape "sphere" "float radius" 0.3\nAttributeEnd\n'
            + extra +
            'Material "diffuse" "rgb reflectance" [0.4 0.4 0.4]\n'
            'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-5 0 -5 5 0 -5 5 0 5 -5 0 5]\n'
            f'AttributeBegin\nMaterial "measured" "string filename" "{fn}"\nTranslate 0 0.7 0\nShape "sphere" "float radius" 0.7\nAttributeEnd\n'
            f'AttributeBegin\nMaterial "measured" "string filename" "{fn}"\nTranslate 1.5 0.4 0.5\nShape "sphere" "float radius" 0.4\nAttributeEnd\n')


@pytest.fixture
def bsdf(tmp_path):
    make_bsdf(tmp_path / "m.bsdf")
    make_bsdf(tmp_path / "a.bsdf", n_phi=5, alpha=0.2, tint=(0.3, 0.7, 0.9), jitter=0.2, seed=1)
    return tmp_path


def queries(n=3000, seed=0):
    rng = np.random.default_rng(seed)
    q = np.zeros((n, 8), np.float32)
    for o in (0, 3):
        d = rng.normal(size=(n, 3))
        d[:, 2] = np.abs(d[:, 2]) * np.where(rng.random(n) < 0.9, 1, -1)
        q[:, o:o + 3] = d / np.linalg.norm(d, axis=1, keepdims=True)
    q[:, 6:] = rng.random((n, 2))
    return q


LAMBDA = np.float32(395 + (705 - 395) / 31 * np.arange(31) + 3.7)


def test_measured_loader(pa, bsdf):
    sc = pa.Scene.from_string(scene_text(), bsdf)
    f = sc.flat()
    assert f.n_measured == 1  # one file, read once for both spheres
    assert f.measured_files[0].decode().endswith("m.bsdf")
    types = np.ctypeslib.as_array(f.material_type, shape=(f.n_materials,))
    assert (types == 10).sum() == 2


def test_measured_loader_errors(pa, bsdf):
    with pytest.raises(pa.PbrtError, match="Filename must be provided"):
        pa.Scene.from_string(scene_text().replace('"string filename" "m.bsdf"', ''), bsdf)
    (bsdf / "bad.bsdf").write_bytes(b"not a tensor file at all")
    with pytest.raises(pa.PbrtError, match="invalid header"):
        pa.Scene.from_string(scene_text("bad.bsdf"), bsdf)
    write_tensor(bsdf / "nofield.bsdf", {"theta_i": np.zeros(3, np.float32)})
    with pytest.raises(pa.PbrtError, match="invalid BRDF file structure"):
        pa.Scene.from_string(scene_text("nofield.bsdf"), bsdf)
    # phi_i over half the circle: reduction 2 (bxdfs.cpp:945-951)
    make_bsdf(bsdf / "half.bsdf", n_phi=5, phi_range=(0, np.pi))
    with pytest.raises(pa.PbrtError, match="reduction 2"):
        pa.Scene.from_string(scene_text("half.bsdf"), bsdf)


@pytest.mark.parametrize("fn", ["m.bsdf", "a.bsdf"])
def test_measured_host_matches_oracle(pa, oracle, bsdf, fn):
    sc = pa.Scene.from_string(scene_text(fn), bsdf)
    q = queries()
    got = sc.measured_eval(0, q, LAMBDA)
    with oracle.math_mode(oracle.MATH_LIBM):
        ref = oracle.measured_eval(bsdf / fn, q, LAMBDA)
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert np.isfinite(got).all()
    assert (got[:, :31] > 0).any() and got[:, 32].mean() > 0.5


@pytest.mark.parametrize("fn", ["m.bsdf", "a.bsdf"])
def test_measured_sampling_invariants(oracle, bsdf, fn):
    """Sample_f's pdf is PDF(wo, wi) of its own direction and its f is f(wo, wi) (the vndf
    warp's Invert undoes Sample), to float round-off, on almost every sample"""
    q = queries(4000, seed=2)
    q[:, 2] = np.abs(q[:, 2])
    out = oracle.measured_eval(bsdf / fn, q, LAMBDA)
    ok = out[:, 32] == 1
    assert ok.mean() > 0.5
    q2 = q[ok].copy()
    q2[:, 3:6] = out[ok, 33:36]
    back = oracle.measured_eval(bsdf / fn, q2, LAMBDA)
    rel_pdf = np.abs(back[:, 31] / out[ok, 36] - 1)
    rel_f = np.abs(back[:, :31] / np.maximum(out[ok, 37:], 1e-30) - 1).max(axis=1)
    assert np.median(rel_pdf) < 1e-4 and np.quantile(rel_pdf, 0.99) < 1e-2, np.quantile(rel_pdf, [0.5, 0.99])
    assert np.median(rel_f) < 1e-4 and np.quantile(rel_f, 0.99) < 1e-2, np.quantile(rel_f, [0.5, 0.99])


def test_measured_oracle_render(pa, oracle, bsdf):
    sc = pa.Scene.from_string(scene_text(res=16, spp=4), bsdf)
    film = oracle.render(sc, threads=8)
    assert np.isfinite(film).all() and film[:3].sum() > 0


FOG = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.05 0.05 0.05] "rgb sigma_s" [0.3 0.3 0.3]\n'
       'AttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\nTranslate -1.4 0.5 0\n'
       'Shape "sphere" "float radius" 0.5\nAttributeEnd\n')


@pytest.mark.gpu
@pytest.mark.parametrize("fn", ["m.bsdf", "a.bsdf"])
@pytest.mark.parametrize("medium", [False, True])
def test_measured_matches_oracle_gpu(pa, oracle, bsdf, fn, medium):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(scene_text(fn, extra=FOG if medium else "", spp=16), bsdf)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"measured {fn} (medium={medium}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")
