"""GPU parity through the C ABI: the MI355X wavefront path vs the CPU oracle on the same
scene, sampler and seed.

Tolerance (north star: "per-channel float tolerance"): per-pixel output RGB
within 1e-3 relative (abs floor 1e-4) on >= 99.5 % of pixels, image mean within 1e-4
relative.  The oracle runs in its libm mode -- glibc's float transcendentals, the reference CPU
build's arithmetic (conftest) -- and the device's core/detmath.h returns glibc's bits for every
input, so GPU paths follow the reference's decisions; what remains are exact-t closest-hit ties
resolved in a different BVH order and film-only reciprocal roundings (Numerics).
C1 (full), C2 (rows 300-315, 8 spp) and C3 (192x108, 16 spp) below are the north star's
"match the reference CPU VolPathIntegrator" checks at that bar.
Integer results (closest-hit primitive ids) must match exactly except documented
exact-t ties."""
import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu

REL, ABS_FLOOR, FRAC_OK, MEAN_REL = 1e-3, 1e-4, 0.995, 1e-4


def gpu_film(pa, sc, rows=None, first=0, n=None, max_paths=1 << 20):
    integ = pa.WavefrontPathIntegrator(sc, max_paths=max_paths)
    integ.render(rows=rows, first_sample=first, n_samples=n)
    integ.synchronize()
    return integ.film_raw(), integ


def to_rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def oracle_film(oracle, sc, integ=None, **kw):
    """The oracle's film of the scene, rendered with libm's float transcendentals (the reference's
    arithmetic, which the kernels' core/detmath.h reproduces bit for bit), so every path decision
    -- alpha tests and mix choices that hash a ray, the medium RNG seeded from one -- is the same."""
    kw.setdefault("threads", 16)
    with oracle.math_mode(oracle.MATH_LIBM):
        return oracle.render(sc, **kw)


def check_parity(a, b):
    d = np.abs(a - b)
    ok = d <= np.maximum(REL * np.abs(b), ABS_FLOOR)
    frac = ok.all(axis=-1).mean()
    mean_rel = np.abs(a.mean(axis=(0, 1)) / b.mean(axis=(0, 1)) - 1).max()
    assert frac >= FRAC_OK, frac
    assert mean_rel <= MEAN_REL, mean_rel
    return frac, mean_rel


def test_cornell_c1_matches_oracle(pa, oracle):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")  # C1: 256x256, 16 spp, maxdepth 5
    film, _ = gpu_film(pa, sc)
    ref = oracle_film(oracle, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"C1 parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.parametrize("randomization", ["fastowen", "owen"])
def test_cornell_zsobol_matches_oracle(pa, oracle, randomization):
    """pbrt's default sampler (ZSobolSampler, fork default scene.cpp:93) end to end."""
    from conftest import cornell_with_sampler
    line = f'Sampler "zsobol" "integer pixelsamples" [ 16 ] "string randomization" "{randomization}"'
    sc = cornell_with_sampler(pa, line, xresolution=160, yresolution=120)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"ZSobol ({randomization}) parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_cornell_c2_rows_match_oracle(pa, oracle):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64)
    rows = np.arange(300, 316, dtype=np.int32)
    film, _ = gpu_film(pa, sc, rows=rows, first=0, n=8)
    ref = oracle_film(oracle, sc, rows=rows, first_sample=0, n_samples=8)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film)[300:316], to_rgb(oracle, sc, ref)[300:316])
    print(f"C2 rows 300-315 x 8 spp parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_furnace_known_answer_gpu(pa, oracle):
    sc = pa.load_scene(SCENES / "furnace.pbrt")
    film, _ = gpu_film(pa, sc)
    img = to_rgb(oracle, sc, film)
    assert abs(img.mean() - 1.0) < 0.025, img.mean()
    check_parity(img, to_rgb(oracle, sc, oracle.render(sc, threads=16)))


def _c3(pa, xres=192, yres=108, spp=16, sampler="zsobol", regularize=False):
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c3
    text = gen_c3.scene_text(xres, yres, spp, sampler=sampler)
    if regularize:
        text = text.replace('"integer maxdepth" [ 5 ]', '"integer maxdepth" [ 5 ] "bool regularize" true')
    return pa.Scene.from_string(text, SCENES)


@pytest.mark.parametrize("sampler", ["zsobol", "halton"])
def test_c3_dielectric_conductor_matches_oracle(pa, oracle, sampler):
    """C3: specular dielectric shell + rough conductor floor + diffuse backdrop, 30k triangles."""
    sc = _c3(pa, sampler=sampler)
    film, integ = gpu_film(pa, sc)
    counts = integ.queue_counts()
    ref = oracle_film(oracle, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"C3 ({sampler}) parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
    # every material queue saw work (per-type queues of EvaluateMaterialsAndBSDFs)
    assert counts[0][1] > 0 and counts[0][5] > 0 and counts[0][6] > 0, counts[:2]


def test_c3_regularize_matches_oracle(pa, oracle):
    sc = _c3(pa, 128, 72, 8, regularize=True)
    film, _ = gpu_film(pa, sc)
    check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))


@pytest.mark.parametrize("skies", [1, 2, 0], ids=["one-sky", "two-skies", "distant-only"])
def test_c3_escaped_rays_match_oracle(pa, oracle, skies):
    """HandleEscapedRays (integrator.cpp:495-537) in both k_escaped forms: one infinite light
    with Le (sky spectrum and sensor curves staged in LDS), two (the general loop, per-light
    sums in pbrt's order) and a distant light alone in the infinite list (no Le: escaped rays
    add nothing)."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c3
    text = gen_c3.scene_text(96, 54, 8)
    assert text.count('LightSource "infinite"') == 1
    if skies == 2:
        text = text.replace("WorldBegin", 'WorldBegin\nLightSource "infinite" "rgb L" [ 0.3 0.2 0.1 ] "float scale" 0.7\n', 1)
    elif skies == 0:
        text = "\n".join(l for l in text.splitlines() if not l.lstrip().startswith('LightSource "infinite"'))
        text = text.replace("WorldBegin", 'WorldBegin\nLightSource "distant" "rgb L" [ 1 1 1 ] "point3 from" [ 1 2 -1 ] '
                            '"point3 to" [ 0 0 0 ]\n', 1)
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    assert f.n_infinite_lights == (skies if skies else 1)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"C3 escaped rays ({skies} skies): {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_c4_named_metals_match_oracle(pa, oracle, tmp_path):
    """C4's generator at a small size: rough conductors with pbrt's named metal spectra (56-knot
    piecewise-linear eta / k, walked knot by knot over each path's wavelengths) beside diffuse
    copies, PLY meshes, area light and sky."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c4
    path, _ = gen_c4.generate(tmp_path, copies=12, level=3, xres=96, yres=54, spp=8)
    sc = pa.load_scene(path)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"C4 small (named metals): {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_index_matched_glass_invisible_gpu(pa, oracle):
    import sys
    sys.path.insert(0, str(SCENES.parent / "tests"))
    from test_c3 import furnace_glass_text
    sc = pa.Scene.from_string(furnace_glass_text(1.0, 0.0), SCENES)
    empty = pa.Scene.from_string(furnace_glass_text(1.0, 0.0, sphere=False), SCENES)
    img = to_rgb(oracle, sc, gpu_film(pa, sc)[0])
    sky = to_rgb(oracle, empty, gpu_film(pa, empty)[0])
    np.testing.assert_allclose(img, sky, rtol=1e-5)


@pytest.mark.parametrize("sampler", ["zsobol", "halton"])
def test_vertex_normals_and_uv_match_oracle(pa, oracle, sampler):
    """Smooth-shaded conductor sphere with uv, an area light with vertex normals, uv floor."""
    import sys
    sys.path.insert(0, str(SCENES.parent / "tests"))
    from test_shading_ply import smooth_sphere_text
    sc = pa.Scene.from_string(smooth_sphere_text(res=96, spp=16, sampler=sampler), SCENES)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"vertex normals/uv ({sampler}) parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_c4_small_variant_matches_oracle(pa, oracle, tmp_path):
    """C4's construction (PLY copies, named-metal conductors, 124 materials) at 1/1000 size."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c4
    path, _ = gen_c4.generate(tmp_path, copies=12, level=3, xres=160, yres=90, spp=8)
    sc = pa.load_scene(path)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"C4 small parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.parametrize("scene", ["c4", "cornell", "mix"])
def test_ray_binning_leaves_films_bit_identical(pa, monkeypatch, tmp_path, scene):
    """Closest hits of depth >= 1 traced in ray-bin order (origin cell x direction octant, then
    k_classify enqueues in record order) against record order: every path's arithmetic is the
    same, so the films must match bit for bit -- C4's HBM-resident tree (binning by default),
    Cornell's LDS tree and a mix-material scene (binning forced)."""
    import sys
    if scene == "c4":
        sys.path.insert(0, str(SCENES))
        import gen_c4
        path, _ = gen_c4.generate(tmp_path, copies=12, level=3, xres=160, yres=90, spp=8)
        load = lambda: pa.load_scene(path)
    elif scene == "cornell":
        load = lambda: pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=96, yresolution=64, spp=8)
    else:
        sys.path.insert(0, str(SCENES.parent / "tests"))
        from test_mix import MIXED
        load = lambda: pa.Scene.from_string(MIXED, SCENES)
    films = []
    for on in ("0", "1"):
        monkeypatch.setenv("PBRT_AMD_RAY_SORT", on)
        film, integ = gpu_film(pa, load())
        films.append(film)
        del integ
    assert np.abs(films[0]).sum() > 0
    assert np.array_equal(films[0], films[1])


@pytest.mark.parametrize("fmt", ["wide", "compressed"])
def test_bvh_node_formats_match_oracle(pa, oracle, monkeypatch, fmt):
    """Both BVH8 node formats (256-B wide, 80-B quantised) on C3 geometry: the quantised boxes
    are conservative, so closest hits -- and the image -- must not change."""
    monkeypatch.setenv("PBRT_AMD_BVH", fmt)
    sc = _c3(pa, 128, 72, 8)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"BVH {fmt} parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_compressed_bvh_intersections_match_oracle(pa, oracle, monkeypatch):
    import torch
    monkeypatch.setenv("PBRT_AMD_BVH", "compressed")
    sc = _c3(pa, 64, 36, 4)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    rng = np.random.default_rng(11)
    n = 50000
    o = rng.uniform([-3, 0.2, -3], [3, 3, 3], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    o = o - np.array([0, 1.7, -5.2], np.float32)  # world -> render space ("cameraworld": minus the eye)
    rays = np.concatenate([o.T, d.T, np.full((1, n), np.inf, np.float32)]).astype(np.float32)
    gp, gh = agg.IntersectClosest(torch.from_numpy(rays).cuda())
    gp, gh = gp.cpu().numpy(), gh.cpu().numpy()
    op, oh = oracle.intersect(sc, rays)
    np.testing.assert_array_equal(gp >= 0, op >= 0)
    hit = op >= 0
    assert hit.sum() > n // 4
    same = gp[hit] == op[hit]
    tie = ~same & (gh[3][hit] == oh[3][hit])
    assert (same | tie).all()
    np.testing.assert_array_equal(gh[3][hit], oh[3][hit])


def test_sample_splits_bit_exact(pa):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=64, yresolution=48, spp=8)
    full, _ = gpu_film(pa, sc)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)  # forces several passes
    integ.render(first_sample=0, n_samples=3)
    integ.render(first_sample=3, n_samples=5)
    integ.synchronize()
    np.testing.assert_array_equal(integ.film_raw(), full)


def test_row_stripes_bit_exact(pa):
    from pbrt_amd.tiles import rows_for_rank
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=96, yresolution=80, spp=4)
    full, _ = gpu_film(pa, sc)
    parts = [gpu_film(pa, sc, rows=rows_for_rank(0, 80, r, 3, block=16))[0] for r in range(3)]
    np.testing.assert_array_equal(parts[0] + parts[1] + parts[2], full)


def test_intersect_closest_and_shadow_match_oracle(pa, oracle):
    import torch
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    rng = np.random.default_rng(7)
    n = 20000
    o = rng.uniform([-50, -50, -50], [600, 600, 600], size=(n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    tmax = np.where(rng.uniform(size=n) < 0.3, rng.uniform(1, 800, size=n), np.inf).astype(np.float32)
    # express in render space (cameraworld): subtract the camera position
    f = sc.flat()
    m = np.array(list(f.render_from_camera), np.float32).reshape(4, 4)
    o = o + m[:3, 3]
    rays = np.concatenate([o.T, d.T, tmax[None]], axis=0).astype(np.float32)
    for any_hit in (False, True):
        gp, gh = agg.IntersectShadow(torch.from_numpy(rays).cuda()) if any_hit else agg.IntersectClosest(
            torch.from_numpy(rays).cuda())
        gp, gh = gp.cpu().numpy(), gh.cpu().numpy()
        op, oh = oracle.intersect(sc, rays, any_hit)
        np.testing.assert_array_equal(gp >= 0, op >= 0)
        if not any_hit:
            hit = op >= 0
            same = gp[hit] == op[hit]
            # exact-t ties between coplanar triangles of one quad may pick either triangle
            tie = ~same & (gh[3][hit] == oh[3][hit])
            assert (same | tie).all()
            np.testing.assert_array_equal(gh[3][hit], oh[3][hit])
            np.testing.assert_array_equal(gh[:3, hit][:, same], oh[:3, hit][:, same])


@pytest.mark.parametrize("line", ['PixelFilter "gaussian"', 'PixelFilter "mitchell" "float xradius" [ 1.5 ]',
                                  'PixelFilter "triangle"', 'PixelFilter "sinc" "float xradius" [ 2 ] "float yradius" [ 2 ]'])
def test_pixel_filters_match_oracle(pa, oracle, line):
    """Filter::Sample offsets and weights (FilterSampler tables on the device) end to end."""
    from test_filters import scene_with_filter
    sc = scene_with_filter(pa, line)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    np.testing.assert_array_equal(film[3], ref[3])  # the filter weight sums are the same floats summed
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"{line}: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


def test_instanced_scene_matches_oracle(pa, oracle):
    """ObjectBegin / ObjectInstance scenes render through the flattened triangle list."""
    from test_instancing import HEAD, TRI
    text = HEAD + f"""
ObjectBegin "thing"
  Material "diffuse" "rgb reflectance" [ 0.7 0.5 0.3 ]
  {TRI}
ObjectEnd
AttributeBegin Translate -0.5 -0.5 0  ObjectInstance "thing" AttributeEnd
AttributeBegin Translate 0.2 0 -0.3  Rotate 60 0 1 0  ObjectInstance "thing" AttributeEnd
"""
    sc = pa.Scene.from_string(text, SCENES, xresolution=96, yresolution=96, spp=8)
    film, _ = gpu_film(pa, sc)
    check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))


def test_full_c2_size_split_invariance_and_mean(pa, oracle):
    """BASELINE configs[1] at full size (1280x720, 64 spp, maxdepth 5) through size-independent
    properties: the film is bit-identical when the same samples are rendered as two sample
    ranges or as interleaved row sets (every path depends only on its pixel, sample index and
    dimension, so any split must sum to the same floats), and the image mean agrees with the
    oracle's 1-spp render of every pixel within its statistical error."""
    from pbrt_amd.tiles import rows_for_rank
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=64)
    full, integ = gpu_film(pa, sc, max_paths=0)
    assert np.isfinite(full).all()
    integ.film_clear()
    integ.render(first_sample=0, n_samples=24)
    integ.render(first_sample=24, n_samples=40)
    integ.synchronize()
    np.testing.assert_array_equal(integ.film_raw(), full)
    integ.film_clear()
    for r in range(4):
        integ.render(rows=rows_for_rank(0, 720, r, 4, block=1))
    integ.synchronize()
    np.testing.assert_array_equal(integ.film_raw(), full)
    # mean radiance vs the oracle at 1 spp (921,600 independent samples)
    sc1 = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=1280, yresolution=720, spp=1)
    ref = to_rgb(oracle, sc1, oracle.render(sc1, threads=16))
    gpu = to_rgb(oracle, sc, full)
    m_ref, m_gpu = ref.mean(axis=(0, 1)), gpu.mean(axis=(0, 1))
    sigma = ref.std(axis=(0, 1)) / np.sqrt(ref.shape[0] * ref.shape[1])
    assert (np.abs(m_gpu - m_ref) <= 5 * sigma + 1e-6).all(), (m_gpu, m_ref, sigma)
