"""BASELINE configs[3] geometry at full size on the GPU: the default C4 scene (scenes/gen_c4.py:
122 copied displaced icospheres from PLY files, 9,994,244 triangles), whose BVH8 (3.2 M nodes,
810 MB wide / 253 MB quantised) is HBM-resident with only the top of the tree in LDS.

* ``pbrt_intersect`` (WavefrontAggregate::IntersectClosest / IntersectShadow, the contract of
  cpu/aggregates.cpp:529-624 and shapes.cpp:172-273) against the oracle's independent binary
  BVH on 250k rays -- camera rays, rays leaving a surface point into the inside of its mesh,
  grazing rays in a triangle's plane, random rays through the scene box -- for both node
  formats.  Hit/miss must agree for every ray; hit triangle ids exactly except equal-t ties
  (two triangles sharing the hit point); t bit for bit.
* A 16-row x 16-spp image stripe vs the oracle at test_gpu_parity's tolerance.

The scene carries gen_c4's alpha-tested leaf canopy (20,000 cut-out quads, "texture alpha"), so
every candidate hit on a leaf runs the stochastic alpha test inside the full-size traversal; the
intersection classes include rays from the leaves' own triangles."""
import os

import numpy as np
import pytest

from conftest import SCENES

pytestmark = pytest.mark.gpu
LEAVES = 20000  # alpha-tested leaf quads (gen_c4 leaf canopy): the any-hit alpha test at full size


@pytest.fixture(scope="module")
def c4(tmp_path_factory, pa):
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c4
    path, n_tris = gen_c4.generate(tmp_path_factory.mktemp("c4full"), xres=1920, yres=1080, spp=16,
                                   leaves=LEAVES)
    sc = pa.load_scene(path)
    assert sc.info.n_triangles == n_tris == 9994244 + 2 * LEAVES
    # a deep tree: the traversal's LDS group stack (8 B per entry and lane) is 18 KB per block,
    # admitted beside the static LDS with a smaller node cache (capi.hip BuildDevice)
    st = sc.bvh_stats()
    assert st["max_stack"] >= 8 and st["nodes"] > 2_000_000, st
    return sc


def _context(pa, sc, fmt):
    old = os.environ.get("PBRT_AMD_BVH")
    os.environ["PBRT_AMD_BVH"] = fmt
    try:
        return pa.WavefrontPathIntegrator(sc, max_paths=1 << 16)
    finally:
        if old is None:
            del os.environ["PBRT_AMD_BVH"]
        else:
            os.environ["PBRT_AMD_BVH"] = old


def _rays(sc, n_each=62500, seed=3):
    """[7, 4 * n_each] float32 rays (o, d, tMax) in render space."""
    rng = np.random.default_rng(seed)
    f = sc.flat()
    i = sc.info
    V = np.ctypeslib.as_array(f.vertices, shape=(f.n_vertices * 3,)).reshape(-1, 3).astype(np.float64)
    T = np.ctypeslib.as_array(f.triangles, shape=(f.n_triangles * 3,)).reshape(-1, 3)
    out = []
    # camera rays: raster points -> camera space (PerspectiveCamera::GenerateRay, cameras.cpp:433-456)
    cfr = np.array(list(f.camera_from_raster), np.float64).reshape(4, 4)
    rfc = np.array(list(f.render_from_camera), np.float64).reshape(4, 4)
    pr = np.stack([rng.uniform(0, i.xres, n_each), rng.uniform(0, i.yres, n_each), np.zeros(n_each),
                   np.ones(n_each)])
    pc = cfr @ pr
    dc = pc[:3] / pc[3]
    dc /= np.linalg.norm(dc, axis=0)
    d = rfc[:3, :3] @ dc
    o = np.repeat(rfc[:3, 3:4], n_each, axis=1)
    out.append(np.concatenate([o, d, np.full((1, n_each), np.inf)]))
    # from just inside a random triangle of a copy (below its centroid, against the outward
    # normal) in random directions: hits on the inner side of the same closed mesh
    t = rng.integers(4, len(T), n_each)  # skip the light's and the ground's quads
    p0, p1, p2 = V[T[t, 0]], V[T[t, 1]], V[T[t, 2]]
    c = (p0 + p1 + p2) / 3
    nrm = np.cross(p1 - p0, p2 - p0)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    o = c - 1e-3 * nrm
    d = rng.normal(size=(n_each, 3))
    out.append(np.concatenate([o.T, d.T, np.full((1, n_each), np.inf)]))
    # grazing: in the plane of a triangle, aimed across it with a tiny normal component
    t = rng.integers(4, len(T), n_each)
    p0, p1, p2 = V[T[t, 0]], V[T[t, 1]], V[T[t, 2]]
    c = (p0 + p1 + p2) / 3
    nrm = np.cross(p1 - p0, p2 - p0)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    e = p1 - p0
    o = c - 3 * e
    d = e + nrm * rng.uniform(-1e-4, 1e-4, (n_each, 1)) * np.linalg.norm(e, axis=1, keepdims=True)
    out.append(np.concatenate([o.T, d.T, np.full((1, n_each), np.inf)]))
    # random rays in the scene's box, some with a finite tMax (shadow-ray style)
    lo, hi = V[8:].min(axis=0), V[8:].max(axis=0)
    o = rng.uniform(lo, hi, (n_each, 3))
    d = rng.normal(size=(n_each, 3))
    tmax = np.where(rng.uniform(size=n_each) < 0.4, rng.uniform(0.05, 5, n_each), np.inf)
    out.append(np.concatenate([o.T, d.T, tmax[None]]))
    return np.ascontiguousarray(np.concatenate(out, axis=1), dtype=np.float32)


@pytest.fixture(scope="module")
def c4_rays(c4, oracle):
    rays = _rays(c4)
    closest = oracle.intersect(c4, rays, False)
    anyhit = oracle.intersect(c4, rays, True)
    return rays, closest, anyhit


@pytest.mark.parametrize("fmt", ["wide", "compressed"])
def test_c4_full_intersections_match_oracle(pa, c4, c4_rays, fmt):
    import torch
    rays, (op, oh), (ap, _) = c4_rays
    n = rays.shape[1]
    assert n >= 200000
    integ = _context(pa, c4, fmt)
    agg = pa.HIPAggregate(integ)
    dev = torch.from_numpy(rays).cuda()
    gp, gh = (x.cpu().numpy() for x in agg.IntersectClosest(dev))
    np.testing.assert_array_equal(gp >= 0, op >= 0)
    hit = op >= 0
    assert hit.mean() > 0.5
    for k in range(4):  # every ray class hits something
        assert hit[k * n // 4:(k + 1) * n // 4].mean() > 0.2
    same = gp[hit] == op[hit]
    tie = ~same & (gh[3][hit] == oh[3][hit])
    assert (same | tie).all(), np.flatnonzero(hit)[~(same | tie)][:10]
    assert same.mean() > 0.999
    np.testing.assert_array_equal(gh[3][hit], oh[3][hit])
    np.testing.assert_array_equal(gh[:3, hit][:, same], oh[:3, hit][:, same])
    # any hit: occlusion agrees for every ray; the reported triangle is a real hit
    sp, _ = (x.cpu().numpy() for x in agg.IntersectShadow(dev))
    np.testing.assert_array_equal(sp >= 0, ap >= 0)
    np.testing.assert_array_equal(sp >= 0, op >= 0)
    print(f"C4 full ({fmt}): {n} rays, {hit.mean()*100:.1f}% hit, {(~same).sum()} equal-t ties")


def test_c4_full_image_stripe_matches_oracle(pa, oracle, c4):
    """16 rows x 16 spp of the full C4 scene, canopy included, at test_gpu_parity's per-pixel
    bar: the canopy's alpha tests hash ray bits, which the device's portable transcendentals keep
    identical to the oracle's (test_gpu_parity.oracle_film)."""
    from test_gpu_parity import check_parity, oracle_film, to_rgb
    rows = np.arange(16, dtype=np.int32) * 67 + 20  # 16 rows spread over the 1080
    integ = _context(pa, c4, "wide")
    integ.render(rows=rows, first_sample=0, n_samples=16)
    integ.synchronize()
    gpu = integ.film_raw()
    ref = oracle_film(oracle, c4, integ, rows=rows, first_sample=0, n_samples=16)
    a, b = to_rgb(oracle, c4, gpu)[rows], to_rgb(oracle, c4, ref)[rows]
    assert np.isfinite(a).all()
    frac, mean_rel = check_parity(a, b)
    print(f"C4 full stripe (16 rows x 16 spp): {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
