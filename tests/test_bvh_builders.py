"""The BVH builders (csrc/host/bvh.cpp) against each other on the host: the object-split tree
(all-axes binned SAH, the default) and the spatial-split tree (PBRT_AMD_BVH_SBVH=1: a triangle
may be listed by several leaves, each through a clipped box) must return the same closest hit
for every ray, since the triangle test (shapes.cpp:172-273) is the same and only the visit order
differs.  pbrt_debug_bvh_trace walks the device's BVH8 nodes on the host with an exact slab test,
so a clipped box that lost part of its triangle would show up as a missed or farther hit."""
import numpy as np
import pytest

HEAD = ('LookAt 0 0 -5 0 0 0 0 1 0\nCamera "perspective" "float fov" 40\nSampler "halton" "integer pixelsamples" 1\n'
        'Film "rgb" "integer xresolution" 16 "integer yresolution" 16 "string filename" "x.exr"\nWorldBegin\n'
        'LightSource "point" "point3 from" [0 3 0]\nMaterial "diffuse"\n')


def slivers(n=400, seed=3):
    """Long thin triangles across a unit cube: the case spatial splits exist for."""
    rng = np.random.default_rng(seed)
    a = rng.uniform(-1, 1, (n, 3))
    b = rng.uniform(-1, 1, (n, 3))
    c = a + rng.normal(scale=0.3, size=(n, 3))
    p = np.stack([a, b, c], 1).reshape(-1, 3)
    idx = " ".join(str(i) for i in range(3 * n))
    pts = " ".join(f"{x:.6f}" for x in p.ravel())
    return HEAD + f'Shape "trianglemesh" "integer indices" [{idx}] "point3 P" [{pts}]\n'


def bounds(sc):
    """The scene's render-space bounds (the loader's vertices, camera-world space)."""
    f = sc.flat()
    v = np.ctypeslib.as_array(f.vertices, shape=(f.n_vertices * 3,)).reshape(-1, 3)
    return v.min(0), v.max(0)


def rays(sc, n, seed=5):
    rng = np.random.default_rng(seed)
    lo, hi = bounds(sc)
    o = lo + rng.uniform(-0.1, 1.1, (n, 3)) * (hi - lo)
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.hstack([o, d]).astype(np.float32)


def compare(sc, r):
    t0, p0, s0 = sc.bvh_trace(r, spatial=0)
    t1, p1, s1 = sc.bvh_trace(r, spatial=1)
    assert (t0 >= 0).sum() > len(r) // 10
    np.testing.assert_array_equal(t0, t1)
    tie = t0 == t1
    assert (p0[tie] == p1[tie]).mean() > 0.999  # equal t on two triangles may resolve either way
    return s0, s1


def test_spatial_splits_duplicate_slivers_and_keep_every_hit(pa, tmp_path):
    sc = pa.Scene.from_string(slivers(), tmp_path)
    s0, s1 = compare(sc, rays(sc, 20000))
    assert s0["references"] == 400
    assert s1["references"] > 400  # straddling slivers were split into several leaves
    assert s1["tri_tests"] < s0["tri_tests"]


def test_spatial_splits_on_cornell_box(pa):
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    sc = pa.load_scene(root / "scenes" / "cornell-box.pbrt", xresolution=16, yresolution=16, spp=1)
    compare(sc, rays(sc, 20000))


@pytest.mark.parametrize("seed", [1, 2])
def test_grazing_rays_along_split_planes(pa, tmp_path, seed):
    """Axis-aligned rays through a grid of large triangles: hits sit on bin planes."""
    rng = np.random.default_rng(seed)
    sc = pa.Scene.from_string(slivers(200, seed), tmp_path)
    n = 6000
    lo, hi = bounds(sc)
    o = lo + np.round(rng.uniform(0, 1, (n, 3)) * 32) / 32 * (hi - lo)
    axis = rng.integers(0, 3, n)
    d = np.zeros((n, 3))
    d[np.arange(n), axis] = rng.choice([-1.0, 1.0], n)
    o[np.arange(n), axis] = np.where(d[np.arange(n), axis] > 0, lo[axis] - 1, hi[axis] + 1)
    compare(sc, np.hstack([o, d]).astype(np.float32))
