"""Host-side comparison of the BVH builders (pbrt_debug_bvh_trace): node visits and triangle
tests per ray for object-split and spatial-split trees, and the closest hits of both (which must
agree: the trees hold the same triangles).  Rays: uniformly random directions from points on
random triangles (secondary rays) and from random points in the scene bounds.

    python tools/bvh_explore.py c2|c3 [n_rays]
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pbrt-v4_amd"))
sys.path.insert(0, str(ROOT / "scenes"))
import pbrt_amd as pa  # noqa: E402


def load(name):
    if name == "c3":
        import gen_c3
        return pa.Scene.from_string(gen_c3.scene_text(64, 36, 1), ROOT / "scenes")
    return pa.load_scene(ROOT / "scenes" / "cornell-box.pbrt", xresolution=64, yresolution=36, spp=1)


def rays_for(sc, n, seed=1):
    f = sc.flat()
    v = np.ctypeslib.as_array(f.vertices, shape=(f.n_vertices * 3,)).reshape(-1, 3).astype(np.float64)
    t = np.ctypeslib.as_array(f.triangles, shape=(f.n_triangles * 3,)).reshape(-1, 3)
    rng = np.random.default_rng(seed)
    p0, p1, p2 = v[t[:, 0]], v[t[:, 1]], v[t[:, 2]]
    area = 0.5 * np.linalg.norm(np.cross(p1 - p0, p2 - p0), axis=1)
    k = rng.choice(len(t), size=n // 2, p=area / area.sum())
    u, w = rng.random(n // 2), rng.random(n // 2)
    su = np.sqrt(u)
    pts = (1 - su)[:, None] * p0[k] + (su * (1 - w))[:, None] * p1[k] + (su * w)[:, None] * p2[k]
    lo, hi = v.min(0), v.max(0)
    scale = np.abs(hi - lo).max()
    nrm = np.cross(p1[k] - p0[k], p2[k] - p0[k])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    d = rng.normal(size=(n // 2, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    side = np.sign((d * nrm).sum(1))[:, None]
    o1 = pts + side * nrm * 1e-4 * scale
    o2 = lo + rng.random((n - n // 2, 3)) * (hi - lo)
    d2 = rng.normal(size=(n - n // 2, 3))
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    return np.concatenate([np.hstack([o1, d]), np.hstack([o2, d2])]).astype(np.float32)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200000
    sc = load(name)
    rays = rays_for(sc, n)
    res = {}
    for sp in (0, 1):
        t, prim, st = sc.bvh_trace(rays, spatial=sp)
        res[sp] = (t, prim)
        print(f"{name} spatial={sp}: {st['node_visits'] / n:.3f} nodes/ray, {st['tri_tests'] / n:.3f} tris/ray, "
              f"{st['references']} refs, {st['nodes']} nodes")
    (t0, p0), (t1, p1) = res[0], res[1]
    print("t mismatches:", int((t0 != t1).sum()), " prim mismatches (t equal):", int(((t0 == t1) & (p0 != p1)).sum()),
          " hits:", int((t0 >= 0).sum()))


if __name__ == "__main__":
    main()
