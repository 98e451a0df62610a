"""Shape "plymesh" with "texture displacement" (shapes.cpp:1418-1458): TriQuadMesh::Displace
(util/mesh.h:91-191) -- quads to triangles, vertex normals when the file has none, edge
bisection until every edge is shorter than "edgelength" in render space, p += d n with the
texture evaluated at each vertex's object-space position and uv, normals recomputed.

The refinement and displacement (host/displace.cpp) are pinned bit-exact against the reference's
own TriQuadMesh::Displace run by oracle/ref/refgold.cpp with closed-form displacements
("displace" goldens); the loader path is checked against the same routine, and on the GPU the
displaced mesh renders as the oracle renders it."""
import numpy as np
import pytest

from conftest import fl
from test_shading_ply import write_ply


def test_displace_matches_reference(pa, golden):
    cases = golden["displace"]
    assert len(cases) == 3
    for c in cases:
        P, N, uv, tri = pa.debug_displace(fl(c["P"]), fl(c["uv"]), fl(c["N"]) or None, c["tri"], c["quad"], fl(c["m"]),
                                          c["edge"], c["mode"])
        o = c["out"]
        np.testing.assert_array_equal(tri.ravel(), np.asarray(o["tri"], np.int32))
        np.testing.assert_array_equal(P.ravel(), np.asarray(fl(o["P"]), np.float32))
        np.testing.assert_array_equal(N.ravel(), np.asarray(fl(o["N"]), np.float32))
        np.testing.assert_array_equal(uv.ravel(), np.asarray(fl(o["uv"]), np.float32))
        assert len(tri) > len(c["tri"]) // 3 + len(c["quad"]) // 2  # refined


GRID_N = 4
GRID_P = [[x / GRID_N * 2 - 1, y / GRID_N * 2 - 1, 0.1 * np.sin(x + y)] for y in range(GRID_N + 1) for x in range(GRID_N + 1)]
GRID_UV = [[x / GRID_N, y / GRID_N] for y in range(GRID_N + 1) for x in range(GRID_N + 1)]
GRID_F = []
for _y in range(GRID_N):
    for _x in range(GRID_N):
        _a = _y * (GRID_N + 1) + _x
        GRID_F += [[_a, _a + 1, _a + GRID_N + 2], [_a, _a + GRID_N + 2, _a + GRID_N + 1]]


def scene(pa, tmp_path, shape, tex='Texture "d" "float" "constant" "float value" 0.1\n', spp=4, res=16):
    text = f"""LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" [ 40 ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "zsobol" "integer pixelsamples" [ {spp} ]
WorldBegin
LightSource "infinite" "rgb L" [ 1 1 1 ]
{tex}Material "diffuse" "rgb reflectance" [ 0.5 0.4 0.3 ]
{shape}
"""
    return pa.Scene.from_string(text, tmp_path)


def flat(sc):
    f = sc.flat()
    nv, nt = sc.info.n_vertices, sc.info.n_triangles
    v = np.ctypeslib.as_array(f.vertices, shape=(nv * 3,)).reshape(-1, 3).copy()
    t = np.ctypeslib.as_array(f.triangles, shape=(nt * 3,)).reshape(-1, 3).copy()
    n = np.ctypeslib.as_array(f.vertex_normals, shape=(nv * 3,)).reshape(-1, 3).copy()
    return v, t, n


def test_loader_displaces_plymesh(pa, tmp_path):
    write_ply(tmp_path / "m.ply", GRID_P, GRID_F, UV=GRID_UV)
    base = flat(scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply"'))
    v, t, n = flat(scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "d" '
                                        '"float edgelength" 0.3'))
    # the same refinement and a constant d = 0.1 through the pinned routine (identity object
    # transform; render space is camera-world, a translation, which leaves the edge lengths)
    P, N, uv, tri = pa.debug_displace(np.ravel(GRID_P), np.ravel(GRID_UV), None, np.ravel(GRID_F), [], np.eye(4), 0.3, 2)
    assert len(t) == len(tri) > 4 * len(base[1])
    np.testing.assert_array_equal(t, tri)
    shift = base[0][0] - np.asarray(GRID_P[0], np.float32)  # camera-world offset
    np.testing.assert_allclose(v - shift, P, atol=2e-6)
    np.testing.assert_allclose(n, N, atol=1e-6)  # recomputed vertex normals become shading normals


def test_displacement_needs_uv(pa, tmp_path):
    write_ply(tmp_path / "m.ply", GRID_P, GRID_F)
    with pytest.raises(pa.PbrtError, match="uvs are currently required"):
        scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "d"')


def test_displacement_texture_must_exist(pa, tmp_path):
    write_ply(tmp_path / "m.ply", GRID_P, GRID_F, UV=GRID_UV)
    with pytest.raises(pa.PbrtError):
        scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "nope"')


def test_quads_are_split_and_displaced(pa, tmp_path):
    quads = [[0, 1, 6, 5], [1, 2, 7, 6]]  # p00 p10 p11 p01 face order in the PLY
    write_ply(tmp_path / "m.ply", GRID_P, quads, UV=GRID_UV)
    v, t, n = flat(scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "d" '
                                        '"float edgelength" 10'))
    assert len(t) == 4  # two quads -> four triangles, no patches left


@pytest.mark.gpu
def test_displaced_plymesh_matches_oracle_gpu(pa, oracle, tmp_path):
    from test_gpu_media import check, gpu_rgb, oracle_rgb

    write_ply(tmp_path / "m.ply", GRID_P, GRID_F, UV=GRID_UV)
    tex = 'Texture "d" "float" "checkerboard" "float uscale" 4 "float vscale" 4 "float tex1" 0 "float tex2" 0.15\n'
    sc = scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "d" "float edgelength" 0.1',
               tex=tex, spp=8, res=48)
    assert sc.info.n_triangles > 500
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"displaced plymesh parity: {frac * 100:.3f}% pixels, mean rel {mr:.2e}")


def test_instanced_displaced_plymesh(pa, tmp_path):
    """A displaced plymesh inside ObjectBegin is refined once and each instance copies it."""
    write_ply(tmp_path / "m.ply", GRID_P, GRID_F, UV=GRID_UV)
    one = flat(scene(pa, tmp_path, 'Shape "plymesh" "string filename" "m.ply" "texture displacement" "d" '
                                    '"float edgelength" 0.3'))
    inst = ('ObjectBegin "g"\nShape "plymesh" "string filename" "m.ply" "texture displacement" "d" "float edgelength" 0.3\n'
            'ObjectEnd\nObjectInstance "g"\nAttributeBegin\nTranslate 3 0 0\nObjectInstance "g"\nAttributeEnd\n')
    v, t, n = flat(scene(pa, tmp_path, inst))
    nt, nv = len(one[1]), len(one[0])
    assert len(t) == 2 * nt and len(v) == 2 * nv
    np.testing.assert_array_equal(v[:nv], one[0])
    np.testing.assert_allclose(v[nv:] - v[:nv], np.tile([3, 0, 0], (nv, 1)), atol=1e-5)
