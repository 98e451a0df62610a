"""Vertex normals / uv (Triangle::InteractionFromIntersection shading geometry, Triangle::Sample
normal, shapes.h:884-1046) against the reference's own outputs, and Shape "plymesh"
(TriQuadMesh::ReadPLY, util/mesh.cpp:322-420) through the loader."""
import struct

import numpy as np
import pytest

from conftest import SCENES, fl


def same(a, b):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    return bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def _args(e):
    n = fl(e["n"]) or None
    uv = fl(e["uv"]) or None
    return fl(e["p"]), n, uv, int(e["flip"]), fl(e["b"]), fl(e["u"])


def test_shading_geometry_matches_reference(pa, oracle, golden):
    cases = golden["shading_triangles"]
    assert len(cases) == 300
    n_flipped = 0
    for e in cases:
        want = np.asarray(fl(e["out"]), np.float32)
        got_o = oracle.triangle_shading(*_args(e))
        got_p = pa.debug_triangle_shading(*_args(e))
        assert same(got_o, want), (e, got_o, want)
        assert same(got_p, want), (e, got_p, want)
        geo = np.cross(np.subtract(e["p"][0:3], e["p"][6:9]), np.subtract(e["p"][3:6], e["p"][6:9]))
        n_flipped += np.dot(geo, want[:3]) < 0
    assert n_flipped > 20  # FaceForward toward the shading normal happens


# ------------------------------------------------------------------ PLY
def write_ply(path, P, F, N=None, UV=None, fmt="binary_little_endian", extra_face=None):
    P = np.asarray(P, np.float32)
    F = [list(f) for f in F] + (extra_face or [])
    props = ["x", "y", "z"] + (["nx", "ny", "nz"] if N is not None else []) + (["u", "v"] if UV is not None else [])
    head = ["ply", f"format {fmt} 1.0", "comment pbrt-v4_amd test", f"element vertex {len(P)}"]
    head += [f"property float {p}" for p in props]
    head += [f"element face {len(F)}", "property list uchar int vertex_indices", "end_header"]
    cols = [P] + ([np.asarray(N, np.float32)] if N is not None else []) + ([np.asarray(UV, np.float32)] if UV is not None else [])
    V = np.concatenate(cols, axis=1)
    with open(path, "wb") as f:
        f.write(("\n".join(head) + "\n").encode())
        if fmt == "ascii":
            for row in V:
                f.write((" ".join(repr(float(x)) for x in row) + "\n").encode())
            for face in F:
                f.write((" ".join(map(str, [len(face)] + face)) + "\n").encode())
        else:
            e = "<" if fmt == "binary_little_endian" else ">"
            for row in V:
                f.write(struct.pack(e + "f" * len(row), *row))
            for face in F:
                f.write(struct.pack(e + "B" + "i" * len(face), len(face), *face))


def _scene(pa, shape_line, tmp_path):
    text = f"""LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" [ 40 ]
Film "rgb" "integer xresolution" [ 16 ] "integer yresolution" [ 16 ]
Sampler "zsobol" "integer pixelsamples" [ 4 ]
WorldBegin
LightSource "infinite" "rgb L" [ 1 1 1 ]
Translate 0.25 0 0
{shape_line}
"""
    return pa.Scene.from_string(text, tmp_path)


MESH_P = [[-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0], [0, 0, 1]]
MESH_F = [[0, 1, 2], [0, 2, 3], [0, 1, 4]]
MESH_N = [[0, 0, -1], [0.1, 0, -1], [0, 0.2, -1], [0, 0, -1], [0.3, 0.3, -0.5]]
MESH_UV = [[0, 0], [1, 0], [1, 1], [0, 1], [0.5, 0.5]]


def _flat_arrays(sc):
    f = sc.flat()
    nv, nt = sc.info.n_vertices, sc.info.n_triangles
    verts = np.ctypeslib.as_array(f.vertices, shape=(nv * 3,)).copy()
    tris = np.ctypeslib.as_array(f.triangles, shape=(nt * 3,)).copy()
    normals = np.ctypeslib.as_array(f.vertex_normals, shape=(nv * 3,)).copy() if f.vertex_normals else None
    uv = np.ctypeslib.as_array(f.vertex_uv, shape=(nv * 2,)).copy() if f.vertex_uv else None
    shade = np.ctypeslib.as_array(f.tri_shading, shape=(nt,)).copy()
    return verts, tris, normals, uv, shade


def _trianglemesh_line(with_n=True, with_uv=True):
    s = 'Shape "trianglemesh" "integer indices" [ ' + " ".join(str(i) for f in MESH_F for i in f) + ' ]'
    s += ' "point3 P" [ ' + " ".join(repr(float(x)) for p in MESH_P for x in p) + ' ]'
    if with_n:
        s += ' "normal N" [ ' + " ".join(repr(float(x)) for n in MESH_N for x in n) + ' ]'
    if with_uv:
        s += ' "point2 uv" [ ' + " ".join(repr(float(x)) for t in MESH_UV for x in t) + ' ]'
    return s


@pytest.mark.parametrize("fmt", ["binary_little_endian", "binary_big_endian", "ascii"])
def test_plymesh_equals_trianglemesh(pa, tmp_path, fmt):
    write_ply(tmp_path / "m.ply", MESH_P, MESH_F, MESH_N, MESH_UV, fmt=fmt)
    a = _flat_arrays(_scene(pa, 'Shape "plymesh" "string filename" "m.ply"', tmp_path))
    b = _flat_arrays(_scene(pa, _trianglemesh_line(), tmp_path))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert list(a[4]) == [3, 3, 3]
    # normals are transformed to render space and kept unnormalised (TriangleMesh ctor)
    assert not np.allclose(np.linalg.norm(a[2].reshape(-1, 3), axis=1), 1)


def test_plymesh_without_attributes(pa, tmp_path):
    write_ply(tmp_path / "m.ply", MESH_P, MESH_F)
    verts, tris, normals, uv, shade = _flat_arrays(_scene(pa, 'Shape "plymesh" "string filename" "m.ply"', tmp_path))
    assert normals is None and uv is None and list(shade) == [0, 0, 0]


def test_reverse_orientation_negates_normals(pa, tmp_path):
    a = _flat_arrays(_scene(pa, _trianglemesh_line(), tmp_path))[2]
    b = _flat_arrays(_scene(pa, "ReverseOrientation\n" + _trianglemesh_line(), tmp_path))[2]
    np.testing.assert_array_equal(a, -b)


@pytest.mark.parametrize("kind,msg", [
    ("missing", "Couldn't open PLY file"),
    ("badindex", "out of bounds"),
])
def test_plymesh_errors_are_loud(pa, tmp_path, kind, msg):
    if kind == "badindex":
        write_ply(tmp_path / "m.ply", MESH_P, MESH_F + [[0, 1, 9]])
    with pytest.raises(pa.PbrtError, match=msg):
        _scene(pa, 'Shape "plymesh" "string filename" "m.ply"', tmp_path)


def test_plymesh_quad_becomes_a_patch(pa, tmp_path):
    """A quad face loads as a bilinear patch beside the TriangleMesh (tests/test_bilinear.py)."""
    write_ply(tmp_path / "m.ply", MESH_P, MESH_F, extra_face=[[0, 1, 2, 3]])
    sc = _scene(pa, 'Shape "plymesh" "string filename" "m.ply"', tmp_path)
    assert (sc.info.n_triangles, sc.flat().n_shapes) == (3, 1)


def test_plymesh_skips_polygons(pa, tmp_path):
    """rply_face_callback ignores faces that are neither triangles nor quads."""
    write_ply(tmp_path / "m.ply", MESH_P, MESH_F, extra_face=[[0, 1, 2, 3, 4]])
    assert _scene(pa, 'Shape "plymesh" "string filename" "m.ply"', tmp_path).info.n_triangles == 3


def smooth_sphere_text(res=48, spp=8, normals=True, sampler="zsobol"):
    """An icosphere with per-vertex normals (smooth shading) under a sky + area light."""
    import sys
    sys.path.insert(0, str(SCENES))
    import gen_c3
    P, F = gen_c3.icosphere(2)
    N = P.copy()
    UV = np.stack([0.5 + 0.5 * P[:, 0], 0.5 + 0.5 * P[:, 1]], 1)
    nline = f' "normal N" [ {gen_c3.fmt(N)} ]' if normals else ""
    return f"""LookAt 0 0.5 -4  0 0 0  0 1 0
Camera "perspective" "float fov" [ 35 ]
Film "rgb" "integer xresolution" [ {res} ] "integer yresolution" [ {res} ]
Sampler "{sampler}" "integer pixelsamples" [ {spp} ]
Integrator "volpath" "integer maxdepth" [ 5 ]
WorldBegin
LightSource "infinite" "rgb L" [ 0.2 0.25 0.3 ]
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [ 6 6 6 ]
  Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ] "point3 P" [ -1 3 -1  1 3 -1  1 3 1  -1 3 1 ]
    "normal N" [ 0 -1 0  0 -1 0.2  0 -1 0  0.2 -1 0 ]
AttributeEnd
Material "conductor" "float roughness" [ 0.05 ]
Shape "trianglemesh" "integer indices" [ {" ".join(map(str, F.ravel()))} ] "point3 P" [ {gen_c3.fmt(P)} ]
  {nline} "point2 uv" [ {gen_c3.fmt(UV)} ]
Material "diffuse" "rgb reflectance" [ 0.5 0.5 0.5 ]
Shape "trianglemesh" "integer indices" [ 0 1 2 0 2 3 ] "point3 P" [ -4 -1 -4  4 -1 -4  4 -1 4  -4 -1 4 ]
  "point2 uv" [ 0 0 3 0 3 3 0 3 ]
"""


def test_oracle_smooth_shading_changes_image(pa, oracle):
    def render(normals):
        sc = pa.Scene.from_string(smooth_sphere_text(normals=normals), SCENES)
        f = sc.flat()
        film = oracle.render(sc, threads=8)
        return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    a, b = render(True), render(False)
    assert np.isfinite(a).all() and a.min() >= 0
    assert np.abs(a - b).mean() > 1e-3 * np.abs(b).mean()
