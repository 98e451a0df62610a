"""Per-vertex shading tangents: trianglemesh "vector3 S" (shapes.cpp:408-413, TriangleMesh s in
render space, util/mesh.cpp:58-63) setting the shading dpdu of Triangle::InteractionFromIntersection
(shapes.h:940-1010: the interpolated S, made perpendicular to the shading normal; the geometric
dpdu when it interpolates to zero).  An anisotropic conductor shows the frame.

* loader: S transformed as a vector, tri_shading bit2; a count mismatch is reported and the
  tangents discarded (pbrt's Error(), not fatal);
* bump mapping on such a mesh (round 6): the shading bitangent ts = Cross(ns, S) and dndu /
  dndv as Triangle::InteractionFromIntersection leaves them (shapes.h:940-1006; zero without
  vertex normals), the oracle's restatement and the texture stage alike;
* oracle: the tangents change an anisotropic render; S along the geometric dpdu leaves it as is;
* GPU film parity against the oracle on the surface and the volumetric paths.
"""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 1.2 -2.4  0 0.2 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 48 "integer yresolution" 36
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 4
WorldBegin
LightSource "infinite" "rgb L" [0.2 0.2 0.25]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [8 8 8]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.5 2 -0.5  0.5 2 -0.5  0.5 2 0.5  -0.5 2 0.5]
AttributeEnd
"""
MAT = 'Material "conductor" "float uroughness" 0.02 "float vroughness" 0.5 "bool remaproughness" false'
# a gently curved sheet with per-vertex normals and tangents that rotate across it
N = 6


def sheet(with_s=True, s_kind="rotate", with_n=True, bump=""):
    P, Nn, S, uv, idx = [], [], [], [], []
    for j in range(N + 1):
        for i in range(N + 1):
            x, z = -1 + 2 * i / N, -1 + 2 * j / N
            y = 0.15 * (x * x + z * z)
            P += [x, y, z]
            n = np.array([-0.3 * x, 1.0, -0.3 * z])
            Nn += list(n / np.linalg.norm(n))
            a = 0.6 * x + 0.4 * z if s_kind == "rotate" else 0.0
            S += [np.cos(a), 0.0, np.sin(a)] if s_kind != "zero" else [0.0, 0.0, 0.0]
            uv += [i / N, j / N]
    for j in range(N):
        for i in range(N):
            a = j * (N + 1) + i
            idx += [a, a + 1, a + N + 2, a, a + N + 2, a + N + 1]
    fmt = lambda v: " ".join(f"{x:.6g}" for x in v)
    s = f'Shape "trianglemesh" "integer indices" [{fmt(idx)}] "point3 P" [{fmt(P)}] "point2 uv" [{fmt(uv)}]'
    if with_n:
        s += f' "normal N" [{fmt(Nn)}]'
    if with_s:
        s += f' "vector3 S" [{fmt(S)}]'
    return f"AttributeBegin\n{bump or MAT}\n{s}\nAttributeEnd\n"


def scene(*a, medium=False, **kw):
    extra = ""
    if medium:  # a fog ball (interface material) puts the scene on the volumetric path
        extra = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.3 0.3 0.3] '
                 '"rgb sigma_s" [0.4 0.4 0.4]\nAttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\n'
                 'Translate 0.7 0.6 -0.2\nShape "sphere" "float radius" 0.25\nAttributeEnd\n')
    return HEAD + extra + sheet(*a, **kw)


def oracle_rgb(oracle, sc):
    f = sc.flat()
    return oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_tangents_loader(pa):
    sc = pa.Scene.from_string(scene(), SCENES)
    f = sc.flat()
    ts = np.ctypeslib.as_array(f.tri_shading, shape=(f.n_triangles,))
    assert (ts[-2 * N * N:] & 4).all() and f.n_vertex_s >= (N + 1) ** 2
    vs = np.ctypeslib.as_array(f.vertex_s, shape=(f.n_vertex_s * 3,)).reshape(-1, 3)
    # render space is camera-world here up to a translation: the tangents keep unit length
    np.testing.assert_allclose(np.linalg.norm(vs[-(N + 1) ** 2:], axis=1), 1, rtol=1e-5)
    # a count mismatch: reported, tangents discarded
    bad = scene().replace('"vector3 S" [', '"vector3 S" [1 0 0 ')
    sc2 = pa.Scene.from_string(bad, SCENES)
    ts2 = np.ctypeslib.as_array(sc2.flat().tri_shading, shape=(sc2.flat().n_triangles,))
    assert not (ts2 & 4).any()


BUMP = ('Texture "f" "float" "fbm" "integer octaves" 4\nTexture "b" "float" "scale" "texture tex" "f" '
        '"float scale" 0.03\nMaterial "conductor" "float uroughness" 0.05 "float vroughness" 0.4 '
        '"texture displacement" "b"')


@pytest.mark.parametrize("with_n", [True, False])
def test_tangents_bump_changes_oracle_render(pa, oracle, with_n):
    plain = pa.Scene.from_string(scene(with_n=with_n), SCENES, xresolution=48, yresolution=32, spp=8)
    bumped = pa.Scene.from_string(scene(with_n=with_n, bump=BUMP), SCENES, xresolution=48, yresolution=32, spp=8)
    a, b = oracle_rgb(oracle, bumped), oracle_rgb(oracle, plain)
    assert np.isfinite(a).all()
    assert np.abs(a - b).mean() > 1e-3


def test_tangents_change_oracle_render(pa, oracle):
    base = oracle_rgb(oracle, pa.Scene.from_string(scene(with_s=False), SCENES))
    rot = oracle_rgb(oracle, pa.Scene.from_string(scene(), SCENES))
    zero = oracle_rgb(oracle, pa.Scene.from_string(scene(s_kind="zero"), SCENES))
    assert np.isfinite(rot).all()
    assert np.abs(rot - base).max() > 0.05  # the anisotropic lobe turns with S
    # S interpolating to zero falls back to the geometric dpdu: the render without S
    np.testing.assert_array_equal(zero, base)


@pytest.mark.gpu
@pytest.mark.parametrize("medium", [False, True])
@pytest.mark.parametrize("with_n", [True, False])
def test_tangents_bump_match_oracle_gpu(pa, oracle, medium, with_n):
    from test_gpu_media import check, gpu_rgb
    sc = pa.Scene.from_string(scene(with_n=with_n, medium=medium, bump=BUMP), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"bumped tangents (medium={medium}, normals={with_n}): {frac*100:.2f}% pixels, mean rel {mr:.2e}")


@pytest.mark.gpu
@pytest.mark.parametrize("medium", [False, True])
@pytest.mark.parametrize("with_n", [True, False])
def test_tangents_match_oracle_gpu(pa, oracle, medium, with_n):
    from test_gpu_media import check, gpu_rgb
    sc = pa.Scene.from_string(scene(with_n=with_n, medium=medium), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"tangents (medium={medium}, normals={with_n}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")
