"""Bilinear patches (shapes.h:1150-1560, shapes.cpp:914-1372): the "bilinearmesh" loader and
plymesh quads, the product's shared host/device intersection / SurfaceInteraction / Sample /
PDF code against the oracle's independent restatement (bit for bit, both on the host) for
rectangles (spherical-rectangle sampling, with and without the cos-weighted warp), non-planar
patches (bilinear area sampling), patches with uv (InvertBilinear in the pdf) and shading
normals, and a degenerate (triangle-shaped) patch; a rectangle emitter's known answer; GPU
parity in the wavefront and volumetric kernels and through the C-ABI intersector."""
import numpy as np
import pytest

from conftest import SCENES

PATCHES = """LookAt 0 1 -6  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.2 0.2 0.25]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [6 6 6]
Shape "bilinearmesh" "point3 P" [-0.5 2.5 -0.5  0.5 2.5 -0.5  -0.5 2.5 0.5  0.5 2.5 0.5]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.7 0.5 0.3]
AttributeBegin
Translate -1.2 -0.3 0.4
Rotate 20 0 1 0
Shape "bilinearmesh" "point3 P" [-0.8 0 -0.6  0.8 0.6 -0.6  -0.8 0.9 0.7  0.8 -0.2 0.8]
    "point2 uv" [0 0  2 0  0 1.5  2.2 1.7]
    "normal N" [0.1 1 -0.2  -0.3 1 0  0 1 0.3  0.2 0.8 0.1]
AttributeEnd
Material "conductor" "float roughness" 0.1
AttributeBegin
ReverseOrientation
Translate 1.3 0 0.2
Rotate -35 0 0 1
Shape "bilinearmesh" "point3 P" [-0.6 -0.4 -0.5  0.6 0.2 -0.5  -0.5 0.3 0.6  0.7 -0.5 0.5]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.3 0.6 0.4]
AttributeBegin
Translate 0.1 0.2 -1.2
Shape "bilinearmesh" "point3 P" [-0.4 0 0  0.4 0 0  -0.4 0.6 0  0.4 0 0]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
Shape "bilinearmesh" "point3 P" [-4 -1 -4  0 -1 -4  4 -1 -4  -4 -1 4  0 -1 4  4 -1 4]
    "integer indices" [0 1 3 4  1 2 4 5]
AttributeBegin
Translate 2 1.5 1
AreaLightSource "diffuse" "rgb L" [3 2 1] "bool twosided" true
Shape "bilinearmesh" "point3 P" [-0.5 0 -0.4  0.5 0.3 -0.4  -0.4 -0.3 0.5  0.4 0.1 0.3]
    "point2 uv" [0.1 0  1 0.2  0 0.9  1.1 1.2]
AttributeEnd
AttributeBegin
Translate 0.2 0.3 -2
Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [-0.3 0 0 0.3 0 0 0 0.5 0]
AttributeEnd
"""

EYE = np.array([0, 1, -6])  # render space is "cameraworld": world minus the eye
CENTERS = [(0, 2.5, 0), (-1.2, 0, 0.4), (1.3, 0, 0.2), (0.1, 0.4, -1.2), (-2, -1, 0), (2, -1, 0), (2, 1.5, 1)]


def _rays(rng, center, n, spread=1.0):
    o = rng.uniform(-5, 5, (n, 3))
    t = np.asarray(center) + rng.uniform(-spread, spread, (n, 3))
    return np.concatenate([o - EYE, t - o], 1).astype(np.float32)


def _flat(pa, text=PATCHES):
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    n = f.n_shapes
    info = np.ctypeslib.as_array(f.shape_info, shape=(n * 8,)).reshape(n, 8).copy()
    par = np.ctypeslib.as_array(f.shape_params, shape=(n * 32,)).reshape(n, 32).copy()
    nrm = np.ctypeslib.as_array(f.shape_normals, shape=(n * 12,)).reshape(n, 12).copy()
    return sc, f, info, par, nrm


def test_bilinear_loader_records(pa):
    sc, f, info, par, nrm = _flat(pa)
    assert (f.n_shapes, f.n_triangles, f.n_area_lights) == (7, 1, 2)
    assert list(info[:, 0]) == [3] * 7
    assert list(info[:, 3]) == [0, -1, -1, -1, -1, -1, 1]
    # corners in render space (world minus the eye), p00 p10 p01 p11
    np.testing.assert_allclose(par[0, :12].reshape(4, 3) + EYE,
                               [[-0.5, 2.5, -0.5], [0.5, 2.5, -0.5], [-0.5, 2.5, 0.5], [0.5, 2.5, 0.5]], atol=1e-6)
    # IsRectangle and area: the emitter and the two floor patches are rectangles
    assert list(par[:, 25]) == [1, 0, 0, 0, 1, 1, 0]
    np.testing.assert_allclose(par[[0, 4, 5], 24], [1, 32, 32], rtol=1e-6)
    # flags: bit0 ReverseOrientation, bit2 uv, bit3 N
    assert [int(x) & 13 for x in info[:, 1]] == [0, 12, 1, 0, 0, 0, 4]
    np.testing.assert_allclose(par[1, 12:20], [0, 0, 2, 0, 0, 1.5, 2.2, 1.7])
    # vertex normals through the (rotation-only) normal transform
    th = np.radians(20)
    ry = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
    np.testing.assert_allclose(nrm[1, :3], ry @ np.array([0.1, 1, -0.2]), atol=1e-6)


def test_bilinear_excess_indices_and_errors(pa):
    base = 'LookAt 0 0 -5 0 0 0 0 1 0\nCamera "perspective"\nWorldBegin\nLightSource "infinite"\n'
    sc = pa.Scene.from_string(base + 'Shape "bilinearmesh" "point3 P" [0 0 0 1 0 0 0 1 0 1 1 0 2 0 0] '
                              '"integer indices" [0 1 2 3 1 4]\n', SCENES)
    assert sc.flat().n_shapes == 1  # "Discarding excess" indices
    with pytest.raises(pa.PbrtError, match="indices"):
        pa.Scene.from_string(base + 'Shape "bilinearmesh" "point3 P" [0 0 0 1 0 0 0 1 0 1 1 0 2 0 0]\n', SCENES)
    with pytest.raises(pa.PbrtError, match="out of-bounds"):
        pa.Scene.from_string(base + 'Shape "bilinearmesh" "point3 P" [0 0 0 1 0 0 0 1 0 1 1 0] '
                             '"integer indices" [0 1 2 4]\n', SCENES)


def test_plymesh_quads_become_patches(pa, tmp_path):
    """plymesh: triangles become a TriangleMesh and quads bilinear patches in rply's
    0 1 3 2 corner order (scene.cpp plymesh, util/mesh.cpp ReadPly)."""
    ply = tmp_path / "tq.ply"
    ply.write_text("ply\nformat ascii 1.0\nelement vertex 6\nproperty float x\nproperty float y\n"
                   "property float z\nelement face 2\nproperty list uchar int vertex_indices\nend_header\n"
                   "0 0 0\n1 0 0\n1 1 0\n0 1 0\n2 0 0\n2 1 0\n4 0 1 2 3\n3 1 4 5\n")
    text = ('LookAt 0 0 -5 0 0 0 0 1 0\nCamera "perspective"\nWorldBegin\nLightSource "infinite"\n'
            f'Shape "plymesh" "string filename" "{ply}"\n')
    sc = pa.Scene.from_string(text, SCENES)
    f = sc.flat()
    assert (f.n_triangles, f.n_shapes) == (1, 1)
    par = np.ctypeslib.as_array(f.shape_params, shape=(32,))
    np.testing.assert_allclose(par[:12].reshape(4, 3) + [0, 0, -5], [[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]],
                               atol=1e-6)
    assert par[25] == 1 and par[24] == pytest.approx(1)


@pytest.mark.parametrize("shape", range(7))
def test_bilinear_code_matches_oracle_bitwise(pa, oracle, shape):
    """Intersection, SurfaceInteraction (uv remap, shading normals through RotateFromTo),
    Sample(ctx) and PDF(ctx) — odd rows carry a shading normal so rectangles take the
    cos-weighted warp and InvertSphericalRectangleSample — of the product's shared code vs
    the oracle."""
    sc = pa.Scene.from_string(PATCHES, SCENES)
    rng = np.random.default_rng(40 + shape)
    rays = _rays(rng, CENTERS[shape], 6000, 3.5 if shape in (4, 5) else 0.9)
    u = rng.random((6000, 2), dtype=np.float32)
    a = sc.shape_eval(shape, rays, u)
    b = oracle.shape_eval(sc, shape, rays, u)
    assert a[:, 0].sum() > 200
    assert (a[:, 37] > 0).sum() > 200  # pdfs evaluated
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _render(pa, oracle, text, **kw):
    sc = pa.Scene.from_string(text, SCENES, **kw)
    f = sc.flat()
    return oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def _rect_form_factor(x, y):
    """Differential area to a parallel rectangle x by y (in units of the height) above one corner."""
    a, b = np.sqrt(1 + x * x), np.sqrt(1 + y * y)
    return (x / a * np.arctan(y / a) + y / b * np.arctan(x / b)) / (2 * np.pi)


@pytest.mark.parametrize("twist", [False, True])
def test_rectangle_emitter_known_answer(pa, oracle, twist):
    """A white Lambertian floor under a downward square emitter (side s, radiance 1, height h):
    the floor's radiance below the centre is the form factor 4 F(s/2h, s/2h). twist=False is a
    rectangle (spherical-rectangle sampling with the cos warp), twist=True lifts one corner by
    1e-3 so the patch is not planar and takes bilinear area sampling instead."""
    s, h = 1.0, 1.0
    dz = 1e-3 if twist else 0
    text = ("""LookAt 0 0.6 -0.001  0 0 0  0 1 0
Camera "perspective" "float fov" 8
Film "rgb" "integer xresolution" 16 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 256
Integrator "volpath" "integer maxdepth" 1
WorldBegin
Material "diffuse" "rgb reflectance" [1 1 1]
Shape "bilinearmesh" "point3 P" [-20 0 -20  20 0 -20  -20 0 20  20 0 20]
Material "diffuse" "rgb reflectance" [0 0 0]
AreaLightSource "diffuse" "rgb L" [1 1 1]
""" + f'Shape "bilinearmesh" "point3 P" [-0.5 {h} -0.5  0.5 {h} -0.5  -0.5 {h} 0.5  0.5 {h + dz} 0.5]\n')
    sc, f, info, par, nrm = _flat(pa, text)
    assert list(par[:, 25]) == [1, 0 if twist else 1]
    img = _render(pa, oracle, text)
    want = 4 * _rect_form_factor(s / (2 * h), s / (2 * h))
    assert img[6:10, 6:10].mean() == pytest.approx(want, rel=0.02)


@pytest.mark.gpu
def test_patches_scene_matches_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.Scene.from_string(PATCHES, SCENES)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"patches parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_patches_volumetric_matches_oracle_gpu(pa, oracle):
    """The volumetric kernels: coated patches and a fog-filled box of patches (interface)."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    text = PATCHES.replace('Material "conductor" "float roughness" 0.1',
                           'Material "coateddiffuse" "rgb reflectance" [0.3 0.5 0.7] "float roughness" 0.1')
    text += ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.2 0.3 0.4] '
             '"rgb sigma_s" [1.5 1.2 1] "float g" 0.3\nAttributeBegin\nMediumInterface "fog" ""\n'
             'Material "interface"\nTranslate -1.8 0.9 -0.8\nShape "bilinearmesh" "point3 P" '
             '[-0.5 -0.5 -0.5  0.5 -0.5 -0.5  -0.5 -0.5 0.5  0.5 -0.5 0.5  -0.5 0.5 -0.5  0.5 0.5 -0.5  '
             '-0.5 0.5 0.5  0.5 0.5 0.5] "integer indices" [0 2 1 3  4 5 6 7  0 1 4 5  2 6 3 7  0 4 2 6  1 3 5 7]\n'
             'AttributeEnd\n')
    sc = pa.Scene.from_string(text, SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"patches volumetric parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_patch_intersections_match_oracle_gpu(pa, oracle):
    """pbrt_intersect closest and any-hit over patches and a triangle against the oracle."""
    import torch
    sc = pa.Scene.from_string(PATCHES, SCENES)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    rng = np.random.default_rng(9)
    n = 40000
    o = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    d = (rng.uniform(-1.5, 1.5, (n, 3)) - o).astype(np.float32)
    f = sc.flat()
    o = (o - EYE).astype(np.float32)
    rays = np.concatenate([o.T, d.T, np.full((1, n), np.inf, np.float32)]).astype(np.float32)
    for any_hit in (False, True):
        call = agg.IntersectShadow if any_hit else agg.IntersectClosest
        gp, gh = call(torch.from_numpy(rays).cuda())
        gp, gh = gp.cpu().numpy(), gh.cpu().numpy()
        op, oh = oracle.intersect(sc, rays, any_hit)
        np.testing.assert_array_equal(gp >= 0, op >= 0)
        if not any_hit:
            hit = op >= 0
            assert (op[hit] >= f.n_triangles).sum() > n // 10
            np.testing.assert_array_equal(gp[hit], op[hit])
            np.testing.assert_allclose(gh[3][hit], oh[3][hit], rtol=1e-5)
