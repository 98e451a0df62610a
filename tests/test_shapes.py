"""Spheres and disks (shapes.h:106-571, shapes.cpp:33-119): loader, the product's shared
host/device intersection / SurfaceInteraction / sampling / pdf code against the oracle's
independent restatement (bit for bit, both on the host), known answers for sphere and disk
emitters, and GPU parity (wavefront and volumetric kernels, C-ABI intersections).

Interval arithmetic follows pbrt's CPU build (AddRoundUp(a, b) = NextFloatUp(a + b), ...);
pbrt's GPU build rounds each interval operation directionally instead, which only moves the
conservative bounds by an ulp."""
import numpy as np
import pytest

from conftest import SCENES

SHAPES = """LookAt 0 1 -6  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.2 0.2 0.25]
AttributeBegin
Translate 0 2.5 0
AreaLightSource "diffuse" "rgb L" [8 8 8]
Shape "sphere" "float radius" 0.4
AttributeEnd
Material "diffuse" "rgb reflectance" [0.7 0.5 0.3]
AttributeBegin
Translate -1 0 0.5
Rotate 30 1 0 0
Shape "sphere" "float radius" 0.8 "float zmin" -0.5 "float zmax" 0.6 "float phimax" 300
AttributeEnd
Material "conductor" "float roughness" 0.1
AttributeBegin
Translate 1.2 -0.2 0
Scale 0.7 0.7 0.7
Shape "sphere"
AttributeEnd
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
AttributeBegin
Translate 0 -1 0
Rotate -90 1 0 0
Shape "disk" "float radius" 4 "float innerradius" 0.5
AttributeEnd
AttributeBegin
Translate 2 1.5 1
Rotate 120 1 0 0
AreaLightSource "diffuse" "rgb L" [3 2 1] "bool twosided" true
Shape "disk" "float radius" 0.5 "float phimax" 270
AttributeEnd
AttributeBegin
ReverseOrientation
Translate 0.2 0.3 -1.5
Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [-0.3 0 0 0.3 0 0 0 0.5 0]
AttributeEnd
"""


EYE = np.array([0, 1, -6])  # render space is "cameraworld": world minus the eye


def _rays(rng, center, n, spread=1.5):
    o = rng.uniform(-5, 5, (n, 3))
    t = np.asarray(center) + rng.uniform(-spread, spread, (n, 3))
    return np.concatenate([o - EYE, t - o], 1).astype(np.float32)


def test_shape_loader_records(pa):
    sc = pa.Scene.from_string(SHAPES, SCENES)
    f = sc.flat()
    assert (f.n_shapes, f.n_triangles, f.n_area_lights) == (5, 1, 2)
    info = np.ctypeslib.as_array(f.shape_info, shape=(5 * 8,)).reshape(5, 8)
    par = np.ctypeslib.as_array(f.shape_params, shape=(5 * 32,)).reshape(5, 32)
    assert list(info[:, 0]) == [1, 1, 1, 2, 2]
    assert list(info[:, 3]) == [0, -1, -1, -1, 1]  # area lights in shape order
    # partial sphere: zMin, zMax clamped; thetaZMin = acos(zmin / r); phiMax in radians
    np.testing.assert_allclose(par[1, 24:30], [0.8, -0.5, 0.6, np.radians(300), np.arccos(-0.5 / 0.8),
                                               np.arccos(0.6 / 0.8)], rtol=1e-6)
    np.testing.assert_allclose(par[3, 24:28], [0, 4, 0.5, 2 * np.pi], rtol=1e-6)
    lp = np.ctypeslib.as_array(f.light_prim, shape=(2,))
    assert list(lp) == [f.n_triangles + 0, f.n_triangles + 4]


@pytest.mark.parametrize("shape, center", [(0, (0, 2.5, 0)), (1, (-1, 0, 0.5)), (2, (1.2, -0.2, 0)),
                                           (3, (0, -1, 0)), (4, (2, 1.5, 1))])
def test_shape_code_matches_oracle_bitwise(pa, oracle, shape, center):
    """Intersection (interval quadratic), the render-space SurfaceInteraction, Shape::Sample(ctx)
    (cone / area sampling) and Shape::PDF(ctx) of the product's shared code vs the oracle."""
    sc = pa.Scene.from_string(SHAPES, SCENES)
    rng = np.random.default_rng(shape)
    rays = _rays(rng, center, 6000, 1.0 if shape != 3 else 4.0)
    u = rng.random((6000, 2), dtype=np.float32)
    a = sc.shape_eval(shape, rays, u)
    b = oracle.shape_eval(sc, shape, rays, u)
    assert a[:, 0].sum() > 500
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def _render(pa, oracle, text, **kw):
    sc = pa.Scene.from_string(text, SCENES, **kw)
    f = sc.flat()
    return oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


KAT = """LookAt 0 3 -0.001  0 0 0  0 1 0
Camera "perspective" "float fov" 8
Film "rgb" "integer xresolution" 16 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 256
Integrator "volpath" "integer maxdepth" 1
WorldBegin
Material "diffuse" "rgb reflectance" [1 1 1]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-20 0 -20 20 0 -20 20 0 20 -20 0 20]
"""


def test_sphere_emitter_irradiance_known_answer(pa, oracle):
    """A Lambertian white floor under a sphere emitter of radiance L, radius r at height h:
    E = pi L r^2 / h^2 below it, so the floor's radiance is L r^2 / h^2 (cone sampling, MIS)."""
    r, h = 0.25, 1.0
    text = KAT.replace("LookAt 0 3", "LookAt 0 0.6") + (
        f'AttributeBegin\nTranslate 0 {h} 0\nMaterial "diffuse" "rgb reflectance" [0 0 0]\n'
        f'AreaLightSource "diffuse" "rgb L" [1 1 1]\nShape "sphere" "float radius" {r}\nAttributeEnd\n')
    img = _render(pa, oracle, text)
    assert img[6:10, 6:10].mean() == pytest.approx(r * r / (h * h), rel=0.02)


def test_disk_emitter_irradiance_known_answer(pa, oracle):
    """A downward disk emitter of radius R at height h: E = pi L R^2 / (h^2 + R^2) below its
    centre, the floor's radiance L R^2 / (h^2 + R^2) (area sampling converted to solid angle)."""
    R, h = 0.5, 1.0
    text = KAT.replace("LookAt 0 3", "LookAt 0 0.6") + (f'AttributeBegin\nTranslate 0 {h} 0\nRotate 90 1 0 0\nMaterial "diffuse" "rgb reflectance" [0 0 0]\n'
                  f'AreaLightSource "diffuse" "rgb L" [1 1 1]\nShape "disk" "float radius" {R}\nAttributeEnd\n')
    img = _render(pa, oracle, text)
    assert img[6:10, 6:10].mean() == pytest.approx(R * R / (h * h + R * R), rel=0.02)


def test_sphere_under_uniform_sky_known_answer(pa, oracle):
    """A convex diffuse sphere of albedo 0.5 under a unit uniform sky, one bounce: 0.5."""
    text = """LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 10
Film "rgb" "integer xresolution" 16 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 64
Integrator "volpath" "integer maxdepth" 1
WorldBegin
LightSource "infinite" "rgb L" [1 1 1]
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
Shape "sphere" "float radius" 1
"""
    img = _render(pa, oracle, text)
    assert img[4:12, 4:12].mean() == pytest.approx(0.5, abs=0.01)


def test_inside_emitting_sphere(pa, oracle):
    """The camera inside a reversed emitting sphere sees exactly its radiance."""
    text = """LookAt 0 0 0  0 0 1  0 1 0
Camera "perspective" "float fov" 60
Film "rgb" "integer xresolution" 8 "integer yresolution" 8
Sampler "halton" "integer pixelsamples" 4
Integrator "volpath" "integer maxdepth" 3
WorldBegin
ReverseOrientation
Material "diffuse" "rgb reflectance" [0 0 0]
AreaLightSource "diffuse" "rgb L" [0.5 0.5 0.5]
Shape "sphere" "float radius" 3
"""
    img = _render(pa, oracle, text)
    np.testing.assert_allclose(img, 0.5, rtol=2e-3)


@pytest.mark.gpu
def test_shapes_scene_matches_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.Scene.from_string(SHAPES, SCENES)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"shapes parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_shapes_volumetric_matches_oracle_gpu(pa, oracle):
    """The volumetric kernels: a medium-filled sphere (interface material) and a coated sphere
    beside the emitters (oracle in its libm mode, as the media tests)."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    text = SHAPES.replace('Material "conductor" "float roughness" 0.1',
                          'Material "coateddiffuse" "rgb reflectance" [0.3 0.5 0.7] "float roughness" 0.1')
    text += ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.2 0.3 0.4] '
             '"rgb sigma_s" [1.5 1.2 1] "float g" 0.3\nAttributeBegin\nMediumInterface "fog" ""\n'
             'Material "interface"\nTranslate -1.8 0.9 -0.8\nShape "sphere" "float radius" 0.6\nAttributeEnd\n')
    sc = pa.Scene.from_string(text, SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"shapes volumetric parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_shape_intersections_match_oracle_gpu(pa, oracle):
    """pbrt_intersect closest and any-hit over spheres, disks and a triangle: ids (n_triangles + k
    for shapes) and t against the oracle."""
    import torch
    sc = pa.Scene.from_string(SHAPES, SCENES)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    rng = np.random.default_rng(5)
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


CYL = """LookAt 0 1 -6  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.2 0.2 0.25]
AttributeBegin
Translate 0 2.2 0
Rotate 90 0 1 0
AreaLightSource "diffuse" "rgb L" [4 4 4] "bool twosided" true
Shape "cylinder" "float radius" 0.2 "float zmin" -0.8 "float zmax" 0.8
AttributeEnd
Material "diffuse" "rgb reflectance" [0.6 0.5 0.4]
AttributeBegin
Translate -1 0 0.5
Rotate -90 1 0 0
Shape "cylinder" "float radius" 0.6 "float zmin" 1 "float zmax" -0.9 "float phimax" 250
AttributeEnd
AttributeBegin
ReverseOrientation
Translate 1.3 0 0
Rotate 30 0 0 1
Shape "cylinder"
AttributeEnd
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-4 -1 -4 4 -1 -4 4 -1 4 -4 -1 4]
"""


def test_cylinder_loader_records(pa):
    sc = pa.Scene.from_string(CYL, SCENES)
    f = sc.flat()
    assert (f.n_shapes, f.n_triangles, f.n_area_lights) == (3, 2, 1)
    info = np.ctypeslib.as_array(f.shape_info, shape=(3 * 8,)).reshape(3, 8)
    par = np.ctypeslib.as_array(f.shape_params, shape=(3 * 32,)).reshape(3, 32)
    assert list(info[:, 0]) == [4, 4, 4]
    # Cylinder ctor: zMin / zMax ordered, phiMax in radians; defaults radius 1, z -1..1
    np.testing.assert_allclose(par[1, 24:28], [0.6, -0.9, 1, np.radians(250)], rtol=1e-6)
    np.testing.assert_allclose(par[2, 24:28], [1, -1, 1, 2 * np.pi], rtol=1e-6)


@pytest.mark.parametrize("shape, center", [(0, (0, 2.2, 0)), (1, (-1, 0, 0.5)), (2, (1.3, 0, 0))])
def test_cylinder_code_matches_oracle_bitwise(pa, oracle, shape, center):
    """Cylinder::BasicIntersect (interval quadratic in x-y, reprojection, partial-phi retry),
    the render-space SurfaceInteraction, Sample(ctx, u) through Sample(u) and PDF(ctx, wi)."""
    sc = pa.Scene.from_string(CYL, SCENES)
    rng = np.random.default_rng(70 + shape)
    rays = _rays(rng, center, 6000, 1.2)
    u = rng.random((6000, 2), dtype=np.float32)
    a = sc.shape_eval(shape, rays, u)
    b = oracle.shape_eval(sc, shape, rays, u)
    assert a[:, 0].sum() > 500
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_inside_emitting_cylinder(pa, oracle):
    """The camera on the axis of a long reversed emitting cylinder, looking across it, sees
    exactly its radiance."""
    text = """LookAt 0 0 0  1 0 0  0 0 1
Camera "perspective" "float fov" 20
Film "rgb" "integer xresolution" 8 "integer yresolution" 8
Sampler "halton" "integer pixelsamples" 4
Integrator "volpath" "integer maxdepth" 3
WorldBegin
ReverseOrientation
Material "diffuse" "rgb reflectance" [0 0 0]
AreaLightSource "diffuse" "rgb L" [0.5 0.5 0.5]
Shape "cylinder" "float radius" 2 "float zmin" -50 "float zmax" 50
"""
    img = _render(pa, oracle, text)
    np.testing.assert_allclose(img, 0.5, rtol=2e-3)


@pytest.mark.gpu
def test_cylinders_match_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.Scene.from_string(CYL, SCENES)
    film, _ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle.render(sc, threads=16)))
    print(f"cylinders parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")



# ---------------------------------------------------------------- reference goldens
# tests/golden/reference_components.json "shapes": the reference's own Sphere, Disk, Cylinder and
# BilinearPatch (shapes.h / shapes.cpp compiled unmodified into oracle/_ref/refgold) on seeded
# rays, in pbrt_debug_shape_eval's row layout (oracle/ref/refgold.cpp ShapeGoldens).  The
# transforms are Translate * ConcatTransform(signed permutation) * Scale with dyadic values, so
# the loader's double-precision composition and inversion equal pbrt's float ones bit for bit.
_PERM = {0: None,
         1: [[0, 0, 1, 0], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 0, 1]],
         2: [[0, 0, 1, 0], [0, 1, 0, 0], [1, 0, 0, 0], [0, 0, 0, 1]]}


def _fmt(v):
    return " ".join(repr(float(x)) for x in v)


def golden_shape_scene(case):
    """The one-shape scene of a golden case (camera at the origin: render space = world)."""
    lines = ['LookAt 0 0 0  0 0 1  0 1 0', 'Camera "perspective"', 'WorldBegin', 'LightSource "infinite"',
             'AttributeBegin']
    if case["reverse"]:
        lines.append("ReverseOrientation")
    lines.append("Translate " + _fmt(case["translate"]))
    if _PERM[case["perm"]] is not None:
        m = np.array(_PERM[case["perm"]], float)
        lines.append("ConcatTransform [" + _fmt(m.T.reshape(-1)) + "]")  # column-major, as pbrt reads it
    lines.append("Scale " + _fmt(case["scale"]))
    a, b, c, d = case["params"]
    kind = case["kind"]
    if kind == "sphere":
        shape = f'Shape "sphere" "float radius" {a!r} "float zmin" {b!r} "float zmax" {c!r} "float phimax" {d!r}'
    elif kind == "disk":
        shape = f'Shape "disk" "float height" {a!r} "float radius" {b!r} "float innerradius" {c!r} "float phimax" {d!r}'
    elif kind == "cylinder":
        shape = f'Shape "cylinder" "float radius" {a!r} "float zmin" {b!r} "float zmax" {c!r} "float phimax" {d!r}'
    else:
        shape = f'Shape "bilinearmesh" "point3 P" [{_fmt(case["P"])}]'
        if case["N"]:
            shape += f' "normal N" [{_fmt(case["N"])}]'
        if case["uv"]:
            shape += f' "point2 uv" [{_fmt(case["uv"])}]'
    lines += [shape, "AttributeEnd", ""]
    return "\n".join(lines)


def _golden_rows(case):
    rays = np.array([r["ray"] for r in case["rows"]], np.float32)
    u = np.array([r["u"] for r in case["rows"]], np.float32)
    want = np.array([[float(x) for x in r["out"]] for r in case["rows"]], np.float32)
    return rays, u, want


def _assert_rows_equal(got, want, label):
    """Bit for bit, except that +0 and -0 compare equal: the loader composes and inverts
    transforms in double (Gauss-Jordan), pbrt in float (compensated inner products and the
    cofactor inverse, util/math.h), so an exactly-zero matrix entry may carry the other sign
    and so may a zero component it produces; every value is the same float."""
    cols = list(range(38))
    g, w = got[:, cols].copy(), want[:, cols].copy()
    g[g == 0] = 0
    w[w == 0] = 0
    bad = np.nonzero((g.view(np.uint32) != w.view(np.uint32)).any(axis=1))[0]
    if len(bad):
        i = bad[0]
        diff = [j for j in cols if got[i, j].view(np.uint32) != want[i, j].view(np.uint32)]
        raise AssertionError(f"{label}: {len(bad)} of {len(got)} rows differ; row {i} columns {diff}: "
                             f"got {got[i, diff]} want {want[i, diff]}")


@pytest.mark.parametrize("ci", range(13))
def test_shapes_match_reference_goldens(pa, oracle, golden, ci):
    """Intersection, SurfaceInteraction, Sample(ctx, u) and PDF(ctx, wi) of spheres, disks,
    cylinders and bilinear patches against the reference's own code, bit for bit: the product's
    shared host/device code and the oracle's restatement."""
    case = golden["shapes"][ci]
    sc = pa.Scene.from_string(golden_shape_scene(case), SCENES)
    assert sc.flat().n_shapes == 1
    rays, u, want = _golden_rows(case)
    assert want[:, 0].sum() >= 10 and want[:, 26].sum() >= 10  # hits and samples exercised
    _assert_rows_equal(sc.shape_eval(0, rays, u), want, f"product {case['kind']} #{ci}")
    _assert_rows_equal(oracle.shape_eval(sc, 0, rays, u), want, f"oracle {case['kind']} #{ci}")
