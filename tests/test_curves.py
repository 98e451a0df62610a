"""Curves (Shape "curve") as pbrt's wavefront integrator renders them: OptiXAggregate::
diceCurveToBLP (gpu/aggregate.cpp:547-760, called with 5 steps along and 5 around at
:800-806) dices every curve into a bilinear patch mesh on the host -- a tube of 5 x 5 patches
with per-vertex normals for "flat" and "cylinder" curves, a strip of 5 patches across the
slerped normals for "ribbon" -- which the patch kernels then intersect and shade.

* the diced mesh bit for bit against tests/golden "curves" (oracle/ref/refgold.cpp restates
  the dicing loop over the reference's own Lerp / EvaluateCubicBezier / basis conversions /
  CoordinateSystem / AngleBetween / Cross / Normalize, since aggregate.cpp needs OptiX);
* Curve::Create's parameter errors (shapes.cpp:1004-1105);
* GPU film parity of a curve scene, surface and volumetric kernels (the patch paths)."""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 0 0  0 0 1  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 32 "integer yresolution" 32
Sampler "halton" "integer pixelsamples" 4
WorldBegin
LightSource "infinite" "rgb L" [0.5 0.5 0.5]
"""


def curve_line(c):
    n = f' "normal N" [{" ".join(f"{v:.9g}" for v in c["N"])}]' if c["N"] else ""
    return (f'Shape "curve" "point3 P" [{" ".join(f"{v:.9g}" for v in c["P"])}] "string basis" "{c["basis"]}" '
            f'"integer degree" {c["degree"]} "string type" "{c["type"]}" "float width0" {c["width0"]:.9g} '
            f'"float width1" {c["width1"]:.9g}{n}\n')


@pytest.mark.parametrize("case", range(8))
def test_curve_dicing_matches_reference(pa, golden, case):
    c = golden["curves"][case]
    sc = pa.Scene.from_string(HEAD + curve_line(c), SCENES)
    f = sc.flat()
    m = c["mesh"]
    idx = np.array(m["indices"]).reshape(-1, 4)
    P = np.array(m["P"], np.float32).reshape(-1, 3)
    uv = np.array(m["uv"], np.float32).reshape(-1, 2)
    n = f.n_shapes
    assert n == len(idx) and f.n_triangles == 0
    info = np.ctypeslib.as_array(f.shape_info, shape=(n * 8,)).reshape(n, 8)
    par = np.ctypeslib.as_array(f.shape_params, shape=(n * 32,)).reshape(n, 32)
    assert (info[:, 0] == 3).all()
    # render space is world minus the eye (at the origin): the object-space corners exactly
    np.testing.assert_array_equal(par[:, :12].reshape(n, 4, 3), P[idx])
    np.testing.assert_array_equal(par[:, 12:20].reshape(n, 4, 2), uv[idx])
    if c["type"] == "ribbon":
        assert not (info[:, 1] & 8).any()
    else:
        N = np.array(m["N"], np.float32).reshape(-1, 3)
        assert (info[:, 1] & 8).all()
        nrm = np.ctypeslib.as_array(f.shape_normals, shape=(n * 12,)).reshape(n, 4, 3)
        np.testing.assert_array_equal(nrm, N[idx])


@pytest.mark.parametrize("params, msg", [
    ('"point3 P" [0 0 1 0 1 1 1 1 1 1 0 1] "integer degree" 4', "only degree 2 and 3"),
    ('"point3 P" [0 0 1 0 1 1 1 1 1 1 0 1] "string basis" "hermite"', "Invalid basis"),
    ('"point3 P" [0 0 1 0 1 1 1 1 1 1 0 1 2 0 1]', "Invalid number of control points"),
    ('"point3 P" [0 0 1 0 1 1 1 1 1] "string basis" "bspline"', "must have >= 4"),
    ('"point3 P" [0 0 1 0 1 1 1 1 1 1 0 1] "string type" "ribbon"', "Must provide normals"),
    ('"point3 P" [0 0 1 0 1 1 1 1 1 1 0 1] "string type" "ribbon" "normal N" [0 0 1]', "Invalid number of normals"),
])
def test_curve_errors(pa, params, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(HEAD + f'Shape "curve" {params}\n', SCENES)


def test_curve_area_light_refused_and_defaults(pa):
    with pytest.raises(pa.PbrtError, match="area lights on curves"):
        pa.Scene.from_string(HEAD + 'AreaLightSource "diffuse"\nShape "curve" "point3 P" [0 0 1 0 1 1 1 1 1 1 0 1]\n',
                             SCENES)
    # defaults: bezier, degree 3, flat (a tube), width 1; "N" on a flat curve is ignored
    # (a warning) and "splitdepth" is accepted
    sc = pa.Scene.from_string(HEAD + 'Shape "curve" "point3 P" [0 0 1 0 1 1 1 1 1 1 0 1] "normal N" [0 0 1 0 0 1] '
                              '"integer splitdepth" 5\n', SCENES)
    f = sc.flat()
    assert f.n_shapes == 25
    par = np.ctypeslib.as_array(f.shape_params, shape=(25 * 32,)).reshape(25, 32)
    # the first ring sits at distance width / 2 = 0.5 from the curve start (0, 0, 1)
    r = np.linalg.norm(par[:5, :3] - [0, 0, 1], axis=1)
    np.testing.assert_allclose(r, 0.5, rtol=1e-6)


SCENE = """LookAt 0 1.2 -3.5  0 0.6 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.3 0.32 0.35]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [6 6 6]
Shape "bilinearmesh" "point3 P" [-0.6 2.6 -0.6  0.6 2.6 -0.6  -0.6 2.6 0.6  0.6 2.6 0.6]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.5 0.5 0.5]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-3 0 -3 3 0 -3 3 0 3 -3 0 3]
Material "coateddiffuse" "rgb reflectance" [0.6 0.35 0.15] "float roughness" 0.2
"""


def strands(seed=3, n=40):
    rng = np.random.default_rng(seed)
    out = []
    kinds = ["flat", "cylinder", "ribbon"]
    for i in range(n):
        x, z = rng.uniform(-1, 1, 2)
        h = rng.uniform(0.8, 1.6)
        bend = rng.uniform(-0.4, 0.4, 2)
        P = [x, 0, z, x + bend[0] * 0.3, h * 0.35, z + bend[1] * 0.3, x + bend[0] * 0.8, h * 0.7, z + bend[1] * 0.8,
             x + bend[0], h, z + bend[1]]
        t = kinds[i % 3]
        extra = ' "normal N" [0 0 -1 0.3 0 -1]' if t == "ribbon" else ""
        out.append(f'Shape "curve" "point3 P" [{" ".join(f"{v:.5f}" for v in P)}] "string type" "{t}" '
                   f'"float width0" 0.08 "float width1" 0.02{extra}\n')
    return "".join(out)


def test_curve_scene_oracle_renders(pa, oracle):
    sc = pa.Scene.from_string(SCENE + strands(n=12), SCENES, xresolution=32, yresolution=24, spp=4)
    assert sc.flat().n_shapes == 4 * 25 + 4 * 25 + 4 * 5 + 1
    f = sc.flat()
    img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert np.isfinite(img).all() and img.mean() > 0.01


@pytest.mark.gpu
def test_curve_scene_matches_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.Scene.from_string(SCENE + strands(), SCENES)
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"curves parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_curve_scene_volumetric_matches_oracle_gpu(pa, oracle):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    fog = ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.05 0.05 0.05] '
           '"rgb sigma_s" [0.3 0.3 0.3]\nAttributeBegin\nMediumInterface "fog" ""\nMaterial "interface"\n'
           'Shape "bilinearmesh" "point3 P" [-1.5 0.01 -1.5  1.5 0.01 -1.5  -1.5 2 -1.5  1.5 2 -1.5  '
           '-1.5 0.01 1.5  1.5 0.01 1.5  -1.5 2 1.5  1.5 2 1.5] "integer indices" [0 2 1 3  4 5 6 7  0 1 4 5  '
           '2 6 3 7  0 4 2 6  1 3 5 7]\nAttributeEnd\n')
    sc = pa.Scene.from_string(SCENE + fog + strands(n=20), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"curves volumetric parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mr:.2e}")
