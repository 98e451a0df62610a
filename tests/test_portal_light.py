"""PortalImageInfiniteLight: LightSource "infinite" with "filename" and "point3 portal"
(lights.h:644-744, lights.cpp:1140-1297, 1558-1694).  The map is rectified over the portal
frame's angles and sampled with a WindowedPiecewiseConstant2D (util/sampling.h:830-989)
restricted to the portal as seen from the shading point; Le of an escaped ray and PDF_Li depend
on the ray origin / previous vertex, so portal scenes render on the volumetric kernels.

* the product's host code (pbrt_debug_portal_eval: rectified image, distribution, Le, PDF_Li,
  SampleLi) against the oracle's restatement, bit for bit in libm mode;
* pbrt's loader errors; the portal light and the plain image light of the same map agree on a
  room lit through a window (the portal only changes the sampling);
* GPU film parity against the oracle (libm mode).
"""
import numpy as np
import pytest

from conftest import SCENES

ROOM = [  # a closed room x [-1, 1], y [0, 2], z [-1, 1] with a window in its z = 1 wall
    "-1 0 -1  1 0 -1  1 0 1  -1 0 1",        # floor
    "-1 2 -1  -1 2 1  1 2 1  1 2 -1",        # ceiling
    "-1 0 -1  -1 2 -1  1 2 -1  1 0 -1",      # back wall
    "-1 0 -1  -1 0 1  -1 2 1  -1 2 -1",      # left
    "1 0 -1  1 2 -1  1 2 1  1 0 1",          # right
    "-1 0 1  -0.5 0 1  -0.5 2 1  -1 2 1",    # front wall around the window
    "0.5 0 1  1 0 1  1 2 1  0.5 2 1",
    "-0.5 0 1  0.5 0 1  0.5 0.6 1  -0.5 0.6 1",
    "-0.5 1.4 1  0.5 1.4 1  0.5 2 1  -0.5 2 1",
]
PORTAL = "-0.5 0.6 1  -0.5 1.4 1  0.5 1.4 1  0.5 0.6 1"  # p01 = +y, p03 = +x: frame z points out


def scene(portal=True, res=(48, 36), spp=16, maxdepth=4, extra=""):
    walls = "\n".join(f'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [{q}]' for q in ROOM)
    light = 'LightSource "infinite" "string filename" "textures/env_sky.pfm" "float scale" 2'
    if portal:
        light += f' "point3 portal" [{PORTAL}]'
    return f"""LookAt 0.3 0.8 -0.9  -0.1 1.0 1  0 1 0
Camera "perspective" "float fov" 70
Film "rgb" "integer xresolution" {res[0]} "integer yresolution" {res[1]}
Sampler "halton" "integer pixelsamples" {spp}
Integrator "volpath" "integer maxdepth" {maxdepth}
WorldBegin
AttributeBegin
Rotate -90 1 0 0
{light}
AttributeEnd
Material "diffuse" "rgb reflectance" [0.7 0.65 0.6]
{walls}
{extra}"""


def queries(n=4000, seed=3):
    rng = np.random.default_rng(seed)
    q = np.zeros((n, 8), np.float32)
    # points inside the room (render space = camera-world here up to the camera translation,
    # which the flat scene's coordinates already include: use world points, then shift)
    q[:, 0] = rng.uniform(-0.95, 0.95, n)
    q[:, 1] = rng.uniform(0.05, 1.95, n)
    q[:, 2] = rng.uniform(-0.95, 0.9, n)
    d = rng.normal(size=(n, 3))
    d[:, 2] = np.abs(d[:, 2])  # mostly towards the window wall
    q[:, 3:6] = d / np.linalg.norm(d, axis=1, keepdims=True)
    q[:, 6:8] = rng.uniform(size=(n, 2))
    return q


def to_render(sc, q):
    """the queries' points from world to render space (camera-world: a translation by -eye)"""
    eye = np.array([0.3, 0.8, -0.9], np.float32)
    q = q.copy()
    q[:, :3] -= eye
    return q


def test_portal_host_matches_oracle(pa, oracle):
    sc = pa.Scene.from_string(scene(), SCENES)
    f = sc.flat()
    assert f.env_info[1] == 1
    res = f.env_info[0]
    q = to_render(sc, queries())
    got, rect, func = sc.portal_eval(0, q, res=res)
    with oracle.math_mode(oracle.MATH_LIBM):
        ref, rrect, rfunc = oracle.portal_eval(sc, 0, q, res=res)
    np.testing.assert_array_equal(rect.view(np.uint32), rrect.view(np.uint32))
    np.testing.assert_array_equal(func.view(np.uint32), rfunc.view(np.uint32))
    np.testing.assert_array_equal(got.view(np.uint32), ref.view(np.uint32))
    assert got[:, 14].mean() > 0.5 and got[:, 5].mean() > 0.5  # bounds and samples mostly exist
    assert (got[:, :4] > 0).any() and np.isfinite(got).all()
    # a sample's pdf equals PDF_Li of its direction from the same point
    ok = got[:, 5] == 1
    qs = q[ok].copy()
    qs[:, 3:6] = got[ok, 6:9]
    back = sc.portal_eval(0, qs)
    np.testing.assert_allclose(back[:, 4], got[ok, 9], rtol=2e-3)


@pytest.mark.parametrize("src, msg", [
    (scene().replace(PORTAL, "-0.5 0.6 1  -0.5 1.4 1  0.5 1.4 1"), "Expected 4 vertices"),
    (scene().replace('"string filename" "textures/env_sky.pfm"', '"rgb L" [1 1 1]'), "not supported"),
])
def test_portal_loader_errors(pa, src, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(src, SCENES)


def test_portal_agrees_with_image_light(pa, oracle):
    """the same map seen through the window, sampled through the portal or over the whole sphere"""
    imgs = []
    for portal in (True, False):
        sc = pa.Scene.from_string(scene(portal, res=(16, 12), spp=256, maxdepth=3), SCENES)
        f = sc.flat()
        imgs.append(oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)]))
    a, b = imgs
    assert np.isfinite(a).all() and a.mean() > 1e-3
    rel = abs(a.mean() / b.mean() - 1)
    assert rel < 0.05, (a.mean(), b.mean())
    # the portal estimate is the less noisy one: its pixels vary less around a smooth image
    assert np.abs(np.diff(a, axis=1)).mean() < np.abs(np.diff(b, axis=1)).mean()


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["plain", "glossy"])
def test_portal_matches_oracle_gpu(pa, oracle, variant):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    extra = ""
    if variant == "glossy":
        extra = ('Material "conductor" "float roughness" 0.2\n'
                 'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.6 0.01 -0.4  0.2 0.01 -0.4  0.2 0.01 0.4  -0.6 0.01 0.4]')
    sc = pa.Scene.from_string(scene(extra=extra), SCENES)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(a, oracle_rgb(oracle, sc))
    print(f"portal ({variant}): {frac*100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")
