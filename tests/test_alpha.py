"""Alpha-tested geometry (GeometricPrimitive alpha: scene.cpp:1369-1384 getAlphaTexture,
cpu/primitive.cpp:56-80; the GPU any-hit programs gpu/optix.cu:197-243, 368-381, 449-461): the
loader's "float alpha" / "texture alpha", the oracle's restatement against known answers, and
GPU parity of closest hits, any-hit shadow rays, films (surface and volumetric kernels) and the
C-ABI intersector against the oracle.

Semantics are pbrt's GPU ones: every candidate hit is tested against its alpha texture at the
candidate's SurfaceInteraction (no derivatives); alpha <= 0 kills it, alpha < 1 kills it when
HashFloat(ray o, ray d) > alpha, so a ray keeps the nearest surviving candidate and a shadow ray
is blocked by any surviving one (pbrt's CPU aggregate instead re-spawns the ray past a killed
hit, which draws a new hash per crossing)."""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 1 -5  0 0.5 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 96 "integer yresolution" 64
Sampler "halton" "integer pixelsamples" 16
Integrator "volpath" "integer maxdepth" 5
WorldBegin
LightSource "infinite" "rgb L" [0.3 0.3 0.35]
AttributeBegin
AreaLightSource "diffuse" "rgb L" [6 6 6]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.5 3 -0.5 0.5 3 -0.5 0.5 3 0.5 -0.5 3 0.5]
AttributeEnd
Material "diffuse" "rgb reflectance" [0.6 0.6 0.6]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-4 0 -4 4 0 -4 4 0 4 -4 0 4]
"""

LEAVES = """Texture "leaf" "float" "imagemap" "string filename" "leaf.png" "string encoding" "linear"
Material "diffuse" "rgb reflectance" [0.2 0.6 0.2]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1.5 0.2 0.3 0 0.2 0.3 0 1.7 0.6 -1.5 1.7 0.6]
    "point2 uv" [0 0 1 0 1 1 0 1] "texture alpha" "leaf"
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [0.2 0.1 -0.5 1.6 0.1 -0.3 1.6 1.5 0 0.2 1.5 -0.2]
    "point2 uv" [0 0 2 0 2 2 0 2] "texture alpha" "leaf"
Material "diffuse" "rgb reflectance" [0.7 0.3 0.2]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.4 0.05 -1.2 0.4 0.05 -1.2 0.4 0.9 -1 -0.4 0.9 -1]
    "float alpha" 0.5
AttributeBegin
Translate 1.4 0.6 1.2
Material "conductor" "float roughness" 0.2
Shape "sphere" "float radius" 0.5 "texture alpha" "leaf"
AttributeEnd
AttributeBegin
Translate -1.6 0.2 -1
Shape "bilinearmesh" "point3 P" [-0.5 0 -0.4  0.5 0.3 -0.4  -0.4 0.9 0.5  0.4 1.1 0.3] "texture alpha" "leaf"
AttributeEnd
"""


def write_leaf(path, n=64):
    """An 8-bit grey alpha map: a disc of 1 with a soft rim (0 < alpha < 1) and holes of 0."""
    from PIL import Image
    y, x = np.mgrid[0:n, 0:n]
    r = np.hypot(x - n / 2 + 0.5, y - n / 2 + 0.5) / (n / 2)
    a = np.clip((1.0 - r) * 4, 0, 1)
    a[(x // 8 + y // 8) % 5 == 0] = 0
    Image.fromarray((a * 255).astype(np.uint8), mode="L").save(path)


def _scene(pa, tmp_path, body=LEAVES, head=HEAD, **kw):
    write_leaf(tmp_path / "leaf.png")
    return pa.Scene.from_string(head + body, tmp_path, **kw)


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def _prim_alpha(sc):
    f = sc.flat()
    n = f.n_triangles + f.n_shapes
    return np.ctypeslib.as_array(f.prim_alpha, shape=(n,)).copy() if f.prim_alpha else None


def test_alpha_loader(pa, tmp_path):
    sc = _scene(pa, tmp_path)
    f = sc.flat()
    pa_ = _prim_alpha(sc)
    assert (f.n_triangles, f.n_shapes) == (10, 2)
    # emitter and floor: none; the two leaves share the texture's node; the pane a constant node
    assert (pa_[:4] == -1).all()
    assert len(set(pa_[4:8])) == 1 and pa_[4] >= 0
    assert pa_[8] == pa_[9] and pa_[8] >= 0 and pa_[8] != pa_[4]
    assert pa_[10] == pa_[4] and pa_[11] == pa_[4]  # sphere and patch
    # "float alpha" 1 is no alpha test at all (scene.cpp: alpha < 1 only)
    sc1 = pa.Scene.from_string(HEAD + 'Shape "sphere" "float alpha" 1\n', SCENES)
    assert not sc1.flat().prim_alpha


@pytest.mark.parametrize("body, msg", [
    ('Shape "sphere" "texture alpha" "nope"\n', "couldn't find float texture"),
    ('Shape "sphere" "rgb alpha" [1 1 1]\n', "must be a float or a texture"),
    ('AttributeBegin\nAreaLightSource "diffuse"\nShape "sphere" "float alpha" 0.5\nAttributeEnd\n',
     "alpha\\\" on area lights"),
])
def test_alpha_loader_errors(pa, body, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(HEAD + body, SCENES)


def test_alpha_zero_and_one_known_answers(pa, oracle, tmp_path):
    """A shape with alpha 0 is invisible (every candidate killed: the film equals the scene
    without it, bit for bit), alpha 1 is opaque (the film equals the scene without the
    parameter)."""
    occluder = ('Material "diffuse" "rgb reflectance" [0.9 0.1 0.1]\n'
                'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] '
                '"point3 P" [-1 0.1 -1 1 0.1 -1 1 1.5 0 -1 1.5 0]')
    kw = dict(xresolution=48, yresolution=32, spp=8)
    base = oracle.render(pa.Scene.from_string(HEAD, SCENES, **kw), threads=8)
    zero = oracle.render(pa.Scene.from_string(HEAD + occluder + ' "float alpha" 0\n', SCENES, **kw), threads=8)
    one = oracle.render(pa.Scene.from_string(HEAD + occluder + ' "float alpha" 1\n', SCENES, **kw), threads=8)
    opaque = oracle.render(pa.Scene.from_string(HEAD + occluder + '\n', SCENES, **kw), threads=8)
    assert np.array_equal(zero, base)
    assert np.array_equal(one, opaque)
    assert not np.array_equal(opaque, base)


def test_half_alpha_pane_transmits_half(pa, oracle):
    """A black pane of alpha 0.5 filling the view in front of a uniform emitter: half of the
    camera rays survive (HashFloat is uniform), so the image is half the emitter's radiance."""
    text = """LookAt 0 0 -3  0 0 0  0 1 0
Camera "perspective" "float fov" 10
Film "rgb" "integer xresolution" 16 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 256
Integrator "volpath" "integer maxdepth" 1
WorldBegin
AttributeBegin
Material "diffuse" "rgb reflectance" [0 0 0]
AreaLightSource "diffuse" "rgb L" [1 1 1]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-5 -5 2 -5 5 2 5 5 2 5 -5 2]
AttributeEnd
Material "diffuse" "rgb reflectance" [0 0 0]
Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-5 -5 0 5 -5 0 5 5 0 -5 5 0] "float alpha" 0.5
"""
    sc = pa.Scene.from_string(text, SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8))
    assert img.mean() == pytest.approx(0.5, abs=0.01)


def test_alpha_texture_cutout_oracle(pa, oracle, tmp_path):
    """Rays through the leaf texture's holes pass, rays through its opaque disc stop: closest
    hits of rays aimed at the first leaf against the texture's value at the hit's uv."""
    sc = _scene(pa, tmp_path, body="\n".join(LEAVES.splitlines()[:4]) + "\n")  # the texture and the first leaf
    n = 4000
    rng = np.random.default_rng(1)
    uv = rng.random((n, 2)).astype(np.float32)
    # the first leaf: P0 + u (P1 - P0) + v (P3 - P0), uv = (u, v)
    p0, p1, p3 = np.array([-1.5, 0.2, 0.3]), np.array([0, 0.2, 0.3]), np.array([-1.5, 1.7, 0.6])
    target = p0 + uv[:, :1] * (p1 - p0) + uv[:, 1:] * (p3 - p0)
    eye = np.array([0, 1, -5.0])
    o = np.tile(eye, (n, 1)) - eye  # render space: world minus the eye
    d = target - eye
    rays = np.concatenate([o.T, d.T, np.full((1, n), np.inf)]).astype(np.float32)
    prim, _ = oracle.intersect(sc, rays, False)
    f = sc.flat()
    assert f.n_triangles == 6
    hit_leaf = np.isin(prim, [4, 5])
    from PIL import Image
    a = np.pad(np.asarray(Image.open(tmp_path / "leaf.png"), np.float32) / 255, 1, mode="edge")
    # level 0, bilinear: where the 3x3 texel neighbourhood is uniform the filtered alpha is
    # exactly that value (1: always kept, 0: always killed)
    tx = np.clip((uv[:, 0] * 64).astype(int), 0, 63) + 1
    ty = np.clip(((1 - uv[:, 1]) * 64).astype(int), 0, 63) + 1
    nb = np.stack([a[ty + dy, tx + dx] for dy in (-1, 0, 1) for dx in (-1, 0, 1)], 1)
    opaque, clear = (nb == 1).all(1), (nb == 0).all(1)
    assert opaque.sum() > 300 and clear.sum() > 300
    assert hit_leaf[opaque].all()
    assert not hit_leaf[clear].any()


def _gpu_rays(n, seed):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-3, 3, (n, 3)) + [0, 1, 0]
    t = rng.uniform(-1.5, 1.5, (n, 3)) + [0, 0.7, 0]
    eye = np.array([0, 1, -5.0])
    return np.concatenate([(o - eye).T, (t - o).T, np.full((1, n), np.inf)]).astype(np.float32)


@pytest.mark.gpu
def test_alpha_intersections_match_oracle_gpu(pa, oracle, tmp_path):
    """pbrt_intersect closest and any-hit on the alpha scene: ids equal the oracle's."""
    import torch
    sc = _scene(pa, tmp_path)
    integ = pa.WavefrontPathIntegrator(sc, max_paths=1 << 12)
    agg = pa.HIPAggregate(integ)
    rays = _gpu_rays(60000, 3)
    for any_hit in (False, True):
        call = agg.IntersectShadow if any_hit else agg.IntersectClosest
        gp, gh = call(torch.from_numpy(rays).cuda())
        gp, gh = gp.cpu().numpy(), gh.cpu().numpy()
        op, oh = oracle.intersect(sc, rays, any_hit)
        np.testing.assert_array_equal(gp >= 0, op >= 0)
        if not any_hit:
            np.testing.assert_array_equal(gp, op)
            hit = op >= 0
            np.testing.assert_allclose(gh[3][hit], oh[3][hit], rtol=1e-5)


@pytest.mark.gpu
def test_alpha_first_hits_match_oracle_gpu(pa, oracle, tmp_path):
    """maxdepth 0: camera rays (bit-identical to the oracle's) through the leaves onto the
    emitters and the sky; every alpha decision is the oracle's, so pixels agree to 1e-3."""
    from test_gpu_parity import check_parity, gpu_film, oracle_film, to_rgb
    head = HEAD.replace('"integer maxdepth" 5', '"integer maxdepth" 0').replace("LookAt 0 1 -5  0 0.5 0", "LookAt 0 0.3 -5  0 1.2 0")
    sc = _scene(pa, tmp_path, head=head)
    film, integ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle_film(oracle, sc, integ)))
    print(f"alpha first-hit parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_alpha_scene_matches_oracle_gpu(pa, oracle, tmp_path):
    """Five bounces through alpha-tested leaves: every candidate's keep/kill hashes the ray's
    bits, so a bounce direction one ulp off the oracle's would re-roll it: the device's
    transcendentals are the portable polynomials the oracle restates (core/detmath.h), so every
    alpha decision is the oracle's and the standard per-pixel bar applies."""
    from test_gpu_parity import check_parity, gpu_film, oracle_film, to_rgb
    sc = _scene(pa, tmp_path, spp=64)
    film, integ = gpu_film(pa, sc)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, oracle_film(oracle, sc, integ)))
    print(f"alpha 5-bounce: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_alpha_volumetric_matches_oracle_gpu(pa, oracle, tmp_path):
    """The volumetric kernels' closest hits and transmittance shadow rays with alpha-tested
    leaves beside a fog sphere."""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    body = LEAVES + ('MakeNamedMedium "fog" "string type" "homogeneous" "rgb sigma_a" [0.2 0.3 0.4] '
                     '"rgb sigma_s" [1.5 1.2 1] "float g" 0.3\nAttributeBegin\nMediumInterface "fog" ""\n'
                     'Material "interface"\nTranslate -0.3 0.8 0.8\nShape "sphere" "float radius" 0.6\nAttributeEnd\n')
    sc = _scene(pa, tmp_path, body=body, spp=64)
    a, _ = gpu_rgb(pa, oracle, sc)
    frac, mean_rel = check(a, oracle_rgb(oracle, sc))
    print(f"alpha volumetric: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")
