"""Scene-file `Option` and `Attribute` directives.

Option (BasicSceneBuilder::Option, scene.cpp:492-560; the name normalised as util/args.h:23-30
does, the value one raw token, parser.cpp:877-880) with the wavefront integrator's refusals
(wavefront/integrator.cpp:202-212):
* disablepixeljitter -- every camera sample at the pixel centre, lens centre, filter weight 1
  (GetCameraSample, samplers.h:807-812), and the full-pixel footprint in Approximate_dp_dxy
  (cameras.h:187-190);
* disablewavelengthjitter -- lu = 0.5 (wavefront/camera.cpp:55);
* disabletexturefiltering -- zero uv differentials (wavefront/surfscatter.cpp:77);
* seed -- Options->seed, the default of every sampler's "seed" (samplers.cpp:73 etc.);
* rendercoordsys -- camera / cameraworld / world rendering space (cameras.cpp:43-73);
* forcediffuse, pixelstats, msereferenceimage -- refused, as the wavefront integrator refuses them;
* wavefront, displacementedgescale, msereferenceout -- accepted (no effect on this path);
* anything else -- "unknown option".

Attribute "shape" | "light" | "material" | "medium" | "texture" (scene.cpp:189-215): parameters
appended to the graphics state's list for that target, scoped by AttributeBegin/End, consulted after
a directive's own parameters (latest attribute first, paramdict.cpp:150-159), never reported as
unused."""
import numpy as np
import pytest

from conftest import SCENES

HEAD = """LookAt 0 0 -4  0 0 0  0 1 0
Camera "perspective" "float fov" 30
Film "rgb" "integer xresolution" {res} "integer yresolution" {res}
Sampler "halton" "integer pixelsamples" {spp}
Integrator "volpath" "integer maxdepth" {maxdepth}
"""


def scene(body, opts="", res=24, spp=8, maxdepth=5, world_head='LightSource "infinite" "rgb L" [0.4 0.45 0.5]\n'):
    return opts + HEAD.format(res=res, spp=spp, maxdepth=maxdepth) + "WorldBegin\n" + world_head + body


SPHERES = """AttributeBegin
  Material "diffuse" "rgb reflectance" [0.7 0.3 0.2]
  Translate -0.6 0 0
  Shape "sphere" "float radius" 0.5
AttributeEnd
AttributeBegin
  Material "conductor" "float roughness" 0.2
  Translate 0.6 0 0
  Shape "sphere" "float radius" 0.5
AttributeEnd
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [4 4 4]
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 1.5 -1  1 1.5 -1  1 1.5 1  -1 1.5 1]
AttributeEnd
"""


def rgb(oracle, sc, **kw):
    f = sc.flat()
    return oracle.film_to_rgb(oracle.render(sc, threads=8, **kw), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


# ------------------------------------------------------------------------------------ Option
def test_option_seed_precedence(pa):
    """Options->seed: --seed (the "seed" override), then a scene's Option "seed" (parsed later), and
    a sampler's own "integer seed" over both."""
    base = scene(SPHERES)
    assert pa.Scene.from_string(base, SCENES).info.seed == 0
    assert pa.Scene.from_string('Option "seed" 5\n' + base, SCENES).info.seed == 5
    assert pa.Scene.from_string('Option "seed" 5\n' + base, SCENES, seed=3).info.seed == 5
    assert pa.Scene.from_string(base, SCENES, seed=3).info.seed == 3
    own = base.replace('Sampler "halton"', 'Sampler "halton" "integer seed" 7')
    assert pa.Scene.from_string('Option "seed" 5\n' + own, SCENES).info.seed == 7


def test_option_seed_changes_the_image(pa, oracle):
    a = rgb(oracle, pa.Scene.from_string(scene(SPHERES), SCENES))
    b = rgb(oracle, pa.Scene.from_string(scene(SPHERES, 'Option "seed" 1\n'), SCENES))
    c = rgb(oracle, pa.Scene.from_string(scene(SPHERES), SCENES, seed=1))
    assert not np.array_equal(a, b)
    np.testing.assert_array_equal(b, c)


def test_option_names_are_normalised(pa):
    for name in ("disablepixeljitter", "disable-pixel-jitter", "Disable_Pixel_Jitter"):
        sc = pa.Scene.from_string(scene(SPHERES, f'Option "{name}" true\n'), SCENES)
        assert sc.flat().options & 1


@pytest.mark.parametrize("opt,match", [
    ('Option "forcediffuse" true', "force-diffuse"),
    ('Option "pixelstats" true', "pixelstats"),
    ('Option "msereferenceimage" "ref.exr"', "mse-reference-image"),
    ('Option "rendercoordsys" "screen"', "unknown rendering coordinate system"),
    ('Option "rendercoordsys" world', "quoted string"),
    ('Option "disablepixeljitter" 1', "true"),
    ('Option "disablepixeljitter" "true"', "true"),
    ('Option "displacementedgescale" "x"', "floating-point"),
    ('Option "bogus" true', "unknown option"),
])
def test_option_refusals(pa, opt, match):
    with pytest.raises(RuntimeError, match=match):
        pa.Scene.from_string(scene(SPHERES, opt + "\n"), SCENES)


@pytest.mark.parametrize("opt", ['Option "forcediffuse" false', 'Option "pixelstats" false', 'Option "wavefront" true',
                                 'Option "wavefront" false', 'Option "displacementedgescale" 2.5',
                                 'Option "msereferenceout" "mse.txt"', 'Option "rendercoordsys" "cameraworld"'])
def test_options_without_effect_are_accepted(pa, oracle, opt):
    ref = rgb(oracle, pa.Scene.from_string(scene(SPHERES), SCENES))
    got = rgb(oracle, pa.Scene.from_string(scene(SPHERES, opt + "\n"), SCENES))
    np.testing.assert_array_equal(got, ref)


EDGE = """AttributeBegin
  AreaLightSource "diffuse" "rgb L" [1 1 1] "bool twosided" true
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-0.37 -0.41 0  0.53 -0.41 0  0.53 0.47 0  -0.37 0.47 0]
AttributeEnd
"""


def test_disablepixeljitter_known_answer(pa, oracle):
    """Emission seen directly (maxdepth 1, black sky): with the pixel jitter off every sample of a
    pixel takes the pixel-centre ray, so each pixel shows all or nothing of the emitter; with it on,
    the pixels along the emitter's edges are fractional."""
    kw = dict(maxdepth=1, spp=16, world_head="")
    on = rgb(oracle, pa.Scene.from_string(scene(EDGE, **kw), SCENES))[..., 1]
    off = rgb(oracle, pa.Scene.from_string(scene(EDGE, 'Option "disablepixeljitter" true\n', **kw), SCENES))[..., 1]
    lit = off.max()
    assert lit > 0
    frac_off = (off > 1e-6) & (off < lit * (1 - 1e-3))
    assert frac_off.sum() == 0
    assert ((on > 1e-6) & (on < lit * 0.9)).sum() > 10  # antialiased edges
    assert abs((off > 0).mean() - (on > 0).mean()) < 0.2


def test_disablewavelengthjitter_known_answer(pa, oracle):
    """With both jitters off every sample of a pixel is the same path (one ray, the same 31
    wavelengths), so an emitter seen directly gives the 1-spp value at any sample count."""
    opts = 'Option "disablepixeljitter" true\nOption "disablewavelengthjitter" true\n'
    kw = dict(maxdepth=1, world_head="")
    one = rgb(oracle, pa.Scene.from_string(scene(EDGE, opts, spp=1, **kw), SCENES))
    many = rgb(oracle, pa.Scene.from_string(scene(EDGE, opts, spp=8, **kw), SCENES))
    np.testing.assert_allclose(many, one, rtol=1e-6)
    jit = rgb(oracle, pa.Scene.from_string(scene(EDGE, 'Option "disablepixeljitter" true\n', spp=8, **kw), SCENES))
    assert not np.allclose(jit, one, rtol=1e-6)


TEXTURED = """Texture "checks" "spectrum" "imagemap" "string filename" "textures/bricks_rgb8.png" "string filter" "{filt}"
  "float uscale" 6 "float vscale" 6
AttributeBegin
  Material "diffuse" "texture reflectance" "checks"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-4 -1 -1  4 -1 -1  4 -1 8  -4 -1 8]
    "point2 uv" [0 0 1 0 1 1 0 1]
AttributeEnd
"""


def _textured(pa, filt, opts=""):
    return pa.Scene.from_string(scene(TEXTURED.format(filt=filt), opts, spp=4), SCENES)


def test_disabletexturefiltering_known_answer(pa, oracle):
    """Zero uv differentials: a trilinear lookup then reads the finest level bilinearly, which is
    the bilinear filter's lookup -- the same bits; without the option the grazing floor's trilinear
    lookups blur."""
    if not (SCENES / "textures" / "bricks_rgb8.png").exists():
        pytest.skip("no checker texture")
    opt = 'Option "disabletexturefiltering" true\n'
    tri = rgb(oracle, _textured(pa, "trilinear", opt))
    bil = rgb(oracle, _textured(pa, "bilinear", opt))
    np.testing.assert_array_equal(tri, bil)
    tri_on = rgb(oracle, _textured(pa, "trilinear"))
    assert not np.array_equal(tri_on, tri)


def test_rendercoordsys(pa, oracle):
    """The three rendering spaces render the same image up to float rounding of the transforms."""
    ref = rgb(oracle, pa.Scene.from_string(scene(SPHERES, spp=16), SCENES))
    for cs in ("camera", "world"):
        sc = pa.Scene.from_string(scene(SPHERES, f'Option "rendercoordsys" "{cs}"\n', spp=16), SCENES)
        img = rgb(oracle, sc)
        assert abs(img.mean() / ref.mean() - 1) < 0.02, cs
        assert np.mean(np.abs(img - ref) <= 1e-3 * np.abs(ref) + 1e-4) > 0.5, cs


# ------------------------------------------------------------------------------------ Attribute
def test_attribute_shape_defaults(pa, oracle):
    explicit = scene('Shape "sphere" "float radius" 0.8\n')
    via_attr = scene('Attribute "shape" "float radius" 0.8\nShape "sphere"\n')
    own_wins = scene('Attribute "shape" "float radius" 0.3\nShape "sphere" "float radius" 0.8\n')
    latest = scene('Attribute "shape" "float radius" 0.3\nAttribute "shape" "float radius" 0.8\nShape "sphere"\n')
    ref = rgb(oracle, pa.Scene.from_string(explicit, SCENES))
    for t in (via_attr, own_wins, latest):
        np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(t, SCENES)), ref)
    scoped = scene('AttributeBegin\nAttribute "shape" "float radius" 0.3\nAttributeEnd\nShape "sphere" "float radius" 0.8\n')
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scoped, SCENES)), ref)
    default = scene('AttributeBegin\nAttribute "shape" "float radius" 0.3\nAttributeEnd\nShape "sphere"\n')
    assert not np.array_equal(rgb(oracle, pa.Scene.from_string(default, SCENES)), ref)


def test_attribute_material_light_medium_texture(pa, oracle):
    mat = ('Material "diffuse" "rgb reflectance" [0.2 0.6 0.3]\nShape "sphere" "float radius" 0.8\n')
    mat_attr = ('Attribute "material" "rgb reflectance" [0.2 0.6 0.3]\nMaterial "diffuse"\n'
                'Shape "sphere" "float radius" 0.8\n')
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scene(mat_attr), SCENES)),
                                  rgb(oracle, pa.Scene.from_string(scene(mat), SCENES)))
    sky = 'LightSource "infinite" "rgb L" [0.4 0.45 0.5] "float scale" 2\n'
    sky_attr = 'Attribute "light" "float scale" 2\nLightSource "infinite" "rgb L" [0.4 0.45 0.5]\n'
    body = 'Shape "sphere" "float radius" 0.8\n'
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scene(body, world_head=sky_attr), SCENES)),
                                  rgb(oracle, pa.Scene.from_string(scene(body, world_head=sky), SCENES)))
    area = 'AttributeBegin\nAreaLightSource "diffuse" "rgb L" [3 3 3]\nShape "sphere" "float radius" 0.3\nAttributeEnd\n'
    area_attr = ('AttributeBegin\nAttribute "light" "rgb L" [3 3 3]\nAreaLightSource "diffuse"\n'
                 'Shape "sphere" "float radius" 0.3\nAttributeEnd\n')
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scene(area_attr, world_head=""), SCENES)),
                                  rgb(oracle, pa.Scene.from_string(scene(area, world_head=""), SCENES)))
    med = ('MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.2 0.2 0.2] "rgb sigma_s" [1 1 1]\n'
           'AttributeBegin\nMediumInterface "m" ""\nMaterial "interface"\nShape "sphere" "float radius" 0.8\nAttributeEnd\n')
    med_attr = ('Attribute "medium" "rgb sigma_s" [1 1 1]\n'
                'MakeNamedMedium "m" "string type" "homogeneous" "rgb sigma_a" [0.2 0.2 0.2]\n'
                'AttributeBegin\nMediumInterface "m" ""\nMaterial "interface"\nShape "sphere" "float radius" 0.8\nAttributeEnd\n')
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scene(med_attr), SCENES)),
                                  rgb(oracle, pa.Scene.from_string(scene(med), SCENES)))
    tex = ('Texture "c" "spectrum" "checkerboard" "float uscale" 8 "float vscale" 8 "rgb tex1" [0.9 0.1 0.1]\n'
           'Material "diffuse" "texture reflectance" "c"\nShape "sphere" "float radius" 0.8\n')
    tex_attr = ('Attribute "texture" "float uscale" 8\nAttribute "texture" "float vscale" 8\n'
                'Texture "c" "spectrum" "checkerboard" "rgb tex1" [0.9 0.1 0.1]\n'
                'Material "diffuse" "texture reflectance" "c"\nShape "sphere" "float radius" 0.8\n')
    np.testing.assert_array_equal(rgb(oracle, pa.Scene.from_string(scene(tex_attr), SCENES)),
                                  rgb(oracle, pa.Scene.from_string(scene(tex), SCENES)))


def test_attribute_unused_is_not_an_error(pa):
    pa.Scene.from_string(scene('Attribute "shape" "float radius" 0.8 "float bogus" 3\n'
                               'Shape "trianglemesh" "integer indices" [0 1 2] "point3 P" [0 0 0 1 0 0 0 1 0]\n'), SCENES)
    with pytest.raises(RuntimeError, match="not supported"):  # a directive's own unused parameter still is
        pa.Scene.from_string(scene('Shape "sphere" "float bogus" 3\n'), SCENES)


def test_attribute_unknown_target(pa):
    with pytest.raises(RuntimeError, match="Unknown attribute target"):
        pa.Scene.from_string(scene('Attribute "camera" "float fov" 20\n'), SCENES)


# ------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("opts", ['Option "disablepixeljitter" true', 'Option "disablewavelengthjitter" true',
                                  'Option "seed" 9', 'Option "rendercoordsys" "world"',
                                  'Option "rendercoordsys" "camera"'])
def test_options_gpu_match_oracle(pa, oracle, opts):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = pa.Scene.from_string(scene(SPHERES, opts + "\n", res=48, spp=16), SCENES)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(gpu, oracle_rgb(oracle, sc))
    print(f"{opts}: {frac * 100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_disabletexturefiltering_gpu_matches_oracle(pa, oracle):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    if not (SCENES / "textures" / "bricks_rgb8.png").exists():
        pytest.skip("no checker texture")
    for filt in ("trilinear", "ewa"):
        sc = _textured(pa, filt, 'Option "disabletexturefiltering" true\n')
        gpu, _ = gpu_rgb(pa, oracle, sc)
        check(gpu, oracle_rgb(oracle, sc))
