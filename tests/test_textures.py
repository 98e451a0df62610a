"""Textures: image and procedural textures on the wavefront material stage.

CPU tests pin the pieces: the PNG / PFM readers against an independent decoder (PIL) and the
generator's arrays, the MIPMap pyramid (product vs the oracle's own build, byte for byte), the
camera's minimum differentials (product vs oracle), the texture evaluation at random hits
(product's shared host/device code vs the oracle's recursive restatement, bit for bit), the
reference data tables, loader semantics (scale folding, errors) and known answers.
GPU tests render the textured Cornell box against the oracle at test_gpu_parity's tolerance.

Parity with pbrt itself: util/image.cpp and util/mipmap.cpp need OpenEXR / lodepng / stb,
which are empty submodules here, so the pyramid and filtering are restated, not pinned; the
tables they read (SRGBToLinearLUT, MIPFilterLUT) are the reference's literals, and the
RGB->spectrum table is the rgb2spec_opt output pinned by the golden columns."""
import numpy as np
import pytest

from conftest import SCENES

LAMBDAS = np.linspace(395, 705, 31).astype(np.float32)


@pytest.fixture(scope="module")
def tex_scene(pa):
    return pa.load_scene(SCENES / "textured.pbrt")


def _gen():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_textured", SCENES / "gen_textured.py")
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _raw(flat, i):
    info = np.ctypeslib.as_array(flat.image_raw_info, shape=(flat.n_images * 8,)).reshape(-1, 8)[i]
    w, h, fmt, nc = info[:4]
    off = flat.image_raw_offset[i]
    n = int(w) * int(h) * int(nc) * [1, 2, 4][fmt]
    buf = np.ctypeslib.as_array(flat.image_raw_data, shape=(off + n,))[off:off + n]
    dt = [np.uint8, np.float16, np.float32][fmt]
    return buf.view(dt).reshape(h, w, nc), info


def test_png_and_pfm_readers_match_independent_decoders(tex_scene):
    from PIL import Image
    f = tex_scene.flat()
    # image order in the scene: bricks, marble, bumps, tiles, sky, gloss
    bricks, _ = _raw(f, 0)
    assert np.array_equal(bricks, np.asarray(Image.open(SCENES / "textures/bricks_rgb8.png").convert("RGB")))
    marble, info = _raw(f, 1)
    assert info[3] == 3  # RGBA with alpha 1 everywhere drops to RGB (mipmap.cpp:395-403)
    assert np.array_equal(marble, np.asarray(Image.open(SCENES / "textures/marble_rgba8.png"))[..., :3])
    tiles, _ = _raw(f, 3)
    assert np.array_equal(tiles, np.asarray(Image.open(SCENES / "textures/tiles_pal.png").convert("RGB")))
    # 16-bit grey: Half(SRGBToLinear(v / 65535)) (image.cpp:1287-1297)
    bumps, info = _raw(f, 2)
    assert info[2] == 1 and info[3] == 1
    src = np.asarray(Image.open(SCENES / "textures/bumps_grey16.png")).astype(np.float64) / 65535
    lin = np.where(src <= 0.04045, src / 12.92, ((src + 0.055) / 1.055) ** 2.4)
    assert np.abs(bumps[..., 0].astype(np.float64) - lin).max() < 2e-3
    # PFM: rows bottom-up, |scale| applied
    sky, _ = _raw(f, 4)
    y, x = np.mgrid[0:8, 0:16]
    ref = np.stack([0.2 + 0.1 * x, 0.3 + 0.05 * y, 0.9 - 0.02 * x], axis=-1).astype(np.float32)
    assert np.array_equal(sky, ref)


def test_mipmap_pyramids_match_oracle(tex_scene, oracle):
    """Image::GeneratePyramid: the product's stored levels equal the oracle's own build (both
    re-quantise every level into the file's pixel format, as pbrt does)."""
    f = tex_scene.flat()
    info = np.ctypeslib.as_array(f.image_info, shape=(f.n_images * 8,)).reshape(-1, 8)
    nlev = int(info[:, 2].sum())
    lv = np.ctypeslib.as_array(f.image_levels, shape=(nlev * 4,)).reshape(-1, 4)
    for i in range(f.n_images):
        fmt, nc, nl, _, base = info[i][:5]
        bpp = [1, 2, 4][fmt] * nc
        for level in range(nl):
            w, h, lo, hi = lv[base + level]
            off = (int(hi) << 32) | (int(lo) & 0xffffffff)
            prod = np.ctypeslib.as_array(f.image_data, shape=(off + w * h * bpp,))[off:]
            orc, ow, oh = oracle.image_level(tex_scene, i, level)
            assert (ow, oh) == (w, h)
            assert np.array_equal(prod, orc), (i, level)
    # non-power-of-two images were resampled up: bricks 48x40 -> 64x64 base, 7 levels
    assert tuple(lv[info[0][4]][:2]) == (64, 64) and info[0][2] == 7


def test_camera_minimum_differentials_match_oracle(tex_scene, oracle):
    f = tex_scene.flat()
    prod = np.array(f.camera_min_diff, dtype=np.float32)
    assert np.array_equal(prod, oracle.camera_min_diff(tex_scene))
    # a pinhole camera: no position differential; the direction differentials are about one
    # pixel's angle (fov 39.3 deg over 128 px, FindMinimumDifferentials takes the smallest)
    assert np.all(prod[:6] == 0)
    assert 1e-3 < np.linalg.norm(prod[6:9]) < 1e-2


def _random_hits(rng, n):
    for _ in range(n):
        p = rng.uniform([-300, -280, 780], [300, 280, 1370])
        nrm = rng.normal(size=3)
        nrm /= np.linalg.norm(nrm)
        dpdu = rng.normal(size=3) * rng.uniform(10, 600)
        dpdv = rng.normal(size=3) * rng.uniform(10, 600)
        uv = rng.uniform(-0.5, 1.5, 2)
        yield np.concatenate([p, nrm, dpdu, dpdv, uv]).astype(np.float32)


def test_texture_eval_matches_oracle_bitwise(tex_scene, oracle):
    """Every textured parameter of the scene (image / checkerboard / mix / scale / bilerp /
    directionmix / planar mapping; point, bilinear, trilinear and EWA filtering; 8-bit, half
    and float pyramids) at 400 random hits: the product's device code run on the host equals
    the oracle's restatement exactly, differentials included."""
    f = tex_scene.flat()
    mt = np.ctypeslib.as_array(f.material_tex, shape=(f.n_materials * 4,)).reshape(-1, 4)
    rng = np.random.default_rng(3)
    checked = 0
    for m in range(f.n_materials):
        for slot in range(3):
            if mt[m][slot] < 0:
                continue
            for hit in _random_hits(rng, 400):
                d1, v1 = tex_scene.texture_eval(m, slot, hit, LAMBDAS)
                d2, v2 = oracle.texture_eval(tex_scene, m, slot, hit, LAMBDAS)
                assert np.array_equal(d1, d2), (m, slot, hit)
                assert np.array_equal(np.atleast_1d(v1), np.atleast_1d(v2)), (m, slot, hit)
                checked += 1
    assert checked >= 11 * 400


def test_reference_tables_are_the_literals(pa):
    data = (pa.DATA_DIR / "spectral_data.txt").read_text().splitlines()
    tabs = {ln.split()[0]: np.array(ln.split()[2:], dtype=np.float64) for ln in data}
    lut = tabs["SRGBToLinearLUT"]
    assert lut.size == 256 and lut[0] == 0 and lut[255] == 1
    # the literals follow the sRGB curve to their printed precision
    v = np.arange(256) / 255
    assert np.abs(lut - np.where(v <= 0.04045, v / 12.92, ((v + 0.055) / 1.055) ** 2.4)).max() < 1e-6
    ewa = tabs["MIPFilterLUT"]
    assert ewa.size == 128 and ewa[-1] == 0
    assert np.abs(ewa - (np.exp(-2 * np.arange(128) / 127) - np.exp(-2))).max() < 1e-6


def test_full_rgb_table_matches_column_generator(pa):
    """data/rgbspec_srgb.bin (the table the texture kernels read) holds exactly the columns of
    the rgb2spec_opt restatement that the golden rgb2spec columns pin."""
    import ctypes
    table = np.fromfile(pa.DATA_DIR / "rgbspec_srgb.bin", dtype=np.float32)
    assert table.size == 64 + 3 * 64 ** 3 * 3
    data = table[64:].reshape(3, 64, 64, 64, 3)
    rng = np.random.default_rng(5)
    for _ in range(6):
        l, j, i = rng.integers(0, 3), rng.integers(0, 64), rng.integers(0, 64)
        col = (ctypes.c_float * 192)()
        assert pa._lib().pbrt_debug_rgb2spec_column(int(l), int(j), int(i), col) == 0
        assert np.array_equal(np.array(col[:], np.float32).reshape(64, 3), data[l, :, j, i, :])


def test_scale_texture_folds_into_image_scale(tex_scene):
    """SpectrumScaledTexture::Create (textures.cpp:971-1001): a constant scale of an image
    texture becomes the image's own scale -- "tiles80" is an imagemap node with scale 0.8."""
    f = tex_scene.flat()
    mt = np.ctypeslib.as_array(f.material_tex, shape=(f.n_materials * 4,)).reshape(-1, 4)
    info = np.ctypeslib.as_array(f.tex_node_info, shape=(f.n_tex_nodes * 8,)).reshape(-1, 8)
    par = np.ctypeslib.as_array(f.tex_node_params, shape=(f.n_tex_nodes * 28,)).reshape(-1, 28)
    right = mt[3][0]  # MakeNamedMaterial "right": texture reflectance "tiles80"
    assert info[right][0] == 6 and par[right][26] == np.float32(0.8)


BASE = """LookAt 0 0 -5  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" 24 "integer yresolution" 16
Sampler "halton" "integer pixelsamples" 4
WorldBegin
LightSource "infinite" "rgb L" [1 1 1]
"""
QUAD = 'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0 1 -1 0 1 1 0 -1 1 0]\n'


@pytest.mark.parametrize("body, msg", [
    ('Texture "t" "spectrum" "fbm"\nMaterial "diffuse" "texture reflectance" "t"\n', "not supported"),
    ('Material "diffuse" "texture reflectance" "nope"\n', "Couldn't find spectrum texture"),
    ('Texture "t" "spectrum" "constant" "rgb value" [2 0 0]\nMaterial "diffuse" "texture reflectance" "t"\n',
     "albedo has > 1 component"),
    ('Texture "t" "color" "constant"\n', "texture type unknown"),
    ('Texture "t" "float" "constant"\nTexture "t" "float" "constant"\n', "Redefining texture"),
    ('Texture "t" "spectrum" "imagemap" "string filename" "textures/missing.png"\n'
     'Material "diffuse" "texture reflectance" "t"\n', "unable to open"),
])
def test_texture_loader_errors(pa, body, msg):
    with pytest.raises(pa.PbrtError, match=msg):
        pa.Scene.from_string(BASE + body + QUAD, SCENES)


def test_constant_texture_renders_like_rgb_reflectance(pa, oracle):
    """A "constant" spectrum texture of an rgb value is the same SpectrumConstantTexture pbrt
    builds for an "rgb reflectance" parameter: the oracle's films are bit-identical."""
    a = pa.Scene.from_string(BASE + 'Material "diffuse" "rgb reflectance" [0.7 0.3 0.2]\n' + QUAD, SCENES)
    b = pa.Scene.from_string(BASE + 'Texture "c" "spectrum" "constant" "rgb value" [0.7 0.3 0.2]\n'
                             'Material "diffuse" "texture reflectance" "c"\n' + QUAD, SCENES)
    assert np.array_equal(oracle.render(a, threads=4), oracle.render(b, threads=4))


def test_checkerboard_known_answer(pa, oracle):
    """A 2x2 checkerboard of albedo 1 and 0 seen under a uniform sky of radiance 1: pixels deep
    inside a white square reflect about 1 (single-bounce furnace), inside a black one 0."""
    text = (BASE.replace("xresolution\" 24", "xresolution\" 32").replace("yresolution\" 16", "yresolution\" 32")
            .replace('"perspective" "float fov" 40', '"perspective" "float fov" 22')
            + 'Texture "c" "spectrum" "checkerboard" "float uscale" 2 "float vscale" 2 '
              '"rgb tex1" [1 1 1] "rgb tex2" [0 0 0]\nMaterial "diffuse" "texture reflectance" "c"\n'
            + 'Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0 1 -1 0 1 1 0 -1 1 0] '
              '"point2 uv" [0 0 1 0 1 1 0 1]\n')
    sc = pa.Scene.from_string(text.replace('"integer pixelsamples" 4', '"integer pixelsamples" 16')
                              .replace("WorldBegin", 'Integrator "volpath" "integer maxdepth" 1\nWorldBegin'), SCENES)
    f = sc.flat()
    img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    # the camera looks down +z at the quad: image x runs along -u (Scale-free LookAt), so the
    # white (tex1 where floor(s) + floor(t) is even) quadrants are where u, v are both < .5 or > .5
    lum = img.mean(axis=-1)
    q = [lum[4:12, 4:12].mean(), lum[4:12, 20:28].mean(), lum[20:28, 4:12].mean(), lum[20:28, 20:28].mean()]
    assert sorted(q)[:2] == pytest.approx([0, 0], abs=1e-6)
    assert sorted(q)[2:] == pytest.approx([1, 1], abs=0.03)


@pytest.mark.gpu
def test_textured_scene_matches_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    sc = pa.load_scene(SCENES / "textured.pbrt")
    film, _ = gpu_film(pa, sc)
    ref = oracle.render(sc, threads=16)
    frac, mean_rel = check_parity(to_rgb(oracle, sc, film), to_rgb(oracle, sc, ref))
    print(f"textured Cornell parity: {frac*100:.3f}% pixels within 1e-3, mean rel {mean_rel:.2e}")


@pytest.mark.gpu
def test_textured_zsobol_rows_match_oracle_gpu(pa, oracle):
    from test_gpu_parity import check_parity, gpu_film, to_rgb
    text = (SCENES / "textured.pbrt").read_text().replace(
        'Sampler "halton" "integer pixelsamples" [ 16 ]', 'Sampler "zsobol" "integer pixelsamples" [ 8 ]')
    sc = pa.Scene.from_string(text, SCENES, xresolution=320, yresolution=240)
    rows = np.arange(100, 140, dtype=np.int32)
    film, _ = gpu_film(pa, sc, rows=rows)
    ref = oracle.render(sc, rows=rows, threads=16)
    check_parity(to_rgb(oracle, sc, film)[100:140], to_rgb(oracle, sc, ref)[100:140])


@pytest.mark.gpu
def test_constant_texture_film_bit_identical_gpu(pa):
    """The textured kernels with a constant texture give the same film bits as the untextured
    kernels with the rgb reflectance."""
    from test_gpu_parity import gpu_film
    a = pa.Scene.from_string(BASE + 'Material "diffuse" "rgb reflectance" [0.7 0.3 0.2]\n' + QUAD, SCENES)
    b = pa.Scene.from_string(BASE + 'Texture "c" "spectrum" "constant" "rgb value" [0.7 0.3 0.2]\n'
                             'Material "diffuse" "texture reflectance" "c"\n' + QUAD, SCENES)
    fa, _ = gpu_film(pa, a)
    fb, _ = gpu_film(pa, b)
    assert np.array_equal(fa, fb)
