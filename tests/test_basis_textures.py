"""Multispectral basis image textures -- the fork's "basisfilename" (--zhenyi) on spectrum imagemap
textures, with the GPU renderer's semantics (GPUSpectrumImageTexture::Evaluate, textures.h:652-686;
basis array of GPUSpectrumImageTexture::Create, textures.cpp:1148-1176):

    value at wavelength sample i = sum over channels c of  basis[3 + i + c * 31] * (texel_c - offset)

* the basis array is {channels, first channel's basis length, int(first channel's offset[0]),
  every channel's basis values}, read with clamp addressing;
* the basis is indexed by the wavelength's *sample index* i, not by its value;
* offset is truncated to an int; the texel is the filtered RGB without "scale" / "invert";
* an empty channel array leaves the texture an ordinary RGB image (nChannels == 0).

The reference reads the file with nlohmann::json; the product has its own small reader and refuses
what the reference would choke on (malformed JSON, a channel without a numeric basis of the first
channel's length, no offset, more than 3 channels -- Evaluate reads an RGB texel).  Pinning: the
product's texture code (run on the host through pbrt_debug_texture_eval) equals the oracle's
independent restatement bit for bit, known answers below, GPU film parity at the end.  No basis file
ships with the reference, so the files here are synthetic; against pbrt's own renders this is
parity unpinned (its GPU path needs CUDA)."""
import json

import numpy as np
import pytest

from conftest import SCENES

LAMBDAS = (400 + 10 * np.arange(31) + 3.3).astype(np.float32)

HEAD = """LookAt 0 0 -3  0 0 0  0 1 0
Camera "perspective" "float fov" 40
Film "rgb" "integer xresolution" {res} "integer yresolution" {res}
Sampler "halton" "integer pixelsamples" {spp}
Integrator "volpath" "integer maxdepth" 4
WorldBegin
LightSource "infinite" "rgb L" [0.6 0.6 0.6]
AttributeBegin
  AreaLightSource "diffuse" "rgb L" [3 3 3]
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 1.6 -1  1 1.6 -1  1 1.6 1  -1 1.6 1]
AttributeEnd
"""


def write_pfm(path, rgb):
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(rgb[::-1], dtype="<f4").tobytes())


def write_basis(path, channels, offset=0.0):
    json.dump([{"basis": list(map(float, b)), "offset": [offset]} for b in channels], open(path, "w"))


def textured(tmp_path, pa, basis_file, img="img.pfm", filt="bilinear", res=24, spp=8, extra=""):
    text = HEAD.format(res=res, spp=spp) + f"""
Texture "ms" "spectrum" "imagemap" "string filename" "{img}" "string filter" "{filt}"
  "string basisfilename" "{basis_file}" "float uscale" 2 "float vscale" 2 {extra}
AttributeBegin
  Material "diffuse" "texture reflectance" "ms"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0.5  1 -1 0.5  1 1 0.5  -1 1 0.5]
    "point2 uv" [0 0 1 0 1 1 0 1]
AttributeEnd
"""
    return pa.Scene.from_string(text, tmp_path)


@pytest.fixture
def tex_dir(tmp_path):
    rng = np.random.default_rng(4)
    write_pfm(tmp_path / "img.pfm", rng.uniform(0, 1, (16, 16, 3)).astype(np.float32))
    write_pfm(tmp_path / "const.pfm", np.tile(np.array([0.5, 0.2, 0.1], np.float32), (4, 4, 1)))
    write_basis(tmp_path / "b3.json", rng.uniform(-0.5, 1, (3, 31)), offset=0.0)
    write_basis(tmp_path / "b2_36.json", rng.uniform(0, 1, (2, 36)), offset=1.7)  # int(1.7) = 1
    write_basis(tmp_path / "b1_10.json", rng.uniform(0, 1, (1, 10)))  # indices past 12 clamp
    write_basis(tmp_path / "ramp.json", [np.arange(31) / 30.0, np.zeros(31), np.zeros(31)])
    json.dump([], open(tmp_path / "empty.json", "w"))
    return tmp_path


def _mat(sc):
    """the textured material's index"""
    f = sc.flat()
    mt = np.ctypeslib.as_array(f.material_tex, shape=(f.n_materials * 4,)).reshape(-1, 4)
    return int(np.nonzero(mt[:, 0] >= 0)[0][0])


def _hits(rng, n):
    for _ in range(n):
        p = rng.uniform([-1, -1, 0.5], [1, 1, 0.5])
        yield np.concatenate([p, [0, 0, -1], [2, 0, 0], [0, 2, 0], rng.uniform(0, 1, 2)]).astype(np.float32)


@pytest.mark.parametrize("basis,filt", [("b3.json", "bilinear"), ("b3.json", "ewa"), ("b2_36.json", "trilinear"),
                                        ("b1_10.json", "point")])
def test_basis_texture_matches_oracle_bitwise(pa, oracle, tex_dir, basis, filt):
    sc = textured(tex_dir, pa, basis, filt=filt)
    rng = np.random.default_rng(8)
    for hit in _hits(rng, 300):
        d1, v1 = sc.texture_eval(_mat(sc), 0, hit, LAMBDAS)
        d2, v2 = oracle.texture_eval(sc, _mat(sc), 0, hit, LAMBDAS)
        assert np.array_equal(d1, d2)
        assert np.array_equal(v1, v2), (basis, hit, v1, v2)


def test_basis_known_answers(pa, tex_dir):
    """A constant image (0.5, 0.2, 0.1) under a ramp basis on channel 0: the value at sample i is
    0.5 i / 30 whatever the wavelengths -- the basis follows the sample index."""
    sc = textured(tex_dir, pa, "ramp.json", img="const.pfm", filt="point")
    hit = next(_hits(np.random.default_rng(1), 1))
    _, v = sc.texture_eval(_mat(sc), 0, hit, LAMBDAS)
    want = (np.arange(31) / 30.0).astype(np.float32) * (np.float32(0.5) - np.float32(0))
    np.testing.assert_array_equal(v, want.astype(np.float32))
    _, v_rev = sc.texture_eval(_mat(sc), 0, hit, LAMBDAS[::-1].copy())
    np.testing.assert_array_equal(v_rev, v)
    # "scale" and "invert" do not apply on the basis branch
    sc2 = textured(tex_dir, pa, "ramp.json", img="const.pfm", filt="point", extra='"float scale" 3 "bool invert" true')
    np.testing.assert_array_equal(sc2.texture_eval(_mat(sc2), 0, hit, LAMBDAS)[1], v)


def test_offset_truncates_and_table_clamps(pa, tex_dir):
    """int(1.7) = 1 (textures.cpp:1163); with one channel of 10 values, samples past index 9 read
    the table's last entry (clamp addressing)."""
    hit = next(_hits(np.random.default_rng(2), 1))
    sc = textured(tex_dir, pa, "b1_10.json", img="const.pfm", filt="point")
    b = np.array(json.load(open(tex_dir / "b1_10.json"))[0]["basis"], np.float32)
    _, v = sc.texture_eval(_mat(sc), 0, hit, LAMBDAS)
    idx = np.minimum(np.arange(31), 9)
    np.testing.assert_array_equal(v, b[idx] * np.float32(0.5))
    sc = textured(tex_dir, pa, "b2_36.json", img="const.pfm", filt="point")
    bb = json.load(open(tex_dir / "b2_36.json"))
    flat = np.array(bb[0]["basis"] + bb[1]["basis"], np.float32)
    _, v = sc.texture_eval(_mat(sc), 0, hit, LAMBDAS)
    i = np.arange(31)
    s = np.zeros(31, np.float32)
    for c, t in enumerate((0.5, 0.2)):
        s = (flat[np.minimum(i + 31 * c, 71)] * (np.float32(t) - np.float32(1)) + s).astype(np.float32)
    np.testing.assert_array_equal(v, s)


def test_empty_basis_is_an_rgb_texture(pa, oracle, tex_dir):
    a = textured(tex_dir, pa, "empty.json")
    text = HEAD.format(res=24, spp=8) + """
Texture "ms" "spectrum" "imagemap" "string filename" "img.pfm" "float uscale" 2 "float vscale" 2
AttributeBegin
  Material "diffuse" "texture reflectance" "ms"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0.5  1 -1 0.5  1 1 0.5  -1 1 0.5]
    "point2 uv" [0 0 1 0 1 1 0 1]
AttributeEnd
"""
    b = pa.Scene.from_string(text, tex_dir)
    assert np.array_equal(oracle.render(a, threads=4), oracle.render(b, threads=4))


@pytest.mark.parametrize("content,match", [
    ("[{\"basis\": [1, 2, 3], \"offset\": [0]", "malformed"),
    ("{\"basis\": [1]}", "array of channels"),
    ("[{\"offset\": [0]}]", "no \"basis\""),
    ("[{\"basis\": [1, 2]}]", "offset"),
    ("[{\"basis\": [1, \"x\"], \"offset\": [0]}]", "non-numeric"),
    ("[{\"basis\": [1, 2, 3], \"offset\": [0]}, {\"basis\": [1, 2]}]", "shorter"),
    (json.dumps([{"basis": [1.0], "offset": [0]}] * 4), "more than 3"),
])
def test_malformed_basis_files_are_refused(pa, tex_dir, content, match):
    (tex_dir / "bad.json").write_text(content)
    with pytest.raises(RuntimeError, match=match):
        textured(tex_dir, pa, "bad.json")


def test_basis_needs_rgb_image_and_file(pa, tex_dir):
    write_pfm(tex_dir / "grey.pfm", np.ones((4, 4, 3), np.float32))
    with pytest.raises(RuntimeError, match="cannot open"):
        textured(tex_dir, pa, "missing.json")
    # a float imagemap reads no basis (FloatImageTexture ignores it)
    text = HEAD.format(res=8, spp=1) + """
Texture "r" "float" "imagemap" "string filename" "img.pfm" "string basisfilename" "b3.json"
Material "conductor" "texture roughness" "r"
Shape "sphere" "float radius" 0.5
"""
    pa.Scene.from_string(text, tex_dir)


def test_basis_texture_renders(pa, oracle, tex_dir):
    sc = textured(tex_dir, pa, "b3.json")
    f = sc.flat()
    img = oracle.film_to_rgb(oracle.render(sc, threads=8), [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert np.isfinite(img).all() and np.abs(img).mean() > 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("basis,filt", [("b3.json", "bilinear"), ("b2_36.json", "ewa")])
def test_basis_texture_gpu_matches_oracle(pa, oracle, tex_dir, basis, filt):
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    sc = textured(tex_dir, pa, basis, filt=filt, res=48, spp=16)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    frac, mr = check(gpu, oracle_rgb(oracle, sc))
    print(f"basis texture {basis} ({filt}): {frac * 100:.2f}% pixels within 1e-3, mean rel {mr:.2e}")


@pytest.mark.gpu
def test_basis_texture_volumetric_gpu_matches_oracle(pa, oracle, tex_dir):
    """the same texture on the volumetric kernels (k_vtexture): a homogeneous haze around the scene"""
    from test_gpu_media import check, gpu_rgb, oracle_rgb
    haze = ('MakeNamedMedium "haze" "string type" "homogeneous" "rgb sigma_a" [0.01 0.01 0.01] '
            '"rgb sigma_s" [0.05 0.05 0.05]\n')
    body = HEAD.format(res=32, spp=8).replace('Camera "perspective"', haze + 'MediumInterface "" "haze"\nCamera "perspective"')
    body += """
Texture "ms" "spectrum" "imagemap" "string filename" "img.pfm" "string basisfilename" "b3.json"
AttributeBegin
  Material "diffuse" "texture reflectance" "ms"
  Shape "trianglemesh" "integer indices" [0 1 2 0 2 3] "point3 P" [-1 -1 0.5  1 -1 0.5  1 1 0.5  -1 1 0.5]
    "point2 uv" [0 0 1 0 1 1 0 1]
AttributeEnd
"""
    sc = pa.Scene.from_string(body, tex_dir)
    gpu, _ = gpu_rgb(pa, oracle, sc)
    check(gpu, oracle_rgb(oracle, sc))
