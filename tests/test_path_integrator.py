"""configs[0]'s integrator: the oracle's restatement of the CPU PathIntegrator
(cpu/integrators.cpp:629-805, oracle.cpp Renderer::PathLi) and a mean-within-noise check of the
product's C1 image against it.

pbrt's GPU renders every "path" / "volpath" scene with the wavefront integrator's semantics
(balance-heuristic MIS through r_u / r_l, seven fixed sampler dimensions per bounce), and so does
the product.  The CPU PathIntegrator is a different estimator of the same image (power heuristic,
the CPU sampler's sequential dimensions, roulette after the second bounce), so the two agree in
expectation, not per sample:

* RenderTest.RadianceMatches (cpu/integrators_test.cpp:51-156) runs PathIntegrator on its
  furnace scenes: the emissive furnace (scenes/furnace.pbrt) and the point-light furnaces, image
  average 1.0 +- 0.025 -- the same known answers the wavefront oracle meets.
* C1 Cornell: the path image's mean and its 8x8-pixel block means agree with the wavefront
  oracle's (and, on the GPU, with the product's) within 4.5 standard errors estimated from the
  per-pixel differences."""
import numpy as np
import pytest

from conftest import SCENES
from test_known_answers import point_furnace_text


def _rgb(oracle, sc, film):
    f = sc.flat()
    return oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])


def test_path_emissive_furnace(pa, oracle):
    sc = pa.load_scene(SCENES / "furnace.pbrt")
    img = _rgb(oracle, sc, oracle.render(sc, threads=8, path=True))
    assert abs(img.mean() - 1.0) < 0.025, img.mean()


@pytest.mark.parametrize("sampler", ["halton", "zsobol"])
@pytest.mark.parametrize("n_lights", [1, 4])
def test_path_point_light_furnace(pa, oracle, n_lights, sampler):
    sc = pa.Scene.from_string(point_furnace_text(n_lights, sampler), SCENES)
    img = _rgb(oracle, sc, oracle.render(sc, threads=8, path=True))
    assert abs(img.mean() - 1.0) <= 0.025, img.mean()


def test_path_refuses_media(pa, oracle):
    sys_path = str(SCENES)
    import sys
    sys.path.insert(0, sys_path)
    import gen_c5
    sc = pa.Scene.from_string(gen_c5.scene_text(16, 12, 1, grid=8), SCENES)
    with pytest.raises(AssertionError):
        oracle.render(sc, threads=2, path=True)


def mean_within_noise(a, b, k=4.5, block=8):
    """a, b: [h, w, 3] images of the same scene by independent unbiased estimators.  The image
    mean and every block x block mean of a - b must be within k standard errors, the error of a
    block mean estimated from the spread of its pixels' differences."""
    d = (a - b).astype(np.float64)
    n = d.shape[0] * d.shape[1]
    se = d.reshape(n, 3).std(axis=0, ddof=1) / np.sqrt(n)
    z = np.abs(d.reshape(n, 3).mean(axis=0)) / np.maximum(se, 1e-12)
    assert (z <= k).all(), (z, d.reshape(n, 3).mean(axis=0), se)
    h, w = d.shape[0] // block * block, d.shape[1] // block * block
    blocks = d[:h, :w].reshape(h // block, block, w // block, block, 3).transpose(0, 2, 1, 3, 4)
    blocks = blocks.reshape(-1, block * block, 3)
    bse = blocks.std(axis=1, ddof=1) / np.sqrt(block * block)
    bz = np.abs(blocks.mean(axis=1)) / np.maximum(bse, 1e-9)
    # k standard errors per block, over many blocks: allow the normal tail's share past k
    frac = (bz > k).mean()
    assert frac <= 0.01, (frac, bz.max())
    return z, frac


def c1(pa, res=64, spp=64):
    return pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=res, yresolution=res, spp=spp)


def test_path_vs_wavefront_cornell_oracle(pa, oracle):
    sc = c1(pa)
    vol = _rgb(oracle, sc, oracle.render(sc, threads=8))
    path = _rgb(oracle, sc, oracle.render(sc, threads=8, path=True))
    assert np.isfinite(path).all() and path.mean() > 0
    z, frac = mean_within_noise(vol, path)
    # different estimators: the images are not the same bits
    assert np.abs(vol - path).max() > 0


@pytest.mark.gpu
def test_gpu_c1_vs_path_integrator(pa, oracle):
    """The product's configs[0] image (C1 Cornell 256x256 16 spp, wavefront semantics on the GPU)
    against the CPU PathIntegrator restatement: mean within noise, and 8x8 blocks."""
    from test_gpu_parity import gpu_film
    sc = pa.load_scene(SCENES / "cornell-box.pbrt")
    film, _ = gpu_film(pa, sc)
    gpu = _rgb(oracle, sc, film)
    path = _rgb(oracle, sc, oracle.render(sc, threads=16, path=True))
    z, frac = mean_within_noise(gpu, path)
    print(f"C1 GPU vs PathIntegrator: mean z {np.round(z, 2)}, blocks past 4.5 se {frac:.4f}")
