"""CPU oracle integrator: determinism, decomposition invariants and the reference's own
known-answer test (RenderTest.RadianceMatches furnace scene, cpu/integrators_test.cpp)."""
import numpy as np

from conftest import SCENES


def render(oracle, sc, rows=None, first=0, n=None, film=None):
    f = oracle.render(sc, rows=rows, first_sample=first, n_samples=n, threads=8)
    return f if film is None else film + f


def test_row_stripes_stitch_bit_exact(pa, oracle):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=48, yresolution=40, spp=4)
    full = oracle.render(sc, threads=8)
    from pbrt_amd.tiles import rows_for_rank
    parts = [oracle.render(sc, rows=rows_for_rank(0, 40, r, 3, block=4), threads=3) for r in range(3)]
    np.testing.assert_array_equal(full, parts[0] + parts[1] + parts[2])


def test_deterministic(pa, oracle):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=32, yresolution=32, spp=4)
    np.testing.assert_array_equal(oracle.render(sc, threads=1), oracle.render(sc, threads=8))


def test_pixel_bounds_crop(pa, oracle):
    full_sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=32, yresolution=32, spp=2)
    crop_sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=32, yresolution=32, spp=2,
                            pixelbounds="8,24,4,20")
    full = oracle.render(full_sc, threads=8)
    crop = oracle.render(crop_sc, threads=8)
    np.testing.assert_array_equal(full[:, 4:20, 8:24], crop[:, 4:20, 8:24])
    assert not crop[:, :4].any() and not crop[:, :, :8].any()


def test_furnace_known_answer(pa, oracle):
    """integrators_test.cpp:128-155 + CheckSceneAverage (:51-64): average 1.0 +- 0.025."""
    sc = pa.load_scene(SCENES / "furnace.pbrt")
    film = oracle.render(sc, threads=8)
    f = sc.flat()
    img = oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    assert abs(img.mean() - 1.0) < 0.025, img.mean()


def test_cornell_plausible(pa, oracle):
    sc = pa.load_scene(SCENES / "cornell-box.pbrt", xresolution=32, yresolution=32, spp=8)
    f = sc.flat()
    film = oracle.render(sc, threads=8)
    assert np.isfinite(film).all() and (film >= 0).all()  # sensor XYZ sums are non-negative
    img = oracle.film_to_rgb(film, [f.output_rgb_from_sensor_rgb[i] for i in range(9)])
    # red wall left / green wall right after the "Scale -1 1 1" flip, light is brightest
    assert img[:, :4, 0].mean() > img[:, :4, 1].mean() and img[:, -4:, 1].mean() > img[:, -4:, 0].mean()


def test_oracle_zsobol_render_runs(pa, oracle):
    """The oracle renders the default-sampler (ZSobol) Cornell; finite, nonzero image."""
    from conftest import cornell_with_sampler
    sc = cornell_with_sampler(pa, 'Sampler "zsobol" "integer pixelsamples" [ 4 ]', xresolution=32, yresolution=24)
    film = oracle.render(sc, threads=4)
    assert np.isfinite(film).all() and film[:3].sum() > 0
