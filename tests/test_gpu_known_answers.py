"""The closed-form known answers of tests/test_known_answers.py on the GPU (point-light
RadianceMatches furnaces, tilted spot light), plus parity with the oracle on the same scenes."""
import numpy as np
import pytest

from test_known_answers import check_spot, point_furnace_text, render_rgb, spot_scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sampler", ["halton", "zsobol"])
@pytest.mark.parametrize("n_lights", [1, 4])
def test_point_light_furnace_gpu(pa, oracle, n_lights, sampler):
    text = point_furnace_text(n_lights, sampler)
    img, _ = render_rgb(pa, oracle, text, gpu=True)
    assert abs(img.mean() - 1.0) <= 0.025, img.mean()
    ref, _ = render_rgb(pa, oracle, text)
    np.testing.assert_allclose(img.mean(), ref.mean(), rtol=1e-4)


def test_tilted_spot_light_gpu(pa, oracle):
    img, _ = render_rgb(pa, oracle, spot_scene(), gpu=True)
    check_spot(img)
    ref, _ = render_rgb(pa, oracle, spot_scene())
    np.testing.assert_allclose(img, ref, rtol=1e-4, atol=1e-7)
