"""WindowedPiecewiseConstant2D and PiecewiseLinear2D pinned to the reference's own classes.

tests/golden/reference_components.json keys `windowed_pc2d` and `piecewise_linear_2d` are written
by oracle/ref/refgold.cpp, which links the unmodified reference sources
(util/sampling.h:830-980 SummedAreaTable / WindowedPiecewiseConstant2D, 1299-1749
PiecewiseLinear2D): seeded functions of 16x16, 7x7 (zero rows and columns) and 32x32 with 400
windows each (every 9th degenerate, every 13th the unit square), and PiecewiseLinear2D<0> with and
without a CDF and PiecewiseLinear2D<2> with parameter grids {-3, .5, 3.1} x {0, .3, .55, 1} queried
inside and outside the grids. The portal light and the measured BxDF use these two classes; here
both the oracle's restatements and the product's host code (the same PHD functions the kernels
run) are held to every golden row bit for bit.

The one intended difference: the product's (and oracle's) SampleBisection stops after 128 halvings
where pbrt's loop has no cap; none of the golden windows comes near it.
"""
import json
import pathlib

import numpy as np
import pytest

GOLD = json.loads((pathlib.Path(__file__).parent / "golden" / "reference_components.json").read_text())


@pytest.mark.parametrize("case", range(3))
def test_windowed_oracle_matches_reference(oracle, case):
    c = GOLD["windowed_pc2d"][case]
    rows = np.array(c["rows"], np.float32)
    out = oracle.windowed2d(np.array(c["f"], np.float32), rows[:, :8])
    np.testing.assert_array_equal(out, rows[:, 8:])


@pytest.mark.parametrize("case", range(3))
def test_windowed_product_matches_reference(pa, case):
    c = GOLD["windowed_pc2d"][case]
    rows = np.array(c["rows"], np.float32)
    out = pa.debug_windowed2d(np.array(c["f"], np.float32), rows[:, :8])
    np.testing.assert_array_equal(out, rows[:, 8:])


def test_windowed_golden_covers_edges():
    """The fixture holds failed samples (zero windows), degenerate windows and the unit square."""
    rows = np.concatenate([np.array(c["rows"], np.float32) for c in GOLD["windowed_pc2d"]])
    assert (rows[:, 8] == 0).sum() > 10 and (rows[:, 8] == 1).sum() > 900
    assert ((rows[:, 2] == 0) & (rows[:, 4] == 1)).sum() >= 3 * 30
    assert (rows[:, 12] == 0).sum() > 0


@pytest.mark.parametrize("case", range(4))
def test_pl2d_oracle_matches_reference(oracle, case):
    c = GOLD["piecewise_linear_2d"][case]
    rows = np.array(c["rows"], np.float32)
    out = oracle.pl2d(c["dim"], c["cdf"], c["data"], c["xs"], c["ys"], c["pr"], c["pv0"], c["pv1"], rows[:, :6])
    np.testing.assert_array_equal(out, rows[:, 6:])


@pytest.mark.parametrize("case", range(4))
def test_pl2d_product_matches_reference(pa, case):
    c = GOLD["piecewise_linear_2d"][case]
    rows = np.array(c["rows"], np.float32)
    out = pa.debug_pl2d(c["dim"], c["cdf"], c["data"], c["xs"], c["ys"], c["pr"], c["pv0"], c["pv1"],
                        rows[:, :6])
    np.testing.assert_array_equal(out, rows[:, 6:])


def test_pl2d_sample_invert_round_trip(pa):
    """Invert(Sample(u)) == u and the two pdfs agree, on the golden dim-2 table (a property the
    reference's sampling tests check for the warps)."""
    c = GOLD["piecewise_linear_2d"][2]
    rng = np.random.default_rng(7)
    q = np.zeros((256, 6), np.float32)
    q[:, :2] = rng.uniform(0.02, 0.98, (256, 2))
    q[:, 4] = rng.uniform(-3, 3.1, 256)
    q[:, 5] = rng.uniform(0, 1, 256)
    s = pa.debug_pl2d(c["dim"], c["cdf"], c["data"], c["xs"], c["ys"], c["pr"], c["pv0"], c["pv1"], q)
    q2 = q.copy()
    q2[:, 2:4] = s[:, :2]
    r = pa.debug_pl2d(c["dim"], c["cdf"], c["data"], c["xs"], c["ys"], c["pr"], c["pv0"], c["pv1"], q2)
    np.testing.assert_allclose(r[:, 3:5], q[:, :2], atol=2e-4)
    np.testing.assert_allclose(r[:, 5], s[:, 2], rtol=2e-4)
    np.testing.assert_allclose(r[:, 6], s[:, 2], rtol=2e-4)


def test_windowed_pdf_integrates_to_one(pa):
    """PDF(p, b) integrates to 1 over any window with mass (midpoint rule on the 16x16 table)."""
    c = GOLD["windowed_pc2d"][0]
    f = np.array(c["f"], np.float32)
    b = np.array([0.1, 0.25, 0.8, 0.9], np.float32)
    m = 512
    xs = b[0] + (np.arange(m) + 0.5) / m * (b[2] - b[0])
    ys = b[1] + (np.arange(m) + 0.5) / m * (b[3] - b[1])
    gx, gy = np.meshgrid(xs, ys)
    q = np.zeros((m * m, 8), np.float32)
    q[:, 2:6] = b
    q[:, 6], q[:, 7] = gx.ravel(), gy.ravel()
    pdf = pa.debug_windowed2d(f, q)[:, 4]
    assert abs(pdf.mean() * (b[2] - b[0]) * (b[3] - b[1]) - 1) < 5e-3


def test_bad_tables_refused(pa):
    with pytest.raises(Exception):
        pa.debug_pl2d(1, 1, np.ones(16), 4, 4, [1, 1], [0], [0], np.zeros((1, 6)))
    with pytest.raises(Exception):
        pa.debug_pl2d(0, 1, np.ones(4), 1, 4, [1, 1], [0], [0], np.zeros((1, 6)))
