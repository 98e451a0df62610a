"""RGBSigmoidPolynomial (util/color.h:341) on the device forms its correctly rounded sqrt and
division without the compiler's range-scaling / fix-up steps (core.h); it must equal the plain
IEEE expression bit for bit on every input, in the tables' range or not.  The same device
self-check covers SinCosf against the separate calls, DenseOffset's 32-bit form against lround,
and DivByRcp (a spectrum divided by one scalar through its correctly rounded reciprocal and two
residual corrections) against the IEEE division, on any operands and on quotients placed next
to a rounding midpoint."""
import numpy as np
import pytest


@pytest.mark.gpu
def test_sigmoid_fast_sqrt_div_bit_exact(pa):
    for seed in (1, 987654321):
        bad = pa.check_rn_math(n=1 << 28, seed=seed)
        np.set_printoptions(precision=9)
        assert bad == 0, f"{bad} mismatches, e.g. (c0 c1 c2 lambda kernel plain):\n{pa.check_rn_math.examples}"
