"""The kernels' transcendentals (pbrt-v4_amd/csrc/core/detmath.h): sin, cos, sincos, asin, acos,
atan, atan2, log, exp, tan, expm1 and sinh restated from glibc's own algorithms (Arm's
double-precision sinf / cosf / expf / logf in glibc's -mfma build, the fdlibm float conversions for
the rest), so the GPU, the product's host code and pbrt's CPU build (std::sin(float) = glibc sinf)
compute the same bits.  That is what lets every GPU parity test hold the oracle's per-sample
decisions in its libm mode -- the reference's arithmetic: the medium RNG seeded from a ray's bits
(wavefront/media.cpp:44), alpha tests hashing the ray (gpu/optix.cu:197-243), mix choices hashing
the hit (materials.h:285-294).

* glibc: the product == glibc (the oracle's libm mode) bit for bit, on seeded samples of each
  function's domain plus a stride over all 2^32 bit patterns (tools/detmath_exhaustive.cpp checks
  every input; its last output is profiles/r06_detmath_exhaustive.txt);
* glibc itself is not correctly rounded: the fraction differing from the correctly rounded value is
  reported and bounded below, which is why a merely accurate polynomial cannot match it;
* GPU == host, bit for bit (gpu).
"""
import numpy as np
import pytest

FNS = ["sin", "cos", "asin", "acos", "atan2", "log", "exp", "sinh", "tan", "atan", "expm1"]


def inputs(fn, n=400000, seed=7):
    rng = np.random.default_rng(seed)
    if fn in ("sin", "cos", "sincos_sin", "sincos_cos", "tan"):
        a = np.concatenate([rng.uniform(-7, 7, n // 2), rng.uniform(-1e4, 1e4, n // 4), rng.uniform(-1e-3, 1e-3, n // 8),
                            rng.uniform(-1e6, 1e6, n // 8), [0.0, -0.0, 1e-30, np.pi, -np.pi / 2, 8192.0, 8193.0, 120.0,
                                                             119.99, 1e38, -3e37]])
        b = np.zeros_like(a)
    elif fn in ("asin", "acos"):
        a = np.concatenate([rng.uniform(-1, 1, n // 2), 1 - np.ldexp(rng.uniform(0, 1, n // 4), -rng.integers(1, 24, n // 4)),
                            -1 + np.ldexp(rng.uniform(0, 1, n // 4), -rng.integers(1, 24, n // 4)), [0.0, -0.0, 0.5, -0.5, 1, -1]])
        b = np.zeros_like(a)
    elif fn == "atan2":
        a = np.concatenate([rng.uniform(-5, 5, n // 2), rng.uniform(-1e-5, 1e-5, n // 4), rng.normal(size=n // 4),
                            np.ldexp(rng.uniform(-1, 1, n // 4), rng.integers(-70, 70, n // 4)),
                            [0.0, -0.0, 0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.inf, 3.0]])
        b = np.concatenate([rng.uniform(-5, 5, n // 2), rng.normal(size=n // 4), rng.uniform(-1e-5, 1e-5, n // 4),
                            np.ldexp(rng.uniform(-1, 1, n // 4), rng.integers(-70, 70, n // 4)),
                            [1.0, 1.0, -1.0, -1.0, 0.0, -0.0, np.inf, -np.inf, -np.inf, 1.0]])
    elif fn in ("exp", "expm1"):
        a = np.concatenate([rng.uniform(-104, 89, n // 2), rng.uniform(-1, 1, n // 4), rng.uniform(-20, 0, n // 4),
                            [0.0, -0.0, 1.0, -1.0, 88.7, -87.3, -100.0, -104.0, 89.0, 1e-9, -1e-9]])
        b = np.zeros_like(a)
    elif fn == "sinh":
        a = np.concatenate([rng.uniform(0.1, 30, n // 2), rng.uniform(-30, -0.1, n // 4), rng.uniform(1, 10, n // 4),
                            rng.uniform(-100, 100, n // 8), [0.0, -0.0, 1e-5, 0.5, 1.0, 10.0, 22.0, 89.0, 90.0]])
        b = np.zeros_like(a)
    elif fn == "atan":
        a = np.concatenate([rng.uniform(-3, 3, n // 2), np.ldexp(rng.uniform(-1, 1, n // 2), rng.integers(-40, 40, n // 2)),
                            [0.0, -0.0, 2.0 ** 25, -2.0 ** 25, 0.4375, 1.1875, 2.4375, np.inf]])
        b = np.zeros_like(a)
    else:  # log
        a = np.concatenate([np.exp(rng.uniform(-87, 88, n // 2)), rng.uniform(0.5, 2, n // 4), rng.uniform(0, 1, n // 4),
                            [1.0, 2.0, 0.5, 1e-40, 1e-45, 3e38]])
        b = np.zeros_like(a)
    a, b = a.astype(np.float32), b.astype(np.float32)
    if fn != "atan2":  # plus a stride over every bit pattern (NaNs and infinities included)
        a = np.concatenate([a, np.arange(0, 1 << 32, 4099, dtype=np.uint64).astype(np.uint32).view(np.float32)])
        b = np.zeros_like(a)
    return a, b


def bits_equal(x, y):
    """bitwise equality, any NaN equal to any NaN"""
    return (x.view(np.uint32) == y.view(np.uint32)) | (np.isnan(x) & np.isnan(y))


@pytest.mark.parametrize("fn", FNS + ["sincos_sin", "sincos_cos"])
def test_det_math_equals_glibc(pa, oracle, fn):
    """product host code == glibc (the oracle's libm mode, which calls std::sin(float) etc.)"""
    a, b = inputs(fn)
    got = pa.det_math(fn, a, b)
    with np.errstate(all="ignore"):
        ref = oracle.math_eval(fn.replace("sincos_", ""), a, b)
    ok = bits_equal(got, ref)
    assert ok.all(), (fn, (~ok).sum(), a[~ok][:4], b[~ok][:4], got[~ok][:4], ref[~ok][:4])


CR_DIFF = {"sin": 0.005, "cos": 0.005, "asin": 0.03, "acos": 0.03, "atan2": 0.05, "tan": 0.01, "sinh": 0.05}


@pytest.mark.parametrize("fn", sorted(CR_DIFF))
def test_glibc_is_not_correctly_rounded(oracle, fn):
    """Why a correctly rounded (or any other accurate) implementation would not do: glibc's float
    functions differ from the correctly rounded value on a measurable share of inputs."""
    rng = np.random.default_rng(5)
    lo, hi = {"asin": (-1, 1), "acos": (-1, 1), "sinh": (0.1, 20), "tan": (-1.5, 1.5)}.get(fn, (-7, 7))
    a = rng.uniform(lo, hi, 200000).astype(np.float32)
    b = rng.uniform(-5, 5, 200000).astype(np.float32)
    with oracle.math_mode(oracle.MATH_LIBM):
        lm = oracle.math_eval(fn, a, b)
    with oracle.math_mode(oracle.MATH_CR):
        cr = oracle.math_eval(fn, a, b)
    frac = 1 - bits_equal(lm, cr).mean()
    print(f"{fn}: glibc differs from correctly rounded on {frac * 100:.2f}% of inputs")
    assert frac > CR_DIFF[fn], frac


def test_det_math_special_values(pa):
    z = np.float32
    assert np.signbit(pa.det_math("sin", [-0.0])[0]) and pa.det_math("cos", [-0.0])[0] == 1
    at = pa.det_math("atan2", [0.0, -0.0, 0.0, -0.0, 1.0, -1.0], [1.0, 1.0, -1.0, -1.0, 0.0, 0.0])
    np.testing.assert_array_equal(at, np.arctan2(z([0.0, -0.0, 0.0, -0.0, 1.0, -1.0]), z([1.0, 1.0, -1.0, -1.0, 0.0, 0.0])))
    assert np.signbit(at[1]) and not np.signbit(at[0])
    lg = pa.det_math("log", [0.0, 1.0, np.inf, -1.0])
    assert lg[0] == -np.inf and lg[1] == 0 and lg[2] == np.inf and np.isnan(lg[3])
    assert np.isnan(pa.det_math("sin", [np.inf, np.nan])).all()
    assert np.isnan(pa.det_math("tan", [np.inf])).all() and pa.det_math("expm1", [-np.inf])[0] == -1


@pytest.mark.gpu
@pytest.mark.parametrize("fn", FNS + ["sincos_sin", "sincos_cos"])
def test_det_math_gpu_equals_host_bitwise(pa, fn):
    """The same source compiled for gfx950 and for the host gives the same bits on every input
    (IEEE operations only; -ffp-contract=off), including SinCosf against the separate calls."""
    a, b = inputs(fn, n=1 << 20, seed=13)
    dev = pa.det_math(fn, a, b, device=0)
    host = pa.det_math(fn, a, b)
    ok = bits_equal(dev, host)
    assert ok.all(), (fn, (~ok).sum(), a[~ok][:4], dev[~ok][:4], host[~ok][:4])
    if fn.startswith("sincos_"):
        assert bits_equal(dev, pa.det_math(fn[7:], a, b, device=0)).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fn", FNS)
def test_det_math_gpu_equals_glibc(pa, oracle, fn):
    """the GPU's values against glibc directly (host libm on the GPU box)"""
    a, b = inputs(fn, n=1 << 18, seed=17)
    dev = pa.det_math(fn, a, b, device=0)
    with np.errstate(all="ignore"):
        ref = oracle.math_eval(fn, a, b)
    assert bits_equal(dev, ref).all()
