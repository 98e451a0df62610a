"""The CPU oracle (oracle/oracle.cpp) against the reference's own outputs
(tests/golden/reference_components.json, produced by oracle/ref from the unmodified
reference sources).  Integer/index results must match exactly; floating-point results
bit-exactly where the arithmetic is the same IEEE sequence, and to a few ulp where the
reference calls libm transcendentals (sin/cos/asin/atan2) that the test machine may round
differently."""
import ctypes

import numpy as np
import pytest

from conftest import fl


_KEEP = []


def arr(a):
    """float32 contiguous copy that stays alive until the next test (ctypes gets raw pointers)"""
    x = np.ascontiguousarray(np.asarray(fl(a), dtype=np.float32))
    _KEEP.append(x)
    if len(_KEEP) > 64:
        del _KEEP[:32]
    return x


def ulp_close(a, b, ulps=4, atol=0.0):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    tol = ulps * np.spacing(np.maximum(np.abs(a), np.abs(b))) + atol
    return np.all((np.abs(a - b) <= tol) | (a == b))


def test_triangle_intersection_bit_exact(oracle, golden):
    lib = oracle.lib()
    n_hit = 0
    for e in golden["triangles"]:
        out = np.zeros(19, np.float32)
        r = lib.oracle_intersect_triangle(arr(e["p"]).ctypes.data, arr(e["o"]).ctypes.data, arr(e["d"]).ctypes.data,
                                          float(fl(e["tMax"])), int(e["flip"]), out.ctypes.data)
        if e["hit"] is None:
            assert r == 0, e
            continue
        n_hit += 1
        assert r == 1, e
        np.testing.assert_array_equal(out[0:4], arr(e["hit"]))        # b0 b1 b2 t
        np.testing.assert_array_equal(out[4:7], arr(e["si_p"]))
        np.testing.assert_array_equal(out[7:10], arr(e["si_err"]))
        np.testing.assert_array_equal(out[10:13], arr(e["si_n"]))
        np.testing.assert_array_equal(out[13:16], arr(e["si_dpdu"]))
        np.testing.assert_array_equal(out[16:19], arr(e["si_wo"]))
    assert n_hit > 100


def test_triangle_bad_case_misses(oracle, golden):
    # Triangle.BadCases (shapes_test.cpp:435-449) is the first golden entry
    assert golden["triangles"][0]["hit"] is None


def test_warps(oracle, golden):
    lib = oracle.lib()
    for e in golden["warps"]:
        out = np.zeros(11, np.float32)
        lib.oracle_warps(arr(e["u"]).ctypes.data, arr(e["w"]).ctypes.data, out.ctypes.data)
        assert ulp_close(out[0:2], arr(e["disk"]), 4), e
        assert ulp_close(out[2:5], arr(e["cos"]), 8, 1e-7), e
        np.testing.assert_array_equal(out[5:8], arr(e["tri"]))
        np.testing.assert_array_equal(out[8:10], arr(e["bilinear"]))
        np.testing.assert_array_equal(out[10], np.float32(fl(e["bilinear_pdf"])))


def test_spherical_triangles(oracle, golden):
    lib = oracle.lib()
    for e in golden["spherical_triangles"]:
        out = np.zeros(10, np.float32)
        lib.oracle_spherical_triangle(arr(e["v"]).ctypes.data, arr(e["p"]).ctypes.data, arr(e["u"]).ctypes.data,
                                      out.ctypes.data)
        assert ulp_close(out[0:3], arr(e["b"]), 64, 1e-6), e
        assert ulp_close(out[3], np.float32(fl(e["pdf"])), 16), e
        assert ulp_close(out[7:9], arr(e["inv"]), 256, 1e-5), e
        assert ulp_close(out[9], np.float32(fl(e["area"])), 16), e


def test_triangle_light_sampling(oracle, golden):
    lib = oracle.lib()
    quad = np.array([[343, 548.7, 227], [343, 548.7, 332], [213, 548.7, 332], [213, 548.7, 227]], np.float32)
    tris = [np.ascontiguousarray(quad[[0, 1, 2]].ravel()), np.ascontiguousarray(quad[[0, 2, 3]].ravel())]
    n = 0
    for e in golden["triangle_light_sampling"]:
        out = np.zeros(12, np.float32)
        r = lib.oracle_triangle_sample(tris[e["tri"]].ctypes.data, 0, arr(e["ref"]).ctypes.data,
                                       arr(e["n"]).ctypes.data, arr(e["ns"]).ctypes.data, arr(e["u"]).ctypes.data,
                                       out.ctypes.data)
        if e["p"] is None:
            assert r == 0
            continue
        assert r == 1
        n += 1
        assert ulp_close(out[0:3], arr(e["p"]), 64, 1e-3), e
        assert ulp_close(out[6:9], arr(e["nrm"]), 0), e
        assert ulp_close(out[9], np.float32(fl(e["pdf"])), 1024), (out[9], e)
        assert ulp_close(out[10], np.float32(fl(e["pdf_wi"])), 1024), (out[10], e)
        assert ulp_close(out[11], np.float32(fl(e["solid_angle"])), 16), e
    assert n > 250


def test_light_importance(oracle, golden):
    lib = oracle.lib()
    for e in golden["light_importance"]:
        imp = lib.oracle_light_importance(arr(e["decoded"]).ctypes.data, ctypes.c_float(fl(e["phi"])), int(e["two"]),
                                          arr(e["p"]).ctypes.data, arr(e["n"]).ctypes.data)
        assert ulp_close(imp, np.float32(fl(e["importance"])), 8), (imp, e)


def test_offset_ray_origin_bit_exact(oracle, golden):
    lib = oracle.lib()
    for e in golden["offset_ray_origin"]:
        out = np.zeros(3, np.float32)
        lib.oracle_offset_ray_origin(arr(e["p"]).ctypes.data, arr(e["e"]).ctypes.data, arr(e["n"]).ctypes.data,
                                     arr(e["w"]).ctypes.data, out.ctypes.data)
        np.testing.assert_array_equal(out, arr(e["po"]))


def test_sample_uniform_wavelengths_bit_exact(oracle, golden):
    lib = oracle.lib()
    for e in golden["sample_uniform_wavelengths"]:
        lam = np.zeros(31, np.float32)
        pdf = np.zeros(1, np.float32)
        lib.oracle_sample_wavelengths(ctypes.c_float(fl(e["u"])), lam.ctypes.data, pdf.ctypes.data)
        np.testing.assert_array_equal(lam, arr(e["lambda"]))
        assert pdf[0] == np.float32(fl(e["pdf"]))


@pytest.mark.parametrize("cfg_index", [0, 1, 2])
def test_halton_bit_exact(oracle, golden, cfg_index):
    lib = oracle.lib()
    cfg = golden["halton"][cfg_index]
    for px, py, si, dim, p0, p1, vals in cfg["samples"]:
        got = [lib.oracle_halton(cfg["xres"], cfg["yres"], cfg["seed"], px, py, si, dim + j) for j in range(7)]
        np.testing.assert_array_equal(np.float32(got), arr(vals))
        assert lib.oracle_halton(cfg["xres"], cfg["yres"], cfg["seed"], px, py, si, -1) == np.float32(p0)
        assert lib.oracle_halton(cfg["xres"], cfg["yres"], cfg["seed"], px, py, si, -2) == np.float32(p1)


RANDOMIZE = {"none": 0, "permutedigits": 1, "fastowen": 2, "owen": 3}


@pytest.mark.parametrize("cfg_index", range(6))
def test_zsobol_bit_exact(oracle, golden, cfg_index):
    """The oracle's ZSobolSampler restatement against the reference's (samplers.h:225-370)."""
    cfg = golden["zsobol"][cfg_index]
    out = (ctypes.c_float * 7)()
    for px, py, si, dim, vals in cfg["samples"]:
        oracle.lib().oracle_zsobol(cfg["spp"], cfg["xres"], cfg["yres"], cfg["seed"], RANDOMIZE[cfg["randomization"]],
                                   px, py, si, dim, out)
        np.testing.assert_array_equal(np.array(out[:], np.float32), np.array(vals, np.float32))
