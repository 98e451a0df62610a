"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/_build/liboracle.so, the CPU
restatement of pbrt-v4's wavefront integrator (see oracle/oracle.cpp).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "liboracle.so"
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", str(HERE)])


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = ctypes.CDLL(str(LIB))
        _lib.oracle_render.restype = ctypes.c_int
        _lib.oracle_light_importance.restype = ctypes.c_float
        _lib.oracle_halton.restype = ctypes.c_float
        _lib.oracle_intersect_triangle.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
        _lib.oracle_light_importance.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        _lib.oracle_sample_wavelengths.argtypes = [ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
        _lib.oracle_halton.argtypes = [ctypes.c_int] * 7
        _lib.oracle_zsobol.argtypes = [ctypes.c_int] * 9 + [ctypes.c_void_p]
        _lib.oracle_sampler.argtypes = [ctypes.c_int] * 9 + [ctypes.c_void_p] * 3 + [ctypes.c_int] * 4 + [ctypes.c_void_p]
        _lib.oracle_rng.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        _lib.oracle_procedural.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]
        _lib.oracle_sss_table.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
        _lib.oracle_catmull_rom.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                            ctypes.c_void_p]
        vp = ctypes.c_void_p
        _lib.oracle_warps.argtypes = [vp, vp, vp]
        _lib.oracle_spherical_triangle.argtypes = [vp, vp, vp, vp]
        _lib.oracle_triangle_sample.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp]
        _lib.oracle_offset_ray_origin.argtypes = [vp, vp, vp, vp, vp]
        _lib.oracle_trowbridge.argtypes = [vp, vp]
        _lib.oracle_fresnel.argtypes = [vp, vp]
        _lib.oracle_named_spectrum.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp]
        _lib.oracle_bxdf.argtypes = [ctypes.c_int] + [vp] * 7
        _lib.oracle_layered.argtypes = [vp] * 8
        _lib.oracle_hair_eval.argtypes = [vp, ctypes.c_int, vp]
        _lib.oracle_measured_eval.argtypes = [ctypes.c_char_p, vp, ctypes.c_int, vp, vp]
        _lib.oracle_portal_eval.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp, vp]
        _lib.oracle_pl2d.argtypes = [ctypes.c_int, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int] + [vp] * 4 + [
            ctypes.c_int, vp]
        _lib.oracle_windowed2d.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int, vp]
        _lib.oracle_triangle_shading.argtypes = [vp] * 3 + [ctypes.c_int] + [vp] * 3
        _lib.oracle_render.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, vp]
        _lib.oracle_render_path.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, vp]
        _lib.oracle_render_path.restype = ctypes.c_int
        _lib.oracle_set_cr_math.argtypes = [ctypes.c_int]
        _lib.oracle_set_math_mode.argtypes = [ctypes.c_int]
        _lib.oracle_get_math_mode.restype = ctypes.c_int
        _lib.oracle_math_eval.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        _lib.oracle_light_bvh.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp, ctypes.c_int]
        _lib.oracle_intersect_tr.argtypes = [vp, vp, vp, vp, vp, ctypes.c_int, vp]
        _lib.oracle_set_rgb_table.argtypes = [vp, vp]
        _lib.oracle_texture_eval.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, ctypes.c_int, vp]
        _lib.oracle_env_eval.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, vp]
        _lib.oracle_shape_eval.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, vp]
        _lib.oracle_equal_area.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp]
        _lib.oracle_cloud_density.argtypes = [vp, vp, ctypes.c_int, vp]
        _lib.oracle_medium_point.argtypes = [vp, ctypes.c_int, vp, vp, ctypes.c_int, vp]
        _lib.oracle_camera_min_diff.argtypes = [vp, vp, vp]
        _lib.oracle_image_level.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int64,
                                            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        _lib.oracle_image_level.restype = ctypes.c_int64
        _set_tables(_lib)
    return _lib


# Reference data tables the oracle's texture code reads: the rgb2spec_opt coefficient table
# (pbrt-v4_amd/data/rgbspec_srgb.bin, written by the build) and MIPFilterLUT
# (pbrt-v4_amd/data/spectral_data.txt, the literals of util/mipmap.cpp)
_TABLES = {}


def _set_tables(l):
    data = HERE.parent / "pbrt-v4_amd" / "data"
    rgb = data / "rgbspec_srgb.bin"
    if not rgb.exists():
        return
    _TABLES["rgb"] = np.fromfile(rgb, dtype=np.float32)
    for line in (data / "spectral_data.txt").read_text().splitlines():
        if line.startswith("MIPFilterLUT "):
            _TABLES["ewa"] = np.array(line.split()[2:], dtype=np.float32)
    l.oracle_set_rgb_table(_TABLES["rgb"].ctypes.data, _TABLES["ewa"].ctypes.data)


def texture_eval(scene, material, slot, hit14, lambdas=()):
    """The oracle's evaluation of a textured material parameter at a hit (p, n, dpdu, dpdv, uv):
    ((dudx, dudy, dvdx, dvdy), values) as pbrt_amd.Scene.texture_eval returns them."""
    info, flat = scene.info, scene.flat()
    lam, hit = f32(lambdas), f32(hit14)
    out = np.zeros(5 + lam.size, np.float32)
    rc = lib().oracle_texture_eval(ctypes.byref(flat), ctypes.byref(info), material, slot, hit.ctypes.data,
                                   lam.ctypes.data, lam.size, out.ctypes.data)
    assert rc == 0, rc
    return out[:4].copy(), (out[4:4 + lam.size].copy() if slot == 0 else float(out[4]))


def env_eval(scene, env, dirs, u):
    """The oracle's ImageInfiniteLight lookups, rows as pbrt_amd.Scene.env_eval returns them"""
    flat = scene.flat()
    d = f32(dirs).reshape(-1, 3)
    uu = f32(u).reshape(-1, 2)
    out = np.zeros((len(d), 16), np.float32)
    rc = lib().oracle_env_eval(ctypes.byref(flat), env, d.ctypes.data, uu.ctypes.data, len(d), out.ctypes.data)
    assert rc == 0, rc
    return out


def cloud_density(params3, points):
    """The oracle's Noise / DNoise / CloudMedium density rows, as pbrt_amd.cloud_density"""
    import json
    perm = json.loads((HERE.parent / "pbrt-v4_amd" / "data" / "spectral_data.json").read_text())["NoisePerm"]
    c = f32(list(params3) + perm)
    pts = f32(points).reshape(-1, 3)
    out = np.zeros((len(pts), 5), np.float32)
    assert lib().oracle_cloud_density(c.ctypes.data, pts.ctypes.data, len(pts), out.ctypes.data) == 0
    return out


def medium_point(scene, medium, points, lambdas):
    """Medium::SamplePoint at render-space points and wavelengths [n, 31] -> float32 [n, 3, 31]
    (sigma_a, sigma_s, Le)"""
    flat = scene.flat()
    pts = f32(points).reshape(-1, 3)
    lam = f32(lambdas).reshape(-1, 31)
    out = np.zeros((len(pts), 3, 31), np.float32)
    assert lib().oracle_medium_point(ctypes.byref(flat), medium, pts.ctypes.data, lam.ctypes.data, len(pts),
                                     out.ctypes.data) == 0
    return out


def equal_area(points, to_sphere):
    """The oracle's EqualAreaSquareToSphere / EqualAreaSphereToSquare, as pbrt_amd.equal_area"""
    k_in, k_out = (2, 3) if to_sphere else (3, 2)
    a = f32(points).reshape(-1, k_in)
    out = np.zeros((len(a), k_out), np.float32)
    assert lib().oracle_equal_area(1 if to_sphere else 0, a.ctypes.data, len(a), out.ctypes.data) == 0
    return out


def shape_eval(scene, shape, rays, u):
    """The oracle's sphere / disk evaluation, rows as pbrt_amd.Scene.shape_eval returns them"""
    flat = scene.flat()
    r = f32(rays).reshape(-1, 6)
    uu = f32(u).reshape(-1, 2)
    out = np.zeros((len(r), 40), np.float32)
    rc = lib().oracle_shape_eval(ctypes.byref(flat), shape, r.ctypes.data, uu.ctypes.data, len(r), out.ctypes.data)
    assert rc == 0, rc
    return out


def camera_min_diff(scene):
    """The oracle's own FindMinimumDifferentials: [pos dx, pos dy, dir dx, dir dy] x 3"""
    info, flat = scene.info, scene.flat()
    out = np.zeros(12, np.float32)
    lib().oracle_camera_min_diff(ctypes.byref(flat), ctypes.byref(info), out.ctypes.data)
    return out


def image_level(scene, image, level):
    """Level `level` of the oracle's own MIPMap pyramid of image `image`, as stored bytes"""
    flat = scene.flat()
    w, h = ctypes.c_int(), ctypes.c_int()
    n = lib().oracle_image_level(ctypes.byref(flat), image, level, None, 0, ctypes.byref(w), ctypes.byref(h))
    assert n >= 0
    buf = np.zeros(n, np.uint8)
    lib().oracle_image_level(ctypes.byref(flat), image, level, buf.ctypes.data, n, ctypes.byref(w), ctypes.byref(h))
    return buf, w.value, h.value


MATH_LIBM, MATH_CR = 0, 1


class math_mode:
    """Context manager: the oracle's transcendentals inside the block -- MATH_LIBM (its default:
    glibc's float functions, as pbrt's CPU build calls them, and what the device kernels' detmath.h
    reproduces bit for bit) or MATH_CR (correctly rounded, for sensitivity checks)."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        self.prev = lib().oracle_get_math_mode()
        lib().oracle_set_math_mode(self.mode)
        return self

    def __exit__(self, *exc):
        lib().oracle_set_math_mode(self.prev)
        return False


def set_math_mode(mode):
    lib().oracle_set_math_mode(mode)


def math_eval(fn, a, b=None):
    """The oracle's transcendental `fn` (sin cos asin acos atan2 log exp sinh tan atan expm1) in its
    current mode: libm's float functions (MATH_LIBM) or correctly rounded (MATH_CR)."""
    names = ["sin", "cos", "asin", "acos", "atan2", "log", "exp", "sinh", "tan", "atan", "expm1"]
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), np.float32)
    out = np.zeros_like(a)
    lib().oracle_math_eval(names.index(fn), a.ctypes.data, b.ctypes.data, len(a), out.ctypes.data)
    return out


def f32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def render(scene, rows=None, first_sample=0, n_samples=None, threads=None, path=False):
    """Render `rows` of a pbrt_amd.Scene on the CPU; returns film [4, yres, xres] float64.
    path=False: WavefrontPathIntegrator semantics (the product's); path=True: the CPU
    PathIntegrator (cpu/integrators.cpp:629-805, surfaces only) -- configs[0]'s integrator."""
    info = scene.info
    flat = scene.flat()
    if rows is None:
        rows = np.arange(info.py0, info.py1, dtype=np.int32)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    if n_samples is None:
        n_samples = info.spp - first_sample
    threads = threads or os.cpu_count() or 1
    film = np.zeros((4, info.yres, info.xres), dtype=np.float64)
    fn = lib().oracle_render_path if path else lib().oracle_render
    rc = fn(ctypes.byref(flat), ctypes.byref(info), rows.ctypes.data_as(ctypes.c_void_p),
                             len(rows), int(first_sample), int(n_samples), int(info.uniform_light_sampler),
                             int(threads), film.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return film


def intersect(scene, rays, any_hit=False):
    """rays: float32 [7, n] (o, d, tMax) -> (prim int32 [n], hit float32 [4, n])"""
    info = scene.info
    flat = scene.flat()
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    n = rays.shape[1]
    prim = np.zeros(n, np.int32)
    hit = np.zeros((4, n), np.float32)
    lib().oracle_intersect_batch(ctypes.byref(flat), ctypes.byref(info), rays.ctypes.data_as(ctypes.c_void_p), n,
                                 int(any_hit), prim.ctypes.data_as(ctypes.c_void_p),
                                 hit.ctypes.data_as(ctypes.c_void_p))
    return prim, hit


def intersect_one_random(scene, segs, materials):
    """IntersectOneRandom per probe segment: segs float32 [6, n] (p0, p1), materials int32 [n]
    -> (prim int32 [n], hit float32 [3, n], pdf float32 [n])"""
    info = scene.info
    flat = scene.flat()
    segs = np.ascontiguousarray(segs, dtype=np.float32)
    mats = np.ascontiguousarray(materials, dtype=np.int32)
    n = segs.shape[1]
    prim = np.zeros(n, np.int32)
    hit = np.zeros((3, n), np.float32)
    pdf = np.zeros(n, np.float32)
    vp = ctypes.c_void_p
    lib().oracle_intersect_one_random(ctypes.byref(flat), ctypes.byref(info), vp(segs.ctypes.data), vp(mats.ctypes.data), n,
                                      vp(prim.ctypes.data), vp(hit.ctypes.data), vp(pdf.ctypes.data))
    return prim, hit, pdf


def intersect_tr(scene, rays, medium, lambda0):
    """TraceTransmittance per ray (see pbrt_intersect_tr): rays float32 [7, n], medium int32 [n],
    lambda0 float32 [n] -> float32 [3, 31, n] (T_ray, r_u, r_l)."""
    info = scene.info
    flat = scene.flat()
    rays = np.ascontiguousarray(rays, dtype=np.float32)
    medium = np.ascontiguousarray(medium, dtype=np.int32)
    lambda0 = np.ascontiguousarray(lambda0, dtype=np.float32)
    n = rays.shape[1]
    out = np.zeros((3, 31, n), np.float32)
    lib().oracle_intersect_tr(ctypes.byref(flat), ctypes.byref(info), rays.ctypes.data, medium.ctypes.data,
                              lambda0.ctypes.data, n, out.ctypes.data)
    return out


def film_to_rgb(film, m3x3):
    """RGBFilm::GetPixelRGB: normalise by the weight sum and apply outputRGBFromSensorRGB."""
    w = film[3]
    rgb = film[:3] / np.where(w == 0, 1, w)
    m = np.asarray(m3x3, dtype=np.float64).reshape(3, 3)
    return np.einsum("ij,jhw->hwi", m, rgb).astype(np.float32)


def light_bvh(scene=None, lights13=None):
    """The oracle's own BVHLightSampler tree, over the scene's lights or given [n][13] LightBounds
    rows -> (nodes [m][12] decoded bounds, info [m][3] childOrLight / isLeaf / twoSided, trails)."""
    flat = None if scene is None else scene.flat()
    fp = ctypes.byref(flat) if flat is not None else None
    if lights13 is not None:
        lights13 = np.ascontiguousarray(lights13, dtype=np.float32).reshape(-1, 13)
        n, lp = len(lights13), lights13.ctypes.data
    else:
        n, lp = flat.n_area_lights + flat.n_point_spot, None
    m = lib().oracle_light_bvh(fp, lp, n, None, None, None, 0)
    nodes = np.zeros((max(m, 1), 12), np.float32)
    info = np.zeros((max(m, 1), 3), np.int32)
    trails = np.zeros(max(n, 1), np.uint32)
    lib().oracle_light_bvh(fp, lp, n, nodes.ctypes.data, info.ctypes.data, trails.ctypes.data, m)
    return nodes[:m], info[:m], trails[:n]


def trowbridge(in13):
    i = f32(in13)
    out = np.zeros(14, np.float32)
    lib().oracle_trowbridge(i.ctypes.data, out.ctypes.data)
    return out


def fresnel(in10):
    i = f32(in10)
    out = np.zeros(10, np.float32)
    lib().oracle_fresnel(i.ctypes.data, out.ctypes.data)
    return out


def named_spectrum(interleaved, lambdas):
    src, lam = f32(interleaved), f32(lambdas)
    out = np.zeros(lam.size, np.float32)
    lib().oracle_named_spectrum(src.ctypes.data, src.size, lam.ctypes.data, lam.size, out.ctypes.data)
    return out


def bxdf(bxdf_type, params3, wo, wi, u3, eta31=None, k31=None):
    arrs = [f32(params3), f32(eta31 if eta31 is not None else np.ones(31)),
            f32(k31 if k31 is not None else np.zeros(31)), f32(wo), f32(wi), f32(u3)]
    out = np.zeros(70, np.float32)
    lib().oracle_bxdf(int(bxdf_type), *[a.ctypes.data for a in arrs], out.ctypes.data)
    return out


def layered(params12, a31, b31, alb31, wo, wi, u3):
    arrs = [f32(params12), f32(a31), f32(b31), f32(alb31), f32(wo), f32(wi), f32(u3)]
    out = np.zeros(72, np.float32)
    lib().oracle_layered(*[a.ctypes.data for a in arrs], out.ctypes.data)
    return out


def triangle_shading(p9, n9, uv6, flip, b3, u2):
    p, b, u = f32(p9), f32(b3), f32(u2)
    n = None if n9 is None else f32(n9)
    t = None if uv6 is None else f32(uv6)
    out = np.zeros(15, np.float32)
    lib().oracle_triangle_shading(p.ctypes.data, None if n is None else n.ctypes.data,
                                  None if t is None else t.ctypes.data, int(flip), b.ctypes.data, u.ctypes.data,
                                  out.ctypes.data)
    return out


SAMPLER_KINDS = {"independent": 2, "stratified": 3, "sobol": 4, "paddedsobol": 5}
RANDOMIZE = {"none": 0, "permutedigits": 1, "fastowen": 2, "owen": 3}


def sampler(name, px, py, sample_index, dim, spp=16, seed=0, xsamples=4, ysamples=4, jitter=1,
            randomization="fastowen", xres=256, yres=256, tables=None):
    """The oracle's independent / stratified / sobol / paddedsobol sampler: 7 values in the
    wavefront's call order from StartPixelSample((px, py), sample_index, dim).  tables =
    (SobolMatrices32, VdCSobolMatrices, VdCSobolMatricesInv) numpy arrays (sobol only)."""
    out = np.zeros(7, np.float32)
    m32, vdc, inv = tables if tables is not None else (None, None, None)
    ptr = lambda a: None if a is None else a.ctypes.data
    lib().oracle_sampler(SAMPLER_KINDS[name], spp, seed, xsamples, ysamples, jitter, RANDOMIZE[randomization],
                         xres, yres, ptr(m32), ptr(vdc), ptr(inv), px, py, sample_index, dim, out.ctypes.data)
    return out


def rng(seq, advance):
    """RNG::SetSequence(seq), Advance(advance), two Uniform<uint32_t>() (oracle restatement)."""
    out = np.zeros(2, np.uint32)
    lib().oracle_rng(int(seq), int(advance), out.ctypes.data)
    return int(out[0]), int(out[1])


SSS_TABLE_FLOATS = 100 + 64 + 2 * 100 * 64 + 100


def sss_table(g, eta):
    """The oracle's BSSRDF table for (g, eta): rho[100], radius[64], profile[100][64], rhoEff[100],
    profileCDF[100][64] (ComputeBeamDiffusionBSSRDF restated)."""
    out = np.zeros(SSS_TABLE_FLOATS, np.float32)
    lib().oracle_sss_table(float(g), float(eta), out.ctypes.data)
    return out


def catmull_rom(op, nodes1, nodes2, values, cdf, x):
    """The oracle's spline restatements: op 0 weights [n][6], 1 invert [n], 3 sample2d (x: [n][2])."""
    a = [np.ascontiguousarray(v, np.float32) for v in (nodes1, nodes2, values, cdf, x)]
    n = len(a[4]) // 2 if op == 3 else len(a[4])
    out = np.zeros(n * 6 if op == 0 else n, np.float32)
    lib().oracle_catmull_rom(op, a[0].ctypes.data, len(a[0]), a[1].ctypes.data, len(a[1]), a[2].ctypes.data,
                             a[3].ctypes.data, a[4].ctypes.data, n, out.ctypes.data)
    return out.reshape(-1, 6) if op == 0 else out


def portal_eval(scene, env, queries, res=0):
    """The oracle's PortalImageInfiniteLight on [n][8] queries {p, d, u0, u1} -> [n][16] (see
    oracle_portal_eval); with res > 0 also its rectified image [res][res][3] and function."""
    f = scene.flat()
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 8)
    out = np.zeros((len(q), 16), np.float32)
    img = np.zeros(res * res * 4, np.float32) if res else None
    rc = lib().oracle_portal_eval(ctypes.byref(f), env, q.ctypes.data, len(q), out.ctypes.data,
                                  img.ctypes.data if img is not None else None)
    if rc != 0:
        raise RuntimeError(f"oracle_portal_eval failed ({rc})")
    if img is None:
        return out
    np_ = res * res
    return out, img[:3 * np_].reshape(res, res, 3), img[3 * np_:].reshape(res, res)


def hair_eval(queries):
    """The oracle's HairBxDF (f, PDF, Sample_f) on [n][16] queries laid out as the product's
    hair_eval -> [n][68], in the current math mode."""
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 16)
    out = np.zeros((len(q), 68), np.float32)
    lib().oracle_hair_eval(q.ctypes.data, len(q), out.ctypes.data)
    return out


def measured_eval(path, queries, lambdas):
    """The oracle's MeasuredBxDF read from the tensor file `path` (its own reader and
    PiecewiseLinear2D) on [n][8] queries {wo, wi, u0, u1} -> [n][68], in the current math mode."""
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 8)
    lam = np.ascontiguousarray(lambdas, np.float32).reshape(31)
    out = np.zeros((len(q), 68), np.float32)
    if lib().oracle_measured_eval(str(path).encode(), q.ctypes.data, len(q), lam.ctypes.data, out.ctypes.data) != 0:
        raise OSError(f"oracle: cannot read {path}")
    return out


def pl2d(dim, cdf, data, xs, ys, pr, pv0, pv1, queries):
    """The oracle's PiecewiseLinear2D<dim> (normalised; CDF iff cdf) over data [pr0][pr1][ys][xs] on
    [n][6] queries {u0, u1, px, py, p0, p1} -> [n][7] {Sample xy pdf, Invert xy pdf, Evaluate}."""
    d = np.ascontiguousarray(data, np.float32)
    pr = np.ascontiguousarray(pr, np.int32)
    a0, a1 = np.ascontiguousarray(pv0, np.float32), np.ascontiguousarray(pv1, np.float32)
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 6)
    out = np.zeros((len(q), 7), np.float32)
    if lib().oracle_pl2d(dim, cdf, d.ctypes.data, xs, ys, pr.ctypes.data, a0.ctypes.data, a1.ctypes.data,
                         q.ctypes.data, len(q), out.ctypes.data) != 0:
        raise ValueError("oracle_pl2d: bad table")
    return out


def windowed2d(func, queries):
    """The oracle's WindowedPiecewiseConstant2D over func [n][n] on [k][8] queries
    {u0, u1, b0, b1, b2, b3, qx, qy} -> [k][5] {ok, x, y, pdf, PDF(q, b)}."""
    f = np.ascontiguousarray(func, np.float32)
    n = int(round(np.sqrt(f.size)))
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 8)
    out = np.zeros((len(q), 5), np.float32)
    if lib().oracle_windowed2d(f.ctypes.data, n, q.ctypes.data, len(q), out.ctypes.data) != 0:
        raise ValueError("oracle_windowed2d: bad table")
    return out


def procedural(kind, perm, params4, in9):
    """The oracle's procedural textures (fbm, turbulence, windy, polka dot, marble): [n][6]."""
    perm = np.ascontiguousarray(perm, np.float32)
    par = np.ascontiguousarray(params4, np.float32)
    x = np.ascontiguousarray(in9, np.float32).reshape(-1, 9)
    out = np.zeros((len(x), 6), np.float32)
    lib().oracle_procedural(kind, perm.ctypes.data, par.ctypes.data, x.ctypes.data, len(x), out.ctypes.data)
    return out
