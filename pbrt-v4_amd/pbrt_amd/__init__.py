"""pbrt_amd — Python host mirror of pbrt-v4's wavefront rendering entry points, bound to
the MI355X C ABI in ``include/pbrt_amd.h`` (``lib/libpbrt_amd.so``).

Reference interfaces mirrored (scienstanford/pbrt-v4):

* ``RenderWavefront(scene)``            -> ``pbrt::RenderWavefront(BasicScene&)``
                                            (src/pbrt/wavefront/wavefront.cpp:14-72)
* ``WavefrontPathIntegrator``           -> ``pbrt::WavefrontPathIntegrator``
                                            (src/pbrt/wavefront/integrator.h:57-190)
* ``HIPAggregate.IntersectClosest/Shadow`` -> ``pbrt::WavefrontAggregate``
                                            (src/pbrt/wavefront/integrator.h:32-54)
* ``load_scene``                        -> ``pbrt::ParseFiles`` + ``BasicScene`` (scene.h:260)

Errors follow pbrt's fail-fast convention: every C-ABI failure raises ``PbrtError`` with
the library's message.  There is no CPU fallback: if the HIP library is missing the import
of ``_lib()`` raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
ROOT = PKG_DIR.parent
# PBRT_AMD_LIB selects a profiling build (lib/libpbrt_amd_prof.so, tools only)
LIB_PATH = Path(os.environ.get("PBRT_AMD_LIB", ROOT / "lib" / "libpbrt_amd.so"))
DATA_DIR = ROOT / "data"


class PbrtError(RuntimeError):
    pass


class SceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "xres yres px0 px1 py0 py1 spp seed max_depth n_triangles n_vertices n_materials "
        "n_area_lights n_infinite_lights n_light_nodes uniform_light_sampler").split()] + [
        ("filter_radius_x", ctypes.c_float), ("filter_radius_y", ctypes.c_float)]


class SceneFlat(ctypes.Structure):
    _fields_ = [
        ("n_vertices", ctypes.c_int), ("n_triangles", ctypes.c_int), ("n_materials", ctypes.c_int),
        ("n_area_lights", ctypes.c_int), ("n_infinite_lights", ctypes.c_int), ("n_spectra", ctypes.c_int),
        ("vertices", ctypes.POINTER(ctypes.c_float)), ("triangles", ctypes.POINTER(ctypes.c_int32)),
        ("tri_material", ctypes.POINTER(ctypes.c_int32)), ("tri_light", ctypes.POINTER(ctypes.c_int32)),
        ("tri_flip", ctypes.POINTER(ctypes.c_uint8)), ("material_coeffs", ctypes.POINTER(ctypes.c_float)),
        ("material_constant", ctypes.POINTER(ctypes.c_int32)), ("light_prim", ctypes.POINTER(ctypes.c_int32)),
        ("light_scale", ctypes.POINTER(ctypes.c_float)), ("light_spectrum", ctypes.POINTER(ctypes.c_int32)),
        ("light_two_sided", ctypes.POINTER(ctypes.c_int32)), ("light_spread", ctypes.POINTER(ctypes.c_float)),
        ("light_image", ctypes.POINTER(ctypes.c_int32)), ("area_images", ctypes.POINTER(ctypes.c_float)), ("inf_spectrum", ctypes.POINTER(ctypes.c_int32)),
        ("inf_scale", ctypes.POINTER(ctypes.c_float)), ("dense_spectra", ctypes.POINTER(ctypes.c_float)),
        ("sensor_xyz", ctypes.POINTER(ctypes.c_float)), ("imaging_ratio", ctypes.c_float),
        ("camera_from_raster", ctypes.c_float * 16), ("render_from_camera", ctypes.c_float * 16),
        ("lens_radius", ctypes.c_float), ("focal_distance", ctypes.c_float),
        ("output_rgb_from_sensor_rgb", ctypes.c_double * 9),
        ("n_light_nodes", ctypes.c_int), ("light_node_bounds", ctypes.POINTER(ctypes.c_float)),
        ("light_node_info", ctypes.POINTER(ctypes.c_int32)), ("light_bit_trail", ctypes.POINTER(ctypes.c_uint32)),
        ("halton_base_scales", ctypes.c_int * 2), ("halton_base_exponents", ctypes.c_int * 2),
        ("halton_mult_inverse", ctypes.c_int * 2), ("n_dims", ctypes.c_int),
        ("perm_table", ctypes.POINTER(ctypes.c_uint16)), ("perm_offset", ctypes.POINTER(ctypes.c_uint32)),
        ("perm_ndigits", ctypes.POINTER(ctypes.c_uint32)), ("perm_base", ctypes.POINTER(ctypes.c_uint32)),
        ("sampler_type", ctypes.c_int), ("zs_randomize", ctypes.c_int), ("zs_log2_spp", ctypes.c_int),
        ("zs_nbase4_digits", ctypes.c_int),
        ("material_type", ctypes.POINTER(ctypes.c_int32)), ("material_params", ctypes.POINTER(ctypes.c_float)),
        ("material_spectra", ctypes.POINTER(ctypes.c_int32)), ("n_pl_spectra", ctypes.c_int),
        ("pl_offsets", ctypes.POINTER(ctypes.c_int32)), ("pl_lambda", ctypes.POINTER(ctypes.c_float)),
        ("pl_value", ctypes.POINTER(ctypes.c_float)), ("regularize", ctypes.c_int),
        ("vertex_normals", ctypes.POINTER(ctypes.c_float)), ("vertex_uv", ctypes.POINTER(ctypes.c_float)),
        ("tri_shading", ctypes.POINTER(ctypes.c_uint8)),
        ("n_media", ctypes.c_int), ("camera_medium", ctypes.c_int),
        ("medium_info", ctypes.POINTER(ctypes.c_int32)), ("medium_params", ctypes.POINTER(ctypes.c_float)),
        ("medium_values", ctypes.POINTER(ctypes.c_float)), ("tri_medium", ctypes.POINTER(ctypes.c_int16)),
        ("filter_type", ctypes.c_int), ("filter_a", ctypes.c_float), ("filter_b", ctypes.c_float),
        ("material_layer", ctypes.POINTER(ctypes.c_float)),
        ("n_delta_lights", ctypes.c_int), ("n_point_spot", ctypes.c_int),
        ("delta_lights", ctypes.POINTER(ctypes.c_float)), ("delta_images", ctypes.POINTER(ctypes.c_float)), ("inf_distant", ctypes.POINTER(ctypes.c_int32)),
        ("uniform_order", ctypes.POINTER(ctypes.c_int32)), ("scene_radius", ctypes.c_float),
        ("n_tex_nodes", ctypes.c_int), ("n_images", ctypes.c_int),
        ("tex_node_info", ctypes.POINTER(ctypes.c_int32)), ("tex_node_params", ctypes.POINTER(ctypes.c_float)),
        ("tex_node_spec", ctypes.POINTER(ctypes.c_float)), ("image_info", ctypes.POINTER(ctypes.c_int32)),
        ("image_levels", ctypes.POINTER(ctypes.c_int32)), ("image_data", ctypes.POINTER(ctypes.c_uint8)),
        ("image_luts", ctypes.POINTER(ctypes.c_float)), ("image_raw_info", ctypes.POINTER(ctypes.c_int32)),
        ("image_raw_gamma", ctypes.POINTER(ctypes.c_float)), ("image_raw_offset", ctypes.POINTER(ctypes.c_uint64)),
        ("image_raw_data", ctypes.POINTER(ctypes.c_uint8)), ("material_tex", ctypes.POINTER(ctypes.c_int32)),
        ("camera_from_render", ctypes.c_float * 12), ("camera_min_diff", ctypes.c_float * 12),
        ("material_mix", ctypes.POINTER(ctypes.c_int32)),
        ("n_env", ctypes.c_int),
        ("inf_image", ctypes.POINTER(ctypes.c_int32)),
        ("env_info", ctypes.POINTER(ctypes.c_int32)),
        ("env_xform", ctypes.POINTER(ctypes.c_float)),
        ("env_offset", ctypes.POINTER(ctypes.c_uint64)),
        ("env_rgb", ctypes.POINTER(ctypes.c_float)),
        ("n_shapes", ctypes.c_int),
        ("shape_info", ctypes.POINTER(ctypes.c_int32)),
        ("shape_params", ctypes.POINTER(ctypes.c_float)),
        ("shape_normals", ctypes.POINTER(ctypes.c_float)),
        ("prim_alpha", ctypes.POINTER(ctypes.c_int32)),
        ("max_component_value", ctypes.c_float),
        ("xyz_from_sensor_rgb", ctypes.c_float * 9),
        ("material_bump", ctypes.POINTER(ctypes.c_int32)),
        ("strat_xsamples", ctypes.c_int), ("strat_ysamples", ctypes.c_int), ("strat_jitter", ctypes.c_int),
        ("sobol_log2_scale", ctypes.c_int), ("sobol_matrices32", ctypes.POINTER(ctypes.c_uint32)),
        ("vdc_sobol", ctypes.POINTER(ctypes.c_uint64)), ("vdc_sobol_inv", ctypes.POINTER(ctypes.c_uint64)),
        ("noise_perm", ctypes.POINTER(ctypes.c_float)),
        ("n_sss", ctypes.c_int),
        ("dims_per_depth", ctypes.c_int),
        ("material_sss", ctypes.POINTER(ctypes.c_int32)),
        ("sss_params", ctypes.POINTER(ctypes.c_float)),
        ("sss_tables", ctypes.POINTER(ctypes.c_float)),
        ("vertex_s", ctypes.POINTER(ctypes.c_float)), ("n_vertex_s", ctypes.c_int),
        ("env_portal", ctypes.POINTER(ctypes.c_float)),
        ("n_measured", ctypes.c_int),
        ("measured_files", ctypes.POINTER(ctypes.c_char_p)),
        ("options", ctypes.c_int),
        ("tex_basis", ctypes.POINTER(ctypes.c_float)),
        ("material_hair_tex", ctypes.POINTER(ctypes.c_int32)),
        ("material_sss_tex", ctypes.POINTER(ctypes.c_int32)),
    ]


class RenderParams(ctypes.Structure):
    _fields_ = [("rows", ctypes.POINTER(ctypes.c_int32)), ("n_rows", ctypes.c_int),
                ("first_sample", ctypes.c_int), ("n_samples", ctypes.c_int), ("time_closest", ctypes.c_int)]


class RenderStats(ctypes.Structure):
    _fields_ = [("camera_rays", ctypes.c_uint64), ("closest_rays", ctypes.c_uint64),
                ("shadow_rays", ctypes.c_uint64), ("closest_launches", ctypes.c_int),
                ("closest_ms", ctypes.c_double), ("timed_closest_rays", ctypes.c_uint64), ("passes", ctypes.c_int),
                ("paths_per_pass", ctypes.c_uint64), ("bvh_hbm_node_bytes", ctypes.c_uint64),
                ("bvh_hbm_tri_bytes", ctypes.c_uint64)]


class KernelStat(ctypes.Structure):
    _fields_ = [("description", ctypes.c_char * 96), ("launches", ctypes.c_int), ("total_ms", ctypes.c_double),
                ("min_ms", ctypes.c_double), ("max_ms", ctypes.c_double)]


# Symbols declared in include/pbrt_amd.h (tests check every one is exported)
EXPORTED_SYMBOLS = [
    "pbrt_last_error", "pbrt_set_data_dir", "pbrt_scene_load", "pbrt_scene_load_string", "pbrt_scene_free",
    "pbrt_scene_get_info", "pbrt_scene_get_flat", "pbrt_device_count", "pbrt_context_create",
    "pbrt_context_free", "pbrt_render", "pbrt_synchronize", "pbrt_get_stats", "pbrt_reset_stats",
    "pbrt_film_clear", "pbrt_film_device_ptr", "pbrt_film_read", "pbrt_film_get_rgb", "pbrt_intersect",
    "pbrt_debug_halton", "pbrt_debug_halton_fastpath_mismatches", "pbrt_debug_catmull_rom", "pbrt_debug_check_rn_math", "pbrt_debug_rgb_coeffs", "pbrt_debug_rgb2spec_column", "pbrt_debug_kernel_sections",
    "pbrt_debug_queue_counts", "pbrt_debug_zsobol", "pbrt_debug_sampler", "pbrt_debug_rng", "pbrt_debug_det_math", "pbrt_debug_hair", "pbrt_debug_measured", "pbrt_debug_catmull_rom_gpu", "pbrt_debug_portal_eval", "pbrt_debug_procedural", "pbrt_debug_trowbridge", "pbrt_debug_fresnel",
    "pbrt_debug_named_spectrum", "pbrt_debug_bxdf", "pbrt_debug_layered", "pbrt_debug_triangle_shading", "pbrt_film_write_image",
    "pbrt_image_read_size", "pbrt_image_read", "pbrt_image_write", "pbrt_image_error", "pbrt_debug_filter_sample",
    "pbrt_debug_bvh_stats", "pbrt_debug_bvh_trace", "pbrt_debug_light_bvh", "pbrt_intersect_tr", "pbrt_intersect_one_random", "pbrt_image_flip", "pbrt_set_kernel_profiling", "pbrt_get_kernel_stats",
    "pbrt_debug_texture_eval",
    "pbrt_debug_env_eval",
    "pbrt_debug_shape_eval",
    "pbrt_debug_set_queue_check", "pbrt_debug_queue_holes",
    "pbrt_debug_equal_area", "pbrt_debug_cloud_density",
    "pbrt_debug_pl2d", "pbrt_debug_windowed2d", "pbrt_debug_displace",
    "pbrt_color_space_index", "pbrt_debug_color_space", "pbrt_debug_rgb_spectrum", "pbrt_debug_rgb2spec_column_cs",
]

_LIB = None


def _lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not LIB_PATH.exists():
        raise PbrtError(f"HIP library {LIB_PATH} is missing: build it with __graft_entry__.build() "
                        "(make -C pbrt-v4_amd); there is no CPU fallback")
    # One HIP runtime per process: torch ships its own libamdhip64 with the same soname as
    # /opt/rocm's.  Whichever loads first serves both, and torch cannot initialise on the
    # system runtime ("No HIP GPUs are available"), so torch (when installed) goes first.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(str(LIB_PATH))
    c = ctypes
    lib.pbrt_last_error.restype = c.c_char_p
    lib.pbrt_set_data_dir.argtypes = [c.c_char_p]
    lib.pbrt_scene_load.argtypes = [c.c_char_p, c.c_char_p, c.POINTER(c.c_void_p)]
    lib.pbrt_scene_load_string.argtypes = [c.c_char_p, c.c_char_p, c.c_char_p, c.POINTER(c.c_void_p)]
    lib.pbrt_scene_free.argtypes = [c.c_void_p]
    lib.pbrt_debug_filter_sample.argtypes = [c.c_void_p, c.c_float, c.c_float, c.c_void_p]
    lib.pbrt_film_write_image.argtypes = [c.c_void_p, c.c_char_p, c.c_int]
    lib.pbrt_image_read_size.argtypes = [c.c_char_p, c.POINTER(c.c_int), c.POINTER(c.c_int)]
    lib.pbrt_image_read.argtypes = [c.c_char_p, c.c_void_p, c.c_int, c.c_int]
    lib.pbrt_image_write.argtypes = [c.c_char_p, c.c_void_p, c.c_int, c.c_int, c.c_int]
    lib.pbrt_image_error.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_char_p, c.c_void_p]
    lib.pbrt_scene_get_info.argtypes = [c.c_void_p, c.POINTER(SceneInfo)]
    lib.pbrt_scene_get_flat.argtypes = [c.c_void_p, c.POINTER(SceneFlat)]
    lib.pbrt_device_count.argtypes = [c.POINTER(c.c_int)]
    lib.pbrt_context_create.argtypes = [c.c_void_p, c.c_int, c.c_int64, c.POINTER(c.c_void_p)]
    lib.pbrt_context_free.argtypes = [c.c_void_p]
    lib.pbrt_render.argtypes = [c.c_void_p, c.POINTER(RenderParams)]
    lib.pbrt_synchronize.argtypes = [c.c_void_p]
    lib.pbrt_get_stats.argtypes = [c.c_void_p, c.POINTER(RenderStats)]
    lib.pbrt_reset_stats.argtypes = [c.c_void_p]
    lib.pbrt_film_clear.argtypes = [c.c_void_p]
    lib.pbrt_film_device_ptr.argtypes = [c.c_void_p, c.POINTER(c.c_void_p), c.POINTER(c.c_size_t)]
    lib.pbrt_film_read.argtypes = [c.c_void_p, c.c_void_p]
    lib.pbrt_film_get_rgb.argtypes = [c.c_void_p, c.c_void_p]
    lib.pbrt_intersect.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p]
    lib.pbrt_debug_bvh_stats.argtypes = [c.c_void_p, c.c_void_p]
    lib.pbrt_debug_bvh_trace.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p]
    lib.pbrt_image_flip.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_int, c.c_void_p]
    lib.pbrt_intersect_tr.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_intersect_one_random.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p, c.c_void_p,
                                              c.c_void_p]
    lib.pbrt_set_kernel_profiling.argtypes = [c.c_void_p, c.c_int]
    lib.pbrt_debug_light_bvh.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p, c.c_int,
                                         c.POINTER(c.c_int)]
    lib.pbrt_get_kernel_stats.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.POINTER(c.c_int)]
    lib.pbrt_debug_halton.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int]
    lib.pbrt_debug_halton.restype = c.c_float
    lib.pbrt_debug_catmull_rom.argtypes = [c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_void_p,
                                           c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_halton_fastpath_mismatches.argtypes = [c.c_void_p, c.c_int, c.c_uint32, c.c_uint32, c.c_uint32]
    lib.pbrt_debug_halton_fastpath_mismatches.restype = c.c_int64
    lib.pbrt_debug_check_rn_math.argtypes = [c.c_int, c.c_uint64, c.c_int64, c.POINTER(c.c_int64),
                                             c.POINTER(c.c_float)]
    lib.pbrt_debug_rgb_coeffs.argtypes = [c.c_float, c.c_float, c.c_float, c.POINTER(c.c_float)]
    lib.pbrt_debug_rgb2spec_column.argtypes = [c.c_int, c.c_int, c.c_int, c.POINTER(c.c_float)]
    lib.pbrt_debug_kernel_sections.argtypes = [c.c_void_p, c.POINTER(c.c_uint64), c.c_int]
    lib.pbrt_debug_zsobol.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.POINTER(c.c_float)]
    lib.pbrt_debug_sampler.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_int, c.c_int, c.POINTER(c.c_float)]
    lib.pbrt_debug_rng.argtypes = [c.c_uint64, c.c_uint64, c.POINTER(c.c_uint32)]
    lib.pbrt_debug_det_math.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_hair.argtypes = [c.c_int, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_catmull_rom_gpu.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p,
                                               c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_portal_eval.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_void_p]
    lib.pbrt_debug_measured.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_void_p]
    lib.pbrt_debug_displace.argtypes = [c.c_void_p, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p, c.c_int,
                                        c.c_void_p, c.c_float, c.c_int, c.c_int, c.c_int] + [c.c_void_p] * 5
    lib.pbrt_debug_pl2d.argtypes = [c.c_int, c.c_int, c.c_void_p, c.c_int, c.c_int] + [c.c_void_p] * 4 + [
        c.c_int, c.c_void_p]
    lib.pbrt_debug_windowed2d.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_color_space_index.argtypes = [c.c_char_p]
    lib.pbrt_debug_color_space.argtypes = [c.c_int, c.c_void_p]
    lib.pbrt_debug_rgb_spectrum.argtypes = [c.c_int, c.c_void_p, c.c_int, c.c_float, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_rgb2spec_column_cs.argtypes = [c.c_int] * 4 + [c.c_void_p]
    lib.pbrt_debug_procedural.argtypes = [c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_queue_counts.argtypes = [c.c_void_p, c.POINTER(c.c_int32), c.c_int]
    lib.pbrt_debug_trowbridge.argtypes = [c.c_void_p, c.c_void_p]
    lib.pbrt_debug_fresnel.argtypes = [c.c_void_p, c.c_void_p]
    lib.pbrt_debug_named_spectrum.argtypes = [c.c_char_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_bxdf.argtypes = [c.c_int] + [c.c_void_p] * 7
    lib.pbrt_debug_layered.argtypes = [c.c_void_p] * 8
    lib.pbrt_debug_triangle_shading.argtypes = [c.c_void_p] * 3 + [c.c_int] + [c.c_void_p] * 3
    lib.pbrt_debug_texture_eval.argtypes = [c.c_void_p, c.c_int, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_env_eval.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_shape_eval.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_set_queue_check.argtypes = [c.c_int]
    lib.pbrt_debug_queue_holes.argtypes = [c.POINTER(c.c_int)]
    lib.pbrt_debug_equal_area.argtypes = [c.c_int, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_debug_cloud_density.argtypes = [c.c_void_p, c.c_void_p, c.c_int, c.c_void_p]
    lib.pbrt_set_data_dir(str(DATA_DIR).encode())
    _LIB = lib
    return lib


def cloud_density(params3, points):
    """pbrt_debug_cloud_density: [n, 5] rows Noise(p), DNoise(p) xyz, CloudMedium Density(p)."""
    import numpy as np
    p = np.ascontiguousarray(np.asarray(params3, np.float32).reshape(3))
    pts = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 3))
    out = np.zeros((len(pts), 5), np.float32)
    _check(_lib().pbrt_debug_cloud_density(p.ctypes.data, pts.ctypes.data, len(pts), out.ctypes.data))
    return out


def equal_area(points, to_sphere):
    """EqualAreaSquareToSphere (to_sphere: points[n][2] -> [n][3]) or EqualAreaSphereToSquare
    ([n][3] -> [n][2]) with the product's shared host/device code (pbrt_debug_equal_area)."""
    k_in, k_out = (2, 3) if to_sphere else (3, 2)
    a = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, k_in)
    out = np.zeros((len(a), k_out), np.float32)
    _check(_lib().pbrt_debug_equal_area(1 if to_sphere else 0, a.ctypes.data, len(a), out.ctypes.data))
    return out


def _f32(a, n=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32))
    if n is not None and a.size != n:
        raise PbrtError(f"expected {n} values, got {a.size}")
    return a


def set_queue_check(on):
    """Turns the volumetric wavefront's queue-integrity check on or off (diagnostics)."""
    _check(_lib().pbrt_debug_set_queue_check(1 if on else 0))


def queue_holes():
    """Queue slots counted but never written since the last call (0 with the check off)."""
    n = ctypes.c_int(0)
    _check(_lib().pbrt_debug_queue_holes(ctypes.byref(n)))
    return n.value


def debug_light_bvh(lights13):
    """The loader's light-BVH build over [n][13] LightBounds rows -> (nodes [m][12] decoded bounds,
    info [m][3] childOrLight / isLeaf / twoSided, trails [n] uint32)."""
    lights13 = np.ascontiguousarray(lights13, dtype=np.float32).reshape(-1, 13)
    n = len(lights13)
    m = ctypes.c_int(0)
    _check(_lib().pbrt_debug_light_bvh(lights13.ctypes.data, n, None, None, None, 0, ctypes.byref(m)))
    nodes = np.zeros((max(m.value, 1), 12), np.float32)
    info = np.zeros((max(m.value, 1), 3), np.int32)
    trails = np.zeros(max(n, 1), np.uint32)
    _check(_lib().pbrt_debug_light_bvh(lights13.ctypes.data, n, nodes.ctypes.data, info.ctypes.data,
                                       trails.ctypes.data, m.value, ctypes.byref(m)))
    return nodes[:m.value], info[:m.value], trails[:n]


def debug_trowbridge(in13):
    """TrowbridgeReitzDistribution terms as the product computes them (see pbrt_amd.h)."""
    i, o = _f32(in13, 13), np.zeros(14, np.float32)
    _check(_lib().pbrt_debug_trowbridge(i.ctypes.data, o.ctypes.data))
    return o


def debug_fresnel(in10):
    i, o = _f32(in10, 10), np.zeros(10, np.float32)
    _check(_lib().pbrt_debug_fresnel(i.ctypes.data, o.ctypes.data))
    return o


def named_spectrum(name, lambdas):
    """GetNamedSpectrum(name)(lambda) for the metal / glass tables."""
    lam = _f32(lambdas)
    o = np.zeros(lam.size, np.float32)
    _check(_lib().pbrt_debug_named_spectrum(name.encode(), lam.ctypes.data, lam.size, o.ctypes.data))
    return o


def debug_triangle_shading(p9, n9, uv6, flip, b3, u2):
    """TriangleSurface (+ Triangle::Sample normal) with optional vertex normals / uv: 15 floats."""
    p, b, u = _f32(p9, 9), _f32(b3, 3), _f32(u2, 2)
    n = None if n9 is None else _f32(n9, 9)
    t = None if uv6 is None else _f32(uv6, 6)
    o = np.zeros(15, np.float32)
    _check(_lib().pbrt_debug_triangle_shading(p.ctypes.data, None if n is None else n.ctypes.data,
                                              None if t is None else t.ctypes.data, int(flip), b.ctypes.data,
                                              u.ctypes.data, o.ctypes.data))
    return o


def debug_bxdf(bxdf_type, params3, wo, wi, u3, eta31=None, k31=None):
    """Sample_f / f / PDF of DielectricBxDF (1) or ConductorBxDF (2): 70 floats (pbrt_amd.h)."""
    p, a, b, u = _f32(params3, 3), _f32(wo, 3), _f32(wi, 3), _f32(u3, 3)
    e = _f32(eta31 if eta31 is not None else np.ones(31), 31)
    k = _f32(k31 if k31 is not None else np.zeros(31), 31)
    o = np.zeros(70, np.float32)
    _check(_lib().pbrt_debug_bxdf(int(bxdf_type), p.ctypes.data, e.ctypes.data, k.ctypes.data, a.ctypes.data,
                                  b.ctypes.data, u.ctypes.data, o.ctypes.data))
    return o


def debug_pl2d(dim, cdf, data, xs, ys, pr, pv0, pv1, queries):
    """PiecewiseLinear2D<dim> on the host (pbrt_debug_pl2d): [n][6] queries {u0, u1, px, py, p0, p1}
    -> [n][7] {Sample xy pdf, Invert xy pdf, Evaluate}."""
    d = np.ascontiguousarray(data, np.float32)
    p = np.ascontiguousarray(pr, np.int32)
    a0, a1 = np.ascontiguousarray(pv0, np.float32), np.ascontiguousarray(pv1, np.float32)
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 6)
    o = np.zeros((len(q), 7), np.float32)
    _check(_lib().pbrt_debug_pl2d(int(dim), int(cdf), d.ctypes.data, int(xs), int(ys), p.ctypes.data, a0.ctypes.data,
                                  a1.ctypes.data, q.ctypes.data, len(q), o.ctypes.data))
    return o


def debug_displace(P, uv, N, tri, quad, render_from_object, edge_length, mode):
    """The plymesh displacement (pbrt_debug_displace) with a closed-form displacement (mode 0:
    0.1 u - 0.05 v, mode 1: 0.25 p.y u + 0.125, mode 2: 0.1): returns (P, N, uv, tri) of the refined mesh."""
    p = np.ascontiguousarray(P, np.float32).reshape(-1, 3)
    t = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
    n = None if N is None or len(N) == 0 else np.ascontiguousarray(N, np.float32).reshape(-1, 3)
    tr = np.ascontiguousarray(tri, np.int32).reshape(-1)
    qd = np.ascontiguousarray(quad, np.int32).reshape(-1)
    m = np.ascontiguousarray(render_from_object, np.float32).reshape(16)
    cap_v, cap_t = 1 << 16, 1 << 17
    po, no = np.zeros((cap_v, 3), np.float32), np.zeros((cap_v, 3), np.float32)
    uo, to = np.zeros((cap_v, 2), np.float32), np.zeros((cap_t, 3), np.int32)
    cnt = np.zeros(2, np.int32)
    _check(_lib().pbrt_debug_displace(p.ctypes.data, t.ctypes.data, None if n is None else n.ctypes.data, len(p),
                                      tr.ctypes.data, len(tr) // 3, qd.ctypes.data, len(qd) // 4, m.ctypes.data,
                                      float(edge_length), int(mode), cap_v, cap_t, po.ctypes.data, no.ctypes.data,
                                      uo.ctypes.data, to.ctypes.data, cnt.ctypes.data))
    nv, nt = int(cnt[0]), int(cnt[1])
    return po[:nv], no[:nv], uo[:nv], to[:nt]


COLOR_SPACES = ("srgb", "dci-p3", "rec2020", "aces2065-1")


def color_space_index(name):
    """ColorSpace directive name -> index 0..3 (RGBColorSpace::GetNamed; raises when unknown)."""
    k = _lib().pbrt_color_space_index(name.encode())
    if k < 0:
        raise PbrtError(_lib().pbrt_last_error().decode())
    return k


def debug_color_space(cs):
    """One colour space's constants (pbrt_debug_color_space): dict of prim[6], w[2],
    xyz_from_rgb / rgb_from_xyz [3][3], photometric, illuminant[311]."""
    o = np.zeros(338, np.float32)
    _check(_lib().pbrt_debug_color_space(int(cs), o.ctypes.data))
    return {"prim": o[:6], "w": o[6:8], "xyz_from_rgb": o[8:17].reshape(3, 3), "rgb_from_xyz": o[17:26].reshape(3, 3),
            "photometric": o[26], "illuminant": o[27:]}


def debug_rgb_spectrum(cs, rgbs, lambdas, unbounded_scale=1.0):
    """RGB -> spectrum in colour space cs (pbrt_debug_rgb_spectrum): [n][3 + 3 nl] rows of
    coefficients, albedo(lambda), unbounded(s rgb)(lambda), illuminant(s rgb)(lambda)."""
    x = np.ascontiguousarray(rgbs, np.float32).reshape(-1, 3)
    lam = np.ascontiguousarray(lambdas, np.float32).ravel()
    o = np.zeros((len(x), 3 + 3 * len(lam)), np.float32)
    _check(_lib().pbrt_debug_rgb_spectrum(int(cs), x.ctypes.data, len(x), float(unbounded_scale), lam.ctypes.data,
                                          len(lam), o.ctypes.data))
    return o


def debug_rgb2spec_column(cs, maxc, j, i):
    """Column (maxc, j, i) of colour space cs's RGBToSpectrumTable: [64][3]."""
    o = np.zeros(192, np.float32)
    _check(_lib().pbrt_debug_rgb2spec_column_cs(int(cs), int(maxc), int(j), int(i), o.ctypes.data))
    return o.reshape(64, 3)


def debug_windowed2d(func, queries):
    """WindowedPiecewiseConstant2D on the host (pbrt_debug_windowed2d) over func [n][n]: [k][8]
    queries {u0, u1, b0, b1, b2, b3, qx, qy} -> [k][5] {ok, x, y, pdf, PDF(q, b)}."""
    f = np.ascontiguousarray(func, np.float32)
    n = int(round(np.sqrt(f.size)))
    if n * n != f.size:
        raise ValueError("debug_windowed2d: func must be square")
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, 8)
    o = np.zeros((len(q), 5), np.float32)
    _check(_lib().pbrt_debug_windowed2d(f.ctypes.data, n, q.ctypes.data, len(q), o.ctypes.data))
    return o


def debug_layered(params12, a31, b31, alb31, wo, wi, u3):
    """Sample_f / f / PDF / Flags of a LayeredBxDF (coated diffuse or conductor): 72 floats
    (pbrt_amd.h pbrt_debug_layered)."""
    arrs = [_f32(params12, 12), _f32(a31, 31), _f32(b31, 31), _f32(alb31, 31), _f32(wo, 3), _f32(wi, 3), _f32(u3, 3)]
    o = np.zeros(72, np.float32)
    _check(_lib().pbrt_debug_layered(*[a.ctypes.data for a in arrs], o.ctypes.data))
    return o


def _check(rc):
    if rc != 0:
        raise PbrtError(_lib().pbrt_last_error().decode())


def _overrides(d):
    return ";".join(f"{k}={v}" for k, v in (d or {}).items()).encode()


class Scene:
    """A parsed .pbrt scene (BasicScene analogue)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load(cls, path, **overrides):
        h = ctypes.c_void_p()
        _check(_lib().pbrt_scene_load(str(path).encode(), _overrides(overrides), ctypes.byref(h)))
        return cls(h)

    @classmethod
    def from_string(cls, text, base_dir=".", **overrides):
        h = ctypes.c_void_p()
        _check(_lib().pbrt_scene_load_string(text.encode(), str(base_dir).encode(), _overrides(overrides),
                                             ctypes.byref(h)))
        return cls(h)

    @property
    def info(self) -> SceneInfo:
        i = SceneInfo()
        _check(_lib().pbrt_scene_get_info(self._h, ctypes.byref(i)))
        return i

    def flat(self) -> SceneFlat:
        f = SceneFlat()
        _check(_lib().pbrt_scene_get_flat(self._h, ctypes.byref(f)))
        f._owner = self  # keep the scene alive
        return f

    def zsobol(self, px, py, sample_index, dim):
        out = (ctypes.c_float * 7)()
        _check(_lib().pbrt_debug_zsobol(self._h, px, py, sample_index, dim, out))
        return np.array(out[:], dtype=np.float32)

    def sampler_values(self, px, py, sample_index, dim):
        """The scene's independent / stratified / sobol / paddedsobol sampler from
        StartPixelSample((px, py), sample_index, dim): 7 values in the wavefront's call order
        (pbrt_debug_sampler)."""
        out = (ctypes.c_float * 7)()
        _check(_lib().pbrt_debug_sampler(self._h, px, py, sample_index, dim, out))
        return np.array(out[:], dtype=np.float32)

    def filter_sample(self, u0, u1):
        """Filter::Sample((u0, u1)) of the scene's pixel filter -> (p.x, p.y, weight)"""
        out = (ctypes.c_float * 3)()
        _check(_lib().pbrt_debug_filter_sample(self._h, ctypes.c_float(u0), ctypes.c_float(u1), out))
        return np.array(out[:], dtype=np.float32)

    def halton(self, px, py, sample_index, dim):
        return _lib().pbrt_debug_halton(self._h, px, py, sample_index, dim)

    def bvh_stats(self):
        """Host BVH8 build statistics (pbrt_debug_bvh_stats)."""
        out = (ctypes.c_int64 * 8)()
        _check(_lib().pbrt_debug_bvh_stats(self._h, out))
        keys = ("nodes", "triangles", "depth", "max_stack", "wide_bytes", "quantised_bytes")
        return dict(zip(keys, list(out)[:6]))

    def bvh_trace(self, rays, spatial=-1):
        """Closest hits of rays (n x 6: origin, direction) by a host traversal of the device BVH8
        (pbrt_debug_bvh_trace): (t, triangle, stats); t = -1 and triangle = -1 for a miss."""
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = r.shape[0]
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.int32)
        st = (ctypes.c_int64 * 4)()
        _check(_lib().pbrt_debug_bvh_trace(self._h, int(spatial), r.ctypes.data, n, t.ctypes.data, prim.ctypes.data, st))
        return t, prim, dict(zip(("node_visits", "tri_tests", "references", "nodes"), list(st)))

    def texture_eval(self, material, slot, hit14, lambdas=()):
        """The product's texture evaluation of a material's textured parameter at a hit
        (pbrt_debug_texture_eval): returns ((dudx, dudy, dvdx, dvdy), values) where values are
        the reflectance at each wavelength (slot 0) or the roughness (slot 1 u, 2 v)."""
        lam = np.ascontiguousarray(lambdas, dtype=np.float32)
        hit = np.ascontiguousarray(hit14, dtype=np.float32)
        out = np.zeros(5 + len(lam), dtype=np.float32)
        _check(_lib().pbrt_debug_texture_eval(self._h, material, slot, hit.ctypes.data, lam.ctypes.data, len(lam),
                                              out.ctypes.data))
        return out[:4].copy(), (out[4:4 + len(lam)].copy() if slot == 0 else float(out[4]))

    def env_eval(self, env, dirs, u):
        """The product's ImageInfiniteLight lookups for directions dirs[n][3] and sample pairs
        u[n][2] (pbrt_debug_env_eval): [n][16] rows as include/pbrt_amd.h documents."""
        d = np.ascontiguousarray(dirs, dtype=np.float32).reshape(-1, 3)
        uu = np.ascontiguousarray(u, dtype=np.float32).reshape(-1, 2)
        assert len(d) == len(uu)
        out = np.zeros((len(d), 16), dtype=np.float32)
        _check(_lib().pbrt_debug_env_eval(self._h, env, d.ctypes.data, uu.ctypes.data, len(d), out.ctypes.data))
        return out

    def measured_eval(self, brdf, queries, lambdas):
        """The product's MeasuredBxDF on the host (pbrt_debug_measured) for [n][8] queries {wo, wi,
        u0, u1} at 31 wavelengths -> [n][68]: f[31], PDF, Sample_f ok, wi, pdf, f[31]."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, 8)
        lam = np.ascontiguousarray(lambdas, dtype=np.float32).reshape(31)
        out = np.zeros((len(q), 68), dtype=np.float32)
        _check(_lib().pbrt_debug_measured(self._h, brdf, q.ctypes.data, len(q), lam.ctypes.data, out.ctypes.data))
        return out

    def portal_eval(self, env, queries, res=0):
        """The product's PortalImageInfiniteLight on the host for [n][8] queries {p, d, u0, u1}
        (pbrt_debug_portal_eval) -> [n][16]; with res > 0 also the rectified image [res][res][3]
        and the windowed distribution's function [res][res]."""
        q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, 8)
        out = np.zeros((len(q), 16), dtype=np.float32)
        img = np.zeros(res * res * 4, np.float32) if res else None
        _check(_lib().pbrt_debug_portal_eval(self._h, env, q.ctypes.data, len(q), out.ctypes.data,
                                             img.ctypes.data if img is not None else None))
        if img is None:
            return out
        n = res * res
        return out, img[:3 * n].reshape(res, res, 3), img[3 * n:].reshape(res, res)

    def shape_eval(self, shape, rays, u):
        """The product's sphere / disk intersection, surface, sampling and pdf for rays[n][6]
        and sample pairs u[n][2] (pbrt_debug_shape_eval): [n][40] rows as the header documents."""
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        uu = np.ascontiguousarray(u, dtype=np.float32).reshape(-1, 2)
        out = np.zeros((len(r), 40), dtype=np.float32)
        _check(_lib().pbrt_debug_shape_eval(self._h, shape, r.ctypes.data, uu.ctypes.data, len(r), out.ctypes.data))
        return out

    def halton_fastpath_mismatches(self, dim, a0, a1, step=1):
        """Indices in [a0, a1) (stride step) whose 24-bit fast-path ScrambledRadicalInverse
        differs from the 64-bit restatement (core.h); -1 on bad arguments."""
        return _lib().pbrt_debug_halton_fastpath_mismatches(self._h, dim, a0, a1, step)

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.pbrt_scene_free(self._h)
            self._h = None


def load_scene(path, **overrides) -> Scene:
    return Scene.load(path, **overrides)


def check_rn_math(n=1 << 28, seed=1, device=0):
    """Bitwise mismatches of the kernels' RGBSigmoidPolynomial (device sqrt / division without
    range scaling) against the plain IEEE expression over ~n hashed inputs (runs on the GPU)."""
    out = ctypes.c_int64(0)
    ex = (ctypes.c_float * 96)()
    _check(_lib().pbrt_debug_check_rn_math(device, seed, n, ctypes.byref(out), ex))
    check_rn_math.examples = np.array(ex[:], np.float32).reshape(16, 6)[:min(out.value, 16)]
    return out.value


def debug_rng(seq, advance):
    """RNG::SetSequence(seq), Advance(advance), then two Uniform<uint32_t>() (pbrt_debug_rng)."""
    out = (ctypes.c_uint32 * 2)()
    _check(_lib().pbrt_debug_rng(int(seq), int(advance), out))
    return int(out[0]), int(out[1])


DET_MATH_FNS = ["sin", "cos", "asin", "acos", "atan2", "log", "sincos_sin", "sincos_cos", "exp", "sinh", "tan", "atan",
                "expm1"]


def det_math(fn, a, b=None, device=-1):
    """The kernels' portable transcendental `fn` (DET_MATH_FNS) on a (and b for atan2), run on GPU
    `device` or compiled for the host (device < 0): pbrt_debug_det_math."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b if b is not None else np.zeros_like(a), np.float32)
    out = np.zeros_like(a)
    _check(_lib().pbrt_debug_det_math(device, DET_MATH_FNS.index(fn), a.ctypes.data, b.ctypes.data, len(a),
                                      out.ctypes.data))
    return out


HAIR_IN, HAIR_OUT = 16, 68


def hair_eval(queries, device=-1):
    """HairBxDF f / PDF / Sample_f (core/hair.h) on [n][16] queries {h, eta, beta_m, beta_n,
    alpha, sigma_a0, wo, wi, uc, u0, u1, slope} -> [n][68] {f[31], pdf, ok, wi', pdf', f'[31]}, on
    GPU `device` or compiled for the host (device < 0): pbrt_debug_hair."""
    q = np.ascontiguousarray(queries, np.float32).reshape(-1, HAIR_IN)
    out = np.zeros((len(q), HAIR_OUT), np.float32)
    _check(_lib().pbrt_debug_hair(device, q.ctypes.data, len(q), out.ctypes.data))
    return out


def catmull_rom(op, nodes1, nodes2, values, cdf, x, device=-1):
    """The product's Catmull-Rom spline utilities (core/bssrdf.h) on the host, or compiled for
    gfx950 on GPU `device`: op 0 weights [n][6] (ok, offset, w0..w3), 1 InvertCatmullRom [n], 3
    SampleCatmullRom2D (x: alpha, u pairs)."""
    a = [np.ascontiguousarray(v, np.float32) for v in (nodes1, nodes2, values, cdf, x)]
    n = len(a[4]) // 2 if op == 3 else len(a[4])
    out = np.zeros(n * 6 if op == 0 else n, np.float32)
    args = (op, a[0].ctypes.data, len(a[0]), a[1].ctypes.data, len(a[1]), a[2].ctypes.data, a[3].ctypes.data,
            a[4].ctypes.data, n, out.ctypes.data)
    if device >= 0:
        _check(_lib().pbrt_debug_catmull_rom_gpu(device, *args))
    else:
        _check(_lib().pbrt_debug_catmull_rom(*args))
    return out.reshape(-1, 6) if op == 0 else out


def procedural(kind, params4, in9):
    """The procedural textures' code on the host (pbrt_debug_procedural): kind 0 fbm, 1
    turbulence, 2 windy, 3 polka dot, 4 marble; in9 rows = p, dpdx, dpdy; [n][6] out."""
    par = np.ascontiguousarray(params4, np.float32)
    x = np.ascontiguousarray(in9, np.float32).reshape(-1, 9)
    out = np.zeros((len(x), 6), np.float32)
    _check(_lib().pbrt_debug_procedural(kind, par.ctypes.data, x.ctypes.data, len(x), out.ctypes.data))
    return out


def device_count() -> int:
    n = ctypes.c_int(0)
    _lib().pbrt_device_count(ctypes.byref(n))
    return n.value


class WavefrontPathIntegrator:
    """Device-resident wavefront integrator (WavefrontPathIntegrator analogue).

    ``render(rows, first_sample, n_samples)`` runs the per-sample / per-depth stage loop of
    ``WavefrontPathIntegrator::Render`` (wavefront/integrator.cpp:290-493) over the given
    film rows, asynchronously on the context's HIP stream."""

    def __init__(self, scene: Scene, device: int = 0, max_paths: int = 0):
        self.scene = scene
        self.info = scene.info
        self._h = ctypes.c_void_p()
        _check(_lib().pbrt_context_create(scene._h, device, int(max_paths), ctypes.byref(self._h)))
        self._rows_cache = None

    def all_rows(self):
        i = self.info
        return np.arange(i.py0, i.py1, dtype=np.int32)

    def render(self, rows=None, first_sample=0, n_samples=None, time_closest=False):
        if rows is None:
            rows = self.all_rows()
        rows = np.ascontiguousarray(rows, dtype=np.int32)
        if n_samples is None:
            n_samples = self.info.spp - first_sample
        p = RenderParams(rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(rows), int(first_sample),
                         int(n_samples), 1 if time_closest else 0)
        self._rows_cache = rows
        _check(_lib().pbrt_render(self._h, ctypes.byref(p)))

    def synchronize(self):
        _check(_lib().pbrt_synchronize(self._h))

    def stats(self) -> RenderStats:
        s = RenderStats()
        _check(_lib().pbrt_get_stats(self._h, ctypes.byref(s)))
        return s

    def reset_stats(self):
        _check(_lib().pbrt_reset_stats(self._h))

    def set_kernel_profiling(self, enable=True):
        """Bracket every stage launch with HIP events (GetProfilerEvents, gpu/util.cpp:178-205)."""
        _check(_lib().pbrt_set_kernel_profiling(self._h, 1 if enable else 0))

    def kernel_stats(self):
        """Per-stage profile as of the last synchronize(): list of dicts in first-launch order."""
        n = ctypes.c_int(0)
        _check(_lib().pbrt_get_kernel_stats(self._h, None, 0, ctypes.byref(n)))
        arr = (KernelStat * max(n.value, 1))()
        _check(_lib().pbrt_get_kernel_stats(self._h, arr, n.value, ctypes.byref(n)))
        return [{"description": k.description.decode(), "launches": k.launches, "total_ms": k.total_ms,
                 "min_ms": k.min_ms, "max_ms": k.max_ms} for k in arr[:n.value]]

    def report_kernel_stats(self, file=None):
        """ReportKernelStats (gpu/util.cpp:211-246): one line per stage, stages under 0.1 % of the
        total folded into "Other"."""
        import sys
        out = file or sys.stdout
        ks = self.kernel_stats()
        total = sum(k["total_ms"] for k in ks) or 1.0
        print("Wavefront Kernel Profile:", file=out)
        other_n, other_ms = 0, 0.0
        for k in ks:
            if k["total_ms"] > 0.001 * total:
                print(f"  {k['description']:<49s} {k['launches']:5d} launches {k['total_ms']:9.2f} ms / "
                      f"{100 * k['total_ms'] / total:5.1f}% (avg {k['total_ms'] / k['launches']:6.3f}, min "
                      f"{k['min_ms']:6.3f}, max {k['max_ms']:7.3f})", file=out)
            else:
                other_n += k["launches"]
                other_ms += k["total_ms"]
        print(f"  {'Other':<49s} {other_n:5d} launches {other_ms:9.2f} ms / {100 * other_ms / total:5.1f}% "
              f"(avg {other_ms / max(other_n, 1):6.3f})", file=out)
        print(f"\nTotal rendering time: {total:9.2f} ms\n", file=out)

    def queue_counts(self):
        """Per-depth queue sizes of the last pass: rows of (rays, diffuse material, shadow, escaped,
        emissive, dielectric material, conductor material)."""
        n = 8 * (self.info.max_depth + 3)
        out = (ctypes.c_int32 * n)()
        _check(_lib().pbrt_debug_queue_counts(self._h, out, n))
        return np.array(out[:], dtype=np.int64).reshape(-1, 8)[:, :7]

    def kernel_sections(self, n=32):
        """Summed wave cycles per instrumented kernel section (profiling build only)."""
        out = (ctypes.c_uint64 * n)()
        _check(_lib().pbrt_debug_kernel_sections(self._h, out, n))
        return list(out)

    def film_clear(self):
        _check(_lib().pbrt_film_clear(self._h))

    def film_device_ptr(self):
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _check(_lib().pbrt_film_device_ptr(self._h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def film_raw(self) -> np.ndarray:
        i = self.info
        out = np.zeros((4, i.yres, i.xres), dtype=np.float64)
        _check(_lib().pbrt_film_read(self._h, out.ctypes.data))
        return out

    def film_rgb(self) -> np.ndarray:
        i = self.info
        out = np.zeros((i.yres, i.xres, 3), dtype=np.float32)
        _check(_lib().pbrt_film_get_rgb(self._h, out.ctypes.data))
        return out

    def write_image(self, path, write_fp16=True):
        """RGBFilm::WriteImage: .exr (half unless write_fp16=False), .pfm or .png by extension."""
        _check(_lib().pbrt_film_write_image(self._h, str(path).encode(), 1 if write_fp16 else 0))

    def __del__(self):
        if getattr(self, "_h", None) and _LIB is not None:
            _LIB.pbrt_context_free(self._h)
            self._h = None


class HIPAggregate:
    """WavefrontAggregate over device SoA ray batches (IntersectClosest / IntersectShadow)."""

    def __init__(self, integrator: WavefrontPathIntegrator):
        self.integrator = integrator

    def _run(self, rays, any_hit):
        import torch
        if not (rays.is_cuda and rays.dtype == torch.float32 and rays.dim() == 2 and rays.shape[0] == 7):
            raise PbrtError("rays must be a float32 device tensor of shape [7, n]")
        rays = rays.contiguous()
        n = rays.shape[1]
        prim = torch.empty(n, dtype=torch.int32, device=rays.device)
        hit = torch.empty((4, n), dtype=torch.float32, device=rays.device)
        torch.cuda.synchronize(rays.device)
        _check(_lib().pbrt_intersect(self.integrator._h, ctypes.c_void_p(rays.data_ptr()), n, int(any_hit),
                                     ctypes.c_void_p(prim.data_ptr()), ctypes.c_void_p(hit.data_ptr())))
        self.integrator.synchronize()  # results are written on the context's stream
        return prim, hit

    def IntersectClosest(self, rays):
        return self._run(rays, False)

    def IntersectShadow(self, rays):
        return self._run(rays, True)

    def IntersectShadowTr(self, rays, medium, lambda0):
        """TraceTransmittance (wavefront/intersect.h:164-274) per ray: rays [7, n] float32, medium
        [n] int32 (-1 vacuum), lambda0 [n] float32 device tensors -> (T_ray, r_u, r_l), each
        [31, n] float32."""
        import torch
        if not (rays.is_cuda and rays.dtype == torch.float32 and rays.dim() == 2 and rays.shape[0] == 7):
            raise PbrtError("rays must be a float32 device tensor of shape [7, n]")
        n = rays.shape[1]
        rays = rays.contiguous()
        medium = medium.to(device=rays.device, dtype=torch.int32).contiguous()
        lambda0 = lambda0.to(device=rays.device, dtype=torch.float32).contiguous()
        if medium.numel() != n or lambda0.numel() != n:
            raise PbrtError("medium and lambda0 need one entry per ray")
        out = torch.empty((3, 31, n), dtype=torch.float32, device=rays.device)
        torch.cuda.synchronize(rays.device)
        _check(_lib().pbrt_intersect_tr(self.integrator._h, ctypes.c_void_p(rays.data_ptr()),
                                        ctypes.c_void_p(medium.data_ptr()), ctypes.c_void_p(lambda0.data_ptr()), n,
                                        ctypes.c_void_p(out.data_ptr())))
        self.integrator.synchronize()
        return out[0], out[1], out[2]


    def IntersectOneRandom(self, segs, materials):
        """IntersectOneRandom (optix.cu:478-518) per probe segment: segs [6, n] float32 (p0, p1)
        and materials [n] int32 device tensors -> (prim [n] int32, hit [3, n], pdf [n])."""
        import torch
        if not (segs.is_cuda and segs.dtype == torch.float32 and segs.dim() == 2 and segs.shape[0] == 6):
            raise PbrtError("segs must be a float32 device tensor of shape [6, n]")
        n = segs.shape[1]
        segs = segs.contiguous()
        materials = materials.to(device=segs.device, dtype=torch.int32).contiguous()
        if materials.numel() != n:
            raise PbrtError("materials needs one entry per segment")
        prim = torch.empty(n, dtype=torch.int32, device=segs.device)
        hit = torch.empty((3, n), dtype=torch.float32, device=segs.device)
        pdf = torch.empty(n, dtype=torch.float32, device=segs.device)
        torch.cuda.synchronize(segs.device)
        _check(_lib().pbrt_intersect_one_random(self.integrator._h, ctypes.c_void_p(segs.data_ptr()),
                                                ctypes.c_void_p(materials.data_ptr()), n,
                                                ctypes.c_void_p(prim.data_ptr()), ctypes.c_void_p(hit.data_ptr()),
                                                ctypes.c_void_p(pdf.data_ptr())))
        self.integrator.synchronize()
        return prim, hit, pdf


def RenderWavefront(scene_path, device=0, **overrides):
    """Render a whole .pbrt file on one GPU and return the output-colour-space RGB image."""
    scene = Scene.load(scene_path, **overrides)
    integ = WavefrontPathIntegrator(scene, device=device)
    integ.render()
    integ.synchronize()
    return integ.film_rgb()


def write_pfm(path, rgb):
    """Write an RGB float image as PFM (pbrt's own PFM layout, util/image.cpp:1009)."""
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1\n".encode())
        f.write(np.ascontiguousarray(rgb[::-1], dtype="<f4").tobytes())


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = map(int, f.readline().split())
        scale = float(f.readline())
        data = np.frombuffer(f.read(), dtype="<f4" if scale < 0 else ">f4").reshape(h, w, 3)
    return data[::-1].copy()


# ---------------------------------------------------------------- image I/O and imgtool metrics
def write_image(path, rgb, write_fp16=True):
    """Image::Write for a [h, w, 3] float image: .exr / .pfm / .png by extension."""
    a = np.ascontiguousarray(rgb, dtype=np.float32)
    if a.ndim != 3 or a.shape[2] != 3:
        raise PbrtError("write_image expects an [h, w, 3] image")
    _check(_lib().pbrt_image_write(str(path).encode(), a.ctypes.data, a.shape[1], a.shape[0], 1 if write_fp16 else 0))


def read_image(path) -> np.ndarray:
    """Image::Read of a .pfm or uncompressed .exr file -> [h, w, 3] float32 (R, G, B)."""
    w, h = ctypes.c_int(), ctypes.c_int()
    _check(_lib().pbrt_image_read_size(str(path).encode(), ctypes.byref(w), ctypes.byref(h)))
    out = np.zeros((h.value, w.value, 3), np.float32)
    _check(_lib().pbrt_image_read(str(path).encode(), out.ctypes.data, w.value, h.value))
    return out


def image_error(image, reference, metric="MSE") -> np.ndarray:
    """Image::MAE / MSE / MRSE per channel, or the FLIP map's mean (imgtool diff/error,
    cmd/imgtool.cpp:960-1255).  Like imgtool diff, infinite pixel values are set to 0 first."""
    a = np.array(image, dtype=np.float32, copy=True)
    b = np.array(reference, dtype=np.float32, copy=True)
    if a.shape != b.shape or a.ndim != 3 or a.shape[2] != 3:
        raise PbrtError(f"image resolution {a.shape[:2]} doesn't match reference {b.shape[:2]}")
    a[np.isinf(a)] = 0
    b[np.isinf(b)] = 0
    out = np.zeros(3, np.float64)
    _check(_lib().pbrt_image_error(a.ctypes.data, b.ctypes.data, a.shape[1], a.shape[0], metric.encode(),
                                   out.ctypes.data))
    return out


def flip_error_map(image, reference) -> np.ndarray:
    """FLIP error per pixel [h, w] (imgtool --metric FLIP; inputs clamped to [0, 1])."""
    a = np.ascontiguousarray(image, dtype=np.float32)
    b = np.ascontiguousarray(reference, dtype=np.float32)
    if a.shape != b.shape or a.ndim != 3 or a.shape[2] != 3:
        raise PbrtError("FLIP needs two [h, w, 3] images of one resolution")
    out = np.zeros(a.shape[:2], np.float32)
    _check(_lib().pbrt_image_flip(a.ctypes.data, b.ctypes.data, a.shape[1], a.shape[0], out.ctypes.data))
    return out


def imgtool_diff(image_file, reference_file, metric="MSE"):
    """imgtool diff (cmd/imgtool.cpp:1105-1275): reads both images, returns
    {"image_average", "reference_average", "delta_percent", metric: average over channels}."""
    a, b = read_image(image_file), read_image(reference_file)
    a[np.isinf(a)] = 0
    b[np.isinf(b)] = 0
    err = image_error(a, b, metric)
    ia, ra = float(a.mean()), float(b.mean())
    return {"image_average": ia, "reference_average": ra,
            "delta_percent": 100.0 * (ia - ra) / ra if ra != 0 else float("inf"), metric: float(err.mean())}
