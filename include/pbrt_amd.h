/*
 * pbrt_amd.h — C ABI of the MI355X-native wavefront hot path (drop-in for pbrt-v4's
 * WavefrontPathIntegrator + WavefrontAggregate).
 *
 * Every entry point replaces a reference interface (file:line in scienstanford/pbrt-v4):
 *
 *   pbrt_scene_load / pbrt_scene_load_string
 *       pbrt::ParseFiles + BasicScene (cmd/pbrt.cpp:291-293, scene.h:260) for the .pbrt
 *       subset the hot path needs; overrides mirror --spp / --seed / --pixelbounds.
 *   pbrt_context_create
 *       WavefrontPathIntegrator ctor (wavefront/integrator.cpp:80-287): device scene
 *       upload, BVH build (replaces OptiXAggregate ctor, gpu/aggregate.cpp:1179-1663), queue
 *       allocation sized for maxPathsPerPass (integrator.cpp:227-236 uses 1M).
 *   pbrt_render
 *       WavefrontPathIntegrator::Render (wavefront/integrator.cpp:290-493) restricted to a
 *       set of film rows and a range of sample indices; asynchronous on the context stream.
 *   pbrt_intersect / pbrt_intersect_tr / pbrt_intersect_one_random
 *       WavefrontAggregate::IntersectClosest / IntersectShadow / IntersectShadowTr
 *       (wavefront/integrator.h:32-54) over caller-owned device SoA ray buffers.
 *   pbrt_film_*
 *       RGBFilm pixel storage (film.h:305-310), GetPixelRGB (film.h:261-277) and
 *       RGBFilm::WriteImage (film.cpp) to EXR / PFM / PNG.
 *   pbrt_image_*
 *       imgtool's diff / error metrics (cmd/imgtool.cpp:960-1105) and Image::Read.
 *
 * Conventions: 0 = success, nonzero = error with text from pbrt_last_error(); device
 * buffers are caller-owned where passed in; one hipStream per context; nothing blocks
 * except pbrt_synchronize / pbrt_film_read / pbrt_film_get_rgb.
 */
#ifndef PBRT_AMD_H
#define PBRT_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pbrt_scene pbrt_scene;
typedef struct pbrt_context pbrt_context;

typedef struct pbrt_scene_info {
    int xres, yres;
    int px0, px1, py0, py1; /* pixel bounds [px0,px1) x [py0,py1) */
    int spp, seed, max_depth;
    int n_triangles, n_vertices, n_materials, n_area_lights, n_infinite_lights;
    int n_light_nodes, uniform_light_sampler;
    float filter_radius_x, filter_radius_y;
} pbrt_scene_info;

/* Flattened, read-only view of a loaded scene (pointers into scene-owned memory). Used
 * by the CPU oracle and by tests; layout documented in DESIGN.md. */
typedef struct pbrt_scene_flat {
    int n_vertices, n_triangles, n_materials, n_area_lights, n_infinite_lights, n_spectra;
    const float *vertices;        /* [n_vertices][3] render space */
    const int32_t *triangles;     /* [n_triangles][3] */
    const int32_t *tri_material;  /* [n_triangles] */
    const int32_t *tri_light;     /* [n_triangles], -1 if not emissive */
    const uint8_t *tri_flip;      /* [n_triangles] reverseOrientation ^ swapsHandedness */
    const float *material_coeffs; /* [n_materials][4]: c0 c1 c2 constant */
    const int32_t *material_constant;
    const int32_t *light_prim;    /* [n_area_lights]: triangle, or n_triangles + k for shape k */
    const float *light_scale;
    const int32_t *light_spectrum;
    const int32_t *light_two_sided;
    /* [n_area_lights][3]: the fork's "spread" (lights.cpp:715-717): cosFalloffEnd (> 0 only for a
     * spread below 90 degrees), tanFalloffEnd, normalize_falloffEnd */
    const float *light_spread;
    /* [n_area_lights]: offset of the light's emission image in area_images, or -1; an image
     * is {w, h} then linear R, G, B [h][w][3] (row 0 = top); the light's spectrum is then the
     * colour space's illuminant (DiffuseAreaLight with "filename", lights.cpp:909-936) */
    const int32_t *light_image;
    const float *area_images;
    const int32_t *inf_spectrum;  /* [n_infinite_lights] */
    const float *inf_scale;
    const float *dense_spectra;   /* [n_spectra][311] at 395..705 nm */
    const float *sensor_xyz;      /* [3][311] */
    float imaging_ratio;
    float camera_from_raster[16];
    float render_from_camera[16];
    float lens_radius, focal_distance;
    double output_rgb_from_sensor_rgb[9];
    /* light BVH: [n_light_nodes][12] floats pMin3 pMax3 w3 phi cosO cosE, plus ints */
    int n_light_nodes;
    const float *light_node_bounds;
    const int32_t *light_node_info; /* [n][3]: childOrLight, isLeaf, twoSided */
    const uint32_t *light_bit_trail;
    /* Halton */
    int halton_base_scales[2], halton_base_exponents[2], halton_mult_inverse[2];
    int n_dims;
    const uint16_t *perm_table;
    const uint32_t *perm_offset, *perm_ndigits, *perm_base;
    /* sampler: 0 halton, 1 zsobol, 2 independent, 3 stratified, 4 sobol, 5 paddedsobol
     * (randomization of zsobol / sobol / paddedsobol: 0 none, 1 permutedigits, 2 fastowen, 3 owen;
     * stratified and Sobol' fields at the end of this struct) */
    int sampler_type, zs_randomize, zs_log2_spp, zs_nbase4_digits;
    /* materials: type 0 diffuse, 1 dielectric, 2 conductor (materials.h DiffuseMaterial,
     * DielectricMaterial, ConductorMaterial), 3 interface, 4 coateddiffuse, 5 coatedconductor,
     * 6 thindielectric, 7 diffusetransmission (reflectance in material_coeffs, transmittance in
     * material_layer's albedo fields, scale = material_params[3]) */
    const int32_t *material_type;     /* [n_materials] */
    const float *material_params;     /* [n_materials][4]: alpha_x alpha_y eta 0 (TrowbridgeReitz
                                         alphas after remap + clamp; dielectric eta) */
    const int32_t *material_spectra;  /* [n_materials][2]: conductor eta, k indices into the
                                         piecewise-linear spectra; -1 -1 = "reflectance" (coeffs) */
    int n_pl_spectra;
    const int32_t *pl_offsets;        /* [n_pl_spectra + 1] into pl_lambda / pl_value */
    const float *pl_lambda, *pl_value;
    int regularize;                   /* integrator "regularize" */
    /* shading attributes (TriangleMesh n / uv): per vertex, or NULL when no mesh has any;
     * tri_shading[t] bit0 = triangle t uses vertex normals, bit1 = uv, bit2 = tangents S
     * (vertex_s below) */
    const float *vertex_normals;      /* [n_vertices][3] render space */
    const float *vertex_uv;           /* [n_vertices][2] */
    const uint8_t *tri_shading;       /* [n_triangles] */
    /* participating media (HomogeneousMedium / GridMedium); index -1 = vacuum */
    int n_media, camera_medium;
    const int32_t *medium_info;       /* [n_media][16]: type (0 homogeneous, 1 grid, 2 cloud,
                                         3 rgbgrid), sigma_a, sigma_s, Le (dense_spectra
                                         indices, pbrt's scales applied), emissive, nx, ny, nz,
                                         lnx, lny, lnz, density offset, LeScale offset,
                                         majorant offset (into medium_values), grey (sigma_a and
                                         sigma_s constant over wavelength); last: grid: offset
                                         of {temperatureoffset, temperaturescale, T[nz][ny][nx]}
                                         or -1, rgbgrid: bit k = block k given, else 0 */
    const float *medium_params;       /* [n_media][24]: g, bounds p0 xyz, p1 xyz, 0,
                                         mediumFromRender 4x4 row-major */
    const float *medium_values;       /* density / LeScale / 16^3 majorant grids */
    const int16_t *tri_medium;        /* [n_triangles][2] inside, outside (NULL without media) */
    /* pixel filter (filters.h): type 0 box, 1 gaussian (a = sigma), 2 mitchell (a = B, b = C),
     * 3 sinc (a = tau), 4 triangle; radius in pbrt_scene_info */
    int filter_type;
    float filter_a, filter_b;
    /* layered materials, type 4 coateddiffuse / 5 coatedconductor (LayeredBxDF, bxdfs.h:565):
     * material_params = interface alphas + eta, material_coeffs = diffuse or conductor
     * "reflectance", material_spectra = conductor.eta / .k; per material [12] floats:
     * thickness g maxdepth nsamples, albedo c0 c1 c2 value constant(1/0), conductor
     * alpha_x alpha_y, spectral interface eta (index into the piecewise-linear spectra, -1
     * for the constant eta of material_params) */
    const float *material_layer;
    /* point / spot / distant lights (PointLight, SpotLight, DistantLight: lights.h, lights.cpp:
     * 192-276, 1376-1495) in render space, [n_delta_lights][24] floats: type (0 point, 1 spot,
     * 2 distant), dense spectrum index, final scale, cosFalloffStart, cosFalloffEnd, p xyz, w xyz
     * (spot axis / direction toward a distant light), renderFromLight^-1 upper 3x3 row-major
     * (spot, goniometric, projection), then LightBounds' phi, the light's offset into
     * delta_images (-1: none), image width, height.  Types 3 (goniometric) and 4 (projection)
     * keep LightBounds' cosTheta_o / cosTheta_e in the cosFalloff slots and their bounds axis in
     * w.  The first n_point_spot are the point, spot, goniometric and projection lights: light-BVH members
     * with global light index n_area_lights + i.  Infinite-list entry j (global index
     * n_area_lights + n_point_spot + j) is a distant light when inf_distant[j] >= 0.
     * uniform_order[k]: global index of pbrt's k-th light (area lights, then LightSource order);
     * scene_radius: DistantLight::Preprocess's bounding-sphere radius. */
    int n_delta_lights, n_point_spot;
    const float *delta_lights;
    /* per goniometric / projection light at its offset: a 4-float header {1 / tan(fov / 2)
     * (projection), 0, 0, 0}, then the goniometric light's Y values [h][w] or the projection
     * light's linear R, G, B [h][w][3] (row 0 = top) */
    const float *delta_images;
    const int32_t *inf_distant;       /* [n_infinite_lights] */
    const int32_t *uniform_order;     /* [n_area_lights + n_point_spot + n_infinite_lights] */
    float scene_radius;
    /* textures (textures.h, textures.cpp, util/mipmap.*): expression nodes in the device layout
     * (core/texture_eval.h DeviceTexNode) -- [n][8] ints kind (0 constant, 1 scale, 2 mix,
     * 3 directionmix, 4 checkerboard, 5 bilerp, 6 imagemap), flags (bit0 spectrum, bits 1-2
     * SpectrumType 0 albedo / 1 unbounded, bit3 invert, bit4 3D checkerboard), child0..2, image,
     * mapping (0 uv, 1 spherical, 2 cylindrical, 3 planar), MIP filter (0 point, 1 bilinear,
     * 2 trilinear, 3 EWA); [n][28] floats textureFromRender 3x4, planar vs vt, uv su sv du dv
     * (planar ds dt), float constant / bilerp v00 v01 v10 v11 / directionmix dir, image scale,
     * maxanisotropy; [n][4][8] constant spectra {rgb, value, c0, c1, c2, scale} (bilerp corners
     * in v00 v10 v01 v11 order).  Images: [n][8] format (0 u8, 1 half, 2 float), channels,
     * levels, wrap (0 repeat, 1 black, 2 clamp, 3 octahedral), first level, lut offset; per
     * level [4] w, h, byte offset lo, hi into image_data; 8-bit decode tables [n][256]; the
     * decoded files before the pyramid ([n][8] w, h, format, channels, encoding 0 linear /
     * 1 sRGB / 2 gamma; image_raw_gamma, bytes at image_raw_offset).  material_tex [n][4]: root
     * node of the reflectance, u and v roughness textures (-1 none), remaproughness.
     * camera_from_render (3x4) and camera_min_diff (minPosDifferentialX/Y,
     * minDirDifferentialX/Y, cameras.cpp:170-216) for Approximate_dp_dxy (cameras.h:167-195). */
    int n_tex_nodes, n_images;
    const int32_t *tex_node_info;
    const float *tex_node_params;
    const float *tex_node_spec;
    const int32_t *image_info;
    const int32_t *image_levels;
    const uint8_t *image_data;
    const float *image_luts;
    const int32_t *image_raw_info;
    const float *image_raw_gamma;
    const uint64_t *image_raw_offset;
    const uint8_t *image_raw_data;
    const int32_t *material_tex;
    float camera_from_render[12];
    float camera_min_diff[12];
    /* MixMaterial (materials.h:271-350, type 8): [n_materials][4] material 0, material 1, root
     * node of the float "amount" texture (constant or image), 0; -1 for other materials */
    const int32_t *material_mix;
    /* ImageInfiniteLight (lights.h:557-641): infinite-list entry j is an image light when
     * inf_image[j] >= 0 (its index here); per image light env_info [n_env][4] res (square),
     * portal flag, 0, 0, env_xform [n_env][18] renderFromLight then its inverse (upper 3x3, row major),
     * and its linear R, G, B pixels (Image::GetChannel) at env_rgb + 3 * env_offset[k]
     * ([res][res][3], row y = v * res).  inf_spectrum / inf_scale hold the colour space's
     * illuminant and the light's scale. */
    int n_env;
    const int32_t *inf_image;
    const int32_t *env_info;
    const float *env_xform;
    const uint64_t *env_offset;
    const float *env_rgb;
    /* Sphere / Disk (shapes.h:106-571), render space: primitive id n_triangles + k (light_prim
     * of a shape emitter).  shape_info [n][8] kind (1 sphere, 2 disk), flags (bit0
     * ReverseOrientation, bit1 transformSwapsHandedness), material, area light (-1), medium
     * inside, outside, 0, 0; shape_params [n][32] objectFromRender 3x4, renderFromObject 3x4
     * (row major), then sphere radius, zMin, zMax, phiMax, thetaZMin, thetaZMax or disk height,
     * radius, innerRadius, phiMax (radians), 2 unused. */
    int n_shapes;
    const int32_t *shape_info;
    const float *shape_params;
    /* kind 3 (bilinear patch, shapes.h:1272-1540): shape_params holds the render-space corners
     * p00 p10 p01 p11 in its first 12 floats, their uv in the next 8, then area and
     * isRectangle; flags bit2 uv present, bit3 vertex normals present (shape_normals [n][12],
     * render space) */
    const float *shape_normals;
    /* alpha-tested primitives (GeometricPrimitive alpha, cpu/primitive.cpp:56-80; gpu/optix.cu
     * alphaKilled): [n_triangles + n_shapes] in scene order, the float texture node (index into
     * the tex_node tables) of the primitive's alpha, or -1; NULL when no shape has one */
    const int32_t *prim_alpha;
    /* RGBFilm / PixelSensor (film.cpp:222-262, 582-600): "maxcomponentvalue" (inf when not
     * given) and the sensor's XYZFromSensorRGB (row major); sensor_xyz holds its r/g/b curves */
    float max_component_value;
    float xyz_from_sensor_rgb[9];
    /* bump / normal mapping (materials.h:86-160) per material [n][2]: the displacement
     * texture's root node and the normal map image (indices into the tex_node / image tables,
     * -1 none) */
    const int32_t *material_bump;
    /* StratifiedSampler xsamples, ysamples, jitter; SobolSampler log2(RoundUpPow2(max(xres,
     * yres))) and util/sobolmatrices.cpp's tables (SobolMatrices32 [1024 * 52], VdCSobolMatrices
     * and VdCSobolMatricesInv [25 * 52]; NULL unless the sampler is sobol) */
    int strat_xsamples, strat_ysamples, strat_jitter, sobol_log2_scale;
    const uint32_t *sobol_matrices32;
    const uint64_t *vdc_sobol, *vdc_sobol_inv;
    /* util/noise.cpp NoisePerm[512] (as floats), for the procedural textures (dots, fbm,
     * wrinkled, windy, marble: tex_node_info kinds 7-11; their params [22..24] = octaves,
     * roughness, variation and [26] = marble scale) */
    const float *noise_perm;
    /* SubsurfaceMaterial (materials.h:772-866): material_sss [n_materials] = its subsurface
     * description or -1 (NULL when n_sss == 0; such a material is otherwise a dielectric);
     * sss_params [n_sss][20] = mode (0 sigma_a / sigma_s, 1 reflectance / mfp), scale, eta,
     * 1 - 2 FresnelMoment1(1 / eta), two spectra {kind (0 constant, 1 scale * sigmoid, 2
     * piecewise-linear), value, c0, c1, c2, scale, pl_spectra index}, g, 0; sss_tables
     * [n_sss][13064] = the BSSRDFTable (rho[100], radius[64], profile[100][64], rhoEff[100],
     * profileCDF[100][64]); dims_per_depth: sampler dimensions per path depth (7, or 10 with
     * subsurface scattering: samples.cpp:39-41) */
    int n_sss, dims_per_depth;
    const int32_t *material_sss;
    const float *sss_params;
    const float *sss_tables;
    /* per-vertex shading tangents (TriangleMesh s, "vector3 S"), render space, or NULL; used by
     * the triangles whose tri_shading bit2 is set (entries past the array are zero) */
    const float *vertex_s;            /* [n_vertex_s][3] */
    int n_vertex_s;
    /* PortalImageInfiniteLight: env_info[4k + 1] = 1 for a portal light, whose render-space
     * portal corners are env_portal [n_env][4][3] (zeros for the others) */
    const float *env_portal;
    /* MeasuredMaterial (materials.h:925-967, type 10): material_layer[12 * m] = its BRDF index;
     * measured_files [n_measured] the resolved RGL tensor files (".bsdf") */
    int n_measured;
    const char *const *measured_files;
    /* scene Options (BasicSceneBuilder::Option, scene.cpp:492-560) that change the hot path:
     * bit 0 disablepixeljitter (samplers.h:807-812), bit 1 disablewavelengthjitter
     * (wavefront/camera.cpp:55), bit 2 disabletexturefiltering (wavefront/surfscatter.cpp:77) */
    int options;
    /* multispectral basis image textures (tex_node_info flags bit 5, the fork's "basisfilename"):
     * the node's table starts at tex_basis[params[22]], params[24] floats long, laid out as the
     * reference's GPU basis array (textures.cpp:1148-1176): channels, basis length, int(offset),
     * then each channel's basis values */
    const float *tex_basis;
    /* textured hair floats (GetFloatTexture, materials.cpp:135-184): per material the tex_node
     * roots of eta, beta_m, beta_n, alpha, eumelanin, pheomelanin, or -1 for the material_layer
     * constant; the concentrations are textured as a pair (sigma_a = SigmaAFromConcentration
     * per hit); NULL when no hair material is textured */
    const int32_t *material_hair_tex;
    /* textured subsurface spectra (SubsurfaceMaterial::GetBSSRDF, materials.h:823-841): per
     * material the tex_node roots of sigma_a and of sigma_s (sss mode 0) or mfp (mode 1),
     * Unbounded, or -1 for the sss_params constant; NULL when none is textured */
    const int32_t *material_sss_tex;
} pbrt_scene_flat;

typedef struct pbrt_render_params {
    const int32_t *rows; /* host array of absolute film rows to render (within bounds) */
    int n_rows;
    int first_sample;    /* first sample index */
    int n_samples;       /* number of consecutive sample indices */
    int time_closest;    /* 1: record HIP events around every closest-hit launch */
} pbrt_render_params;

typedef struct pbrt_render_stats {
    uint64_t camera_rays, closest_rays, shadow_rays; /* valid after pbrt_synchronize */
    int closest_launches;   /* event-timed closest-hit launches (first pass of each render) */
    double closest_ms;      /* sum of their durations */
    uint64_t timed_closest_rays; /* rays those launches processed */
    int passes;
    uint64_t paths_per_pass;
    /* the BVH the closest-hit traversal reads from HBM (SURVEY 8(d)'s "touched once per
     * launch" term): node bytes in the format traversed, less the top nodes cached in LDS,
     * and triangle bytes (0 when every triangle is cached in LDS) */
    uint64_t bvh_hbm_node_bytes, bvh_hbm_tri_bytes;
} pbrt_render_stats;

/* Per-stage kernel profile (GetProfilerEvents / ReportKernelStats, gpu/util.cpp:128-246): with
 * profiling on, every stage launch of pbrt_render is bracketed by HIP events on the stream it
 * runs on; pbrt_synchronize folds them into one record per stage. */
typedef struct pbrt_kernel_stat {
    char description[96];
    int launches;
    double total_ms, min_ms, max_ms;
} pbrt_kernel_stat;

const char *pbrt_last_error(void);
int pbrt_set_data_dir(const char *dir);

int pbrt_scene_load(const char *path, const char *overrides, pbrt_scene **out);
int pbrt_scene_load_string(const char *text, const char *base_dir, const char *overrides, pbrt_scene **out);
void pbrt_scene_free(pbrt_scene *scene);
int pbrt_scene_get_info(const pbrt_scene *scene, pbrt_scene_info *info);
int pbrt_scene_get_flat(const pbrt_scene *scene, pbrt_scene_flat *flat);

int pbrt_device_count(int *count);
/* max_paths_per_pass <= 0: every sample of the film in one pass, up to 64 Mi paths (16 Mi for
 * scenes with media) */
int pbrt_context_create(const pbrt_scene *scene, int device, int64_t max_paths_per_pass, pbrt_context **out);
void pbrt_context_free(pbrt_context *ctx);

int pbrt_render(pbrt_context *ctx, const pbrt_render_params *params);
int pbrt_synchronize(pbrt_context *ctx);
int pbrt_get_stats(pbrt_context *ctx, pbrt_render_stats *stats);
int pbrt_reset_stats(pbrt_context *ctx); /* also clears the kernel profile */
int pbrt_set_kernel_profiling(pbrt_context *ctx, int enable);
/* the profile as of the last pbrt_synchronize: min(*n_stats, max_stats) records in first-launch
 * order; *n_stats = number of stages profiled */
int pbrt_get_kernel_stats(pbrt_context *ctx, pbrt_kernel_stat *out, int max_stats, int *n_stats);

int pbrt_film_clear(pbrt_context *ctx);
int pbrt_film_device_ptr(pbrt_context *ctx, double **film, size_t *n_doubles);
int pbrt_film_read(pbrt_context *ctx, double *out);     /* [4][xres*yres] sensor RGB sums + weight */
int pbrt_film_get_rgb(pbrt_context *ctx, float *rgb);   /* [yres*xres][3] output colour space */

/* Film output (RGBFilm::WriteImage, film.cpp; Image::Write, util/image.cpp:990-1012): the
 * film's output-colour-space RGB written by extension: .exr (OpenEXR scanline, uncompressed;
 * half floats unless write_fp16 = 0, pbrt's "writefp16"), .pfm (Image::WritePFM), .png (8-bit
 * sRGB). */
int pbrt_film_write_image(pbrt_context *ctx, const char *path, int write_fp16);
/* imgtool (cmd/imgtool.cpp:960-1105) image access and error metrics, host only.
 * pbrt_image_read_size then pbrt_image_read into a caller-owned [h][w][3] float buffer
 * (.pfm, uncompressed .exr).  pbrt_image_error: metric "MAE" (pbrt's signed mean
 * difference), "MSE", "MRSE" or "FLIP" per channel over [h][w][3] images (Image::MAE / MSE /
 * MRSE, util/image.cpp:543-639; FLIP below). */
int pbrt_image_read_size(const char *path, int *width, int *height);
int pbrt_image_read(const char *path, float *rgb, int width, int height);
int pbrt_image_write(const char *path, const float *rgb, int width, int height, int write_fp16);
int pbrt_image_error(const float *image, const float *reference, int width, int height, const char *metric,
                     double *error3);
/* FLIP error map [h][w] (imgtool --metric FLIP, cmd/imgtool.cpp:1224-1255 over src/ext/flip):
 * inputs clamped to [0, 1]; "FLIP" in pbrt_image_error reports the map's mean per channel */
int pbrt_image_flip(const float *image, const float *reference, int width, int height, float *error_map);

/* WavefrontAggregate boundary: rays_dev = [7][n] SoA (o.xyz, d.xyz, tMax) on the device;
 * prim_dev [n] receives the original triangle index or -1; hit_dev [4][n] b0 b1 b2 t.
 * Asynchronous on the context stream (no host round trip): the results are valid after
 * pbrt_synchronize, or for work the caller orders after the context stream. */
int pbrt_intersect(pbrt_context *ctx, const float *rays_dev, int n, int any_hit, int32_t *prim_dev, float *hit_dev);
/* WavefrontAggregate::IntersectOneRandom (wavefront/integrator.h:53; gpu/aggregate.cpp:1811-1847,
 * optix.cu:478-518): per caller segment segs_dev[6][n] (p0.xyz, p1.xyz) the closest hits from p0
 * towards p1, each continued by SpawnRayTo(p1), reservoir-sampled among the hits on
 * materials_dev[i] (the scene's material index) with pbrt's RNG seeding (Hash(p0, p1)) ->
 * prim_dev[n] (triangle in the caller's numbering, n_triangles + k for shape k, or -1),
 * hit_dev[3][n] (b0, b1, b2; a shape's coordinates), pdf_dev[n] (SampleProbability, 0: none).
 * Device pointers, asynchronous on the context stream. */
int pbrt_intersect_one_random(pbrt_context *ctx, const float *segs_dev, const int32_t *materials_dev, int n,
                              int32_t *prim_dev, float *hit_dev, float *pdf_dev);
/* WavefrontAggregate::IntersectShadowTr (wavefront/integrator.h:49-51; TraceTransmittance,
 * wavefront/intersect.h:164-274) over device SoA buffers: rays_dev [7][n] (o, d, tMax: the light
 * point is o + tMax d), medium_dev [n] the medium each ray starts in (NULL or -1: vacuum; indices
 * of the scene's media), lambda0_dev [n] the path's first wavelength (the other 30 follow
 * SampleUniform's 10 nm stratification, as every SampledWavelengths of this wavefront); out_dev
 * [3][31][n] receives T_ray, r_u, r_l after ratio tracking through every medium and interface
 * up to the light (T_ray = 0 when an opaque surface blocks the ray; RNG seeded as pbrt's,
 * Hash(ray.o), Hash(ray.d)).  The caller applies intersect.h:262-266: Ld *= T_ray /
 * avg(sr.r_u * r_u + sr.r_l * r_l).  Asynchronous on the context stream. */
int pbrt_intersect_tr(pbrt_context *ctx, const float *rays_dev, const int32_t *medium_dev, const float *lambda0_dev,
                      int n, float *out_dev);


/* ColorSpace directive name (srgb, dci-p3, rec2020, aces2065-1; any case, RGBColorSpace::GetNamed)
 * -> 0..3, or -1 with pbrt_last_error set */
int pbrt_color_space_index(const char *name);

#ifdef __cplusplus
}
#endif

#endif /* PBRT_AMD_H */
