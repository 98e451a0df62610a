/*
 * pbrt_amd_debug.h -- test and tooling entry points of libpbrt_amd.so (not the renderer API).
 *
 * Each function runs one product component -- the same host / device code the wavefront kernels
 * use -- on caller-supplied inputs, so tests/ can hold it to the oracle and to the reference's
 * golden vectors component by component (tests/test_golden_product_host.py and friends), and
 * tools/ can profile it.  Conventions as include/pbrt_amd.h: 0 on success, non-zero with
 * pbrt_last_error() set.  A maintainer binding the renderer needs only pbrt_amd.h.
 */
#ifndef PBRT_AMD_DEBUG_H
#define PBRT_AMD_DEBUG_H

#include "pbrt_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* host-side evaluation of product components (no GPU): used by golden-vector tests */
float pbrt_debug_halton(const pbrt_scene *scene, int px, int py, int sample_index, int dim);
/* GPU arithmetic self-check: the kernels' RGBSigmoidPolynomial evaluation (core.h, correctly
 * rounded sqrt / division without the range-scaling steps) against the plain IEEE expression, and
 * SinCosf against separate sin / cos, on about n hashed inputs from seed; *mismatches = bitwise
 * mismatch count of both;
 * examples96 (optional): up to 16 mismatches as {c0, c1, c2, lambda, kernel value, plain value} */
int pbrt_debug_check_rn_math(int device, uint64_t seed, int64_t n, int64_t *mismatches, float *examples96);
/* Halton fast path check: ScrambledRadicalInverse of the scene's dimension dim (its digit
 * permutations) by the kernels' 24-bit float-reciprocal digit loop against the 64-bit
 * restatement of util/lowdiscrepancy.h:115-134, for a = a0, a0 + step, ... < a1 (a1 <= 2^24);
 * returns the number of indices whose floats differ (bitwise), or -1 on error */
/* The Catmull-Rom spline utilities of the tabulated BSSRDF (core/bssrdf.h; util/math.cpp:157-265,
 * util/sampling.cpp:424-488), run on the host: op 0 CatmullRomWeights(nodes1, x[i]) -> out[n][6]
 * = ok, offset, w0..w3; 1 InvertCatmullRom(nodes1, values, x[i]) -> out[n]; 3
 * SampleCatmullRom2D(nodes1, nodes2, values[n1][n2], cdf[n1][n2], alpha = x[2i], u = x[2i+1]) */
int pbrt_debug_catmull_rom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                           const float *cdf, const float *x, int n, float *out);
/* The same utilities compiled for gfx950 and run on GPU `device` (one thread per query). */
int pbrt_debug_catmull_rom_gpu(int device, int op, const float *nodes1, int n1, const float *nodes2, int n2,
                               const float *values, const float *cdf, const float *x, int n, float *out);
int64_t pbrt_debug_halton_fastpath_mismatches(const pbrt_scene *scene, int dim, uint32_t a0, uint32_t a1,
                                              uint32_t step);
int pbrt_debug_rgb_coeffs(float r, float g, float b, float *coeffs3);
int pbrt_debug_rgb2spec_column(int maxc, int j, int i, float *out192);
/* The RGB colour spaces (util/colorspace.cpp:83-105), indexed as pbrt_color_space_index returns:
 * info[338] = r, g, b, white chromaticities (8), XYZFromRGB (9), RGBFromXYZ (9),
 * SpectrumToPhotometric(illuminant), the illuminant densely sampled at 395..705 */
int pbrt_debug_color_space(int cs, float *info338);
/* RGB -> spectrum in colour space cs for n RGB triples at nl wavelengths: per triple
 * out[3 + 3 nl] = the table's sigmoid coefficients of rgb, RGBAlbedoSpectrum(rgb)(lambda),
 * RGBUnboundedSpectrum(s rgb)(lambda), RGBIlluminantSpectrum(s rgb)(lambda) with s = unboundedScale */
int pbrt_debug_rgb_spectrum(int cs, const float *rgb3, int n, float unboundedScale, const float *lambda, int nl,
                            float *out);
/* Column (maxc, j, i) of colour space cs's RGBToSpectrumTable as rgb2spec_opt builds it (64 x 3) */
int pbrt_debug_rgb2spec_column_cs(int cs, int maxc, int j, int i, float *out192);
/* Texture evaluation of material `material`'s textured parameter (slot 0 reflectance, 1 u / 2 v
 * roughness) at a hit given as p, n, dpdu, dpdv (render space) and uv (14 floats), with the
 * product's shared host/device code (surfscatter.cpp:74-137, textures.h): out[0..3] = dudx,
 * dudy, dvdx, dvdy, then the spectrum texture at each of the n wavelengths, or out[4] = the
 * float texture */
int pbrt_debug_texture_eval(const pbrt_scene *scene, int material, int slot, const float *hit14, const float *lambda,
                            int n, float *out);
/* ImageInfiniteLight `env` of the scene with the product's shared host/device code
 * (lights.h:587-631, lights.cpp:1073-1083): for n directions dirs[n][3] and sample pairs
 * u[n][2], out[n][16] = Le's (u, v) of the direction, PDF_Li(allowIncompletePDF), the pixel's
 * RGBIlluminantSpectrum at 400 / 500 / 600 / 700 nm (light scale and illuminant 1), the
 * compensated distribution's sample (u, v), its mapPDF, wi = renderFromLight(
 * EqualAreaSquareToSphere(u, v)), PiecewiseConstant2D::PDF at that sample, PDF at u taken as a
 * point of [0,1]^2, 1 unused */
int pbrt_debug_env_eval(const pbrt_scene *scene, int env, const float *dirs, const float *u, int n, float *out);
/* PortalImageInfiniteLight `env` (lights.cpp:1140-1297) on the host: per query q8 = {p[3], d[3],
 * u0, u1}: out16 = {Le(ray p, d) at 400 / 500 / 600 / 700 nm (light scale 1, illuminant 1),
 * PDF_Li(p, d), SampleLi(p, u) ok, wi[3], pdf, the sample's Le at the four wavelengths,
 * ImageBounds(p) ok, 0}; img (optional, res * res * 4 floats): the rectified image [res][res][3]
 * then the windowed distribution's function [res][res] */
int pbrt_debug_portal_eval(const pbrt_scene *scene, int env, const float *q8, int n, float *out16, float *img);
/* EqualAreaSquareToSphere (to_sphere != 0: in[n][2] -> out[n][3]) or EqualAreaSphereToSquare
 * (in[n][3] -> out[n][2]) with the product's shared host/device code (util/math.cpp:292-361) */
/* util/noise.cpp Noise / DNoise and CloudMedium::Density (media.h:493-517) as the media
 * kernels evaluate them: out5 per point = Noise(p), DNoise(p) xyz, Density(p) for params3 =
 * {density, wispiness, frequency} (host) */
int pbrt_debug_cloud_density(const float *params3, const float *pts, int n, float *out5);
int pbrt_debug_equal_area(int to_sphere, const float *in, int n, float *out);
/* Sphere / disk `shape` of the scene with the product's shared host/device code (shapes.h:
 * 106-571): for n rays rays[n][6] (o, d) and sample pairs u[n][2], out[n][40] = hit flag, tHit,
 * pObj xyz, then the render-space SurfaceInteraction p xyz, pError xyz, n xyz, shading n xyz,
 * dpdu xyz, dpdv xyz, uv; then Shape::Sample(ctx = (o, no error, no normal), u): ok flag, p
 * xyz, pError xyz, n xyz, pdf; then Shape::PDF(ctx, d); 2 unused.  Odd rows give the context the
 * shading normal -d (the bilinear patch's cosine-weighted warp), even rows none. */
int pbrt_debug_shape_eval(const pbrt_scene *scene, int shape, const float *rays, const float *u, int n, float *out);
/* Filter::Sample(u) of the scene's pixel filter (FilterSampler over PiecewiseConstant2D for
 * gaussian / mitchell / sinc, SampleTent for triangle, filters.h): out3 = p.x p.y weight */
int pbrt_debug_filter_sample(const pbrt_scene *scene, float u0, float u1, float *out3);
/* ZSobolSampler (samplers.h:225-370) from StartPixelSample((px,py), sample_index, dim) with the
 * wavefront's call pattern Get1D, Get2D, Get1D, Get2D, Get1D -> 7 values (scene's sampler
 * parameters: spp, resolution, seed, randomization) */
int pbrt_debug_zsobol(const pbrt_scene *scene, int px, int py, int sample_index, int dim, float *out7);
/* IndependentSampler / StratifiedSampler / SobolSampler / PaddedSobolSampler (samplers.h:144-224,
 * 442-633) of the scene from StartPixelSample((px,py), sample_index, dim): for dim 0 the
 * camera's Get1D, GetPixel2D, Get1D, Get2D, Get1D, otherwise Get1D, Get2D, Get1D, Get2D, Get1D
 * -> 7 values.  Fails for halton / zsobol scenes (pbrt_debug_halton / pbrt_debug_zsobol). */
int pbrt_debug_sampler(const pbrt_scene *scene, int px, int py, int sample_index, int dim, float *out7);
/* The kernels' portable transcendentals (core/detmath.h) on n inputs: fn 0 sin, 1 cos, 2 asin, 3
 * acos (inputs clamped to [-1, 1] as SafeASin / SafeACos), 4 atan2(a, b), 5 log, 6 / 7 the sin /
 * cos of SinCosf, 8 exp, 9 sinh; on GPU `device`, or compiled for the host when device < 0 (the two must agree
 * bit for bit, and the oracle's device-math mode with both) */
int pbrt_debug_det_math(int device, int fn, const float *a, const float *b, int n, float *out);
/* HairBxDF (bxdfs.h:1054-1152, bxdfs.cpp:279-573; the BxDF HairMaterial::GetBxDF builds,
 * materials.h:380-404) on n queries of 16 floats {h, eta, beta_m, beta_n, alpha, sigma_a0, wo[3],
 * wi[3], uc, u0, u1, slope} with sigma_a[i] = sigma_a0 + slope * i at the 31 wavelengths:
 * out[68] per query = {f(wo, wi)[31], PDF(wo, wi), Sample_f ok, wi[3], pdf, f[31]} (zeros when
 * BSDF::Sample_f returns {}).  On GPU `device`, or compiled for the host when device < 0. */
int pbrt_debug_hair(int device, const float *in16, int n, float *out);
/* MeasuredBxDF (bxdfs.cpp:1003-1124) on the host over a loaded scene's measured BRDF `brdf`:
 * per query in8 {wo xyz, wi xyz, u0, u1} (local frame) at the 31 wavelengths `lambda`; out
 * [n][68] = f(wo, wi)[31], PDF(wo, wi), Sample_f ok, wi xyz, pdf, f[31] */
int pbrt_debug_measured(const pbrt_scene *scene, int brdf, const float *in8, int n, const float *lambda, float *out);
/* PiecewiseLinear2D<dim> alone (util/sampling.h:1299-1749; dim 0 or 2, normalised, CDF iff cdf)
 * over data [pr2[0]][pr2[1]][ys][xs] with parameter grids pv0 [pr2[0]], pv1 [pr2[1]] (dim 2); per
 * query q6 = {u0, u1, px, py, p0, p1}: out7 = Sample(u, p) xy pdf, Invert(p_xy, p) xy pdf,
 * Evaluate(p_xy, p) (Sample / Invert left 0 without a CDF).  The measured BxDF's tables. */
int pbrt_debug_pl2d(int dim, int cdf, const float *data, int xs, int ys, const int *pr2, const float *pv0,
                    const float *pv1, const float *q6, int n, float *out7);
/* WindowedPiecewiseConstant2D alone (util/sampling.h:890-980) over func [res][res] (the portal
 * light's sampling distribution): per query q8 = {u0, u1, window b0 b1 b2 b3, qx, qy}: out5 =
 * Sample ok, x, y, pdf, PDF(q, b) */
int pbrt_debug_windowed2d(const float *func, int res, const float *q8, int n, float *out5);
/* The procedural textures' kernels code on the host (core/texture_eval.h): kind 0 FBm, 1
 * Turbulence (wrinkled), 2 windy, 3 InsidePolkaDot (in9[0..1] = s, t), 4 marble; params4 =
 * octaves, roughness, scale, variation; in9 per point = p, dpdx, dpdy; out6 per point = value
 * (marble: RGB, then its RGBAlbedoSpectrum sigmoid coefficients) */
int pbrt_debug_procedural(int kind, const float *params4, const float *in9, int n, float *out6);
/* RNG::SetSequence(seq); RNG::Advance(advance); two Uniform<uint32_t>() (util/rng.h:119-150) */
int pbrt_debug_rng(uint64_t seq, uint64_t advance, uint32_t *out2);
/* util/scattering.h components as the product evaluates them (core.h), host side.
 * trowbridge: in13 = ax ay wo3 wi3 wm3 u0 u1 (TrowbridgeReitzDistribution(ax, ay)) ->
 *   out14 = alpha_x alpha_y smooth D(wm) D(wo,wm) Lambda(wo) G1(wo) G(wo,wi) PDF(wo,wm)
 *           Sample_wm(wo,u)3 regularized alpha_x alpha_y
 * fresnel: in10 = cos eta eta_re eta_im wi3 n3 -> out10 = FrDielectric FrComplex
 *   refract_ok etap wt3 reflect3 */
int pbrt_debug_trowbridge(const float *in13, float *out14);
int pbrt_debug_fresnel(const float *in10, float *out10);
/* Triangle::InteractionFromIntersection with optional vertex normals n9 / uv6 (NULL = absent)
 * at barycentrics b3, and the normal of Triangle::Sample(u2): out15 = n3 shading.n3 dpdu3
 * shading.dpdu3 sample_n3 (shapes.h:884-1046) */
int pbrt_debug_triangle_shading(const float *p9, const float *n9, const float *uv6, int flip, const float *b3,
                                const float *u2, float *out15);
/* GetNamedSpectrum(name)(lambda_i) for the metal / glass tables */
int pbrt_debug_named_spectrum(const char *name, const float *lambda, int n, float *out);
/* DielectricBxDF (type 1) / ConductorBxDF (type 2) / this fork's RetroreflectiveBxDF (type 11,
 * bxdfs.h:102-215) in the shading frame: params3 = alpha_x
 * alpha_y eta (alphas as the constructor leaves them); eta31 / k31 the conductor's sampled
 * spectra; u3 = uc u0 u1.  out70 = sample_ok wi3 pdf flags etap f_sample[31] f(wo,wi)[31]
 * PDF(wo,wi) (Sample_f / f / PDF of bxdfs.h:300-517, bxdfs.cpp:77-245) */
int pbrt_debug_bxdf(int type, const float *params3, const float *eta31, const float *k31, const float *wo3,
                    const float *wi3, const float *u3, float *out70);
/* LayeredBxDF (CoatedDiffuseBxDF / CoatedConductorBxDF, bxdfs.h:565-1052) in the shading
 * frame: params12 = top alpha_x alpha_y eta, bottom type (0 diffuse, 2 conductor) alpha_x
 * alpha_y, thickness g maxdepth nsamples radiance(1/0) 0; a31 = diffuse R or conductor eta,
 * b31 = conductor k, alb31 = layer albedo; u3 = uc u0 u1.  out72 = sample_ok wi3 pdf flags
 * f_sample[31] f(wo,wi)[31] PDF(wo,wi) Flags() 0 0 (stochastic estimates: RNGs seeded from
 * the directions as the reference's) */
int pbrt_debug_layered(const float *params12, const float *a31, const float *b31, const float *alb31,
                       const float *wo3, const float *wi3, const float *u3, float *out72);
/* host-side BVH8 build of the scene (what pbrt_context_create uploads): out8 = nodes, leaf-order
 * triangles, tree depth, worst-case traversal stack entries, wide node bytes, quantised node
 * bytes, 0, 0 */
int pbrt_debug_bvh_stats(const pbrt_scene *scene, int64_t *out8);
/* Host traversal of the device BVH8 (builder: spatial = 1 spatial splits, 0 object splits,
   -1 the environment's choice) for n rays (ox oy oz dx dy dz); writes the closest t (-1 for
   a miss) and the original triangle index, and stats4 = {node visits, triangle tests, leaf
   references, nodes}.  Checks the builders against a brute-force search without a GPU. */
int pbrt_debug_bvh_trace(const pbrt_scene *scene, int spatial, const float *rays, int n, float *tOut, int *primOut,
                         int64_t *stats4);
/* BVHLightSampler::buildBVH (lightsamplers.cpp:135-238) as the loader runs it, over given
 * LightBounds lights13 [n][13] = pMin3 pMax3 w3 phi cosTheta_o cosTheta_e twoSided: nodes12
 * [n_nodes][12] decoded CompactLightBounds (pMin3 pMax3 w3 phi cosTheta_o cosTheta_e), info3
 * [n_nodes][3] childOrLight isLeaf twoSided, trails [n] bit trails (0xffffffff: not in the
 * tree); at most max_nodes nodes are written, *n_nodes = the tree's node count (host only) */
int pbrt_debug_light_bvh(const float *lights13, int n, float *nodes12, int32_t *info3, uint32_t *trails, int max_nodes,
                         int *n_nodes);
/* queue counters of the last pass: [depth][8] = rays, material hits, shadow rays, escaped,
 * emissive hits (diagnostics) */
int pbrt_debug_queue_counts(pbrt_context *ctx, int32_t *counts, int n);
/* profiling build only (PBRT_AMD_SECTION_TIMING): summed wave cycles per kernel section
 * since the last pbrt_reset_stats; zeros in the product build */
int pbrt_debug_kernel_sections(pbrt_context *ctx, uint64_t *cycles, int n);
/* queue-integrity check of the volumetric wavefront (diagnostics): with it on, every queue
 * slot the surface, layered and medium-scattering stages count must be written; a slot that is
 * counted but left unwritten (a "hole") is counted and printed by the device, and pbrt_render
 * stops with an error before any stage reads it.
 * pbrt_debug_queue_holes returns the holes found since its last call and resets the count.
 * PBRT_AMD_QUEUE_CHECK=1 turns the check on from the environment. */
/* The plymesh displacement of shapes.cpp:1436-1452 (TriQuadMesh::Displace, util/mesh.h:91-191:
   quads to triangles, normals when n is null, refinement to edges below edgeLength in render
   space, p += d n, normals recomputed) with a closed-form d (mode 0: 0.1 u - 0.05 v; mode 1:
   0.25 p.y u + 0.125; mode 2: 0.1) in place of the texture.  counts2 = {vertices, triangles} of the result;
   fails when they exceed capVerts / capTris. */
int pbrt_debug_displace(const float *p, const float *uv, const float *n, int nVerts, const int *tri, int nTri,
                        const int *quad, int nQuad, const float *renderFromObject16, float edgeLength, int mode,
                        int capVerts, int capTris, float *pOut, float *nOut, float *uvOut, int *triOut, int *counts2);
int pbrt_debug_set_queue_check(int on);
int pbrt_debug_queue_holes(int *holes);

#ifdef __cplusplus
}
#endif

#endif /* PBRT_AMD_DEBUG_H */
