// Device-resident scene and path-state layout of the MI355X wavefront.
//
// Path state is structure-of-arrays; every spectral quantity is stored wavelength-major
// ([31][N]) so a wave64 access to one wavelength is a single 256-byte coalesced segment
// (the reference's SOA<SampledSpectrum> keeps 31 floats per item contiguous, soa.h:51-57).
// Surface-only scenes keep r_u == 1 and r_l spectrally constant (wavefront/surfscatter.cpp:
// 181-187), so r_l is one float per path; radiance L is accumulated directly as PixelSensor
// RGB (film.h:95-100 is linear in L and maxComponentValue is infinite by default).
#pragma once

#include <cstdint>

#include "../core/core.h"
#include "../core/texture_eval.h"
#include "../host/bvh.h"

namespace pbrt_amd {

constexpr int kDenseN = 311;
constexpr int kMaxLightBVHDepth = 64;

struct DeviceLightNode {
    LightNodeBounds b;
    int childOrLight;
    int isLeaf;
};

// One area light (a triangle of a DiffuseAreaLight shape) as the light-sampling code reads it:
// the triangle's vertices and the light's parameters in one 64-byte record.
struct DeviceAreaLight {
    float4 v0, v1, v2;  // render-space vertices; v0.w: prim bits; v1.w / v2.w: the spread's
                        // cosFalloffEnd (> 0: a spread below 90 degrees) / tanFalloffEnd
    float scale;
    int spectrum, twoSided, flip;
};
static_assert(sizeof(DeviceAreaLight) == 64, "DeviceAreaLight must be 64 bytes");

// Dynamic-LDS layout of k_shade_diffuse (byte offsets; host-computed per scene).  The block
// stages everything its lanes look up per wavelength or per sample: sensor tables, light
// spectra, the Halton permutations of the launch's 7 dimensions, lights and materials.
constexpr int kShadeLdsDepths = 16;
struct ShadeLdsLayout {
    int sensor, dense, perm, lights, lightNodes, mats, matConst, total;
    int denseInLds, lightsInLds, matsInLds, permEntries;
    int plInLds, plCount;  // conductor eta / k knots (lambdas, then values) after the perm tables
    int totalByDepth[kShadeLdsDepths];  // bytes a launch at that depth needs (perm tables last)
};

// Work queues are sharded: a producer block appends to shard (blockIdx.x % kShards), each
// shard with its own counter on its own cache line.  Same-line atomics serialise at ~11 ns
// each on MI355X (tools/microbench/atomics.hip); kShards lines take the queue appends off the
// critical path.  Producer grids are multiples of kShards and grid-stride in 256-item
// chunks, so one producer kernel gives shard s at most its count/kShards + 256 items; a queue
// fed by several producers (surface, layered, medium, subsurface stages) can overshoot by one
// chunk per producer, so capS = N/kShards + 256 kShards, and every pass ends with a check that
// no shard overflowed (k_queue_overflow).
constexpr int kShards = 8;
constexpr int kQueueTrash = 64;  // record slots past the shards (PathState::NR - 1: overflow writes)
constexpr int kCounterPad = 64;  // ints between counters (256 B)
constexpr int kNumQueues = 8;
constexpr int kCntRay = 0, kCntMat = 1, kCntShadow = 2, kCntEscaped = 3, kCntEmissive = 4;
// per-material-type queues (pbrt's MaterialEvalQueue per Material::Types, surfscatter.cpp:39-55):
// diffuse uses kCntMat, dielectric kCntMat + 4, conductor kCntMat + 5
constexpr int kNumMatTypes = 3;  // == host kMatNumTypes (diffuse, dielectric, conductor)
constexpr int kMatDiffuseT = 0, kMatDielectricT = 1, kMatConductorT = 2;
constexpr int kMatCoatedDiffuseT = 4, kMatCoatedConductorT = 5;  // layered (volumetric path only)
constexpr int kMatThinDielectricT = 6;                           // volumetric path only
constexpr int kMatDiffuseTransmissionT = 7;                      // k_vlayered
constexpr int kMatMixT = 8;  // MixMaterial: resolved per hit by k_closest<kClosestMix>
constexpr int kMatHairT = 9;  // HairBxDF: k_vlayered (volumetric path only)
constexpr int kMatMeasuredT = 10;  // MeasuredBxDF: k_vlayered (volumetric path only)
constexpr int kMatRetroreflectiveT = 11;  // RetroreflectiveBxDF: k_vlayered (volumetric path only)
PHD int MatCounter(int type) { return type == 0 ? kCntMat : kCntMat + 3 + type; }
PHD int CounterIndex(int depth, int queue, int shard) {
    return ((depth * kNumQueues + queue) * kShards + shard) * kCounterPad;
}
// device stats slots: [0..7] ray counters, [16..47] per-section wave cycles (profiling build)
constexpr int kStatsSlots = 48, kStatsSectionBase = 16;
constexpr int kStatQueueOverflow = 4;  // stats slot: queue counters found above capS (k_queue_overflow)
constexpr int kMaxStackSize = 32;  // traversal stack entries per lane (uint2: 64 KB of LDS per block)
constexpr int kSceneLdsBudget = 16 * 1024;  // bytes of BVH nodes + triangles cached in LDS per block (at most)
// Traversal kernels run 256-thread blocks at PBRT_TRAVERSAL_WAVES blocks (= waves per SIMD) per
// CU; the node cache gets what static LDS and the group stack leave of kLdsPerCU / that
constexpr int kLdsPerCU = 160 * 1024;
// Traversal modes (one kernel instantiation each): every node and triangle in LDS, wide nodes
// with the tree top in LDS, quantised nodes
constexpr int kTravLds = 0, kTravWide = 1, kTravQuant = 2;
constexpr int kLdsNodeStride = 17;  // float4 per LDS-cached wide node (68 dwords: conflict-free)
constexpr int kLdsQNodeStride = 5;  // float4 per LDS-cached compressed node (20 dwords: conflict-free)
PHD int LdsNodeStride(int compressed) { return compressed ? kLdsQNodeStride : kLdsNodeStride; }

// Participating media (MakeNamedMedium homogeneous / uniformgrid), as the flat tables of
// pbrt_scene_flat::medium_* (capi.hip MediumTables): per medium 16 ints (type, sigma_a, sigma_s,
// Le dense-spectrum ids, emissive, density nx ny nz, LeScale nx ny nz, value offsets of the
// density / LeScale / 16^3 majorant grids) and 24 floats (g, bounds lo hi, pad,
// mediumFromRender 4x4).  primMedium: {inside, outside} per leaf-order triangle (-1 = none),
// nullptr when no triangle is a medium boundary.
constexpr int kDevMediumGrid = 1;   // info[0] (scene.h MediumType)
constexpr int kDevMediumCloud = 2;  // density / wispiness / frequency + noise permutation at info[11]
// RGBGridMedium: per voxel {c0, c1, c2, scale} of sigma_a, sigma_s and Le (three [nz][ny][nx]
// blocks at info[11]), info[15] bit 0 / 1 / 2: the grid is given; params[7] = sigmaScale,
// values[info[12]] = LeScale
constexpr int kDevMediumRGBGrid = 3;
constexpr int kMajorantRes = 16;
struct DeviceMedia {
    int n;             // media in the scene (0: the surface-only kernels run)
    int cameraMedium;  // medium the camera sits in, or -1
    int allGrey;       // every medium grey (info[14]): the scalar-majorant kernels run
    int hasCloud;      // some medium is a CloudMedium: the grey kernels' cloud instantiations run
    int denseInLds;    // the media kernels stage every dense spectrum in LDS (nDense small)
    const int *info;
    const float *params;
    const float *values;
    const int *primMedium;
};

// PointLight / SpotLight / DistantLight / GoniometricLight / ProjectionLight in render space
// (scene.h DeltaLightDesc): p.xyz position (.w type bits: 0 point, 1 spot, 2 distant,
// 3 goniometric, 4 projection), w.xyz spot axis or direction toward a distant light (.w scale),
// cone = cosFalloffStart, cosFalloffEnd, spectrum bits, offset of the goniometric / projection
// image in DeviceScene::deltaImg (int bits); m0..m2: rows of renderFromLight's inverse 3x3
// (Transform::ApplyInverse on vectors), .w: image width / height bits, projection 1/tan(fov/2)
struct DeviceDeltaLight {
    float4 p, w, cone, m0, m1, m2;
};

struct DeviceScene {
    // geometry (leaf order)
    const BVH8Node *nodes;
    const float4 *qnodes;     // the same tree, quantised (80 B/node) at qStride float4 per node:
    int qStride;              // 5 (packed) or 8 (one 128-B cache line per node)
    int compressed;           // traverse qnodes (HBM-resident scenes) instead of nodes
    const float4 *triVerts;  // 3 per triangle at triStride (3, or 4: 64-B slots)
    int triStride;
    int nTris;
    const int *primMaterial;
    const int *primLight;
    const uint8_t *primFlip;
    // alpha-tested primitives (GeometricPrimitive alpha): leaf order, the alpha texture's
    // program or -1; nAlpha = 0 (and primAlpha null) when no shape has an alpha texture
    const int *primAlpha;
    int nAlpha;
    // bump / normal mapping per material: {displacement program, normal map image, flag, 0};
    // hasBump = 0 (matBump null) when no material perturbs its shading normal
    const int4 *matBump;
    int hasBump;
    const int *primOrig;  // leaf order -> the scene's triangle index (boundary results)
    // per-triangle shading attributes (leaf order, 4 float4 each: n0|flags, n1|u0, n2|v0,
    // u1 v1 u2 v2), nullptr when no mesh has vertex normals or uv
    const float4 *triShade;
    const float4 *triTangent;  // [3][nTris] shading tangents S (triShade bit2), or nullptr
    // measured BRDFs (core/measured.h): kMeasHdr ints each (hdr[7] = the BRDF's blob offset)
    const int *measHdr;
    const float *measData;
    // materials
    const float4 *matCoeffs;  // c0, c1, c2, constant value
    const int *matConstant;
    int nMaterials;
    const int *matType;        // [nMaterials] 0 diffuse, 1 dielectric, 2 conductor
    const float4 *matParams;   // alpha_x, alpha_y (TrowbridgeReitz), dielectric eta, 0
    const int *matSpectra;     // [nMaterials][2] conductor eta / k piecewise-linear spectra
    const float4 *matLayer;    // [nMaterials][3] layered: thickness g maxDepth nSamples | albedo c0..c2 value |
                               // albedo constant, conductor alpha_x alpha_y, interface eta spectrum (-1)
    int matTypeMask;           // bit t: some material of type t exists
    int regularize;            // integrator "regularize" (surfscatter.cpp:127-128)
    int smoothDielectrics;     // every dielectric is EffectivelySmooth and no regularize
    int dispersive;            // some dielectric has a spectral eta (matSpectra[2 * mat] >= 0)
    // piecewise-linear spectra (conductor eta / k): spectrum s spans [plOffsets[s], plOffsets[s+1])
    const int *plOffsets;
    const float *plLambda, *plValue;
    // per spectrum and integer wavelength 360..830 nm: the segment FindInterval picks at that
    // wavelength (PiecewiseLinearEvalIdx starts its search there)
    const uint16_t *plIndex;  // [nPL][kPlIndexN]
    // area lights
    int nAreaLights;
    const int *lightPrim;  // leaf-order prim
    const float *lightScale;
    const int *lightSpectrum;
    const int *lightTwoSided;
    const float *lightArea;
    const DeviceAreaLight *lights;  // [nAreaLights]
    const uint32_t *lightBitTrail;  // 0xffffffff when not in the light BVH
    // infinite-light list (UniformInfiniteLight, or DistantLight when infDistant[j] >= 0)
    int nInfinite;
    const int *infSpectrum;
    const float *infScale;
    const int *infDistant;
    // spheres and disks: prim ids nTris + k (leaf-order triangles first), their BVH
    int nShapes;
    const DeviceShape *shapes;
    const ShapeBVHNode *shapeNodes;
    const float *shapeN;  // [nShapes][12]: a bilinear patch's vertex normals (flags bit 3)
    // ImageInfiniteLight entries: infImage[j] indexes env[] (-1: not an image light)
    const int *infImage;
    const DeviceEnvLight *env;
    int nEnv;
    // point / spot / distant lights: the first nPointSpot are light-BVH members with global light
    // index nAreaLights + i; the infinite-list entry j has global index nAreaLights + nPointSpot + j
    int nDelta, nPointSpot;
    const DeviceDeltaLight *delta;
    const float *deltaImg;  // goniometric Y images and projection per-pixel EnvCoef
    const float *lightSpreadNorm;  // per area light: the spread's normalize_falloffEnd
    const float *lightImg;         // DiffuseAreaLight emission images ({w, h} bits, R G B [h][w][3])
    const int *lightImgOff;        // per area light: its image's offset in lightImg, or -1
    int nImageAreaLights;          // image emitters (their kernels are the Ext ones)
    int hasSpread;                 // some area light has a spread below 90 degrees
    int nImageDelta;        // goniometric + projection lights (their kernels are the Ext ones)
    const int *uniformOrder;  // UniformLightSampler: pbrt's light order -> global index
    float sceneRadius;
    // light sampler
    int uniformLightSampler;
    const DeviceLightNode *lightNodes;
    int nLightNodes;
    const float *dense;  // [nDense][311]
    int nDense;
    // sensor (PixelSensor cie1931): x,y,z bar dense tables [3][311]
    const float *sensor;
    const float4 *sensor4;  // same tables interleaved: {xbar, ybar, zbar, 0} per dense entry
    float imagingRatio;
    float maxComponentValue;  // RGBFilm: a sample's sensor RGB is scaled down to this maximum
    // camera
    float cameraFromRaster[16];
    float renderFromCamera[16];
    float lensRadius, focalDistance;
    int options;  // scene Options: kOptNoPixelJitter / kOptNoWavelengthJitter (camera rays)
    // film / filter
    int xres, yres, px0, px1, py0, py1;
    float filterRadiusX, filterRadiusY;
    int boxFilter;  // box filter: every sample weight is 1 (filters.h:67-71)
    FilterParams filter;       // the pixel filter (core.h)
    FilterTableView filterTab; // FilterSampler tables on the device (tabulated filters)
    // halton
    const uint16_t *perm;
    const uint32_t *permOffset, *permNDigits, *permBase;
    const HaltonDimDesc *haltonDim;  // per dimension (core.h)
    // the 7 permutation tables of each depth's dims (6+7d .. 12+7d) stored contiguously, each
    // depth's block starting on a 4-byte boundary; permDepthInfo[8d] = block start (uint16
    // units), [8d+1+k] = dim k's offset inside the block; [8*maxDepth] = end of the last block
    const uint16_t *permByDepth;
    const uint32_t *permDepthInfo;
    int nDims;
    int baseScales[2], baseExponents[2], multInverse[2];
    int haltonFast32;  // pixel offsets computable in 32 bits (StartPixelSample fast path)
    // sampler: 0 Halton, 1 ZSobol, 2 independent, 3 stratified, 4 Sobol, 5 padded Sobol (core.h kSampler*)
    int samplerType;
    SamplerDesc samp;  // the last four (core.h GenericSampler)
    // sampler dimensions per path depth: 7, or 10 when a material has subsurface scattering
    // (samples.cpp:39-41: direct 3, indirect 4, subsurface 3)
    int dimsPerDepth;
    // SubsurfaceMaterial (materials.h:772-866): per material its SubsurfaceDesc index or -1
    // (nullptr: no subsurface material); per desc kSssParams floats (volpath.hip SssParam*) and
    // a kSssTableFloats BSSRDF table (core/bssrdf.h)
    const int *matSss;
    const float *sssParams;
    const float *sssTables;
    ZSobolParams zs;
    const uint8_t (*zsPerms)[4];  // [24][4]
    const uint32_t *sobolM1;      // Sobol' dimension-1 matrix rows [52]
    int maxDepth;
    int stackSize;  // BVH traversal stack entries (uint2 groups) per lane (BVH8::maxStack)
    float bvhAbsMax[3];  // bound on |plane coordinate| per axis (traversal box-test margins)
    float rayBinLo[3], rayBinScale[3];  // ray-binning grid: cell = (o - lo) * scale, 8 per axis
    int rayBinMode;                     // RayBinKey's key layout (PBRT_AMD_RAY_BIN_KEY)
    int xcdGroups;  // chunks per super-chunk of the traversal kernels' XCD-grouped walk, 0 = off (XcdChunks; PBRT_AMD_XCD_GROUPS)
    int ldsNodes, ldsTris;  // BVH8 nodes / triangles cached in LDS by the traversal kernels
    ShadeLdsLayout shadeLds;
    DeviceMedia media;
    // textures (core/texture_eval.h): expression tables, MIPMap pyramids, the RGB->spectrum
    // table, the camera's differential estimate, and per material the texture programs of
    // reflectance / u roughness / v roughness (-1: the constant parameters apply) + remap flag
    int textured;
    TexView tex;
    CameraDiff camDiff;
    const int4 *matTex;
    // textured hair floats: per material 2 int4 of programs {eta, beta_m, beta_n, alpha},
    // {eumelanin, pheomelanin, -, -} (-1: constant); nullptr when no hair is textured
    const int4 *matHairTex;
    // textured subsurface spectra: per material {sigma_a, sigma_s | mfp} programs (-1: constant);
    // nullptr when none is textured
    const int2 *matSssTex;
    // MixMaterial: per material {material 0, material 1, amount program, 0}
    const int4 *matMix;
    // this struct's copy in device memory (static scene fields only): out-of-line functions
    // that need many scene tables take it, so no kernel copies its DeviceScene into scratch
    const DeviceScene *self;
};

// One depth's path records, compacted: record i is the i-th ray of that depth (pbrt's
// RayWorkItem, workitems.h, in SoA).  Each shade pass writes the surviving paths densely into
// the other parity's records, so every later depth reads contiguous memory instead of the
// thinning-out slots of the original pixel samples.
struct PathRecords {
    float *beta;      // [31][NR] wavelength-major
    float *ray;       // [6][NR] o, d
    float *lambda0;   // [NR] first wavelength (the other 30 follow by pbrt's +10 nm rule)
    float *rl;        // [NR] r_l (spectrally constant for surface-only paths); depth > 0
    float *etaScale;  // [NR]
    int *flags;       // [NR] bit0 specularBounce, bit1 anyNonSpecular
    int *pixel;       // [NR] pixel-sample slot (index of L / film sample); depth > 0
    int *prevIdx;     // [NR] record index at the previous depth (its hit = the MIS context)
    uint32_t *sidx;   // [NR] the pixel sample's Halton index (kNoSampleIndex: recompute it)
};
constexpr uint32_t kNoSampleIndex = 0xffffffffu;

// Per-pass wavefront buffers; N = paths per pass = P pixels x S samples.
struct PathState {
    int N;
    int P;              // pixels per sample in this pass
    int width;          // pixel row width (px1 - px0)
    const int *rows;    // P / width row indices (absolute y)
    int firstSample;    // sample index of slot block 0
    int capS;           // capacity of one queue shard
    int NR;             // record stride = kShards * capS (>= N)
    PathRecords rec[2]; // by depth parity
    // hit records of each depth's rays (by record index), double-buffered by depth parity:
    // the previous depth's hit is the emissive-hit MIS context (pbrt's prevIntrCtx)
    int *hitPrim[2];    // [NR] each
    float *hitB[2];     // [4][NR] each: b0, b1, b2, t
    // shadow-ray queue, compacted (pbrt's ShadowRayWorkItem)
    float *shadowRay;   // [6][NR]
    float *shadowL;     // [3][NR] sensor RGB to add when unoccluded
    int *shadowPixel;   // [NR]
    // per pixel-sample slot
    float *L;           // [3][N] sensor RGB
    // dispersion (SampledWavelengths::TerminateSecondary): the lambda_0-only sensor RGB of the
    // same contributions, and whether the path terminated its secondary wavelengths; null
    // unless the scene has a dielectric with spectral eta
    float *L0;          // [3][N]
    int *lamTerm;       // [N]
    float *filterW;     // [N]
    // work queues: record indices of the current depth
    int *matQ[kNumMatTypes];  // [NR] each: hits per material type
    // textured materials (k_texture, before each shade launch), by record index: the hit's
    // reflectance as sigmoid coefficients c0 c1 c2 + a flag (1: the per-wavelength values are
    // in texR), then the TrowbridgeReitz alphas of a textured roughness; null when untextured
    float *texCoef;     // [8][NR]
    float *texS;        // [2][31][NR] textured subsurface sigma_a, sigma_s | mfp per wavelength
    float *texBump[2];  // by depth parity, [6][NR]: the bump / normal-mapped shading normal and
                        // dpdu of a record (null without such materials)
    float *texR;        // [31][NR] general reflectance expressions (null when none)
    // scenes with mix materials: each hit's resolved material, by depth parity (null otherwise)
    int *hitMat[2];
    int *escQ;          // [NR] escaped rays (only with infinite lights)
    int *emitQ;         // [NR] hits on emissive triangles
    int *counters;      // [CounterIndex(maxDepth + 2, 0, 0)]: per depth, queue and shard
    // ray binning (HBM-resident trees, depth >= 1; null when off): binned rays (o, record
    // index), (d, 0) and the bin counts / running offsets
    float4 *raySort;    // [2][NR]
    int *rayBins;       // [2][kRayBins]
    double *film;       // [4][xres*yres]: rgbSum[3], weightSum (sensor RGB)
    unsigned long long *stats;  // [kStatsSlots]
};

// Path records of the participating-media wavefront (volpath.hip), one per ray of a wavefront
// iteration, double-buffered by iteration parity.  With media r_u and r_l are spectral
// (SampleT_maj's T_maj / T_maj[0] ratios differ per wavelength), the path depth may lag the
// iteration (an interface crossing continues at the same depth, integrator.cpp:374 and
// media.cpp:196-203), each ray carries its medium, and the MIS context of the previous vertex
// is stored (a medium scattering vertex has no surface to rebuild it from).
struct VolRecords {
    float *beta, *ru, *rl;     // [31][NR] wavelength-major
    float *ray;                // [6][NR] o, d
    float *prev;               // [12][NR] prevIntrCtx: p, pErr, n, ns
    float *lambda0, *etaScale; // [NR]
    int *flags;                // [NR] bit0 specularBounce, bit1 anyNonSpecularBounces, bits 2-4:
                               // beta / r_u / r_l stored uniform (entry 0 only, volpath.hip)
    int *pixel, *depth, *medium;
};
// queues of one iteration (counters at CounterIndex(iteration, queue, shard))
constexpr int kVRay = 0, kVSurf = 1, kVShadow = 2, kVMed = 3, kVScat = 4;
constexpr int kVIface = 5;  // surface hits on Material "interface" (k_viface)
constexpr int kVEsc = 6;    // escaped rays (k_vescaped)
constexpr int kVSss = 7;    // transmitted rays into a subsurface material (k_vsss_probe / _scatter)
constexpr int kSssParams = 20;
// BSSRDF work items (GetBSSRDFAndProbeRayWorkItem + SubsurfaceScatterWorkItem,
// wavefront/workitems.h:202-240), compacted: the entry point's state, then the probe's result
struct SssRecords {
    float *beta, *ru;          // [31][NR] after the entry BSDF sample and Russian roulette
    float *po, *ns;            // [3][NR] entry point and shading normal (TabulatedBSSRDF)
    float *lambda0, *etaScale; // [NR]
    float *hitB, *resPdf;      // [3][NR] the reservoir's hit (barycentrics / shape coords), [NR]
    int *mat, *pixel, *depth, *mIn, *mOut, *flags, *hitPrim;  // [NR] (flags: kUni* bits)
    int *src;  // [NR] the entry's record index in this iteration (its texture-stage results)
};
struct VolState {
    VolRecords rec[2];
    int *hitPrim;  // [NR] this iteration's closest hit (-1: none)
    float *hitB;   // [4][NR] b0 b1 b2 t; a medium scattering event stores its point in b0..b2
    int *medQ, *surfQ, *scatQ, *ifaceQ, *escQ;  // record indices
    // shadow rays (ShadowRayWorkItem with spectral Ld, r_u, r_l), compacted
    float *shRay;              // [6][NR] o, d (d unnormalised, tMax = 1 - ShadowEpsilon)
    float *shLd, *shRu, *shRl; // [31][NR]
    float *shLambda0;          // [NR]
    int *shPixel, *shMedium;   // [NR]
    int *shFlags;              // [NR] uniform-spectrum bits (volpath.hip kShUni*)
    int *holes;                // [1] queue-integrity diagnostic: unwritten queue slots found
    SssRecords sss;            // allocated when a material has subsurface scattering
};

}  // namespace pbrt_amd
