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
#include "../host/bvh.h"

namespace pbrt_amd {

constexpr int kDenseN = 311;
constexpr int kMaxLightBVHDepth = 64;

struct DeviceLightNode {
    LightNodeBounds b;
    int childOrLight;
    int isLeaf;
};

constexpr int kMaxStackSize = 64;  // traversal stack entries per lane (64 KB of LDS per block)

struct DeviceScene {
    // geometry (leaf order)
    const BVH8Node *nodes;
    const float4 *triVerts;  // 3 per triangle
    int nTris;
    const int *primMaterial;
    const int *primLight;
    const uint8_t *primFlip;
    // materials
    const float4 *matCoeffs;  // c0, c1, c2, constant value
    const int *matConstant;
    int nMaterials;
    // area lights
    int nAreaLights;
    const int *lightPrim;  // leaf-order prim
    const float *lightScale;
    const int *lightSpectrum;
    const int *lightTwoSided;
    const float *lightArea;
    const uint32_t *lightBitTrail;  // 0xffffffff when not in the light BVH
    // infinite (uniform) lights
    int nInfinite;
    const int *infSpectrum;
    const float *infScale;
    // light sampler
    int uniformLightSampler;
    const DeviceLightNode *lightNodes;
    int nLightNodes;
    const float *dense;  // [nSpectra][311]
    // sensor (PixelSensor cie1931): x,y,z bar dense tables [3][311]
    const float *sensor;
    const float4 *sensor4;  // same tables interleaved: {xbar, ybar, zbar, 0} per dense entry
    float imagingRatio;
    // camera
    float cameraFromRaster[16];
    float renderFromCamera[16];
    float lensRadius, focalDistance;
    // film / filter
    int xres, yres, px0, px1, py0, py1;
    float filterRadiusX, filterRadiusY;
    // halton
    const uint16_t *perm;
    const uint32_t *permOffset, *permNDigits, *permBase;
    const uint4 *haltonDim;  // per dimension {base, nDigits | shift << 8, permOffset, magic}
    int nDims;
    int baseScales[2], baseExponents[2], multInverse[2];
    int maxDepth;
    int stackSize;  // BVH traversal stack entries per lane (BVH8::maxStack)
};

// Per-pass wavefront buffers; N = paths per pass = P pixels x S samples.
struct PathState {
    int N;
    int P;              // pixels per sample in this pass
    int width;          // pixel row width (px1 - px0)
    const int *rows;    // P / width row indices (absolute y)
    int firstSample;    // sample index of slot block 0
    float *beta;        // [31][N]
    float *rl;          // [N]
    float *L;           // [3][N] sensor RGB
    float *lambda0;     // [N]
    float *filterW;     // [N]
    float *etaScale;    // [N]
    int *flags;         // [N]: bit0 specularBounce, bit1 anyNonSpecular
    float *ray;         // [6][N]
    float *ctx;         // [12][N]: prev p, n, ns, pError
    int *hitPrim;       // [N]
    float *hitB;        // [4][N]: b0, b1, b2, t
    float *shadowRay;   // [6][N]
    float *shadowL;     // [3][N]
    int *rayQ[2];       // [N]
    int *matQ;          // [N]
    int *shadowQ;       // [N]
    int *escQ;          // [N] escaped rays (only with infinite lights)
    int *counters;      // [(maxDepth+2) * 4]: ray, mat, shadow, spare per depth
    double *film;       // [4][xres*yres]: rgbSum[3], weightSum (sensor RGB)
    unsigned long long *stats;  // [8]: camera rays, closest rays, shadow rays, node visits
};

}  // namespace pbrt_amd
