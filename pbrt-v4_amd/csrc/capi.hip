// C ABI and render driver of pbrt-v4_amd (declared in include/pbrt_amd.h; the component entry
// points tests and tools use in include/pbrt_amd_debug.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pbrt_amd.h"
#include "../../include/pbrt_amd_debug.h"
#include "core/bssrdf.h"
#include "core/hair.h"
#include "core/measured.h"
#include "host/bvh.h"
#include "host/displace.h"
#include "host/image.h"
#include "host/scene.h"
#include "host/texture.h"
#include "kernels/device.h"

namespace pbrt_amd {
hipError_t LaunchCamera(const DeviceScene &S, const PathState &st, int nActive, hipStream_t s);
hipError_t LaunchClosest(const DeviceScene &S, const PathState &st, int depth, int maxCount, int timed,
                         hipStream_t s, bool sorted);
hipError_t LaunchRayBin(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s);
hipError_t LaunchClassify(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s);
hipError_t LaunchShadeDiffuse(const DeviceScene &S, const PathState &st, int depth, int maxCount, bool lean,
                              hipStream_t s);
hipError_t LaunchTexture(const DeviceScene &S, const PathState &st, int depth, int type, bool full, int maxCount,
                         hipStream_t s);
hipError_t LaunchShadeMicrofacet(const DeviceScene &S, const PathState &st, int depth, int type, int maxCount,
                                 hipStream_t s);
hipError_t LaunchEscaped(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s);
hipError_t LaunchEmissive(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s);
hipError_t LaunchShadow(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s);
hipError_t LaunchFilm(const DeviceScene &S, const PathState &st, int nSamples, hipStream_t s);
hipError_t LaunchCheckRNMath(uint64_t seed, int blocks, int perThread, unsigned long long *bad, hipStream_t s);
hipError_t LaunchDetMath(int fn, const float *a, const float *b, int n, float *out, hipStream_t s);
hipError_t LaunchHairEval(const float *in, int n, float *out, hipStream_t s);
hipError_t LaunchCatmullRom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                            const float *cdf, const float *x, int n, float *out, hipStream_t s);
hipError_t LaunchQueueOverflowCheck(const PathState &st, int nDepths, hipStream_t s);
hipError_t LaunchIntersectBatch(const DeviceScene &S, const float *rays, int n, int anyHit, int *outPrim,
                                float *outHit, hipStream_t s);
size_t SurfaceTraversalStaticLds(int tm);
int TraversalBlocksCompiled(int compressed);
hipError_t LaunchVolCamera(const DeviceScene &S, const PathState &st, const VolState &v, int nActive, hipStream_t s);
hipError_t LaunchVolClosest(const DeviceScene &S, const PathState &st, const VolState &v, int wf, int maxCount,
                            int timed, hipStream_t s);
hipError_t LaunchVolIteration(const DeviceScene &S, const PathState &st, const VolState &v, int wf, int maxCount,
                              hipStream_t s);
void SetQueueCheck(int on);
int TakeQueueHoles();
hipError_t LaunchIntersectOneRandom(const DeviceScene &S, const float *segs, const int *mats, int n, int *prim,
                                    float *hit, float *pdf, hipStream_t s);
hipError_t LaunchIntersectTr(const DeviceScene &S, const float *rays, const int *medium, const float *lambda0, int n,
                             float *out, hipStream_t s);
size_t VolTraversalStaticLds(int tm);
}  // namespace pbrt_amd

using namespace pbrt_amd;

static thread_local std::string g_lastError;
static int Fail(const std::string &msg) {
    g_lastError = msg;
    return 1;
}
#define HIPCHECK(x)                                                                                     \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) throw Error(std::string("HIP error ") + hipGetErrorString(e_) + " at " #x); \
    } while (0)

// Media as flat tables (pbrt_scene_flat::medium_*; the device upload uses the same layout)
static void MediumTables(const SceneDesc &s, std::vector<int32_t> *info, std::vector<float> *params,
                         std::vector<float> *values) {
    info->clear();
    params->clear();
    values->clear();
    for (const MediumDesc &m : s.media) {
        const int dOff = (int)values->size();
        values->insert(values->end(), m.density.begin(), m.density.end());
        const int lOff = (int)values->size();
        values->insert(values->end(), m.LeScale.begin(), m.LeScale.end());
        const int mOff = (int)values->size();
        values->insert(values->end(), m.majorant.begin(), m.majorant.end());
        // GridMedium temperature: {offset, scale, T[nz][ny][nx]} at info[15] (-1: none)
        int tOff = -1;
        if (!m.temperature.empty()) {
            tOff = (int)values->size();
            values->push_back(m.temperatureOffset);
            values->push_back(m.temperatureScale);
            values->insert(values->end(), m.temperature.begin(), m.temperature.end());
        }
        // grey: sigma_a and sigma_s are the same at every wavelength, so every SampledSpectrum
        // built from them (T_maj, sigma_n, ...) has 31 equal entries (the kernels' scalar path)
        auto flat = [&](int idx) {
            const auto &d = s.denseSpectra[idx];
            return std::all_of(d.begin(), d.end(), [&](float v) { return v == d[0]; });
        };
        // (a temperature grid's Le is a blackbody per point: the spectral kernels evaluate it)
        const int grey = m.type != kMediumRGBGrid && tOff < 0 && flat(m.sigmaA) && flat(m.sigmaS) ? 1 : 0;
        info->insert(info->end(), {m.type, m.sigmaA, m.sigmaS, m.Le, m.emissive ? 1 : 0, m.nx, m.ny, m.nz, m.lnx, m.lny,
                                   m.lnz, dOff, lOff, mOff, grey, m.type == kMediumGrid ? tOff : m.rgbGrids});
        const V3 lo(std::min(m.p0.x, m.p1.x), std::min(m.p0.y, m.p1.y), std::min(m.p0.z, m.p1.z));
        const V3 hi(std::max(m.p0.x, m.p1.x), std::max(m.p0.y, m.p1.y), std::max(m.p0.z, m.p1.z));
        params->insert(params->end(), {m.g, lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, m.sigmaScale});
        Mat4 inv = m.type != kMediumHomogeneous ? Inverse4(m.renderFromMedium) : Identity4();
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) params->push_back((float)inv[i][j]);
    }
}

// A hair material's 12 per-material floats in the matLayer slot (k_vlayered, the oracle's
// MakeBSDF): {mode, sigma_a | color: kind value c0 c1 c2 scale pl, eta, beta_m, beta_n, alpha}
static void HairLayer(const MaterialDesc &m, std::vector<float> *out) {
    const SssSpectrumDesc &q = m.hairSpec;
    out->insert(out->end(), {(float)m.hairMode, (float)q.kind, q.value, q.c0, q.c1, q.c2, q.scale, (float)q.pl, m.eta,
                             m.hairBetaM, m.hairBetaN, m.hairAlpha});
}

// Subsurface tables (pbrt_scene_flat::material_sss / sss_params / sss_tables; the device
// upload uses the same layout): per material its SubsurfaceDesc or -1, per desc kSssParams
// floats {mode, scale, eta, fresnelC, a: kind value c0 c1 c2 scale pl, b: the same, g, 0} and
// its kSssTableFloats table.  Empty when no material has subsurface scattering.
static void SssTables(const SceneDesc &s, std::vector<int32_t> *matSss, std::vector<float> *params,
                      std::vector<float> *tables) {
    matSss->clear();
    params->clear();
    tables->clear();
    if (s.sss.empty()) return;
    for (const MaterialDesc &m : s.materials) matSss->push_back(m.sss);
    auto spec = [&](const SssSpectrumDesc &q) {
        params->insert(params->end(), {(float)q.kind, q.value, q.c0, q.c1, q.c2, q.scale, (float)q.pl});
    };
    for (const SubsurfaceDesc &d : s.sss) {
        if ((int)d.table.size() != kSssTableFloats) throw Error("subsurface table has the wrong size");
        params->insert(params->end(), {(float)d.mode, d.scale, d.eta, d.fresnelC});
        spec(d.a);
        spec(d.b);
        params->insert(params->end(), {d.g, 0.f});
        tables->insert(tables->end(), d.table.begin(), d.table.end());
    }
    static_assert(kSssParams == 20, "SubsurfaceDesc packing");
}

static CameraDiff MakeCameraDiff(const SceneDesc &s) {
    CameraDiff c{};
    for (int k = 0; k < 12; ++k) c.cameraFromRender[k] = s.cameraFromRender[k];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) c.renderFromCamera[3 * i + j] = (float)s.camera.renderFromCamera[i][j];
    c.minPosDx = V3(s.minPosDx[0], s.minPosDx[1], s.minPosDx[2]);
    c.minPosDy = V3(s.minPosDy[0], s.minPosDy[1], s.minPosDy[2]);
    c.minDirDx = V3(s.minDirDx[0], s.minDirDx[1], s.minDirDx[2]);
    c.minDirDy = V3(s.minDirDy[0], s.minDirDy[1], s.minDirDy[2]);
    // cameras.h:187-190; Option "disablepixeljitter" takes the full pixel footprint
    c.sppScale = (s.options & kOptNoPixelJitter) ? 1.f : std::max<float>(.125f, 1 / std::sqrt((float)s.spp));
    c.noFilter = (s.options & kOptNoTextureFiltering) ? 1 : 0;  // surfscatter.cpp:77
    return c;
}
// ImageInfiniteLight::ImageLe's RGBIlluminantSpectrum per pixel (lights.h:625-631,
// util/spectrum.cpp:246-251): ClampZero(rgb), scale = 2 max, coefficients of rgb / scale
static std::vector<EnvCoef> BuildEnvCoefs(const EnvLightDesc &e) {
    const std::vector<float> &tab = RGBToSpectrumTableData();
    TexView T{};
    T.rgbZNodes = tab.data();
    T.rgbCoeffs = tab.data() + 64;
    const size_t np = (size_t)e.res * e.res;
    std::vector<EnvCoef> out(np);
    const std::vector<float> &rgb = e.portal ? e.rect : e.rgb;  // a portal light's rectified image
    for (size_t p = 0; p < np; ++p) {
        const float r = std::max(0.f, rgb[3 * p]), g = std::max(0.f, rgb[3 * p + 1]), b = std::max(0.f, rgb[3 * p + 2]);
        const float m = std::max(r, std::max(g, b));
        const float scale = 2 * m;
        float c[3];
        if (scale != 0) RGBToCoeffs(T, r / scale, g / scale, b / scale, c);
        else RGBToCoeffs(T, 0, 0, 0, c);
        out[p] = EnvCoef{c[0], c[1], c[2], scale};
    }
    return out;
}

struct pbrt_scene {
    SceneDesc desc;
    // flattened copies for pbrt_scene_get_flat
    std::vector<float> verts, matCoeffs, lightScale, infScale, dense, sensor, nodeBounds, matParams, plLambda, plValue,
        mediumParams, mediumValues, matLayer;
    std::vector<int32_t> mediumInfo, matSss;
    std::vector<float> sssParams, sssTables;
    std::vector<int32_t> tris, lightPrim, lightSpectrum, lightTwoSided, infSpectrum, matConstant, nodeInfo, matType,
        matSpectra, plOffsets, infDistant, uniformOrder;
    std::vector<float> deltaLights, deltaImages, lightSpread, areaImages;
    std::vector<int32_t> lightImage;
    std::vector<int32_t> infImage, envInfo, shapeInfo, primAlpha;
    std::vector<float> shapeParams, shapeNormals;
    std::vector<float> envXform, envRgb, envPortal;
    mutable std::vector<const char *> measuredFiles;
    std::vector<uint64_t> envOffset;
    TexTables tex;
    void Flatten() {
        const SceneDesc &s = desc;
        infImage.clear();
        for (auto &l : s.infiniteLights) infImage.push_back(l.image);
        shapeInfo.clear();
        shapeParams.clear();
        shapeNormals.clear();
        primAlpha.clear();
        if (!s.alphaTex.empty()) {
            for (int id : s.triAlpha) primAlpha.push_back(id >= 0 ? s.alphaTex[id][0] : -1);
            for (const AnalyticShapeDesc &a : s.shapes) primAlpha.push_back(a.alpha >= 0 ? s.alphaTex[a.alpha][0] : -1);
        }
        for (const AnalyticShapeDesc &a : s.shapes) {
            shapeInfo.insert(shapeInfo.end(), {a.dev.kind, a.dev.flags, a.material, a.light, a.medium[0], a.medium[1], 0, 0});
            shapeParams.insert(shapeParams.end(), a.dev.r2o, a.dev.r2o + 12);
            shapeParams.insert(shapeParams.end(), a.dev.o2r, a.dev.o2r + 12);
            shapeParams.insert(shapeParams.end(), {a.dev.a, a.dev.b, a.dev.c, a.dev.d, a.dev.e, a.dev.f, 0.f, 0.f});
            shapeNormals.insert(shapeNormals.end(), a.normals.begin(), a.normals.end());
        }
        envInfo.clear();
        envXform.clear();
        envPortal.clear();
        envRgb.clear();
        envOffset.clear();
        for (const EnvLightDesc &e : s.envLights) {
            envInfo.insert(envInfo.end(), {e.res, e.portal ? 1 : 0, 0, 0});
            for (int k = 0; k < 4; ++k) envPortal.insert(envPortal.end(), e.portalP[k], e.portalP[k] + 3);
            envXform.insert(envXform.end(), e.renderFromLight, e.renderFromLight + 9);
            envXform.insert(envXform.end(), e.lightFromRender, e.lightFromRender + 9);
            envOffset.push_back(envRgb.size() / 3);
            envRgb.insert(envRgb.end(), e.rgb.begin(), e.rgb.end());
        }
        BuildTexTables(s, &tex);
        verts.clear();
        for (V3 v : s.verts) {
            verts.push_back(v.x);
            verts.push_back(v.y);
            verts.push_back(v.z);
        }
        tris.clear();
        for (auto &t : s.tris) tris.insert(tris.end(), t.begin(), t.end());
        matCoeffs.clear();
        matConstant.clear();
        matType.clear();
        matParams.clear();
        matSpectra.clear();
        matLayer.clear();
        for (auto &m : s.materials) {
            if (m.type == kMatHair) HairLayer(m, &matLayer);
            else if (m.type == kMatMeasured) matLayer.insert(matLayer.end(), {(float)m.measured, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0});
            else
                matLayer.insert(matLayer.end(), {m.thickness, m.g, (float)m.maxDepth, (float)m.nSamples, m.a0, m.a1, m.a2,
                                                 m.albedoValue, m.albedoConstant ? 1.f : 0.f, m.cAlphaX, m.cAlphaY,
                                                 (float)m.ifaceEtaSpec});
            matCoeffs.insert(matCoeffs.end(), {m.c0, m.c1, m.c2, m.constantValue});
            matConstant.push_back(m.constant ? 1 : 0);
            matType.push_back(m.type);
            matParams.insert(matParams.end(), {m.alphaX, m.alphaY, m.eta, m.scale});
            matSpectra.insert(matSpectra.end(), {m.etaSpec, m.kSpec});
        }
        MediumTables(s, &mediumInfo, &mediumParams, &mediumValues);
        SssTables(s, &matSss, &sssParams, &sssTables);
        plOffsets.assign(1, 0);
        plLambda.clear();
        plValue.clear();
        for (auto &sp : s.plSpectra) {
            plLambda.insert(plLambda.end(), sp.lambda.begin(), sp.lambda.end());
            plValue.insert(plValue.end(), sp.value.begin(), sp.value.end());
            plOffsets.push_back((int32_t)plLambda.size());
        }
        lightPrim.clear();
        lightScale.clear();
        lightSpectrum.clear();
        lightTwoSided.clear();
        lightSpread.clear();
        lightImage.clear();
        areaImages.clear();
        std::vector<int> areaImageOff;
        for (const AreaLightImage &im : s.areaLightImages) {
            areaImageOff.push_back((int)areaImages.size());
            areaImages.push_back((float)im.w);
            areaImages.push_back((float)im.h);
            areaImages.insert(areaImages.end(), im.rgb.begin(), im.rgb.end());
        }
        for (auto &l : s.areaLights) {
            lightPrim.push_back(l.shape >= 0 ? (int32_t)s.tris.size() + l.shape : l.prim);
            lightScale.push_back(l.scale);
            lightSpectrum.push_back(l.spectrum);
            lightTwoSided.push_back(l.twoSided ? 1 : 0);
            lightSpread.insert(lightSpread.end(), {l.cosFalloffEnd, l.tanFalloffEnd, l.normFalloffEnd});
            lightImage.push_back(l.image >= 0 ? areaImageOff[l.image] : -1);
        }
        infSpectrum.clear();
        infScale.clear();
        infDistant.clear();
        for (auto &l : s.infiniteLights) {
            infSpectrum.push_back(l.spectrum);
            infScale.push_back(l.scale);
            infDistant.push_back(l.distant);
        }
        deltaLights.clear();
        deltaImages.clear();
        for (auto &d : s.deltaLights) {
            deltaLights.insert(deltaLights.end(), {(float)d.type, (float)d.spectrum, d.scale, d.cosFalloffStart,
                                                   d.cosFalloffEnd, d.p.x, d.p.y, d.p.z, d.w.x, d.w.y, d.w.z});
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) deltaLights.push_back(d.m[i][j]);
            float off = -1;
            if (!d.img.empty()) {
                off = (float)deltaImages.size();
                deltaImages.insert(deltaImages.end(), {d.invTanAng, 0.f, 0.f, 0.f});
                deltaImages.insert(deltaImages.end(), d.img.begin(), d.img.end());
            }
            deltaLights.insert(deltaLights.end(), {d.phi, off, (float)d.imgW, (float)d.imgH});
        }
        uniformOrder.assign(s.uniformOrder.begin(), s.uniformOrder.end());
        dense.clear();
        for (auto &d : s.denseSpectra) dense.insert(dense.end(), d.begin(), d.end());
        sensor.clear();
        sensor.insert(sensor.end(), s.sensorX.begin(), s.sensorX.end());
        sensor.insert(sensor.end(), s.sensorY.begin(), s.sensorY.end());
        sensor.insert(sensor.end(), s.sensorZ.begin(), s.sensorZ.end());
        nodeBounds.clear();
        nodeInfo.clear();
        for (auto &n : s.lightNodes) {
            const LightNodeBounds &b = n.bounds;
            nodeBounds.insert(nodeBounds.end(), {b.pMin.x, b.pMin.y, b.pMin.z, b.pMax.x, b.pMax.y, b.pMax.z, b.w.x, b.w.y,
                                                 b.w.z, b.phi, b.cosTheta_o, b.cosTheta_e});
            nodeInfo.insert(nodeInfo.end(), {n.childOrLight, n.isLeaf, b.twoSided});
        }
    }
};

template <typename T>
struct DevBuf {
    T *p = nullptr;
    size_t n = 0;
    void Alloc(size_t count) {
        Free();
        n = count;
        if (count) HIPCHECK(hipMalloc((void **)&p, count * sizeof(T)));
    }
    void Upload(const std::vector<T> &v) {
        Alloc(v.size());
        if (!v.empty()) HIPCHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    }
    void Free() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DevBuf() { Free(); }
};

struct pbrt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    // side stream for the short emission kernels (HandleEmissiveIntersection / HandleEscapedRays):
    // they are latency-bound on small queues and independent of the same depth's material
    // stage, so they run beside it; per depth, eClosest orders them after the closest-hit
    // launch and eEmit orders the shadow stage (which also adds to L) after them
    hipStream_t sideStream = nullptr;
    std::vector<hipEvent_t> eClosest, eEmit;
    SceneDesc desc;
    BVH8 bvh;
    DeviceScene S{};
    DevBuf<DeviceScene> sceneSelf;
    // scene buffers
    DevBuf<BVH8Node> nodes;
    DevBuf<float4> qnodes;  // qStride float4 per node
    int qStride = 5;
    int triStride = 3;  // float4 per triangle in triVerts
    DevBuf<float> triVerts, matCoeffs, lightScale, lightArea, infScale, dense, sensor;
    DevBuf<int> primMaterial, primLight, matConstant, lightPrim, lightSpectrum, lightTwoSided, infSpectrum, infDistant,
        uniformOrder;
    DevBuf<DeviceDeltaLight> deltaLights;
    DevBuf<float> lightSpreadNorm;  // per area light: normalize_falloffEnd of its spread
    bool hasSpread = false;
    DevBuf<float> deltaImg, lightImg;
    DevBuf<int> lightImgOff;
    DevBuf<int> primOrig, matType, matSpectra, plOffsets, matSss;
    DevBuf<float> sssParams, sssTables, sssF;
    DevBuf<int> sssI;
    DevBuf<float> matParams, plLambda, plValue, triShade, triTangent, matLayer, dispL0;
    DevBuf<uint16_t> plIndex;
    DevBuf<int> dispTerm;
    DevBuf<uint8_t> primFlip;
    DevBuf<int> primAlpha;  // leaf order: alpha texture program or -1 (scenes with alpha only)
    DevBuf<uint32_t> lightBitTrail, permOffset, permNDigits, permBase;
    DevBuf<uint16_t> perm;
    DevBuf<HaltonDimDesc> haltonDim;
    uint64_t haltonIndexBound = 0;  // Lean launches: every Halton index below it (HaltonDimDesc::nz)
    DevBuf<uint16_t> permByDepth;
    DevBuf<uint8_t> zsPerms;
    DevBuf<uint32_t> sobolM1;
    DevBuf<uint32_t> sobol32;           // SobolSampler: SobolMatrices32 (only for that sampler)
    DevBuf<uint64_t> vdcSobol, vdcSobolInv;
    DevBuf<uint32_t> permDepthInfo;
    DevBuf<float> sensor4;
    DevBuf<DeviceLightNode> lightNodes;
    DevBuf<DeviceAreaLight> lights;
    DevBuf<int> mediumInfo, primMedium;
    DevBuf<float> mediumParams, mediumValues, filterTab;
    // textures
    DevBuf<DeviceTexNode> texNodes;
    DevBuf<DeviceTexSpec> texSpec;
    DevBuf<DeviceImage> texImages;
    DevBuf<DeviceImageLevel> texLevels;
    DevBuf<uint8_t> texData;
    DevBuf<float> texLuts, rgbTable, ewaLut, noisePerm, texBasis;
    DevBuf<DeviceTexInstr> texInstrs;
    DevBuf<DeviceTexProgram> texProgs;
    DevBuf<int> matTex;
    DevBuf<float> texCoef, texR, texS;  // k_texture results (PathState::texCoef / texR / texS)
    DevBuf<int> infImage;
    DevBuf<DeviceShape> shapes;
    DevBuf<ShapeBVHNode> shapeNodes;
    DevBuf<float> shapeN;
    DevBuf<EnvCoef> envCoef;
    DevBuf<float> envDist;
    DevBuf<DeviceEnvLight> envLights;
    DevBuf<float> portalTab;  // portal lights: SummedAreaTable values then function, per light
    DevBuf<int> measHdr;      // measured BRDFs: headers, then their tables
    DevBuf<float> measData;
    DevBuf<int> queueHoles;       // VolState::holes
    DevBuf<int> matMix, hitMat;   // mix materials: {m0, m1, amount program} and resolved materials
    bool hasMix = false;
    // ray binning before closest hits at depth >= 1 (HBM-resident trees; PBRT_AMD_RAY_SORT=0/1
    // overrides): st.raySort / st.rayBins
    bool rayBinning = false;
    DevBuf<float4> raySort;
    DevBuf<int> rayBins;
    bool texGeneral = false;      // some textured reflectance is not a single image leaf
    DevBuf<int> matBump, matHairTex, matSssTex;
    DevBuf<float> texBump;        // [2][6][NR] (bump / normal-mapped materials only)
    int texTypeMask = 0;          // bit t: some material of type t is textured
    int texFullMask = 0;          // bit t: ... with an expression beyond one non-EWA image leaf
    // wavefront buffers
    int64_t maxPaths = 0;
    DevBuf<float> fState;
    DevBuf<int> iState;
    DevBuf<int> rows;
    DevBuf<double> film;
    DevBuf<unsigned long long> devStats;
    DevBuf<float> vfState;  // media scenes: VolState records
    DevBuf<int> viState;
    PathState st{};
    VolState vs{};
    bool volumetric = false;  // media or interface materials: the volpath.hip kernels render
    // timing
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    int eventsUsed = 0;
    // per-stage kernel profile (pbrt_set_kernel_profiling; ReportKernelStats, gpu/util.cpp:128-246):
    // an event pair around every stage launch, folded into stageStats at pbrt_synchronize
    bool profiling = false;
    struct StageStat {
        std::string name;
        int launches = 0;
        double sum = 0, mn = 0, mx = 0;
    };
    std::vector<StageStat> stageStats;
    struct StageEvents {
        hipEvent_t a, b;
        int stat;
    };
    std::vector<StageEvents> stageEvents;
    int stageEventsUsed = 0;
    pbrt_render_stats stats{};
    std::vector<int> hostCounters;
    std::vector<int> lastRows;

    ~pbrt_context() {
        for (auto &e : events) {
            (void)hipEventDestroy(e.first);
            (void)hipEventDestroy(e.second);
        }
        for (auto &e : stageEvents) {
            (void)hipEventDestroy(e.a);
            (void)hipEventDestroy(e.b);
        }
        for (hipEvent_t e : eClosest) (void)hipEventDestroy(e);
        for (hipEvent_t e : eEmit) (void)hipEventDestroy(e);
        if (sideStream) (void)hipStreamDestroy(sideStream);
        if (stream) (void)hipStreamDestroy(stream);
    }
};

// An RGB reflectance's sigmoid polynomial x(lambda) = c0 lambda^2 + c1 lambda + c2 bounded below
// over every wavelength SampleUniform produces (within [390, 710]), with a generous allowance for
// the float evaluation: x > -1000 gives clamp(.5 + x / (2 sqrt(1 + x^2)), 0, 1) >= 2e-7, so R
// is nonzero at every sampled wavelength (it first rounds to zero near x = -2900).
static bool SigmoidNeverZero(float c0, float c1, float c2) {
    if (!std::isfinite(c0) || !std::isfinite(c1) || !std::isfinite(c2)) return false;
    const double lo = 390, hi = 710;
    auto x = [&](double l) { return ((double)c0 * l + c1) * l + c2; };
    double m = std::min(x(lo), x(hi));
    if (c0 > 0) {
        const double v = -(double)c1 / (2.0 * c0);
        if (v > lo && v < hi) m = std::min(m, x(v));
    }
    const double err = (std::fabs((double)c0) * hi * hi + std::fabs((double)c1) * hi + std::fabs((double)c2)) * 1e-5;
    return m - err > -1000.0;
}

// Binary BVH over the spheres and disks (ShapeBVHNode): median split of the centroids along the
// widest axis down to one shape per leaf (a leaf's child is the shape index, so the device
// array stays in scene order)
static std::vector<ShapeBVHNode> BuildShapeBVH(const std::vector<AnalyticShapeDesc> &shapes) {
    std::vector<ShapeBVHNode> nodes;
    const int n = (int)shapes.size();
    if (n == 0) {
        nodes.push_back(ShapeBVHNode{{0, 0, 0}, {0, 0, 0}, 0, 0});
        return nodes;
    }
    std::vector<V3> lo(n), hi(n), cen(n);
    for (int i = 0; i < n; ++i) {
        ShapeBounds(shapes[i].dev, &lo[i], &hi[i]);
        cen[i] = (lo[i] + hi[i]) * 0.5f;
    }
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    std::function<int(int, int)> build = [&](int a, int e) -> int {
        const int idx = (int)nodes.size();
        nodes.push_back(ShapeBVHNode{});
        V3 bl(kInfinity, kInfinity, kInfinity), bh(-kInfinity, -kInfinity, -kInfinity);
        V3 cl = bl, ch = bh;
        for (int i = a; i < e; ++i) {
            const int k = order[i];
            bl = V3(std::fmin(bl.x, lo[k].x), std::fmin(bl.y, lo[k].y), std::fmin(bl.z, lo[k].z));
            bh = V3(std::fmax(bh.x, hi[k].x), std::fmax(bh.y, hi[k].y), std::fmax(bh.z, hi[k].z));
            cl = V3(std::fmin(cl.x, cen[k].x), std::fmin(cl.y, cen[k].y), std::fmin(cl.z, cen[k].z));
            ch = V3(std::fmax(ch.x, cen[k].x), std::fmax(ch.y, cen[k].y), std::fmax(ch.z, cen[k].z));
        }
        for (int j = 0; j < 3; ++j) {
            nodes[idx].lo[j] = bl[j];
            nodes[idx].hi[j] = bh[j];
        }
        if (e - a == 1) {
            nodes[idx].child = order[a];
            nodes[idx].count = 1;
            return idx;
        }
        const V3 ext = ch - cl;
        const int axis = ext.x > ext.y ? (ext.x > ext.z ? 0 : 2) : (ext.y > ext.z ? 1 : 2);
        const int mid = (a + e) / 2;
        std::nth_element(order.begin() + a, order.begin() + mid, order.begin() + e,
                         [&](int x, int y) { return cen[x][axis] < cen[y][axis]; });
        build(a, mid);
        const int right = build(mid, e);
        nodes[idx].child = right;
        nodes[idx].count = 0;
        return idx;
    };
    build(0, n);
    return nodes;
}

static void BuildDevice(pbrt_context *c) {
    SceneDesc &s = c->desc;
    HIPCHECK(hipSetDevice(c->device));
    HIPCHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHECK(hipStreamCreateWithFlags(&c->sideStream, hipStreamNonBlocking));
    c->eClosest.resize(s.maxDepth + 1);
    c->eEmit.resize(s.maxDepth + 1);
    for (int d = 0; d <= s.maxDepth; ++d) {
        HIPCHECK(hipEventCreateWithFlags(&c->eClosest[d], hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&c->eEmit[d], hipEventDisableTiming));
    }
    c->bvh = BuildBVH8(s.verts, s.tris, 4);
    if (c->bvh.maxStack > kMaxStackSize)
        throw Error("BVH needs a " + std::to_string(c->bvh.maxStack) + "-entry traversal stack (limit " +
                    std::to_string(kMaxStackSize) + ")");
    BVH8 &b = c->bvh;
    // leaf-order positions: with spatial splits (PBRT_AMD_BVH_SBVH) a triangle may sit at several,
    // each carrying the same per-prim data, so a hit on any copy shades the same triangle; the
    // light records name the first
    int nt = (int)b.triPrim.size();
    std::vector<int> origToLeaf(s.tris.size(), -1);
    for (int i = nt - 1; i >= 0; --i) origToLeaf[b.triPrim[i]] = i;
    const int nsh = (int)s.shapes.size();
    std::vector<int> pm(nt + nsh), pl(nt + nsh), po(b.triPrim.begin(), b.triPrim.end());
    std::vector<uint8_t> pf(nt + nsh, 0);
    for (int i = 0; i < nt; ++i) {
        int o = b.triPrim[i];
        pm[i] = s.triMaterial[o];
        pl[i] = s.triLight[o];
        pf[i] = s.triFlip[o];
    }
    // spheres and disks follow the leaf-order triangles (prim nt + k; original id nt + k)
    for (int k = 0; k < nsh; ++k) {
        pm[nt + k] = s.shapes[k].material;
        pl[nt + k] = s.shapes[k].light;
        po.push_back(nt + k);
    }
    if (!s.alphaTex.empty()) {
        std::vector<int> pa(nt + nsh, -1);
        for (int i = 0; i < nt; ++i) {
            const int id = s.triAlpha[b.triPrim[i]];
            pa[i] = id >= 0 ? s.alphaTex[id][1] : -1;
        }
        for (int k = 0; k < nsh; ++k) pa[nt + k] = s.shapes[k].alpha >= 0 ? s.alphaTex[s.shapes[k].alpha][1] : -1;
        c->primAlpha.Upload(pa);
    }
    c->nodes.Upload(b.nodes);
    {
        // quantised nodes packed (80 B) or one per 128-B line (PBRT_AMD_QNODE_LINE=1): a packed
        // node straddles two lines 3 times in 5
        c->qStride = getenv("PBRT_AMD_QNODE_LINE") && atoi(getenv("PBRT_AMD_QNODE_LINE")) ? 8 : 5;
        std::vector<float4> q(b.qnodes.size() * c->qStride, make_float4(0.f, 0.f, 0.f, 0.f));
        for (size_t n = 0; n < b.qnodes.size(); ++n) memcpy(&q[n * c->qStride], &b.qnodes[n], sizeof(BVH8QNode));
        c->qnodes.Upload(q);
    }
    {
        // triangles at 48 B (packed) or 64 B (PBRT_AMD_TRI_LINE=1: never across a 128-B line)
        c->triStride = getenv("PBRT_AMD_TRI_LINE") && atoi(getenv("PBRT_AMD_TRI_LINE")) ? 4 : 3;
        if (c->triStride == 3) {
            c->triVerts.Upload(b.triVerts);
        } else {
            std::vector<float> t(b.triVerts.size() / 12 * 16, 0.f);
            for (size_t i = 0; i < b.triVerts.size() / 12; ++i) memcpy(&t[i * 16], &b.triVerts[i * 12], 48);
            c->triVerts.Upload(t);
        }
    }
    c->primMaterial.Upload(pm);
    c->primLight.Upload(pl);
    c->primFlip.Upload(pf);
    c->primOrig.Upload(po);
    {
        std::vector<DeviceShape> ds;
        for (const AnalyticShapeDesc &a : s.shapes) ds.push_back(a.dev);
        c->shapes.Upload(ds);
        c->shapeNodes.Upload(BuildShapeBVH(s.shapes));
        std::vector<float> sn((size_t)std::max(nsh, 1) * 12, 0.f);
        for (int k = 0; k < nsh; ++k) std::copy(s.shapes[k].normals.begin(), s.shapes[k].normals.end(), sn.begin() + 12 * k);
        c->shapeN.Upload(sn);
    }
    // vertex normals / uv per leaf triangle (only when some mesh has them)
    if (std::any_of(s.triShade.begin(), s.triShade.end(), [](uint8_t f) { return f != 0; })) {
        std::vector<float> ts((size_t)nt * 16, 0.f);
        for (int i = 0; i < nt; ++i) {
            const int o = b.triPrim[i];
            const int flags = s.triShade[o];
            if (!flags) continue;
            const auto &t = s.tris[o];
            float *d = &ts[(size_t)i * 16];
            for (int k = 0; k < 3; ++k) {
                d[4 * k] = s.vertN[t[k]].x;
                d[4 * k + 1] = s.vertN[t[k]].y;
                d[4 * k + 2] = s.vertN[t[k]].z;
            }
            int fl = flags;
            memcpy(&d[3], &fl, 4);
            d[7] = s.vertUV[t[0]][0];
            d[11] = s.vertUV[t[0]][1];
            d[12] = s.vertUV[t[1]][0];
            d[13] = s.vertUV[t[1]][1];
            d[14] = s.vertUV[t[2]][0];
            d[15] = s.vertUV[t[2]][1];
        }
        c->triShade.Upload(ts);
    }
    // shading tangents per leaf triangle (triShade bit2): s0 s1 s2 as float4
    if (std::any_of(s.triShade.begin(), s.triShade.end(), [](uint8_t f) { return (f & 4) != 0; })) {
        std::vector<float> tt((size_t)nt * 12, 0.f);
        for (int i = 0; i < nt; ++i) {
            const int o = b.triPrim[i];
            if (!(s.triShade[o] & 4)) continue;
            const auto &t = s.tris[o];
            for (int k = 0; k < 3; ++k) {
                const V3 v = t[k] < (int)s.vertS.size() ? s.vertS[t[k]] : V3(0, 0, 0);
                tt[(size_t)i * 12 + 4 * k] = v.x;
                tt[(size_t)i * 12 + 4 * k + 1] = v.y;
                tt[(size_t)i * 12 + 4 * k + 2] = v.z;
            }
        }
        c->triTangent.Upload(tt);
    }
    std::vector<float> mc;
    std::vector<int> mk;
    for (auto &m : s.materials) {
        // An RGB albedo whose sigmoid has c0 = c1 = 0 (a grey rgb) is the same value at every
        // wavelength: upload it as a constant, so the kernels skip 31 sigmoid evaluations
        // (identical bits: SigmoidPolynomial(0, 0, c2, lambda) does not depend on lambda).
        const bool grey = !m.constant && m.c0 == 0 && m.c1 == 0;
        const float cv = grey ? SigmoidPolynomial(0.f, 0.f, m.c2, 500.f) : m.constantValue;
        mc.insert(mc.end(), {m.c0, m.c1, m.c2, cv});
        // bit 0: constant R; bit 1: R != 0 at every sampled wavelength (k_shade_diffuse then
        // needs no pass over the wavelengths to learn the BSDF's flags)
        const bool constant = m.constant || grey;
        const bool neverZero = constant ? Clampf(cv, 0, 1) != 0 : SigmoidNeverZero(m.c0, m.c1, m.c2);
        mk.push_back((constant ? 1 : 0) | (neverZero ? 2 : 0));
    }
    c->matCoeffs.Upload(mc);
    c->matConstant.Upload(mk);
    {
        static_assert(kNumMatTypes == kMatNumTypes, "material type count");
        std::vector<int> mt, msp, po{0};
        std::vector<float> mp, pll, plv;
        for (auto &m : s.materials) {
            mt.push_back(m.type);
            mp.insert(mp.end(), {m.alphaX, m.alphaY, m.eta, m.scale});
            msp.insert(msp.end(), {m.etaSpec, m.kSpec});
        }
        for (auto &sp : s.plSpectra) {
            pll.insert(pll.end(), sp.lambda.begin(), sp.lambda.end());
            plv.insert(plv.end(), sp.value.begin(), sp.value.end());
            po.push_back((int)pll.size());
        }
        if (pll.empty()) pll.push_back(0), plv.push_back(0);
        std::vector<float> ml;
        for (auto &m : s.materials) {
            if (m.type == kMatHair) {
                HairLayer(m, &ml);
                continue;
            }
            if (m.type == kMatMeasured) {  // the BRDF's index; its tables are measHdr / measData
                ml.insert(ml.end(), {(float)m.measured, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0});
                continue;
            }
            // grey layer albedo uploaded as a constant (same bits, as the reflectances above)
            const bool grey = !m.albedoConstant && m.a0 == 0 && m.a1 == 0;
            const float av = grey ? SigmoidPolynomial(0.f, 0.f, m.a2, 500.f) : m.albedoValue;
            ml.insert(ml.end(), {m.thickness, m.g, (float)m.maxDepth, (float)m.nSamples, m.a0, m.a1, m.a2, av,
                                 (m.albedoConstant || grey) ? 1.f : 0.f, m.cAlphaX, m.cAlphaY, (float)m.ifaceEtaSpec});
        }
        c->matLayer.Upload(ml);
        {
            std::vector<int> mh;
            std::vector<float> md;
            for (const MeasuredDesc &b : s.measured) {
                std::vector<int> h = b.hdr;
                if (md.size() > (size_t)INT32_MAX - b.blob.size()) throw Error("measured BRDFs too large");
                h[7] = (int)md.size();
                mh.insert(mh.end(), h.begin(), h.end());
                md.insert(md.end(), b.blob.begin(), b.blob.end());
            }
            if (mh.empty()) mh.assign(kMeasHdr, 0), md.push_back(0.f);
            c->measHdr.Upload(mh);
            c->measData.Upload(md);
        }
        {
            std::vector<int32_t> ms;
            std::vector<float> sp, stb;
            SssTables(s, &ms, &sp, &stb);
            if (!ms.empty()) {
                c->matSss.Upload(ms);
                c->sssParams.Upload(sp);
                c->sssTables.Upload(stb);
            }
        }
        c->matType.Upload(mt);
        c->matParams.Upload(mp);
        c->matSpectra.Upload(msp);
        c->plOffsets.Upload(po);
        c->plLambda.Upload(pll);
        c->plValue.Upload(plv);
        // PiecewiseLinearEvalIdx's start segments: FindInterval at each integer wavelength
        std::vector<uint16_t> pli;
        for (size_t j = 0; j + 1 < po.size(); ++j) {
            pli.resize(pli.size() + kPlIndexN);
            BuildPlIndex(pll.data() + po[j], po[j + 1] - po[j], pli.data() + pli.size() - kPlIndexN);
        }
        if (pli.empty()) pli.push_back(0);
        c->plIndex.Upload(pli);
    }
    std::vector<int> lp, ls, lt;
    std::vector<float> lsc, la;
    for (auto &l : s.areaLights) {
        lp.push_back(l.shape >= 0 ? nt + l.shape : origToLeaf[l.prim]);
        ls.push_back(l.spectrum);
        lt.push_back(l.twoSided);
        lsc.push_back(l.scale);
        la.push_back(l.area);
    }
    c->lightPrim.Upload(lp);
    c->lightSpectrum.Upload(ls);
    c->lightTwoSided.Upload(lt);
    c->lightScale.Upload(lsc);
    c->lightArea.Upload(la);
    std::vector<DeviceAreaLight> dl;
    for (auto &l : s.areaLights) {
        DeviceAreaLight d{};
        if (l.shape >= 0) {
            // a sphere or disk emitter: .w holds its prim id nt + shape (no vertices)
            const int prim = nt + l.shape;
            float bits;
            memcpy(&bits, &prim, 4);
            d.v0 = make_float4(0.f, 0.f, 0.f, bits);
            d.v1 = make_float4(0.f, 0.f, 0.f, l.cosFalloffEnd);
            d.v2 = make_float4(0.f, 0.f, 0.f, l.tanFalloffEnd);
            d.scale = l.scale;
            d.spectrum = l.spectrum;
            d.twoSided = l.twoSided;
            dl.push_back(d);
            continue;
        }
        int leaf = origToLeaf[l.prim];
        const float *v = &b.triVerts[(size_t)leaf * 12];
        float leafBits;  // .w: the light's leaf prim (its shading data), as int bits
        memcpy(&leafBits, &leaf, 4);
        d.v0 = make_float4(v[0], v[1], v[2], leafBits);
        d.v1 = make_float4(v[4], v[5], v[6], l.cosFalloffEnd);
        d.v2 = make_float4(v[8], v[9], v[10], l.tanFalloffEnd);
        d.scale = l.scale;
        d.spectrum = l.spectrum;
        d.twoSided = l.twoSided;
        d.flip = pf[leaf];
        dl.push_back(d);
    }
    c->lights.Upload(dl);
    {
        std::vector<float> norm;
        c->hasSpread = false;
        for (const AreaLightDesc &l : s.areaLights) {
            norm.push_back(l.normFalloffEnd);
            c->hasSpread = c->hasSpread || l.cosFalloffEnd > 0;
        }
        c->lightSpreadNorm.Upload(norm);
    }
    std::vector<int> is;
    std::vector<float> isc;
    for (auto &l : s.infiniteLights) {
        is.push_back(l.spectrum);
        isc.push_back(l.scale);
    }
    c->infSpectrum.Upload(is);
    c->infScale.Upload(isc);
    {
        std::vector<int> idist;
        for (auto &l : s.infiniteLights) idist.push_back(l.distant);
        c->infDistant.Upload(idist);
        // image infinite lights: per-pixel spectra and the compensated sampling distribution
        std::vector<int> iimg;
        for (auto &l : s.infiniteLights) iimg.push_back(l.image);
        c->infImage.Upload(iimg);
        std::vector<EnvCoef> coefs;
        std::vector<float> dist;
        std::vector<DeviceEnvLight> els;
        std::vector<std::pair<size_t, size_t>> offs;
        for (const EnvLightDesc &e : s.envLights) {
            const std::vector<EnvCoef> ec = BuildEnvCoefs(e);
            const std::vector<float> dt = BuildEnvDistribution(e);
            offs.push_back({coefs.size(), dist.size()});
            coefs.insert(coefs.end(), ec.begin(), ec.end());
            dist.insert(dist.end(), dt.begin(), dt.end());
        }
        c->envCoef.Upload(coefs);
        c->envDist.Upload(dist);
        // portal lights' windowed distributions: SummedAreaTable values and function
        std::vector<float> ptab;
        std::vector<size_t> poff;
        for (const EnvLightDesc &e : s.envLights) {
            poff.push_back(ptab.size());
            if (!e.portal) continue;
            ptab.insert(ptab.end(), e.portalSat.begin(), e.portalSat.end());
            ptab.insert(ptab.end(), e.portalFunc.begin(), e.portalFunc.end());
        }
        if (ptab.empty()) ptab.push_back(0.f);
        c->portalTab.Upload(ptab);
        for (size_t k = 0; k < s.envLights.size(); ++k) {
            const EnvLightDesc &e = s.envLights[k];
            DeviceEnvLight d{};
            std::memcpy(d.m, e.renderFromLight, sizeof(d.m));
            std::memcpy(d.mi, e.lightFromRender, sizeof(d.mi));
            d.res = e.res;
            d.coef = c->envCoef.p + offs[k].first;
            d.dist = FilterTableView{e.res, e.res, c->envDist.p + offs[k].second};
            if (e.portal) {
                d.portal = 1;
                std::memcpy(d.pf, e.portalFrame, sizeof(d.pf));
                std::memcpy(d.pc0, e.portalP[0], sizeof(d.pc0));
                std::memcpy(d.pc2, e.portalP[2], sizeof(d.pc2));
                d.sat = c->portalTab.p + poff[k];
                d.func = d.sat + (size_t)e.res * e.res;
            }
            els.push_back(d);
        }
        c->envLights.Upload(els);
        std::vector<DeviceDeltaLight> dd;
        std::vector<float> dimg;  // goniometric Y values / projection per-pixel EnvCoef
        for (auto &d : s.deltaLights) {
            DeviceDeltaLight x{};
            x.p = make_float4(d.p.x, d.p.y, d.p.z, BitsToFloat((uint32_t)d.type));
            x.w = make_float4(d.w.x, d.w.y, d.w.z, d.scale);
            int off = -1;
            if (d.type == kDeltaGonio) {
                off = (int)dimg.size();
                dimg.insert(dimg.end(), d.img.begin(), d.img.end());
            } else if (d.type == kDeltaProjection) {
                // ProjectionLight::I's RGBIlluminantSpectrum of the nearest pixel, per pixel
                // (float4 records: 16-byte aligned)
                while (dimg.size() % 4) dimg.push_back(0.f);
                off = (int)dimg.size();
                EnvLightDesc e;
                e.res = 1;
                e.rgb = d.img;
                const size_t np = (size_t)d.imgW * d.imgH;
                for (size_t q = 0; q < np; ++q) {
                    e.rgb.assign(d.img.begin() + 3 * q, d.img.begin() + 3 * q + 3);
                    const EnvCoef ec = BuildEnvCoefs(e)[0];
                    dimg.insert(dimg.end(), {ec.c0, ec.c1, ec.c2, ec.s});
                }
            }
            x.cone = make_float4(d.cosFalloffStart, d.cosFalloffEnd, BitsToFloat((uint32_t)d.spectrum),
                                 BitsToFloat((uint32_t)off));
            x.m0 = make_float4(d.m[0][0], d.m[0][1], d.m[0][2], BitsToFloat((uint32_t)d.imgW));
            x.m1 = make_float4(d.m[1][0], d.m[1][1], d.m[1][2], BitsToFloat((uint32_t)d.imgH));
            x.m2 = make_float4(d.m[2][0], d.m[2][1], d.m[2][2], d.invTanAng);
            dd.push_back(x);
        }
        c->deltaLights.Upload(dd);
        c->deltaImg.Upload(dimg);
        c->uniformOrder.Upload(std::vector<int>(s.uniformOrder.begin(), s.uniformOrder.end()));
    }
    std::vector<float> dense;
    for (auto &d : s.denseSpectra) dense.insert(dense.end(), d.begin(), d.end());
    c->dense.Upload(dense);
    std::vector<float> sensor;
    sensor.insert(sensor.end(), s.sensorX.begin(), s.sensorX.end());
    sensor.insert(sensor.end(), s.sensorY.begin(), s.sensorY.end());
    sensor.insert(sensor.end(), s.sensorZ.begin(), s.sensorZ.end());
    c->sensor.Upload(sensor);
    std::vector<float> sensor4(4 * kDenseN, 0.f);
    for (int i = 0; i < kDenseN; ++i) {
        sensor4[4 * i] = s.sensorX[i];
        sensor4[4 * i + 1] = s.sensorY[i];
        sensor4[4 * i + 2] = s.sensorZ[i];
    }
    c->sensor4.Upload(sensor4);
    std::vector<uint32_t> bt(s.areaLights.size() + s.nPointSpot, 0xffffffffu);  // light-BVH members
    if (!s.uniformLightSampler)
        for (auto &n : s.lightNodes)
            if (n.isLeaf) bt[n.childOrLight] = s.lightBitTrail[n.childOrLight];
    c->lightBitTrail.Upload(bt);
    std::vector<DeviceLightNode> ln;
    for (auto &n : s.lightNodes) ln.push_back(DeviceLightNode{n.bounds, n.childOrLight, n.isLeaf});
    c->lightNodes.Upload(ln);
    c->perm.Upload(s.permTable);
    c->permOffset.Upload(s.permOffset);
    c->permNDigits.Upload(s.permNDigits);
    c->permBase.Upload(s.permBase);
    std::vector<HaltonDimDesc> hd;
    for (size_t d = 0; d < s.permBase.size(); ++d)
        hd.push_back(MakeHaltonDimDesc(s.permBase[d], s.permNDigits[d], s.permOffset[d]));
    // the shade stage's dimensions 6 + 7 depth + {0..6}: one digit count per depth, enough for
    // every Halton index below spp * stride (samplers.h:53-71), the Lean launches' bound
    {
        const uint64_t stride = (uint64_t)s.haltonBaseScales[0] * (uint64_t)s.haltonBaseScales[1];
        c->haltonIndexBound = std::min<uint64_t>((uint64_t)std::max(s.spp, 1) * stride, 1ull << 24);
        for (size_t d = 0; d < hd.size(); ++d) {
            uint32_t nz = 6;
            if (d >= 6 && hd[d].base >= 17) {
                const size_t d0 = 6 + (d - 6) / 7 * 7;
                nz = 0;
                for (size_t j = d0; j < std::min(d0 + 7, hd.size()); ++j)
                    nz = std::max(nz, HaltonDigitsFor(hd[j].base, c->haltonIndexBound));
                nz = std::min(std::max(nz, 1u), 6u);
            }
            HaltonDimTail(&hd[d], s.permTable.data() + hd[d].permOffset, nz);
        }
    }
    c->haltonDim.Upload(hd);
    {
        std::vector<uint8_t> zp(&kZSobolPermutations[0][0], &kZSobolPermutations[0][0] + 96);
        c->zsPerms.Upload(zp);
        std::vector<uint32_t> m1(kSobolMatrixSize);
        for (int k = 0; k < kSobolMatrixSize; ++k) m1[k] = SobolMatrix1Row(k);
        c->sobolM1.Upload(m1);
    }
    {
        std::vector<uint16_t> pb;
        std::vector<uint32_t> info((size_t)8 * (s.maxDepth + 1), 0);
        for (int depth = 0; depth < s.maxDepth; ++depth) {
            if (pb.size() & 1) pb.push_back(0);  // 4-byte aligned block start
            uint32_t start = (uint32_t)pb.size();
            info[8 * depth] = start;
            for (int k = 0; k < 7; ++k) {
                int d = 6 + 7 * depth + k;
                info[8 * depth + 1 + k] = (uint32_t)pb.size() - start;
                if (d < (int)s.permBase.size()) {
                    size_t n = (size_t)s.permBase[d] * s.permNDigits[d];
                    pb.insert(pb.end(), s.permTable.begin() + s.permOffset[d], s.permTable.begin() + s.permOffset[d] + n);
                }
            }
        }
        if (pb.size() & 1) pb.push_back(0);
        info[8 * s.maxDepth] = (uint32_t)pb.size();
        if (pb.empty()) pb.push_back(0);
        c->permByDepth.Upload(pb);
        c->permDepthInfo.Upload(info);
    }

    // participating media: the flat tables, and {inside, outside} per leaf-order triangle
    if (!s.media.empty()) {
        std::vector<int32_t> mi;
        std::vector<float> mp, mv;
        MediumTables(s, &mi, &mp, &mv);
        if (mv.empty()) mv.push_back(0.f);
        c->mediumInfo.Upload(std::vector<int>(mi.begin(), mi.end()));
        c->mediumParams.Upload(mp);
        c->mediumValues.Upload(mv);
        if (!s.triMedium.empty() || nsh > 0) {
            std::vector<int> tm((size_t)(nt + nsh) * 2, -1);
            for (int i = 0; i < nt && !s.triMedium.empty(); ++i) {
                tm[2 * i] = s.triMedium[b.triPrim[i]][0];
                tm[2 * i + 1] = s.triMedium[b.triPrim[i]][1];
            }
            for (int k = 0; k < nsh; ++k) {
                tm[2 * (nt + k)] = s.shapes[k].medium[0];
                tm[2 * (nt + k) + 1] = s.shapes[k].medium[1];
            }
            c->primMedium.Upload(tm);
        }
    }

    DeviceScene &S = c->S;
    S.media.n = (int)s.media.size();
    c->volumetric = !s.media.empty() ||
                    std::any_of(s.materials.begin(), s.materials.end(), [](const MaterialDesc &m) {
                        return m.type == kMatInterface || m.type == kMatCoatedDiffuse || m.type == kMatCoatedConductor ||
                               m.type == kMatThinDielectric || m.type == kMatDiffuseTransmission || m.type == kMatHair ||
                               m.type == kMatMeasured || m.type == kMatRetroreflective;
                    });
    S.dispersive = std::any_of(s.materials.begin(), s.materials.end(),
                               [](const MaterialDesc &m) { return ((m.type == kMatDielectric || m.type == kMatThinDielectric) && m.etaSpec >= 0) || m.ifaceEtaSpec >= 0;
                               });
    if (S.dispersive && !s.media.empty())
        throw std::runtime_error("a dielectric with spectral eta (dispersion) together with participating media is not supported yet");
    c->volumetric = c->volumetric || S.dispersive;
    // subsurface scattering: its r_u becomes spectral (subsurface.cpp:61), so the volumetric
    // kernels (spectral r_u / r_l records) render it
    c->volumetric = c->volumetric || !s.sss.empty();
    // portal lights: Le and PDF_Li depend on the ray origin and the previous vertex, which the
    // volumetric records carry
    c->volumetric = c->volumetric || std::any_of(s.envLights.begin(), s.envLights.end(), [](const EnvLightDesc &e) { return e.portal; });
    S.media.cameraMedium = s.cameraMedium;
    S.media.allGrey = 1;
    for (size_t m = 0; m < s.media.size(); ++m) {
        const auto &a = s.denseSpectra[s.media[m].sigmaA], &b = s.denseSpectra[s.media[m].sigmaS];
        if (!std::all_of(a.begin(), a.end(), [&](float x) { return x == a[0]; }) ||
            !std::all_of(b.begin(), b.end(), [&](float x) { return x == b[0]; }) ||
            s.media[m].type == kMediumRGBGrid ||  // spectra per voxel (its dense sigma_a / sigma_s are 1 / 0)
            !s.media[m].temperature.empty())      // blackbody Le per point
            S.media.allGrey = 0;
    }
    if (getenv("PBRT_AMD_SPECTRAL_MEDIA")) S.media.allGrey = 0;
    S.media.hasCloud = std::any_of(s.media.begin(), s.media.end(), [](const MediumDesc &m) { return m.type == kMediumCloud; }) ? 1 : 0;
    S.media.denseInLds = s.denseSpectra.size() <= 12 ? 1 : 0;  // <= 15 KB of LDS per block  // force the spectral kernels (tests)
    S.media.info = c->mediumInfo.p;
    S.media.params = c->mediumParams.p;
    S.media.values = c->mediumValues.p;
    S.media.primMedium = c->primMedium.p;
    S.nodes = c->nodes.p;
    S.qnodes = c->qnodes.p;
    S.qStride = c->qStride;
    S.triStride = c->triStride;
    S.triVerts = (const float4 *)c->triVerts.p;
    S.nTris = nt;
    S.primMaterial = c->primMaterial.p;
    S.primLight = c->primLight.p;
    S.primFlip = c->primFlip.p;
    S.primAlpha = c->primAlpha.p;
    S.nAlpha = (int)s.alphaTex.size();
    S.primOrig = c->primOrig.p;
    S.nShapes = nsh;
    S.shapes = c->shapes.p;
    S.shapeNodes = c->shapeNodes.p;
    S.shapeN = c->shapeN.p;
    S.triShade = (const float4 *)c->triShade.p;
    S.triTangent = (const float4 *)c->triTangent.p;
    S.measHdr = c->measHdr.p;
    S.measData = c->measData.p;
    S.matCoeffs = (const float4 *)c->matCoeffs.p;
    S.matConstant = c->matConstant.p;
    S.nMaterials = (int)s.materials.size();
    S.matType = c->matType.p;
    S.matSss = s.sss.empty() ? nullptr : c->matSss.p;
    S.sssParams = c->sssParams.p;
    S.sssTables = c->sssTables.p;
    S.dimsPerDepth = s.sss.empty() ? 7 : 10;  // samples.cpp:39-41
    S.matParams = (const float4 *)c->matParams.p;
    S.matSpectra = c->matSpectra.p;
    S.matLayer = (const float4 *)c->matLayer.p;
    S.plOffsets = c->plOffsets.p;
    S.plLambda = c->plLambda.p;
    S.plValue = c->plValue.p;
    S.plIndex = c->plIndex.p;
    S.matTypeMask = 0;
    for (auto &m : s.materials) S.matTypeMask |= 1 << m.type;
    S.regularize = s.regularize ? 1 : 0;
    S.smoothDielectrics = !s.regularize;
    for (auto &m : s.materials)
        if (m.type == kMatDielectricT && (!(std::fmax(m.alphaX, m.alphaY) < 1e-3f) || m.texURough >= 0))
            S.smoothDielectrics = 0;
    // textures: expression tables, pyramids, the RGB->spectrum table, camera differentials
    {
        TexTables tt;
        BuildTexTables(s, &tt);
        c->matTex.Upload(tt.matTex);
        S.matTex = (const int4 *)c->matTex.p;
        std::vector<int> mm;
        for (const MaterialDesc &m : s.materials) {
            mm.insert(mm.end(), {m.mixMat[0], m.mixMat[1], m.texAmount, 0});
            c->hasMix = c->hasMix || m.type == kMatMix;
        }
        c->matMix.Upload(mm);
        S.matMix = (const int4 *)c->matMix.p;
        // textured: some material evaluates a program (the textured shade / texture kernels);
        // the alpha tests of the traversal kernels may need the tables on their own
        {
            std::vector<bool> alphaOnly(s.texPrograms.size(), false);
            for (const auto &a : s.alphaTex) alphaOnly[a[1]] = true;
            for (const MaterialDesc &m : s.materials)
                for (int p : {m.texReflectance, m.texURough, m.texVRough, m.texAmount, m.texDisp, m.texHair[0], m.texHair[1],
                              m.texHair[2], m.texHair[3], m.texHair[4], m.texHair[5], m.texSss[0], m.texSss[1]})
                    if (p >= 0) alphaOnly[p] = false;
            S.textured = std::any_of(alphaOnly.begin(), alphaOnly.end(), [](bool a) { return !a; }) ? 1 : 0;
        }
        // bump / normal mapping (surfscatter.cpp:109-127): evaluated in k_texture
        std::vector<int> mb;
        S.hasBump = 0;
        for (const MaterialDesc &m : s.materials) {
            const bool bump = m.texDisp >= 0 || m.normalMap >= 0;
            mb.insert(mb.end(), {m.texDisp, m.normalMap, bump ? 1 : 0, 0});
            if (bump) S.hasBump = 1;
        }
        if (S.hasBump) S.textured = 1;
        c->matBump.Upload(mb);
        S.matHairTex = nullptr;
        if (tt.anyHairTex) {
            std::vector<int> mh;
            for (const MaterialDesc &m : s.materials)
                mh.insert(mh.end(), {m.texHair[0], m.texHair[1], m.texHair[2], m.texHair[3], m.texHair[4], m.texHair[5], -1, -1});
            c->matHairTex.Upload(mh);
            S.matHairTex = (const int4 *)c->matHairTex.p;
        }
        S.matSssTex = nullptr;
        if (tt.anySssTex) {
            std::vector<int> ms;
            for (const MaterialDesc &m : s.materials) ms.insert(ms.end(), {m.texSss[0], m.texSss[1]});
            c->matSssTex.Upload(ms);
            S.matSssTex = (const int2 *)c->matSssTex.p;
        }
        S.matBump = S.hasBump ? (const int4 *)c->matBump.p : nullptr;
        S.tex = TexView{};
        if (!s.texPrograms.empty() || S.hasBump) {
            // textures on the volumetric path: k_vtexture + k_vsurface<..., Tex> (diffuse,
            // dielectric, conductor) and k_vlayered (bump / normal maps, hair sigma_a and
            // reflectance); mix materials resolve in k_vclosest<TM, true>
            c->texNodes.Upload(tt.nodes);
            c->texSpec.Upload(tt.spec);
            c->texImages.Upload(tt.images);
            c->texLevels.Upload(tt.levels);
            if (tt.data.empty()) tt.data.push_back(0);
            c->texData.Upload(tt.data);
            c->texLuts.Upload(tt.luts);
            c->texInstrs.Upload(tt.instrs);
            c->texProgs.Upload(tt.progs);
            c->rgbTable.Upload(RGBToSpectrumTableData());
            c->ewaLut.Upload(std::vector<float>(GetSpectralData().mipFilterLUT.begin(), GetSpectralData().mipFilterLUT.end()));
            S.tex.nodes = c->texNodes.p;
            S.tex.spec = c->texSpec.p;
            S.tex.images = c->texImages.p;
            S.tex.levels = c->texLevels.p;
            S.tex.data = c->texData.p;
            S.tex.luts = c->texLuts.p;
            S.tex.instrs = c->texInstrs.p;
            S.tex.progs = c->texProgs.p;
            S.tex.rgbZNodes = c->rgbTable.p;
            S.tex.rgbCoeffs = c->rgbTable.p + 64;
            S.tex.ewaLut = c->ewaLut.p;
            c->noisePerm.Upload(GetSpectralData().noisePerm);  // procedural textures' Perlin noise
            S.tex.noisePerm = c->noisePerm.p;
            c->texBasis.Upload(tt.basis);
            S.tex.basis = c->texBasis.p;
            S.tex.nProgs = (int)tt.progs.size();
            S.tex.nLuts = (int)tt.images.size();
            S.camDiff = MakeCameraDiff(s);
            // a program k_texture's lean instantiation evaluates: one image leaf without EWA
            // (reflectance: the albedo RGB leaf; roughness: a float image or a constant)
            auto leanProg = [&](int p, bool spectrum) {
                if (p < 0) return true;
                const DeviceTexProgram &pg = tt.progs[p];
                if (spectrum && !pg.simple) return false;
                if (!spectrum && pg.n1 != 1) return false;
                const DeviceTexInstr &in = tt.instrs[pg.p1];
                const int op = in.op & 0xff;
                if (!spectrum && op != kT1FConst && op != kT1FImage) return false;
                return op == kT1FConst || s.textures[in.node].filter != kMipEWA;
            };
            for (const MaterialDesc &m : s.materials) {
                if (m.texReflectance >= 0 && !tt.progs[m.texReflectance].simple) c->texGeneral = true;
                if (m.texHair[4] >= 0) c->texGeneral = true;  // sigma_a from textured concentrations, per wavelength
                if (m.texReflectance >= 0 || m.texURough >= 0 || m.texDisp >= 0 || m.normalMap >= 0)
                    c->texTypeMask |= 1 << m.type;
                if (m.texDisp >= 0 && !leanProg(m.texDisp, false)) c->texFullMask |= 1 << m.type;
                if (!leanProg(m.texReflectance, true) || !leanProg(m.texURough, false) || !leanProg(m.texVRough, false))
                    c->texFullMask |= 1 << m.type;
            }
        }
    }
    S.nAreaLights = (int)s.areaLights.size();
    S.lightPrim = c->lightPrim.p;
    S.lightScale = c->lightScale.p;
    S.lightSpectrum = c->lightSpectrum.p;
    S.lightTwoSided = c->lightTwoSided.p;
    S.lightSpreadNorm = c->lightSpreadNorm.p;
    S.hasSpread = c->hasSpread ? 1 : 0;
    S.lightArea = c->lightArea.p;
    S.lights = c->lights.p;
    S.lightBitTrail = c->lightBitTrail.p;
    S.nInfinite = (int)s.infiniteLights.size();
    S.infSpectrum = c->infSpectrum.p;
    S.infScale = c->infScale.p;
    S.infDistant = c->infDistant.p;
    S.infImage = c->infImage.p;
    S.env = c->envLights.p;
    S.nEnv = (int)s.envLights.size();
    S.nDelta = (int)s.deltaLights.size();
    S.nPointSpot = s.nPointSpot;
    S.delta = c->deltaLights.p;
    S.deltaImg = c->deltaImg.p;
    S.nImageDelta = 0;
    for (auto &d : s.deltaLights) S.nImageDelta += d.type == kDeltaGonio || d.type == kDeltaProjection;
    {
        // DiffuseAreaLight emission images: per area light the offset of its image in lightImg
        // ({w, h} as int bits, then linear R, G, B [h][w][3]) or -1; their RGBIlluminantSpectrum
        // needs the RGB -> spectrum table (uploaded here when no texture did)
        std::vector<float> img;
        std::vector<int> offOf;
        for (const AreaLightImage &im : s.areaLightImages) {
            offOf.push_back((int)img.size());
            img.push_back(BitsToFloat((uint32_t)im.w));
            img.push_back(BitsToFloat((uint32_t)im.h));
            img.insert(img.end(), im.rgb.begin(), im.rgb.end());
        }
        std::vector<int> lo;
        S.nImageAreaLights = 0;
        for (const AreaLightDesc &l : s.areaLights) {
            lo.push_back(l.image >= 0 ? offOf[l.image] : -1);
            S.nImageAreaLights += l.image >= 0;
        }
        if (S.nImageAreaLights > 0) {
            c->lightImg.Upload(img);
            c->lightImgOff.Upload(lo);
            if (!S.tex.rgbZNodes) {
                c->rgbTable.Upload(RGBToSpectrumTableData());
                S.tex.rgbZNodes = c->rgbTable.p;
                S.tex.rgbCoeffs = c->rgbTable.p + 64;
            }
        }
        S.lightImg = S.nImageAreaLights ? c->lightImg.p : nullptr;
        S.lightImgOff = S.nImageAreaLights ? c->lightImgOff.p : nullptr;
    }
    S.uniformOrder = c->uniformOrder.p;
    S.sceneRadius = s.sceneRadius;
    S.uniformLightSampler = s.uniformLightSampler ? 1 : 0;
    S.lightNodes = c->lightNodes.p;
    S.nLightNodes = (int)s.lightNodes.size();
    S.dense = c->dense.p;
    S.nDense = (int)s.denseSpectra.size();
    S.sensor = c->sensor.p;
    S.sensor4 = (const float4 *)c->sensor4.p;
    S.imagingRatio = s.imagingRatio;
    S.maxComponentValue = s.maxComponentValue;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            S.cameraFromRaster[4 * i + j] = (float)s.camera.cameraFromRaster[i][j];
            S.renderFromCamera[4 * i + j] = (float)s.camera.renderFromCamera[i][j];
        }
    S.lensRadius = s.camera.lensRadius;
    S.options = s.options;
    S.focalDistance = s.camera.focalDistance;
    S.xres = s.xres;
    S.yres = s.yres;
    S.px0 = s.px0;
    S.px1 = s.px1;
    S.py0 = s.py0;
    S.py1 = s.py1;
    S.filterRadiusX = s.filterRadiusX;
    S.filterRadiusY = s.filterRadiusY;
    S.boxFilter = s.filterType == kFilterBox ? 1 : 0;
    S.filter = FilterParams{s.filterType, s.filterRadiusX, s.filterRadiusY, s.filterA, s.filterB};
    c->filterTab.Upload(s.filterTable.empty() ? std::vector<float>{0.f} : s.filterTable);
    S.filterTab = FilterTableView{s.filterNu, s.filterNv, c->filterTab.p};
    S.perm = c->perm.p;
    S.permOffset = c->permOffset.p;
    S.permNDigits = c->permNDigits.p;
    S.permBase = c->permBase.p;
    S.haltonDim = c->haltonDim.p;
    S.permByDepth = c->permByDepth.p;
    S.permDepthInfo = c->permDepthInfo.p;
    S.nDims = (int)s.permBase.size();
    for (int i = 0; i < 2; ++i) {
        S.baseScales[i] = s.haltonBaseScales[i];
        S.baseExponents[i] = s.haltonBaseExponents[i];
        S.multInverse[i] = s.haltonMultInverse[i];
    }
    {
        uint64_t s0 = (uint64_t)S.baseScales[0], s1 = (uint64_t)S.baseScales[1];
        // every pixel coordinate passed to the kernels is >= 0 (pixel bounds start at >= 0)
        S.haltonFast32 = s.px0 >= 0 && s.py0 >= 0 && s0 * s1 * (s0 + s1) < (1ull << 32) ? 1 : 0;
    }
    S.maxDepth = s.maxDepth;
    S.samplerType = s.samplerType;
    S.zs = ZSobolParams{s.zsLog2SamplesPerPixel, s.zsNBase4Digits, s.seed, (Randomize)s.zsRandomize};
    S.zsPerms = reinterpret_cast<const uint8_t(*)[4]>(c->zsPerms.p);
    S.sobolM1 = c->sobolM1.p;
    // IndependentSampler / StratifiedSampler / SobolSampler / PaddedSobolSampler (core.h GenericSampler)
    S.samp = SamplerDesc{s.samplerType, s.spp, s.seed, s.stratXs, s.stratYs, s.stratJitter,
                         (Randomize)s.zsRandomize, s.sobolLog2Scale, nullptr, nullptr, nullptr};
    if (s.samplerType == kSamplerSobol) {
        const SobolTableData &sob = SobolTables();
        c->sobol32.Upload(sob.m32);
        c->vdcSobol.Upload(sob.vdc);
        c->vdcSobolInv.Upload(sob.vdcInv);
        S.samp.sobol32 = c->sobol32.p;
        S.samp.vdc = c->vdcSobol.p;
        S.samp.vdcInv = c->vdcSobolInv.p;
    }
    {
        // k_shade_diffuse dynamic LDS: [beta*f 31x256 floats][sensor][light spectra][Halton
        // permutations of 7 dims][lights][light BVH][materials]
        ShadeLdsLayout &L = S.shadeLds;
        L = ShadeLdsLayout{};
        auto align16 = [](int v) { return (v + 15) & ~15; };
        int off = kNSpectrumSamples * 256 * (int)sizeof(float);
        L.sensor = off;
        off += kDenseN * 16;
        L.denseInLds = s.denseSpectra.size() <= 4 ? 1 : 0;
        L.dense = off;
        if (L.denseInLds) off = align16(off + (int)s.denseSpectra.size() * kDenseN * 4);
        L.lightsInLds = (s.areaLights.size() <= 64 && s.lightNodes.size() <= 127) ? 1 : 0;
        L.lights = off;
        L.lightNodes = off;
        if (L.lightsInLds) {
            off += (int)s.areaLights.size() * (int)sizeof(DeviceAreaLight);
            L.lightNodes = off;
            off = align16(off + (int)s.lightNodes.size() * (int)sizeof(DeviceLightNode));
        }
        L.matsInLds = s.materials.size() <= 256 ? 1 : 0;
        L.mats = off;
        L.matConst = off;
        if (L.matsInLds) {
            off += (int)s.materials.size() * 16;
            L.matConst = off;
            off = align16(off + (int)s.materials.size() * 4);
        }
        // the Halton permutations of the launch's 7 dimensions come last, so a launch asks for
        // the LDS its own depth's tables need (depth 0's prime bases are the smallest)
        int permEntries = 0;
        L.perm = off;
        for (int depth = 0; depth < s.maxDepth; ++depth) {
            int n = 0;
            for (int k = 0; k < 7; ++k) {
                int d = 6 + 7 * depth + k;
                if (d < (int)s.permBase.size()) n += (int)(s.permBase[d] * s.permNDigits[d]);
            }
            permEntries = std::max(permEntries, n);
            if (depth < kShadeLdsDepths) L.totalByDepth[depth] = align16(off + (n + 1) * 2);  // whole 4-byte words
        }
        L.permEntries = permEntries + 1;
        off = align16(off + (permEntries + 1) * 2);
        for (int depth = s.maxDepth; depth < kShadeLdsDepths; ++depth) L.totalByDepth[depth] = off;
        L.total = off;
        // conductor eta / k knots, searched per wavelength: the microfacet launches stage a
        // small set (up to one named-metal pair, 2 x 56 knots) after their depth's permutation
        // tables.  C3 (two 2-knot spectra): +2.7 %; C4's ten 56-knot spectra ran 1 % slower
        // from LDS than through L1, so larger sets stay in global memory.
        L.plCount = (int)c->plLambda.n;
        L.plInLds = ((S.matTypeMask >> kMatConductorT) & 1) && L.plCount <= 128 ? 1 : 0;
        if (L.total > 64 * 1024 && !c->volumetric) throw Error("shade kernel LDS layout exceeds 64 KB");
    }
    S.stackSize = c->bvh.maxStack;
    // |plane coordinate| bound per axis for the traversal's box-test margins (common.h
    // MakeCwRay): the scene bounds, widened by twice the extent for the quantised planes'
    // outward rounding (each lies within its node's grid of 255 steps of at most 2 ext / 255)
    for (int a = 0; a < 3; ++a) {
        const float lo = c->bvh.boundsMin[a], hi = c->bvh.boundsMax[a];
        const float ext = std::isfinite(hi - lo) && hi >= lo ? hi - lo : 0.f;
        S.bvhAbsMax[a] = std::isfinite(lo) && std::isfinite(hi) ? std::max(std::fabs(lo), std::fabs(hi)) + 2 * ext : 0.f;
        S.rayBinLo[a] = std::isfinite(lo) ? lo : 0.f;
        S.rayBinScale[a] = ext > 0 ? 8.f / ext : 0.f;
    }
    {
        // Node format.  A tree that fits the LDS cache whole (nodes + pre-rotated triangles:
        // Cornell) traverses wide nodes from LDS.  An HBM-resident tree traverses the 80-B
        // quantised nodes with kernels compiled for TraversalWaves(kTravQuant) = 6 waves per
        // SIMD: the traversal is bound by dependent-load latency, and the smaller node loads
        // (20 VGPRs instead of 60) buy the waves in flight (C4 k_closest -16 %).
        // PBRT_AMD_BVH=wide / compressed forces a format.
        const char *fmt = getenv("PBRT_AMD_BVH");
        const bool forceWide = fmt && strcmp(fmt, "wide") == 0, forceQuant = fmt && strcmp(fmt, "compressed") == 0;
        int maxLds = 0;
        HIPCHECK(hipDeviceGetAttribute(&maxLds, hipDeviceAttributeMaxSharedMemoryPerBlock, c->device));
        const size_t stackLds = (size_t)c->bvh.maxStack * 256 * sizeof(uint2);  // kBlock lanes
        const int nNodes = (int)c->bvh.nodes.size();
        // A traversal block's LDS = static (queue staging) + the group stack + the node /
        // triangle cache (top BVH8 nodes first, BFS order, then all triangles or none).  The
        // cache gets what the other two leave of the block's share of the CU at the mode's
        // occupancy (C4 wide: 10 KB + 18 KB of 40 KB -> 12 KB); a tree whose stack does not fit
        // the per-block limit is rejected here rather than failing at launch.
        auto layout = [&](bool compressed, int tm) {
            const size_t staticLds = std::max(SurfaceTraversalStaticLds(tm), VolTraversalStaticLds(tm));
            if (staticLds + stackLds > (size_t)maxLds)
                throw Error("BVH needs a " + std::to_string(c->bvh.maxStack) + "-entry traversal stack (" +
                            std::to_string(stackLds) + " B of LDS per block beside " + std::to_string(staticLds) +
                            " B static; the device allows " + std::to_string(maxLds) + ")");
            const size_t share =
                std::min<size_t>((size_t)maxLds, kLdsPerCU / TraversalBlocksCompiled(compressed ? 1 : 0) - 512);
            const size_t left = share > staticLds + stackLds ? share - staticLds - stackLds : 0;
            const int stride = 16 * LdsNodeStride(compressed);
            int budget = (int)std::min<size_t>(kSceneLdsBudget, left);
            S.compressed = compressed ? 1 : 0;
            S.ldsNodes = std::min(nNodes, budget / stride);
            budget -= S.ldsNodes * stride;
            // all or none, in three pre-rotated copies (one per ray permutation)
            S.ldsTris = (!compressed && S.ldsNodes == nNodes && nt * 3 * 48 <= budget) ? nt : 0;
        };
        layout(false, kTravWide);
        const bool allInLds = S.ldsTris > 0;
        if (forceQuant || (!forceWide && !allInLds)) layout(true, kTravQuant);
        else if (allInLds) layout(false, kTravLds);
        // ray binning before the closest hits of depth >= 1 when the tree lives in HBM (the
        // surface wavefront; PBRT_AMD_RAY_SORT=0/1 overrides)
        const char *rs = getenv("PBRT_AMD_RAY_SORT");
        c->rayBinning = !c->volumetric && (rs ? atoi(rs) != 0 : S.ldsTris == 0);
        const char *rk = getenv("PBRT_AMD_RAY_BIN_KEY");
        S.rayBinMode = rk ? std::max(0, std::min(4, atoi(rk))) : 0;
        const char *xg = getenv("PBRT_AMD_XCD_GROUPS");
        S.xcdGroups = xg ? std::max(0, atoi(xg)) : 0;  // measured neutral on C4 (k_closest 7434 vs 7410 us)
    }

    // the scene struct's device copy (DeviceScene::self)
    c->sceneSelf.Alloc(1);
    S.self = c->sceneSelf.p;
    HIPCHECK(hipMemcpy(c->sceneSelf.p, &S, sizeof(DeviceScene), hipMemcpyHostToDevice));

    // film
    size_t npix = (size_t)s.xres * s.yres;
    c->film.Alloc(4 * npix);
    HIPCHECK(hipMemset(c->film.p, 0, 4 * npix * sizeof(double)));
}

// floats: records 2 x (beta 31, ray 6, lambda0, rl, etaScale) = 80, hitB 2x4, shadowRay 6,
// shadowL 3, L 3, filterW 1 = 101; ints: records 2 x (flags, pixel, prevIdx), hitPrim 2,
// shadowPixel, matQ x 3 (per material type), escQ, emitQ, records 2 x sidx = 16
constexpr int kPathFloats = 101, kPathInts = 16;
// VolState: records 2 x (beta, r_u, r_l 93 + ray 6 + prev 12 + lambda0, etaScale 2) = 226,
// hitB 4, shadow ray 6 + Ld/r_u/r_l 93 + lambda0 = 100 floats; records 2 x (flags, pixel,
// depth, medium) = 8, hitPrim, 5 queues, shadow pixel + medium + flags = 17 ints
constexpr int kVolFloats = 330, kVolInts = 17;
static int64_t PathStateBytesPerPath(bool volumetric, bool dispersive, bool textured = false, bool texGeneral = false,
                                     bool mix = false, bool bump = false, bool sssTex = false) {
    return 4 * (kPathFloats + kPathInts) + (volumetric ? 4 * (kVolFloats + kVolInts) : 0) + (dispersive ? 16 : 0) +
           (textured ? 32 : 0) + (texGeneral ? 124 : 0) + (mix ? 8 : 0) + (bump ? 48 : 0) + (sssTex ? 248 : 0);
}

static void AllocPaths(pbrt_context *c, int64_t N) {
    if (N <= c->maxPaths) return;
    const int nf = kPathFloats, ni = kPathInts;
    // per-shard capacity: the fair share plus one 256-item chunk per producer kernel of a queue
    // (a producer's block b pushes into shard b % kShards and its grid is a multiple of kShards,
    // so each producer overshoots a shard's share by less than one chunk; up to kShards producers)
    const int64_t capS = ((N + kShards - 1) / kShards + 256 * kShards + 63) / 64 * 64;
    // record stride: the shards plus a trash area whose last slot takes the writes of a full
    // shard (ShardSlot), so an overflow never lands in another shard or past the arrays
    const int64_t NR = capS * kShards + kQueueTrash;
    // kernels index [k][NR] arrays with 32-bit k * NR for k <= 11 (spectral ones use size_t)
    if (NR > INT32_MAX / 12) throw Error("max_paths too large: " + std::to_string(N));
    // per pixel-sample arrays (L, filterW) use N; the rest NR (>= N)
    c->fState.Alloc((size_t)nf * NR);
    c->iState.Alloc((size_t)ni * NR + CounterIndex(c->desc.maxDepth + 3, 0, 0));
    if (c->S.dispersive) {
        c->dispL0.Alloc((size_t)3 * NR);
        c->dispTerm.Alloc((size_t)NR);
    }
    if (c->S.textured) {
        c->texCoef.Alloc((size_t)8 * NR);
        if (c->S.hasBump) c->texBump.Alloc((size_t)12 * NR);
        if (c->texGeneral) c->texR.Alloc((size_t)kNSpectrumSamples * NR);
        if (c->S.matSssTex) c->texS.Alloc((size_t)2 * kNSpectrumSamples * NR);
    }
    if (c->hasMix) c->hitMat.Alloc((size_t)2 * NR);
    if (c->rayBinning) {
        c->raySort.Alloc((size_t)2 * NR);
        c->rayBins.Alloc(2 * 4096);
        HIPCHECK(hipMemset(c->rayBins.p, 0, 2 * 4096 * sizeof(int)));
    }
    c->maxPaths = N;
    PathState &st = c->st;
    st.capS = (int)capS;
    st.NR = (int)NR;
    float *f = c->fState.p;
    auto take = [&](int k) {
        float *r = f;
        f += (size_t)k * NR;
        return r;
    };
    int *ip = c->iState.p;
    auto takei = [&](int k) {
        int *r = ip;
        ip += (size_t)k * NR;
        return r;
    };
    for (int b = 0; b < 2; ++b) {
        PathRecords &r = st.rec[b];
        r.beta = take(31);
        r.ray = take(6);
        r.lambda0 = take(1);
        r.rl = take(1);
        r.etaScale = take(1);
        r.flags = takei(1);
        r.pixel = takei(1);
        r.prevIdx = takei(1);
        r.sidx = reinterpret_cast<uint32_t *>(takei(1));
        st.hitB[b] = take(4);
        st.hitPrim[b] = takei(1);
    }
    st.shadowRay = take(6);
    st.shadowL = take(3);
    st.L = take(3);
    st.L0 = c->S.dispersive ? c->dispL0.p : nullptr;
    st.lamTerm = c->S.dispersive ? c->dispTerm.p : nullptr;
    st.filterW = take(1);
    st.shadowPixel = takei(1);
    for (int t = 0; t < kNumMatTypes; ++t) st.matQ[t] = takei(1);
    st.escQ = takei(1);
    st.emitQ = takei(1);
    st.counters = ip;
    st.texCoef = c->texCoef.p;
    st.texBump[0] = c->S.hasBump ? c->texBump.p : nullptr;
    st.texBump[1] = c->S.hasBump ? c->texBump.p + (size_t)6 * NR : nullptr;
    st.texR = c->texR.p;
    st.texS = c->texS.p;
    st.hitMat[0] = c->hasMix ? c->hitMat.p : nullptr;
    st.hitMat[1] = c->hasMix ? c->hitMat.p + NR : nullptr;
    st.raySort = c->rayBinning ? c->raySort.p : nullptr;
    st.rayBins = c->rayBinning ? c->rayBins.p : nullptr;
    if (c->volumetric) {
        const int vf = kVolFloats, vi = kVolInts;
        c->vfState.Alloc((size_t)vf * NR);
        c->viState.Alloc((size_t)vi * NR);
        float *g = c->vfState.p;
        int *gi = c->viState.p;
        auto tf = [&](int k) {
            float *r = g;
            g += (size_t)k * NR;
            return r;
        };
        auto ti = [&](int k) {
            int *r = gi;
            gi += (size_t)k * NR;
            return r;
        };
        VolState &v = c->vs;
        for (int b = 0; b < 2; ++b) {
            VolRecords &r = v.rec[b];
            r.beta = tf(31);
            r.ru = tf(31);
            r.rl = tf(31);
            r.ray = tf(6);
            r.prev = tf(12);
            r.lambda0 = tf(1);
            r.etaScale = tf(1);
            r.flags = ti(1);
            r.pixel = ti(1);
            r.depth = ti(1);
            r.medium = ti(1);
        }
        v.hitB = tf(4);
        v.shRay = tf(6);
        v.shLd = tf(31);
        v.shRu = tf(31);
        v.shRl = tf(31);
        v.shLambda0 = tf(1);
        v.hitPrim = ti(1);
        v.medQ = ti(1);
        v.surfQ = ti(1);
        v.scatQ = ti(1);
        v.ifaceQ = ti(1);
        v.escQ = ti(1);
        v.shPixel = ti(1);
        v.shMedium = ti(1);
        v.shFlags = ti(1);
        if (g - c->vfState.p > (ptrdiff_t)vf * NR || gi - c->viState.p > (ptrdiff_t)vi * NR)
            throw Error("VolState layout overflow");
        // the queue-integrity diagnostic's hole counter (PBRT_AMD_QUEUE_CHECK), this context's own
        if (!c->queueHoles.p) {
            c->queueHoles.Alloc(1);
            HIPCHECK(hipMemset(c->queueHoles.p, 0, sizeof(int)));
        }
        v.holes = c->queueHoles.p;
        v.sss = SssRecords{};
        if (!c->desc.sss.empty()) {
            c->sssF.Alloc((size_t)(2 * 31 + 3 + 3 + 2 + 3 + 1) * NR);
            c->sssI.Alloc((size_t)8 * NR);
            float *sf = c->sssF.p;
            int *si = c->sssI.p;
            auto sF = [&](int k) {
                float *r = sf;
                sf += (size_t)k * NR;
                return r;
            };
            auto sI = [&](int k) {
                int *r = si;
                si += (size_t)k * NR;
                return r;
            };
            SssRecords &q = v.sss;
            q.beta = sF(31);
            q.ru = sF(31);
            q.po = sF(3);
            q.ns = sF(3);
            q.lambda0 = sF(1);
            q.etaScale = sF(1);
            q.hitB = sF(3);
            q.resPdf = sF(1);
            q.mat = sI(1);
            q.pixel = sI(1);
            q.depth = sI(1);
            q.mIn = sI(1);
            q.mOut = sI(1);
            q.flags = sI(1);
            q.hitPrim = sI(1);
            q.src = sI(1);
        }
    }
    if (!c->devStats.p) {
        c->devStats.Alloc(kStatsSlots);
        HIPCHECK(hipMemset(c->devStats.p, 0, kStatsSlots * sizeof(unsigned long long)));
    }
    st.stats = c->devStats.p;
}

static void RecordEvent(pbrt_context *c, bool start) {
    if (start) {
        if (c->eventsUsed == (int)c->events.size()) {
            hipEvent_t a, b;
            HIPCHECK(hipEventCreate(&a));
            HIPCHECK(hipEventCreate(&b));
            c->events.push_back({a, b});
        }
        HIPCHECK(hipEventRecord(c->events[c->eventsUsed].first, c->stream));
    } else {
        HIPCHECK(hipEventRecord(c->events[c->eventsUsed].second, c->stream));
        ++c->eventsUsed;
    }
}

// Brackets one stage launch with events on the stream it runs on (profiling on); the pair is
// read back at pbrt_synchronize
struct StageTimer {
    pbrt_context *c;
    hipStream_t s;
    int slot = -1;
    StageTimer(pbrt_context *ctx, const char *name, hipStream_t stream) : c(ctx), s(stream) {
        if (!c->profiling) return;
        int stat = -1;
        for (size_t i = 0; i < c->stageStats.size(); ++i)
            if (c->stageStats[i].name == name) stat = (int)i;
        if (stat < 0) {
            c->stageStats.push_back({name});
            stat = (int)c->stageStats.size() - 1;
        }
        if (c->stageEventsUsed == (int)c->stageEvents.size()) {
            pbrt_context::StageEvents e{};
            HIPCHECK(hipEventCreate(&e.a));
            HIPCHECK(hipEventCreate(&e.b));
            c->stageEvents.push_back(e);
        }
        slot = c->stageEventsUsed++;
        c->stageEvents[slot].stat = stat;
        HIPCHECK(hipEventRecord(c->stageEvents[slot].a, s));
    }
    ~StageTimer() noexcept(false) {
        if (slot >= 0) HIPCHECK(hipEventRecord(c->stageEvents[slot].b, s));
    }
};

static void CollectStageEvents(pbrt_context *c) {
    for (int i = 0; i < c->stageEventsUsed; ++i) {
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, c->stageEvents[i].a, c->stageEvents[i].b));
        auto &st = c->stageStats[c->stageEvents[i].stat];
        st.mn = st.launches ? std::min(st.mn, (double)ms) : ms;
        st.mx = st.launches ? std::max(st.mx, (double)ms) : ms;
        st.sum += ms;
        ++st.launches;
    }
    c->stageEventsUsed = 0;
}

static void RenderImpl(pbrt_context *c, const pbrt_render_params *p) {
    HIPCHECK(hipSetDevice(c->device));
    const SceneDesc &s = c->desc;
    int width = s.px1 - s.px0;
    if (width <= 0) throw Error("empty pixel bounds");
    std::vector<int> rows;
    for (int i = 0; i < p->n_rows; ++i) {
        int y = p->rows[i];
        if (y < s.py0 || y >= s.py1) throw Error("row outside the film pixel bounds");
        rows.push_back(y);
    }
    if (rows.empty() || p->n_samples <= 0) return;
    int64_t maxPaths = c->maxPaths;
    // rows per chunk so that one sample of the chunk fits
    int64_t rowsPerChunk = std::max<int64_t>(1, maxPaths / width);
    if (rows != c->lastRows) {
        HIPCHECK(hipStreamSynchronize(c->stream));  // earlier passes may still read the row table
        c->rows.Alloc(rows.size());
        HIPCHECK(hipMemcpy(c->rows.p, rows.data(), rows.size() * sizeof(int), hipMemcpyHostToDevice));
        c->lastRows = rows;
    }
    const int countersBytes = CounterIndex(s.maxDepth + 3, 0, 0) * sizeof(int);
    for (size_t r0 = 0; r0 < rows.size(); r0 += rowsPerChunk) {
        int nRows = (int)std::min<int64_t>(rowsPerChunk, rows.size() - r0);
        int64_t P = (int64_t)nRows * width;
        int64_t samplesPerPass = std::max<int64_t>(1, std::min<int64_t>(p->n_samples, maxPaths / P));
        for (int s0 = 0; s0 < p->n_samples; s0 += (int)samplesPerPass) {
            int nS = (int)std::min<int64_t>(samplesPerPass, p->n_samples - s0);
            int64_t nActive = P * nS;
            PathState st = c->st;
            st.N = (int)c->maxPaths;
            st.P = (int)P;
            st.width = width;
            st.rows = c->rows.p + r0;
            st.firstSample = p->first_sample + s0;
            st.film = c->film.p;
            HIPCHECK(hipMemsetAsync(st.counters, 0, countersBytes, c->stream));
            if (c->volumetric) {
                // participating media: the volumetric wavefront (volpath.hip), same film update
                {
                    StageTimer t(c, "Generate camera rays (k_vcamera)", c->stream);
                    HIPCHECK(LaunchVolCamera(c->S, st, c->vs, (int)nActive, c->stream));
                }
                for (int wf = 0; wf <= s.maxDepth; ++wf) {
                    const bool timed = p->time_closest && r0 == 0 && s0 == 0;
                    if (timed) RecordEvent(c, true);
                    {
                        StageTimer t(c, "Tracing closest hit rays (k_vclosest)", c->stream);
                        HIPCHECK(LaunchVolClosest(c->S, st, c->vs, wf, (int)nActive, timed ? 1 : 0, c->stream));
                    }
                    if (timed) RecordEvent(c, false);
                    StageTimer t(c, "Media, surfaces, scattering and shadow rays (volpath iteration)", c->stream);
                    const hipError_t e = LaunchVolIteration(c->S, st, c->vs, wf, (int)nActive, c->stream);
                    if (e == hipErrorIllegalState)
                        throw Error("queue-integrity check (PBRT_AMD_QUEUE_CHECK): a volumetric stage counted queue slots "
                                    "it never wrote (iteration " + std::to_string(wf) + "); render aborted");
                    HIPCHECK(e);
                }
                HIPCHECK(LaunchQueueOverflowCheck(st, s.maxDepth + 2, c->stream));
                {
                    StageTimer t(c, "Update film (k_film)", c->stream);
                    HIPCHECK(LaunchFilm(c->S, st, nS, c->stream));
                }
                c->stats.passes++;
                c->stats.paths_per_pass = std::max<uint64_t>(c->stats.paths_per_pass, nActive);
                continue;
            }
            {
                StageTimer t(c, "Generate camera rays (k_camera)", c->stream);
                HIPCHECK(LaunchCamera(c->S, st, (int)nActive, c->stream));
            }
            // k_shade_diffuse<Lean>: Halton indices of this pass all below 2^24 (index <
            // (sample + 1) * stride, samplers.h:53-71), lights, light BVH and dense spectra in
            // LDS, no shading normals or uv, no point / spot / distant lights
            static const bool noLean = getenv("PBRT_AMD_NO_LEAN") != nullptr;
            const uint64_t haltonStride = (uint64_t)c->S.baseScales[0] * (uint64_t)c->S.baseScales[1];
            const bool lean = !noLean && c->S.samplerType == 0 &&
                              (uint64_t)(st.firstSample + nS) * haltonStride <= c->haltonIndexBound &&
                              c->S.shadeLds.lightsInLds && c->S.shadeLds.denseInLds && c->S.triShade == nullptr &&
                              c->S.nDelta == 0 && c->S.nEnv == 0 && c->S.nShapes == 0 && !c->S.textured && !c->hasMix &&
                              !c->S.hasSpread && c->S.nImageAreaLights == 0;
            for (int depth = 0; depth <= s.maxDepth; ++depth) {
                // closest-hit launches are event-timed in the first pass of a render only: the
                // passes are statistically identical and each event pair costs a queue gap
                const bool timed = p->time_closest && r0 == 0 && s0 == 0;
                const bool bin = c->rayBinning && depth > 0;
                if (bin) {
                    StageTimer t(c, "Bin rays by origin cell and direction octant (k_raybin_*)", c->stream);
                    HIPCHECK(LaunchRayBin(c->S, st, depth, (int)nActive, c->stream));
                }
                if (timed) RecordEvent(c, true);
                {
                    StageTimer t(c, "Tracing closest hit rays (k_closest)", c->stream);
                    HIPCHECK(LaunchClosest(c->S, st, depth, (int)nActive, timed ? 1 : 0, c->stream, bin));
                }
                if (timed) RecordEvent(c, false);
                if (bin) {
                    StageTimer t(c, "Enqueue binned hits in record order (k_classify)", c->stream);
                    HIPCHECK(LaunchClassify(c->S, st, depth, (int)nActive, c->stream));
                }
                // emission (escaped rays, emissive hits) on the side stream, beside the material
                // stage; the shadow stage and the next depth's closest hits wait for it
                static const bool emitSerial = getenv("PBRT_AMD_EMIT_SERIAL") != nullptr;
                const bool emit = (s.infiniteLights.size() || s.areaLights.size()) && !emitSerial;
                if (emitSerial) {
                    if (s.infiniteLights.size()) {
                        StageTimer t(c, "Handle escaped rays (k_escaped)", c->stream);
                        HIPCHECK(LaunchEscaped(c->S, st, depth, (int)nActive, c->stream));
                    }
                    if (s.areaLights.size()) {
                        StageTimer t(c, "Handle emitters hit by indirect rays (k_emissive)", c->stream);
                        HIPCHECK(LaunchEmissive(c->S, st, depth, (int)nActive, c->stream));
                    }
                }
                if (emit) {
                    HIPCHECK(hipEventRecord(c->eClosest[depth], c->stream));
                    HIPCHECK(hipStreamWaitEvent(c->sideStream, c->eClosest[depth], 0));
                    if (s.infiniteLights.size()) {
                        StageTimer t(c, "Handle escaped rays (k_escaped)", c->sideStream);
                        HIPCHECK(LaunchEscaped(c->S, st, depth, (int)nActive, c->sideStream));
                    }
                    if (s.areaLights.size()) {
                        StageTimer t(c, "Handle emitters hit by indirect rays (k_emissive)", c->sideStream);
                        HIPCHECK(LaunchEmissive(c->S, st, depth, (int)nActive, c->sideStream));
                    }
                    HIPCHECK(hipEventRecord(c->eEmit[depth], c->sideStream));
                }
                if (depth == s.maxDepth) {
                    if (emit) HIPCHECK(hipStreamWaitEvent(c->stream, c->eEmit[depth], 0));
                    break;
                }
                // EvaluateMaterialsAndBSDFs: one launch per material type present (surfscatter.cpp:39-55),
                // preceded by that type's texture stage when some material of it is textured
                for (int t = 0; t < kNumMatTypes; ++t)
                    if (c->texTypeMask & (1 << t)) {
                        StageTimer tm(c, "Evaluate textures (k_texture)", c->stream);
                        HIPCHECK(LaunchTexture(c->S, st, depth, t, (c->texFullMask >> t) & 1, (int)nActive, c->stream));
                    }
                if (c->S.matTypeMask & (1 << kMatDiffuseT)) {
                    StageTimer t(c, "Evaluate materials/BSDFs for DiffuseMaterial (k_shade_diffuse)", c->stream);
                    HIPCHECK(LaunchShadeDiffuse(c->S, st, depth, (int)nActive, lean, c->stream));
                }
                for (int t = kMatDielectricT; t < kNumMatTypes; ++t)
                    if (c->S.matTypeMask & (1 << t)) {
                        StageTimer tm(c, t == kMatDielectricT ? "Evaluate materials/BSDFs for DielectricMaterial (k_shade_microfacet)"
                                                             : "Evaluate materials/BSDFs for ConductorMaterial (k_shade_microfacet)",
                                      c->stream);
                        HIPCHECK(LaunchShadeMicrofacet(c->S, st, depth, t, (int)nActive, c->stream));
                    }
                if (emit) HIPCHECK(hipStreamWaitEvent(c->stream, c->eEmit[depth], 0));
                {
                    StageTimer t(c, "Tracing shadow rays (k_shadow)", c->stream);
                    HIPCHECK(LaunchShadow(c->S, st, depth, (int)nActive, c->stream));
                }
            }
            HIPCHECK(LaunchQueueOverflowCheck(st, s.maxDepth + 2, c->stream));
            {
                StageTimer t(c, "Update film (k_film)", c->stream);
                HIPCHECK(LaunchFilm(c->S, st, nS, c->stream));
            }
            c->stats.passes++;
            c->stats.paths_per_pass = std::max<uint64_t>(c->stats.paths_per_pass, nActive);
        }
    }
}

extern "C" {

const char *pbrt_last_error(void) { return g_lastError.c_str(); }

int pbrt_set_data_dir(const char *dir) {
    SetDataDirectory(dir ? dir : "");
    return 0;
}

static std::map<std::string, std::string> ParseOverrides(const char *ov) {
    std::map<std::string, std::string> m;
    if (!ov) return m;
    std::stringstream ss(ov);
    std::string item;
    while (std::getline(ss, item, ';')) {
        auto eq = item.find('=');
        if (eq == std::string::npos) continue;
        m[item.substr(0, eq)] = item.substr(eq + 1);
    }
    return m;
}

int pbrt_scene_load(const char *path, const char *overrides, pbrt_scene **out) {
    try {
        auto s = std::make_unique<pbrt_scene>();
        s->desc = LoadPbrtFile(path, ParseOverrides(overrides));
        s->Flatten();
        *out = s.release();
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_scene_load_string(const char *text, const char *base_dir, const char *overrides, pbrt_scene **out) {
    try {
        auto s = std::make_unique<pbrt_scene>();
        s->desc = LoadPbrtString(text, base_dir ? base_dir : "", ParseOverrides(overrides));
        s->Flatten();
        *out = s.release();
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

void pbrt_scene_free(pbrt_scene *scene) { delete scene; }

int pbrt_scene_get_info(const pbrt_scene *scene, pbrt_scene_info *info) {
    if (!scene || !info) return Fail("null argument");
    const SceneDesc &s = scene->desc;
    info->xres = s.xres;
    info->yres = s.yres;
    info->px0 = s.px0;
    info->px1 = s.px1;
    info->py0 = s.py0;
    info->py1 = s.py1;
    info->spp = s.spp;
    info->seed = s.seed;
    info->max_depth = s.maxDepth;
    info->n_triangles = (int)s.tris.size();
    info->n_vertices = (int)s.verts.size();
    info->n_materials = (int)s.materials.size();
    info->n_area_lights = (int)s.areaLights.size();
    info->n_infinite_lights = (int)s.infiniteLights.size();
    info->n_light_nodes = (int)s.lightNodes.size();
    info->uniform_light_sampler = s.uniformLightSampler;
    info->filter_radius_x = s.filterRadiusX;
    info->filter_radius_y = s.filterRadiusY;
    return 0;
}

int pbrt_scene_get_flat(const pbrt_scene *scene, pbrt_scene_flat *f) {
    if (!scene || !f) return Fail("null argument");
    const SceneDesc &s = scene->desc;
    memset(f, 0, sizeof(*f));
    f->n_vertices = (int)s.verts.size();
    f->n_triangles = (int)s.tris.size();
    f->n_materials = (int)s.materials.size();
    f->n_area_lights = (int)s.areaLights.size();
    f->n_infinite_lights = (int)s.infiniteLights.size();
    f->n_spectra = (int)s.denseSpectra.size();
    f->vertices = scene->verts.data();
    f->triangles = scene->tris.data();
    f->tri_material = s.triMaterial.data();
    f->tri_light = s.triLight.data();
    f->tri_flip = s.triFlip.data();
    f->material_coeffs = scene->matCoeffs.data();
    f->material_constant = scene->matConstant.data();
    f->light_prim = scene->lightPrim.data();
    f->light_scale = scene->lightScale.data();
    f->light_spectrum = scene->lightSpectrum.data();
    f->light_two_sided = scene->lightTwoSided.data();
    f->light_spread = scene->lightSpread.data();
    f->light_image = scene->lightImage.data();
    f->area_images = scene->areaImages.data();
    f->inf_spectrum = scene->infSpectrum.data();
    f->inf_scale = scene->infScale.data();
    f->n_delta_lights = (int)s.deltaLights.size();
    f->n_point_spot = s.nPointSpot;
    f->delta_lights = scene->deltaLights.data();
    f->delta_images = scene->deltaImages.data();
    f->inf_distant = scene->infDistant.data();
    f->n_env = (int)scene->desc.envLights.size();
    f->inf_image = scene->infImage.data();
    f->env_info = scene->envInfo.data();
    f->env_xform = scene->envXform.data();
    f->env_offset = scene->envOffset.data();
    f->env_rgb = scene->envRgb.data();
    f->n_shapes = (int)scene->desc.shapes.size();
    f->shape_info = scene->shapeInfo.data();
    f->shape_params = scene->shapeParams.data();
    f->shape_normals = scene->shapeNormals.data();
    f->prim_alpha = scene->primAlpha.empty() ? nullptr : scene->primAlpha.data();
    f->uniform_order = scene->uniformOrder.data();
    f->scene_radius = s.sceneRadius;
    {
        const TexTables &t = scene->tex;
        f->n_tex_nodes = (int)s.textures.size();
        f->n_images = (int)s.images.size();
        f->tex_node_info = t.nodeInfo.data();
        f->tex_node_params = t.nodeParams.data();
        f->noise_perm = GetSpectralData().noisePerm.data();
        f->tex_node_spec = t.specFlat.data();
        f->tex_basis = t.basis.data();
        f->image_info = t.imageInfo.data();
        f->image_levels = t.levelInfo.data();
        f->image_data = t.data.data();
        f->image_luts = t.luts.data();
        f->image_raw_info = t.rawInfo.data();
        f->image_raw_gamma = t.rawGamma.data();
        f->image_raw_offset = t.rawOffset.data();
        f->image_raw_data = t.rawData.data();
        f->material_tex = t.matTexNode.data();
        f->material_mix = t.matMixNode.data();
        f->material_bump = t.matBumpNode.data();
        f->material_hair_tex = t.anyHairTex ? t.matHairNode.data() : nullptr;
        f->material_sss_tex = t.anySssTex ? t.matSssNode.data() : nullptr;
        for (int k = 0; k < 12; ++k) f->camera_from_render[k] = s.cameraFromRender[k];
        for (int k = 0; k < 3; ++k) {
            f->camera_min_diff[k] = s.minPosDx[k];
            f->camera_min_diff[3 + k] = s.minPosDy[k];
            f->camera_min_diff[6 + k] = s.minDirDx[k];
            f->camera_min_diff[9 + k] = s.minDirDy[k];
        }
    }
    f->dense_spectra = scene->dense.data();
    f->sensor_xyz = scene->sensor.data();
    f->imaging_ratio = s.imagingRatio;
    f->max_component_value = s.maxComponentValue;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) f->xyz_from_sensor_rgb[3 * i + j] = s.xyzFromSensorRGB[i][j];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            f->camera_from_raster[4 * i + j] = (float)s.camera.cameraFromRaster[i][j];
            f->render_from_camera[4 * i + j] = (float)s.camera.renderFromCamera[i][j];
        }
    f->lens_radius = s.camera.lensRadius;
    f->focal_distance = s.camera.focalDistance;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) f->output_rgb_from_sensor_rgb[3 * i + j] = s.outputRGBFromSensorRGB[i][j];
    f->n_light_nodes = (int)s.lightNodes.size();
    f->light_node_bounds = scene->nodeBounds.data();
    f->light_node_info = scene->nodeInfo.data();
    f->light_bit_trail = s.lightBitTrail.data();
    for (int i = 0; i < 2; ++i) {
        f->halton_base_scales[i] = s.haltonBaseScales[i];
        f->halton_base_exponents[i] = s.haltonBaseExponents[i];
        f->halton_mult_inverse[i] = s.haltonMultInverse[i];
    }
    f->n_dims = (int)s.permBase.size();
    f->perm_table = s.permTable.data();
    f->perm_offset = s.permOffset.data();
    f->perm_ndigits = s.permNDigits.data();
    f->perm_base = s.permBase.data();
    f->sampler_type = s.samplerType;
    f->zs_randomize = s.zsRandomize;
    f->zs_log2_spp = s.zsLog2SamplesPerPixel;
    f->zs_nbase4_digits = s.zsNBase4Digits;
    f->strat_xsamples = s.stratXs;
    f->strat_ysamples = s.stratYs;
    f->strat_jitter = s.stratJitter;
    f->sobol_log2_scale = s.sobolLog2Scale;
    if (s.samplerType == kSamplerSobol) {
        const SobolTableData &sob = SobolTables();
        f->sobol_matrices32 = sob.m32.data();
        f->vdc_sobol = sob.vdc.data();
        f->vdc_sobol_inv = sob.vdcInv.data();
    }
    f->material_type = scene->matType.data();
    f->n_sss = (int)s.sss.size();
    f->material_sss = s.sss.empty() ? nullptr : scene->matSss.data();
    f->sss_params = s.sss.empty() ? nullptr : scene->sssParams.data();
    f->sss_tables = s.sss.empty() ? nullptr : scene->sssTables.data();
    f->vertex_s = s.vertS.empty() ? nullptr : &s.vertS[0].x;
    f->n_vertex_s = (int)s.vertS.size();
    f->env_portal = scene->envPortal.empty() ? nullptr : scene->envPortal.data();
    scene->measuredFiles.clear();
    for (const MeasuredDesc &b : s.measured) scene->measuredFiles.push_back(b.path.c_str());
    f->options = s.options;
    f->n_measured = (int)s.measured.size();
    f->measured_files = s.measured.empty() ? nullptr : scene->measuredFiles.data();
    f->dims_per_depth = s.sss.empty() ? 7 : 10;
    f->material_params = scene->matParams.data();
    f->material_layer = scene->matLayer.data();
    f->material_spectra = scene->matSpectra.data();
    f->n_pl_spectra = (int)s.plSpectra.size();
    f->pl_offsets = scene->plOffsets.data();
    f->pl_lambda = scene->plLambda.data();
    f->pl_value = scene->plValue.data();
    f->regularize = s.regularize ? 1 : 0;
    static_assert(sizeof(V3) == 12, "vertex normals are handed out as float[3] arrays");
    f->vertex_normals = s.vertN.empty() ? nullptr : &s.vertN[0].x;
    f->vertex_uv = s.vertUV.empty() ? nullptr : s.vertUV[0].data();
    f->tri_shading = s.triShade.data();
    f->n_media = (int)s.media.size();
    f->camera_medium = s.cameraMedium;
    f->medium_info = scene->mediumInfo.data();
    f->medium_params = scene->mediumParams.data();
    f->medium_values = scene->mediumValues.data();
    f->tri_medium = s.triMedium.empty() ? nullptr : s.triMedium[0].data();
    f->filter_type = s.filterType;
    f->filter_a = s.filterA;
    f->filter_b = s.filterB;
    return 0;
}

int pbrt_device_count(int *count) {
    hipError_t e = hipGetDeviceCount(count);
    if (e != hipSuccess) {
        *count = 0;
        return Fail(std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    return 0;
}

int pbrt_context_create(const pbrt_scene *scene, int device, int64_t maxPaths, pbrt_context **out) {
    try {
        if (!scene) return Fail("null scene");
        auto c = std::make_unique<pbrt_context>();
        c->device = device;
        c->desc = scene->desc;
        BuildDevice(c.get());
        if (maxPaths <= 0) {
            // default: every sample of the film in one pass (one launch per stage and depth for
            // the whole image -- per-pass launch, tail and LDS-staging costs paid once), up to
            // 64 Mi paths (~31 GB of surface path state; 16 Mi with the media records, ~23 GB)
            const SceneDesc &d = c->desc;
            const int64_t all = (int64_t)(d.px1 - d.px0) * (d.py1 - d.py0) * std::max(d.spp, 1);
            maxPaths = std::min<int64_t>(all, c->volumetric ? (1 << 24) : (1 << 26));
            // ... and within 3/4 of the device memory still free (several contexts per GPU,
            // smaller cards): path-state bytes per path from AllocPaths' layout
            size_t freeB = 0, totalB = 0;
            HIPCHECK(hipMemGetInfo(&freeB, &totalB));
            const int64_t perPath = PathStateBytesPerPath(c->volumetric, c->S.dispersive, c->S.textured, c->texGeneral, c->hasMix,
                                                       c->S.hasBump, c->S.matSssTex != nullptr) +
                                    (c->rayBinning ? 32 : 0);
            const int64_t fit = (int64_t)(freeB / 4 * 3) / perPath - kShards * 320;
            if (fit < 4096) throw Error("not enough free device memory for path state");
            maxPaths = std::min<int64_t>(maxPaths, fit);
        }
        AllocPaths(c.get(), maxPaths);
        *out = c.release();
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

void pbrt_context_free(pbrt_context *ctx) { delete ctx; }

int pbrt_render(pbrt_context *ctx, const pbrt_render_params *params) {
    try {
        if (!ctx || !params) return Fail("null argument");
        RenderImpl(ctx, params);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_synchronize(pbrt_context *ctx) {
    try {
        if (!ctx) return Fail("null context");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        for (int i = 0; i < ctx->eventsUsed; ++i) {
            float ms = 0;
            HIPCHECK(hipEventElapsedTime(&ms, ctx->events[i].first, ctx->events[i].second));
            ctx->stats.closest_ms += ms;
            ctx->stats.closest_launches++;
        }
        ctx->eventsUsed = 0;
        CollectStageEvents(ctx);
        unsigned long long ds[8];
        HIPCHECK(hipMemcpy(ds, ctx->devStats.p, sizeof ds, hipMemcpyDeviceToHost));
        if (ds[kStatQueueOverflow]) {
            HIPCHECK(hipMemset(ctx->devStats.p + kStatQueueOverflow, 0, sizeof(unsigned long long)));
            return Fail("queue overflow: " + std::to_string(ds[kStatQueueOverflow]) +
                        " queue shard(s) exceeded their capacity; the film of this render is invalid");
        }
        ctx->stats.camera_rays = ds[0];
        ctx->stats.closest_rays = ds[1];
        ctx->stats.shadow_rays = ds[2];
        ctx->stats.timed_closest_rays = ds[3];
        {
            const DeviceScene &S = ctx->S;
            const uint64_t nodeB = S.compressed ? sizeof(BVH8QNode) : sizeof(BVH8Node);
            const uint64_t nNodes = S.compressed ? ctx->qnodes.n / S.qStride : ctx->nodes.n;
            ctx->stats.bvh_hbm_node_bytes = nNodes > (uint64_t)S.ldsNodes ? (nNodes - S.ldsNodes) * nodeB : 0;
            ctx->stats.bvh_hbm_tri_bytes = S.ldsTris > 0 ? 0 : (uint64_t)ctx->triVerts.n / S.triStride * 3 * sizeof(float);
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_set_kernel_profiling(pbrt_context *ctx, int enable) {
    try {
        if (!ctx) return Fail("null argument");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        HIPCHECK(hipStreamSynchronize(ctx->sideStream));
        CollectStageEvents(ctx);
        ctx->profiling = enable != 0;
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_get_kernel_stats(pbrt_context *ctx, pbrt_kernel_stat *out, int max_stats, int *n_stats) {
    if (!ctx || !n_stats || (max_stats > 0 && !out)) return Fail("null argument");
    const int n = (int)ctx->stageStats.size();
    *n_stats = n;
    for (int i = 0; i < std::min(n, max_stats); ++i) {
        const auto &st = ctx->stageStats[i];
        pbrt_kernel_stat &o = out[i];
        memset(&o, 0, sizeof o);
        strncpy(o.description, st.name.c_str(), sizeof o.description - 1);
        o.launches = st.launches;
        o.total_ms = st.sum;
        o.min_ms = st.mn;
        o.max_ms = st.mx;
    }
    return 0;
}

int pbrt_get_stats(pbrt_context *ctx, pbrt_render_stats *stats) {
    if (!ctx || !stats) return Fail("null argument");
    *stats = ctx->stats;
    return 0;
}

int pbrt_reset_stats(pbrt_context *ctx) {
    try {
        if (!ctx) return Fail("null context");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        HIPCHECK(hipMemset(ctx->devStats.p, 0, kStatsSlots * sizeof(unsigned long long)));
        ctx->stats = pbrt_render_stats{};
        ctx->eventsUsed = 0;
        ctx->stageEventsUsed = 0;
        ctx->stageStats.clear();
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_film_clear(pbrt_context *ctx) {
    try {
        if (!ctx) return Fail("null context");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipMemsetAsync(ctx->film.p, 0, ctx->film.n * sizeof(double), ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_film_device_ptr(pbrt_context *ctx, double **film, size_t *n) {
    if (!ctx || !film || !n) return Fail("null argument");
    *film = ctx->film.p;
    *n = ctx->film.n;
    return 0;
}

int pbrt_film_read(pbrt_context *ctx, double *out) {
    try {
        if (!ctx || !out) return Fail("null argument");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        HIPCHECK(hipMemcpy(out, ctx->film.p, ctx->film.n * sizeof(double), hipMemcpyDeviceToHost));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_film_get_rgb(pbrt_context *ctx, float *rgb) {
    try {
        if (!ctx || !rgb) return Fail("null argument");
        std::vector<double> f(ctx->film.n);
        if (pbrt_film_read(ctx, f.data())) return 1;
        size_t npix = (size_t)ctx->desc.xres * ctx->desc.yres;
        const auto &m = ctx->desc.outputRGBFromSensorRGB;
        for (size_t i = 0; i < npix; ++i) {
            // RGBFilm::GetPixelRGB (film.h:261-277)
            float c[3] = {(float)f[i], (float)f[npix + i], (float)f[2 * npix + i]};
            float w = (float)f[3 * npix + i];
            if (w != 0)
                for (float &v : c) v /= w;
            for (int k = 0; k < 3; ++k)
                rgb[3 * i + k] = (float)(m[k][0] * c[0] + m[k][1] * c[1] + m[k][2] * c[2]);
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_film_write_image(pbrt_context *ctx, const char *path, int writeFP16) {
    try {
        if (!ctx || !path) return Fail("null argument");
        // RGBFilm::GetImage (film.cpp) covers pixelBounds only; Image::WriteEXR records it as
        // the dataWindow of the full-resolution displayWindow
        const SceneDesc &d = ctx->desc;
        std::vector<float> rgb((size_t)d.xres * d.yres * 3);
        if (pbrt_film_get_rgb(ctx, rgb.data())) return 1;
        const int w = d.px1 - d.px0, h = d.py1 - d.py0;
        std::vector<float> crop((size_t)w * h * 3);
        for (int y = 0; y < h; ++y)
            std::copy(rgb.begin() + ((size_t)(d.py0 + y) * d.xres + d.px0) * 3,
                      rgb.begin() + ((size_t)(d.py0 + y) * d.xres + d.px0 + w) * 3, crop.begin() + (size_t)y * w * 3);
        const int window[4] = {d.px0, d.py0, d.xres, d.yres};
        const float *chroma = nullptr;
        float chroma8[8];
        if (d.filmColorSpace != kColorSpaceSRGB) {
            const ColorSpaceDesc &cs = GetColorSpace(d.filmColorSpace);
            const std::string p(path);
            const std::string ext = p.size() >= 4 ? p.substr(p.size() - 4) : p;
            if (ext == ".exr" || ext == ".EXR") {
                // Image::WriteEXR keeps the film's colour space and records its chromaticities
                std::copy(cs.prim, cs.prim + 6, chroma8);
                chroma8[6] = cs.w[0], chroma8[7] = cs.w[1];
                chroma = chroma8;
            } else {
                // Image::Write (util/image.cpp:989-1005): PNG / PFM pixels are converted to sRGB by
                // ConvertRGBColorSpace(film, sRGB) = sRGB.RGBFromXYZ * film.XYZFromRGB, Mul<RGB>
                float m[3][3];
                MulCompensated3(GetColorSpace(kColorSpaceSRGB).rgbFromXYZf, cs.xyzFromRGBf, m);
                for (size_t q = 0; q < (size_t)w * h; ++q) {
                    float *c = &crop[3 * q];
                    float o[3];
                    for (int i = 0; i < 3; ++i) {
                        o[i] = 0;
                        for (int j = 0; j < 3; ++j) o[i] += m[i][j] * c[j];
                    }
                    std::copy(o, o + 3, c);
                }
            }
        }
        WriteImage(path, crop.data(), w, h, writeFP16 != 0, window, chroma);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_image_read_size(const char *path, int *width, int *height) {
    try {
        Image im = ReadImage(path);
        *width = im.width;
        *height = im.height;
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_image_read(const char *path, float *rgb, int width, int height) {
    try {
        Image im = ReadImage(path);
        if (im.width != width || im.height != height) return Fail(std::string(path) + ": resolution mismatch");
        std::copy(im.rgb.begin(), im.rgb.end(), rgb);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_image_write(const char *path, const float *rgb, int width, int height, int writeFP16) {
    try {
        WriteImage(path, rgb, width, height, writeFP16 != 0);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_image_error(const float *image, const float *reference, int width, int height, const char *metric,
                     double *error3) {
    try {
        const std::string m = metric ? metric : "MSE";
        ErrorMetric em;
        if (m == "MAE") em = ErrorMetric::MAE;
        else if (m == "MSE") em = ErrorMetric::MSE;
        else if (m == "MRSE") em = ErrorMetric::MRSE;
        else if (m == "FLIP") em = ErrorMetric::FLIP;
        else return Fail("--metric must be \"MAE\", \"MSE\", \"MRSE\", or \"FLIP\"");
        const auto e = ImageError(image, reference, width, height, em);
        for (int c = 0; c < 3; ++c) error3[c] = e[c];
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_image_flip(const float *image, const float *reference, int width, int height, float *error_map) {
    try {
        if (!image || !reference || !error_map || width <= 0 || height <= 0) return Fail("bad arguments");
        const std::vector<float> m = FlipErrorMap(image, reference, width, height);
        std::copy(m.begin(), m.end(), error_map);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_intersect(pbrt_context *ctx, const float *rays, int n, int anyHit, int32_t *prim, float *hit) {
    try {
        if (!ctx || n < 0 || (n > 0 && (!rays || !prim || !hit))) return Fail("bad arguments");
        HIPCHECK(hipSetDevice(ctx->device));
        if (n == 0) return 0;
        if ((int64_t)n * 7 > INT32_MAX) return Fail("ray batch too large");
        // asynchronous on the context stream; the kernel writes the scene's triangle numbering
        HIPCHECK(LaunchIntersectBatch(ctx->S, rays, n, anyHit, prim, hit, ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_intersect_one_random(pbrt_context *ctx, const float *segs, const int32_t *materials, int n, int32_t *prim,
                              float *hit, float *pdf) {
    try {
        if (!ctx || n < 0 || (n > 0 && (!segs || !materials || !prim || !hit || !pdf))) return Fail("bad arguments");
        HIPCHECK(hipSetDevice(ctx->device));
        if (n == 0) return 0;
        if ((int64_t)n * 6 > INT32_MAX) return Fail("segment batch too large");
        HIPCHECK(LaunchIntersectOneRandom(ctx->S, segs, materials, n, prim, hit, pdf, ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_intersect_tr(pbrt_context *ctx, const float *rays, const int32_t *medium, const float *lambda0, int n,
                      float *out) {
    try {
        if (!ctx || n < 0 || (n > 0 && (!rays || !lambda0 || !out))) return Fail("bad arguments");
        if (n == 0) return 0;
        if ((int64_t)n * 93 > INT32_MAX) return Fail("ray batch too large");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(LaunchIntersectTr(ctx->S, rays, medium, lambda0, n, out, ctx->stream));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_check_rn_math(int device, uint64_t seed, int64_t n, int64_t *mismatches, float *examples96) {
    try {
        if (!mismatches || n <= 0) return Fail("bad arguments");
        HIPCHECK(hipSetDevice(device));
        const int blocks = 4096, perThread = (int)std::max<int64_t>(1, n / ((int64_t)blocks * 256));
        unsigned long long *bad = nullptr;
        const size_t bytes = (2 + 48 + 3) * sizeof(unsigned long long);
        HIPCHECK(hipMalloc(&bad, bytes));
        HIPCHECK(hipMemset(bad, 0, bytes));
        HIPCHECK(LaunchCheckRNMath(seed, blocks, perThread, bad, nullptr));
        std::vector<unsigned long long> h(2 + 48 + 3);
        HIPCHECK(hipMemcpy(h.data(), bad, bytes, hipMemcpyDeviceToHost));
        HIPCHECK(hipFree(bad));
        *mismatches = (int64_t)(h[0] + h[50] + h[51] + h[52]);
        if (examples96) memcpy(examples96, h.data() + 2, 96 * sizeof(float));
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_catmull_rom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                           const float *cdf, const float *x, int n, float *out) {
    if (!nodes1 || !x || !out || n < 0 || n1 < 2 || (op == 3 && (!nodes2 || n2 < 2 || !values || !cdf)) ||
        (op == 1 && !values) || (op != 0 && op != 1 && op != 3))
        return Fail("pbrt_debug_catmull_rom: bad arguments");
    for (int i = 0; i < n; ++i) {
        if (op == 0) {
            int off = 0;
            float w[4] = {0, 0, 0, 0};
            const bool ok = CatmullRomWeights(nodes1, n1, x[i], &off, w);
            const float r[6] = {ok ? 1.f : 0.f, (float)(ok ? off : 0), w[0], w[1], w[2], w[3]};
            std::copy(r, r + 6, out + 6 * i);
        } else if (op == 1) {
            out[i] = InvertCatmullRom(nodes1, values, n1, x[i]);
        } else {
            out[i] = SampleCatmullRom2D(nodes1, n1, nodes2, n2, values, cdf, x[2 * i], x[2 * i + 1]);
        }
    }
    return 0;
}

int pbrt_debug_catmull_rom_gpu(int device, int op, const float *nodes1, int n1, const float *nodes2, int n2,
                               const float *values, const float *cdf, const float *x, int n, float *out) {
    try {
        if (!nodes1 || !x || !out || n < 0 || n1 < 2 || (op == 3 && (!nodes2 || n2 < 2 || !values || !cdf)) ||
            (op == 1 && !values) || (op != 0 && op != 1 && op != 3))
            return Fail("pbrt_debug_catmull_rom_gpu: bad arguments");
        HIPCHECK(hipSetDevice(device));
        DevBuf<float> dn1, dn2, dv, dc, dx, dout;
        dn1.Upload(std::vector<float>(nodes1, nodes1 + n1));
        dn2.Upload(op == 3 ? std::vector<float>(nodes2, nodes2 + n2) : std::vector<float>(1, 0.f));
        // values: [n1][n2] for sample2d, [n1] for invert; cdf [n1][n2]
        const size_t nv = op == 3 ? (size_t)n1 * n2 : (op == 1 ? (size_t)n1 : 1);
        dv.Upload(values ? std::vector<float>(values, values + nv) : std::vector<float>(1, 0.f));
        dc.Upload(op == 3 ? std::vector<float>(cdf, cdf + (size_t)n1 * n2) : std::vector<float>(1, 0.f));
        const size_t nx = op == 3 ? 2 * (size_t)n : (size_t)n;
        dx.Upload(std::vector<float>(x, x + std::max<size_t>(nx, 1)));
        const size_t no = op == 0 ? 6 * (size_t)n : (size_t)n;
        dout.Alloc(std::max<size_t>(no, 1));
        if (n > 0) {
            HIPCHECK(LaunchCatmullRom(op, dn1.p, n1, dn2.p, n2, dv.p, dc.p, dx.p, n, dout.p, nullptr));
            HIPCHECK(hipMemcpy(out, dout.p, no * sizeof(float), hipMemcpyDeviceToHost));
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int64_t pbrt_debug_halton_fastpath_mismatches(const pbrt_scene *scene, int dim, uint32_t a0, uint32_t a1,
                                              uint32_t step) {
    if (!scene || step == 0 || a1 > (1u << 24)) return -1;
    const SceneDesc &s = scene->desc;
    if (dim < 0 || dim >= (int)s.permBase.size()) return -1;
    HaltonDimDesc d = MakeHaltonDimDesc(s.permBase[dim], s.permNDigits[dim], s.permOffset[dim]);
    const uint16_t *perm = s.permTable.data() + d.permOffset;
    HaltonDimTail(&d, perm);
    int64_t bad = 0;
    for (uint64_t a = a0; a < a1; a += step) {
        // the shade stage's form for bases >= 17 (a < 2^24 < base^6), the unrolled loop otherwise
        const float f = d.base >= 17 ? ScrambledRadicalInverse24x6(d, (uint32_t)a, perm)
                        : d.nDigits <= (uint32_t)kMaxShadeHaltonDigits
                            ? ScrambledRadicalInverse24<kMaxShadeHaltonDigits>(d, (uint32_t)a, perm)
                            : ScrambledRadicalInverse24<kMaxHaltonDigits24>(d, (uint32_t)a, perm);
        const float g = ScrambledRadicalInverse(d.base, d.nDigits, a, perm);
        uint32_t fb, gb;
        memcpy(&fb, &f, 4);
        memcpy(&gb, &g, 4);
        bad += fb != gb;
    }
    // the Lean shade stage's digit-major form (HaltonDepthSamples) over this dimension's depth
    // group, with the digit count of indices below a1
    if (dim >= 6 && 6 + ((size_t)dim - 6) / 7 * 7 + 7 <= s.permBase.size()) {
        const int d0 = 6 + (dim - 6) / 7 * 7;
        HaltonDimDesc g7[7];
        const uint16_t *p7[7];
        uint32_t nz = 1;
        for (int j = 0; j < 7; ++j) {
            g7[j] = MakeHaltonDimDesc(s.permBase[d0 + j], s.permNDigits[d0 + j], s.permOffset[d0 + j]);
            p7[j] = s.permTable.data() + g7[j].permOffset;
            nz = std::max(nz, HaltonDigitsFor(g7[j].base, a1));
        }
        for (int j = 0; j < 7; ++j) HaltonDimTail(&g7[j], p7[j], std::min(nz, 6u));
        for (uint64_t a = a0; a < a1; a += step) {
            float u[7];
            HaltonDepthSamples<false>(g7, (uint32_t)a, p7, u);
            const float g = ScrambledRadicalInverse(d.base, d.nDigits, a, perm);
            bad += memcmp(&u[dim - d0], &g, 4) != 0;
        }
    }
    return bad;
}

float pbrt_debug_halton(const pbrt_scene *scene, int px, int py, int sampleIndex, int dim) {
    const SceneDesc &s = scene->desc;
    uint64_t stride = (uint64_t)s.haltonBaseScales[0] * s.haltonBaseScales[1];
    uint64_t index = 0;
    if (stride > 1) {
        int pm[2] = {((px % 128) + 128) % 128, ((py % 128) + 128) % 128};
        for (int i = 0; i < 2; ++i) {
            uint64_t off = InverseRadicalInverse((uint64_t)pm[i], i == 0 ? 2 : 3, s.haltonBaseExponents[i]);
            index += off * (stride / s.haltonBaseScales[i]) * (uint64_t)s.haltonMultInverse[i];
        }
        index %= stride;
    }
    index += (uint64_t)sampleIndex * stride;
    // the camera kernel's evaluation (32-bit digit loop below 2^30)
    if (dim == -1) {
        const uint64_t a = index >> s.haltonBaseExponents[0];
        return a < (1ull << 30) ? RadicalInverse32<2>((uint32_t)a) : RadicalInverse(2, a);
    }
    if (dim == -2) {
        const uint64_t a = index / s.haltonBaseScales[1];
        return a < (1ull << 30) ? RadicalInverse32<3>((uint32_t)a) : RadicalInverse(3, a);
    }
    if (dim < 0 || dim >= (int)s.permBase.size()) return -1;
    // the device's evaluation path
    HaltonDimDesc d = MakeHaltonDimDesc(s.permBase[dim], s.permNDigits[dim], s.permOffset[dim]);
    return HaltonSampleDimension(d, index, s.permTable.data());
}

int pbrt_debug_rgb_coeffs(float r, float g, float b, float *c) {
    try {
        auto v = RGBToSigmoidCoeffs(r, g, b);
        c[0] = v[0];
        c[1] = v[1];
        c[2] = v[2];
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

// The product's texture evaluation (core/texture_eval.h, the same code the shade kernels run)
// on the host, for one material slot at a given hit: out[0..3] = dudx dudy dvdx dvdy, then the
// texture's value at each of the n wavelengths (reflectance) or out[4] (a roughness).
int pbrt_debug_texture_eval(const pbrt_scene *scene, int material, int slot, const float *hit14, const float *lambda,
                            int n, float *out) {
    try {
        if (!scene || !hit14 || !out) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        if (material < 0 || material >= (int)s.materials.size()) return Fail("material index out of range");
        const MaterialDesc &m = s.materials[material];
        const int prog = slot == 0 ? m.texReflectance : (slot == 1 ? m.texURough : m.texVRough);
        if (prog < 0) return Fail("material parameter is not textured");
        const TexView T = HostTexView(scene->tex);
        const CameraDiff cd = MakeCameraDiff(s);
        TexEvalCtx c;
        c.p = V3(hit14[0], hit14[1], hit14[2]);
        c.n = V3(hit14[3], hit14[4], hit14[5]);
        const V3 dpdu(hit14[6], hit14[7], hit14[8]), dpdv(hit14[9], hit14[10], hit14[11]);
        c.u = hit14[12];
        c.v = hit14[13];
        UVDerivatives(cd, c.p, c.n, dpdu, dpdv, &c);
        out[0] = c.dudx;
        out[1] = c.dudy;
        out[2] = c.dvdx;
        out[3] = c.dvdy;
        const DeviceTexProgram pg = T.progs[prog];
        float R[kTexMaxRegs];
        TexPhase1(T, pg, c, R);
        if (slot != 0) {
            out[4] = R[pg.result];
            return 0;
        }
        for (int i = 0; i < n; ++i)
            out[4 + i] = pg.simple ? SigmoidPolynomial(R[0], R[1], R[2], lambda[i]) : TexPhase2(T, pg, R, lambda[i], i % kNSpectrumSamples);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_pl2d(int dim, int cdf, const float *data, int xs, int ys, const int *pr2, const float *pv0,
                    const float *pv1, const float *q6, int n, float *out7) {
    try {
        if (!data || !q6 || !out7 || n < 0) return Fail("pbrt_debug_pl2d: null argument");
        if (dim != 0 && dim != 2) return Fail("pbrt_debug_pl2d: dim must be 0 or 2");
        if (xs < 2 || ys < 2) return Fail("pbrt_debug_pl2d: the table needs at least 2x2 values");
        if (dim == 2 && (!pr2 || !pv0 || !pv1 || pr2[0] < 1 || pr2[1] < 1))
            return Fail("pbrt_debug_pl2d: bad parameter grids");
        std::vector<float> blob;
        if (dim == 2) {
            blob.assign(pv0, pv0 + pr2[0]);
            blob.insert(blob.end(), pv1, pv1 + pr2[1]);
        }
        const uint32_t slices = dim == 2 ? (uint32_t)(pr2[0] * pr2[1]) : 1u;
        int h[5];
        BuildPL2D(data, xs, ys, slices, true, cdf != 0, &blob, h);
        PL2D d{};
        d.sx = h[0];
        d.sy = h[1];
        d.np = dim;
        d.data = blob.data() + h[2];
        d.marg = h[3] >= 0 ? blob.data() + h[3] : nullptr;
        d.cond = h[4] >= 0 ? blob.data() + h[4] : nullptr;
        // the parameter grids lead the blob (BuildPL2D appends after them)
        for (int i = 0; i < 3; ++i) {
            d.pn[i] = (dim == 2 && i < 2) ? pr2[i] : 1;
            d.pv[i] = blob.data() + (dim == 2 && i == 1 ? pr2[0] : 0);
        }
        for (int k = 0; k < n; ++k) {
            const float *x = q6 + 6 * (size_t)k;
            float *o = out7 + 7 * (size_t)k;
            std::fill(o, o + 7, 0.f);
            const float par[2] = {x[4], x[5]};
            if (dim == 0) {
                if (cdf) {
                    PLSample<0>(d, x[0], x[1], par, &o[0], &o[1], &o[2]);
                    PLInvert<0>(d, x[2], x[3], par, &o[3], &o[4], &o[5]);
                }
                o[6] = PLEvaluate<0>(d, x[2], x[3], par);
            } else {
                if (cdf) {
                    PLSample<2>(d, x[0], x[1], par, &o[0], &o[1], &o[2]);
                    PLInvert<2>(d, x[2], x[3], par, &o[3], &o[4], &o[5]);
                }
                o[6] = PLEvaluate<2>(d, x[2], x[3], par);
            }
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_windowed2d(const float *func, int res, const float *q8, int n, float *out5) {
    try {
        if (!func || !q8 || !out5 || n < 0 || res < 1) return Fail("pbrt_debug_windowed2d: bad arguments");
        const std::vector<float> f(func, func + (size_t)res * res);
        const std::vector<float> sat = SummedAreaTable(f, res);
        DeviceEnvLight E{};
        E.res = res;
        E.sat = sat.data();
        E.func = f.data();
        for (int k = 0; k < n; ++k) {
            const float *x = q8 + 8 * (size_t)k;
            float *o = out5 + 5 * (size_t)k;
            std::fill(o, o + 5, 0.f);
            const float b[4] = {x[2], x[3], x[4], x[5]};
            float px, py, pdf;
            if (PortalWindowedSample(E, x[0], x[1], b, &px, &py, &pdf)) o[0] = 1, o[1] = px, o[2] = py, o[3] = pdf;
            const float bi = SatIntegral(E, b[0], b[1], b[2], b[3]);
            o[4] = bi == 0 ? 0.f : PortalFuncAt(E, x[6], x[7]) / bi;
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_measured(const pbrt_scene *scene, int brdf, const float *in8, int n, const float *lambda, float *out) {
    try {
        if (!scene || !in8 || !lambda || !out || n < 0) return Fail("pbrt_debug_measured: bad arguments");
        const SceneDesc &s = scene->desc;
        if (brdf < 0 || brdf >= (int)s.measured.size()) return Fail("pbrt_debug_measured: not a measured BRDF index");
        const MeasuredView m = MeasuredAt(s.measured[brdf].hdr.data(), s.measured[brdf].blob.data());
        for (int i = 0; i < n; ++i) MeasuredDebugEval(m, in8 + (size_t)kMeasDebugIn * i, lambda, out + (size_t)kMeasDebugOut * i);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_portal_eval(const pbrt_scene *scene, int env, const float *q8, int n, float *out16, float *img) {
    try {
        if (!scene || !q8 || !out16) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        if (env < 0 || env >= (int)s.envLights.size() || !s.envLights[env].portal) return Fail("not a portal light index");
        const EnvLightDesc &e = s.envLights[env];
        const std::vector<EnvCoef> coef = BuildEnvCoefs(e);
        DeviceEnvLight E{};
        std::memcpy(E.m, e.renderFromLight, sizeof(E.m));
        std::memcpy(E.mi, e.lightFromRender, sizeof(E.mi));
        E.res = e.res;
        E.portal = 1;
        E.coef = coef.data();
        std::memcpy(E.pf, e.portalFrame, sizeof(E.pf));
        std::memcpy(E.pc0, e.portalP[0], sizeof(E.pc0));
        std::memcpy(E.pc2, e.portalP[2], sizeof(E.pc2));
        E.sat = e.portalSat.data();
        E.func = e.portalFunc.data();
        static const float kLam[4] = {400.f, 500.f, 600.f, 700.f};
        for (int i = 0; i < n; ++i) {
            const float *x = q8 + 8 * (size_t)i;
            float *o = out16 + 16 * (size_t)i;
            std::fill(o, o + 16, 0.f);
            const V3 p(x[0], x[1], x[2]), d(x[3], x[4], x[5]);
            const EnvCoef c = PortalLeCoef(E, p, d);
            for (int k = 0; k < 4; ++k) o[k] = EnvLe(c, 1.f, 1.f, kLam[k]);
            o[4] = PortalPDFLi(E, p, d);
            V3 wi;
            float pdf;
            EnvCoef sc;
            if (PortalSampleLi(E, p, x[6], x[7], &wi, &pdf, &sc)) {
                o[5] = 1;
                o[6] = wi.x, o[7] = wi.y, o[8] = wi.z;
                o[9] = pdf;
                for (int k = 0; k < 4; ++k) o[10 + k] = EnvLe(sc, 1.f, 1.f, kLam[k]);
            }
            float b[4];
            o[14] = PortalImageBounds(E, p, b) ? 1.f : 0.f;
        }
        if (img) {
            const size_t np = (size_t)e.res * e.res;
            std::copy(e.rect.begin(), e.rect.end(), img);
            std::copy(e.portalFunc.begin(), e.portalFunc.end(), img + 3 * np);
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_env_eval(const pbrt_scene *scene, int env, const float *dirs, const float *u, int n, float *out) {
    try {
        if (!scene || !dirs || !u || !out) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        if (env < 0 || env >= (int)s.envLights.size()) return Fail("environment light index out of range");
        const EnvLightDesc &e = s.envLights[env];
        const std::vector<EnvCoef> coef = BuildEnvCoefs(e);
        const std::vector<float> dist = BuildEnvDistribution(e);
        DeviceEnvLight E{};
        std::memcpy(E.m, e.renderFromLight, sizeof(E.m));
        std::memcpy(E.mi, e.lightFromRender, sizeof(E.mi));
        E.res = e.res;
        E.coef = coef.data();
        E.dist = FilterTableView{e.res, e.res, dist.data()};
        static const float kLam[4] = {400.f, 500.f, 600.f, 700.f};
        for (int i = 0; i < n; ++i) {
            float *o = out + 16 * (size_t)i;
            const V3 d(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
            float uu, vv;
            EqualAreaSphereToSquare(Normalize(MulM3(E.mi, d)), &uu, &vv);
            o[0] = uu;
            o[1] = vv;
            float pu, pv;
            EqualAreaSphereToSquare(MulM3(E.mi, d), &pu, &pv);
            o[2] = EnvPDF(E, pu, pv) / (4 * kPi);
            const EnvCoef c = EnvCoefAt(E, uu, vv);
            for (int k = 0; k < 4; ++k) o[3 + k] = EnvLe(c, 1.f, 1.f, kLam[k]);
            float su, sv, mp;
            EnvSampleUV(E, u[2 * i], u[2 * i + 1], &su, &sv, &mp);
            o[7] = su;
            o[8] = sv;
            o[9] = mp;
            const V3 wi = MulM3(E.m, EqualAreaSquareToSphere(su, sv));
            o[10] = wi.x;
            o[11] = wi.y;
            o[12] = wi.z;
            o[13] = EnvPDF(E, su, sv);                // PiecewiseConstant2D::PDF at the sample
            o[14] = EnvPDF(E, u[2 * i], u[2 * i + 1]);  // ... and at u taken as a point of [0,1]^2
            o[15] = 0;
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_shape_eval(const pbrt_scene *scene, int shape, const float *rays, const float *u, int n, float *out) {
    try {
        if (!scene || !rays || !u || !out) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        if (shape < 0 || shape >= (int)s.shapes.size()) return Fail("shape index out of range");
        const DeviceShape &d = s.shapes[shape].dev;
        const float *N = s.shapes[shape].normals.data();
        for (int i = 0; i < n; ++i) {
            float *o = out + 40 * (size_t)i;
            std::fill(o, o + 40, 0.f);
            const V3 ro(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), rd(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
            // the sampling context's shading normal: every other row uses -d (patch cosine warp)
            const V3 cns = (i & 1) ? Normalize(-rd) : V3(0, 0, 0);
            float th;
            V3 pObj;
            if (ShapeIntersect(d, ro, rd, kInfinity, &th, &pObj)) {
                const TriSurface si = ShapeSurface(d, pObj, N);
                const V3 v[8] = {pObj, si.p, si.pErr, si.n, si.ns, si.dpdu, si.dpdv, V3(si.uv[0], si.uv[1], 0)};
                o[0] = 1;
                o[1] = th;
                for (int k = 0; k < 8; ++k)
                    for (int j = 0; j < (k == 7 ? 2 : 3); ++j) o[2 + 3 * k + j] = v[k][j];
            }
            ShapeSamplePt ss;
            if (ShapeSampleSolidAngle(d, ro, V3(0, 0, 0), V3(0, 0, 0), u[2 * i], u[2 * i + 1], &ss, N, cns)) {
                o[26] = 1;
                for (int j = 0; j < 3; ++j) {
                    o[27 + j] = ss.p[j];
                    o[30 + j] = ss.pErr[j];
                    o[33 + j] = ss.n[j];
                }
                o[36] = ss.pdf;
            }
            o[37] = ShapePDFSolidAngle(d, ro, V3(0, 0, 0), V3(0, 0, 0), rd, N, cns);
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_cloud_density(const float *params3, const float *pts, int n, float *out) {
    try {
        const auto &perm = GetSpectralData().noisePerm;
        if (perm.size() != 512) return Fail("spectral data lacks the noise permutation (NoisePerm)");
        std::vector<float> c(params3, params3 + 3);
        c.insert(c.end(), perm.begin(), perm.end());
        for (int i = 0; i < n; ++i) {
            const V3 p(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
            // rows: Noise(p), DNoise(p) xyz, Density(p) with params3
            const float nz = Noise3(c.data() + 3, p.x, p.y, p.z);
            const float d = .01f;
            out[5 * i] = nz;
            out[5 * i + 1] = (Noise3(c.data() + 3, p.x + d, p.y + 0.f, p.z + 0.f) - nz) / d;
            out[5 * i + 2] = (Noise3(c.data() + 3, p.x + 0.f, p.y + d, p.z + 0.f) - nz) / d;
            out[5 * i + 3] = (Noise3(c.data() + 3, p.x + 0.f, p.y + 0.f, p.z + d) - nz) / d;
            out[5 * i + 4] = CloudDensity(c.data(), p);
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_equal_area(int to_sphere, const float *in, int n, float *out) {
    if (!in || !out || n < 0) return Fail("null argument");
    for (int i = 0; i < n; ++i) {
        if (to_sphere) {
            const V3 w = EqualAreaSquareToSphere(in[2 * i], in[2 * i + 1]);
            out[3 * i] = w.x;
            out[3 * i + 1] = w.y;
            out[3 * i + 2] = w.z;
        } else {
            EqualAreaSphereToSquare(V3(in[3 * i], in[3 * i + 1], in[3 * i + 2]), &out[2 * i], &out[2 * i + 1]);
        }
    }
    return 0;
}

int pbrt_debug_color_space(int cs, float *info) {
    try {
        if (!info) return Fail("null argument");
        if (cs < 0 || cs >= kNumColorSpaces) return Fail("pbrt_debug_color_space: colour space index out of range");
        const ColorSpaceDesc &c = GetColorSpace(cs);
        float *o = info;
        o = std::copy(c.prim, c.prim + 6, o);
        o = std::copy(c.w, c.w + 2, o);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) *o++ = c.xyzFromRGBf[i][j];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) *o++ = c.rgbFromXYZf[i][j];
        *o++ = c.photometric;
        std::copy(c.illuminant.begin(), c.illuminant.end(), o);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_color_space_index(const char *name) {
    if (!name) {
        Fail("null argument");
        return -1;
    }
    const int cs = ColorSpaceByName(name);
    if (cs < 0) Fail(std::string(name) + ": color space unknown");
    return cs;
}

int pbrt_debug_rgb_spectrum(int cs, const float *rgb3, int n, float unboundedScale, const float *lambda, int nl,
                            float *out) {
    try {
        if (!rgb3 || !lambda || !out || n < 0 || nl < 0) return Fail("null argument");
        if (cs < 0 || cs >= kNumColorSpaces) return Fail("pbrt_debug_rgb_spectrum: colour space index out of range");
        const ColorSpaceDesc &c = GetColorSpace(cs);
        const int stride = 3 + 3 * nl;
        for (int k = 0; k < n; ++k) {
            const float *x = rgb3 + 3 * (size_t)k;
            float *o = out + (size_t)stride * k;
            // RGBAlbedoSpectrum(cs, rgb): the table's coefficients of rgb itself
            const auto a = RGBToSigmoidCoeffs(x[0], x[1], x[2], cs);
            std::copy(a.begin(), a.end(), o);
            // RGBUnboundedSpectrum / RGBIlluminantSpectrum(cs, unboundedScale * rgb): scale 2 max,
            // the coefficients of rgb / scale; the illuminant is DenselySampled (nearest nm)
            const float r = unboundedScale * x[0], g = unboundedScale * x[1], b = unboundedScale * x[2];
            const float scale = 2 * std::max({r, g, b});
            const auto u = scale ? RGBToSigmoidCoeffs(r / scale, g / scale, b / scale, cs) : RGBToSigmoidCoeffs(0, 0, 0, cs);
            for (int i = 0; i < nl; ++i) {
                const float l = lambda[i];
                o[3 + i] = SigmoidPolynomial(a[0], a[1], a[2], l);
                o[3 + nl + i] = scale * SigmoidPolynomial(u[0], u[1], u[2], l);
                const int off = (int)std::lround(l) - 395;
                const float ill = off >= 0 && off < 311 ? c.illuminant[off] : 0.f;
                o[3 + 2 * nl + i] = scale * SigmoidPolynomial(u[0], u[1], u[2], l) * ill;
            }
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_rgb2spec_column_cs(int cs, int maxc, int j, int i, float *out) {
    try {
        if (!out) return Fail("null argument");
        if (cs < 0 || cs >= kNumColorSpaces || maxc < 0 || maxc > 2 || j < 0 || j > 63 || i < 0 || i > 63)
            return Fail("pbrt_debug_rgb2spec_column_cs: index out of range");
        auto v = RGB2SpecColumn(maxc, j, i, cs);
        std::copy(v.begin(), v.end(), out);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_rgb2spec_column(int maxc, int j, int i, float *out) {
    try {
        auto v = RGB2SpecColumn(maxc, j, i);
        std::copy(v.begin(), v.end(), out);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_filter_sample(const pbrt_scene *scene, float u0, float u1, float *out3) {
    try {
        const SceneDesc &s = scene->desc;
        const FilterParams fp{s.filterType, s.filterRadiusX, s.filterRadiusY, s.filterA, s.filterB};
        FilterSample(fp, FilterTableView{s.filterNu, s.filterNv, s.filterTable.data()}, u0, u1, &out3[0], &out3[1],
                     &out3[2]);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_zsobol(const pbrt_scene *scene, int px, int py, int sampleIndex, int dim, float *out7) {
    try {
        if (!scene || !out7) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        ZSobolParams z{s.zsLog2SamplesPerPixel, s.zsNBase4Digits, s.seed, (Randomize)s.zsRandomize};
        uint32_t m1[kSobolMatrixSize];
        for (int k = 0; k < kSobolMatrixSize; ++k) m1[k] = SobolMatrix1Row(k);
        const uint64_t morton = ZSobolMortonIndex(z, px, py, sampleIndex);
        // the wavefront's call pattern from `dim`: Get1D, Get2D, Get1D, Get2D, Get1D
        out7[0] = ZSobolGet1D(z, morton, dim, kZSobolPermutations, m1);
        ZSobolGet2D(z, morton, dim + 1, kZSobolPermutations, m1, &out7[1], &out7[2]);
        out7[3] = ZSobolGet1D(z, morton, dim + 3, kZSobolPermutations, m1);
        ZSobolGet2D(z, morton, dim + 4, kZSobolPermutations, m1, &out7[4], &out7[5]);
        out7[6] = ZSobolGet1D(z, morton, dim + 6, kZSobolPermutations, m1);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_sampler(const pbrt_scene *scene, int px, int py, int sampleIndex, int dim, float *out7) {
    try {
        if (!scene || !out7) return Fail("null argument");
        const SceneDesc &s = scene->desc;
        if (s.samplerType < kSamplerIndependent) return Fail("pbrt_debug_sampler: the scene's sampler is halton or zsobol");
        SamplerDesc d{s.samplerType, s.spp, s.seed, s.stratXs, s.stratYs, s.stratJitter, (Randomize)s.zsRandomize,
                      s.sobolLog2Scale, nullptr, nullptr, nullptr};
        if (s.samplerType == kSamplerSobol) {
            const SobolTableData &sob = SobolTables();
            d.sobol32 = sob.m32.data();
            d.vdc = sob.vdc.data();
            d.vdcInv = sob.vdcInv.data();
        }
        GenericSampler g;
        g.Start(d, px, py, sampleIndex, dim);
        // dimension 0: the camera's Get1D, GetPixel2D, Get1D, Get2D, Get1D; otherwise the ray
        // samples' Get1D, Get2D, Get1D, Get2D, Get1D
        out7[0] = g.Get1D(d);
        if (dim == 0) g.GetPixel2D(d, &out7[1], &out7[2]);
        else g.Get2D(d, &out7[1], &out7[2]);
        out7[3] = g.Get1D(d);
        g.Get2D(d, &out7[4], &out7[5]);
        out7[6] = g.Get1D(d);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_det_math(int device, int fn, const float *a, const float *b, int n, float *out) {
    try {
        if (!a || !b || !out || n < 0 || fn < 0 || fn >= detm::kNumEvalFns)
            return Fail("pbrt_debug_det_math: bad arguments");
        if (device < 0) {  // the same code compiled for the host
            for (int i = 0; i < n; ++i) out[i] = detm::Eval(fn, a[i], b[i]);
            return 0;
        }
        HIPCHECK(hipSetDevice(device));
        DevBuf<float> da, db, dout;
        da.Upload(std::vector<float>(a, a + n));
        db.Upload(std::vector<float>(b, b + n));
        dout.Alloc(n);
        if (n > 0) {
            HIPCHECK(LaunchDetMath(fn, da.p, db.p, n, dout.p, nullptr));
            HIPCHECK(hipMemcpy(out, dout.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_hair(int device, const float *in16, int n, float *out) {
    try {
        if (!in16 || !out || n < 0) return Fail("pbrt_debug_hair: bad arguments");
        if (device < 0) {  // the same code compiled for the host (libm transcendentals)
            for (int i = 0; i < n; ++i) HairDebugEval(in16 + (size_t)kHairDebugIn * i, out + (size_t)kHairDebugOut * i);
            return 0;
        }
        HIPCHECK(hipSetDevice(device));
        DevBuf<float> din, dout;
        din.Upload(std::vector<float>(in16, in16 + (size_t)kHairDebugIn * n));
        dout.Alloc((size_t)kHairDebugOut * n);
        if (n > 0) {
            HIPCHECK(LaunchHairEval(din.p, n, dout.p, nullptr));
            HIPCHECK(hipMemcpy(out, dout.p, (size_t)kHairDebugOut * n * sizeof(float), hipMemcpyDeviceToHost));
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_procedural(int kind, const float *params4, const float *in9, int n, float *out6) {
    try {
        if (!params4 || !in9 || !out6 || n < 0 || kind < 0 || kind > 4) return Fail("pbrt_debug_procedural: bad arguments");
        const auto &perm = GetSpectralData().noisePerm;
        if (perm.size() != 512) return Fail("spectral data lacks the noise permutation (NoisePerm)");
        TexTables none;
        const TexView T = HostTexView(none);  // the RGB -> spectrum table for marble
        for (int i = 0; i < n; ++i) {
            const float *q = in9 + 9 * i;
            float *o = out6 + 6 * i;
            const V3 p(q[0], q[1], q[2]), dx(q[3], q[4], q[5]), dy(q[6], q[7], q[8]);
            for (int k = 0; k < 6; ++k) o[k] = 0;
            switch (kind) {
            case 0: o[0] = FBmNoise(perm.data(), p, dx, dy, params4[1], (int)params4[0]); break;
            case 1: o[0] = TurbulenceNoise(perm.data(), p, dx, dy, params4[1], (int)params4[0]); break;
            case 2: o[0] = WindyNoise(perm.data(), p, dx, dy); break;
            case 3: o[0] = InsidePolkaDot(perm.data(), q[0], q[1]) ? 1.f : 0.f; break;
            default:
                MarbleRGB(perm.data(), p, dx, dy, (int)params4[0], params4[1], params4[2], params4[3], o);
                RGBToCoeffs(T, o[0], o[1], o[2], o + 3);
                break;
            }
        }
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_rng(uint64_t seq, uint64_t advance, uint32_t *out2) {
    if (!out2) return Fail("null argument");
    PCG32 r;
    r.SetSequence(seq);
    r.Advance(advance);
    out2[0] = r.NextU32();
    out2[1] = r.NextU32();
    return 0;
}

int pbrt_debug_trowbridge(const float *in, float *out) {
    if (!in || !out) return Fail("null argument");
    TrowbridgeReitz d = TrowbridgeReitz::Make(in[0], in[1]);
    V3 wo(in[2], in[3], in[4]), wi(in[5], in[6], in[7]), wm(in[8], in[9], in[10]);
    V3 sw = d.SampleWm(wo, in[11], in[12]);
    TrowbridgeReitz r = d;
    r.Regularize();
    const float v[14] = {d.ax,        d.ay,      (float)d.EffectivelySmooth(), d.D(wm), d.D(wo, wm), d.Lambda(wo),
                         d.G1(wo),    d.G(wo, wi), d.PDF(wo, wm),             sw.x,    sw.y,        sw.z,
                         r.ax,        r.ay};
    memcpy(out, v, sizeof v);
    return 0;
}

int pbrt_debug_fresnel(const float *in, float *out) {
    if (!in || !out) return Fail("null argument");
    V3 wi(in[4], in[5], in[6]), n(in[7], in[8], in[9]);
    float etap = 0;
    V3 wt(0, 0, 0);
    bool ok = Refract(wi, n, in[1], &etap, &wt);
    V3 rf = Reflect(wi, n);
    const float v[10] = {FrDielectric(in[0], in[1]), FrComplex(in[0], in[2], in[3]), (float)ok, etap, wt.x, wt.y,
                         wt.z, rf.x, rf.y, rf.z};
    memcpy(out, v, sizeof v);
    return 0;
}

int pbrt_debug_triangle_shading(const float *p9, const float *n9, const float *uv6, int flip, const float *b3,
                                const float *u2, float *out) {
    if (!p9 || !b3 || !u2 || !out) return Fail("null argument");
    const V3 p0(p9[0], p9[1], p9[2]), p1(p9[3], p9[4], p9[5]), p2(p9[6], p9[7], p9[8]);
    TriShading sh;
    sh.flags = (n9 ? 1 : 0) | (uv6 ? 2 : 0);
    if (n9) {
        sh.n0 = V3(n9[0], n9[1], n9[2]);
        sh.n1 = V3(n9[3], n9[4], n9[5]);
        sh.n2 = V3(n9[6], n9[7], n9[8]);
    }
    if (uv6)
        for (int k = 0; k < 3; ++k) sh.uv[k][0] = uv6[2 * k], sh.uv[k][1] = uv6[2 * k + 1];
    TriSurface s = TriangleSurface(p0, p1, p2, b3[0], b3[1], b3[2], flip != 0, &sh);
    float b[3];
    SampleUniformTriangle(u2[0], u2[1], b);
    V3 sn = TriangleSampleNormal(p0, p1, p2, b[0], b[1], flip != 0, &sh);
    const float v[15] = {s.n.x, s.n.y, s.n.z, s.ns.x, s.ns.y, s.ns.z, s.dpdu.x, s.dpdu.y, s.dpdu.z,
                         s.dpdus.x, s.dpdus.y, s.dpdus.z, sn.x, sn.y, sn.z};
    memcpy(out, v, sizeof v);
    return 0;
}

int pbrt_debug_named_spectrum(const char *name, const float *lambda, int n, float *out) {
    try {
        if (!name || !lambda || !out) return Fail("null argument");
        PLSpectrumDesc d = NamedPiecewiseLinear(name);
        // the kernels' indexed evaluation (the same segment and arithmetic as PiecewiseLinearEval)
        uint16_t idx[kPlIndexN];
        BuildPlIndex(d.lambda.data(), (int)d.lambda.size(), idx);
        for (int i = 0; i < n; ++i)
            out[i] = PiecewiseLinearEvalIdx(d.lambda.data(), d.value.data(), (int)d.lambda.size(), idx, lambda[i]);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_bxdf(int type, const float *params, const float *eta31, const float *k31, const float *wo3,
                    const float *wi3, const float *u3, float *out) {
    if (!params || !wo3 || !wi3 || !u3 || !out) return Fail("null argument");
    if ((type == kMatConductor || type == kMatRetroreflective) && (!eta31 || !k31))
        return Fail("conductor / retroreflective needs eta and k");
    if (type != kMatDielectric && type != kMatConductor && type != kMatRetroreflective)
        return Fail("type must be 1 (dielectric), 2 (conductor) or 11 (retroreflective)");
    const TrowbridgeReitz tr{params[0], params[1]};
    const float eta = params[2];
    const V3 wo(wo3[0], wo3[1], wo3[2]), wi(wi3[0], wi3[1], wi3[2]);
    memset(out, 0, 70 * sizeof(float));
    if (type == kMatDielectric) {
        BxSample bs = DielectricSample(eta, tr, wo, u3[0], u3[1], u3[2]);
        if (bs.ok) {
            const float v[7] = {1, bs.wi.x, bs.wi.y, bs.wi.z, bs.pdf, (float)bs.flags, bs.etap};
            memcpy(out, v, sizeof v);
            for (int i = 0; i < kNSpectrumSamples; ++i) out[7 + i] = bs.f;
        }
        float pdf;
        float f = DielectricEval(eta, tr, wo, wi, &pdf);
        for (int i = 0; i < kNSpectrumSamples; ++i) out[38 + i] = f;
        out[69] = pdf;
    } else if (type == kMatRetroreflective) {
        const ConductorTerms ct = RetroSample(tr, wo, u3[1], u3[2]);
        if (ct.ok) {
            const float v[7] = {1, ct.wi.x, ct.wi.y, ct.wi.z, ct.pdf, (float)(kBxReflection | (ct.specular ? kBxSpecular : kBxGlossy)), 1};
            memcpy(out, v, sizeof v);
            for (int i = 0; i < kNSpectrumSamples; ++i) out[7 + i] = ConductorF(ct, eta31[i], k31[i]);
        }
        const RetroTerms rt = RetroEval(tr, wo, wi);
        if (rt.ok)
            for (int i = 0; i < kNSpectrumSamples; ++i) out[38 + i] = RetroF(rt, eta31[i], k31[i]);
        out[69] = RetroPDF(tr, wo, wi);
    } else {
        ConductorTerms ct = ConductorSample(tr, wo, u3[1], u3[2]);
        if (ct.ok) {
            const int flags = kBxReflection | (ct.specular ? kBxSpecular : kBxGlossy);
            const float v[7] = {1, ct.wi.x, ct.wi.y, ct.wi.z, ct.pdf, (float)flags, 1};
            memcpy(out, v, sizeof v);
            for (int i = 0; i < kNSpectrumSamples; ++i) out[7 + i] = ConductorF(ct, eta31[i], k31[i]);
        }
        ConductorTerms ce = ConductorEval(tr, wo, wi);
        if (ce.ok) {
            for (int i = 0; i < kNSpectrumSamples; ++i) out[38 + i] = ConductorF(ce, eta31[i], k31[i]);
            out[69] = ce.pdf;
        }
    }
    return 0;
}

namespace {
struct DebugLayerSpec {
    const float *a, *b, *alb;
    float R(int i) const { return a[i]; }
    void EtaK(int i, float *e, float *k) const {
        *e = a[i];
        *k = b[i];
    }
    float Albedo(int i) const { return alb[i]; }
};
}  // namespace

int pbrt_debug_layered(const float *params, const float *a31, const float *b31, const float *alb31, const float *wo3,
                       const float *wi3, const float *u3, float *out) {
    if (!params || !a31 || !b31 || !alb31 || !wo3 || !wi3 || !u3 || !out) return Fail("null argument");
    if (params[3] != 0 && params[3] != 2) return Fail("bottom type must be 0 (diffuse) or 2 (conductor)");
    if (params[8] < 0 || params[9] < 1) return Fail("maxdepth >= 0 and nsamples >= 1 required");
    const DebugLayerSpec sp{a31, b31, alb31};
    bool bottomNz = false, albNz = false;
    for (int i = 0; i < kNSpectrumSamples; ++i) {
        bottomNz |= a31[i] != 0;
        albNz |= alb31[i] != 0;
    }
    const LayeredBxDF<DebugLayerSpec> L{params[2],
                                        TrowbridgeReitz{params[0], params[1]},
                                        TrowbridgeReitz{params[4], params[5]},
                                        params[3] == 2,
                                        std::max(params[6], std::numeric_limits<float>::min()),
                                        params[7],
                                        albNz,
                                        (int)params[8],
                                        (int)params[9],
                                        0,
                                        sp,
                                        bottomNz};
    const bool radiance = params[10] != 0;
    const V3 wo(wo3[0], wo3[1], wo3[2]), wi(wi3[0], wi3[1], wi3[2]);
    memset(out, 0, 72 * sizeof(float));
    float f[kNSpectrumSamples];
    const LayerSample bs = L.Sample_f(wo, u3[0], u3[1], u3[2], radiance, f);
    if (bs.ok) {
        const float v[6] = {1, bs.wi.x, bs.wi.y, bs.wi.z, bs.pdf, (float)bs.flags};
        memcpy(out, v, sizeof v);
        for (int i = 0; i < kNSpectrumSamples; ++i) out[6 + i] = f[i];
    }
    L.f(wo, wi, radiance, f);
    for (int i = 0; i < kNSpectrumSamples; ++i) out[37 + i] = f[i];
    out[68] = L.PDF(wo, wi, radiance);
    out[69] = (float)L.LayerFlags();
    return 0;
}

int pbrt_debug_light_bvh(const float *lights13, int n, float *nodes12, int32_t *info3, uint32_t *trails, int max_nodes,
                         int *n_nodes) {
    try {
        if (!lights13 || n < 0 || !n_nodes) return Fail("bad arguments");
        std::vector<LightBVHNodeDesc> nodes;
        std::vector<uint32_t> tr;
        DebugBuildLightBVH(lights13, n, &nodes, &tr);
        *n_nodes = (int)nodes.size();
        for (int i = 0; i < std::min((int)nodes.size(), max_nodes); ++i) {
            const LightNodeBounds &b = nodes[i].bounds;
            const float v[12] = {b.pMin.x, b.pMin.y, b.pMin.z, b.pMax.x, b.pMax.y, b.pMax.z, b.w.x, b.w.y, b.w.z,
                                 b.phi, b.cosTheta_o, b.cosTheta_e};
            if (nodes12) memcpy(nodes12 + 12 * i, v, sizeof v);
            if (info3) {
                info3[3 * i] = nodes[i].childOrLight;
                info3[3 * i + 1] = nodes[i].isLeaf;
                info3[3 * i + 2] = b.twoSided;
            }
        }
        if (trails) std::copy(tr.begin(), tr.end(), trails);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_bvh_stats(const pbrt_scene *scene, int64_t *out8) {
    try {
        if (!scene || !out8) return Fail("null argument");
        const BVH8 b = BuildBVH8(scene->desc.verts, scene->desc.tris, 4);
        const int64_t v[8] = {(int64_t)b.nodes.size(), (int64_t)b.triPrim.size(), b.maxDepth, b.maxStack,
                              (int64_t)(b.nodes.size() * sizeof(BVH8Node)), (int64_t)(b.qnodes.size() * sizeof(BVH8QNode)),
                              0, 0};
        memcpy(out8, v, sizeof v);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_bvh_trace(const pbrt_scene *scene, int spatial, const float *rays, int n, float *tOut, int *primOut,
                         int64_t *stats4) {
    try {
        if (!scene || !rays || n < 0 || !tOut || !primOut || !stats4) return Fail("null argument");
        const BVH8 b = BuildBVH8(scene->desc.verts, scene->desc.tris, 4, spatial);
        int64_t nodeVisits = 0, triTests = 0;
        std::vector<int> stack;
        for (int i = 0; i < n; ++i) {
            const V3 o(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), d(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
            float tMax = kInfinity;
            int hit = -1;
            stack.assign(1, 0);
            while (!stack.empty()) {
                const int ni = stack.back();
                stack.pop_back();
                ++nodeVisits;
                const BVH8Node &nd = b.nodes[ni];
                for (int c = 0; c < 8; ++c) {
                    if (!(nd.occ >> c & 1)) continue;
                    // exact slab test in double precision (a box that misses part of its
                    // triangle shows up as a missed hit against the brute-force answer)
                    double t0 = 0, t1 = tMax;
                    const double lo[3] = {nd.lox[c], nd.loy[c], nd.loz[c]}, hi[3] = {nd.hix[c], nd.hiy[c], nd.hiz[c]};
                    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
                    bool in = true;
                    for (int a = 0; a < 3 && in; ++a) {
                        if (dd[a] == 0) {
                            if (oo[a] < lo[a] || oo[a] > hi[a]) in = false;
                            continue;
                        }
                        double ta = (lo[a] - oo[a]) / dd[a], tb = (hi[a] - oo[a]) / dd[a];
                        if (ta > tb) std::swap(ta, tb);
                        t0 = std::max(t0, ta), t1 = std::min(t1, tb);
                        if (t0 > t1) in = false;
                    }
                    if (!in) continue;
                    const int ref = b.childRef[ni][c];
                    if (ref >= 0) {
                        stack.push_back(ref);
                        continue;
                    }
                    const int enc = ~ref, first = enc >> 3, count = (enc & 7) + 1;
                    for (int k = first; k < first + count; ++k) {
                        ++triTests;
                        const float *v = &b.triVerts[(size_t)k * 12];
                        TriHit h;
                        if (IntersectTriangle(o, d, tMax, V3(v[0], v[1], v[2]), V3(v[4], v[5], v[6]), V3(v[8], v[9], v[10]), &h))
                            tMax = h.t, hit = b.triPrim[k];
                    }
                }
            }
            tOut[i] = hit >= 0 ? tMax : -1.f;
            primOut[i] = hit;
        }
        const int64_t v[4] = {nodeVisits, triTests, (int64_t)b.triPrim.size(), (int64_t)b.nodes.size()};
        memcpy(stats4, v, sizeof v);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_displace(const float *p, const float *uv, const float *n, int nVerts, const int *tri, int nTri,
                        const int *quad, int nQuad, const float *renderFromObject16, float edgeLength, int mode,
                        int capVerts, int capTris, float *pOut, float *nOut, float *uvOut, int *triOut, int *counts2) {
    try {
        if (!p || !uv || nVerts <= 0 || (nTri > 0 && !tri) || (nQuad > 0 && !quad) || !renderFromObject16 || !pOut ||
            !nOut || !uvOut || !triOut || !counts2)
            return Fail("null argument");
        DisplaceMesh m;
        for (int i = 0; i < nVerts; ++i) {
            m.p.push_back(V3(p[3 * i], p[3 * i + 1], p[3 * i + 2]));
            m.uv.push_back({uv[2 * i], uv[2 * i + 1]});
            if (n) m.n.push_back(V3(n[3 * i], n[3 * i + 1], n[3 * i + 2]));
        }
        for (int i = 0; i < 3 * nTri; ++i) {
            if (tri[i] < 0 || tri[i] >= nVerts) return Fail("triangle index out of range");
            m.tri.push_back(tri[i]);
        }
        for (int i = 0; i < 4 * nQuad; ++i) {
            if (quad[i] < 0 || quad[i] >= nVerts) return Fail("quad index out of range");
            m.quad.push_back(quad[i]);
        }
        // the closed-form displacements of oracle/ref/refgold.cpp DisplaceGoldens
        DisplaceTriQuadMesh(&m, renderFromObject16, edgeLength, [mode](V3 q, float u, float v) {
            return mode == 0 ? 0.1f * u - 0.05f * v : mode == 1 ? 0.25f * q.y * u + 0.125f : 0.1f;
        });
        counts2[0] = (int)m.p.size();
        counts2[1] = (int)m.tri.size() / 3;
        if (counts2[0] > capVerts || counts2[1] > capTris) return Fail("pbrt_debug_displace: output capacity too small");
        for (size_t i = 0; i < m.p.size(); ++i) {
            pOut[3 * i] = m.p[i].x, pOut[3 * i + 1] = m.p[i].y, pOut[3 * i + 2] = m.p[i].z;
            nOut[3 * i] = m.n[i].x, nOut[3 * i + 1] = m.n[i].y, nOut[3 * i + 2] = m.n[i].z;
            uvOut[2 * i] = m.uv[i][0], uvOut[2 * i + 1] = m.uv[i][1];
        }
        std::copy(m.tri.begin(), m.tri.end(), triOut);
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_set_queue_check(int on) {
    SetQueueCheck(on);
    return 0;
}
int pbrt_debug_queue_holes(int *holes) {
    if (!holes) return Fail("pbrt_debug_queue_holes: null output");
    *holes = TakeQueueHoles();
    return 0;
}
int pbrt_debug_queue_counts(pbrt_context *ctx, int32_t *counts, int n) {
    try {
        if (!ctx || !counts || n <= 0) return Fail("null argument");
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        const int depths = ctx->desc.maxDepth + 3;
        std::vector<int32_t> raw(CounterIndex(depths, 0, 0));
        HIPCHECK(hipMemcpy(raw.data(), ctx->st.counters, raw.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
        // [depth][8]: totals over shards of the kNumQueues queues, zero padded
        for (int i = 0; i < n; ++i) counts[i] = 0;
        for (int d = 0; d < depths; ++d)
            for (int q = 0; q < kNumQueues; ++q)
                for (int sh = 0; sh < kShards; ++sh)
                    if (d * 8 + q < n) counts[d * 8 + q] += raw[CounterIndex(d, q, sh)];
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

int pbrt_debug_kernel_sections(pbrt_context *ctx, uint64_t *cycles, int n) {
    try {
        if (!ctx || !cycles || n <= 0) return Fail("null argument");
        n = std::min(n, kStatsSlots - kStatsSectionBase);
        HIPCHECK(hipSetDevice(ctx->device));
        HIPCHECK(hipStreamSynchronize(ctx->stream));
        std::vector<unsigned long long> h(kStatsSlots);
        HIPCHECK(hipMemcpy(h.data(), ctx->devStats.p, kStatsSlots * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (int i = 0; i < n; ++i) cycles[i] = h[kStatsSectionBase + i];
        return 0;
    } catch (const std::exception &e) {
        return Fail(e.what());
    }
}

}  // extern "C"
