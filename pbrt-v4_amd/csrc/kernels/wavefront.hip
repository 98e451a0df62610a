// MI355X wavefront kernels for pbrt's WavefrontPathIntegrator hot path.
//
// Stage <-> reference mapping:
//   k_camera          GenerateCameraRays<HaltonSampler> (wavefront/camera.cpp:31-80)
//   k_closest         WavefrontAggregate::IntersectClosest + EnqueueWorkAfterIntersection/Miss
//                     (wavefront/intersect.h:16-156), escaped rays (integrator.cpp:495-537)
//   k_shade_diffuse   HandleEmissiveIntersection (integrator.cpp:539-573) fused with
//                     GenerateRaySamples (samples.cpp:29-66) and
//                     EvaluateMaterialAndBSDF<DiffuseMaterial> (surfscatter.cpp:57-328)
//   k_shadow          IntersectShadow + RecordShadowRayResult (intersect.h:31-46)
//   k_film            UpdateFilm / RGBFilm::AddSample (wavefront/film.cpp:13-39, film.h:241-258)
//
// Queues are compacted with one wave64 ballot + one atomic per wave; per-material streams
// are separate queues (one per material tag present).  Launches are grid-stride over the
// device-side queue counters so the host never synchronises inside the render loop.
#include <hip/hip_runtime.h>

#include "device.h"

namespace pbrt_amd {

constexpr int kBlock = 256;
constexpr float kInvWavelengthPDF = kLambdaMax - kLambdaMin;  // 1 / SampleUniformWavelengths pdf

// ------------------------------------------------------------------ helpers
__device__ inline int WavePush(int *counter, bool pred) {
    unsigned long long mask = __ballot(pred);
    if (mask == 0) return -1;
    int lane = __lane_id();
    int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader);
    return pred ? base + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

__device__ inline V3 XfPoint(const float *m, V3 p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1) return V3(xp, yp, zp);
    return V3(xp, yp, zp) / wp;
}
__device__ inline V3 XfVector(const float *m, V3 v) {
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}

struct Halton {
    uint64_t index;
    int dimension;
};

__device__ inline Halton StartPixelSample(const DeviceScene &S, int px, int py, int sampleIndex, int dim) {
    // samplers.h:53-71
    Halton h;
    h.index = 0;
    uint64_t sampleStride = (uint64_t)S.baseScales[0] * S.baseScales[1];
    if (sampleStride > 1) {
        int pmx = px % 128, pmy = py % 128;
        if (pmx < 0) pmx += 128;
        if (pmy < 0) pmy += 128;
        h.index += InverseRadicalInverse((uint64_t)pmx, 2, S.baseExponents[0]) * (sampleStride / S.baseScales[0]) *
                   (uint64_t)S.multInverse[0];
        h.index += InverseRadicalInverse((uint64_t)pmy, 3, S.baseExponents[1]) * (sampleStride / S.baseScales[1]) *
                   (uint64_t)S.multInverse[1];
        h.index %= sampleStride;
    }
    h.index += (uint64_t)sampleIndex * sampleStride;
    h.dimension = dim < 2 ? 2 : dim;
    return h;
}
__device__ inline float SampleDim(const DeviceScene &S, uint64_t index, int dim) {
    if ((index >> 32) == 0) {  // 32-bit digit extraction: same digits, division by multiply
        const uint4 hd = S.haltonDim[dim];
        return ScrambledRadicalInverse32Magic(hd.x, hd.y & 0xffu, hd.w, hd.y >> 8, (uint32_t)index, S.perm + hd.z);
    }
    return ScrambledRadicalInverse(S.permBase[dim], S.permNDigits[dim], index, S.perm + S.permOffset[dim]);
}
__device__ inline float Get1D(const DeviceScene &S, Halton &h) {
    if (h.dimension >= S.nDims) h.dimension = 2;
    return SampleDim(S, h.index, h.dimension++);
}
__device__ inline void Get2D(const DeviceScene &S, Halton &h, float *u0, float *u1) {
    if (h.dimension + 1 >= S.nDims) h.dimension = 2;
    int dim = h.dimension;
    h.dimension += 2;
    *u0 = SampleDim(S, h.index, dim);
    *u1 = SampleDim(S, h.index, dim + 1);
}

__device__ inline void PixelOf(const PathState &st, int slot, int *px, int *py, int *sampleIndex) {
    int s = slot / st.P, pl = slot - s * st.P;
    int r = pl / st.width;
    *px = pl - r * st.width;
    *py = st.rows[r];
    *sampleIndex = st.firstSample + s;
}

// ------------------------------------------------------------------ BVH8 traversal
// One ray per lane.  The node's 8 child boxes are read as 12 float4 loads (SoA inside the
// 256-byte node), the 8 slab tests run fully unrolled in registers, leaves are intersected
// nearest-first and interior children are pushed farthest-first onto a per-lane stack that
// lives in LDS ([depth][lane] layout: consecutive lanes hit consecutive banks), so nothing
// spills to scratch.  Box test = Bounds3::IntersectP (util/vecmath.h:1576-1611) including the
// 1 + 2 gamma(3) far-plane slack; triangle test = IntersectTriangle (shapes.cpp:172-273).
// Stack entries per lane = DeviceScene::stackSize (the BVH's exact worst case, host-computed,
// at most kMaxStackSize), allocated as dynamic LDS at launch so small scenes keep occupancy.

struct RayPre {
    V3 o, invDir;
    int neg[3];
};

__device__ inline void SlabTest4(const float4 *__restrict__ q, int g, const RayPre &r, float raytMax, float tn[8],
                                 unsigned *mask) {
    // children 4g..4g+3: lox,loy,loz at float4 index 2a+g, hix,hiy,hiz at 6+2a+g
    float4 L[3], H[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        L[a] = q[2 * a + g];
        H[a] = q[6 + 2 * a + g];
    }
    const float slack = 1 + 2 * gamma(3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float lo[3], hi[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = k == 0 ? L[a].x : k == 1 ? L[a].y : k == 2 ? L[a].z : L[a].w;
            hi[a] = k == 0 ? H[a].x : k == 1 ? H[a].y : k == 2 ? H[a].z : H[a].w;
        }
        float nx = r.neg[0] ? hi[0] : lo[0], fx = r.neg[0] ? lo[0] : hi[0];
        float ny = r.neg[1] ? hi[1] : lo[1], fy = r.neg[1] ? lo[1] : hi[1];
        float nz = r.neg[2] ? hi[2] : lo[2], fz = r.neg[2] ? lo[2] : hi[2];
        float tMin = (nx - r.o.x) * r.invDir.x;
        float tMax = (fx - r.o.x) * r.invDir.x * slack;
        float tyMin = (ny - r.o.y) * r.invDir.y;
        float tyMax = (fy - r.o.y) * r.invDir.y * slack;
        bool ok = !(tMin > tyMax || tyMin > tMax);
        tMin = tyMin > tMin ? tyMin : tMin;
        tMax = tyMax < tMax ? tyMax : tMax;
        float tzMin = (nz - r.o.z) * r.invDir.z;
        float tzMax = (fz - r.o.z) * r.invDir.z * slack;
        ok = ok && !(tMin > tzMax || tzMin > tMax);
        tMin = tzMin > tMin ? tzMin : tMin;
        tMax = tzMax < tMax ? tzMax : tMax;
        ok = ok && (tMin < raytMax) && (tMax > 0);
        tn[4 * g + k] = tMin;
        *mask |= ok ? (1u << (4 * g + k)) : 0u;
    }
}

__device__ inline void SlabTest8(const BVH8Node *__restrict__ np, const RayPre &r, float raytMax, float tn[8],
                                 unsigned *mask) {
    const float4 *q = reinterpret_cast<const float4 *>(np);
    *mask = 0;
    SlabTest4(q, 0, r, raytMax, tn, mask);
    SlabTest4(q, 1, r, raytMax, tn, mask);
}

template <bool AnyHit>
__device__ inline int Traverse(const DeviceScene &S, V3 o, V3 d, float tMax, TriHit *best, int *lds) {
    const TriRay tr = MakeTriRay(o, d);
    RayPre r;
    r.o = o;
    r.invDir = V3(1 / d.x, 1 / d.y, 1 / d.z);
    r.neg[0] = r.invDir.x < 0;
    r.neg[1] = r.invDir.y < 0;
    r.neg[2] = r.invDir.z < 0;
    const int lane = threadIdx.x, stride = blockDim.x;
    int sp = 0;
    int node = 0;
    int hitPrim = -1;
    while (true) {
        const BVH8Node *np = S.nodes + node;
        float tn[8];
        unsigned mask;
        SlabTest8(np, r, tMax, tn, &mask);
        // empty slots carry an inverted box, so they never pass the slab test
        unsigned leaves = 0, inner = 0;
        int4 ch0 = reinterpret_cast<const int4 *>(np->child)[0], ch1 = reinterpret_cast<const int4 *>(np->child)[1];
        int ch[8] = {ch0.x, ch0.y, ch0.z, ch0.w, ch1.x, ch1.y, ch1.z, ch1.w};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            if (mask & (1u << c)) {
                if (ch[c] < 0) leaves |= 1u << c;
                else inner |= 1u << c;
            }
        }
        // leaves nearest-first
        while (leaves) {
            int bc = 0;
            float bt = kInfinity;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if ((leaves & (1u << c)) && tn[c] <= bt) {
                    bt = tn[c];
                    bc = c;
                }
            leaves &= ~(1u << bc);
            if (bt >= tMax) continue;
            int enc = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) enc = (c == bc) ? ~ch[c] : enc;
            int first = enc >> 3, count = (enc & 7) + 1;
            for (int t = first; t < first + count; ++t) {
                float4 a = S.triVerts[3 * t], b = S.triVerts[3 * t + 1], c = S.triVerts[3 * t + 2];
                TriHit h;
                if (IntersectTriangleRay(tr, tMax, V3(a.x, a.y, a.z), V3(b.x, b.y, b.z), V3(c.x, c.y, c.z), &h)) {
                    if (AnyHit) return t;
                    tMax = h.t;
                    *best = h;
                    hitPrim = t;
                }
            }
        }
        // interior children farthest-first onto the stack (closest popped next)
        while (inner) {
            int bc = 0;
            float bt = -kInfinity;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if ((inner & (1u << c)) && tn[c] >= bt) {
                    bt = tn[c];
                    bc = c;
                }
            inner &= ~(1u << bc);
            if (bt >= tMax) continue;
            int child = 0;
#pragma unroll
            for (int c = 0; c < 8; ++c) child = (c == bc) ? ch[c] : child;
            lds[(sp++) * stride + lane] = child;  // sp < S.stackSize by construction
        }
        if (sp == 0) break;
        node = lds[(--sp) * stride + lane];
    }
    return hitPrim;
}

// ------------------------------------------------------------------ lights
struct LightSample {
    float Le[kNSpectrumSamples];
    V3 wi, p, pErr, n;
    float pdf;
};

// Triangle geometry of a leaf-order prim
__device__ inline void PrimVerts(const DeviceScene &S, int prim, V3 *p0, V3 *p1, V3 *p2) {
    float4 a = S.triVerts[3 * prim], b = S.triVerts[3 * prim + 1], c = S.triVerts[3 * prim + 2];
    *p0 = V3(a.x, a.y, a.z);
    *p1 = V3(b.x, b.y, b.z);
    *p2 = V3(c.x, c.y, c.z);
}

__device__ inline float TriArea(V3 p0, V3 p1, V3 p2) { return 0.5f * Length(Cross(p1 - p0, p2 - p0)); }

__device__ inline float SolidAngleOf(V3 p0, V3 p1, V3 p2, V3 p) {
    return SphericalTriangleArea(Normalize(p0 - p), Normalize(p1 - p), Normalize(p2 - p));
}

// Triangle::Sample(ctx, u) (shapes.h:1053-1130); returns false for {}
__device__ inline bool SampleTriangle(V3 p0, V3 p1, V3 p2, bool flip, V3 refP, V3 refN, V3 refNs, float u0,
                                      float u1, V3 *ps, V3 *pErr, V3 *ns, float *pdfOut) {
    (void)refN;
    float solidAngle = SolidAngleOf(p0, p1, p2, refP);
    if (solidAngle < kMinSphericalSampleArea || solidAngle > kMaxSphericalSampleArea) {
        float b[3];
        SampleUniformTriangle(u0, u1, b);
        V3 p = b[0] * p0 + b[1] * p1 + b[2] * p2;
        V3 n = Normalize(Cross(p1 - p0, p2 - p0));
        if (flip) n = n * -1.f;
        V3 pAbsSum = Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2);
        ToPoint3fi(p, gamma(6) * pAbsSum, &p, pErr);
        float pdf = 1 / TriArea(p0, p1, p2);
        V3 wi = p - refP;
        if (LengthSquared(wi) == 0) return false;
        wi = Normalize(wi);
        pdf /= AbsDotN(n, -wi) / DistanceSquared(refP, p);
        if (isinf(pdf)) return false;
        *ps = p;
        *ns = n;
        *pdfOut = pdf;
        return true;
    }
    float pdf = 1;
    if (refNs != V3(0, 0, 0)) {
        V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
        float w[4] = {fmaxf(0.01f, AbsDotN(refNs, wi1)), fmaxf(0.01f, AbsDotN(refNs, wi1)),
                      fmaxf(0.01f, AbsDotN(refNs, wi0)), fmaxf(0.01f, AbsDotN(refNs, wi2))};
        float px, py;
        SampleBilinear(u0, u1, w, &px, &py);
        u0 = px;
        u1 = py;
        pdf = BilinearPDF(u0, u1, w);
    }
    float triPDF;
    float b[3];
    SampleSphericalTriangle(p0, p1, p2, refP, u0, u1, b, &triPDF);
    if (triPDF == 0) return false;
    pdf *= triPDF;
    V3 pAbsSum = Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2);
    V3 p;
    ToPoint3fi(b[0] * p0 + b[1] * p1 + b[2] * p2, gamma(6) * pAbsSum, &p, pErr);
    V3 n = Normalize(Cross(p1 - p0, p2 - p0));
    if (flip) n = n * -1.f;
    *ps = p;
    *ns = n;
    *pdfOut = pdf;
    return true;
}

// Triangle::PDF(ctx, wi) (shapes.h:1133-1174)
__device__ inline float TrianglePDF(const DeviceScene &S, int prim, V3 refP, V3 refPErr, V3 refN, V3 refNs, V3 wi) {
    V3 p0, p1, p2;
    PrimVerts(S, prim, &p0, &p1, &p2);
    float solidAngle = SolidAngleOf(p0, p1, p2, refP);
    if (solidAngle < kMinSphericalSampleArea || solidAngle > kMaxSphericalSampleArea) {
        // ShapeSampleContext::SpawnRay(wi) then Triangle::Intersect
        V3 o = OffsetRayOrigin(refP, refPErr, refN, wi);
        TriHit h;
        if (!IntersectTriangle(o, wi, kInfinity, p0, p1, p2, &h)) return 0;
        TriSurface hs = TriangleSurface(p0, p1, p2, h.b0, h.b1, h.b2, S.primFlip[prim]);
        V3 pHit = hs.p, n = hs.n;
        float pdf = (1 / TriArea(p0, p1, p2)) / (AbsDotN(n, -wi) / DistanceSquared(refP, pHit));
        if (isinf(pdf)) pdf = 0;
        return pdf;
    }
    float pdf = 1 / solidAngle;
    if (refNs != V3(0, 0, 0)) {
        float u0, u1;
        InvertSphericalTriangleSample(p0, p1, p2, refP, wi, &u0, &u1);
        V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
        float w[4] = {fmaxf(0.01f, AbsDotN(refNs, wi1)), fmaxf(0.01f, AbsDotN(refNs, wi1)),
                      fmaxf(0.01f, AbsDotN(refNs, wi0)), fmaxf(0.01f, AbsDotN(refNs, wi2))};
        pdf *= BilinearPDF(u0, u1, w);
    }
    return pdf;
}

// BVHLightSampler::Sample / PMF (lightsamplers.h:266-403) and UniformLightSampler
// light index convention: [0, nAreaLights) area lights, then infinite lights.
__device__ inline bool SampleLight(const DeviceScene &S, V3 p, V3 ns, float u, int *light, float *pmfOut) {
    int nAll = S.nAreaLights + S.nInfinite;
    if (S.uniformLightSampler) {
        if (nAll == 0) return false;
        int li = min((int)(u * nAll), nAll - 1);
        *light = li;
        *pmfOut = 1.f / nAll;
        return true;
    }
    float pInfinite = float(S.nInfinite) / float(S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    if (u < pInfinite) {
        u /= pInfinite;
        int index = min((int)(u * S.nInfinite), S.nInfinite - 1);
        *pmfOut = pInfinite / S.nInfinite;
        *light = S.nAreaLights + index;
        return true;
    }
    if (S.nLightNodes == 0) return false;
    u = fminf((u - pInfinite) / (1 - pInfinite), kOneMinusEpsilon);
    int nodeIndex = 0;
    float pmf = 1 - pInfinite;
    for (int iter = 0; iter < 4 * kMaxLightBVHDepth; ++iter) {
        DeviceLightNode node = S.lightNodes[nodeIndex];
        if (!node.isLeaf) {
            float c0 = LightImportance(S.lightNodes[nodeIndex + 1].b, p, ns);
            float c1 = LightImportance(S.lightNodes[node.childOrLight].b, p, ns);
            if (c0 == 0 && c1 == 0) return false;
            float nodePMF;
            int child = SampleDiscrete2(c0, c1, u, &nodePMF, &u);
            pmf *= nodePMF;
            nodeIndex = (child == 0) ? (nodeIndex + 1) : node.childOrLight;
        } else {
            if (nodeIndex > 0 || LightImportance(node.b, p, ns) > 0) {
                *light = node.childOrLight;
                *pmfOut = pmf;
                return true;
            }
            return false;
        }
    }
    return false;
}

__device__ inline float LightPMF(const DeviceScene &S, V3 p, V3 ns, int light) {
    int nAll = S.nAreaLights + S.nInfinite;
    if (S.uniformLightSampler) return nAll ? 1.f / nAll : 0.f;
    uint32_t bitTrail = light < S.nAreaLights ? S.lightBitTrail[light] : 0xffffffffu;
    if (bitTrail == 0xffffffffu) return 1.f / (S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    float pInfinite = float(S.nInfinite) / float(S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    float pmf = 1 - pInfinite;
    int nodeIndex = 0;
    for (int iter = 0; iter < kMaxLightBVHDepth; ++iter) {
        const DeviceLightNode &node = S.lightNodes[nodeIndex];
        if (node.isLeaf) return pmf;
        float c0 = LightImportance(S.lightNodes[nodeIndex + 1].b, p, ns);
        float c1 = LightImportance(S.lightNodes[node.childOrLight].b, p, ns);
        pmf *= ((bitTrail & 1) ? c1 : c0) / (c0 + c1);
        nodeIndex = (bitTrail & 1) ? node.childOrLight : (nodeIndex + 1);
        bitTrail >>= 1;
    }
    return pmf;
}

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(kBlock) k_camera(DeviceScene S, PathState st, int nActive) {
    int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot == 0) {
        st.counters[0] = nActive;  // depth-0 ray queue = every slot
        atomicAdd(&st.stats[0], (unsigned long long)nActive);
    }
    if (slot >= nActive) return;
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    Halton h = StartPixelSample(S, px, py, sampleIndex, 0);
    float lu = Get1D(S, h);
    float lambda0 = Lerpf(lu, kLambdaMin, kLambdaMax);
    // GetCameraSample (samplers.h:797-813) with the box filter (filters.h:67-71)
    float pix0 = RadicalInverse(2, h.index >> S.baseExponents[0]);
    float pix1 = RadicalInverse(3, h.index / (uint64_t)S.baseScales[1]);
    float fx = Lerpf(pix0, -S.filterRadiusX, S.filterRadiusX), fy = Lerpf(pix1, -S.filterRadiusY, S.filterRadiusY);
    float pFilmX = px + fx + 0.5f, pFilmY = py + fy + 0.5f;
    float time = Get1D(S, h);
    (void)time;
    float l0, l1;
    Get2D(S, h, &l0, &l1);
    // PerspectiveCamera::GenerateRay (cameras.cpp:433-456)
    V3 pCamera = XfPoint(S.cameraFromRaster, V3(pFilmX, pFilmY, 0));
    V3 o(0, 0, 0), d = Normalize(pCamera);
    if (S.lensRadius > 0) {
        float lx, ly;
        SampleUniformDiskConcentric(l0, l1, &lx, &ly);
        lx *= S.lensRadius;
        ly *= S.lensRadius;
        float ft = S.focalDistance / d.z;
        V3 pFocus = o + d * ft;
        o = V3(lx, ly, 0);
        d = Normalize(pFocus - o);
    }
    // CameraBase::RenderFromCamera(ray): Transform::operator()(Ray) with origin error offset
    {
        const float *m = S.renderFromCamera;
        V3 oo = XfPoint(m, o);
        V3 err;
        if (o == V3(0, 0, 0))
            err = gamma(3) * Abs(V3(m[3], m[7], m[11]));
        else
            err = gamma(3) * (Abs(V3(m[0] * o.x, m[4] * o.x, m[8] * o.x)) + Abs(V3(m[1] * o.y, m[5] * o.y, m[9] * o.y)) +
                              Abs(V3(m[2] * o.z, m[6] * o.z, m[10] * o.z)) + Abs(V3(m[3], m[7], m[11])));
        V3 dd = XfVector(m, d);
        float l2 = LengthSquared(dd);
        if (l2 > 0) {
            float dt = Dot(Abs(dd), err) / l2;
            oo = oo + dd * dt;
        }
        o = oo;
        d = dd;
    }
    int N = st.N;
    for (int i = 0; i < kNSpectrumSamples; ++i) st.beta[i * N + slot] = 1.f;
    st.rl[slot] = 1.f;
    st.L[slot] = 0;
    st.L[N + slot] = 0;
    st.L[2 * N + slot] = 0;
    st.lambda0[slot] = lambda0;
    st.filterW[slot] = 1.f;
    st.etaScale[slot] = 1.f;
    st.flags[slot] = 0;
    st.ray[slot] = o.x;
    st.ray[N + slot] = o.y;
    st.ray[2 * N + slot] = o.z;
    st.ray[3 * N + slot] = d.x;
    st.ray[4 * N + slot] = d.y;
    st.ray[5 * N + slot] = d.z;
    st.rayQ[0][slot] = slot;
}

__global__ void __launch_bounds__(kBlock) k_closest(DeviceScene S, PathState st, int depth) {
    extern __shared__ int stackLds[];
    int N = st.N;
    const int *q = st.rayQ[depth & 1];
    const int count = st.counters[depth * 4 + 0];
    int *matCounter = &st.counters[depth * 4 + 1];
    int *escCounter = &st.counters[depth * 4 + 3];
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[1], (unsigned long long)count);
    for (int base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        int qi = base + threadIdx.x;
        bool active = qi < count;
        int slot = active ? q[qi] : 0;
        int prim = -1;
        TriHit h;
        V3 o, d;
        if (active) {
            o = V3(st.ray[slot], st.ray[N + slot], st.ray[2 * N + slot]);
            d = V3(st.ray[3 * N + slot], st.ray[4 * N + slot], st.ray[5 * N + slot]);
            prim = Traverse<false>(S, o, d, kInfinity, &h, stackLds);
            if (prim >= 0) {
                st.hitPrim[slot] = prim;
                st.hitB[slot] = h.b0;
                st.hitB[N + slot] = h.b1;
                st.hitB[2 * N + slot] = h.b2;
                st.hitB[3 * N + slot] = h.t;
            }
        }
        if (S.nInfinite > 0) {
            int epos = WavePush(escCounter, active && prim < 0);
            if (epos >= 0) st.escQ[epos] = slot;
        }
        int pos = WavePush(matCounter, active && prim >= 0);
        if (pos >= 0) st.matQ[pos] = slot;
    }
}

// HandleEscapedRays (integrator.cpp:495-537) for UniformInfiniteLight: Le with MIS where
// PDF_Li(allowIncompletePDF = true) == 0, so r_l contributes nothing.
__global__ void __launch_bounds__(kBlock) k_escaped(DeviceScene S, PathState st, int depth) {
    int N = st.N;
    const int count = st.counters[depth * 4 + 3];
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < count; qi += gridDim.x * blockDim.x) {
        int slot = st.escQ[qi];
        int fl = st.flags[slot];
        float rl = st.rl[slot];
        float denom = (depth == 0 || (fl & 1)) ? Avg31(1.f) : Avg31(1.f + rl * 0.f);
        const float invDenom = 1 / denom;
        float rgb[3] = {0, 0, 0};
        bool any = false;
        for (int li = 0; li < S.nInfinite; ++li) {
            const float *dense = S.dense + S.infSpectrum[li] * kDenseN;
            float scale = S.infScale[li];
            float sx = 0, sy = 0, sz = 0, lam = st.lambda0[slot];
            bool nz = false;
            for (int i = 0; i < kNSpectrumSamples; ++i) {
                if (i > 0) {
                    lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
                    if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
                }
                int off = DenseOffset(lam);
                float Le = scale * (off < 0 ? 0.f : dense[off]);
                nz |= Le != 0;
                float v = (st.beta[i * N + slot] * Le * invDenom) * kInvWavelengthPDF;
                float xb = off < 0 ? 0.f : S.sensor[off], yb = off < 0 ? 0.f : S.sensor[kDenseN + off],
                      zb = off < 0 ? 0.f : S.sensor[2 * kDenseN + off];
                sx = i == 0 ? xb * v : sx + xb * v;
                sy = i == 0 ? yb * v : sy + yb * v;
                sz = i == 0 ? zb * v : sz + zb * v;
            }
            if (!nz) continue;
            any = true;
            rgb[0] += S.imagingRatio * (sx / kNSpectrumSamples);
            rgb[1] += S.imagingRatio * (sy / kNSpectrumSamples);
            rgb[2] += S.imagingRatio * (sz / kNSpectrumSamples);
        }
        if (any) {
            st.L[slot] += rgb[0];
            st.L[N + slot] += rgb[1];
            st.L[2 * N + slot] += rgb[2];
        }
    }
}

// Streaming form of the per-wavelength work: lambda_i, R_i, Le_i and beta_i are produced
// inside each 31-iteration loop (lambda by pbrt's sequential +10 nm recurrence, R by the
// sigmoid polynomial, beta re-read from the wavelength-major SoA through L1/L2) instead of
// being held in 31-entry register arrays, which keeps the kernel at a few waves per SIMD.
struct SpectralIter {
    float lam;
    int i;
    __device__ SpectralIter(float l0) : lam(l0), i(0) {}
    __device__ void Next() {
        lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
        if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
        ++i;
    }
};

__device__ inline float Reflectance(float4 mc, bool constant, float lambda) {
    float r = constant ? mc.w : SigmoidPolynomial(mc.x, mc.y, mc.z, lambda);
    return Clampf(r, 0, 1);
}

// ToSensorRGB accumulation for one wavelength: sx += xbar * (c / pdf) (film.h:95-100)
// Film-only arithmetic (the contribution c and its 1/pdf, 1/denom scalings) uses reciprocal
// multiplies where the reference divides: at most an ulp or two per term in the pixel sums,
// and nothing that steers a path (beta, pdfs and RR keep the reference's exact operations).
struct SensorAcc {
    float sx = 0, sy = 0, sz = 0;
    __device__ void Add(const DeviceScene &S, int off, float c, bool first) {
        float v = c * kInvWavelengthPDF;
        float4 sb = off < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : S.sensor4[off];
        float xb = sb.x, yb = sb.y, zb = sb.z;
        sx = first ? xb * v : sx + xb * v;
        sy = first ? yb * v : sy + yb * v;
        sz = first ? zb * v : sz + zb * v;
    }
};

__global__ void __launch_bounds__(kBlock) k_shade_diffuse(DeviceScene S, PathState st, int depth) {
    __shared__ float bfLds[kNSpectrumSamples * kBlock];  // [lambda][lane]: conflict-free
    int N = st.N;
    const int count = st.counters[depth * 4 + 1];
    int *nextCounter = &st.counters[(depth + 1) * 4 + 0];
    int *shadowCounter = &st.counters[depth * 4 + 2];
    int *nextQ = st.rayQ[(depth + 1) & 1];
    for (int base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        int qi = base + threadIdx.x;
        bool active = qi < count;
        bool pushRay = false, pushShadow = false;
        int slot = active ? st.matQ[qi] : 0;
        if (active) {
            const float lambda0 = st.lambda0[slot];
            const float *betaP = st.beta + slot;
            int prim = st.hitPrim[slot];
            float b0 = st.hitB[slot], b1 = st.hitB[N + slot], b2 = st.hitB[2 * N + slot];
            V3 rd(st.ray[3 * N + slot], st.ray[4 * N + slot], st.ray[5 * N + slot]);
            V3 p0, p1, p2;
            PrimVerts(S, prim, &p0, &p1, &p2);
            TriSurface surf = TriangleSurface(p0, p1, p2, b0, b1, b2, S.primFlip[prim]);
            V3 wo = Normalize(-rd);
            V3 n = surf.n, ns = surf.n;
            int fl = st.flags[slot];
            float rl = st.rl[slot];
            float Lr = 0, Lg = 0, Lb = 0;
            // ---- HandleEmissiveIntersection (integrator.cpp:539-573)
            int light = S.primLight[prim];
            if (light >= 0 && (S.lightTwoSided[light] || DotN(n, wo) >= 0)) {
                float denom;
                if (depth == 0 || (fl & 1)) {
                    denom = Avg31(1.f);
                } else {
                    V3 cp(st.ctx[slot], st.ctx[N + slot], st.ctx[2 * N + slot]);
                    V3 cn(st.ctx[3 * N + slot], st.ctx[4 * N + slot], st.ctx[5 * N + slot]);
                    V3 cns(st.ctx[6 * N + slot], st.ctx[7 * N + slot], st.ctx[8 * N + slot]);
                    V3 cpe(st.ctx[9 * N + slot], st.ctx[10 * N + slot], st.ctx[11 * N + slot]);
                    float lightChoicePDF = LightPMF(S, cp, cns, light);
                    float lightPDF = lightChoicePDF * TrianglePDF(S, S.lightPrim[light], cp, cpe, cn, cns, -wo);
                    denom = Avg31(1.f + rl * lightPDF);
                }
                const float *dense = S.dense + S.lightSpectrum[light] * kDenseN;
                float scale = S.lightScale[light];
                SensorAcc acc;
                const float invDenom = 1 / denom;
#pragma unroll 4
                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                    int off = DenseOffset(it.lam);
                    float Le = scale * (off < 0 ? 0.f : dense[off]);
                    acc.Add(S, off, betaP[it.i * N] * Le * invDenom, it.i == 0);
                }
                Lr = S.imagingRatio * (acc.sx / kNSpectrumSamples);
                Lg = S.imagingRatio * (acc.sy / kNSpectrumSamples);
                Lb = S.imagingRatio * (acc.sz / kNSpectrumSamples);
            }
            if (depth < S.maxDepth) {
                // ---- GenerateRaySamples (samples.cpp:29-66): dimension = 6 + 7 * depth
                int px, py, sampleIndex;
                PixelOf(st, slot, &px, &py, &sampleIndex);
                px += S.px0;
                Halton h = StartPixelSample(S, px, py, sampleIndex, 6 + 7 * depth);
                float dUc = Get1D(S, h);
                float dU0, dU1;
                Get2D(S, h, &dU0, &dU1);
                (void)Get1D(S, h);  // indirect.uc (unused by DiffuseBxDF)
                float iU0, iU1;
                Get2D(S, h, &iU0, &iU1);
                float rr = Get1D(S, h);
                // ---- DiffuseMaterial::GetBxDF: R = clamp(reflectance(lambda), 0, 1); f = R / pi
                // (bxdfs.h DiffuseBxDF::f).  bf_i = beta_i * f_i is formed once per wavelength
                // into LDS; light sampling and the BSDF update both start from that product.
                int mat = S.primMaterial[prim];
                const float4 mc = S.matCoeffs[mat];
                const bool constant = S.matConstant[mat];
                bool Rnz = false;
                float *bf = bfLds + threadIdx.x;
#pragma unroll 4
                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                    float R = Reflectance(mc, constant, it.lam);
                    Rnz |= R != 0;
                    bf[it.i * kBlock] = betaP[it.i * N] * (R * kInvPi);
                }
                Frame frame = Frame::FromXZ(Normalize(surf.dpdu), ns);
                V3 woL = frame.ToLocal(wo);
                V3 pi = surf.p, pe = surf.pErr;
                // ---- light sampling + shadow ray (surfscatter.cpp:254-326); reads the old beta
                if (Rnz) {
                    V3 cp = OffsetRayOrigin(pi, pe, n, wo);  // reflective, not transmissive
                    int li;
                    float lpmf;
                    if (SampleLight(S, cp, ns, dUc, &li, &lpmf) && li < S.nAreaLights) {
                        int lprim = S.lightPrim[li];
                        V3 q0, q1, q2;
                        PrimVerts(S, lprim, &q0, &q1, &q2);
                        V3 lp, lpe, ln;
                        float lpdf;
                        if (SampleTriangle(q0, q1, q2, S.primFlip[lprim], cp, n, ns, dU0, dU1, &lp, &lpe, &ln, &lpdf) &&
                            lpdf != 0 && LengthSquared(lp - cp) != 0) {
                            V3 wi = Normalize(lp - cp);
                            V3 wiL = frame.ToLocal(wi);
                            if ((S.lightTwoSided[li] || DotN(ln, -wi) >= 0) && woL.z != 0 && woL.z * wiL.z > 0) {
                                const float *dense = S.dense + S.lightSpectrum[li] * kDenseN;
                                float scale = S.lightScale[li];
                                float absdot = AbsDotN(ns, wi);
                                float lightPDF = lpdf * lpmf;
                                float bsdfPDF = CosineHemispherePDF(fabsf(wiL.z));
                                float denom = Avg31(bsdfPDF + lightPDF);
                                const float invDenom = 1 / denom;
                                SensorAcc acc;
                                bool nz = false;
#pragma unroll 4
                                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                                    int off = DenseOffset(it.lam);
                                    float Le = scale * (off < 0 ? 0.f : dense[off]);
                                    nz |= Le != 0;
                                    acc.Add(S, off, bf[it.i * kBlock] * absdot * Le * invDenom, it.i == 0);
                                }
                                if (nz) {
                                    // SpawnRayTo(pi, n, time, pLight.pi, pLight.n) (ray.h:106-111)
                                    V3 pf = OffsetRayOrigin(pi, pe, n, lp - pi);
                                    V3 pt = OffsetRayOrigin(lp, lpe, ln, pf - lp);
                                    V3 sd = pt - pf;
                                    st.shadowRay[slot] = pf.x;
                                    st.shadowRay[N + slot] = pf.y;
                                    st.shadowRay[2 * N + slot] = pf.z;
                                    st.shadowRay[3 * N + slot] = sd.x;
                                    st.shadowRay[4 * N + slot] = sd.y;
                                    st.shadowRay[5 * N + slot] = sd.z;
                                    st.shadowL[slot] = S.imagingRatio * (acc.sx / kNSpectrumSamples);
                                    st.shadowL[N + slot] = S.imagingRatio * (acc.sy / kNSpectrumSamples);
                                    st.shadowL[2 * N + slot] = S.imagingRatio * (acc.sz / kNSpectrumSamples);
                                    pushShadow = true;
                                }
                            }
                        }
                    }
                }
                // ---- BSDF::Sample_f<DiffuseBxDF> + RR + indirect ray (surfscatter.cpp:170-250)
                if (woL.z != 0 && Rnz) {
                    V3 wiL = SampleCosineHemisphere(iU0, iU1);
                    if (woL.z < 0) wiL.z *= -1;
                    float pdf = CosineHemispherePDF(fabsf(wiL.z));
                    if (pdf != 0 && wiL.z != 0) {
                        V3 wi = frame.FromLocal(wiL);
                        float absdot = AbsDotN(ns, wi);
                        float etaScale = st.etaScale[slot];
                        float avgRu = Avg31(1.f);
                        float mx = -kInfinity;
#pragma unroll 4
                        for (int i = 0; i < kNSpectrumSamples; ++i) {
                            float nbv = bf[i * kBlock] * absdot / pdf;
                            bf[i * kBlock] = nbv;
                            mx = fmaxf(mx, nbv * etaScale / avgRu);
                        }
                        bool kill = false;
                        float q = 0;
                        if (mx < 1 && depth >= 1) {
                            q = fmaxf(0.f, 1 - mx);
                            kill = rr < q;
                        }
                        if (!kill) {
                            bool rrScale = mx < 1 && depth >= 1;
                            bool nz = false;
                            float *betaW = st.beta + slot;
#pragma unroll 4
                            for (int i = 0; i < kNSpectrumSamples; ++i) {
                                float nbv = bf[i * kBlock];
                                if (rrScale) nbv /= 1 - q;
                                nz |= nbv != 0;
                                betaW[i * N] = nbv;
                            }
                            if (nz) {
                                V3 ro = OffsetRayOrigin(pi, pe, n, wi);
                                pushRay = true;
                                st.ray[slot] = ro.x;
                                st.ray[N + slot] = ro.y;
                                st.ray[2 * N + slot] = ro.z;
                                st.ray[3 * N + slot] = wi.x;
                                st.ray[4 * N + slot] = wi.y;
                                st.ray[5 * N + slot] = wi.z;
                                st.rl[slot] = 1.f / pdf;
                                st.flags[slot] = 2;  // specularBounce = false, anyNonSpecular = true
                                st.ctx[slot] = pi.x;
                                st.ctx[N + slot] = pi.y;
                                st.ctx[2 * N + slot] = pi.z;
                                st.ctx[3 * N + slot] = n.x;
                                st.ctx[4 * N + slot] = n.y;
                                st.ctx[5 * N + slot] = n.z;
                                st.ctx[6 * N + slot] = ns.x;
                                st.ctx[7 * N + slot] = ns.y;
                                st.ctx[8 * N + slot] = ns.z;
                                st.ctx[9 * N + slot] = pe.x;
                                st.ctx[10 * N + slot] = pe.y;
                                st.ctx[11 * N + slot] = pe.z;
                            }
                        }
                    }
                }
            }
            if (Lr != 0 || Lg != 0 || Lb != 0) {
                st.L[slot] += Lr;
                st.L[N + slot] += Lg;
                st.L[2 * N + slot] += Lb;
            }
        }
        int pos = WavePush(nextCounter, pushRay);
        if (pos >= 0) nextQ[pos] = slot;
        int spos = WavePush(shadowCounter, pushShadow);
        if (spos >= 0) st.shadowQ[spos] = slot;
    }
}

__global__ void __launch_bounds__(kBlock) k_shadow(DeviceScene S, PathState st, int depth) {
    extern __shared__ int stackLds[];
    int N = st.N;
    const int count = st.counters[depth * 4 + 2];
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[2], (unsigned long long)count);
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < count; qi += gridDim.x * blockDim.x) {
        int slot = st.shadowQ[qi];
        V3 o(st.shadowRay[slot], st.shadowRay[N + slot], st.shadowRay[2 * N + slot]);
        V3 d(st.shadowRay[3 * N + slot], st.shadowRay[4 * N + slot], st.shadowRay[5 * N + slot]);
        TriHit h;
        int hit = Traverse<true>(S, o, d, 1 - kShadowEpsilon, &h, stackLds);
        if (hit < 0) {
            st.L[slot] += st.shadowL[slot];
            st.L[N + slot] += st.shadowL[N + slot];
            st.L[2 * N + slot] += st.shadowL[2 * N + slot];
        }
    }
}

// UpdateFilm: one thread per pixel walks its samples in sample order (deterministic sums)
__global__ void __launch_bounds__(kBlock) k_film(DeviceScene S, PathState st, int nSamples) {
    int pl = blockIdx.x * blockDim.x + threadIdx.x;
    if (pl >= st.P) return;
    int N = st.N;
    int r = pl / st.width;
    int px = S.px0 + (pl - r * st.width), py = st.rows[r];
    size_t pix = (size_t)py * S.xres + px;
    size_t npix = (size_t)S.xres * S.yres;
    double sr = st.film[pix], sg = st.film[npix + pix], sb = st.film[2 * npix + pix], sw = st.film[3 * npix + pix];
    for (int s = 0; s < nSamples; ++s) {
        int slot = s * st.P + pl;
        float w = st.filterW[slot];
        float rr = st.L[slot], gg = st.L[N + slot], bb = st.L[2 * N + slot];
        sr += w * rr;
        sg += w * gg;
        sb += w * bb;
        sw += w;
    }
    st.film[pix] = sr;
    st.film[npix + pix] = sg;
    st.film[2 * npix + pix] = sb;
    st.film[3 * npix + pix] = sw;
}

// ------------------------------------------------------------------ stand-alone intersection
// The WavefrontAggregate boundary exposed on its own (integrator.h:32-54): closest / any hit
// for an SoA ray batch, used by parity tests and the traversal benchmark.
__global__ void __launch_bounds__(kBlock) k_intersect_batch(DeviceScene S, const float *rays, int n, int anyHit,
                                                              int *outPrim, float *outHit) {
    extern __shared__ int stackLds[];
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        V3 o(rays[i], rays[n + i], rays[2 * n + i]);
        V3 d(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
        float tMax = rays[6 * n + i];
        TriHit h{0, 0, 0, 0};
        int prim = anyHit ? Traverse<true>(S, o, d, tMax, &h, stackLds) : Traverse<false>(S, o, d, tMax, &h, stackLds);
        outPrim[i] = prim;
        outHit[i] = h.b0;
        outHit[n + i] = h.b1;
        outHit[2 * n + i] = h.b2;
        outHit[3 * n + i] = h.t;
    }
}

// ------------------------------------------------------------------ launch helpers (host)
static size_t StackBytes(const DeviceScene &S) { return (size_t)(S.stackSize > 0 ? S.stackSize : 1) * kBlock * sizeof(int); }

static int GridFor(int n) {
    int g = (n + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 8192 ? 8192 : g);
}

hipError_t LaunchCamera(const DeviceScene &S, const PathState &st, int nActive, hipStream_t s) {
    hipLaunchKernelGGL(k_camera, dim3((nActive + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, nActive);
    return hipGetLastError();
}
hipError_t LaunchClosest(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_closest, dim3(GridFor(maxCount)), dim3(kBlock), StackBytes(S), s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchEscaped(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_escaped, dim3(GridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadeDiffuse(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_shade_diffuse, dim3(GridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadow(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_shadow, dim3(GridFor(maxCount)), dim3(kBlock), StackBytes(S), s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchFilm(const DeviceScene &S, const PathState &st, int nSamples, hipStream_t s) {
    hipLaunchKernelGGL(k_film, dim3((st.P + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, nSamples);
    return hipGetLastError();
}
hipError_t LaunchIntersectBatch(const DeviceScene &S, const float *rays, int n, int anyHit, int *outPrim,
                                float *outHit, hipStream_t s) {
    hipLaunchKernelGGL(k_intersect_batch, dim3(GridFor(n)), dim3(kBlock), StackBytes(S), s, S, rays, n, anyHit, outPrim, outHit);
    return hipGetLastError();
}

}  // namespace pbrt_amd
