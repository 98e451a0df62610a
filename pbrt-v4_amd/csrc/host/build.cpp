// Scene finalisation: BVH light sampler construction (lightsamplers.cpp:112-236,
// lights.cpp:803-822, lightsamplers.h:95-229) and Halton digit-permutation tables
// (util/lowdiscrepancy.h:25-55, samplers.cpp:32-52).
#include <fstream>
#include <mutex>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <functional>

#include "scene.h"

namespace pbrt_amd {

const std::vector<int> &Primes() {
    // util/primes.cpp: the first 1000 primes
    static std::vector<int> primes = [] {
        std::vector<int> p;
        for (int n = 2; (int)p.size() < 1000; ++n) {
            bool isPrime = true;
            for (int q : p) {
                if (q * q > n) break;
                if (n % q == 0) {
                    isPrime = false;
                    break;
                }
            }
            if (isPrime) p.push_back(n);
        }
        return p;
    }();
    return primes;
}

uint64_t MurmurHash64A(const unsigned char *key, size_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ (len * m);
    const unsigned char *end = key + 8 * (len / 8);
    while (key != end) {
        uint64_t k;
        std::memcpy(&k, key, sizeof(uint64_t));
        key += 8;
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
    }
    switch (len & 7) {
    case 7: h ^= uint64_t(key[6]) << 48; [[fallthrough]];
    case 6: h ^= uint64_t(key[5]) << 40; [[fallthrough]];
    case 5: h ^= uint64_t(key[4]) << 32; [[fallthrough]];
    case 4: h ^= uint64_t(key[3]) << 24; [[fallthrough]];
    case 3: h ^= uint64_t(key[2]) << 16; [[fallthrough]];
    case 2: h ^= uint64_t(key[1]) << 8; [[fallthrough]];
    case 1:
        h ^= uint64_t(key[0]);
        h *= m;
    };
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}


static int NumDigits(int base) {
    // DigitPermutation ctor digit count (float arithmetic, no contraction)
    int nDigits = 0;
    volatile float invBase = (float)1 / (float)base, invBaseM = 1;
    while (1 - (float)(base - 1) * invBaseM < 1) {
        ++nDigits;
        invBaseM = invBaseM * invBase;
    }
    return nDigits;
}

static void BuildHalton(SceneDesc &s) {
    int fullRes[2] = {s.xres, s.yres};
    for (int i = 0; i < 2; ++i) {
        int base = (i == 0) ? 2 : 3;
        int scale = 1, exp = 0;
        while (scale < std::min(fullRes[i], 128)) {
            scale *= base;
            ++exp;
        }
        s.haltonBaseScales[i] = scale;
        s.haltonBaseExponents[i] = exp;
    }
    auto multInv = [](int64_t a, int64_t n) {
        // extended Euclid (samplers.h multiplicativeInverse)
        std::function<void(uint64_t, uint64_t, int64_t *, int64_t *)> egcd = [&](uint64_t a, uint64_t b, int64_t *x,
                                                                                 int64_t *y) {
            if (b == 0) {
                *x = 1;
                *y = 0;
                return;
            }
            int64_t d = a / b, xp, yp;
            egcd(b, a % b, &xp, &yp);
            *x = yp;
            *y = xp - (d * yp);
        };
        int64_t x, y;
        egcd(a, n, &x, &y);
        int64_t r = x % n;
        return (int)(r < 0 ? r + n : r);
    };
    s.haltonMultInverse[0] = multInv(s.haltonBaseScales[1], s.haltonBaseScales[0]);
    s.haltonMultInverse[1] = multInv(s.haltonBaseScales[0], s.haltonBaseScales[1]);

    // 6 camera dims + 7 per bounce, 10 with subsurface scattering (wavefront/samples.cpp:39-41):
    // pbrt's Halton sampler holds permutations for every dimension below PrimeTableSize, so none
    // of a path's dimensions may wrap here either
    int maxDim = (s.sss.empty() ? 7 : 10) * s.maxDepth + 6;
    maxDim = std::min(maxDim, 999);
    const std::vector<int> &primes = Primes();
    s.permTable.clear();
    s.permOffset.clear();
    s.permNDigits.clear();
    s.permBase.clear();
    for (int dim = 0; dim <= maxDim; ++dim) {
        int base = primes[dim];
        int nDigits = NumDigits(base);
        s.permOffset.push_back((uint32_t)s.permTable.size());
        s.permNDigits.push_back(nDigits);
        s.permBase.push_back(base);
        for (int digitIndex = 0; digitIndex < nDigits; ++digitIndex) {
            // Hash(base, digitIndex, seed): int, int, uint32_t packed = 12 bytes
            unsigned char buf[16];
            int b = base, di = digitIndex;
            uint32_t seed = (uint32_t)s.seed;
            std::memcpy(buf, &b, 4);
            std::memcpy(buf + 4, &di, 4);
            std::memcpy(buf + 8, &seed, 4);
            uint64_t dseed = MurmurHash64A(buf, 12, 0);
            for (int v = 0; v < base; ++v)
                s.permTable.push_back((uint16_t)PermutationElement((uint32_t)v, (uint32_t)base, (uint32_t)dseed));
        }
    }
}

// ---------------------------------------------------------------- light BVH
namespace {
struct Bounds3 {
    V3 pMin{kInfinity, kInfinity, kInfinity}, pMax{-kInfinity, -kInfinity, -kInfinity};
    bool Valid() const { return pMin.x <= pMax.x; }
    void Add(V3 p) {
        pMin = V3(std::min(pMin.x, p.x), std::min(pMin.y, p.y), std::min(pMin.z, p.z));
        pMax = V3(std::max(pMax.x, p.x), std::max(pMax.y, p.y), std::max(pMax.z, p.z));
    }
    void Add(const Bounds3 &b) {
        if (!b.Valid()) return;
        Add(b.pMin);
        Add(b.pMax);
    }
    V3 Diagonal() const { return pMax - pMin; }
    float SurfaceArea() const {
        V3 d = Diagonal();
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    V3 Offset(V3 p) const {
        V3 o = p - pMin;
        if (pMax.x > pMin.x) o.x /= pMax.x - pMin.x;
        if (pMax.y > pMin.y) o.y /= pMax.y - pMin.y;
        if (pMax.z > pMin.z) o.z /= pMax.z - pMin.z;
        return o;
    }
};

struct LightBounds {
    Bounds3 bounds;
    float phi = 0;
    V3 w;
    float cosTheta_o = 0, cosTheta_e = 0;
    bool twoSided = false;
    V3 Centroid() const { return (bounds.pMin + bounds.pMax) / 2; }
};

// util/transform.h Rotate(theta, axis) applied to a vector (float matrix)
V3 RotateVector(float thetaDeg, V3 axis, V3 v) {
    V3 a = Normalize(axis);
    float theta = thetaDeg * (kPi / 180);
    float sinTheta = std::sin(theta), cosTheta = std::cos(theta);
    float m[3][3];
    m[0][0] = a.x * a.x + (1 - a.x * a.x) * cosTheta;
    m[0][1] = a.x * a.y * (1 - cosTheta) - a.z * sinTheta;
    m[0][2] = a.x * a.z * (1 - cosTheta) + a.y * sinTheta;
    m[1][0] = a.x * a.y * (1 - cosTheta) + a.z * sinTheta;
    m[1][1] = a.y * a.y + (1 - a.y * a.y) * cosTheta;
    m[1][2] = a.y * a.z * (1 - cosTheta) - a.x * sinTheta;
    m[2][0] = a.x * a.z * (1 - cosTheta) - a.y * sinTheta;
    m[2][1] = a.y * a.z * (1 - cosTheta) + a.x * sinTheta;
    m[2][2] = a.z * a.z + (1 - a.z * a.z) * cosTheta;
    return V3(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z, m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
              m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z);
}

// util/vecmath.cpp:57 Union(DirectionCone, DirectionCone)
void ConeUnion(V3 aw, float aCos, V3 bw, float bCos, V3 *w, float *cosTheta) {
    float theta_a = SafeACos(aCos), theta_b = SafeACos(bCos);
    float theta_d = AngleBetween(aw, bw);
    if (std::min(theta_d + theta_b, kPi) <= theta_a) {
        *w = aw;
        *cosTheta = aCos;
        return;
    }
    if (std::min(theta_d + theta_a, kPi) <= theta_b) {
        *w = bw;
        *cosTheta = bCos;
        return;
    }
    float theta_o = (theta_a + theta_d + theta_b) / 2;
    if (theta_o >= kPi) {
        *w = V3(0, 0, 1);
        *cosTheta = -1;
        return;
    }
    float theta_r = theta_o - theta_a;
    V3 wr = Cross(aw, bw);
    if (LengthSquared(wr) == 0) {
        *w = V3(0, 0, 1);
        *cosTheta = -1;
        return;
    }
    *w = Normalize(RotateVector(theta_r * (180 / kPi), wr, aw));  // DirectionCone(w, cos theta_o)
    *cosTheta = std::cos(theta_o);
}

LightBounds Union(const LightBounds &a, const LightBounds &b) {
    if (a.phi == 0) return b;
    if (b.phi == 0) return a;
    LightBounds r;
    V3 w;
    float cosTheta;
    // DirectionCone(a.w, ...) normalizes its axis, and so does the LightBounds constructor
    // around the union's (lights.h:128-150): the same normalizations, for the same bits
    ConeUnion(Normalize(a.w), a.cosTheta_o, Normalize(b.w), b.cosTheta_o, &w, &cosTheta);
    r.bounds = a.bounds;
    r.bounds.Add(b.bounds);
    r.w = Normalize(w);
    r.phi = a.phi + b.phi;
    r.cosTheta_o = cosTheta;
    r.cosTheta_e = std::min(a.cosTheta_e, b.cosTheta_e);
    r.twoSided = a.twoSided | b.twoSided;
    return r;
}

float EvaluateCost(const LightBounds &b, const Bounds3 &bounds, int dim) {
    float theta_o = std::acos(b.cosTheta_o), theta_e = std::acos(b.cosTheta_e);
    float theta_w = std::min(theta_o + theta_e, kPi);
    float sinTheta_o = SafeSqrt(1 - Sqr(b.cosTheta_o));
    float M_omega = 2 * kPi * (1 - b.cosTheta_o) +
                    kPi / 2 * (2 * theta_w * sinTheta_o - std::cos(theta_o - 2 * theta_w) - 2 * theta_o * sinTheta_o + b.cosTheta_o);
    V3 d = bounds.Diagonal();
    float Kr = MaxComponentValue(d) / d[dim];
    return b.phi * M_omega * Kr * b.bounds.SurfaceArea();
}

// util/vecmath.h:1735 OctahedralVector encode/decode round trip
V3 OctahedralRoundTrip(V3 v) {
    auto sign = [](float x) { return std::copysign(1.f, x); };
    auto encode = [](float f) { return (uint16_t)std::round(Clampf((f + 1) / 2, 0, 1) * 65535.f); };
    v = v / (std::fabs(v.x) + std::fabs(v.y) + std::fabs(v.z));
    uint16_t x, y;
    if (v.z >= 0) {
        x = encode(v.x);
        y = encode(v.y);
    } else {
        x = encode((1 - std::fabs(v.y)) * sign(v.x));
        y = encode((1 - std::fabs(v.x)) * sign(v.y));
    }
    V3 r;
    r.x = -1 + 2 * (x / 65535.f);
    r.y = -1 + 2 * (y / 65535.f);
    r.z = 1 - (std::fabs(r.x) + std::fabs(r.y));
    if (r.z < 0) {
        float xo = r.x;
        r.x = (1 - std::fabs(r.y)) * sign(xo);
        r.y = (1 - std::fabs(xo)) * sign(r.y);
    }
    return Normalize(r);
}

LightNodeBounds Compact(const LightBounds &lb, const Bounds3 &allb) {
    // CompactLightBounds ctor + decode (lightsamplers.h:95-180)
    LightNodeBounds c;
    c.w = OctahedralRoundTrip(Normalize(lb.w));
    c.phi = lb.phi;
    auto qcos = [](float v) { return (unsigned)std::floor(32767.f * ((v + 1) / 2)); };
    unsigned qo = qcos(lb.cosTheta_o), qe = qcos(lb.cosTheta_e);
    c.cosTheta_o = 2 * (qo / 32767.f) - 1;
    c.cosTheta_e = 2 * (qe / 32767.f) - 1;
    c.twoSided = lb.twoSided;
    auto qb = [](float v, float mn, float mx) {
        if (mn == mx) return 0.f;
        return 65535.f * Clampf((v - mn) / (mx - mn), 0, 1);
    };
    uint16_t q[2][3];
    for (int k = 0; k < 3; ++k) {
        q[0][k] = (uint16_t)std::floor(qb(lb.bounds.pMin[k], allb.pMin[k], allb.pMax[k]));
        q[1][k] = (uint16_t)std::ceil(qb(lb.bounds.pMax[k], allb.pMin[k], allb.pMax[k]));
    }
    for (int k = 0; k < 3; ++k) {
        c.pMin[k] = Lerpf(q[0][k] / 65535.f, allb.pMin[k], allb.pMax[k]);
        c.pMax[k] = Lerpf(q[1][k] / 65535.f, allb.pMin[k], allb.pMax[k]);
    }
    return c;
}

struct LightBVHBuilder {
    SceneDesc &s;
    Bounds3 allLightBounds;
    std::pair<int, LightBounds> Build(std::vector<std::pair<int, LightBounds>> &bvhLights, int start, int end,
                                      uint32_t bitTrail, int depth) {
        if (end - start == 1) {
            int nodeIndex = (int)s.lightNodes.size();
            LightBVHNodeDesc n;
            n.bounds = Compact(bvhLights[start].second, allLightBounds);
            n.childOrLight = bvhLights[start].first;
            n.isLeaf = 1;
            s.lightNodes.push_back(n);
            s.lightBitTrail[bvhLights[start].first] = bitTrail;
            return {nodeIndex, bvhLights[start].second};
        }
        Bounds3 bounds, centroidBounds;
        for (int i = start; i < end; ++i) {
            bounds.Add(bvhLights[i].second.bounds);
            centroidBounds.Add(bvhLights[i].second.Centroid());
        }
        float minCost = kInfinity;
        int minCostSplitBucket = -1, minCostSplitDim = -1;
        constexpr int nBuckets = 12;
        for (int dim = 0; dim < 3; ++dim) {
            if (centroidBounds.pMax[dim] == centroidBounds.pMin[dim]) continue;
            LightBounds bucketLightBounds[nBuckets];
            for (int i = start; i < end; ++i) {
                V3 pc = bvhLights[i].second.Centroid();
                int b = (int)(nBuckets * centroidBounds.Offset(pc)[dim]);
                if (b == nBuckets) b = nBuckets - 1;
                bucketLightBounds[b] = Union(bucketLightBounds[b], bvhLights[i].second);
            }
            float cost[nBuckets - 1];
            for (int i = 0; i < nBuckets - 1; ++i) {
                LightBounds b0, b1;
                for (int j = 0; j <= i; ++j) b0 = Union(b0, bucketLightBounds[j]);
                for (int j = i + 1; j < nBuckets; ++j) b1 = Union(b1, bucketLightBounds[j]);
                cost[i] = EvaluateCost(b0, bounds, dim) + EvaluateCost(b1, bounds, dim);
            }
            for (int i = 1; i < nBuckets - 1; ++i) {
                if (cost[i] > 0 && cost[i] < minCost) {
                    minCost = cost[i];
                    minCostSplitBucket = i;
                    minCostSplitDim = dim;
                }
            }
        }
        int mid;
        if (minCostSplitDim == -1)
            mid = (start + end) / 2;
        else {
            auto *pmid = std::partition(&bvhLights[start], &bvhLights[end - 1] + 1, [&](const std::pair<int, LightBounds> &l) {
                int b = (int)(nBuckets * centroidBounds.Offset(l.second.Centroid())[minCostSplitDim]);
                if (b == nBuckets) b = nBuckets - 1;
                return b <= minCostSplitBucket;
            });
            mid = (int)(pmid - &bvhLights[0]);
            if (mid == start || mid == end) mid = (start + end) / 2;
        }
        int nodeIndex = (int)s.lightNodes.size();
        s.lightNodes.push_back(LightBVHNodeDesc());
        std::pair<int, LightBounds> child0 = Build(bvhLights, start, mid, bitTrail, depth + 1);
        std::pair<int, LightBounds> child1 = Build(bvhLights, mid, end, bitTrail | (1u << depth), depth + 1);
        LightBounds lb = Union(child0.second, child1.second);
        s.lightNodes[nodeIndex].bounds = Compact(lb, allLightBounds);
        s.lightNodes[nodeIndex].childOrLight = child1.first;
        s.lightNodes[nodeIndex].isLeaf = 0;
        return {nodeIndex, lb};
    }
};
}  // namespace

void DebugBuildLightBVH(const float *in13, int n, std::vector<LightBVHNodeDesc> *nodes, std::vector<uint32_t> *trails) {
    SceneDesc s;
    s.lightBitTrail.assign(n, 0xffffffffu);
    LightBVHBuilder b{s, Bounds3()};
    std::vector<std::pair<int, LightBounds>> bvhLights;
    for (int i = 0; i < n; ++i) {
        const float *v = in13 + 13 * i;
        LightBounds lb;
        lb.bounds.Add(V3(v[0], v[1], v[2]));
        lb.bounds.Add(V3(v[3], v[4], v[5]));
        lb.w = V3(v[6], v[7], v[8]);
        lb.phi = v[9];
        lb.cosTheta_o = v[10];
        lb.cosTheta_e = v[11];
        lb.twoSided = v[12] != 0;
        if (lb.phi > 0) {
            bvhLights.push_back({i, lb});
            b.allLightBounds.Add(lb.bounds);
        }
    }
    if (!bvhLights.empty()) b.Build(bvhLights, 0, (int)bvhLights.size(), 0, 0);
    *nodes = s.lightNodes;
    *trails = s.lightBitTrail;
}

static void BuildLightBVH(SceneDesc &s) {
    s.lightNodes.clear();
    s.lightBitTrail.assign(s.areaLights.size() + s.nPointSpot, 0);
    if (s.uniformLightSampler) return;
    LightBVHBuilder b{s, Bounds3()};
    std::vector<std::pair<int, LightBounds>> bvhLights;
    for (size_t i = 0; i < s.areaLights.size(); ++i) {
        const AreaLightDesc &al = s.areaLights[i];
        if (al.shape >= 0) {
            // Sphere / Disk emitters: Shape::Bounds, Shape::NormalBounds (shapes.h:134,
            // shapes.cpp:94-99: the entire sphere; the disk's transformed, oriented normal)
            const DeviceShape &d = s.shapes[al.shape].dev;
            const auto &dense = s.denseSpectra[al.spectrum];
            float phi = *std::max_element(dense.begin(), dense.end());
            phi *= al.scale * al.area * kPi;
            LightBounds lb;
            V3 lo, hi;
            ShapeBounds(d, &lo, &hi);
            lb.bounds.Add(lo);
            lb.bounds.Add(hi);
            if (d.kind == kShapeBilinearT) {
                // BilinearPatch::NormalBounds (shapes.cpp:1083-1129)
                const AnalyticShapeDesc &sh = s.shapes[al.shape];
                const PatchVerts P = PatchP(d);
                const bool hasN = d.flags & 8, flip = ((d.flags & 1) != 0) != ((d.flags & 2) != 0);
                auto N = [&](int k) { return V3(sh.normals[3 * k], sh.normals[3 * k + 1], sh.normals[3 * k + 2]); };
                if (P.p00 == P.p10 || P.p10 == P.p11 || P.p11 == P.p01 || P.p01 == P.p00) {
                    const V3 dpdu = LerpV(0.5f, P.p10, P.p11) - LerpV(0.5f, P.p00, P.p01);
                    const V3 dpdv = LerpV(0.5f, P.p01, P.p11) - LerpV(0.5f, P.p00, P.p10);
                    V3 n = Normalize(Cross(dpdu, dpdv));
                    if (hasN) n = FaceForwardN(n, (N(0) + N(1) + N(2) + N(3)) / 4);
                    else if (flip) n = -n;
                    lb.w = Normalize(Normalize(n));
                    lb.cosTheta_o = 1;
                } else {
                    V3 n00 = Normalize(Cross(P.p10 - P.p00, P.p01 - P.p00));
                    V3 n10 = Normalize(Cross(P.p11 - P.p10, P.p00 - P.p10));
                    V3 n01 = Normalize(Cross(P.p00 - P.p01, P.p11 - P.p01));
                    V3 n11 = Normalize(Cross(P.p01 - P.p11, P.p10 - P.p11));
                    if (hasN) {
                        n00 = FaceForwardN(n00, N(0));
                        n10 = FaceForwardN(n10, N(1));
                        n01 = FaceForwardN(n01, N(2));
                        n11 = FaceForwardN(n11, N(3));
                    } else if (flip) {
                        n00 = -n00, n10 = -n10, n01 = -n01, n11 = -n11;
                    }
                    const V3 n = Normalize(n00 + n10 + n01 + n11);
                    const float cosTheta = std::min(std::min(Dot(n, n00), Dot(n, n01)), std::min(Dot(n, n10), Dot(n, n11)));
                    lb.w = Normalize(n);
                    lb.cosTheta_o = Clampf(cosTheta, -1, 1);
                }
            } else if (d.kind == kShapeSphereT || d.kind == kShapeCylinderT) {  // EntireSphere
                lb.w = Normalize(V3(0, 0, 1));
                lb.cosTheta_o = -1;
            } else {
                V3 n = XfNormal(d.r2o, V3(0, 0, 1));
                if (d.flags & 1) n = -n;
                lb.w = Normalize(Normalize(n));
                lb.cosTheta_o = 1;
            }
            lb.phi = phi;
            lb.cosTheta_e = std::cos(kPi / 2);
            lb.twoSided = al.twoSided;
            if (lb.phi > 0) {
                bvhLights.push_back({(int)i, lb});
                b.allLightBounds.Add(lb.bounds);
            }
            continue;
        }
        const auto &tri = s.tris[al.prim];
        V3 p0 = s.verts[tri[0]], p1 = s.verts[tri[1]], p2 = s.verts[tri[2]];
        const auto &dense = s.denseSpectra[al.spectrum];
        float mx = *std::max_element(dense.begin(), dense.end());
        if (al.image >= 0) {
            // DiffuseAreaLight::Bounds with an image (lights.cpp:806-813): the mean channel value
            const AreaLightImage &im = s.areaLightImages[al.image];
            float sum = 0;
            for (float v : im.rgb) sum += v;
            mx = sum / (3 * im.w * im.h);
        }
        float phi = mx;
        phi *= al.scale * al.area * kPi;
        // Triangle::NormalBounds (shapes.h): with vertex normals the face normal is turned
        // toward their sum, otherwise flipped by reverseOrientation ^ transformSwapsHandedness
        V3 n = Normalize(Cross(p1 - p0, p2 - p0));
        if (!s.triShade.empty() && (s.triShade[al.prim] & 1)) {
            V3 ns = s.vertN[tri[0]] + s.vertN[tri[1]] + s.vertN[tri[2]];
            n = FaceForwardN(n, ns);
        } else if (s.triFlip[al.prim]) {
            n = n * -1.f;
        }
        LightBounds lb;
        lb.bounds.Add(p0);
        lb.bounds.Add(p1);
        lb.bounds.Add(p2);
        // DirectionCone(n) normalizes n, and LightBounds' constructor normalizes the cone's axis
        // (DiffuseAreaLight::Bounds, lights.cpp:819-821): both, for pbrt's bits
        lb.w = Normalize(Normalize(n));
        lb.phi = phi;
        lb.cosTheta_o = 1;
        lb.cosTheta_e = std::cos(kPi / 2);
        lb.twoSided = al.twoSided;
        if (lb.phi > 0) {
            bvhLights.push_back({(int)i, lb});
            b.allLightBounds.Add(lb.bounds);
        }
    }
    // PointLight::Bounds / SpotLight::Bounds (lights.cpp:168-173, 1401-1411), after the area
    // lights in pbrt's light order; phi from the maximum of the dense spectrum, as for area lights
    for (int i = 0; i < s.nPointSpot; ++i) {
        const DeltaLightDesc &d = s.deltaLights[i];
        const auto &dense = s.denseSpectra[d.spectrum];
        const float mx = *std::max_element(dense.begin(), dense.end());
        LightBounds lb;
        lb.bounds.Add(d.p);
        lb.twoSided = false;
        if (d.type == kDeltaGonio || d.type == kDeltaProjection) {
            // GoniometricLight::Bounds (an isotropic point) / ProjectionLight::Bounds, precomputed
            lb.w = Normalize(d.w);
            lb.phi = d.phi;
            lb.cosTheta_o = d.cosFalloffStart;
            lb.cosTheta_e = d.cosFalloffEnd;
        } else if (d.type == kDeltaPoint) {
            lb.w = V3(0, 0, 1);
            lb.phi = 4 * kPi * d.scale * mx;
            lb.cosTheta_o = std::cos(kPi);
            lb.cosTheta_e = std::cos(kPi / 2);
        } else {
            lb.w = Normalize(d.w);  // LightBounds' constructor normalizes SpotLight::Bounds' axis again
            lb.phi = d.scale * mx * 4 * kPi;
            float cosTheta_e = std::cos(std::acos(d.cosFalloffEnd) - std::acos(d.cosFalloffStart));
            if (cosTheta_e == 1 && d.cosFalloffEnd != d.cosFalloffStart) cosTheta_e = 0.999f;
            lb.cosTheta_o = d.cosFalloffStart;
            lb.cosTheta_e = cosTheta_e;
        }
        if (lb.phi > 0) {
            bvhLights.push_back({(int)s.areaLights.size() + i, lb});
            b.allLightBounds.Add(lb.bounds);
        }
    }
    if (!bvhLights.empty()) b.Build(bvhLights, 0, (int)bvhLights.size(), 0, 0);
}

// samplers.h:303-330 (ZSobolSampler::GetSampleIndex permutations)
const uint8_t kZSobolPermutations[24][4] = {
    {0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 2, 1}, {0, 3, 1, 2},
    {1, 0, 2, 3}, {1, 0, 3, 2}, {1, 2, 0, 3}, {1, 2, 3, 0}, {1, 3, 2, 0}, {1, 3, 0, 2},
    {2, 1, 0, 3}, {2, 1, 3, 0}, {2, 0, 1, 3}, {2, 0, 3, 1}, {2, 3, 0, 1}, {2, 3, 1, 0},
    {3, 1, 2, 0}, {3, 1, 0, 2}, {3, 2, 1, 0}, {3, 2, 0, 1}, {3, 0, 2, 1}, {3, 0, 1, 2}};

// ZSobolSampler ctor (samplers.h:228-239)
static void BuildZSobol(SceneDesc &s) {
    auto log2Int = [](int64_t v) {
        int r = -1;
        while (v > 0) {
            v >>= 1;
            ++r;
        }
        return r;
    };
    s.zsLog2SamplesPerPixel = log2Int(s.spp);
    int64_t res = 1;
    while (res < std::max(s.xres, s.yres)) res <<= 1;  // RoundUpPow2
    int log4SamplesPerPixel = (s.zsLog2SamplesPerPixel + 1) / 2;
    s.zsNBase4Digits = log2Int(res) + log4SamplesPerPixel;
    s.sobolLog2Scale = log2Int(res);  // SobolSampler: scale = RoundUpPow2(max(fullResolution))
    if (s.samplerType == kSamplerSobol && s.sobolLog2Scale > kNVdCSobol)
        throw Error("sobol: resolution above 2^25 pixels per side is outside the VdC Sobol' tables");
}

const SobolTableData &SobolTables() {
    static std::once_flag once;
    static SobolTableData t;
    static std::string err;
    std::call_once(once, [] {
        const std::string path = GetDataDirectory() + "/sobol_tables.bin";
        std::ifstream in(path, std::ios::binary);
        const size_t n32 = (size_t)kNSobolDimensions * kSobolMatrixSize, nv = (size_t)kNVdCSobol * kSobolMatrixSize;
        t.m32.resize(n32);
        t.vdc.resize(nv);
        t.vdcInv.resize(nv);
        bool ok = (bool)in;
        if (ok) in.read(reinterpret_cast<char *>(t.m32.data()), (std::streamsize)(n32 * 4));
        if (ok) in.read(reinterpret_cast<char *>(t.vdc.data()), (std::streamsize)(nv * 8));
        if (ok) in.read(reinterpret_cast<char *>(t.vdcInv.data()), (std::streamsize)(nv * 8));
        ok = ok && in.gcount() == (std::streamsize)(nv * 8) && in.peek() == EOF;
        // dimensions 0 and 1 must be the matrices the ZSobol path generates on the fly
        for (int k = 0; ok && k < kSobolMatrixSize; ++k)
            ok = t.m32[k] == (k < 32 ? 0x80000000u >> k : 0u) && t.m32[kSobolMatrixSize + k] == SobolMatrix1Row(k);
        if (!ok) err = "SobolSampler: " + path + " is missing or malformed (oracle/ref/gen_golden.py writes it)";
    });
    if (!err.empty()) throw Error(err);
    return t;
}

void FinalizeScene(SceneDesc &s) {
    BuildLightBVH(s);
    BuildHalton(s);
    BuildZSobol(s);
}

// PiecewiseConstant1D ctor (util/sampling.h:625-649) into func (|f|) and cdf; returns funcInt
float BuildPC1D(const float *f, int n, float mn, float mx, float *func, float *cdf) {
    for (int i = 0; i < n; ++i) func[i] = std::fabs(f[i]);
    cdf[0] = 0;
    for (int i = 1; i < n + 1; ++i) cdf[i] = cdf[i - 1] + func[i - 1] * (mx - mn) / (float)n;
    const float funcInt = cdf[n];
    if (funcInt == 0)
        for (int i = 1; i < n + 1; ++i) cdf[i] = float(i) / float(n);
    else
        for (int i = 1; i < n + 1; ++i) cdf[i] /= funcInt;
    return funcInt;
}

// ImageInfiniteLight's compensatedDistribution (lights.cpp:1060-1070): pixel averages
// (ImageChannelValues::Average, in float), minus their mean accumulated in double, clamped at
// zero (all ones when nothing is left), as a PiecewiseConstant2D over [0,1]^2 in the
// FilterTableView layout
std::vector<float> BuildEnvDistribution(const EnvLightDesc &e) {
    const int n = e.res;
    std::vector<float> t(FilterTableView::Size(n, n), 0.f);
    float *F = t.data(), *func = F + (size_t)n * n, *condCdf = func + (size_t)n * n, *condInt = condCdf + (size_t)n * (n + 1);
    float *margCdf = condInt + n;
    const size_t np = (size_t)n * n;
    for (size_t p = 0; p < np; ++p) {
        float sum = 0;
        for (int c = 0; c < 3; ++c) sum += e.rgb[3 * p + c];
        F[p] = sum / 3;
    }
    double acc = 0.;
    for (size_t p = 0; p < np; ++p) acc += F[p];
    const double average = acc / np;
    bool allZero = true;
    for (size_t p = 0; p < np; ++p) {
        F[p] = std::max<float>((float)(F[p] - average), 0.f);
        allZero = allZero && F[p] == 0;
    }
    if (allZero) std::fill(F, F + np, 1.f);
    for (int v = 0; v < n; ++v) condInt[v] = BuildPC1D(F + (size_t)v * n, n, 0.f, 1.f, func + (size_t)v * n, condCdf + (size_t)v * (n + 1));
    std::vector<float> margFunc(n);
    margCdf[n + 1] = BuildPC1D(condInt, n, 0.f, 1.f, margFunc.data(), margCdf);
    return t;
}

void BuildFilterTable(SceneDesc &s) {
    s.filterTable.clear();
    s.filterNu = s.filterNv = 0;
    if (s.filterType == kFilterBox || s.filterType == kFilterTriangle) return;
    const FilterParams fp{s.filterType, s.filterRadiusX, s.filterRadiusY, s.filterA, s.filterB};
    const int nu = int(32 * fp.rx), nv = int(32 * fp.ry);
    if (nu < 1 || nv < 1) throw Error("pixel filter radius too small to tabulate");
    s.filterNu = nu;
    s.filterNv = nv;
    s.filterTable.assign(FilterTableView::Size(nu, nv), 0.f);
    float *F = s.filterTable.data(), *func = F + nu * nv, *condCdf = func + nu * nv, *condInt = condCdf + nv * (nu + 1);
    float *margCdf = condInt + nv;
    for (int y = 0; y < nv; ++y)
        for (int x = 0; x < nu; ++x) {
            // domain.Lerp((x + 0.5) / nu, (y + 0.5) / nv) over [-r, r]^2
            const float px = Lerpf((x + 0.5f) / nu, -fp.rx, fp.rx), py = Lerpf((y + 0.5f) / nv, -fp.ry, fp.ry);
            F[y * nu + x] = FilterEvaluate(fp, px, py);
        }
    for (int v = 0; v < nv; ++v)
        condInt[v] = BuildPC1D(F + v * nu, nu, -fp.rx, fp.rx, func + v * nu, condCdf + v * (nu + 1));
    std::vector<float> margFunc(nv);
    margCdf[nv + 1] = BuildPC1D(condInt, nv, -fp.ry, fp.ry, margFunc.data(), margCdf);
}

}  // namespace pbrt_amd

namespace pbrt_amd {
// Image::BilerpChannel(uv, c, WrapMode::OctahedralSphere) (util/image.h:279-292, 96-125) of an
// environment map's linear RGB
static float BilerpOctahedral(const EnvLightDesc &e, float u, float v, int c) {
    const int n = e.res;
    const float x = u * n - 0.5f, y = v * n - 0.5f;
    const int xi = (int)std::floor(x), yi = (int)std::floor(y);
    const float dx = x - xi, dy = y - yi;
    auto get = [&](int px, int py) {
        if (px < 0) {
            px = -px;
            py = n - 1 - py;
        } else if (px >= n) {
            px = 2 * n - 1 - px;
            py = n - 1 - py;
        }
        if (py < 0) {
            px = n - 1 - px;
            py = -py;
        } else if (py >= n) {
            px = n - 1 - px;
            py = 2 * n - 1 - py;
        }
        if (n == 1) px = py = 0;
        return e.rgb[((size_t)py * n + px) * 3 + c];
    };
    const float v0 = get(xi, yi), v1 = get(xi + 1, yi), v2 = get(xi, yi + 1), v3 = get(xi + 1, yi + 1);
    return ((1 - dx) * (1 - dy) * v0 + dx * (1 - dy) * v1 + (1 - dx) * dy * v2 + dx * dy * v3);
}

// PortalImageInfiniteLight's constructor (lights.cpp:1140-1212): the portal frame
// (Frame::FromXY(p03, p01)), the map rectified over the portal's (alpha, beta) angles (each
// pixel centre's direction back through renderFromLight to the equal-area map, bilerped), the
// sampling distribution (channel average times duv/dw at the pixel centre,
// Image::GetSamplingDistribution) and its SummedAreaTable (double sums; the device keeps the
// Float values LookupInt returns).  Host float arithmetic with libm, as the reference's CPU build.
void BuildPortal(EnvLightDesc &e, const std::string &loc) {
    auto P = [&](int k) { return V3(e.portalP[k][0], e.portalP[k][1], e.portalP[k][2]); };
    const V3 p01 = Normalize(P(1) - P(0)), p12 = Normalize(P(2) - P(1));
    const V3 p32 = Normalize(P(2) - P(3)), p03 = Normalize(P(3) - P(0));
    if (std::abs(Dot(p01, p32) - 1) > .001 || std::abs(Dot(p12, p03) - 1) > .001 || std::abs(Dot(p01, p12)) > .001 ||
        std::abs(Dot(p12, p32)) > .001 || std::abs(Dot(p32, p03)) > .001 || std::abs(Dot(p03, p01)) > .001)
        std::fprintf(stderr, "%s: Error: Infinite light portal isn't a planar quadrilateral\n", loc.c_str());
    const V3 z = Cross(p03, p01);
    const float fr[9] = {p03.x, p03.y, p03.z, p01.x, p01.y, p01.z, z.x, z.y, z.z};
    std::copy(fr, fr + 9, e.portalFrame);
    const int n = e.res;
    e.rect.assign((size_t)n * n * 3, 0.f);
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
            const float u = (x + 0.5f) / n, v = (y + 0.5f) / n;
            V3 w = PortalRenderFromImage(e.portalFrame, u, v, nullptr);
            w = Normalize(MulM3(e.lightFromRender, w));
            float ue, ve;
            EqualAreaSphereToSquare(w, &ue, &ve);
            for (int c = 0; c < 3; ++c) e.rect[((size_t)y * n + x) * 3 + c] = BilerpOctahedral(e, ue, ve, c);
        }
    e.portalFunc.assign((size_t)n * n, 0.f);
    for (int y = 0; y < n; ++y)
        for (int x = 0; x < n; ++x) {
            const float *c = &e.rect[((size_t)y * n + x) * 3];
            float sum = 0;
            for (int k = 0; k < 3; ++k) sum += c[k];
            const float value = sum / 3;
            float duv_dw;
            (void)PortalRenderFromImage(e.portalFrame, (x + .5f) / n, (y + .5f) / n, &duv_dw);
            e.portalFunc[(size_t)y * n + x] = value * duv_dw;
        }
    e.portalSat = SummedAreaTable(e.portalFunc, n);
}

// SummedAreaTable(values) (util/sampling.h:834-848): double running sums, stored as the Float
// LookupInt returns
std::vector<float> SummedAreaTable(const std::vector<float> &f, int n) {
    std::vector<double> sum((size_t)n * n);
    auto S = [&](int x, int y) -> double & { return sum[(size_t)y * n + x]; };
    auto F = [&](int x, int y) { return f[(size_t)y * n + x]; };
    S(0, 0) = F(0, 0);
    for (int x = 1; x < n; ++x) S(x, 0) = F(x, 0) + S(x - 1, 0);
    for (int y = 1; y < n; ++y) S(0, y) = F(0, y) + S(0, y - 1);
    for (int y = 1; y < n; ++y)
        for (int x = 1; x < n; ++x) S(x, y) = (F(x, y) + S(x - 1, y) + S(x, y - 1) - S(x - 1, y - 1));
    std::vector<float> out(sum.size());
    for (size_t i = 0; i < sum.size(); ++i) out[i] = (float)sum[i];
    return out;
}
}  // namespace pbrt_amd
