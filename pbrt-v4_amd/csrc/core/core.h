// pbrt-v4_amd core: host+device scalar math shared by the HIP kernels and the host
// scene builder.  Every routine restates the reference semantics it names (file:line in
// /root/reference/src/pbrt) with the same operation order, so that device results stay
// within float rounding of pbrt's CPU path.  Compile with -ffp-contract=off: explicit
// fmaf() is used exactly where pbrt calls FMA().
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define PHD __host__ __device__ inline
// Large, cold-ish helpers stay out of line in the kernels: the shade kernel's inlined code
// outgrew the instruction cache, and a call is cheaper than streaming instructions from L2.
#define PHD_NOINLINE __host__ __device__ inline __attribute__((noinline))
#define PHD_UNROLL _Pragma("unroll")
// LightImportance and SampleSphericalTriangleN have an inline body (*Inl, taken by the lean
// diffuse kernel: C2 +2 % over out-of-line calls) and an out-of-line wrapper (every other
// kernel, where inlining them spilled hundreds of VGPRs: the conductor kernel ran 48 % slower).
#define PHD_LI PHD
#define PHD_SPH PHD
#else
#define PHD inline
#define PHD_NOINLINE inline
#define PHD_UNROLL
#define PHD_LI inline
#define PHD_SPH inline
#endif

#include "detmath.h"  // after PHD: the device transcendentals

namespace pbrt_amd {

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kPiOver2 = 1.57079632679489661923f;
constexpr float kPiOver4 = 0.78539816339744830961f;
constexpr float kInfinity = __builtin_huge_valf();
constexpr float kMachineEpsilon = 5.9604644775390625e-08f;  // util/float.h:45
constexpr float kOneMinusEpsilon = 0x1.fffffep-1f;           // util/float.h
constexpr float kShadowEpsilon = 0.0001f;                    // util/math.h:42
constexpr float kLambdaMin = 395.f, kLambdaMax = 705.f;      // util/spectrum.h:34
constexpr int kNSpectrumSamples = 31;                        // util/spectrum.h:36
constexpr float kMinSphericalSampleArea = 3e-4f;             // shapes.h
constexpr float kMaxSphericalSampleArea = 6.22f;

// ---------------------------------------------------------------- float utilities
PHD uint32_t FloatToBits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
PHD float BitsToFloat(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
// util/float.h NextFloatUp/NextFloatDown
PHD float NextFloatUp(float v) {
    if (std::isinf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = FloatToBits(v);
    if (v >= 0) ++ui; else --ui;
    return BitsToFloat(ui);
}
PHD float NextFloatDown(float v) {
    if (std::isinf(v) && v < 0.f) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = FloatToBits(v);
    if (v > 0) --ui; else ++ui;
    return BitsToFloat(ui);
}
// util/float.h:197 gamma(n)
PHD constexpr float gamma(int n) { return (n * kMachineEpsilon) / (1 - n * kMachineEpsilon); }

// Transcendentals.  Host code calls libm's float functions, as the reference CPU build does (the
// host-side tables and debug entries are pinned bit for bit against the reference's goldens).
// Device code evaluates the portable polynomials of detmath.h, built from IEEE operations only,
// so a host restatement reproduces every device result bit for bit: the CPU oracle's device-math
// mode (oracle_set_math_mode(2), which the GPU parity tests select) does, and the GPU path makes every decision
// the oracle makes -- the medium RNG seeded from a ray's bits (wavefront/media.cpp:44), alpha
// tests hashing the ray (gpu/optix.cu:197-243), mix choices hashing the hit (materials.h:285-294).
#if defined(__HIP_DEVICE_COMPILE__)
PHD float Sinf(float x) { return detm::Sin(x); }
PHD float Cosf(float x) { return detm::Cos(x); }
// sin and cos of one angle: one shared argument reduction, the same values as the two calls
PHD void SinCosf(float x, float *s, float *c) { detm::SinCos(x, s, c); }
PHD float ASinf(float x) { return detm::ASin(x); }
PHD float ACosf(float x) { return detm::ACos(x); }
PHD float ATan2f(float y, float x) { return detm::ATan2(y, x); }
PHD float Logf(float x) { return detm::Log(x); }
PHD float Expf(float x) { return detm::Exp(x); }
PHD float Sinhf(float x) { return detm::Sinh(x); }
PHD float Tanf(float x) { return detm::Tan(x); }
#else
PHD float Sinf(float x) { return std::sin(x); }
PHD float Cosf(float x) { return std::cos(x); }
PHD void SinCosf(float x, float *s, float *c) {
    *s = std::sin(x);
    *c = std::cos(x);
}
PHD float ASinf(float x) { return std::asin(x); }
PHD float ACosf(float x) { return std::acos(x); }
PHD float ATan2f(float y, float x) { return std::atan2(y, x); }
PHD float Logf(float x) { return std::log(x); }
PHD float Expf(float x) { return std::exp(x); }
PHD float Sinhf(float x) { return std::sinh(x); }
PHD float Tanf(float x) { return std::tan(x); }
#endif

// Scene Options (BasicSceneBuilder::Option, scene.cpp:492-560) that change the hot path
constexpr int kOptNoPixelJitter = 1;       // GetCameraSample (samplers.h:807-812), Approximate_dp_dxy
constexpr int kOptNoWavelengthJitter = 2;  // wavefront/camera.cpp:55
constexpr int kOptNoTextureFiltering = 4;  // wavefront/surfscatter.cpp:77

PHD float Sqr(float v) { return v * v; }
PHD float Clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }
PHD float Lerpf(float t, float a, float b) { return (1 - t) * a + t * b; }
PHD float SafeSqrt(float x) { return std::sqrt(std::fmax(0.f, x)); }
PHD float SafeASin(float x) { return ASinf(Clampf(x, -1, 1)); }
PHD float SafeACos(float x) { return ACosf(Clampf(x, -1, 1)); }
// util/math.h:570-583
PHD float DifferenceOfProducts(float a, float b, float c, float d) {
    float cd = c * d;
    float dop = fmaf(a, b, -cd);
    float err = fmaf(-c, d, cd);
    return dop + err;
}
PHD float SumOfProducts(float a, float b, float c, float d) {
    float cd = c * d;
    float sop = fmaf(a, b, cd);
    float err = fmaf(c, d, -cd);
    return sop + err;
}

// ---------------------------------------------------------------- vectors (DotN defined below)
struct V3 {
    float x, y, z;
    PHD V3() : x(0), y(0), z(0) {}
    PHD V3(float a, float b, float c) : x(a), y(b), z(c) {}
    PHD float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    PHD float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
PHD V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
PHD V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
PHD V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
PHD V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
PHD V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
PHD V3 operator/(V3 a, float d) { return {a.x / d, a.y / d, a.z / d}; }
PHD bool operator==(V3 a, V3 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
PHD bool operator!=(V3 a, V3 b) { return !(a == b); }
PHD V3 Abs(V3 a) { return {std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)}; }
// util/vecmath.h:966 (plain, left to right)
PHD float Dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PHD float AbsDot(V3 a, V3 b) { return std::fabs(Dot(a, b)); }
// Dot products that involve a Normal3f are FMA-compensated in pbrt (util/vecmath.h:1059-1099):
// FMA(n.x, v.x, SumOfProducts(n.y, v.y, n.z, v.z)).  n is the normal operand.
PHD float DotN(V3 n, V3 v);
PHD float AbsDotN(V3 n, V3 v);
// util/vecmath.h:1001 Cross via DifferenceOfProducts
PHD V3 Cross(V3 v, V3 w) {
    return {DifferenceOfProducts(v.y, w.z, v.z, w.y), DifferenceOfProducts(v.z, w.x, v.x, w.z),
            DifferenceOfProducts(v.x, w.y, v.y, w.x)};
}
PHD float DotN(V3 n, V3 v) { return fmaf(n.x, v.x, SumOfProducts(n.y, v.y, n.z, v.z)); }
PHD float AbsDotN(V3 n, V3 v) { return std::fabs(DotN(n, v)); }
PHD float LengthSquared(V3 v) { return Sqr(v.x) + Sqr(v.y) + Sqr(v.z); }
PHD float Length(V3 v) { return std::sqrt(LengthSquared(v)); }
PHD V3 Normalize(V3 v) { return v / Length(v); }
PHD float DistanceSquared(V3 a, V3 b) { return LengthSquared(a - b); }
PHD float Distance(V3 a, V3 b) { return Length(a - b); }
PHD float MaxComponentValue(V3 v) { return std::fmax(v.x, std::fmax(v.y, v.z)); }
PHD int MaxComponentIndex(V3 v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
PHD V3 Permute(const V3 &v, int a, int b, int c) { return {v[a], v[b], v[c]}; }  // const []: selects, no scratch
PHD V3 FaceForward(V3 n, V3 v) { return (Dot(n, v) < 0.f) ? -n : n; }
// FaceForward(Normal3f, Normal3f): the dot of two normals is FMA-compensated (vecmath.h:1073)
PHD V3 FaceForwardN(V3 n, V3 n2) { return (DotN(n, n2) < 0.f) ? -n : n; }
PHD V3 GramSchmidt(V3 v, V3 w) { return v - Dot(v, w) * w; }
// util/vecmath.h:974 AngleBetween
PHD float AngleBetween(V3 v1, V3 v2) {
    if (Dot(v1, v2) < 0) return kPi - 2 * SafeASin(Length(v1 + v2) / 2);
    return 2 * SafeASin(Length(v2 - v1) / 2);
}
// util/vecmath.h:1009 CoordinateSystem
PHD void CoordinateSystem(V3 v1, V3 *v2, V3 *v3) {
    float sign = std::copysign(1.f, v1.z);
    float a = -1 / (sign + v1.z);
    float b = v1.x * v1.y * a;
    *v2 = V3(1 + sign * Sqr(v1.x) * a, sign * b, -sign * v1.x);
    *v3 = V3(b, sign + Sqr(v1.y) * a, -v1.y);
}
// util/vecmath.h:1640
PHD float SphericalTriangleArea(V3 a, V3 b, V3 c) {
    return std::fabs(2 * ATan2f(Dot(a, Cross(b, c)), 1 + Dot(a, b) + Dot(a, c) + Dot(b, c)));
}

// Frame (util/vecmath.h:1855): FromXZ(x, z) = (x, Cross(z, x), z)
struct Frame {
    V3 x, y, z;
    PHD static Frame FromXZ(V3 x, V3 z) { return Frame{x, Cross(z, x), z}; }
    PHD V3 ToLocal(V3 v) const { return {Dot(v, x), Dot(v, y), Dot(v, z)}; }
    PHD V3 FromLocal(V3 v) const { return x * v.x + y * v.y + z * v.z; }
};

// ---------------------------------------------------------------- sampling (util/sampling.h)
PHD float SampleLinear(float u, float a, float b) {  // :122
    if (u == 0 && a == 0) return 0;
    float x = u * (a + b) / (a + std::sqrt(Lerpf(u, Sqr(a), Sqr(b))));
    return std::fmin(x, kOneMinusEpsilon);
}
PHD float BilinearPDF(float px, float py, const float w[4]) {  // :134
    if (px < 0 || px > 1 || py < 0 || py > 1) return 0;
    if (w[0] + w[1] + w[2] + w[3] == 0) return 1;
    return 4 * ((1 - px) * (1 - py) * w[0] + px * (1 - py) * w[1] + (1 - px) * py * w[2] + px * py * w[3]) /
           (w[0] + w[1] + w[2] + w[3]);
}
PHD void SampleBilinear(float u0, float u1, const float w[4], float *px, float *py) {  // :146
    *py = SampleLinear(u1, w[0] + w[1], w[2] + w[3]);
    *px = SampleLinear(u0, Lerpf(*py, w[0], w[2]), Lerpf(*py, w[1], w[3]));
}
PHD void SampleUniformTriangle(float u0, float u1, float b[3]) {  // :173
    float b0, b1;
    if (u0 < u1) {
        b0 = u0 / 2;
        b1 = u1 - b0;
    } else {
        b1 = u1 / 2;
        b0 = u0 - b1;
    }
    b[0] = b0;
    b[1] = b1;
    b[2] = 1 - b0 - b1;
}
PHD void SampleUniformDiskConcentric(float u0, float u1, float *dx, float *dy) {  // :325
    float ox = 2 * u0 - 1, oy = 2 * u1 - 1;
    if (ox == 0 && oy == 0) {
        *dx = 0;
        *dy = 0;
        return;
    }
    float theta, r;
    if (std::fabs(ox) > std::fabs(oy)) {
        r = ox;
        theta = kPiOver4 * (oy / ox);
    } else {
        r = oy;
        theta = kPiOver2 - kPiOver4 * (ox / oy);
    }
    float sinT, cosT;
    SinCosf(theta, &sinT, &cosT);
    *dx = r * cosT;
    *dy = r * sinT;
}
PHD V3 SampleCosineHemisphere(float u0, float u1) {  // :409
    float dx, dy;
    SampleUniformDiskConcentric(u0, u1, &dx, &dy);
    float z = SafeSqrt(1 - Sqr(dx) - Sqr(dy));
    return V3(dx, dy, z);
}
PHD float CosineHemispherePDF(float cosTheta) { return cosTheta * kInvPi; }

// util/sampling.h:79 SampleDiscrete specialised to two weights (light BVH child choice)
PHD int SampleDiscrete2(float w0, float w1, float u, float *pmf, float *uRemapped) {
    float sumWeights = 0;
    sumWeights += w0;
    sumWeights += w1;
    float up = u * sumWeights;
    if (up == sumWeights) up = NextFloatDown(up);
    // offset walk of the reference loop, unrolled for two weights (no indexed array)
    int offset = 0;
    float sum = 0;
    if (sum + w0 <= up) {
        sum += w0;
        offset = 1;
    }
    float w = offset ? w1 : w0;
    *pmf = w / sumWeights;
    *uRemapped = std::fmin((up - sum) / w, kOneMinusEpsilon);
    return offset;
}

// util/sampling.cpp:28 SampleSphericalTriangle (ok = false when the reference returns {});
// results by value so the out-of-line call needs no stack.
struct SphTriSample {
    float b0, b1, b2, pdf;
    bool ok;
};
// a, bb, c: Normalize(v0 - p), Normalize(v1 - p), Normalize(v2 - p) -- the callers have them
// already (Triangle::Sample's solid angle and bilinear weights use the same three vectors), so
// they are passed in rather than normalised a second time (same values, same bits).
PHD_SPH SphTriSample SampleSphericalTriangleNInl(V3 v0, V3 v1, V3 v2, V3 p, V3 a, V3 bb, V3 c, float u0, float u1) {
    SphTriSample r{0, 0, 0, 0, false};
    float b[3];
    float *pdf = &r.pdf;
    V3 n_ab = Cross(a, bb), n_bc = Cross(bb, c), n_ca = Cross(c, a);
    if (LengthSquared(n_ab) == 0 || LengthSquared(n_bc) == 0 || LengthSquared(n_ca) == 0) {
        return r;
    }
    n_ab = Normalize(n_ab);
    n_bc = Normalize(n_bc);
    n_ca = Normalize(n_ca);
    float alpha = AngleBetween(n_ab, -n_ca);
    float beta = AngleBetween(n_bc, -n_ab);
    float gam = AngleBetween(n_ca, -n_bc);
    float A_pi = alpha + beta + gam;
    float Ap_pi = Lerpf(u0, kPi, A_pi);
    {
        float A = A_pi - kPi;
        *pdf = (A <= 0) ? 0 : 1 / A;
    }
    float cosAlpha, sinAlpha, sinAp, cosAp;
    SinCosf(alpha, &sinAlpha, &cosAlpha);
    SinCosf(Ap_pi, &sinAp, &cosAp);
    float sinPhi = sinAp * cosAlpha - cosAp * sinAlpha;
    float cosPhi = cosAp * cosAlpha + sinAp * sinAlpha;
    float k1 = cosPhi + cosAlpha;
    float k2 = sinPhi - sinAlpha * Dot(a, bb);
    float cosBp = (k2 + (DifferenceOfProducts(k2, cosPhi, k1, sinPhi)) * cosAlpha) /
                  ((SumOfProducts(k2, sinPhi, k1, cosPhi)) * sinAlpha);
    cosBp = Clampf(cosBp, -1, 1);
    float sinBp = SafeSqrt(1 - Sqr(cosBp));
    V3 cp = cosBp * a + sinBp * Normalize(GramSchmidt(c, a));
    float cosTheta = 1 - u1 * (1 - Dot(cp, bb));
    float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    V3 w = cosTheta * bb + sinTheta * Normalize(GramSchmidt(cp, bb));
    V3 e1 = v1 - v0, e2 = v2 - v0;
    V3 s1 = Cross(w, e2);
    float divisor = Dot(s1, e1);
    if (divisor == 0) {
        r.b0 = r.b1 = r.b2 = 1.f / 3.f;
        r.ok = true;
        return r;
    }
    float invDivisor = 1 / divisor;
    V3 s = p - v0;
    float b1 = Dot(s, s1) * invDivisor;
    float b2 = Dot(w, Cross(s, e1)) * invDivisor;
    b1 = Clampf(b1, 0, 1);
    b2 = Clampf(b2, 0, 1);
    if (b1 + b2 > 1) {
        b1 /= b1 + b2;
        b2 /= b1 + b2;  // sic: the reference divides by the updated sum
    }
    r.b0 = 1 - b1 - b2;
    r.b1 = b1;
    r.b2 = b2;
    r.ok = true;
    (void)b;
    return r;
}

PHD_NOINLINE SphTriSample SampleSphericalTriangleN(V3 v0, V3 v1, V3 v2, V3 p, V3 a, V3 bb, V3 c, float u0, float u1) {
    return SampleSphericalTriangleNInl(v0, v1, v2, p, a, bb, c, u0, u1);
}
PHD SphTriSample SampleSphericalTriangle(V3 v0, V3 v1, V3 v2, V3 p, float u0, float u1) {
    return SampleSphericalTriangleN(v0, v1, v2, p, Normalize(v0 - p), Normalize(v1 - p), Normalize(v2 - p), u0, u1);
}

// util/sampling.cpp:110 InvertSphericalTriangleSample
struct SphTriUV {
    float u0, u1;
};
// a, b, c: the normalised (v_i - p), as for SampleSphericalTriangleN
PHD_NOINLINE SphTriUV InvertSphericalTriangleSampleN(V3 v0, V3 v1, V3 v2, V3 p, V3 a, V3 b, V3 c, V3 w) {
    SphTriUV r{0, 0};
    float *u0out = &r.u0, *u1out = &r.u1;
    (void)v0, (void)v1, (void)v2, (void)p;
    V3 n_ab = Cross(a, b), n_bc = Cross(b, c), n_ca = Cross(c, a);
    if (LengthSquared(n_ab) == 0 || LengthSquared(n_bc) == 0 || LengthSquared(n_ca) == 0) {
        return r;
    }
    n_ab = Normalize(n_ab);
    n_bc = Normalize(n_bc);
    n_ca = Normalize(n_ca);
    float alpha = AngleBetween(n_ab, -n_ca);
    float beta = AngleBetween(n_bc, -n_ab);
    float gam = AngleBetween(n_ca, -n_bc);
    V3 cp = Normalize(Cross(Cross(b, w), Cross(c, a)));
    if (Dot(cp, a + c) < 0) cp = -cp;
    float u0;
    if (Dot(a, cp) > 0.99999847691f)
        u0 = 0;
    else {
        V3 n_cpb = Cross(cp, b), n_acp = Cross(a, cp);
        if (LengthSquared(n_cpb) == 0 || LengthSquared(n_acp) == 0) {
            *u0out = 0.5f;
            *u1out = 0.5f;
            return r;
        }
        n_cpb = Normalize(n_cpb);
        n_acp = Normalize(n_acp);
        float Ap = alpha + AngleBetween(n_ab, n_cpb) + AngleBetween(n_acp, -n_cpb) - kPi;
        float A = alpha + beta + gam - kPi;
        u0 = Ap / A;
    }
    float u1 = (1 - Dot(w, b)) / (1 - Dot(cp, b));
    *u0out = Clampf(u0, 0, 1);
    *u1out = Clampf(u1, 0, 1);
    return r;
}

// ---------------------------------------------------------------- rays and triangles
// ray.h:78 OffsetRayOrigin; error vector e is the Point3fi half-width
PHD V3 OffsetRayOrigin(V3 p, V3 e, V3 n, V3 w) {
    float d = DotN(Abs(n), e);
    V3 offset = d * n;
    if (DotN(n, w) < 0) offset = -offset;
    V3 po = p + offset;
    for (int i = 0; i < 3; ++i) {
        if (offset[i] > 0)
            po[i] = NextFloatUp(po[i]);
        else if (offset[i] < 0)
            po[i] = NextFloatDown(po[i]);
    }
    return po;
}

// Point3fi(Point3f p, Vector3f e) (util/vecmath.h:753) stores intervals built with
// Interval::FromValueAndError (util/math.h:829) using the CPU rounding helpers
// AddRoundUp/AddRoundDown = NextFloatUp/Down(a + b) (util/float.h:201-229); Point3f(pi) is
// the interval midpoint and pi.Error() its half width.  Round-trip (p, e) the same way.
PHD void ToPoint3fi(V3 v, V3 e, V3 *p, V3 *err) {
    for (int i = 0; i < 3; ++i) {
        float lo = v[i], hi = v[i];
        if (e[i] != 0) {
            lo = NextFloatDown(v[i] + (-e[i]));
            hi = NextFloatUp(v[i] + e[i]);
        }
        (*p)[i] = (lo + hi) / 2;
        (*err)[i] = (hi - lo) / 2;
    }
}

struct TriHit {
    float b0, b1, b2, t;
};

// shapes.cpp:215-225: recompute the edge functions in double when one is exactly zero.
// Rare, so it is kept out of line (its doubles would otherwise inflate every caller's VGPRs);
// the three results come back by value (in registers, no scratch round trip).
struct EdgeFns {
    float e0, e1, e2;
};
#if defined(__HIPCC__)
__host__ __device__ inline __attribute__((noinline))
#else
inline
#endif
EdgeFns EdgeFunctionsFP64(V3 p0t, V3 p1t, V3 p2t) {
    double p2txp1ty = (double)p2t.x * (double)p1t.y;
    double p2typ1tx = (double)p2t.y * (double)p1t.x;
    EdgeFns e;
    e.e0 = (float)(p2typ1tx - p2txp1ty);
    double p0txp2ty = (double)p0t.x * (double)p2t.y;
    double p0typ2tx = (double)p0t.y * (double)p2t.x;
    e.e1 = (float)(p0typ2tx - p0txp2ty);
    double p1txp0ty = (double)p1t.x * (double)p0t.y;
    double p1typ0tx = (double)p1t.y * (double)p0t.x;
    e.e2 = (float)(p1typ0tx - p1txp0ty);
    return e;
}

// shapes.cpp:172-273 IntersectTriangle (watertight, fp64 edge fallback), split so that the
// per-ray part (permutation and shear, shapes.cpp:180-200) is computed once per ray rather
// than once per triangle; the arithmetic and its order are unchanged.
struct TriRay {
    V3 o;
    int kx, ky, kz;
    float Sx, Sy, Sz;
};
PHD TriRay MakeTriRay(V3 o, V3 dir) {
    TriRay r;
    r.o = o;
    r.kz = MaxComponentIndex(Abs(dir));
    r.kx = r.kz + 1;
    if (r.kx == 3) r.kx = 0;
    r.ky = r.kx + 1;
    if (r.ky == 3) r.ky = 0;
    V3 d = Permute(dir, r.kx, r.ky, r.kz);
    r.Sx = -d.x / d.z;
    r.Sy = -d.y / d.z;
    r.Sz = 1 / d.z;
    return r;
}
// Triangle test for a non-degenerate triangle (callers drop degenerate triangles, the
// shapes.cpp:175 early-out, before calling).
PHD bool IntersectTriangleRay(const TriRay &r, float tMax, V3 p0, V3 p1, V3 p2, TriHit *hit) {
    V3 p0t = Permute(p0 - r.o, r.kx, r.ky, r.kz);
    V3 p1t = Permute(p1 - r.o, r.kx, r.ky, r.kz);
    V3 p2t = Permute(p2 - r.o, r.kx, r.ky, r.kz);
    const float Sx = r.Sx, Sy = r.Sy, Sz = r.Sz;
    p0t.x += Sx * p0t.z;
    p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z;
    p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z;
    p2t.y += Sy * p2t.z;
    float e0 = DifferenceOfProducts(p1t.x, p2t.y, p1t.y, p2t.x);
    float e1 = DifferenceOfProducts(p2t.x, p0t.y, p2t.y, p0t.x);
    float e2 = DifferenceOfProducts(p0t.x, p1t.y, p0t.y, p1t.x);
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        const EdgeFns e = EdgeFunctionsFP64(p0t, p1t, p2t);
        e0 = e.e0, e1 = e.e1, e2 = e.e2;
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz;
    p1t.z *= Sz;
    p2t.z *= Sz;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < tMax * det)) return false;
    if (det > 0 && (tScaled <= 0 || tScaled > tMax * det)) return false;
    float invDet = 1 / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    float t = tScaled * invDet;
    float maxZt = MaxComponentValue(Abs(V3(p0t.z, p1t.z, p2t.z)));
    float deltaZ = gamma(3) * maxZt;
    float maxXt = MaxComponentValue(Abs(V3(p0t.x, p1t.x, p2t.x)));
    float maxYt = MaxComponentValue(Abs(V3(p0t.y, p1t.y, p2t.y)));
    float deltaX = gamma(5) * (maxXt + maxZt);
    float deltaY = gamma(5) * (maxYt + maxZt);
    float deltaE = 2 * (gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = MaxComponentValue(Abs(V3(e0, e1, e2)));
    float deltaT = 3 * (gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::fabs(invDet);
    if (t <= deltaT) return false;
    hit->b0 = b0;
    hit->b1 = b1;
    hit->b2 = b2;
    hit->t = t;
    return true;
}

PHD bool TriangleDegenerate(V3 p0, V3 p1, V3 p2) { return LengthSquared(Cross(p2 - p0, p1 - p0)) == 0; }

PHD bool IntersectTriangle(V3 o, V3 dir, float tMax, V3 p0, V3 p1, V3 p2, TriHit *hit) {
    if (TriangleDegenerate(p0, p1, p2)) return false;
    return IntersectTriangleRay(MakeTriRay(o, dir), tMax, p0, p1, p2, hit);
}

// Surface geometry of a triangle hit without shading normals or uv
// (shapes.h:884-1010, mesh without n/s/uv: default uv (0,0),(1,0),(1,1)).
// Per-triangle shading attributes of TriangleMesh (util/mesh.h:23-46): vertex normals and
// uv, each optional (flags bit0 / bit1).
struct TriShading {
    int flags = 0;      // bit0 vertex normals, bit1 uv, bit2 shading tangents S
    V3 n0, n1, n2;
    float uv[3][2];
    V3 s0, s1, s2;
};
struct TriSurface {
    V3 p, pErr, n, dpdu;
    V3 ns, dpdus;  // shading normal and shading dpdu (== n, dpdu without vertex normals)
    V3 dpdv;       // geometric dpdv and the hit's uv (texture lookups, surfscatter.cpp:74-104)
    float uv[2];
};
// Triangle::InteractionFromIntersection (shapes.h:884-1010) without the dndu/dndv terms (bump
// mapping / ray differentials only) and with SetShadingGeometry(..., true) (interaction.h:194)
PHD TriSurface TriangleSurface(V3 p0, V3 p1, V3 p2, float b0, float b1, float b2, bool flip,
                               const TriShading *sh = nullptr) {
    TriSurface s;
    float uv[3][2] = {{0, 0}, {1, 0}, {1, 1}};
    if (sh && (sh->flags & 2))
        for (int k = 0; k < 3; ++k) uv[k][0] = sh->uv[k][0], uv[k][1] = sh->uv[k][1];
    const float duv02x = uv[0][0] - uv[2][0], duv02y = uv[0][1] - uv[2][1];
    const float duv12x = uv[1][0] - uv[2][0], duv12y = uv[1][1] - uv[2][1];
    V3 dp02 = p0 - p2, dp12 = p1 - p2;
    float determinant = DifferenceOfProducts(duv02x, duv12y, duv02y, duv12x);
    V3 dpdu, dpdv;
    bool degenerateUV = std::fabs(determinant) < 1e-9f;
    if (!degenerateUV) {
        float invdet = 1 / determinant;
        dpdu = V3(DifferenceOfProducts(duv12y, dp02.x, duv02y, dp12.x),
                  DifferenceOfProducts(duv12y, dp02.y, duv02y, dp12.y),
                  DifferenceOfProducts(duv12y, dp02.z, duv02y, dp12.z)) *
               invdet;
        dpdv = V3(DifferenceOfProducts(duv02x, dp12.x, duv12x, dp02.x),
                  DifferenceOfProducts(duv02x, dp12.y, duv12x, dp02.y),
                  DifferenceOfProducts(duv02x, dp12.z, duv12x, dp02.z)) *
               invdet;
    }
    if (degenerateUV || LengthSquared(Cross(dpdu, dpdv)) == 0) {
        V3 ng = Cross(p2 - p0, p1 - p0);
        CoordinateSystem(Normalize(ng), &dpdu, &dpdv);
    }
    V3 pHit = b0 * p0 + b1 * p1 + b2 * p2;
    V3 pAbsSum = Abs(b0 * p0) + Abs(b1 * p1) + Abs(b2 * p2);
    ToPoint3fi(pHit, gamma(7) * pAbsSum, &s.p, &s.pErr);
    s.dpdv = dpdv;
    s.uv[0] = b0 * uv[0][0] + b1 * uv[1][0] + b2 * uv[2][0];
    s.uv[1] = b0 * uv[0][1] + b1 * uv[1][1] + b2 * uv[2][1];
    V3 n = Normalize(Cross(dp02, dp12));
    if (flip) n = -n;
    s.n = n;
    s.dpdu = dpdu;
    s.ns = n;
    s.dpdus = dpdu;
    if (sh && (sh->flags & 5)) {  // mesh->n || mesh->s (shapes.h:940-960)
        V3 ns = s.n;
        if (sh->flags & 1) {
            ns = b0 * sh->n0 + b1 * sh->n1 + b2 * sh->n2;
            ns = LengthSquared(ns) > 0 ? Normalize(ns) : s.n;
        }
        V3 ss = s.dpdu;
        if (sh->flags & 4) {
            ss = b0 * sh->s0 + b1 * sh->s1 + b2 * sh->s2;
            if (LengthSquared(ss) == 0) ss = s.dpdu;
        }
        V3 ts = Cross(ns, ss);
        if (LengthSquared(ts) > 0) ss = Cross(ts, ns);
        else CoordinateSystem(ns, &ss, &ts);
        s.ns = ns;
        s.n = FaceForwardN(s.n, ns);
        while (LengthSquared(ss) > 1e16f || LengthSquared(ts) > 1e16f) {
            ss = ss / 1e8f;
            ts = ts / 1e8f;
        }
        s.dpdus = ss;
    }
    return s;
}
// Triangle::Sample's normal for a sampled point with barycentrics b (shapes.h:1023-1029)
PHD V3 TriangleSampleNormal(V3 p0, V3 p1, V3 p2, float b0, float b1, bool flip, const TriShading *sh) {
    V3 n = Normalize(Cross(p1 - p0, p2 - p0));
    if (sh && (sh->flags & 1)) {
        V3 ns = b0 * sh->n0 + b1 * sh->n1 + (1 - b0 - b1) * sh->n2;
        n = FaceForwardN(n, ns);
    } else if (flip) {
        n = n * -1.f;
    }
    return n;
}

// ---------------------------------------------------------------- spectra
// util/color.h:341 RGBSigmoidPolynomial; EvaluatePolynomial(l, c2, c1, c0) uses FMA.
//
// On the device the correctly rounded sqrt and division are formed without the range-scaling
// and special-case steps of the compiler's IEEE sequences, which cannot act here: the sqrt
// operand 1 + x^2 is >= 1 (v_sqrt + the same one-ulp correction; +inf passes through), and
// the division x / t has t = 2 sqrt(1 + x^2) in [2, inf] with |x| <= t / 2, so the exponent
// difference is small and the quotient is a normal number or below 2^-26 in magnitude --
// where .5 + q is .5 whatever its last bits.  t = inf (|x| > 2^64) divides to 0 as in pbrt.
// Bit-identical to the plain expression (tests/test_gpu_rn_math.py).
PHD float SigmoidPolynomial(float c0, float c1, float c2, float lambda) {
    float x = fmaf(lambda, fmaf(lambda, c0, c1), c2);
    if (std::isinf(x)) return x > 0 ? 1 : 0;
#if defined(__HIP_DEVICE_COMPILE__)
    const float v = 1 + Sqr(x);
    const float s0 = __builtin_amdgcn_sqrtf(v);
    const float dn = __uint_as_float(__float_as_uint(s0) - 1u), up = __uint_as_float(__float_as_uint(s0) + 1u);
    float s = fmaf(-dn, s0, v) <= 0.f ? dn : s0;
    s = fmaf(-up, s0, v) > 0.f ? up : s;
    const float t = 2 * s;
    float y = __builtin_amdgcn_rcpf(t);
    y = fmaf(fmaf(-t, y, 1.0f), y, y);
    float q = x * y;
    float r = fmaf(-t, q, x);
    q = fmaf(r, y, q);
    r = fmaf(-t, q, x);
    q = fmaf(r, y, q);
    if (x == 0.f) q = x * y;       // the correctly signed zero
    if (t == kInfinity) q = x * 0.f;  // x / inf (y is NaN here)
    return .5f + q;
#else
    return .5f + x / (2 * std::sqrt(1 + Sqr(x)));
#endif
}
// the plain expression, for the device self-check
PHD float SigmoidPolynomialPlain(float c0, float c1, float c2, float lambda) {
    float x = fmaf(lambda, fmaf(lambda, c0, c1), c2);
    if (std::isinf(x)) return x > 0 ? 1 : 0;
    return .5f + x / (2 * std::sqrt(1 + Sqr(x)));
}

// x / p, correctly rounded, from y = RN(1 / p): the kernels divide a whole spectrum by one
// scalar (beta * f * |cos| / pdf, beta / (1 - q)), so the reciprocal is one IEEE division per
// path and each element takes q = x y and two residual corrections r = fma(-p, q, x),
// q = fma(r, y, q) instead of the compiler's ten-instruction division.  Markstein: with y the
// correctly rounded reciprocal and q within an ulp of x / p, one correction rounds correctly;
// the first correction brings x y within that ulp.  DivFastOk: exponent in [-60, 60], where the
// quotient, the exact residual (a multiple of 2^(e_x - 46)) and every intermediate are normal
// and finite; any other operand (0, subnormal, inf, NaN, huge) takes the IEEE division.
// Bit-identical to x / p (tests/test_gpu_rn_math.py).
PHD bool DivFastOk(float x) { return ((FloatToBits(x) >> 23) & 0xffu) - 67u <= 120u; }
PHD float DivByRcp(float x, float p, float y, bool pOk) {
#if defined(__HIP_DEVICE_COMPILE__)
    float q = x * y;
    float r = fmaf(-p, q, x);
    q = fmaf(r, y, q);
    r = fmaf(-p, q, x);
    q = fmaf(r, y, q);
    if (!(pOk && DivFastOk(x))) {
        asm volatile("");  // keeps the rare IEEE path a branch (an fdiv alone would be if-converted)
        q = x / p;
    }
    return q;
#else
    (void)y, (void)pOk;
    return x / p;
#endif
}

// util/spectrum.h:318 SampledWavelengths::SampleUniform (sequential adds, wrap)
PHD void SampleWavelengthsUniform(float u, float lambda[kNSpectrumSamples]) {
    lambda[0] = Lerpf(u, kLambdaMin, kLambdaMax);
    const float delta = (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
    for (int i = 1; i < kNSpectrumSamples; ++i) {
        lambda[i] = lambda[i - 1] + delta;
        if (lambda[i] > kLambdaMax) lambda[i] = kLambdaMin + (lambda[i] - kLambdaMax);
    }
}
// DenselySampledSpectrum offset (util/spectrum.h:420): lround(lambda) - 395, 311 entries.
// Only lambda in [394.5, 705.5) has an entry; there lambda + 0.5f is exact (lambda's ulp is
// 2^-15 below 512 and 2^-14 above, the sum stays below 1024 and never crosses a binade edge
// with bits to drop), so floor(lambda + 0.5) is lround(lambda): a 32-bit form of the 64-bit
// lround sequence (tests/test_golden_product_host.py checks every float in the range).
PHD int DenseOffset(float lambda) {
    return (lambda >= 394.5f && lambda < 705.5f) ? (int)std::floor(lambda + 0.5f) - 395 : -1;
}
// Average of 31 copies of x (SampledSpectrum::Average of a constant spectrum)
PHD float Avg31(float x) {
    float s = x;
    for (int i = 1; i < kNSpectrumSamples; ++i) s += x;
    return s / kNSpectrumSamples;
}

// 24-bit unsigned multiply as the full-rate v_mul_u32_u24.  __umul24 masks its operands and
// relies on the backend to see 24-bit operands; once the compiler has folded the masks away by
// range reasoning it selects the quarter-rate 32-bit v_mul_lo_u32 instead.
PHD uint32_t MulU24(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return (a & 0xffffffu) * (b & 0xffffffu);
#endif
}

// ---------------------------------------------------------------- Halton
// util/lowdiscrepancy.h ScrambledRadicalInverse with digit permutations, index < 2^32.
// perm points at the permutation rows for this prime: perm[digit * base + value].
PHD_NOINLINE float ScrambledRadicalInverse(uint32_t base, uint32_t nDigits, uint64_t a, const uint16_t *perm) {
    float invBase = (float)1 / (float)base, invBaseM = 1;
    uint64_t reversedDigits = 0;
    for (uint32_t digitIndex = 0; digitIndex < nDigits; ++digitIndex) {
        uint64_t next = a / base;
        int digitValue = (int)(a - next * base);
        reversedDigits = reversedDigits * base + perm[digitIndex * base + digitValue];
        invBaseM *= invBase;
        a = next;
    }
    return std::fmin(invBaseM * (float)reversedDigits, kOneMinusEpsilon);
}
// One Halton dimension (HaltonSampler::SampleDimension -> ScrambledRadicalInverse with
// DigitPermutation, samplers.h:78-87, util/lowdiscrepancy.h:115-134) as the kernels evaluate it.
// pbrt's loop keeps reversedDigits as an exact uint64 and converts it to Float once at the end,
// so any exact evaluation of the same integer gives the same float.  For indices a < 2^24 the
// kernels form it as:
//  * digits by one float multiply: q = trunc(float(a) * rcp) with rcp = float(1/b): float(a) is
//    exact and the product is within a / b * 2^-23 < 1 of a / b for a < 2^24, so q is
//    floor(a / b) - 1, + 0 or + 1; the remainder's sign and size fix it (the integer products
//    q * b are 24-bit multiplies);
//  * reversedDigits = reversedDigits * b + perm by fma in double, exact because it stays below
//    b^nDigits < 2^53;
//  * invBaseM precomputed by the same float product chain as pbrt's loop.
// Larger indices take the 64-bit restatement above.  No 32/64-bit integer division remains on
// the fast path (pbrt's a / base is a 64-bit division; here it was most of the sampler's cost).
struct HaltonDimDesc {
    uint32_t base, nDigits, permOffset, tail;  // tail, tailMul: HaltonDimTail
    float invBase, invBaseM, rcp, tailMul;
    uint32_t nz;  // digit steps of the fast forms (<= 6): every index they see is < base^nz
};
PHD HaltonDimDesc MakeHaltonDimDesc(uint32_t base, uint32_t nDigits, uint32_t permOffset) {
    HaltonDimDesc d{};
    d.base = base;
    d.nDigits = nDigits;
    d.permOffset = permOffset;
    d.invBase = (float)1 / (float)base;
    float invBaseM = 1;
    for (uint32_t k = 0; k < nDigits; ++k) invBaseM *= d.invBase;
    d.invBaseM = invBaseM;
    d.rcp = (float)(1.0 / base);
    d.tail = 0;
    d.tailMul = 1;
    d.nz = 6;
    return d;
}
// The digits past the nz-th of an index a < base^nz are all zero, so they add the constant
// tail = sum_{k=nz}^{n-1} perm[k base] base^(n-1-k) after scaling the nz-digit value by
// tailMul = base^(n-nz) (ScrambledRadicalInverse24x6, HaltonDepthSamples).  Both are exact
// integers far below 2^24.
PHD void HaltonDimTail(HaltonDimDesc *d, const uint16_t *perm, uint32_t nz = 6) {
    d->nz = nz;
    d->tail = 0;
    d->tailMul = 1;
    if (d->nDigits <= nz) return;
    uint32_t t = 0, m = 1;
    for (uint32_t k = nz; k < d->nDigits; ++k) {
        t = t * d->base + perm[k * d->base];
        m *= d->base;
    }
    d->tail = t;
    d->tailMul = (float)m;
}
// MaxDigits >= d.nDigits: the digit loop is unrolled to that bound (iterations past nDigits are
// skipped by a launch-uniform test) and every permutation load is issued before the first is
// used, so a dimension costs one memory round trip, not nDigits of them.
template <int MaxDigits, typename PermPtr>
PHD float ScrambledRadicalInverse24(const HaltonDimDesc &d, uint32_t a, PermPtr perm) {
    // b < 2^24 made visible to the compiler, so __umul24 is the full-rate v_mul_u32_u24
    const uint32_t b = d.base & 0xffffffu, n = d.nDigits;
    uint32_t pv[MaxDigits];
PHD_UNROLL
    for (int k = 0; k < MaxDigits; ++k) {
        if ((uint32_t)k < n) {
            uint32_t q = (uint32_t)((float)a * d.rcp);
#if defined(__HIP_DEVICE_COMPILE__)
            int r = (int)a - (int)MulU24(q, b);
#else
            int r = (int)a - (int)(q * b);
#endif
            if (r < 0) {
                --q;
                r += (int)b;
            }
            if (r >= (int)b) {
                ++q;
                r -= (int)b;
            }
            pv[k] = perm[k * b + (uint32_t)r];
            a = q;
        }
    }
    double rd = 0;
PHD_UNROLL
    for (int k = 0; k < MaxDigits; ++k)
        if ((uint32_t)k < n) rd = fma(rd, (double)b, (double)pv[k]);
    return std::fmin(d.invBaseM * (float)rd, kOneMinusEpsilon);
}
// ScrambledRadicalInverse24 for a < base^6 (every shade-stage dimension: bases >= 17 and
// a < 2^24 < 17^6): six digit steps without branches -- a step at or past nDigits loads the
// table's first entry and is discarded by a select -- so the compiler can interleave the
// dimensions of a depth, then the remaining (zero) digits as one exact fma with the host's tail.
// reversedDigits stays an exact integer in double throughout, so the result is the same float.
template <typename PermPtr>
PHD float ScrambledRadicalInverse24x6(const HaltonDimDesc &d, uint32_t a, PermPtr perm) {
    const uint32_t b = d.base & 0xffffffu, n = d.nDigits;
    uint32_t pv[6];
PHD_UNROLL
    for (int k = 0; k < 6; ++k) {
        uint32_t q = (uint32_t)((float)a * d.rcp);
#if defined(__HIP_DEVICE_COMPILE__)
        int r = (int)a - (int)MulU24(q, b);
#else
        int r = (int)a - (int)(q * b);
#endif
        q = r < 0 ? q - 1 : q;
        r = r < 0 ? r + (int)b : r;
        q = r >= (int)b ? q + 1 : q;
        r = r >= (int)b ? r - (int)b : r;
        const bool ok = (uint32_t)k < n;
        pv[k] = perm[ok ? (uint32_t)k * b + (uint32_t)r : 0u];
        a = q;
    }
    double rd = 0;
PHD_UNROLL
    for (int k = 0; k < 6; ++k) rd = (uint32_t)k < n && (uint32_t)k < d.nz ? fma(rd, (double)b, (double)pv[k]) : rd;
    rd = fma(rd, (double)d.tailMul, (double)d.tail);
    return std::fmin(d.invBaseM * (float)rd, kOneMinusEpsilon);
}
// HaltonDigitsFor: the digit steps an index below bound needs in base b (bound <= 2^24, b >= 17:
// at most 6)
inline uint32_t HaltonDigitsFor(uint32_t b, uint64_t bound) {
    uint32_t k = 0;
    for (uint64_t p = 1; p < bound; p *= b) ++k;
    return k;
}
// The seven dimensions of one depth (ScrambledRadicalInverse24x6 of each) digit-major: the host
// gave the seven the same nz (digits every index of the render has, HaltonDigitsFor of the
// largest), so the digit steps past nz are skipped by a launch-uniform branch and the seven
// quotient chains interleave inside each step.  The result is the same float per dimension:
// digits past nz are zero and their permuted values sit in the host's tail, as past the sixth.
// Skip3: dimension 3 (indirect.uc) is not needed.
template <bool Skip3, typename PermPtr>
PHD void HaltonDepthSamples(const HaltonDimDesc *d, uint32_t a0, const PermPtr *perm, float *out) {
    const uint32_t nz = d[0].nz;
    uint32_t a[7], pv[6][7];
    double rd[7];
PHD_UNROLL
    for (int j = 0; j < 7; ++j) {
        a[j] = a0;
        rd[j] = 0;
    }
PHD_UNROLL
    for (int k = 0; k < 6; ++k) {
        if ((uint32_t)k < nz) {
PHD_UNROLL
            for (int j = 0; j < 7; ++j) {
                if (Skip3 && j == 3) continue;
                const uint32_t b = d[j].base & 0xffffffu;
                uint32_t q = (uint32_t)((float)a[j] * d[j].rcp);
#if defined(__HIP_DEVICE_COMPILE__)
                int r = (int)a[j] - (int)MulU24(q, b);
#else
                int r = (int)a[j] - (int)(q * b);
#endif
                q = r < 0 ? q - 1 : q;
                r = r < 0 ? r + (int)b : r;
                q = r >= (int)b ? q + 1 : q;
                r = r >= (int)b ? r - (int)b : r;
                const bool ok = (uint32_t)k < d[j].nDigits;
                pv[k][j] = perm[j][ok ? (uint32_t)k * b + (uint32_t)r : 0u];
                a[j] = q;
            }
PHD_UNROLL
            for (int j = 0; j < 7; ++j) {
                if (Skip3 && j == 3) continue;
                if ((uint32_t)k < d[j].nDigits) rd[j] = fma(rd[j], (double)(d[j].base & 0xffffffu), (double)pv[k][j]);
            }
        }
    }
PHD_UNROLL
    for (int j = 0; j < 7; ++j) {
        if (Skip3 && j == 3) {
            out[j] = 0;
            continue;
        }
        rd[j] = fma(rd[j], (double)d[j].tailMul, (double)d[j].tail);
        out[j] = std::fmin(d[j].invBaseM * (float)rd[j], kOneMinusEpsilon);
    }
}
constexpr int kMaxHaltonDigits24 = 25;  // base 2 (the largest digit count of any dimension)
constexpr int kMaxShadeHaltonDigits = 8;  // dimensions >= 6 (bases >= 17)
PHD float HaltonSampleDimension(const HaltonDimDesc &d, uint64_t index, const uint16_t *permTable) {
    if (index < (1ull << 24))
        return d.nDigits <= (uint32_t)kMaxShadeHaltonDigits
                   ? ScrambledRadicalInverse24<kMaxShadeHaltonDigits>(d, (uint32_t)index, permTable + d.permOffset)
                   : ScrambledRadicalInverse24<kMaxHaltonDigits24>(d, (uint32_t)index, permTable + d.permOffset);
    return ScrambledRadicalInverse(d.base, d.nDigits, index, permTable + d.permOffset);
}

// util/lowdiscrepancy.h RadicalInverse (unscrambled), used for the pixel sample
PHD float RadicalInverse(uint32_t base, uint64_t a) {
    uint64_t limit = ~0ull / base - base;
    float invBase = (float)1 / (float)base, invBaseM = 1;
    uint64_t reversedDigits = 0;
    while (a && reversedDigits < limit) {
        uint64_t next = a / base;
        uint64_t digit = a - next * base;
        reversedDigits = reversedDigits * base + digit;
        invBaseM *= invBase;
        a = next;
    }
    return std::fmin((float)reversedDigits * invBaseM, kOneMinusEpsilon);
}
// RadicalInverse for a < 2^30 and Base <= 3: the same digit loop in 32-bit integers.  The
// reversed digits stay below Base * a < 2^32 and the 64-bit limit (~2^62) is never reached,
// so digits and float rounding are identical; no 64-bit division.
template <uint32_t Base>
PHD float RadicalInverse32(uint32_t a) {
    static_assert(Base <= 3, "RadicalInverse32: Base * 2^30 must fit in 32 bits");
    float invBase = (float)1 / (float)Base, invBaseM = 1;
    uint32_t reversedDigits = 0;
    while (a) {
        uint32_t next = a / Base;
        uint32_t digit = a - next * Base;
        reversedDigits = reversedDigits * Base + digit;
        invBaseM *= invBase;
        a = next;
    }
    return std::fmin((float)reversedDigits * invBaseM, kOneMinusEpsilon);
}
PHD uint64_t InverseRadicalInverse(uint64_t inverse, int base, int nDigits) {
    uint64_t index = 0;
    for (int i = 0; i < nDigits; ++i) {
        uint64_t digit = inverse % base;
        inverse /= base;
        index = index * base + digit;
    }
    return index;
}

// ---------------------------------------------------------------- microfacet BxDFs
// TrowbridgeReitzDistribution (util/scattering.h:109-205), Fresnel terms and the dielectric /
// conductor BxDFs (bxdfs.h:300-510, bxdfs.cpp:77-245) in the local shading frame.  Vector dot
// products are plain; a dot with a Normal3f operand (Refract) is FMA-compensated (DotN).
enum BxDFFlagBits : int { kBxReflection = 1, kBxTransmission = 2, kBxDiffuse = 4, kBxGlossy = 8, kBxSpecular = 16 };

PHD float CosTheta(V3 w) { return w.z; }
PHD float Cos2Theta(V3 w) { return Sqr(w.z); }
PHD float AbsCosTheta(V3 w) { return std::fabs(w.z); }
PHD float Sin2Theta(V3 w) { return std::fmax(0.f, 1 - Cos2Theta(w)); }
PHD float SinTheta(V3 w) { return std::sqrt(Sin2Theta(w)); }
PHD float Tan2Theta(V3 w) { return Sin2Theta(w) / Cos2Theta(w); }
PHD float CosPhi(V3 w) {
    float sinTheta = SinTheta(w);
    return (sinTheta == 0) ? 1 : Clampf(w.x / sinTheta, -1, 1);
}
PHD float SinPhi(V3 w) {
    float sinTheta = SinTheta(w);
    return (sinTheta == 0) ? 0 : Clampf(w.y / sinTheta, -1, 1);
}
PHD bool SameHemisphere(V3 w, V3 wp) { return w.z * wp.z > 0; }
PHD V3 Reflect(V3 wo, V3 n) { return -wo + 2 * Dot(wo, n) * n; }
// util/scattering.h Refract: n is a Normal3f
PHD bool Refract(V3 wi, V3 n, float eta, float *etap, V3 *wt) {
    float cosTheta_i = DotN(n, wi);
    if (cosTheta_i < 0) {
        eta = 1 / eta;
        cosTheta_i = -cosTheta_i;
        n = -n;
    }
    float sin2Theta_i = std::fmax(0.f, 1 - Sqr(cosTheta_i));
    float sin2Theta_t = sin2Theta_i / Sqr(eta);
    if (sin2Theta_t >= 1) return false;
    float cosTheta_t = std::sqrt(1 - sin2Theta_t);
    *wt = -wi / eta + (cosTheta_i / eta - cosTheta_t) * n;
    *etap = eta;
    return true;
}
PHD float FrDielectric(float cosTheta_i, float eta) {
    cosTheta_i = Clampf(cosTheta_i, -1, 1);
    if (cosTheta_i < 0) {
        eta = 1 / eta;
        cosTheta_i = -cosTheta_i;
    }
    float sin2Theta_i = 1 - Sqr(cosTheta_i);
    float sin2Theta_t = sin2Theta_i / Sqr(eta);
    if (sin2Theta_t >= 1) return 1.f;
    float cosTheta_t = SafeSqrt(1 - sin2Theta_t);
    float r_parl = (eta * cosTheta_i - cosTheta_t) / (eta * cosTheta_i + cosTheta_t);
    float r_perp = (cosTheta_i - eta * cosTheta_t) / (cosTheta_i + eta * cosTheta_t);
    return (Sqr(r_parl) + Sqr(r_perp)) / 2;
}
// pstd::complex<float> arithmetic exactly as util/pstd.h:1066-1229 writes it
struct Cpx {
    float re, im;
};
PHD Cpx CAdd(Cpx a, Cpx b) { return {a.re + b.re, a.im + b.im}; }
PHD Cpx CSub(Cpx a, Cpx b) { return {a.re - b.re, a.im - b.im}; }
PHD Cpx CMul(Cpx a, Cpx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
PHD Cpx CDiv(Cpx a, Cpx z) {
    float scale = 1 / (z.re * z.re + z.im * z.im);
    return {scale * (a.re * z.re + a.im * z.im), scale * (a.im * z.re - a.re * z.im)};
}
PHD float CNorm(Cpx z) { return z.re * z.re + z.im * z.im; }
PHD Cpx CSqrt(Cpx z) {
    float n = std::sqrt(CNorm(z)), t1 = std::sqrt(0.5f * (n + std::fabs(z.re))), t2 = 0.5f * z.im / t1;
    if (n == 0) return {0, 0};
    if (z.re >= 0) return {t1, t2};
    return {std::fabs(t2), std::copysign(t1, z.im)};
}
// util/scattering.h FrComplex(Float cosTheta_i, complex eta)
PHD float FrComplex(float cosTheta_i, float etaRe, float etaIm) {
    const Cpx eta{etaRe, etaIm};
    cosTheta_i = Clampf(cosTheta_i, 0, 1);
    float sin2Theta_i = 1 - Sqr(cosTheta_i);
    Cpx sin2Theta_t = CDiv(Cpx{sin2Theta_i, 0}, CMul(eta, eta));
    Cpx cosTheta_t = CSqrt(CSub(Cpx{1, 0}, sin2Theta_t));
    Cpx ec = CMul(eta, Cpx{cosTheta_i, 0});
    Cpx r_parl = CDiv(CSub(ec, cosTheta_t), CAdd(ec, cosTheta_t));
    Cpx et = CMul(eta, cosTheta_t);
    Cpx r_perp = CDiv(CSub(Cpx{cosTheta_i, 0}, et), CAdd(Cpx{cosTheta_i, 0}, et));
    return (CNorm(r_parl) + CNorm(r_perp)) / 2;
}
struct TrowbridgeReitz {
    float ax, ay;
    PHD static TrowbridgeReitz Make(float ax, float ay) {
        TrowbridgeReitz t{ax, ay};
        if (!t.EffectivelySmooth()) {
            t.ax = std::fmax(t.ax, 1e-4f);
            t.ay = std::fmax(t.ay, 1e-4f);
        }
        return t;
    }
    PHD bool EffectivelySmooth() const { return std::fmax(ax, ay) < 1e-3f; }
    PHD void Regularize() {
        if (ax < 0.3f) ax = Clampf(2 * ax, 0.1f, 0.3f);
        if (ay < 0.3f) ay = Clampf(2 * ay, 0.1f, 0.3f);
    }
    PHD float D(V3 wm) const {
        float tan2Theta = Tan2Theta(wm);
        if (std::isinf(tan2Theta)) return 0;
        float cos4Theta = Sqr(Cos2Theta(wm));
        if (cos4Theta < 1e-16f) return 0;
        float e = tan2Theta * (Sqr(CosPhi(wm) / ax) + Sqr(SinPhi(wm) / ay));
        return 1 / (kPi * ax * ay * cos4Theta * Sqr(1 + e));
    }
    PHD float Lambda(V3 w) const {
        float tan2Theta = Tan2Theta(w);
        if (std::isinf(tan2Theta)) return 0;
        float alpha2 = Sqr(CosPhi(w) * ax) + Sqr(SinPhi(w) * ay);
        return (std::sqrt(1 + alpha2 * tan2Theta) - 1) / 2;
    }
    PHD float G1(V3 w) const { return 1 / (1 + Lambda(w)); }
    PHD float G(V3 wo, V3 wi) const { return 1 / (1 + Lambda(wo) + Lambda(wi)); }
    PHD float D(V3 w, V3 wm) const { return G1(w) / AbsCosTheta(w) * D(wm) * AbsDot(w, wm); }
    PHD float PDF(V3 w, V3 wm) const { return D(w, wm); }
    PHD V3 SampleWm(V3 w, float u0, float u1) const {
        V3 wh = Normalize(V3(ax * w.x, ay * w.y, w.z));
        if (wh.z < 0) wh = -wh;
        V3 T1 = (wh.z < 0.99999f) ? Normalize(Cross(V3(0, 0, 1), wh)) : V3(1, 0, 0);
        V3 T2 = Cross(wh, T1);
        // SampleUniformDiskPolar (util/sampling.h:311-315)
        float r = std::sqrt(u0), theta = 2 * kPi * u1;
        float px = r * Cosf(theta), py = r * Sinf(theta);
        float h = std::sqrt(1 - Sqr(px));
        py = Lerpf((1 + wh.z) / 2, h, py);
        float pz = std::sqrt(std::fmax(0.f, 1 - (Sqr(px) + Sqr(py))));
        V3 nh = px * T1 + py * T2 + pz * wh;
        return Normalize(V3(ax * nh.x, ay * nh.y, std::fmax(1e-6f, nh.z)));
    }
};
// PiecewiseLinearSpectrum::operator() (util/spectrum.cpp:68-78): FindInterval's result is the
// largest knot index o <= n-2 with lambda[o] <= l
template <typename F>  // const float, or its LDS-qualified form
PHD float PiecewiseLinearEval(F *lam, F *val, int n, float l) {
    if (n == 0 || l < lam[0] || l > lam[n - 1]) return 0;
    int lo = 0, hi = n - 2;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (lam[mid] <= l) lo = mid;
        else hi = mid - 1;
    }
    float t = (l - lam[lo]) / (lam[lo + 1] - lam[lo]);
    return Lerpf(t, val[lo], val[lo + 1]);
}
// The same evaluation started from a per-nanometre segment table: idx[b] = the FindInterval
// result at lambda = kPlIndexLo + b.  FindInterval is monotone in lambda, so for l >= that
// wavelength the answer is idx[b] or a later segment, reached by the forward walk (knots are
// >= 1 nm apart in pbrt's named spectra: at most one step).  Same segment, same arithmetic.
constexpr int kPlIndexLo = 360, kPlIndexN = 471;  // 360..830 nm (SampleVisibleWavelengths)
template <typename F, typename I>
PHD float PiecewiseLinearEvalIdx(F *lam, F *val, int n, I *idx, float l) {
    if (n == 0 || l < lam[0] || l > lam[n - 1]) return 0;
    const int b = (int)l - kPlIndexLo;
    int lo = idx[b < 0 ? 0 : (b >= kPlIndexN ? kPlIndexN - 1 : b)];
    float l1 = lam[lo + 1];
    while (lo < n - 2 && l1 <= l) l1 = lam[++lo + 1];
    const float l0 = lam[lo];
    float t = (l - l0) / (l1 - l0);
    return Lerpf(t, val[lo], val[lo + 1]);
}
// idx[b] for PiecewiseLinearEvalIdx (host): FindInterval at kPlIndexLo + b
inline void BuildPlIndex(const float *lam, int n, uint16_t *idx) {
    for (int b = 0; b < kPlIndexN; ++b) {
        const float l = (float)(kPlIndexLo + b);
        int o = 0;
        while (o < n - 2 && lam[o + 1] <= l) ++o;
        idx[b] = (uint16_t)o;
    }
}
// RoughnessToAlpha (util/scattering.h:192)
PHD float RoughnessToAlpha(float roughness) { return std::sqrt(roughness); }

// A sampled BxDF direction.  f is the scalar BSDF value (dielectric); for the conductor the
// spectral value is evaluated per wavelength from the geometry terms (ConductorTerms).
struct BxSample {
    bool ok;
    V3 wi;
    float f, pdf, etap;
    int flags;
};
PHD int DielectricFlags(float eta, const TrowbridgeReitz &tr) {
    int flags = (eta == 1) ? kBxTransmission : (kBxReflection | kBxTransmission);
    return flags | (tr.EffectivelySmooth() ? kBxSpecular : kBxGlossy);
}
// BxDFReflTransFlags (bxdf.h): which lobes a Sample_f / PDF call may use
constexpr int kSampleR = 1, kSampleT = 2, kSampleAll = 3;
// DielectricBxDF::Sample_f (bxdfs.cpp:77-170); radiance = TransportMode::Radiance (the
// 1/etap^2 factor on transmission), sampleFlags restricts the lobes (LayeredBxDF)
PHD BxSample DielectricSample(float eta, const TrowbridgeReitz &tr, V3 wo, float uc, float u0, float u1,
                              bool radiance = true, int sampleFlags = kSampleAll) {
    BxSample s{false, V3(0, 0, 0), 0, 0, 1, 0};
    if (eta == 1 || tr.EffectivelySmooth()) {
        float R = FrDielectric(CosTheta(wo), eta), T = 1 - R;
        float pr = R, pt = T;
        if (!(sampleFlags & kSampleR)) pr = 0;
        if (!(sampleFlags & kSampleT)) pt = 0;
        if (pr == 0 && pt == 0) return s;
        if (uc < pr / (pr + pt)) {
            V3 wi(-wo.x, -wo.y, wo.z);
            s = BxSample{true, wi, R / AbsCosTheta(wi), pr / (pr + pt), 1, kBxSpecular | kBxReflection};
            return s;
        }
        V3 wi;
        float etap;
        if (!Refract(wo, V3(0, 0, 1), eta, &etap, &wi)) return s;
        float ft = T / AbsCosTheta(wi);
        if (radiance) ft /= Sqr(etap);
        s = BxSample{true, wi, ft, pt / (pr + pt), etap, kBxSpecular | kBxTransmission};
        return s;
    }
    V3 wm = tr.SampleWm(wo, u0, u1);
    float R = FrDielectric(Dot(wo, wm), eta);
    float T = 1 - R;
    float pr = R, pt = T;
    if (!(sampleFlags & kSampleR)) pr = 0;
    if (!(sampleFlags & kSampleT)) pt = 0;
    if (pr == 0 && pt == 0) return s;
    if (uc < pr / (pr + pt)) {
        V3 wi = Reflect(wo, wm);
        if (!SameHemisphere(wo, wi)) return s;
        float pdf = tr.PDF(wo, wm) / (4 * AbsDot(wo, wm)) * pr / (pr + pt);
        float f = tr.D(wm) * tr.G(wo, wi) * R / (4 * CosTheta(wi) * CosTheta(wo));
        s = BxSample{true, wi, f, pdf, 1, kBxGlossy | kBxReflection};
        return s;
    }
    float etap;
    V3 wi;
    bool tir = !Refract(wo, wm, eta, &etap, &wi);
    if (SameHemisphere(wo, wi) || wi.z == 0 || tir) return s;
    float denom = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap);
    float dwm_dwi = AbsDot(wi, wm) / denom;
    float pdf = tr.PDF(wo, wm) * dwm_dwi * pt / (pr + pt);
    float ft = T * tr.D(wm) * tr.G(wo, wi) * std::fabs(Dot(wi, wm) * Dot(wo, wm) / (CosTheta(wi) * CosTheta(wo) * denom));
    if (radiance) ft /= Sqr(etap);
    s = BxSample{true, wi, ft, pdf, etap, kBxGlossy | kBxTransmission};
    return s;
}
// ThinDielectricBxDF::Sample_f (bxdfs.h:355-386): specular reflection / straight-through
// transmission with the inter-reflections of a thin slab folded into R and T
PHD BxSample ThinDielectricSample(float eta, V3 wo, float uc) {
    float R = FrDielectric(AbsCosTheta(wo), eta), T = 1 - R;
    if (R < 1) {
        R += Sqr(T) * R / (1 - Sqr(R));
        T = 1 - R;
    }
    const float pr = R, pt = T;
    if (pr == 0 && pt == 0) return BxSample{false, V3(0, 0, 0), 0, 0, 1, 0};
    if (uc < pr / (pr + pt)) {
        const V3 wi(-wo.x, -wo.y, wo.z);
        return BxSample{true, wi, R / AbsCosTheta(wi), pr / (pr + pt), 1, kBxSpecular | kBxReflection};
    }
    const V3 wi = -wo;
    return BxSample{true, wi, T / AbsCosTheta(wi), pt / (pr + pt), 1, kBxSpecular | kBxTransmission};
}
// DielectricBxDF::f and ::PDF (bxdfs.cpp:172-245); pdfOut may be null
PHD float DielectricEval(float eta, const TrowbridgeReitz &tr, V3 wo, V3 wi, float *pdfOut, bool radiance = true,
                         int sampleFlags = kSampleAll) {
    if (pdfOut) *pdfOut = 0;
    if (eta == 1 || tr.EffectivelySmooth()) return 0;
    float cosTheta_o = CosTheta(wo), cosTheta_i = CosTheta(wi);
    bool reflect = cosTheta_i * cosTheta_o > 0;
    float etap = 1;
    if (!reflect) etap = cosTheta_o > 0 ? eta : (1 / eta);
    V3 wm = wi * etap + wo;
    if (cosTheta_i == 0 || cosTheta_o == 0 || LengthSquared(wm) == 0) return 0;
    wm = FaceForward(Normalize(wm), V3(0, 0, 1));
    if (Dot(wm, wi) * cosTheta_i < 0 || Dot(wm, wo) * cosTheta_o < 0) return 0;
    float F = FrDielectric(Dot(wo, wm), eta);
    float R = F, T = 1 - R, pr = R, pt = T;
    if (!(sampleFlags & kSampleR)) pr = 0;
    if (!(sampleFlags & kSampleT)) pt = 0;
    if (reflect) {
        if (pdfOut && !(pr == 0 && pt == 0)) *pdfOut = tr.PDF(wo, wm) / (4 * AbsDot(wo, wm)) * pr / (pr + pt);
        return tr.D(wm) * tr.G(wo, wi) * F / std::fabs(4 * cosTheta_i * cosTheta_o);
    }
    float denom = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap) * cosTheta_i * cosTheta_o;
    float ft = tr.D(wm) * (1 - F) * tr.G(wo, wi) * std::fabs(Dot(wi, wm) * Dot(wo, wm) / denom);
    if (radiance) ft /= Sqr(etap);
    if (pdfOut && !(pr == 0 && pt == 0)) {
        float denomP = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap);
        float dwm_dwi = AbsDot(wi, wm) / denomP;
        *pdfOut = tr.PDF(wo, wm) * dwm_dwi * pt / (pr + pt);
    }
    return ft;
}
// ConductorBxDF (bxdfs.h:413-510).  f is spectral: the geometry-only terms are returned and
// ConductorF combines them with each wavelength's Fresnel factor in pbrt's operation order.
struct ConductorTerms {
    bool ok, specular;
    V3 wi;
    float pdf;
    float D, G, cosI, cosO;  // rough: f = D * F * G / (4 * cosI * cosO)
    float cosF;              // argument of FrComplex; specular: f = Fr / cosI
};
PHD float ConductorF(const ConductorTerms &t, float eta, float k) {
    float F = FrComplex(t.cosF, eta, k);
    if (t.specular) return F / t.cosI;
    return t.D * F * t.G / (4 * t.cosI * t.cosO);
}
PHD ConductorTerms ConductorSample(const TrowbridgeReitz &tr, V3 wo, float u0, float u1) {
    ConductorTerms c{false, false, V3(0, 0, 0), 0, 0, 0, 0, 0, 0};
    if (tr.EffectivelySmooth()) {
        V3 wi(-wo.x, -wo.y, wo.z);
        c.ok = true;
        c.specular = true;
        c.wi = wi;
        c.pdf = 1;
        c.cosI = AbsCosTheta(wi);
        c.cosF = AbsCosTheta(wi);
        return c;
    }
    if (wo.z == 0) return c;
    V3 wm = tr.SampleWm(wo, u0, u1);
    V3 wi = Reflect(wo, wm);
    if (!SameHemisphere(wo, wi)) return c;
    float pdf = tr.PDF(wo, wm) / (4 * AbsDot(wo, wm));
    float cosTheta_o = AbsCosTheta(wo), cosTheta_i = AbsCosTheta(wi);
    if (cosTheta_i == 0 || cosTheta_o == 0) return c;
    c = ConductorTerms{true, false, wi, pdf, tr.D(wm), tr.G(wo, wi), cosTheta_i, cosTheta_o, AbsDot(wo, wm)};
    return c;
}
// ConductorBxDF::f / ::PDF geometry for a given wi (ok = false: f = 0, pdf = 0)
PHD ConductorTerms ConductorEval(const TrowbridgeReitz &tr, V3 wo, V3 wi) {
    ConductorTerms c{false, false, wi, 0, 0, 0, 0, 0, 0};
    if (!SameHemisphere(wo, wi) || tr.EffectivelySmooth()) return c;
    float cosTheta_o = AbsCosTheta(wo), cosTheta_i = AbsCosTheta(wi);
    V3 wm = wi + wo;
    if (cosTheta_i == 0 || cosTheta_o == 0 || LengthSquared(wm) == 0) return c;
    wm = Normalize(wm);
    // PDF: wm faced forward; f: not (FrComplex uses |dot|, D and G are even in wm)
    V3 wmf = FaceForward(wm, V3(0, 0, 1));
    c = ConductorTerms{true, false, wi, tr.PDF(wo, wmf) / (4 * AbsDot(wo, wmf)), tr.D(wm), tr.G(wo, wi), cosTheta_i,
                       cosTheta_o, AbsDot(wo, wm)};
    return c;
}

// RetroreflectiveBxDF, this fork's material (bxdfs.h:102-215), kept with its quirks:
//  * Sample_f: the smooth case returns wi = wo (FrComplex(|cos wi|) / |cos wi|, pdf 1); the rough
//    case is ConductorBxDF's microfacet reflection sample with the conductor's f (no retro lobe);
//  * f: (1 - (R_i - R_o)) times the sum of a retro lobe (D(wo), Fresnel at |wi . wo|) and the
//    conductor lobe, R_o = FrDielectric(wo . wm, 1.59), R_i = FrDielectric(wi . wo, 1.59);
//  * PDF: the conductor's, which ignores the retro lobe.
PHD int RetroFlags(const TrowbridgeReitz &tr) { return kBxReflection | (tr.EffectivelySmooth() ? kBxSpecular : kBxGlossy); }
PHD ConductorTerms RetroSample(const TrowbridgeReitz &tr, V3 wo, float u0, float u1) {
    if (!tr.EffectivelySmooth()) return ConductorSample(tr, wo, u0, u1);
    ConductorTerms c{true, true, wo, 1, 0, 0, AbsCosTheta(wo), 0, AbsCosTheta(wo)};
    return c;
}
// f's wavelength-independent terms; ok = false: f = 0
struct RetroTerms {
    bool ok;
    float w;                   // 1 - (R_i - R_o)
    float Dr, Dm, G, denom;    // D(wo), D(wm), G(wo, wi), 4 cos_i cos_o
    float cosRetro, cosM;      // FrComplex arguments |wi . wo|, |wo . wm|
};
PHD RetroTerms RetroEval(const TrowbridgeReitz &tr, V3 wo, V3 wi) {
    RetroTerms t{false, 0, 0, 0, 0, 0, 0, 0};
    if (!SameHemisphere(wo, wi) || tr.EffectivelySmooth()) return t;
    const float cosTheta_o = AbsCosTheta(wo), cosTheta_i = AbsCosTheta(wi);
    if (cosTheta_i == 0 || cosTheta_o == 0) return t;
    V3 wm = wo + wi;
    const V3 wmRetro = wo;
    if (LengthSquared(wm) == 0) return t;
    wm = Normalize(wm);
    const float R_o = FrDielectric(Dot(wo, wm), 1.59f), R_i = FrDielectric(Dot(wi, wmRetro), 1.59f);
    t = RetroTerms{true, 1 - (R_i - R_o), tr.D(wmRetro), tr.D(wm), tr.G(wo, wi), 4 * cosTheta_i * cosTheta_o,
                   AbsDot(wi, wmRetro), AbsDot(wo, wm)};
    return t;
}
// one wavelength of f: w * (D(wo) F_retro G / denom) + w * (D(wm) F G / denom), pbrt's order
PHD float RetroF(const RetroTerms &t, float eta, float k) {
    const float Fr = FrComplex(t.cosRetro, eta, k), F = FrComplex(t.cosM, eta, k);
    const float retro = t.Dr * Fr * t.G / t.denom;
    return t.w * retro + t.w * (t.Dm * F * t.G / t.denom);
}
// PDF (bxdfs.h:182-201): the conductor's microfacet reflection density
PHD float RetroPDF(const TrowbridgeReitz &tr, V3 wo, V3 wi) {
    if (!SameHemisphere(wo, wi) || tr.EffectivelySmooth()) return 0;
    V3 wh = wo + wi;
    if (LengthSquared(wh) == 0) return 0;
    wh = FaceForward(Normalize(wh), V3(0, 0, 1));
    return tr.PDF(wo, wh) / (4 * AbsDot(wo, wh));
}

// ---------------------------------------------------------------- ZSobol sampler
// ZSobolSampler (samplers.h:225-370): Morton-ordered pixel samples, base-4 digit
// permutations per dimension, Sobol' dimensions 0/1 with the chosen scrambler.
PHD uint64_t LeftShift2(uint64_t x) {  // util/math.h:83-91
    x &= 0xffffffff;
    x = (x ^ (x << 16)) & 0x0000ffff0000ffffull;
    x = (x ^ (x << 8)) & 0x00ff00ff00ff00ffull;
    x = (x ^ (x << 4)) & 0x0f0f0f0f0f0f0f0full;
    x = (x ^ (x << 2)) & 0x3333333333333333ull;
    x = (x ^ (x << 1)) & 0x5555555555555555ull;
    return x;
}
PHD uint64_t EncodeMorton2(uint32_t x, uint32_t y) { return (LeftShift2(y) << 1) | LeftShift2(x); }
PHD uint64_t MixBits(uint64_t v) {  // util/hash.h:70-77
    v ^= (v >> 31);
    v *= 0x7fb5d329728ea185ull;
    v ^= (v >> 27);
    v *= 0x81dadef4bc2dd44dull;
    v ^= (v >> 33);
    return v;
}
// MurmurHash64A over one 8-byte block with seed 0: pbrt's Hash(int a, int b) (util/hash.h:100-106)
PHD uint64_t HashInt2(int32_t a, int32_t b) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = 0 ^ (8ull * m);
    uint64_t k = (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32);  // little-endian packing
    k *= m;
    k ^= k >> r;
    k *= m;
    h ^= k;
    h *= m;
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}
PHD uint32_t ReverseBits32(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_bitreverse32(v);
#else
    v = (v << 16) | (v >> 16);
    v = ((v & 0x00ff00ff) << 8) | ((v & 0xff00ff00) >> 8);
    v = ((v & 0x0f0f0f0f) << 4) | ((v & 0xf0f0f0f0) >> 4);
    v = ((v & 0x33333333) << 2) | ((v & 0xcccccccc) >> 2);
    v = ((v & 0x55555555) << 1) | ((v & 0xaaaaaaaa) >> 1);
    return v;
#endif
}
// Sobol' generator matrices of dimensions 0 and 1 (the only ones ZSobol reads), 52 rows of
// 32 bits each as in util/sobolmatrices: dimension 0 is the van der Corput matrix; dimension 1
// follows from its primitive polynomial x + 1, V_k = V_{k-1} ^ (V_{k-1} >> 1) on 52-bit rows,
// keeping the top 32 bits.
constexpr int kSobolMatrixSize = 52;
PHD uint32_t SobolMatrix1Row(int k) {
    uint64_t v = 1ull << 51;
    for (int i = 0; i < k; ++i) v ^= v >> 1;
    return (uint32_t)(v >> 20);
}
enum class Randomize : int { None = 0, PermuteDigits = 1, FastOwen = 2, Owen = 3 };
PHD uint32_t FastOwenScramble(uint32_t v, uint32_t seed) {  // lowdiscrepancy.h:221-237
    v = ReverseBits32(v);
    v ^= v * 0x3d20adea;
    v += seed;
    v *= (seed >> 16) | 1;
    v ^= v * 0x05526c56;
    v ^= v * 0x53a22864;
    return ReverseBits32(v);
}
PHD uint32_t OwenScramble(uint32_t v, uint32_t seed) {  // lowdiscrepancy.h:240-258
    if (seed & 1) v ^= 1u << 31;
    for (int b = 1; b < 32; ++b) {
        uint32_t mask = (~0u) << (32 - b);
        if ((uint32_t)MixBits((v & mask) ^ seed) & (1u << b)) v ^= 1u << (31 - b);
    }
    return v;
}
// SobolSample (lowdiscrepancy.h:168-180) for dimension 0 or 1; matrix1 = the 52 rows above
PHD float SobolSampleDim01(uint64_t a, int dim, Randomize rz, uint32_t seed, const uint32_t *matrix1) {
    (void)matrix1;
    uint32_t v = 0;
    if (dim == 0) {
        v = ReverseBits32((uint32_t)a);  // rows >= 32 of dimension 0 are zero
    } else {
        // row i of the dimension-1 matrix generated on the fly (SobolMatrix1Row: the top 32
        // bits of the 52-bit recurrence follow the same recurrence in 32 bits), no table loads
        uint32_t col = 1u << 31;
        for (int i = 0; a != 0 && i < kSobolMatrixSize; a >>= 1, ++i, col ^= col >> 1)
            if (a & 1) v ^= col;
    }
    if (rz == Randomize::PermuteDigits) v ^= seed;
    else if (rz == Randomize::FastOwen) v = FastOwenScramble(v, seed);
    else if (rz == Randomize::Owen) v = OwenScramble(v, seed);
    return std::fmin(v * 0x1p-32f, kOneMinusEpsilon);
}
struct ZSobolParams {
    int log2SamplesPerPixel, nBase4Digits, seed;
    Randomize randomize;
};
// The 24 four-way digit permutations of ZSobolSampler (pbrt's order, host/build.cpp
// kZSobolPermutations) packed 2 bits per entry: perm p, digit d at bit (p & 7) * 8 + 2 d of
// word p >> 3 -- a register lookup instead of a table load per digit.
PHD int ZSobolPermute(int p, int d) {
    const uint64_t w = p < 8 ? 0xb1e19c6c78d8b4e4ull : (p < 16 ? 0x72d236c68d2d39c9ull : 0x93634b1b87271e4eull);
    return (int)((w >> ((p & 7) * 8 + d * 2)) & 3);
}
// (h >> 24) % 24 of a 64-bit hash in 32-bit arithmetic: x = hi 2^32 + lo with hi < 2^8,
// 2^32 = 16 (mod 24)
PHD int Mod24Of40(uint64_t h) {
    const uint32_t lo = (uint32_t)(h >> 24), hi = (uint32_t)(h >> 56);
    return (int)((hi * 16u + lo % 24u) % 24u);
}
// samplers.h:301-356 GetSampleIndex; perms = the 24 four-way permutations in pbrt's order
// (evaluated from the packed ZSobolPermute table; the argument is kept for the callers)
PHD uint64_t ZSobolSampleIndex(const ZSobolParams &z, uint64_t mortonIndex, int dimension,
                               const uint8_t (*perms)[4]) {
    (void)perms;
    uint64_t sampleIndex = 0;
    const bool pow2Samples = z.log2SamplesPerPixel & 1;
    const int lastDigit = pow2Samples ? 1 : 0;
    const uint64_t dimHash = (uint64_t)(0x55555555u * (uint32_t)dimension);
    for (int i = z.nBase4Digits - 1; i >= lastDigit; --i) {
        int digitShift = 2 * i - (pow2Samples ? 1 : 0);
        int digit = (int)((mortonIndex >> digitShift) & 3);
        uint64_t higherDigits = mortonIndex >> (digitShift + 2);
        int p = Mod24Of40(MixBits(higherDigits ^ dimHash));
        digit = ZSobolPermute(p, digit);
        sampleIndex |= uint64_t(digit) << digitShift;
    }
    if (pow2Samples) {
        int digit = (int)(mortonIndex & 1);
        sampleIndex |= digit ^ (MixBits((mortonIndex >> 1) ^ (uint64_t)(0x55555555u * (uint32_t)dimension)) & 1);
    }
    return sampleIndex;
}
// Get1D at state dimension `dimension` (samplers.h:257-271): index from the current dimension,
// hash from the incremented one
PHD float ZSobolGet1D(const ZSobolParams &z, uint64_t morton, int dimension, const uint8_t (*perms)[4],
                      const uint32_t *matrix1) {
    uint64_t sampleIndex = ZSobolSampleIndex(z, morton, dimension, perms);
    uint32_t sampleHash = (uint32_t)HashInt2(dimension + 1, z.seed);
    return SobolSampleDim01(sampleIndex, 0, z.randomize, sampleHash, matrix1);
}
// Get2D at state dimension `dimension` (samplers.h:273-292)
PHD void ZSobolGet2D(const ZSobolParams &z, uint64_t morton, int dimension, const uint8_t (*perms)[4],
                     const uint32_t *matrix1, float *u0, float *u1) {
    uint64_t sampleIndex = ZSobolSampleIndex(z, morton, dimension, perms);
    uint64_t bits = HashInt2(dimension + 2, z.seed);
    *u0 = SobolSampleDim01(sampleIndex, 0, z.randomize, (uint32_t)bits, matrix1);
    *u1 = SobolSampleDim01(sampleIndex, 1, z.randomize, (uint32_t)(bits >> 32), matrix1);
}
// StartPixelSample (samplers.h:252-255)
PHD uint64_t ZSobolMortonIndex(const ZSobolParams &z, int px, int py, int sampleIndex) {
    return (EncodeMorton2((uint32_t)px, (uint32_t)py) << z.log2SamplesPerPixel) | (uint64_t)(uint32_t)sampleIndex;
}

// ---------------------------------------------------------------- light BVH importance
// lightsamplers.h:130 CompactLightBounds::Importance on host-decoded bounds.
struct LightNodeBounds {
    V3 pMin, pMax;  // decoded quantised bounds
    V3 w;           // decoded octahedral direction
    float phi, cosTheta_o, cosTheta_e;
    int twoSided;
};
// util/vecmath.h:1817 BoundSubtendedDirections -> cosTheta
PHD float BoundSubtendedCos(V3 pMin, V3 pMax, V3 p) {
    V3 pCenter = (pMin + pMax) / 2;
    bool inside = pCenter.x >= pMin.x && pCenter.x <= pMax.x && pCenter.y >= pMin.y &&
                  pCenter.y <= pMax.y && pCenter.z >= pMin.z && pCenter.z <= pMax.z;
    float radius = inside ? Distance(pCenter, pMax) : 0;
    if (DistanceSquared(p, pCenter) < Sqr(radius)) return -1;
    float sin2ThetaMax = Sqr(radius) / DistanceSquared(pCenter, p);
    return SafeSqrt(1 - sin2ThetaMax);
}
PHD float CosSubClamped(float sinA, float cosA, float sinB, float cosB) {
    if (cosA > cosB) return 1;
    return cosA * cosB + sinA * sinB;
}
PHD float SinSubClamped(float sinA, float cosA, float sinB, float cosB) {
    if (cosA > cosB) return 0;
    return sinA * cosB - cosA * sinB;
}
PHD_LI float LightImportanceInl(LightNodeBounds lb, V3 p, V3 n) {
    V3 pc = (lb.pMin + lb.pMax) / 2;
    float d2 = DistanceSquared(p, pc);
    d2 = std::fmax(d2, Length(lb.pMax - lb.pMin) / 2);
    V3 wi = Normalize(p - pc);
    float cosTheta_w = Dot(lb.w, wi);
    if (lb.twoSided) cosTheta_w = std::fabs(cosTheta_w);
    float sinTheta_w = SafeSqrt(1 - Sqr(cosTheta_w));
    float cosTheta_b = BoundSubtendedCos(lb.pMin, lb.pMax, p);
    float sinTheta_b = SafeSqrt(1 - Sqr(cosTheta_b));
    float sinTheta_o = SafeSqrt(1 - Sqr(lb.cosTheta_o));
    float cosTheta_x = CosSubClamped(sinTheta_w, cosTheta_w, sinTheta_o, lb.cosTheta_o);
    float sinTheta_x = SinSubClamped(sinTheta_w, cosTheta_w, sinTheta_o, lb.cosTheta_o);
    float cosThetap = CosSubClamped(sinTheta_x, cosTheta_x, sinTheta_b, cosTheta_b);
    if (cosThetap <= lb.cosTheta_e) return 0;
    float importance = lb.phi * cosThetap / d2;
    if (n != V3(0, 0, 0)) {
        float cosTheta_i = AbsDotN(n, wi);
        float sinTheta_i = SafeSqrt(1 - Sqr(cosTheta_i));
        float cosThetap_i = CosSubClamped(sinTheta_i, cosTheta_i, sinTheta_b, cosTheta_b);
        importance *= cosThetap_i;
    }
    importance = std::fmax(importance, 0.f);
    return importance;
}
PHD_NOINLINE float LightImportance(LightNodeBounds lb, V3 p, V3 n) { return LightImportanceInl(lb, p, n); }

// ---------------------------------------------------------------- participating media
// pbrt's Hash(args...) over whole 4-byte words (util/hash.h:91-106): MurmurHash64A (seed 0) of
// the packed arguments, e.g. Hash(ray.o, tMax) = 16 bytes, Hash(ray.d) = 12 bytes.
PHD uint64_t HashWords(const uint32_t *w, int nWords) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = (uint64_t)(4 * nWords) * m;
    for (int i = 0; i + 1 < nWords; i += 2) {
        uint64_t k = (uint64_t)w[i] | ((uint64_t)w[i + 1] << 32);  // little-endian 8-byte block
        k *= m;
        k ^= k >> r;
        k *= m;
        h ^= k;
        h *= m;
    }
    if (nWords & 1) {  // 4-byte tail: bytes 3..0 xor-ed in, then one multiply
        h ^= (uint64_t)w[nWords - 1];
        h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}
PHD uint64_t HashV3(V3 v) {
    const uint32_t w[3] = {FloatToBits(v.x), FloatToBits(v.y), FloatToBits(v.z)};
    return HashWords(w, 3);
}
PHD uint64_t HashV3F(V3 v, float f) {
    const uint32_t w[4] = {FloatToBits(v.x), FloatToBits(v.y), FloatToBits(v.z), FloatToBits(f)};
    return HashWords(w, 4);
}

// PCG32 (util/rng.h:30-140): RNG(seqIndex, offset) = SetSequence(seqIndex, offset)
struct PCG32 {
    uint64_t state, inc;
    PHD PCG32(uint64_t seqIndex, uint64_t offset) {
        state = 0u;
        inc = (seqIndex << 1u) | 1u;
        NextU32();
        state += offset;
        NextU32();
    }
    PHD uint32_t NextU32() {
        const uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        const uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    PHD float Uniform() { return std::fmin(kOneMinusEpsilon, (float)NextU32() * 0x1p-32f); }
    PHD PCG32() : state(0x853c49e6748fea9bULL), inc(0xda3e39cb94b95bdbULL) {}  // PCG32_DEFAULT_STATE / STREAM
    // SetSequence(sequenceIndex) = SetSequence(sequenceIndex, MixBits(sequenceIndex)) (rng.h:43-45, 119-125)
    PHD void SetSequence(uint64_t seqIndex);
    // Advance (rng.h:137-150): the state after idelta draws, by repeated squaring of the LCG step
    PHD void Advance(uint64_t delta) {
        uint64_t curMult = 0x5851f42d4c957f2dULL, curPlus = inc, accMult = 1u, accPlus = 0u;
        while (delta > 0) {
            if (delta & 1) {
                accMult *= curMult;
                accPlus = accPlus * curMult + curPlus;
            }
            curPlus = (curMult + 1) * curPlus;
            curMult *= curMult;
            delta /= 2;
        }
        state = accMult * state + accPlus;
    }
};
PHD void PCG32::SetSequence(uint64_t seqIndex) {
    state = 0u;
    inc = (seqIndex << 1u) | 1u;
    NextU32();
    state += MixBits(seqIndex);
    NextU32();
}

// PermutationElement (util/math.h:728-756): element i of the seeded permutation of [0, l)
PHD int PermutationElement(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1;
    w |= w >> 2;
    w |= w >> 4;
    w |= w >> 8;
    w |= w >> 16;
    do {
        i ^= p;
        i *= 0xe170893d;
        i ^= p >> 16;
        i ^= (i & w) >> 4;
        i ^= p >> 8;
        i *= 0x0929eb3f;
        i ^= p >> 23;
        i ^= (i & w) >> 1;
        i *= 1 | p >> 27;
        i *= 0x6935fa69;
        i ^= (i & w) >> 11;
        i *= 0x74dcb303;
        i ^= (i & w) >> 2;
        i *= 0x9e501cc3;
        i ^= (i & w) >> 2;
        i *= 0xc860a3df;
        i &= w;
        i ^= i >> 5;
    } while (i >= l);
    return (int)((i + p) % l);
}

// ---------------------------------------------------------------- the other samplers
// IndependentSampler, StratifiedSampler, SobolSampler, PaddedSobolSampler (samplers.h:144-224,
// 442-633), behind one state object so every kernel calls them the same way.  Sobol' rows come
// from util/sobolmatrices.cpp's tables (data/sobol_tables.bin, uploaded when the scene uses the
// SobolSampler): SobolMatrices32 [1024][52], VdCSobolMatrices and VdCSobolMatricesInv [25][52].
constexpr int kSamplerHalton = 0, kSamplerZSobol = 1, kSamplerIndependent = 2, kSamplerStratified = 3,
              kSamplerSobol = 4, kSamplerPaddedSobol = 5;
constexpr int kNSobolDimensions = 1024, kNVdCSobol = 25;
struct SamplerDesc {
    int type, spp, seed;
    int xSamples, ySamples, jitter;  // StratifiedSampler
    Randomize randomize;             // SobolSampler / PaddedSobolSampler
    int log2Scale;                   // SobolSampler: Log2Int(RoundUpPow2(max(xres, yres)))
    const uint32_t *sobol32;         // [1024 * 52]
    const uint64_t *vdc, *vdcInv;    // [25][52]
};
// Hash(p, seed) (12 bytes) and Hash(p, dimension, seed) (16 bytes), util/hash.h:91-106
PHD uint64_t HashPixelSeed(int px, int py, int seed) {
    const uint32_t w[3] = {(uint32_t)px, (uint32_t)py, (uint32_t)seed};
    return HashWords(w, 3);
}
PHD uint64_t HashPixelDimSeed(int px, int py, int dim, int seed) {
    const uint32_t w[4] = {(uint32_t)px, (uint32_t)py, (uint32_t)dim, (uint32_t)seed};
    return HashWords(w, 4);
}
// SobolSample (lowdiscrepancy.h:167-180) of any dimension, then the scrambler
PHD float SobolSampleDim(uint64_t a, int dim, Randomize rz, uint32_t seed, const uint32_t *m32) {
    uint32_t v = 0;
    for (int i = dim * kSobolMatrixSize; a != 0; a >>= 1, i++)
        if (a & 1) v ^= m32[i];
    if (rz == Randomize::PermuteDigits) v ^= seed;
    else if (rz == Randomize::FastOwen) v = FastOwenScramble(v, seed);
    else if (rz == Randomize::Owen) v = OwenScramble(v, seed);
    return std::fmin(v * 0x1p-32f, kOneMinusEpsilon);
}
// SobolIntervalToIndex (lowdiscrepancy.h:266-287)
PHD uint64_t SobolIntervalToIndex(const SamplerDesc &d, uint32_t m, uint64_t frame, int px, int py) {
    if (m == 0) return frame;
    const uint32_t m2 = m << 1;
    uint64_t index = uint64_t(frame) << m2;
    uint64_t delta = 0;
    for (int c = 0; frame; frame >>= 1, ++c)
        if (frame & 1) delta ^= d.vdc[(m - 1) * kSobolMatrixSize + c];
    uint64_t b = (((uint64_t)((uint32_t)px) << m) | ((uint32_t)py)) ^ delta;
    for (int c = 0; b; b >>= 1, ++c)
        if (b & 1) index ^= d.vdcInv[(m - 1) * kSobolMatrixSize + c];
    return index;
}
struct GenericSampler {
    int px, py, sampleIndex, dimension;
    uint64_t sobolIndex;
    PCG32 rng;
    // StartPixelSample
    PHD void Start(const SamplerDesc &d, int x, int y, int index, int dim) {
        px = x, py = y, sampleIndex = index, dimension = dim, sobolIndex = 0;
        if (d.type == kSamplerIndependent || d.type == kSamplerStratified) {
            rng.SetSequence(HashPixelSeed(x, y, d.seed));
            rng.Advance((uint64_t)index * 65536ull + (uint64_t)dim);
        } else if (d.type == kSamplerSobol) {
            dimension = dim < 2 ? 2 : dim;
            sobolIndex = SobolIntervalToIndex(d, (uint32_t)d.log2Scale, (uint64_t)index, x, y);
        }
    }
    // SobolSampler::SampleDimension
    PHD float SobolDim(const SamplerDesc &d, int dim) const {
        if (d.randomize == Randomize::None) return SobolSampleDim(sobolIndex, dim, Randomize::None, 0, d.sobol32);
        return SobolSampleDim(sobolIndex, dim, d.randomize, (uint32_t)HashInt2(dim, d.seed), d.sobol32);
    }
    PHD float Get1D(const SamplerDesc &d) {
        if (d.type == kSamplerIndependent) return rng.Uniform();
        if (d.type == kSamplerStratified) {
            const uint64_t hash = HashPixelDimSeed(px, py, dimension, d.seed);
            const int n = d.xSamples * d.ySamples;
            const int stratum = PermutationElement((uint32_t)sampleIndex, (uint32_t)n, (uint32_t)hash);
            ++dimension;
            const float delta = d.jitter ? rng.Uniform() : 0.5f;
            return (stratum + delta) / n;
        }
        if (d.type == kSamplerSobol) {
            if (dimension >= kNSobolDimensions) dimension = 2;
            return SobolDim(d, dimension++);
        }
        // PaddedSobolSampler
        const uint64_t hash = HashPixelDimSeed(px, py, dimension, d.seed);
        const int index = PermutationElement((uint32_t)sampleIndex, (uint32_t)d.spp, (uint32_t)hash);
        ++dimension;
        return SobolSampleDim01((uint64_t)(uint32_t)index, 0, d.randomize, (uint32_t)(hash >> 32), nullptr);
    }
    PHD void Get2D(const SamplerDesc &d, float *u0, float *u1) {
        if (d.type == kSamplerIndependent) {
            *u0 = rng.Uniform();
            *u1 = rng.Uniform();
            return;
        }
        if (d.type == kSamplerStratified) {
            const uint64_t hash = HashPixelDimSeed(px, py, dimension, d.seed);
            const int stratum =
                PermutationElement((uint32_t)sampleIndex, (uint32_t)(d.xSamples * d.ySamples), (uint32_t)hash);
            dimension += 2;
            const int x = stratum % d.xSamples, y = stratum / d.xSamples;
            const float dx = d.jitter ? rng.Uniform() : 0.5f;
            const float dy = d.jitter ? rng.Uniform() : 0.5f;
            *u0 = (x + dx) / d.xSamples;
            *u1 = (y + dy) / d.ySamples;
            return;
        }
        if (d.type == kSamplerSobol) {
            if (dimension + 1 >= kNSobolDimensions) dimension = 2;
            *u0 = SobolDim(d, dimension);
            *u1 = SobolDim(d, dimension + 1);
            dimension += 2;
            return;
        }
        const uint64_t hash = HashPixelDimSeed(px, py, dimension, d.seed);
        const int index = PermutationElement((uint32_t)sampleIndex, (uint32_t)d.spp, (uint32_t)hash);
        dimension += 2;
        *u0 = SobolSampleDim01((uint64_t)(uint32_t)index, 0, d.randomize, (uint32_t)hash, nullptr);
        *u1 = SobolSampleDim01((uint64_t)(uint32_t)index, 1, d.randomize, (uint32_t)(hash >> 32), nullptr);
    }
    PHD void GetPixel2D(const SamplerDesc &d, float *u0, float *u1) {
        if (d.type != kSamplerSobol) {
            Get2D(d, u0, u1);
            return;
        }
        // SobolSampler::GetPixel2D: dimensions 0 and 1 of the pixel's interval, unscrambled,
        // remapped into the pixel
        float u[2] = {SobolSampleDim(sobolIndex, 0, Randomize::None, 0, d.sobol32),
                      SobolSampleDim(sobolIndex, 1, Randomize::None, 0, d.sobol32)};
        const int scale = 1 << d.log2Scale, p[2] = {px, py};
        for (int k = 0; k < 2; ++k) u[k] = Clampf(u[k] * scale - p[k], 0, kOneMinusEpsilon);
        *u0 = u[0];
        *u1 = u[1];
    }
};

// FastExp (util/math.h:450-475), the CPU form (2^x by a cubic on the fraction, exponent bits
// patched in).  |xp| > 256 (and NaN) short-circuit to the values the exponent test gives.
PHD float FastExp(float x) {
    const float xp = x * 1.442695041f;
    if (!(xp > -256.f)) return 0.f;
    if (xp > 256.f) return kInfinity;
    const float fxp = std::floor(xp), f = xp - fxp;
    const int i = (int)fxp;
    const float twoToF = fmaf(f, fmaf(f, fmaf(f, 0.0781455737f, 0.226173572f), 0.695556856f), 1.f);
    const int exponent = (int)((FloatToBits(twoToF) >> 23) & 0xff) - 127 + i;
    if (exponent < -126) return 0.f;
    if (exponent > 127) return kInfinity;
    uint32_t bits = FloatToBits(twoToF);
    bits &= 0b10000000011111111111111111111111u;
    bits |= (uint32_t)(exponent + 127) << 23;
    return BitsToFloat(bits);
}

// Blackbody (util/spectrum.h:69-80): Planck's law with the CPU FastExp, in pbrt's float
// operation order (Pow<5> as (l l)(l l) l); BlackbodySpectrum (util/spectrum.h:530-560) divides
// by its value at Wien's peak, computed once per temperature
PHD float Blackbody(float lambda, float T) {
    if (T <= 0) return 0;
    const float c = 299792458.f, h = 6.62606957e-34f, kb = 1.3806488e-23f;
    const float l = lambda * 1e-9f;
    const float l2 = l * l;
    const float l5 = l2 * l2 * l;
    return (2 * h * c * c) / (l5 * (FastExp((h * c) / (l * kb * T)) - 1));
}
PHD float BlackbodyNorm(float T) { return 1 / Blackbody(2.8977721e-3f / T * 1e9f, T); }

// SampleExponential (util/sampling.h): -log(1 - u) / a
PHD float SampleExponential(float u, float a) { return -Logf(1 - u) / a; }

// HenyeyGreenstein (util/scattering.h:49-58) and SampleHenyeyGreenstein (util/sampling.cpp:347-373)
constexpr float kInv4Pi = 0.07957747154594766788f;
PHD float HenyeyGreenstein(float cosTheta, float g) {
    g = Clampf(g, -.99f, .99f);
    const float denom = 1 + Sqr(g) + 2 * g * cosTheta;
    return kInv4Pi * (1 - Sqr(g)) / (denom * SafeSqrt(denom));
}
PHD V3 SampleHenyeyGreenstein(V3 wo, float g, float u0, float u1, float *pdf) {
    g = Clampf(g, -.99f, .99f);
    float cosTheta;
    if (std::fabs(g) < 1e-3f) cosTheta = 1 - 2 * u0;
    else cosTheta = -1 / (2 * g) * (1 + Sqr(g) - Sqr((1 - Sqr(g)) / (1 + g - 2 * g * u0)));
    const float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    const float phi = 2 * kPi * u1;
    V3 x, y;
    CoordinateSystem(wo, &x, &y);  // Frame::FromZ(wo)
    const float st = Clampf(sinTheta, -1, 1);
    const V3 l(st * Cosf(phi), st * Sinf(phi), Clampf(cosTheta, -1, 1));  // SphericalDirection
    *pdf = HenyeyGreenstein(cosTheta, g);
    return x * l.x + y * l.y + wo * l.z;
}

// SampleDiscrete (util/sampling.h:79-110) over three weights; bounded to the last index
PHD int SampleDiscrete3(float w0, float w1, float w2, float u) {
    const float sum = (w0 + w1) + w2;
    float up = u * sum;
    if (up == sum) up = NextFloatDown(up);
    float acc = 0;
    if (acc + w0 > up) return 0;
    acc += w0;
    if (acc + w1 > up) return 1;
    return 2;
}

// ---------------------------------------------------------------- pixel filters
// filters.h: Box / Gaussian / Mitchell / LanczosSinc / Triangle.  The tabulated filters sample
// through FilterSampler (filters.cpp:133-147): f tabulated at 32 samples per unit radius,
// PiecewiseConstant2D over |f| (util/sampling.h:603-790), weight = f[pi] / pdf.
enum FilterType : int { kFilterBox = 0, kFilterGaussian = 1, kFilterMitchell = 2, kFilterSinc = 3, kFilterTriangle = 4 };
struct FilterParams {
    int type;
    float rx, ry;
    float a, b;  // gaussian sigma; mitchell B, C; sinc tau
};
// util/math.h:478 Gaussian (with the CPU FastExp)
PHD float GaussianF(float x, float mu, float sigma) {
    return 1 / std::sqrt(2 * kPi * sigma * sigma) * FastExp(-Sqr(x - mu) / (2 * sigma * sigma));
}
PHD float Mitchell1D(float x, float b, float c) {  // filters.h:150-162
    x = std::fabs(x);
    if (x <= 1)
        return ((12 - 9 * b - 6 * c) * x * x * x + (-18 + 12 * b + 6 * c) * x * x + (6 - 2 * b)) * (1.f / 6.f);
    else if (x <= 2)
        return ((-b - 6 * c) * x * x * x + (6 * b + 30 * c) * x * x + (-12 * b - 48 * c) * x + (8 * b + 24 * c)) *
               (1.f / 6.f);
    return 0;
}
PHD float SinXOverX(float x) {  // util/math.h:340
    if (1 - x * x == 1) return 1;
    return Sinf(x) / x;
}
PHD float WindowedSinc(float x, float radius, float tau) {  // util/math.h:221
    if (std::fabs(x) > radius) return 0;
    return SinXOverX(kPi * x) * SinXOverX(kPi * (x / tau));
}
// Filter::Evaluate (filters.h)
PHD float FilterEvaluate(const FilterParams &f, float px, float py) {
    switch (f.type) {
    case kFilterGaussian:
        return std::fmax(0.f, GaussianF(px, 0, f.a) - GaussianF(f.rx, 0, f.a)) *
               std::fmax(0.f, GaussianF(py, 0, f.a) - GaussianF(f.ry, 0, f.a));
    case kFilterMitchell:
        return Mitchell1D(2 * px / f.rx, f.a, f.b) * Mitchell1D(2 * py / f.ry, f.a, f.b);
    case kFilterSinc:
        return WindowedSinc(px, f.rx, f.a) * WindowedSinc(py, f.ry, f.a);
    case kFilterTriangle:
        return std::fmax(0.f, f.rx - std::fabs(px)) * std::fmax(0.f, f.ry - std::fabs(py));
    default:
        return (std::fabs(px) <= f.rx && std::fabs(py) <= f.ry) ? 1.f : 0.f;
    }
}
// FindInterval (util/math.h) over a CDF of sz entries: largest i <= sz - 2 with cdf[i] <= u
template <typename P>
PHD int FindIntervalCdf(const P *cdf, int sz, float u) {
    int size = sz - 2, first = 1;
    while (size > 0) {
        const int half = size >> 1, middle = first + half;
        const bool pr = cdf[middle] <= u;
        first = pr ? middle + 1 : first;
        size = pr ? size - (half + 1) : half;
    }
    const int i = first - 1;
    return i < 0 ? 0 : (i > sz - 2 ? sz - 2 : i);
}
// FilterSampler tables of a tabulated filter, one float array (filter.cpp BuildFilterTable):
// [nu*nv] f, [nu*nv] |f|, [nv*(nu+1)] conditional CDFs, [nv] conditional integrals,
// [nv+1] marginal CDF, [1] marginal integral
struct FilterTableView {
    int nu, nv;
    const float *t;
    PHD const float *F() const { return t; }
    PHD const float *Func() const { return t + nu * nv; }
    PHD const float *CondCdf() const { return t + 2 * nu * nv; }
    PHD const float *CondInt() const { return t + 2 * nu * nv + nv * (nu + 1); }
    PHD const float *MargCdf() const { return CondInt() + nv; }
    PHD float MargInt() const { return MargCdf()[nv + 1]; }
    static PHD int Size(int nu, int nv) { return 2 * nu * nv + nv * (nu + 1) + nv + (nv + 1) + 1; }
};
// PiecewiseConstant1D::Sample (util/sampling.h:657-675)
PHD float SamplePC1D(const float *func, const float *cdf, int n, float funcInt, float mn, float mx, float u,
                     float *pdf, int *offset) {
    const int o = FindIntervalCdf(cdf, n + 1, u);
    *offset = o;
    float du = u - cdf[o];
    if (cdf[o + 1] - cdf[o] > 0) du /= cdf[o + 1] - cdf[o];
    *pdf = (funcInt > 0) ? func[o] / funcInt : 0;
    return Lerpf((o + du) / n, mn, mx);
}
// ---------------------------------------------------------------- image infinite lights
// EqualAreaSquareToSphere / EqualAreaSphereToSquare (util/math.cpp:292-361, Clarberg's
// equal-area octahedral mapping); EvaluatePolynomial is FMA-based
PHD V3 EqualAreaSquareToSphere(float px, float py) {
    const float u = 2 * px - 1, v = 2 * py - 1;
    const float up = std::fabs(u), vp = std::fabs(v);
    const float signedDistance = 1 - (up + vp);
    const float d = std::fabs(signedDistance);
    const float r = 1 - d;
    const float phi = (r == 0 ? 1 : (vp - up) / r + 1) * kPi / 4;
    const float z = std::copysign(1 - Sqr(r), signedDistance);
    float sp, cp;
    SinCosf(phi, &sp, &cp);
    const float cosPhi = std::copysign(cp, u);
    const float sinPhi = std::copysign(sp, v);
    return V3(cosPhi * r * SafeSqrt(2 - Sqr(r)), sinPhi * r * SafeSqrt(2 - Sqr(r)), z);
}
PHD void EqualAreaSphereToSquare(V3 d, float *uo, float *vo) {
    const float x = std::fabs(d.x), y = std::fabs(d.y), z = std::fabs(d.z);
    const float r = SafeSqrt(1 - z);
    const float a = std::fmax(x, y);
    float b = std::fmin(x, y);
    b = a == 0 ? 0 : b / a;
    const float t1 = 0.406758566246788489601959989e-5f, t2 = 0.636226545274016134946890922156f,
                t3 = 0.61572017898280213493197203466e-2f, t4 = -0.247333733281268944196501420480f,
                t5 = 0.881770664775316294736387951347e-1f, t6 = 0.419038818029165735901852432784e-1f,
                t7 = -0.251390972343483509333252996350e-1f;
    float phi = fmaf(b, fmaf(b, fmaf(b, fmaf(b, fmaf(b, fmaf(b, t7, t6), t5), t4), t3), t2), t1);
    if (x < y) phi = 1 - phi;
    float v = phi * r;
    float u = r - v;
    if (d.z < 0) {
        const float t = u;
        u = v;
        v = t;
        u = 1 - u;
        v = 1 - v;
    }
    u = std::copysign(u, d.x);
    v = std::copysign(v, d.y);
    *uo = 0.5f * (u + 1);
    *vo = 0.5f * (v + 1);
}
// One ImageInfiniteLight's device tables: per pixel the RGBIlluminantSpectrum of the clamped
// RGB as {c0, c1, c2, scale}, and the compensated PiecewiseConstant2D over [0,1]^2 in the
// FilterTableView layout.  m: renderFromLight, mi: its inverse (upper 3x3, row major).
struct alignas(16) EnvCoef {
    float c0, c1, c2, s;  // sigmoid polynomial coefficients and RGBIlluminantSpectrum::scale
};
struct DeviceEnvLight {
    float m[9], mi[9];
    int res, portal;  // portal != 0: a PortalImageInfiniteLight (coef: the rectified image's)
    const EnvCoef *coef;
    FilterTableView dist;  // ImageInfiniteLight's compensated distribution
    // PortalImageInfiniteLight: portalFrame's rows x, y, z (Frame::FromXY(p03, p01)), portal[0]
    // and portal[2] in render space, the windowed distribution's summed-area table (Float
    // values of its double sums, as SummedAreaTable::LookupInt returns them) and function
    float pf[9], pc0[3], pc2[3];
    const float *sat, *func;
};
PHD V3 MulM3(const float *m, V3 v) {
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
              m[6] * v.x + m[7] * v.y + m[8] * v.z);
}
// Image::LookupNearestChannel(uv, c, OctahedralSphere) (util/image.h:351-356, 96-125)
PHD EnvCoef EnvCoefAt(const DeviceEnvLight &E, float u, float v) {
    int x = (int)(u * E.res), y = (int)(v * E.res);
    const int n = E.res;
    if (x < 0) {
        x = -x;
        y = n - 1 - y;
    } else if (x >= n) {
        x = 2 * n - 1 - x;
        y = n - 1 - y;
    }
    if (y < 0) {
        x = n - 1 - x;
        y = -y;
    } else if (y >= n) {
        x = n - 1 - x;
        y = 2 * n - 1 - y;
    }
    if (n == 1) x = y = 0;
    return E.coef[(size_t)y * n + x];
}
// compensatedDistribution.Sample(u) (util/sampling.h:760-770): marginal in v from u1,
// conditional in u from u0; *pdf = mapPDF
PHD void EnvSampleUV(const DeviceEnvLight &E, float u0, float u1, float *uo, float *vo, float *pdf) {
    const FilterTableView &t = E.dist;
    float pdf1, pdf0;
    int iv, iu;
    *vo = SamplePC1D(t.CondInt(), t.MargCdf(), t.nv, t.MargInt(), 0.f, 1.f, u1, &pdf1, &iv);
    *uo = SamplePC1D(t.Func() + (size_t)iv * t.nu, t.CondCdf() + (size_t)iv * (t.nu + 1), t.nu, t.CondInt()[iv], 0.f,
                     1.f, u0, &pdf0, &iu);
    *pdf = pdf0 * pdf1;
}
// compensatedDistribution.PDF(uv) (util/sampling.h:773-779)
PHD float EnvPDF(const DeviceEnvLight &E, float u, float v) {
    const FilterTableView &t = E.dist;
    int iu = (int)(u * t.nu), iv = (int)(v * t.nv);
    iu = iu < 0 ? 0 : (iu > t.nu - 1 ? t.nu - 1 : iu);
    iv = iv < 0 ? 0 : (iv > t.nv - 1 ? t.nv - 1 : iv);
    return t.Func()[(size_t)iv * t.nu + iu] / t.MargInt();
}
// RGBIlluminantSpectrum::Sample at one wavelength times the light scale (lights.h:625-631):
// scale * ((c.w * rsp(lambda)) * illuminant(lambda))
PHD float EnvLe(const EnvCoef &c, float lightScale, float illum, float lambda) {
    return lightScale * ((c.s * SigmoidPolynomial(c.c0, c.c1, c.c2, lambda)) * illum);
}

// ---------------------------------------------------------------- portal image infinite lights
// PortalImageInfiniteLight (lights.h:644-744, lights.cpp:1140-1297): the environment map
// rectified over the portal frame's angles (alpha, beta) = (atan2(x, z), atan2(y, z)), sampled
// with a WindowedPiecewiseConstant2D (util/sampling.h:830-989) restricted to the portal's image
// bounds as seen from the reference point.
PHD bool PortalImageFromRender(const DeviceEnvLight &E, V3 wr, float *u, float *v, float *duv_dw) {
    const V3 w(Dot(wr, V3(E.pf[0], E.pf[1], E.pf[2])), Dot(wr, V3(E.pf[3], E.pf[4], E.pf[5])),
               Dot(wr, V3(E.pf[6], E.pf[7], E.pf[8])));
    if (w.z <= 0) return false;
    if (duv_dw) *duv_dw = Sqr(kPi) * (1 - Sqr(w.x)) * (1 - Sqr(w.y)) / w.z;
    const float alpha = ATan2f(w.x, w.z), beta = ATan2f(w.y, w.z);
    *u = Clampf((alpha + kPi / 2) / kPi, 0, 1);
    *v = Clampf((beta + kPi / 2) / kPi, 0, 1);
    return true;
}
PHD V3 PortalRenderFromImage(const float *pf, float u, float v, float *duv_dw) {
    const float alpha = -kPi / 2 + u * kPi, beta = -kPi / 2 + v * kPi;
    const float x = Tanf(alpha), y = Tanf(beta);
    const V3 w = Normalize(V3(x, y, 1));
    if (duv_dw) *duv_dw = Sqr(kPi) * (1 - Sqr(w.x)) * (1 - Sqr(w.y)) / w.z;
    return V3(pf[0], pf[1], pf[2]) * w.x + V3(pf[3], pf[4], pf[5]) * w.y + V3(pf[6], pf[7], pf[8]) * w.z;
}
// ImageBounds(p): the image points of portal[0] and portal[2] seen from p, as Bounds2f
// {pMin.x, pMin.y, pMax.x, pMax.y}
PHD bool PortalImageBounds(const DeviceEnvLight &E, V3 p, float b[4]) {
    float u0, v0, u1, v1;
    if (!PortalImageFromRender(E, Normalize(V3(E.pc0[0], E.pc0[1], E.pc0[2]) - p), &u0, &v0, nullptr)) return false;
    if (!PortalImageFromRender(E, Normalize(V3(E.pc2[0], E.pc2[1], E.pc2[2]) - p), &u1, &v1, nullptr)) return false;
    b[0] = u1 < u0 ? u1 : u0;
    b[1] = v1 < v0 ? v1 : v0;
    b[2] = u0 < u1 ? u1 : u0;
    b[3] = v0 < v1 ? v1 : v0;
    return true;
}
// SummedAreaTable::LookupInt / Lookup / Integral (util/sampling.h:851-888)
PHD float SatLookupInt(const DeviceEnvLight &E, int x, int y) {
    if (x == 0 || y == 0) return 0;
    x = x - 1 < E.res - 1 ? x - 1 : E.res - 1;
    y = y - 1 < E.res - 1 ? y - 1 : E.res - 1;
    return E.sat[(size_t)y * E.res + x];
}
PHD float SatLookup(const DeviceEnvLight &E, float x, float y) {
    x *= E.res;
    y *= E.res;
    const int x0 = (int)x, y0 = (int)y;
    const float v00 = SatLookupInt(E, x0, y0), v10 = SatLookupInt(E, x0 + 1, y0);
    const float v01 = SatLookupInt(E, x0, y0 + 1), v11 = SatLookupInt(E, x0 + 1, y0 + 1);
    const float dx = x - (float)(int)x, dy = y - (float)(int)y;
    return (1 - dx) * (1 - dy) * v00 + (1 - dx) * dy * v01 + dx * (1 - dy) * v10 + dx * dy * v11;
}
PHD float SatIntegral(const DeviceEnvLight &E, float x0, float y0, float x1, float y1) {
    const double s = (((double)SatLookup(E, x1, y1) - (double)SatLookup(E, x0, y1)) +
                      ((double)SatLookup(E, x0, y0) - (double)SatLookup(E, x1, y0)));
    const float r = (float)(s / (double)(E.res * E.res));
    return r < 0 ? 0.f : r;
}
// WindowedPiecewiseConstant2D::Eval
PHD float PortalFuncAt(const DeviceEnvLight &E, float u, float v) {
    int x = (int)(u * E.res), y = (int)(v * E.res);
    x = x < E.res - 1 ? x : E.res - 1;
    y = y < E.res - 1 ? y : E.res - 1;
    return E.func[(size_t)y * E.res + x];
}
// SampleBisection over the windowed marginal (Y false: x in [b0, b2] with y over [b1, b3]) or
// conditional (Y true: y with x over the column bounds cx0, cx1); the loop is capped (pbrt has no
// cap; it ends within ~log2(n) halvings)
template <bool Y>
PHD float PortalBisect(const DeviceEnvLight &E, const float b[4], float cx0, float cx1, float norm, float u, float mn,
                       float mx) {
    auto P = [&](float t) {
        return (Y ? SatIntegral(E, cx0, b[1], cx1, t) : SatIntegral(E, b[0], b[1], t, b[3])) / norm;
    };
    const int n = E.res;
    for (int it = 0; it < 128 && std::ceil(n * mx) - std::floor(n * mn) > 1; ++it) {
        const float mid = (mn + mx) / 2;
        if (P(mid) > u) mx = mid;
        else mn = mid;
    }
    const float t = (u - P(mn)) / (P(mx) - P(mn));
    return Clampf((1 - t) * mn + t * mx, mn, mx);
}
// WindowedPiecewiseConstant2D::Sample(u, b, &pdf); false for {}
PHD bool PortalWindowedSample(const DeviceEnvLight &E, float u0, float u1, const float b[4], float *px, float *py,
                              float *pdf) {
    const float bInt = SatIntegral(E, b[0], b[1], b[2], b[3]);
    if (bInt == 0) return false;
    const float x = PortalBisect<false>(E, b, 0, 0, bInt, u0, b[0], b[2]);
    const int nx = E.res;
    const float cx0 = std::floor(x * nx) / nx;
    float cx1 = std::ceil(x * nx) / nx;
    if (cx0 == cx1) cx1 += 1.f / nx;
    const float cInt = SatIntegral(E, cx0, b[1], cx1, b[3]);
    if (cInt == 0) return false;
    const float y = PortalBisect<true>(E, b, cx0, cx1, cInt, u1, b[1], b[3]);
    *px = x;
    *py = y;
    *pdf = PortalFuncAt(E, x, y) / bInt;
    return true;
}
// ImageLookup's pixel: Image::LookupNearestChannel(uv, c) with the default clamp wrap
PHD EnvCoef PortalCoefAt(const DeviceEnvLight &E, float u, float v) {
    int x = (int)(u * E.res), y = (int)(v * E.res);
    x = x < 0 ? 0 : (x > E.res - 1 ? E.res - 1 : x);
    y = y < 0 ? 0 : (y > E.res - 1 ? E.res - 1 : y);
    return E.coef[(size_t)y * E.res + x];
}
// PortalImageInfiniteLight::SampleLi (lights.cpp:1257-1281); false for {} (or pdf 0)
PHD bool PortalSampleLi(const DeviceEnvLight &E, V3 p, float u0, float u1, V3 *wi, float *pdf, EnvCoef *ec) {
    float b[4];
    if (!PortalImageBounds(E, p, b)) return false;
    float uu, vv, mapPDF;
    if (!PortalWindowedSample(E, u0, u1, b, &uu, &vv, &mapPDF)) return false;
    float duv_dw;
    *wi = PortalRenderFromImage(E.pf, uu, vv, &duv_dw);
    if (duv_dw == 0) return false;
    *pdf = mapPDF / duv_dw;
    *ec = PortalCoefAt(E, uu, vv);
    return *pdf != 0;
}
// PortalImageInfiniteLight::Le(ray) (lights.cpp:1239-1246): zero coefficients outside the
// portal's bounds as seen from the ray origin
PHD EnvCoef PortalLeCoef(const DeviceEnvLight &E, V3 o, V3 d) {
    float u, v, b[4];
    if (!PortalImageFromRender(E, Normalize(d), &u, &v, nullptr) || !PortalImageBounds(E, o, b) || !(u >= b[0] && u <= b[2] && v >= b[1] && v <= b[3]))
        return EnvCoef{0, 0, 0, 0};
    return PortalCoefAt(E, u, v);
}
// PortalImageInfiniteLight::PDF_Li(ctx, w) (lights.cpp:1283-1297) from the reference point p
PHD float PortalPDFLi(const DeviceEnvLight &E, V3 p, V3 w) {
    float u, v, duv_dw, b[4];
    if (!PortalImageFromRender(E, w, &u, &v, &duv_dw) || duv_dw == 0) return 0;
    if (!PortalImageBounds(E, p, b)) return 0;
    const float fi = SatIntegral(E, b[0], b[1], b[2], b[3]);
    if (fi == 0) return 0;
    return (PortalFuncAt(E, u, v) / fi) / duv_dw;
}

// ---------------------------------------------------------------- cloud medium
// Perlin gradient noise (util/noise.cpp:53-118) over the permutation stored with a cloud
// medium (as floats); NoiseWeight's powers in pbrt's Pow<n> association
PHD float NoiseGrad(const float *perm, int x, int y, int z, float dx, float dy, float dz) {
    int h = (int)perm[(int)perm[(int)perm[x] + y] + z];
    h &= 15;
    const float u = h < 8 || h == 12 || h == 13 ? dx : dy;
    const float v = h < 4 || h == 12 || h == 13 ? dy : dz;
    return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
}
PHD float NoiseWeight(float t) {
    const float t2 = t * t;
    const float p5 = t2 * t2 * t, p4 = t2 * t2 * 1.f, p3 = t * t * t;
    return 6 * p5 - 15 * p4 + 10 * p3;
}
PHD float Noise3(const float *perm, float x, float y, float z) {
    x = std::fmod(x, float(1 << 30));
    y = std::fmod(y, float(1 << 30));
    z = std::fmod(z, float(1 << 30));
    int ix = (int)std::floor(x), iy = (int)std::floor(y), iz = (int)std::floor(z);
    const float dx = x - ix, dy = y - iy, dz = z - iz;
    ix &= 255;
    iy &= 255;
    iz &= 255;
    const float w000 = NoiseGrad(perm, ix, iy, iz, dx, dy, dz);
    const float w100 = NoiseGrad(perm, ix + 1, iy, iz, dx - 1, dy, dz);
    const float w010 = NoiseGrad(perm, ix, iy + 1, iz, dx, dy - 1, dz);
    const float w110 = NoiseGrad(perm, ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
    const float w001 = NoiseGrad(perm, ix, iy, iz + 1, dx, dy, dz - 1);
    const float w101 = NoiseGrad(perm, ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
    const float w011 = NoiseGrad(perm, ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
    const float w111 = NoiseGrad(perm, ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
    const float wx = NoiseWeight(dx), wy = NoiseWeight(dy), wz = NoiseWeight(dz);
    const float x00 = Lerpf(wx, w000, w100), x10 = Lerpf(wx, w010, w110);
    const float x01 = Lerpf(wx, w001, w101), x11 = Lerpf(wx, w011, w111);
    return Lerpf(wz, Lerpf(wy, x00, x10), Lerpf(wy, x01, x11));
}
// CloudMedium::Density (media.h:493-517) at a medium-space point; c = {density, wispiness,
// frequency, perm[512]}
PHD float CloudDensity(const float *c, V3 p) {
    const float *perm = c + 3;
    const float freq = c[2];
    V3 pp(freq * p.x, freq * p.y, freq * p.z);
    if (c[1] > 0) {
        float vomega = 0.05f * c[1], vlambda = 10.f;
        for (int i = 0; i < 2; ++i) {
            // DNoise(vlambda * pp) (util/noise.cpp:120-126)
            const V3 q(vlambda * pp.x, vlambda * pp.y, vlambda * pp.z);
            const float delta = .01f;
            const float n = Noise3(perm, q.x, q.y, q.z);
            const float nx = Noise3(perm, q.x + delta, q.y + 0.f, q.z + 0.f);
            const float ny = Noise3(perm, q.x + 0.f, q.y + delta, q.z + 0.f);
            const float nz = Noise3(perm, q.x + 0.f, q.y + 0.f, q.z + delta);
            pp = V3(pp.x + vomega * ((nx - n) / delta), pp.y + vomega * ((ny - n) / delta),
                    pp.z + vomega * ((nz - n) / delta));
            vomega *= 0.5f;
            vlambda *= 1.99f;
        }
    }
    float d = 0, omega = 0.5f, lambda = 1.f;
    for (int i = 0; i < 5; ++i) {
        d += omega * Noise3(perm, lambda * pp.x, lambda * pp.y, lambda * pp.z);
        omega *= 0.5f;
        lambda *= 1.99f;
    }
    d = Clampf((1 - p.y) * 4.5f * c[0] * d, 0, 1);
    d += 2 * std::fmax(0.f, 0.5f - p.y);
    return Clampf(d, 0, 1);
}

// ---------------------------------------------------------------- analytic shapes
// Interval (util/math.h:819-1076) with pbrt's CPU rounding helpers AddRoundUp(a, b) =
// NextFloatUp(a + b) etc. (util/float.h:201-301); the constructor orders its bounds
struct Itv {
    float lo, hi;
};
PHD Itv ItvMake(float a, float b) { return Itv{(b < a) ? b : a, (a < b) ? b : a}; }
PHD Itv ItvExact(float v) { return Itv{v, v}; }
PHD Itv ItvFromValueAndError(float v, float err) {
    if (err == 0) return Itv{v, v};
    return Itv{NextFloatDown(v + (-err)), NextFloatUp(v + err)};
}
PHD float ItvMid(Itv i) { return (i.lo + i.hi) / 2; }
PHD float ItvErr(Itv i) { return (i.hi - i.lo) / 2; }
PHD bool ItvHasZero(Itv i) { return 0 >= i.lo && 0 <= i.hi; }
PHD float Min4(float a, float b, float c, float d) {
    float m = a;
    m = (b < m) ? b : m;
    m = (c < m) ? c : m;
    return (d < m) ? d : m;
}
PHD float Max4(float a, float b, float c, float d) {
    float m = a;
    m = (m < b) ? b : m;
    m = (m < c) ? c : m;
    return (m < d) ? d : m;
}
PHD Itv operator+(Itv a, Itv b) { return ItvMake(NextFloatDown(a.lo + b.lo), NextFloatUp(a.hi + b.hi)); }
PHD Itv operator-(Itv a, Itv b) { return ItvMake(NextFloatDown(a.lo + (-b.hi)), NextFloatUp(a.hi + (-b.lo))); }
PHD Itv operator*(Itv a, Itv b) {
    return ItvMake(Min4(NextFloatDown(a.lo * b.lo), NextFloatDown(a.hi * b.lo), NextFloatDown(a.lo * b.hi),
                        NextFloatDown(a.hi * b.hi)),
                   Max4(NextFloatUp(a.lo * b.lo), NextFloatUp(a.hi * b.lo), NextFloatUp(a.lo * b.hi),
                        NextFloatUp(a.hi * b.hi)));
}
PHD Itv operator/(Itv a, Itv b) {
    if (ItvHasZero(b)) return Itv{-kInfinity, kInfinity};
    return ItvMake(Min4(NextFloatDown(a.lo / b.lo), NextFloatDown(a.hi / b.lo), NextFloatDown(a.lo / b.hi),
                        NextFloatDown(a.hi / b.hi)),
                   Max4(NextFloatUp(a.lo / b.lo), NextFloatUp(a.hi / b.lo), NextFloatUp(a.lo / b.hi),
                        NextFloatUp(a.hi / b.hi)));
}
PHD Itv operator*(float f, Itv i) {
    if (f > 0) return ItvMake(NextFloatDown(f * i.lo), NextFloatUp(f * i.hi));
    return ItvMake(NextFloatDown(f * i.hi), NextFloatUp(f * i.lo));
}
PHD Itv ItvSqr(Itv i) {
    float alow = std::fabs(i.lo), ahigh = std::fabs(i.hi);
    if (alow > ahigh) {
        const float t = alow;
        alow = ahigh;
        ahigh = t;
    }
    if (ItvHasZero(i)) return ItvMake(0, NextFloatUp(ahigh * ahigh));
    return ItvMake(NextFloatDown(alow * alow), NextFloatUp(ahigh * ahigh));
}
PHD Itv ItvSqrt(Itv i) { return ItvMake(std::fmax(0.f, NextFloatDown(std::sqrt(i.lo))), NextFloatUp(std::sqrt(i.hi))); }
struct P3i {
    Itv x, y, z;
};
// Transform::operator()(Point3fi) / (Vector3fi) for exact inputs (util/transform.h:133-176,
// 272-306): the affine 3x4 row-major matrix m; the result as Point3fi(value, error)
PHD P3i XfPointExact(const float *m, V3 p) {
    const float x = p.x, y = p.y, z = p.z;
    P3i r;
    Itv *o[3] = {&r.x, &r.y, &r.z};
    for (int i = 0; i < 3; ++i) {
        const float *row = m + 4 * i;
        const float v = (row[0] * x + row[1] * y) + (row[2] * z + row[3]);
        const float e = gamma(3) * (std::fabs(row[0] * x) + std::fabs(row[1] * y) + std::fabs(row[2] * z) +
                                    std::fabs(row[3]));
        *o[i] = ItvFromValueAndError(v, e);
    }
    return r;
}
PHD P3i XfVectorExact(const float *m, V3 v) {
    P3i r;
    Itv *o[3] = {&r.x, &r.y, &r.z};
    for (int i = 0; i < 3; ++i) {
        const float *row = m + 4 * i;
        const float e = gamma(3) * (std::fabs(row[0] * v.x) + std::fabs(row[1] * v.y) + std::fabs(row[2] * v.z));
        const float x = row[0] * v.x + row[1] * v.y + row[2] * v.z;
        *o[i] = ItvFromValueAndError(x, e);
    }
    return r;
}
// Transform::operator()(Point3fi) of an inexact point (value = interval midpoint, error = half
// width): *po, *pe the resulting Point3fi's midpoint and half width
PHD void XfPointInexact(const float *m, P3i p, V3 *po, V3 *pe) {
    const float x = ItvMid(p.x), y = ItvMid(p.y), z = ItvMid(p.z);
    const V3 ein(ItvErr(p.x), ItvErr(p.y), ItvErr(p.z));
    const bool exact = ein.x == 0 && ein.y == 0 && ein.z == 0;
    for (int i = 0; i < 3; ++i) {
        const float *row = m + 4 * i;
        const float v = (row[0] * x + row[1] * y) + (row[2] * z + row[3]);
        float e = gamma(3) * (std::fabs(row[0] * x) + std::fabs(row[1] * y) + std::fabs(row[2] * z) + std::fabs(row[3]));
        if (!exact)
            e = (gamma(3) + 1) * (std::fabs(row[0]) * ein.x + std::fabs(row[1]) * ein.y + std::fabs(row[2]) * ein.z) + e;
        const Itv r = ItvFromValueAndError(v, e);
        (*po)[i] = ItvMid(r);
        (*pe)[i] = ItvErr(r);
    }
}
// Transform::operator()(Vector3f) and (Normal3f) (the normal through the inverse's transpose)
PHD V3 XfVec(const float *m, V3 v) {
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
PHD V3 XfNormal(const float *mInv, V3 n) {
    return V3(mInv[0] * n.x + mInv[4] * n.y + mInv[8] * n.z, mInv[1] * n.x + mInv[5] * n.y + mInv[9] * n.z,
              mInv[2] * n.x + mInv[6] * n.y + mInv[10] * n.z);
}
// Transform::operator()(Point3f) (util/transform.h:310-319), affine
PHD V3 XfPt(const float *m, V3 p) {
    return V3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}

// Sphere and Disk (shapes.h:106-571): affine renderFromObject (o2r) and objectFromRender (r2o)
enum ShapeKindT { kShapeSphereT = 1, kShapeDiskT = 2, kShapeBilinearT = 3, kShapeCylinderT = 4 };
struct alignas(16) DeviceShape {
    float r2o[12], o2r[12];
    // sphere: radius, zMin, zMax, phiMax, thetaZMin, thetaZMax; disk: height, radius,
    // innerRadius, phiMax; bilinear patch: area, isRectangle (render-space corners p00 p10 p01
    // p11 in r2o, their uv in o2r[0..7], vertex normals in a side array)
    float a, b, c, d, e, f;
    int kind, flags;  // flags: bit0 reverseOrientation, bit1 transformSwapsHandedness, bit2 uv, bit3 N
};
static_assert(sizeof(DeviceShape) == 128, "DeviceShape must be 128 bytes");
// binary BVH over the analytic shapes (host-built, median split): count 0 = interior node whose
// children are this + 1 and `child`; count > 0 = leaf of shapes [child, child + count)
struct alignas(16) ShapeBVHNode {
    float lo[3], hi[3];
    int child, count;
};
// ---- bilinear patches (shapes.h:1272-1540, shapes.cpp:1041-1372)
PHD V3 LerpV(float t, V3 a, V3 b) { return (1 - t) * a + t * b; }
// Quadratic(float) (util/math.h:614-637)
PHD bool QuadraticF(float a, float b, float c, float *t0, float *t1) {
    if (a == 0) {
        if (b == 0) return false;
        *t0 = *t1 = -c / b;
        return true;
    }
    const float discrim = DifferenceOfProducts(b, b, 4 * a, c);
    if (discrim < 0) return false;
    const float rootDiscrim = std::sqrt(discrim);
    const float q = -0.5f * (b + std::copysign(rootDiscrim, b));
    *t0 = q / a;
    *t1 = c / q;
    if (*t0 > *t1) {
        const float t = *t0;
        *t0 = *t1;
        *t1 = t;
    }
    return true;
}
// Determinant(SquareMatrix<3>) (util/math.h:1420-1426), rows (a0 a1 a2) (b0 b1 b2) (c0 c1 c2)
PHD float Det3(float a0, float a1, float a2, float b0, float b1, float b2, float c0, float c1, float c2) {
    const float minor12 = DifferenceOfProducts(b1, c2, b2, c1);
    const float minor02 = DifferenceOfProducts(b0, c2, b2, c0);
    const float minor01 = DifferenceOfProducts(b0, c1, b1, c0);
    return fmaf(a2, minor01, DifferenceOfProducts(a0, minor12, a1, minor02));
}
struct PatchVerts {
    V3 p00, p10, p01, p11;
};
PHD PatchVerts PatchP(const DeviceShape &s) {
    const float *q = s.r2o;
    return PatchVerts{V3(q[0], q[1], q[2]), V3(q[3], q[4], q[5]), V3(q[6], q[7], q[8]), V3(q[9], q[10], q[11])};
}
// IntersectBilinearPatch (shapes.h:1279-1347): *u, *v the patch parameters
PHD bool BilinearIntersect(const DeviceShape &s, V3 o, V3 d, float tMax, float *tHit, float *uo, float *vo) {
    const PatchVerts P = PatchP(s);
    const V3 p00 = P.p00, p10 = P.p10, p01 = P.p01, p11 = P.p11;
    const float a = Dot(Cross(p10 - p00, p01 - p11), d);
    const float c = Dot(Cross(p00 - o, d), p01 - p00);
    const float b = Dot(Cross(p10 - o, d), p11 - p10) - (a + c);
    float u1, u2;
    if (!QuadraticF(a, b, c, &u1, &u2)) return false;
    const float eps = gamma(10) * (MaxComponentValue(Abs(o)) + MaxComponentValue(Abs(d)) + MaxComponentValue(Abs(p00)) +
                                   MaxComponentValue(Abs(p10)) + MaxComponentValue(Abs(p01)) + MaxComponentValue(Abs(p11)));
    float t = tMax, u = 0, v = 0;
    if (0 <= u1 && u1 <= 1) {
        const V3 uo1 = LerpV(u1, p00, p10);
        const V3 ud = LerpV(u1, p01, p11) - uo1;
        const V3 deltao = uo1 - o;
        const V3 perp = Cross(d, ud);
        const float p2 = LengthSquared(perp);
        const float v1 = Det3(deltao.x, d.x, perp.x, deltao.y, d.y, perp.y, deltao.z, d.z, perp.z);
        const float t1 = Det3(deltao.x, ud.x, perp.x, deltao.y, ud.y, perp.y, deltao.z, ud.z, perp.z);
        if (t1 > p2 * eps && 0 <= v1 && v1 <= p2) {
            u = u1;
            v = v1 / p2;
            t = t1 / p2;
        }
    }
    if (0 <= u2 && u2 <= 1 && u2 != u1) {
        const V3 uo2 = LerpV(u2, p00, p10);
        const V3 ud = LerpV(u2, p01, p11) - uo2;
        const V3 deltao = uo2 - o;
        const V3 perp = Cross(d, ud);
        const float p2 = LengthSquared(perp);
        const float v2 = Det3(deltao.x, d.x, perp.x, deltao.y, d.y, perp.y, deltao.z, d.z, perp.z);
        float t2 = Det3(deltao.x, ud.x, perp.x, deltao.y, ud.y, perp.y, deltao.z, ud.z, perp.z);
        t2 /= p2;
        if (0 <= v2 && v2 <= p2 && t > t2 && t2 > eps) {
            t = t2;
            u = u2;
            v = v2 / p2;
        }
    }
    if (t >= tMax) return false;
    *tHit = t;
    *uo = u;
    *vo = v;
    return true;
}
// RotateFromTo(from, to) applied to a vector (util/transform.h:249-270)
PHD V3 RotateFromToApply(V3 from, V3 to, V3 w) {
    V3 refl;
    if (std::fabs(from.x) < 0.72f && std::fabs(to.x) < 0.72f) refl = V3(1, 0, 0);
    else if (std::fabs(from.y) < 0.72f && std::fabs(to.y) < 0.72f) refl = V3(0, 1, 0);
    else refl = V3(0, 0, 1);
    const V3 u = refl - from, v = refl - to;
    const float uu = Dot(u, u), vv = Dot(v, v), uv = Dot(u, v);
    float r[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            r[i][j] = ((i == j) ? 1 : 0) - 2 / uu * u[i] * u[j] - 2 / vv * v[i] * v[j] + 4 * uv / (uu * vv) * v[i] * u[j];
    return V3(r[0][0] * w.x + r[0][1] * w.y + r[0][2] * w.z, r[1][0] * w.x + r[1][1] * w.y + r[1][2] * w.z,
              r[2][0] * w.x + r[2][1] * w.y + r[2][2] * w.z);
}
PHD void PatchUV(const DeviceShape &s, int k, float *u, float *v) {
    *u = s.o2r[2 * k];
    *v = s.o2r[2 * k + 1];
}
// a bilinear patch's texture coordinates at parametric (u, v): the mesh uv lerp when the patch
// has uv (flags bit 2), else (u, v) itself
PHD void PatchST(const DeviceShape &s, float uu, float vv, float st[2]) {
    st[0] = uu;
    st[1] = vv;
    if (s.flags & 4) {
        float a[4][2];
        for (int k = 0; k < 4; ++k) PatchUV(s, k, &a[k][0], &a[k][1]);  // uv00 uv10 uv01 uv11
        for (int j = 0; j < 2; ++j) st[j] = Lerpf(uu, Lerpf(vv, a[0][j], a[2][j]), Lerpf(vv, a[1][j], a[3][j]));
    }
}
// BilinearPatch::InteractionFromIntersection (shapes.h:1396-1497) without dndu/dndv; N: the
// four vertex normals (render space, 12 floats) when the mesh has them
PHD TriSurface BilinearSurface(const DeviceShape &s, const float *N, float uu, float vv) {
    const PatchVerts P = PatchP(s);
    const V3 p00 = P.p00, p10 = P.p10, p01 = P.p01, p11 = P.p11;
    const V3 p = LerpV(uu, LerpV(vv, p00, p01), LerpV(vv, p10, p11));
    V3 dpdu = LerpV(vv, p10, p11) - LerpV(vv, p00, p01);
    V3 dpdv = LerpV(uu, p01, p11) - LerpV(uu, p00, p10);
    float st[2] = {uu, vv};
    if (s.flags & 4) {
        float a[4][2];
        for (int k = 0; k < 4; ++k) PatchUV(s, k, &a[k][0], &a[k][1]);  // uv00 uv10 uv01 uv11
        float dstdu[2], dstdv[2];
        for (int j = 0; j < 2; ++j) {
            st[j] = Lerpf(uu, Lerpf(vv, a[0][j], a[2][j]), Lerpf(vv, a[1][j], a[3][j]));
            dstdu[j] = Lerpf(vv, a[1][j], a[3][j]) - Lerpf(vv, a[0][j], a[2][j]);
            dstdv[j] = Lerpf(uu, a[2][j], a[3][j]) - Lerpf(uu, a[0][j], a[1][j]);
        }
        const float duds = std::fabs(dstdu[0]) < 1e-8f ? 0 : 1 / dstdu[0];
        const float dvds = std::fabs(dstdv[0]) < 1e-8f ? 0 : 1 / dstdv[0];
        const float dudt = std::fabs(dstdu[1]) < 1e-8f ? 0 : 1 / dstdu[1];
        const float dvdt = std::fabs(dstdv[1]) < 1e-8f ? 0 : 1 / dstdv[1];
        const V3 dpds = dpdu * duds + dpdv * dvds;
        V3 dpdt = dpdu * dudt + dpdv * dvdt;
        const V3 cst = Cross(dpds, dpdt);
        if (cst.x != 0 || cst.y != 0 || cst.z != 0) {
            if (Dot(Cross(dpdu, dpdv), cst) < 0) dpdt = -dpdt;
            dpdu = dpds;
            dpdv = dpdt;
        }
    }
    const V3 pAbsSum = Abs(p00) + Abs(p01) + Abs(p10) + Abs(p11);
    TriSurface r;
    ToPoint3fi(p, gamma(6) * pAbsSum, &r.p, &r.pErr);
    V3 n = Normalize(Cross(dpdu, dpdv));
    if (((s.flags & 1) != 0) != ((s.flags & 2) != 0)) n = -n;
    r.n = n;
    r.ns = n;
    r.dpdu = r.dpdus = dpdu;
    r.dpdv = dpdv;
    r.uv[0] = st[0];
    r.uv[1] = st[1];
    if ((s.flags & 8) && N) {
        const V3 n00(N[0], N[1], N[2]), n10(N[3], N[4], N[5]), n01(N[6], N[7], N[8]), n11(N[9], N[10], N[11]);
        V3 ns = LerpV(uu, LerpV(vv, n00, n01), LerpV(vv, n10, n11));
        if (LengthSquared(ns) > 0) {
            ns = Normalize(ns);
            V3 sd = RotateFromToApply(Normalize(r.n), ns, dpdu), sv = RotateFromToApply(Normalize(r.n), ns, dpdv);
            // SetShadingGeometry(ns, r(dpdu), r(dpdv), ..., true) (interaction.h:194-214)
            r.ns = ns;
            r.n = FaceForwardN(r.n, ns);
            while (LengthSquared(sd) > 1e16f || LengthSquared(sv) > 1e16f) {
                sd = sd / 1e8f;
                sv = sv / 1e8f;
            }
            r.dpdus = sd;
        }
    }
    return r;
}
// the patch normal at (u, v) for sampling (shapes.cpp:1199-1208)
PHD V3 PatchSampleNormal(const DeviceShape &s, const float *N, V3 n, float uu, float vv) {
    if ((s.flags & 8) && N) {
        const V3 n00(N[0], N[1], N[2]), n10(N[3], N[4], N[5]), n01(N[6], N[7], N[8]), n11(N[9], N[10], N[11]);
        const V3 ns = LerpV(uu, LerpV(vv, n00, n01), LerpV(vv, n10, n11));
        return FaceForwardN(n, ns);
    }
    if (((s.flags & 1) != 0) != ((s.flags & 2) != 0)) return -n;
    return n;
}
// the bilinear warp's corner weights of a non-rectangular patch (shapes.cpp:1173-1175)
PHD void PatchAreaWeights(const PatchVerts &P, float w[4]) {
    w[0] = Length(Cross(P.p10 - P.p00, P.p01 - P.p00));
    w[1] = Length(Cross(P.p10 - P.p00, P.p11 - P.p10));
    w[2] = Length(Cross(P.p01 - P.p00, P.p11 - P.p01));
    w[3] = Length(Cross(P.p11 - P.p10, P.p11 - P.p01));
}
// BilinearPatch::Sample(u) (shapes.cpp:1158-1217): area measure; false for {}
PHD bool BilinearSampleArea(const DeviceShape &s, const float *N, float u0, float u1, V3 *pOut, V3 *pErr, V3 *nOut,
                            float *pdfOut, float *stOut = nullptr) {
    const PatchVerts P = PatchP(s);
    float pdf = 1, uu = u0, vv = u1;
    if (s.b == 0) {
        float w[4];
        PatchAreaWeights(P, w);
        SampleBilinear(u0, u1, w, &uu, &vv);
        pdf = BilinearPDF(uu, vv, w);
    }
    const V3 pu0 = LerpV(vv, P.p00, P.p01), pu1 = LerpV(vv, P.p10, P.p11);
    const V3 p = LerpV(uu, pu0, pu1);
    const V3 dpdu = pu1 - pu0;
    const V3 dpdv = LerpV(uu, P.p01, P.p11) - LerpV(uu, P.p00, P.p10);
    if (LengthSquared(dpdu) == 0 || LengthSquared(dpdv) == 0) return false;
    *nOut = PatchSampleNormal(s, N, Normalize(Cross(dpdu, dpdv)), uu, vv);
    const V3 pAbsSum = Abs(P.p00) + Abs(P.p01) + Abs(P.p10) + Abs(P.p11);
    ToPoint3fi(p, gamma(6) * pAbsSum, pOut, pErr);
    *pdfOut = pdf / Length(Cross(dpdu, dpdv));
    if (stOut) PatchST(s, uu, vv, stOut);
    return true;
}
// SphericalQuadArea (util/vecmath.h:1648-1666)
PHD float SphericalQuadArea(V3 a, V3 b, V3 c, V3 d) {
    V3 axb = Cross(a, b), bxc = Cross(b, c), cxd = Cross(c, d), dxa = Cross(d, a);
    if (LengthSquared(axb) == 0 || LengthSquared(bxc) == 0 || LengthSquared(cxd) == 0 || LengthSquared(dxa) == 0)
        return 0;
    axb = Normalize(axb);
    bxc = Normalize(bxc);
    cxd = Normalize(cxd);
    dxa = Normalize(dxa);
    const float alpha = AngleBetween(dxa, -axb), beta = AngleBetween(axb, -bxc);
    const float gam = AngleBetween(bxc, -cxd), delta = AngleBetween(cxd, -dxa);
    return std::fabs(alpha + beta + gam + delta - 2 * kPi);
}
// SampleSphericalRectangle (util/sampling.cpp:163-220)
PHD V3 SampleSphericalRectangle(V3 pRef, V3 sq, V3 ex, V3 ey, float u0, float u1, float *pdf) {
    const float exl = Length(ex), eyl = Length(ey);
    const V3 rx = ex / exl, ry = ey / eyl;
    V3 rz = Cross(rx, ry);
    const V3 dd0 = sq - pRef;
    float z0 = Dot(dd0, rz);
    const float x0 = Dot(dd0, rx), y0 = Dot(dd0, ry);
    if (z0 > 0) {
        rz = -rz;
        z0 *= -1;
    }
    const float x1 = x0 + exl, y1 = y0 + eyl;
    const V3 v00(x0, y0, z0), v01(x0, y1, z0), v10(x1, y0, z0), v11(x1, y1, z0);
    const V3 n0 = Normalize(Cross(v00, v10)), n1 = Normalize(Cross(v10, v11));
    const V3 n2 = Normalize(Cross(v11, v01)), n3 = Normalize(Cross(v01, v00));
    const float g0 = AngleBetween(-n0, n1), g1 = AngleBetween(-n1, n2);
    const float g2 = AngleBetween(-n2, n3), g3 = AngleBetween(-n3, n0);
    const float solidAngle = g0 + g1 + g2 + g3 - 2 * kPi;
    if (solidAngle <= 0) {
        *pdf = 0;
        return sq + u0 * ex + u1 * ey;
    }
    *pdf = std::fmax(0.f, 1 / solidAngle);
    if (solidAngle < 1e-3f) return sq + u0 * ex + u1 * ey;
    const float b0 = n0.z, b1 = n2.z;
    const float au = u0 * (g0 + g1 - 2 * kPi) + (u0 - 1) * (g2 + g3);
    float sau, cau;
    SinCosf(au, &sau, &cau);
    const float fu = (cau * b0 - b1) / sau;
    float cu = std::copysign(1 / std::sqrt(Sqr(fu) + Sqr(b0)), fu);
    cu = Clampf(cu, -kOneMinusEpsilon, kOneMinusEpsilon);
    float xu = -(cu * z0) / SafeSqrt(1 - Sqr(cu));
    xu = Clampf(xu, x0, x1);
    const float dd = std::sqrt(Sqr(xu) + Sqr(z0));
    const float h0 = y0 / std::sqrt(Sqr(dd) + Sqr(y0));
    const float h1 = y1 / std::sqrt(Sqr(dd) + Sqr(y1));
    const float hv = h0 + u1 * (h1 - h0), hvsq = Sqr(hv);
    const float yv = (hvsq < 1 - 1e-6f) ? (hv * dd) / std::sqrt(1 - hvsq) : y1;
    return pRef + (rx * xu + ry * yv + rz * z0);
}
// InvertSphericalRectangleSample (util/sampling.cpp:222-345)
PHD void InvertSphericalRectangleSample(V3 pRef, V3 sq, V3 ex, V3 ey, V3 pRect, float *uo0, float *uo1) {
    const float exl = Length(ex), eyl = Length(ey);
    const V3 rx = ex / exl, ry = ey / eyl;
    V3 rz = Cross(rx, ry);
    const V3 dd0 = sq - pRef;
    float z0 = Dot(dd0, rz);
    const float x0 = Dot(dd0, rx), y0 = Dot(dd0, ry);
    if (z0 > 0) {
        rz = -rz;
        z0 *= -1;
    }
    const float z0sq = Sqr(z0);
    const float x1 = x0 + exl, y1 = y0 + eyl;
    const float y0sq = Sqr(y0), y1sq = Sqr(y1);
    const V3 v00(x0, y0, z0), v01(x0, y1, z0), v10(x1, y0, z0), v11(x1, y1, z0);
    const V3 n0 = Normalize(Cross(v00, v10)), n1 = Normalize(Cross(v10, v11));
    const V3 n2 = Normalize(Cross(v11, v01)), n3 = Normalize(Cross(v01, v00));
    const float g0 = AngleBetween(-n0, n1), g1 = AngleBetween(-n1, n2);
    const float g2 = AngleBetween(-n2, n3), g3 = AngleBetween(-n3, n0);
    const float b0 = n0.z, b1 = n2.z, b0sq = Sqr(b0);
    const float solidAngle = (float)((double)g0 + (double)g1 + (double)g2 + (double)g3 - 2. * (double)kPi);
    if (solidAngle < 1e-3f) {
        const V3 pq = pRect - sq;
        *uo0 = Dot(pq, ex) / LengthSquared(ex);
        *uo1 = Dot(pq, ey) / LengthSquared(ey);
        return;
    }
    const V3 dv = pRect - pRef;
    float xu = Dot(dv, rx);
    const float yv = Dot(dv, ry);
    xu = Clampf(xu, x0, x1);
    if (xu == 0) xu = 1e-10f;
    const float invcusq = 1 + z0sq / Sqr(xu);
    const float fusq = invcusq - b0sq;
    const float fu = std::copysign(std::sqrt(fusq), xu);
    const float sqr = SafeSqrt(DifferenceOfProducts(b0, b0, b1, b1) + fusq);
    float au = ATan2f(-(b1 * fu) - std::copysign(b0 * sqr, fu * b0), b0 * b1 - sqr * std::fabs(fu));
    if (au > 0) au -= 2 * kPi;
    if (fu == 0) au = kPi;
    const float u0 = (au + g2 + g3) / solidAngle;
    const float ddsq = Sqr(xu) + z0sq;
    const float dd = std::sqrt(ddsq);
    const float h0 = y0 / std::sqrt(ddsq + y0sq);
    const float h1 = y1 / std::sqrt(ddsq + y1sq);
    const float yvsq = Sqr(yv);
    const float root = std::fabs(h0 - h1) * std::sqrt(yvsq * (ddsq + yvsq)) / (ddsq + yvsq);
    const float u1a = (DifferenceOfProducts(h0, h0, h0, h1) - root) / Sqr(h0 - h1);
    const float u1b = (DifferenceOfProducts(h0, h0, h0, h1) + root) / Sqr(h0 - h1);
    const float hva = Lerpf(u1a, h0, h1), hvb = Lerpf(u1b, h0, h1);
    const float yza = (hva * dd) / std::sqrt(1 - Sqr(hva)), yzb = (hvb * dd) / std::sqrt(1 - Sqr(hvb));
    *uo0 = Clampf(u0, 0, 1);
    *uo1 = (std::fabs(yza - yv) < std::fabs(yzb - yv)) ? u1a : u1b;
}
// InvertBilinear (util/vecmath.h:625-654) of st over the corner uvs uv00 uv10 uv01 uv11
PHD void InvertBilinearUV(const DeviceShape &s, float px, float py, float *uo, float *vo) {
    float a[2], b[2], c[2], d[2];
    PatchUV(s, 0, &a[0], &a[1]);
    PatchUV(s, 1, &b[0], &b[1]);
    PatchUV(s, 3, &c[0], &c[1]);
    PatchUV(s, 2, &d[0], &d[1]);
    const float e[2] = {b[0] - a[0], b[1] - a[1]}, f[2] = {d[0] - a[0], d[1] - a[1]};
    const float g[2] = {(a[0] - b[0]) + (c[0] - d[0]), (a[1] - b[1]) + (c[1] - d[1])}, h[2] = {px - a[0], py - a[1]};
    auto cross2d = [](const float *x, const float *y) { return DifferenceOfProducts(x[0], y[1], x[1], y[0]); };
    const float k2 = cross2d(g, f), k1 = cross2d(e, f) + cross2d(h, g), k0 = cross2d(h, e);
    if (std::fabs(k2) < 0.001f) {
        if (std::fabs(e[0] * k1 - g[0] * k0) < 1e-5f) *uo = (h[1] * k1 + f[1] * k0) / (e[1] * k1 - g[1] * k0);
        else *uo = (h[0] * k1 + f[0] * k0) / (e[0] * k1 - g[0] * k0);
        *vo = -k0 / k1;
        return;
    }
    float v0, v1;
    if (!QuadraticF(k2, k1, k0, &v0, &v1)) {
        *uo = *vo = 0;
        return;
    }
    const float u = (h[0] - f[0] * v0) / (e[0] + g[0] * v0);
    if (u < 0 || u > 1 || v0 < 0 || v0 > 1) {
        *uo = (h[0] - f[0] * v1) / (e[0] + g[0] * v1);
        *vo = v1;
        return;
    }
    *uo = u;
    *vo = v0;
}
PHD float ShapeArea(const DeviceShape &s) {
    if (s.kind == kShapeBilinearT) return s.a;
    if (s.kind == kShapeSphereT) return s.d * s.a * (s.c - s.b);  // phiMax radius (zMax - zMin)
    if (s.kind == kShapeCylinderT) return (s.c - s.b) * s.a * s.d;  // (zMax - zMin) radius phiMax
    return s.d * 0.5f * (Sqr(s.b) - Sqr(s.c));                    // phiMax / 2 (r^2 - ri^2)
}
// phi of an object-space hit (atan2, wrapped to [0, 2 pi))
PHD float ShapePhi(V3 p) {
    float phi = ATan2f(p.y, p.x);
    if (phi < 0) phi += 2 * kPi;
    return phi;
}
// Sphere::BasicIntersect (shapes.h:147-229): *pObj the refined object-space hit
PHD bool SphereIntersect(const DeviceShape &s, V3 ro, V3 rd, float tMax, float *tHit, V3 *pObj) {
    const float radius = s.a, zMin = s.b, zMax = s.c, phiMax = s.d;
    const P3i oi = XfPointExact(s.r2o, ro), di = XfVectorExact(s.r2o, rd);
    const Itv a = ItvSqr(di.x) + ItvSqr(di.y) + ItvSqr(di.z);
    const Itv b = 2.f * (di.x * oi.x + di.y * oi.y + di.z * oi.z);
    const Itv c = ItvSqr(oi.x) + ItvSqr(oi.y) + ItvSqr(oi.z) - ItvSqr(ItvExact(radius));
    const Itv f = b / (2.f * a);
    const Itv vx = oi.x - f * di.x, vy = oi.y - f * di.y, vz = oi.z - f * di.z;
    const Itv length = ItvSqrt(ItvSqr(vx) + ItvSqr(vy) + ItvSqr(vz));
    const Itv discrim = 4.f * a * (ItvExact(radius) + length) * (ItvExact(radius) - length);
    if (discrim.lo < 0) return false;
    const Itv rootDiscrim = ItvSqrt(discrim);
    const Itv q = ItvMid(b) < 0 ? -.5f * (b - rootDiscrim) : -.5f * (b + rootDiscrim);
    Itv t0 = q / a, t1 = c / q;
    if (t0.lo > t1.lo) {
        const Itv t = t0;
        t0 = t1;
        t1 = t;
    }
    if (t0.hi > tMax || t1.lo <= 0) return false;
    Itv tShapeHit = t0;
    if (tShapeHit.lo <= 0) {
        tShapeHit = t1;
        if (tShapeHit.hi > tMax) return false;
    }
    const V3 o(ItvMid(oi.x), ItvMid(oi.y), ItvMid(oi.z)), d(ItvMid(di.x), ItvMid(di.y), ItvMid(di.z));
    for (int pass = 0; pass < 2; ++pass) {
        const float th = ItvMid(tShapeHit);
        V3 pHit = o + th * d;
        const float sc = radius / Distance(pHit, V3(0, 0, 0));
        pHit = V3(pHit.x * sc, pHit.y * sc, pHit.z * sc);
        if (pHit.x == 0 && pHit.y == 0) pHit.x = 1e-5f * radius;
        const float phi = ShapePhi(pHit);
        if ((zMin > -radius && pHit.z < zMin) || (zMax < radius && pHit.z > zMax) || phi > phiMax) {
            if (pass == 1 || (tShapeHit.lo == t1.lo && tShapeHit.hi == t1.hi)) return false;
            if (t1.hi > tMax) return false;
            tShapeHit = t1;
            continue;
        }
        *tHit = th;
        *pObj = pHit;
        return true;
    }
    return false;
}
// Cylinder::BasicIntersect (shapes.h:628-722): the sphere's interval quadratic in x and y only,
// the hit refined onto the radius in x-y
PHD bool CylinderIntersect(const DeviceShape &s, V3 ro, V3 rd, float tMax, float *tHit, V3 *pObj) {
    const float radius = s.a, zMin = s.b, zMax = s.c, phiMax = s.d;
    const P3i oi = XfPointExact(s.r2o, ro), di = XfVectorExact(s.r2o, rd);
    const Itv a = ItvSqr(di.x) + ItvSqr(di.y);
    const Itv b = 2.f * (di.x * oi.x + di.y * oi.y);
    const Itv c = ItvSqr(oi.x) + ItvSqr(oi.y) - ItvSqr(ItvExact(radius));
    const Itv f = b / (2.f * a);
    const Itv vx = oi.x - f * di.x, vy = oi.y - f * di.y;
    const Itv length = ItvSqrt(ItvSqr(vx) + ItvSqr(vy));
    const Itv discrim = 4.f * a * (ItvExact(radius) + length) * (ItvExact(radius) - length);
    if (discrim.lo < 0) return false;
    const Itv rootDiscrim = ItvSqrt(discrim);
    const Itv q = ItvMid(b) < 0 ? -.5f * (b - rootDiscrim) : -.5f * (b + rootDiscrim);
    Itv t0 = q / a, t1 = c / q;
    if (t0.lo > t1.lo) {
        const Itv t = t0;
        t0 = t1;
        t1 = t;
    }
    if (t0.hi > tMax || t1.lo <= 0) return false;
    Itv tShapeHit = t0;
    if (tShapeHit.lo <= 0) {
        tShapeHit = t1;
        if (tShapeHit.hi > tMax) return false;
    }
    const V3 o(ItvMid(oi.x), ItvMid(oi.y), ItvMid(oi.z)), d(ItvMid(di.x), ItvMid(di.y), ItvMid(di.z));
    for (int pass = 0; pass < 2; ++pass) {
        const float th = ItvMid(tShapeHit);
        V3 pHit = o + th * d;
        const float hitRad = std::sqrt(Sqr(pHit.x) + Sqr(pHit.y));
        pHit.x *= radius / hitRad;
        pHit.y *= radius / hitRad;
        const float phi = ShapePhi(pHit);
        if (pHit.z < zMin || pHit.z > zMax || phi > phiMax) {
            if (pass == 1 || (tShapeHit.lo == t1.lo && tShapeHit.hi == t1.hi)) return false;
            tShapeHit = t1;
            if (t1.hi > tMax) return false;
            continue;
        }
        *tHit = th;
        *pObj = pHit;
        return true;
    }
    return false;
}
// Disk::BasicIntersect (shapes.h:446-474)
PHD bool DiskIntersect(const DeviceShape &s, V3 ro, V3 rd, float tMax, float *tHit, V3 *pObj) {
    const float height = s.a, radius = s.b, innerRadius = s.c, phiMax = s.d;
    const P3i oi = XfPointExact(s.r2o, ro), di = XfVectorExact(s.r2o, rd);
    if (ItvMid(di.z) == 0) return false;
    const float th = (height - ItvMid(oi.z)) / ItvMid(di.z);
    if (th <= 0 || th >= tMax) return false;
    const V3 pHit = V3(ItvMid(oi.x), ItvMid(oi.y), ItvMid(oi.z)) + th * V3(ItvMid(di.x), ItvMid(di.y), ItvMid(di.z));
    const float dist2 = Sqr(pHit.x) + Sqr(pHit.y);
    if (dist2 > Sqr(radius) || dist2 < Sqr(innerRadius)) return false;
    if (ShapePhi(pHit) > phiMax) return false;
    *tHit = th;
    *pObj = pHit;
    return true;
}
// pObj: the object-space hit (sphere, disk) or (u, v, 0) (bilinear patch)
PHD bool ShapeIntersect(const DeviceShape &s, V3 ro, V3 rd, float tMax, float *tHit, V3 *pObj) {
    if (s.kind == kShapeBilinearT) {
        float u, v;
        if (!BilinearIntersect(s, ro, rd, tMax, tHit, &u, &v)) return false;
        *pObj = V3(u, v, 0);
        return true;
    }
    if (s.kind == kShapeCylinderT) return CylinderIntersect(s, ro, rd, tMax, tHit, pObj);
    return s.kind == kShapeSphereT ? SphereIntersect(s, ro, rd, tMax, tHit, pObj)
                                   : DiskIntersect(s, ro, rd, tMax, tHit, pObj);
}
// Sphere / Disk::InteractionFromIntersection (shapes.h:237-281, 477-501) followed by
// Transform::operator()(SurfaceInteraction) (util/transform.cpp:229-261): render-space p and
// its error, n, shading n (faced to n), dpdu, dpdv and uv
PHD TriSurface ShapeSurface(const DeviceShape &s, V3 pHit, const float *N = nullptr) {
    if (s.kind == kShapeBilinearT) return BilinearSurface(s, N, pHit.x, pHit.y);
    const float phi = ShapePhi(pHit);
    V3 dpdu, dpdv, pError;
    float u, v;
    if (s.kind == kShapeSphereT) {
        const float radius = s.a, phiMax = s.d, thetaZMin = s.e, thetaZMax = s.f;
        u = phi / phiMax;
        const float cosTheta = pHit.z / radius;
        const float theta = SafeACos(cosTheta);
        v = (theta - thetaZMin) / (thetaZMax - thetaZMin);
        const float zRadius = std::sqrt(Sqr(pHit.x) + Sqr(pHit.y));
        const float cosPhi = pHit.x / zRadius, sinPhi = pHit.y / zRadius;
        dpdu = V3(-phiMax * pHit.y, phiMax * pHit.x, 0);
        const float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
        dpdv = (thetaZMax - thetaZMin) * V3(pHit.z * cosPhi, pHit.z * sinPhi, -radius * sinTheta);
        pError = gamma(5) * Abs(pHit);
    } else if (s.kind == kShapeCylinderT) {
        // Cylinder::InteractionFromIntersection (shapes.h:725-760)
        const float zMin = s.b, zMax = s.c, phiMax = s.d;
        u = phi / phiMax;
        v = (pHit.z - zMin) / (zMax - zMin);
        dpdu = V3(-phiMax * pHit.y, phiMax * pHit.x, 0);
        dpdv = V3(0, 0, zMax - zMin);
        pError = gamma(3) * Abs(V3(pHit.x, pHit.y, 0));
    } else {
        const float height = s.a, radius = s.b, innerRadius = s.c, phiMax = s.d;
        u = phi / phiMax;
        const float rHit = std::sqrt(Sqr(pHit.x) + Sqr(pHit.y));
        v = (radius - rHit) / (radius - innerRadius);
        dpdu = V3(-phiMax * pHit.y, phiMax * pHit.x, 0);
        dpdv = V3(pHit.x, pHit.y, 0) * (innerRadius - radius) / rHit;
        pHit.z = height;
        pError = V3(0, 0, 0);
    }
    // SurfaceInteraction ctor (interaction.h): n = Normalize(Cross(dpdu, dpdv)), flipped
    V3 n = Normalize(Cross(dpdu, dpdv));
    if (((s.flags & 1) != 0) != ((s.flags & 2) != 0)) n = -n;
    const P3i pi = {ItvFromValueAndError(pHit.x, pError.x), ItvFromValueAndError(pHit.y, pError.y),
                    ItvFromValueAndError(pHit.z, pError.z)};
    TriSurface r;
    XfPointInexact(s.o2r, pi, &r.p, &r.pErr);
    r.n = Normalize(XfNormal(s.r2o, n));
    r.dpdu = XfVec(s.o2r, dpdu);
    r.dpdv = XfVec(s.o2r, dpdv);
    r.ns = FaceForwardN(Normalize(XfNormal(s.r2o, n)), r.n);
    r.dpdus = r.dpdu;
    r.uv[0] = u;
    r.uv[1] = v;
    return r;
}
// ShapeSample of a sphere or disk light (render space): point, its error, normal
struct ShapeSamplePt {
    V3 p, pErr, n;
    float pdf;
    float uv[2];  // the sample's (u, v): an image emitter's lookup (DiffuseAreaLight::L)
};
// a sphere point's (phi / phiMax, (theta - thetaZMin) / (thetaZMax - thetaZMin)) from its object
// space position (shapes.cpp:54-58, shapes.h:351-357)
PHD void SphereUV(const DeviceShape &s, V3 pObj, float uv[2]) {
    const float theta = SafeACos(pObj.z / s.a);
    float phi = ATan2f(pObj.y, pObj.x);
    if (phi < 0) phi += 2 * kPi;
    uv[0] = phi / s.d;
    uv[1] = (theta - s.e) / (s.f - s.e);
}
// Sphere::Sample(u) / Disk::Sample(u) (shapes.cpp:42-62, shapes.h:509-525): area measure
PHD ShapeSamplePt ShapeSampleArea(const DeviceShape &s, float u0, float u1) {
    ShapeSamplePt r;
    if (s.kind == kShapeSphereT) {
        const float radius = s.a;
        const float z = 1 - 2 * u0, rr = SafeSqrt(1 - Sqr(z)), phi = 2 * kPi * u1;
        float sp, cp;
        SinCosf(phi, &sp, &cp);
        V3 pObj = V3(0, 0, 0) + radius * V3(rr * cp, rr * sp, z);
        const float sc = radius / Distance(pObj, V3(0, 0, 0));
        pObj = V3(pObj.x * sc, pObj.y * sc, pObj.z * sc);
        const V3 pObjError = gamma(5) * Abs(pObj);
        V3 n = Normalize(XfNormal(s.r2o, pObj));
        if (s.flags & 1) n = -n;
        const P3i pi = {ItvFromValueAndError(pObj.x, pObjError.x), ItvFromValueAndError(pObj.y, pObjError.y),
                        ItvFromValueAndError(pObj.z, pObjError.z)};
        XfPointInexact(s.o2r, pi, &r.p, &r.pErr);
        r.n = n;
        SphereUV(s, pObj, r.uv);
    } else if (s.kind == kShapeCylinderT) {
        // Cylinder::Sample(u) (shapes.h:772-793)
        const float radius = s.a, zMin = s.b, zMax = s.c, phiMax = s.d;
        const float z = Lerpf(u0, zMin, zMax), phi = u1 * phiMax;
        float sp, cp;
        SinCosf(phi, &sp, &cp);
        V3 pObj(radius * cp, radius * sp, z);
        const float hitRad = std::sqrt(Sqr(pObj.x) + Sqr(pObj.y));
        pObj.x *= radius / hitRad;
        pObj.y *= radius / hitRad;
        const V3 pObjError = gamma(3) * Abs(V3(pObj.x, pObj.y, 0));
        const P3i pi = {ItvFromValueAndError(pObj.x, pObjError.x), ItvFromValueAndError(pObj.y, pObjError.y),
                        ItvFromValueAndError(pObj.z, pObjError.z)};
        XfPointInexact(s.o2r, pi, &r.p, &r.pErr);
        V3 n = Normalize(XfNormal(s.r2o, V3(pObj.x, pObj.y, 0)));
        if (s.flags & 1) n = -n;
        r.n = n;
        r.uv[0] = phi / phiMax;
        r.uv[1] = (pObj.z - zMin) / (zMax - zMin);
    } else {
        const float height = s.a, radius = s.b;
        float dx, dy;
        SampleUniformDiskConcentric(u0, u1, &dx, &dy);
        const V3 pObj(dx * radius, dy * radius, height);
        const P3i pi = XfPointExact(s.o2r, pObj);
        r.p = V3(ItvMid(pi.x), ItvMid(pi.y), ItvMid(pi.z));
        r.pErr = V3(ItvErr(pi.x), ItvErr(pi.y), ItvErr(pi.z));
        V3 n = Normalize(XfNormal(s.r2o, V3(0, 0, 1)));
        if (s.flags & 1) n = -n;
        r.n = n;
        // Disk::Sample(u)'s (u, v) (shapes.h:517-522)
        float phi = ATan2f(dy, dx);
        if (phi < 0) phi += 2 * kPi;
        const float radiusSample = std::sqrt(Sqr(pObj.x) + Sqr(pObj.y));
        r.uv[0] = phi / s.d;
        r.uv[1] = (radius - radiusSample) / (radius - s.c);
    }
    r.pdf = 1 / ShapeArea(s);
    return r;
}
// Shape::Sample(ctx, u) (shapes.h:293-361 sphere cone sampling, :531-547 disk) with
// ctx = (p, pErr, n): false for {} (also a zero solid-angle pdf); the pdf in solid angle
PHD bool ShapeSampleSolidAngle(const DeviceShape &s, V3 cp, V3 cpErr, V3 cn, float u0, float u1, ShapeSamplePt *out,
                               const float *N = nullptr, V3 cns = V3(0, 0, 0)) {
    if (s.kind == kShapeBilinearT) {
        // BilinearPatch::Sample(ctx, u) (shapes.cpp:1257-1330)
        const PatchVerts P = PatchP(s);
        const V3 v00 = Normalize(P.p00 - cp), v10 = Normalize(P.p10 - cp);
        const V3 v01 = Normalize(P.p01 - cp), v11 = Normalize(P.p11 - cp);
        if (s.b == 0 || SphericalQuadArea(v00, v10, v11, v01) <= 1e-4f) {
            ShapeSamplePt ss;
            if (!BilinearSampleArea(s, N, u0, u1, &ss.p, &ss.pErr, &ss.n, &ss.pdf, ss.uv)) return false;
            V3 wi = ss.p - cp;
            if (LengthSquared(wi) == 0) return false;
            wi = Normalize(wi);
            ss.pdf /= AbsDotN(ss.n, -wi) / DistanceSquared(cp, ss.p);
            if (std::isinf(ss.pdf)) return false;
            *out = ss;
            return true;
        }
        float pdf = 1, uu = u0, vv = u1;
        if (cns.x != 0 || cns.y != 0 || cns.z != 0) {
            const float w[4] = {std::fmax(0.01f, AbsDotN(cns, v00)), std::fmax(0.01f, AbsDotN(cns, v10)),
                                std::fmax(0.01f, AbsDotN(cns, v01)), std::fmax(0.01f, AbsDotN(cns, v11))};
            SampleBilinear(u0, u1, w, &uu, &vv);
            pdf *= BilinearPDF(uu, vv, w);
        }
        const V3 eu = P.p10 - P.p00, ev = P.p01 - P.p00;
        float quadPDF;
        const V3 p = SampleSphericalRectangle(cp, P.p00, eu, ev, uu, vv, &quadPDF);
        pdf *= quadPDF;
        const float su = Dot(p - P.p00, eu) / DistanceSquared(P.p10, P.p00);
        const float sv = Dot(p - P.p00, ev) / DistanceSquared(P.p01, P.p00);
        out->n = PatchSampleNormal(s, N, Normalize(Cross(eu, ev)), su, sv);
        out->p = p;
        out->pErr = V3(0, 0, 0);
        out->pdf = pdf;
        PatchST(s, su, sv, out->uv);
        return true;
    }
    if (s.kind == kShapeSphereT) {
        const float radius = s.a;
        const V3 pCenter = XfPt(s.o2r, V3(0, 0, 0));
        const V3 pOrigin = OffsetRayOrigin(cp, cpErr, cn, pCenter - cp);
        if (!(DistanceSquared(pOrigin, pCenter) <= Sqr(radius))) {
            const float sinThetaMax = radius / Distance(cp, pCenter);
            const float sin2ThetaMax = Sqr(sinThetaMax);
            const float cosThetaMax = SafeSqrt(1 - sin2ThetaMax);
            float oneMinusCosThetaMax = 1 - cosThetaMax;
            float cosTheta = (cosThetaMax - 1) * u0 + 1;
            float sin2Theta = 1 - Sqr(cosTheta);
            if (sin2ThetaMax < 0.00068523f) {
                sin2Theta = sin2ThetaMax * u0;
                cosTheta = std::sqrt(1 - sin2Theta);
                oneMinusCosThetaMax = sin2ThetaMax / 2;
            }
            const float cosAlpha = sin2Theta / sinThetaMax + cosTheta * SafeSqrt(1 - sin2Theta / Sqr(sinThetaMax));
            const float sinAlpha = SafeSqrt(1 - Sqr(cosAlpha));
            const float phi = u1 * 2 * kPi;
            float sp, cpp;
            SinCosf(phi, &sp, &cpp);
            const float st = Clampf(sinAlpha, -1, 1);
            const V3 w(st * cpp, st * sp, Clampf(cosAlpha, -1, 1));
            V3 fx, fy;
            const V3 fz = Normalize(pCenter - cp);
            CoordinateSystem(fz, &fx, &fy);
            const V3 mw = -w;
            V3 n = fx * mw.x + fy * mw.y + fz * mw.z;
            const V3 p = pCenter + radius * V3(n.x, n.y, n.z);
            if (s.flags & 1) n = -n;
            ToPoint3fi(p, gamma(5) * Abs(p), &out->p, &out->pErr);  // Interaction(Point3fi(p, pError))
            out->n = n;
            out->pdf = 1 / (2 * kPi * oneMinusCosThetaMax);
            SphereUV(s, XfPt(s.r2o, p), out->uv);  // (*objectFromRender)(p)
            return true;
        }
    }
    ShapeSamplePt ss = ShapeSampleArea(s, u0, u1);
    V3 wi = ss.p - cp;
    if (LengthSquared(wi) == 0) return false;
    wi = Normalize(wi);
    ss.pdf /= AbsDotN(ss.n, -wi) / DistanceSquared(cp, ss.p);
    if (std::isinf(ss.pdf)) return false;
    *out = ss;
    return true;
}
// Shape::PDF(ctx, wi) (shapes.h:364-392 sphere, :550-564 disk): the ray ctx.SpawnRay(wi)
// against the shape alone where the cone formula does not apply
PHD float ShapePDFSolidAngle(const DeviceShape &s, V3 cp, V3 cpErr, V3 cn, V3 wi, const float *N = nullptr,
                             V3 cns = V3(0, 0, 0)) {
    if (s.kind == kShapeBilinearT) {
        // BilinearPatch::PDF(ctx, wi) (shapes.cpp:1332-1372)
        const V3 ro = OffsetRayOrigin(cp, cpErr, cn, wi);
        float th, iu, iv;
        if (!BilinearIntersect(s, ro, wi, kInfinity, &th, &iu, &iv)) return 0;
        const TriSurface si = BilinearSurface(s, N, iu, iv);
        const PatchVerts P = PatchP(s);
        const V3 v00 = Normalize(P.p00 - cp), v10 = Normalize(P.p10 - cp);
        const V3 v01 = Normalize(P.p01 - cp), v11 = Normalize(P.p11 - cp);
        if (s.b == 0 || SphericalQuadArea(v00, v10, v11, v01) <= 1e-4f) {
            // BilinearPatch::PDF(intr) (shapes.cpp:1219-1255) at the hit's (s, t)
            float uu = si.uv[0], vv = si.uv[1];
            if (s.flags & 4) InvertBilinearUV(s, si.uv[0], si.uv[1], &uu, &vv);
            float pdf = 1;
            if (s.b == 0) {
                float w[4];
                PatchAreaWeights(P, w);
                pdf = BilinearPDF(uu, vv, w);
            }
            const V3 pu0 = LerpV(vv, P.p00, P.p01), pu1 = LerpV(vv, P.p10, P.p11);
            const V3 dpdu = pu1 - pu0;
            const V3 dpdv = LerpV(uu, P.p01, P.p11) - LerpV(uu, P.p00, P.p10);
            pdf = pdf / Length(Cross(dpdu, dpdv));
            pdf = pdf * (DistanceSquared(cp, si.p) / AbsDotN(si.n, -wi));
            return std::isinf(pdf) ? 0.f : pdf;
        }
        const float pdf = 1 / SphericalQuadArea(v00, v10, v11, v01);
        if (cns.x != 0 || cns.y != 0 || cns.z != 0) {
            const float w[4] = {std::fmax(0.01f, AbsDotN(cns, v00)), std::fmax(0.01f, AbsDotN(cns, v10)),
                                std::fmax(0.01f, AbsDotN(cns, v01)), std::fmax(0.01f, AbsDotN(cns, v11))};
            float su, sv;
            InvertSphericalRectangleSample(cp, P.p00, P.p10 - P.p00, P.p01 - P.p00, si.p, &su, &sv);
            return BilinearPDF(su, sv, w) * pdf;
        }
        return pdf;
    }
    if (s.kind == kShapeSphereT) {
        const float radius = s.a;
        const V3 pCenter = XfPt(s.o2r, V3(0, 0, 0));
        const V3 pOrigin = OffsetRayOrigin(cp, cpErr, cn, pCenter - cp);
        if (!(DistanceSquared(pOrigin, pCenter) <= Sqr(radius))) {
            const float sin2ThetaMax = radius * radius / DistanceSquared(cp, pCenter);
            const float cosThetaMax = SafeSqrt(1 - sin2ThetaMax);
            float oneMinusCosThetaMax = 1 - cosThetaMax;
            if (sin2ThetaMax < 0.00068523f) oneMinusCosThetaMax = sin2ThetaMax / 2;
            return 1 / (2 * kPi * oneMinusCosThetaMax);
        }
    }
    const V3 ro = OffsetRayOrigin(cp, cpErr, cn, wi);
    float tHit;
    V3 pObj;
    if (!ShapeIntersect(s, ro, wi, kInfinity, &tHit, &pObj)) return 0;
    const TriSurface si = ShapeSurface(s, pObj);
    float pdf = (1 / ShapeArea(s)) / (AbsDotN(si.n, -wi) / DistanceSquared(cp, si.p));
    if (std::isinf(pdf)) pdf = 0;
    return pdf;
}
// Sphere / Disk::Bounds (shapes.cpp:33-40, 88-92): the transformed object box's 8 corners
PHD void ShapeBounds(const DeviceShape &s, V3 *lo, V3 *hi) {
    if (s.kind == kShapeBilinearT) {  // Union(Bounds3f(p00, p01), Bounds3f(p10, p11))
        const PatchVerts P = PatchP(s);
        *lo = V3(std::fmin(std::fmin(P.p00.x, P.p01.x), std::fmin(P.p10.x, P.p11.x)),
                 std::fmin(std::fmin(P.p00.y, P.p01.y), std::fmin(P.p10.y, P.p11.y)),
                 std::fmin(std::fmin(P.p00.z, P.p01.z), std::fmin(P.p10.z, P.p11.z)));
        *hi = V3(std::fmax(std::fmax(P.p00.x, P.p01.x), std::fmax(P.p10.x, P.p11.x)),
                 std::fmax(std::fmax(P.p00.y, P.p01.y), std::fmax(P.p10.y, P.p11.y)),
                 std::fmax(std::fmax(P.p00.z, P.p01.z), std::fmax(P.p10.z, P.p11.z)));
        return;
    }
    V3 a, b;
    if (s.kind == kShapeSphereT || s.kind == kShapeCylinderT) {  // (-r, -r, zMin), (r, r, zMax)
        a = V3(-s.a, -s.a, s.b);
        b = V3(s.a, s.a, s.c);
    } else {
        a = V3(-s.b, -s.b, s.a);
        b = V3(s.b, s.b, s.a);
    }
    *lo = V3(kInfinity, kInfinity, kInfinity);
    *hi = V3(-kInfinity, -kInfinity, -kInfinity);
    for (int i = 0; i < 8; ++i) {
        const V3 c((i & 1) ? b.x : a.x, (i & 2) ? b.y : a.y, (i & 4) ? b.z : a.z);
        const V3 q = XfPt(s.o2r, c);
        *lo = V3(std::fmin(lo->x, q.x), std::fmin(lo->y, q.y), std::fmin(lo->z, q.z));
        *hi = V3(std::fmax(hi->x, q.x), std::fmax(hi->y, q.y), std::fmax(hi->z, q.z));
    }
}

// SampleTent (util/sampling.h:196-201)
PHD float SampleTent(float u, float r) {
    float pmf;
    if (SampleDiscrete2(0.5f, 0.5f, u, &pmf, &u) == 0) return -r + r * SampleLinear(u, 0, 1);
    return r * SampleLinear(u, 1, 0);
}
// Filter::Sample(u) -> film offset p and weight (filters.h)
PHD void FilterSample(const FilterParams &f, const FilterTableView &tab, float u0, float u1, float *px, float *py,
                      float *weight) {
    if (f.type == kFilterBox) {
        *px = Lerpf(u0, -f.rx, f.rx);
        *py = Lerpf(u1, -f.ry, f.ry);
        *weight = 1.f;
        return;
    }
    if (f.type == kFilterTriangle) {
        *px = SampleTent(u0, f.rx);
        *py = SampleTent(u1, f.ry);
        *weight = 1.f;
        return;
    }
    // PiecewiseConstant2D::Sample (util/sampling.h:761-772): marginal in y, conditional in x
    float pdf1, pdf0;
    int v, u;
    const float *margFunc = tab.CondInt();  // |integral| of each row (all >= 0)
    const float d1 = SamplePC1D(margFunc, tab.MargCdf(), tab.nv, tab.MargInt(), -f.ry, f.ry, u1, &pdf1, &v);
    const float d0 = SamplePC1D(tab.Func() + v * tab.nu, tab.CondCdf() + v * (tab.nu + 1), tab.nu, tab.CondInt()[v],
                                -f.rx, f.rx, u0, &pdf0, &u);
    *px = d0;
    *py = d1;
    *weight = tab.F()[v * tab.nu + u] / (pdf0 * pdf1);
}

// ---------------------------------------------------------------- diffuse transmission
// DiffuseTransmissionBxDF (bxdfs.h:218-296): Lambertian reflection R and transmission T; the
// lobe is chosen by the largest R and T values (pr, pt).  sp.R(i) = R_i, sp.EtaK(i, ...) unused,
// sp.T(i) = T_i.
template <typename Spec>
struct DiffuseTransmission {
    const Spec &sp;
    float pr, pt;  // R.MaxComponentValue(), T.MaxComponentValue()
    PHD int Flags() const {
        return (pr > 0 ? (kBxReflection | kBxDiffuse) : 0) | (pt > 0 ? (kBxTransmission | kBxDiffuse) : 0);
    }
    PHD void f(V3 wo, V3 wi, float fo[kNSpectrumSamples]) const {
        const bool same = SameHemisphere(wo, wi);
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] = (same ? sp.R(i) : sp.T(i)) * kInvPi;
    }
    PHD float PDF(V3 wo, V3 wi) const {
        if (pr == 0 && pt == 0) return 0;
        if (SameHemisphere(wo, wi)) return pr / (pr + pt) * CosineHemispherePDF(AbsCosTheta(wi));
        return pt / (pr + pt) * CosineHemispherePDF(AbsCosTheta(wi));
    }
    PHD bool Sample_f(V3 wo, float uc, float u0, float u1, V3 *wi, float *pdf, int *flags,
                      float fo[kNSpectrumSamples]) const {
        if (pr == 0 && pt == 0) return false;
        V3 w = SampleCosineHemisphere(u0, u1);
        if (uc < pr / (pr + pt)) {
            if (wo.z < 0) w.z *= -1;
            *pdf = CosineHemispherePDF(AbsCosTheta(w)) * pr / (pr + pt);
            *flags = kBxReflection | kBxDiffuse;
        } else {
            if (wo.z > 0) w.z *= -1;
            *pdf = CosineHemispherePDF(AbsCosTheta(w)) * pt / (pr + pt);
            *flags = kBxTransmission | kBxDiffuse;
        }
        *wi = w;
        f(wo, w, fo);
        return true;
    }
};

// ---------------------------------------------------------------- layered BxDFs
// LayeredBxDF<DielectricBxDF, DiffuseBxDF | ConductorBxDF, twoSided = true> (bxdfs.h:565-1052):
// CoatedDiffuseBxDF / CoatedConductorBxDF.  f, Sample_f and PDF are stochastic estimates from a
// random walk between the two interfaces with an RNG seeded from the directions
// (Hash(GetOptions().seed, wo), Hash(wi) ...).  Two pairs of draws the reference writes as
// Point2f(r(), r()) (unspecified argument order in C++) are taken left to right here.
// Spectra are 31-wide (the bottom's per-wavelength values and the albedo come from `sp`):
//   sp.R(i)            diffuse reflectance (clamped) at lambda_i
//   sp.EtaK(i, &e, &k) conductor eta, k at lambda_i
//   sp.Albedo(i)       layer albedo at lambda_i
struct LayerSample {
    bool ok;
    V3 wi;
    float pdf;
    int flags;
    bool pdfIsProportional;
};
PHD float PowerHeuristic(float nf, float fPdf, float ng, float gPdf) {  // util/sampling.h
    const float f = nf * fPdf, g = ng * gPdf;
    if (std::isinf(Sqr(f))) return 1;
    return Sqr(f) / (Sqr(f) + Sqr(g));
}
PHD uint64_t HashIntV3(int a, V3 v) {
    const uint32_t w[4] = {(uint32_t)a, FloatToBits(v.x), FloatToBits(v.y), FloatToBits(v.z)};
    return HashWords(w, 4);
}
PHD uint64_t HashF3(float a, float b, float c) {
    const uint32_t w[3] = {FloatToBits(a), FloatToBits(b), FloatToBits(c)};
    return HashWords(w, 3);
}

template <typename Spec>
struct LayeredBxDF {
    // top: DielectricBxDF(eta, trTop); bottom: diffuse (conductor = false) or ConductorBxDF(trBot)
    float eta;
    TrowbridgeReitz trTop, trBot;
    bool conductor;
    float thickness, g;
    bool albedoNz;
    int maxDepth, nSamples, seed;
    const Spec &sp;
    bool bottomNz;  // diffuse: R != 0 at some wavelength (its Flags() is Unset otherwise)

    PHD static float Tr(float dz, V3 w) {
        if (std::fabs(dz) <= 1.17549435e-38f) return 1;
        return FastExp(-std::fabs(dz / w.z));
    }
    // ---- interfaces (iface 0 = top dielectric, 1 = bottom)
    PHD int Flags(int iface) const {
        if (iface == 0) return DielectricFlags(eta, trTop);
        if (conductor) return kBxReflection | (trBot.EffectivelySmooth() ? kBxSpecular : kBxGlossy);
        return bottomNz ? (kBxReflection | kBxDiffuse) : 0;
    }
    PHD bool IsSpecularI(int iface) const { return Flags(iface) & kBxSpecular; }
    // f of an interface: the top's is a scalar (ft[0] only, isScalar = true)
    PHD void F(int iface, V3 wo, V3 wi, bool radiance, float out[kNSpectrumSamples], bool *isScalar) const {
        if (iface == 0) {
            out[0] = DielectricEval(eta, trTop, wo, wi, nullptr, radiance);
            *isScalar = true;
            return;
        }
        *isScalar = false;
        if (!conductor) {
            const bool same = SameHemisphere(wo, wi);
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) out[i] = same ? sp.R(i) * kInvPi : 0.f;
            return;
        }
        const ConductorTerms ct = ConductorEval(trBot, wo, wi);
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) {
            float e, k;
            sp.EtaK(i, &e, &k);
            out[i] = ct.ok ? ConductorF(ct, e, k) : 0.f;
        }
    }
    PHD float Pdf(int iface, V3 wo, V3 wi, bool radiance, int flags) const {
        if (iface == 0) {
            float pdf;
            DielectricEval(eta, trTop, wo, wi, &pdf, radiance, flags);
            return pdf;
        }
        if (!(flags & kSampleR) || !SameHemisphere(wo, wi)) return 0;
        if (!conductor) return CosineHemispherePDF(std::fabs(wi.z));
        if (trBot.EffectivelySmooth()) return 0;
        return ConductorEval(trBot, wo, wi).pdf;
    }
    // Sample_f of an interface; f into out (scalar for the top).  True when the sample exists
    // with f != 0 and pdf > 0 (callers add the wi.z != 0 test where the reference has it).
    PHD bool Sample(int iface, V3 wo, float uc, float u0, float u1, bool radiance, int flags, BxSample *bs,
                    float out[kNSpectrumSamples], bool *isScalar) const {
        if (iface == 0) {
            *bs = DielectricSample(eta, trTop, wo, uc, u0, u1, radiance, flags);
            out[0] = bs->f;
            *isScalar = true;
            return bs->ok && bs->f != 0 && bs->pdf > 0;
        }
        *isScalar = false;
        if (!(flags & kSampleR)) return false;
        if (!conductor) {
            if (!bottomNz) return false;
            V3 wi = SampleCosineHemisphere(u0, u1);
            if (wo.z < 0) wi.z *= -1;
            const float pdf = CosineHemispherePDF(std::fabs(wi.z));
            *bs = BxSample{true, wi, 0, pdf, 1, kBxReflection | kBxDiffuse};
            bool nz = false;
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) {
                out[i] = sp.R(i) * kInvPi;
                nz |= out[i] != 0;
            }
            return nz && pdf > 0;
        }
        const ConductorTerms ct = ConductorSample(trBot, wo, u0, u1);
        if (!ct.ok) return false;
        *bs = BxSample{true, ct.wi, 0, ct.pdf, 1, kBxReflection | (ct.specular ? kBxSpecular : kBxGlossy)};
        bool nz = false;
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) {
            float e, k;
            sp.EtaK(i, &e, &k);
            out[i] = ConductorF(ct, e, k);
            nz |= out[i] != 0;
        }
        return nz && ct.pdf > 0;
    }
    PHD int LayerFlags() const {  // LayeredBxDF::Flags
        const int t = Flags(0), b = Flags(1);
        int flags = kBxReflection;
        if (t & kBxSpecular) flags |= kBxSpecular;
        if ((t & kBxDiffuse) || (b & kBxDiffuse) || albedoNz) flags |= kBxDiffuse;
        else if ((t & kBxGlossy) || (b & kBxGlossy)) flags |= kBxGlossy;
        if ((t & kBxTransmission) && (b & kBxTransmission)) flags |= kBxTransmission;
        return flags;
    }

    // LayeredBxDF::f (bxdfs.h:611-781)
    PHD void f(V3 wo, V3 wi, bool radiance, float fo[kNSpectrumSamples]) const {
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] = 0;
        if (wo.z < 0) {  // twoSided
            wo = -wo;
            wi = -wi;
        }
        const bool enteredTop = true;
        const int enter = 0;
        const bool exitBottom = SameHemisphere(wo, wi) ^ enteredTop;
        const int exitI = exitBottom ? 1 : 0, nonExitI = exitBottom ? 0 : 1;
        const float exitZ = exitBottom ? 0 : thickness;
        float tmp[kNSpectrumSamples];
        bool sc;
        if (SameHemisphere(wo, wi)) {
            F(enter, wo, wi, radiance, tmp, &sc);
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] = nSamples * (sc ? tmp[0] : tmp[i]);
        }
        PCG32 rng(HashIntV3(seed, wo), HashV3(wi));
        float beta[kNSpectrumSamples], wisF[kNSpectrumSamples];
        for (int s = 0; s < nSamples; ++s) {
            BxSample wos, wis;
            float uc = rng.Uniform(), a0 = rng.Uniform(), a1 = rng.Uniform();
            if (!Sample(enter, wo, uc, a0, a1, radiance, kSampleT, &wos, tmp, &sc) || wos.wi.z == 0) continue;
            uc = rng.Uniform();
            a0 = rng.Uniform();
            a1 = rng.Uniform();
            bool wisSc;
            if (!Sample(exitI, wi, uc, a0, a1, !radiance, kSampleT, &wis, wisF, &wisSc) || wis.wi.z == 0) continue;
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) beta[i] = (sc ? tmp[0] : tmp[i]) * AbsCosTheta(wos.wi) / wos.pdf;
            float z = enteredTop ? thickness : 0;
            V3 w = wos.wi;
            for (int depth = 0; depth < maxDepth; ++depth) {
                if (depth > 3) {
                    float mx = beta[0];
                    PHD_UNROLL
                    for (int i = 1; i < kNSpectrumSamples; ++i) mx = std::fmax(mx, beta[i]);
                    if (mx < 0.25f) {
                        const float q = std::fmax(0.f, 1 - mx);
                        if (rng.Uniform() < q) break;
                        PHD_UNROLL
                        for (int i = 0; i < kNSpectrumSamples; ++i) beta[i] /= 1 - q;
                    }
                }
                if (!albedoNz) {
                    z = (z == thickness) ? 0 : thickness;
                    const float tr = Tr(thickness, w);
                    PHD_UNROLL
                    for (int i = 0; i < kNSpectrumSamples; ++i) beta[i] *= tr;
                } else {
                    const float sigma_t = 1;
                    const float dz = SampleExponential(rng.Uniform(), sigma_t / std::fabs(w.z));
                    const float zp = w.z > 0 ? (z + dz) : (z - dz);
                    if (z == zp) continue;
                    if (0 < zp && zp < thickness) {
                        // scattering in the layer medium: NEE through the exit interface along wis
                        float wt = 1;
                        if (!IsSpecularI(exitI)) wt = PowerHeuristic(1, wis.pdf, 1, HenyeyGreenstein(Dot(-w, -wis.wi), g));
                        const float ph = HenyeyGreenstein(Dot(-w, -wis.wi), g);
                        const float trw = Tr(zp - exitZ, wis.wi);
                        PHD_UNROLL
                        for (int i = 0; i < kNSpectrumSamples; ++i)
                            fo[i] += beta[i] * sp.Albedo(i) * ph * wt * trw * (wisSc ? wisF[0] : wisF[i]) / wis.pdf;
                        const float p0 = rng.Uniform(), p1 = rng.Uniform();
                        float ppdf;
                        const V3 pwi = SampleHenyeyGreenstein(-w, g, p0, p1, &ppdf);
                        if (ppdf == 0 || pwi.z == 0) continue;
                        PHD_UNROLL
                        for (int i = 0; i < kNSpectrumSamples; ++i) beta[i] *= sp.Albedo(i) * ppdf / ppdf;
                        w = pwi;
                        z = zp;
                        if (((z < exitZ && w.z > 0) || (z > exitZ && w.z < 0)) && !IsSpecularI(exitI)) {
                            bool fsc;
                            F(exitI, -w, wi, radiance, tmp, &fsc);
                            bool fnz = false;
                            PHD_UNROLL
                            for (int i = 0; i < kNSpectrumSamples; ++i) fnz |= (fsc ? tmp[0] : tmp[i]) != 0;
                            if (fnz) {
                                const float exitPDF = Pdf(exitI, -w, wi, radiance, kSampleT);
                                const float wt2 = PowerHeuristic(1, ppdf, 1, exitPDF);
                                const float tr2 = Tr(zp - exitZ, pwi);
                                PHD_UNROLL
                                for (int i = 0; i < kNSpectrumSamples; ++i)
                                    fo[i] += beta[i] * tr2 * (fsc ? tmp[0] : tmp[i]) * wt2;
                            }
                        }
                        continue;
                    }
                    z = Clampf(zp, 0, thickness);
                }
                if (z == exitZ) {
                    BxSample bs;
                    const float c = rng.Uniform(), b0 = rng.Uniform(), b1 = rng.Uniform();
                    bool bsc;
                    if (!Sample(exitI, -w, c, b0, b1, radiance, kSampleR, &bs, tmp, &bsc) || bs.wi.z == 0) break;
                    PHD_UNROLL
                    for (int i = 0; i < kNSpectrumSamples; ++i)
                        beta[i] *= (bsc ? tmp[0] : tmp[i]) * AbsCosTheta(bs.wi) / bs.pdf;
                    w = bs.wi;
                } else {
                    if (!IsSpecularI(nonExitI)) {
                        float wt = 1;
                        if (!IsSpecularI(exitI)) wt = PowerHeuristic(1, wis.pdf, 1, Pdf(nonExitI, -w, -wis.wi, radiance, kSampleAll));
                        bool nsc;
                        F(nonExitI, -w, -wis.wi, radiance, tmp, &nsc);
                        const float trw = Tr(thickness, wis.wi);
                        PHD_UNROLL
                        for (int i = 0; i < kNSpectrumSamples; ++i)
                            fo[i] += beta[i] * (nsc ? tmp[0] : tmp[i]) * AbsCosTheta(wis.wi) * wt * trw *
                                     (wisSc ? wisF[0] : wisF[i]) / wis.pdf;
                    }
                    BxSample bs;
                    const float c = rng.Uniform(), b0 = rng.Uniform(), b1 = rng.Uniform();
                    bool bsc;
                    if (!Sample(nonExitI, -w, c, b0, b1, radiance, kSampleR, &bs, tmp, &bsc) || bs.wi.z == 0) break;
                    PHD_UNROLL
                    for (int i = 0; i < kNSpectrumSamples; ++i)
                        beta[i] *= (bsc ? tmp[0] : tmp[i]) * AbsCosTheta(bs.wi) / bs.pdf;
                    w = bs.wi;
                    if (!IsSpecularI(exitI)) {
                        bool fsc;
                        F(exitI, -w, wi, radiance, tmp, &fsc);
                        bool fnz = false;
                        PHD_UNROLL
                        for (int i = 0; i < kNSpectrumSamples; ++i) fnz |= (fsc ? tmp[0] : tmp[i]) != 0;
                        if (fnz) {
                            float wt = 1;
                            if (!IsSpecularI(nonExitI)) {
                                const float exitPDF = Pdf(exitI, -w, wi, radiance, kSampleT);
                                wt = PowerHeuristic(1, bs.pdf, 1, exitPDF);
                            }
                            const float tr2 = Tr(thickness, bs.wi);
                            PHD_UNROLL
                            for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] += beta[i] * tr2 * (fsc ? tmp[0] : tmp[i]) * wt;
                        }
                    }
                }
            }
        }
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] /= nSamples;
    }

    // LayeredBxDF::Sample_f (bxdfs.h:783-911): f into fo, wi / pdf / flags in the result
    PHD LayerSample Sample_f(V3 wo, float uc, float u0, float u1, bool radiance, float fo[kNSpectrumSamples]) const {
        LayerSample res{false, V3(0, 0, 0), 0, 0, false};
        bool flipWi = false;
        if (wo.z < 0) {
            wo = -wo;
            flipWi = true;
        }
        BxSample bs;
        bool sc;
        float tmp[kNSpectrumSamples];
        if (!Sample(0, wo, uc, u0, u1, radiance, kSampleAll, &bs, tmp, &sc) || bs.wi.z == 0) return res;
        if (bs.flags & kBxReflection) {
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] = sc ? tmp[0] : tmp[i];
            res = LayerSample{true, flipWi ? -bs.wi : bs.wi, bs.pdf, bs.flags, true};
            return res;
        }
        V3 w = bs.wi;
        bool specularPath = bs.flags & kBxSpecular;
        PCG32 rng(HashIntV3(seed, wo), HashF3(uc, u0, u1));
        PHD_UNROLL
        for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] = (sc ? tmp[0] : tmp[i]) * AbsCosTheta(bs.wi);
        float pdf = bs.pdf;
        float z = thickness;
        for (int depth = 0; depth < maxDepth; ++depth) {
            float mx = fo[0];
            PHD_UNROLL
            for (int i = 1; i < kNSpectrumSamples; ++i) mx = std::fmax(mx, fo[i]);
            const float rrBeta = mx / pdf;
            if (depth > 3 && rrBeta < 0.25f) {
                const float q = std::fmax(0.f, 1 - rrBeta);
                if (rng.Uniform() < q) return res;
                pdf *= 1 - q;
            }
            if (w.z == 0) return res;
            if (albedoNz) {
                const float sigma_t = 1;
                const float dz = SampleExponential(rng.Uniform(), sigma_t / AbsCosTheta(w));
                const float zp = w.z > 0 ? (z + dz) : (z - dz);
                if (zp == z) return res;
                if (0 < zp && zp < thickness) {
                    const float p0 = rng.Uniform(), p1 = rng.Uniform();
                    float ppdf;
                    const V3 pwi = SampleHenyeyGreenstein(-w, g, p0, p1, &ppdf);
                    if (ppdf == 0 || pwi.z == 0) return res;
                    PHD_UNROLL
                    for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] *= sp.Albedo(i) * ppdf;
                    pdf *= ppdf;
                    specularPath = false;
                    w = pwi;
                    z = zp;
                    continue;
                }
                z = Clampf(zp, 0, thickness);
            } else {
                z = (z == thickness) ? 0 : thickness;
                const float tr = Tr(thickness, w);
                PHD_UNROLL
                for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] *= tr;
            }
            const int iface = z == 0 ? 1 : 0;
            const float c = rng.Uniform(), b0 = rng.Uniform(), b1 = rng.Uniform();
            BxSample is;
            bool isc;
            if (!Sample(iface, -w, c, b0, b1, radiance, kSampleAll, &is, tmp, &isc) || is.wi.z == 0) return res;
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] *= isc ? tmp[0] : tmp[i];
            pdf *= is.pdf;
            specularPath &= (is.flags & kBxSpecular) != 0;
            w = is.wi;
            if (is.flags & kBxTransmission) {
                int flags = SameHemisphere(wo, w) ? kBxReflection : kBxTransmission;
                flags |= specularPath ? kBxSpecular : kBxGlossy;
                res = LayerSample{true, flipWi ? -w : w, pdf, flags, true};
                return res;
            }
            const float ci = AbsCosTheta(is.wi);
            PHD_UNROLL
            for (int i = 0; i < kNSpectrumSamples; ++i) fo[i] *= ci;
        }
        return res;
    }

    // LayeredBxDF::PDF (bxdfs.h:913-1016)
    PHD float PDF(V3 wo, V3 wi, bool radiance) const {
        if (wo.z < 0) {
            wo = -wo;
            wi = -wi;
        }
        PCG32 rng(HashIntV3(seed, wi), HashV3(wo));
        const bool enteredTop = true;
        float pdfSum = 0;
        if (SameHemisphere(wo, wi)) pdfSum += nSamples * Pdf(0, wo, wi, radiance, kSampleR);
        float tmp[kNSpectrumSamples];
        bool sc;
        for (int s = 0; s < nSamples; ++s) {
            if (SameHemisphere(wo, wi)) {
                const int rI = enteredTop ? 1 : 0, tI = enteredTop ? 0 : 1;
                BxSample wos, wis;
                float c = rng.Uniform(), a0 = rng.Uniform(), a1 = rng.Uniform();
                const bool goodO = Sample(tI, wo, c, a0, a1, radiance, kSampleT, &wos, tmp, &sc);
                c = rng.Uniform();
                a0 = rng.Uniform();
                a1 = rng.Uniform();
                const bool goodI = Sample(tI, wi, c, a0, a1, !radiance, kSampleT, &wis, tmp, &sc);
                if (goodO && goodI) {
                    if (!(Flags(tI) & (kBxDiffuse | kBxGlossy))) {
                        pdfSum += Pdf(rI, -wos.wi, -wis.wi, radiance, kSampleAll);
                    } else {
                        BxSample rs;
                        c = rng.Uniform();
                        a0 = rng.Uniform();
                        a1 = rng.Uniform();
                        if (Sample(rI, -wos.wi, c, a0, a1, radiance, kSampleAll, &rs, tmp, &sc)) {
                            if (!(Flags(rI) & (kBxDiffuse | kBxGlossy))) {
                                pdfSum += Pdf(tI, -rs.wi, wi, radiance, kSampleAll);
                            } else {
                                const float rPDF = Pdf(rI, -wos.wi, -wis.wi, radiance, kSampleAll);
                                float wt = PowerHeuristic(1, wis.pdf, 1, rPDF);
                                pdfSum += wt * rPDF;
                                const float tPDF = Pdf(tI, -rs.wi, wi, radiance, kSampleAll);
                                wt = PowerHeuristic(1, rs.pdf, 1, tPDF);
                                pdfSum += wt * tPDF;
                            }
                        }
                    }
                }
            } else {
                // TT term: the opaque bottom never transmits, so every sample is rejected
                const int toI = enteredTop ? 0 : 1, tiI = enteredTop ? 1 : 0;
                BxSample wos, wis;
                float c = rng.Uniform(), a0 = rng.Uniform(), a1 = rng.Uniform();
                if (!Sample(toI, wo, c, a0, a1, radiance, kSampleAll, &wos, tmp, &sc) || wos.wi.z == 0 ||
                    (wos.flags & kBxReflection))
                    continue;
                c = rng.Uniform();
                a0 = rng.Uniform();
                a1 = rng.Uniform();
                if (!Sample(tiI, wi, c, a0, a1, !radiance, kSampleAll, &wis, tmp, &sc) || wis.wi.z == 0 ||
                    (wis.flags & kBxReflection))
                    continue;
                if (Flags(toI) & kBxSpecular) pdfSum += Pdf(tiI, -wos.wi, wi, radiance, kSampleAll);
                else if (Flags(tiI) & kBxSpecular) pdfSum += Pdf(toI, wo, -wis.wi, radiance, kSampleAll);
                else pdfSum += (Pdf(toI, wo, -wis.wi, radiance, kSampleAll) + Pdf(tiI, -wos.wi, wi, radiance, kSampleAll)) / 2;
            }
        }
        return Lerpf(0.9f, 1 / (4 * kPi), pdfSum / nSamples);
    }
};

}  // namespace pbrt_amd
