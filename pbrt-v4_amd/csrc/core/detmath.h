// Portable transcendentals for the device kernels: sin, cos, asin, acos, atan2 and log built
// only from IEEE-754 operations that every conforming implementation rounds the same way
// (+ - * /, fma, sqrt, rint, float <-> int conversion, bit manipulation).  Compiled with
// -ffp-contract=off, the GPU and any CPU produce the same bits for the same input, so the CPU
// oracle (oracle.cpp, its "device math" mode restates these polynomials) follows a device path
// decision for decision: an RNG seeded from a ray's bits (media, wavefront/media.cpp:44), an alpha
// test hashing the ray (gpu/optix.cu:197-243), a mix choice hashing the hit (materials.h:285-294).
//
// The polynomials are the classic minimax fits of the Cephes single-precision library (public
// domain: sinf.c, cosf.c, asinf.c, atanf.c, logf.c) on the reduced ranges below; accuracy
// against the correctly rounded result is within 2 ulp over the float range (host-tested in
// tests/test_det_math.py).  pbrt itself calls libm (CPU) or CUDA's sinf etc. (GPU), which differ
// from the correctly rounded values by an ulp or two in the same way.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#ifndef PHD
#if defined(__HIPCC__)
#define PHD __host__ __device__ inline
#else
#define PHD inline
#endif
#endif

namespace pbrt_amd {
namespace detm {

PHD uint32_t Bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
PHD float FromBits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// pi/2 as a float triple (hi + mid + lo agree with pi/2 to 2^-76) and its reciprocal
constexpr float kRedHi = 0x1.921fb6p+0f, kRedMid = -0x1.777a5cp-25f, kRedLo = -0x1.ee59dap-50f;
constexpr float kTwoOverPi = 0x1.45f306p-1f;
constexpr double kPio2HiD = 0x1.921fb54442d18p+0, kPio2LoD = 0x1.1a62633145c07p-54;
constexpr float kPiF = 0x1.921fb6p+1f, kPio2F = 0x1.921fb6p+0f, kPio4F = 0x1.921fb6p-1f;
// the float constants' remainders: pi = kPiF + kPiLo to 2^-50
constexpr float kPiLo = -0x1.777a5cp-24f, kPio2Lo = -0x1.777a5cp-25f, kPio4Lo = -0x1.777a5cp-26f;

// x = q (pi/2) + r, |r| <= ~pi/4; returns q mod 4.  Cody-Waite with fma for |x| <= 8192, the same
// in double beyond (both exact operation sequences, so every platform agrees).
PHD int ReduceHalfPi(float x, float *r) {
    if (std::fabs(x) <= 8192.f) {
        const float q = rintf(x * kTwoOverPi);
        float t = fmaf(-q, kRedHi, x);
        t = fmaf(-q, kRedMid, t);
        t = fmaf(-q, kRedLo, t);
        *r = t;
        return (int)q & 3;
    }
    const double xd = (double)x;
    const double q = rint(xd * 0.63661977236758134308);
    double t = fma(-q, kPio2HiD, xd);
    t = fma(-q, kPio2LoD, t);
    *r = (float)t;
    return (int)(int64_t)q & 3;
}
// sin and cos on [-pi/4, pi/4] (Cephes sinf / cosf coefficients)
PHD float SinPoly(float r) {
    const float z = r * r;
    float p = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
    p = fmaf(z, p, -1.6666654611e-1f);
    return fmaf(r * z, p, r);
}
PHD float CosPoly(float r) {
    const float z = r * r;
    float p = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
    p = fmaf(z, p, 4.166664568298827e-2f);
    return fmaf(z * z, p, fmaf(-0.5f, z, 1.f));
}
PHD void SinCos(float x, float *s, float *c) {
    if (!(std::fabs(x) <= 3.0e38f)) {  // inf, NaN
        *s = *c = x - x;
        return;
    }
    if (x == 0.f) {  // keeps sin(-0) = -0
        *s = x;
        *c = 1.f;
        return;
    }
    float r;
    const int q = ReduceHalfPi(x, &r);
    const float sp = SinPoly(r), cp = CosPoly(r);
    switch (q) {
    case 0: *s = sp, *c = cp; break;
    case 1: *s = cp, *c = -sp; break;
    case 2: *s = -sp, *c = -cp; break;
    default: *s = -cp, *c = sp; break;
    }
}
PHD float Sin(float x) {
    float s, c;
    SinCos(x, &s, &c);
    return s;
}
PHD float Cos(float x) {
    float s, c;
    SinCos(x, &s, &c);
    return c;
}

// asin on [0, 0.5] in z = x^2 (Cephes asinf), and the half-angle form above 0.5
PHD float ASinPoly(float z, float s) {
    float p = fmaf(z, 4.2163199048e-2f, 2.4181311049e-2f);
    p = fmaf(z, p, 4.5470025998e-2f);
    p = fmaf(z, p, 7.4953002686e-2f);
    p = fmaf(z, p, 1.6666752422e-1f);
    return fmaf(z * s, p, s);
}
PHD float ASin(float x) {
    const float a = std::fabs(x);
    if (!(a <= 1.f)) return (x - x) / (x - x);  // NaN
    float r;
    if (a > 0.5f) {
        const float z = 0.5f * (1.f - a);
        r = kPio2F + (kPio2Lo - 2.f * ASinPoly(z, std::sqrt(z)));
    } else {
        r = ASinPoly(a * a, a);
    }
    return x < 0 ? -r : r;
}
PHD float ACos(float x) {
    if (!(std::fabs(x) <= 1.f)) return (x - x) / (x - x);
    if (x < -0.5f) {
        const float z = 0.5f * (1.f + x);
        return kPiF + (kPiLo - 2.f * ASinPoly(z, std::sqrt(z)));
    }
    if (x > 0.5f) {
        const float z = 0.5f * (1.f - x);
        return 2.f * ASinPoly(z, std::sqrt(z));
    }
    return kPio2F + (kPio2Lo - ASinPoly(x * x, x));
}

// atan on [0, 1] (Cephes atanf: the polynomial below tan(pi/8), pi/4 + atan((t-1)/(t+1)) above)
PHD float ATanUnit(float t) {
    const bool shift = t > 0.4142135623730950f;
    if (shift) t = (t - 1.f) / (t + 1.f);
    const float z = t * t;
    float p = fmaf(z, 8.05374449538e-2f, -1.38776856032e-1f);
    p = fmaf(z, p, 1.99777106478e-1f);
    p = fmaf(z, p, -3.33329491539e-1f);
    const float a = fmaf(z * t, p, t);
    return shift ? kPio4F + (kPio4Lo + a) : a;
}
PHD float ATan2(float y, float x) {
    if (x != x || y != y) return x + y;
    const float ax = std::fabs(x), ay = std::fabs(y);
    const bool yneg = (Bits(y) >> 31) != 0, xneg = (Bits(x) >> 31) != 0;
    float a;
    if (ay == 0.f) {
        a = xneg ? kPiF : 0.f;  // atan2(+-0, -x or -0) = +-pi, atan2(+-0, +x or +0) = +-0
    } else if (ax == 0.f) {
        a = kPio2F;
    } else if (std::isinf(ax) || std::isinf(ay)) {
        a = std::isinf(ax) && std::isinf(ay) ? (xneg ? 3.f * kPio4F : kPio4F)
            : std::isinf(ax)                 ? (xneg ? kPiF : 0.f)
                                             : kPio2F;
    } else {
        // atan(min / max) on [0, 1], reflected about pi/4 and into the left half-plane
        const bool swap = ay > ax;
        a = ATanUnit(swap ? ax / ay : ay / ax);
        if (swap) a = kPio2F + (kPio2Lo - a);
        if (xneg) a = kPiF + (kPiLo - a);
    }
    return yneg ? -a : a;
}

// natural log (Cephes logf): x = 2^e m, m in [sqrt(1/2), sqrt(2)), polynomial in m - 1
PHD float Log(float x) {
    if (x != x || x < 0.f) return (x - x) / (x - x);
    if (x == 0.f) return -__builtin_huge_valf();
    if (std::isinf(x)) return x;
    uint32_t u = Bits(x);
    int e;
    if ((u >> 23) == 0) {  // subnormal: scale into the normal range first
        u = Bits(x * 0x1p25f);
        e = (int)(u >> 23) - 126 - 25;
    } else {
        e = (int)(u >> 23) - 126;
    }
    float m = FromBits((u & 0x007fffffu) | 0x3f000000u);  // [0.5, 1)
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = m + m - 1.f;
    } else {
        m = m - 1.f;
    }
    const float z = m * m;
    float p = fmaf(m, 7.0376836292e-2f, -1.1514610310e-1f);
    p = fmaf(m, p, 1.1676998740e-1f);
    p = fmaf(m, p, -1.2420140846e-1f);
    p = fmaf(m, p, 1.4249322787e-1f);
    p = fmaf(m, p, -1.6668057665e-1f);
    p = fmaf(m, p, 2.0000714765e-1f);
    p = fmaf(m, p, -2.4999993993e-1f);
    p = fmaf(m, p, 3.3333331174e-1f);
    float y = p * m * z;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    return fmaf(fe, 0.693359375f, m + y);
}

// e^x (Cephes expf): n = round(x log2 e), r = x - n ln 2 in two parts, a degree-5 polynomial,
// then 2^n as two exact-then-rounding scalings (subnormal results round once)
PHD float Exp(float x) {
    if (x != x) return x;
    if (x > 88.72283935546875f) return __builtin_huge_valf();
    if (x < -103.97208404541016f) return 0.f;
    const float n = std::floor(fmaf(x, 1.44269502162933349609f, 0.5f));
    float r = fmaf(n, -0.693359375f, x);
    r = fmaf(n, 2.12194440e-4f, r);
    float p = fmaf(r, 1.9875691500e-4f, 1.3981999507e-3f);
    p = fmaf(r, p, 8.3334519073e-3f);
    p = fmaf(r, p, 4.1665795894e-2f);
    p = fmaf(r, p, 1.6666665459e-1f);
    p = fmaf(r, p, 5.0000001201e-1f);
    const float y = fmaf(p, r * r, r) + 1.f;
    const int k = (int)n, k1 = k / 2, k2 = k - k1;
    return y * FromBits((uint32_t)(k1 + 127) << 23) * FromBits((uint32_t)(k2 + 127) << 23);
}
// tan x = sin x / cos x from one shared argument reduction (within a few ulp of tanf away from
// the poles; the portal light evaluates it on (-pi/2, pi/2))
PHD float Tan(float x) {
    float s, c;
    SinCos(x, &s, &c);
    return s / c;
}
// sinh x = (e^|x| - e^-|x|) / 2 with x's sign; x itself below 2^-12
PHD float Sinh(float x) {
    const float a = std::fabs(x);
    if (a < 0x1p-12f) return x;
    const float e = Exp(a);
    const float s = (e - 1.f / e) * 0.5f;
    return x < 0 ? -s : s;
}

}  // namespace detm
}  // namespace pbrt_amd
