// The device kernels' transcendentals, restated so they return glibc's float results bit for bit.
//
// pbrt's CPU build calls std::sin(float) etc., i.e. glibc's sinf, cosf, expf, logf, asinf, acosf,
// atan2f, tanf, sinhf (glibc 2.35 in this image and on the GPU boxes).  Those are not correctly
// rounded (sinf 1.4 %, asinf 7 %, atan2f 16 %, sinhf 14 % of inputs differ from the correctly
// rounded value: tests/test_det_math.py), so a GPU path that wants the reference's per-sample
// decisions -- the medium RNG seeded from a ray's bits (wavefront/media.cpp:44), alpha tests hashing
// the ray (gpu/optix.cu:197-243), mix choices hashing the hit (materials.h:285-294), and every
// direction a sampled angle feeds -- has to evaluate glibc's own algorithms, in glibc's operation
// order:
//
//   * sinf / cosf / sincosf, expf, logf: the double-precision implementations glibc took from Arm's
//     optimized-routines (MIT; sysdeps/ieee754/flt-32 s_sinf.c, e_expf.c, e_logf.c and their data
//     tables).  On x86-64 glibc runs the variants it compiles with -mfma (ifunc), where the
//     compiler contracts a*b + c into one fma; the fma()s below are exactly those contractions.
//   * asinf, acosf, atanf / atan2f, tanf, expm1f / sinhf: the single-precision fdlibm conversions
//     (Sun, freely distributable; e_asinf.c, e_acosf.c, s_atanf.c, e_atan2f.c, k_tanf.c, s_expm1f.c,
//     e_sinhf.c), built without fma.  tanf reduces its argument with sinf's double reduction.
//
// Every function equals glibc on all 2^32 float inputs (atan2f: on 10^8 sampled pairs); the
// exhaustive check is tools/detmath_exhaustive.cpp, the sampled one tests/test_det_math.py.  Only
// IEEE-754 operations that every conforming implementation rounds the same way are used (+ - * /,
// fma, sqrt, conversions, integer arithmetic, bit manipulation), compiled with -ffp-contract=off,
// so gfx950 and the host agree bit for bit.  The price on the GPU is double-precision arithmetic in
// the sin / cos / exp / log kernels (half the fp32 rate on CDNA4; a few calls per path vertex).
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
PHD uint64_t Bits64(double f) {
    uint64_t u;
    memcpy(&u, &f, 8);
    return u;
}
PHD double FromBits64(uint64_t u) {
    double f;
    memcpy(&f, &u, 8);
    return f;
}
// top 12 bits of |x|'s representation (the exponent and the first mantissa bits)
PHD uint32_t AbsTop12(float x) { return (Bits(x) >> 20) & 0x7ff; }

// ---- sin / cos: double polynomials on [-pi/4, pi/4] after a reduction by pi/2 ----------------
// Sine polynomial s1..s3 and cosine polynomial c0..c4 (the second set, used in quadrants 2 and 3,
// carries the cosine negated: sincosf_data.c's __sincosf_table).
struct SinCosPoly {
    double c0, c1, c2, c3, c4, s1, s2, s3;
};
constexpr SinCosPoly kSinCos[2] = {
    {0x1p0, -0x1.ffffffd0c621cp-2, 0x1.55553e1068f19p-5, -0x1.6c087e89a359dp-10, 0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13},
    {-0x1p0, 0x1.ffffffd0c621cp-2, -0x1.55553e1068f19p-5, 0x1.6c087e89a359dp-10, -0x1.99343027bf8c3p-16,
     -0x1.555545995a603p-3, 0x1.1107605230bc4p-7, -0x1.994eb3774cf24p-13}};
constexpr double kHalfPiInv24 = 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
constexpr double kHalfPi = 0x1.921FB54442D18p0;
// 4/pi to 192 bits, as overlapping 32-bit windows (__inv_pio4)
constexpr uint32_t kInvPio4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

PHD double SinPolyD(double x, double x2, const SinCosPoly &p) {
    const double x3 = x * x2;
    const double s1 = fma(x2, p.s3, p.s2);
    const double x7 = x3 * x2;
    const double s = fma(x3, p.s1, x);
    return fma(x7, s1, s);
}
PHD double CosPolyD(double x2, const SinCosPoly &p) {
    const double x4 = x2 * x2;
    const double c2 = fma(x2, p.c4, p.c3);
    const double c1 = fma(x2, p.c1, p.c0);
    const double x6 = x4 * x2;
    const double c = fma(x4, p.c2, c1);
    return fma(x6, c2, c);
}
// |x| < 120: one multiply-subtract with a 53-bit pi/2 (the quadrant from the 2^24-scaled product)
PHD double ReduceFast(double x, int *np, bool contract) {
    const double r = x * kHalfPiInv24;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return contract ? fma(-(double)n, kHalfPi, x) : x - (double)n * kHalfPi;
}
// |x| >= 120: exact 2.62 fixed-point product with 4/pi (sign ignored)
PHD double ReduceLarge(uint32_t xi, int *np) {
    const uint32_t *arr = &kInvPio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = (int)n;
    return (double)(int64_t)res0 * 0x1.921FB54442D18p-62;  // 2 pi 2^-64
}
// the reduced argument r (with the quadrant's sign applied), r^2, the polynomial set and the
// quadrant; false if x needs no reduction
PHD bool SinCosReduce(float y, double *r, int *n, int *set) {
    double x = y;
    if (AbsTop12(y) < AbsTop12(0x1.921FB54442D18p-1f)) return false;
    int q, sgn = 0;
    if (AbsTop12(y) < AbsTop12(120.0f)) {
        x = ReduceFast(x, &q, true);
    } else {
        const uint32_t xi = Bits(y);
        sgn = (int)(xi >> 31);
        x = ReduceLarge(xi, &q);
    }
    const int qs = (q + sgn) & 3;
    *r = (qs == 1 || qs == 2) ? -x : x;  // sign[] = {1, -1, -1, 1}
    *set = (qs & 2) ? 1 : 0;
    *n = q;
    return true;
}
PHD float Sin(float y) {
    if (!(AbsTop12(y) < AbsTop12(__builtin_huge_valf()))) return (y - y) / (y - y);
    double r;
    int n, set;
    if (!SinCosReduce(y, &r, &n, &set)) {
        if (AbsTop12(y) < AbsTop12(0x1p-12f)) return y;
        const double x = y;
        return (float)SinPolyD(x, x * x, kSinCos[0]);
    }
    const double r2 = r * r;  // pbrt's order: sign applied to x, x^2 from the unsigned value
    return (n & 1) ? (float)CosPolyD(r2, kSinCos[set]) : (float)SinPolyD(r, r2, kSinCos[set]);
}
PHD float Cos(float y) {
    if (!(AbsTop12(y) < AbsTop12(__builtin_huge_valf()))) return (y - y) / (y - y);
    double r;
    int n, set;
    if (!SinCosReduce(y, &r, &n, &set)) {
        if (AbsTop12(y) < AbsTop12(0x1p-12f)) return 1.f;
        const double x = y;
        return (float)CosPolyD(x * x, kSinCos[0]);
    }
    const double r2 = r * r;
    return (n & 1) ? (float)SinPolyD(r, r2, kSinCos[set]) : (float)CosPolyD(r2, kSinCos[set]);
}
// sincosf: the same reduction and polynomials as the two calls (glibc's sincosf_poly)
PHD void SinCos(float y, float *s, float *c) {
    if (!(AbsTop12(y) < AbsTop12(__builtin_huge_valf()))) {
        *s = *c = (y - y) / (y - y);
        return;
    }
    double r;
    int n, set;
    if (!SinCosReduce(y, &r, &n, &set)) {
        if (AbsTop12(y) < AbsTop12(0x1p-12f)) {
            *s = y;
            *c = 1.f;
            return;
        }
        const double x = y, x2 = x * x;
        *s = (float)SinPolyD(x, x2, kSinCos[0]);
        *c = (float)CosPolyD(x2, kSinCos[0]);
        return;
    }
    const double r2 = r * r;
    const float sp = (float)SinPolyD(r, r2, kSinCos[set]), cp = (float)CosPolyD(r2, kSinCos[set]);
    *s = (n & 1) ? cp : sp;
    *c = (n & 1) ? sp : cp;
}

// ---- exp: 2^(k/32) from a table times a cubic in the remainder (e_expf.c, e_exp2f_data.c) ------
// kExp2Tab[i] = bits(2^(i/32)) - (i << 47)
constexpr uint64_t kExp2Tab[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51, 0x3fef72b83c7d517b,
    0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1, 0x3fef06fe0a31b715, 0x3feef1a7373aa9cb,
    0x3feedea64c123422, 0x3feece086061892d, 0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429,
    0x3feea47eb03a5585, 0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d, 0x3feee89f995ad3ad,
    0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069, 0x3fef5818dcfba487, 0x3fef7c97337b9b5f,
    0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
PHD float Exp(float x) {
    constexpr double kInvLn2N = 0x1.71547652b82fep+0 * 32, kShift = 0x1.8p+52;
    constexpr double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
                     C2 = 0x1.62e42ff0c52d6p-1 / 32;
    const uint32_t abstop = AbsTop12(x);
    if (abstop >= AbsTop12(88.0f)) {
        if (Bits(x) == Bits(-__builtin_huge_valf())) return 0.f;
        if (abstop >= AbsTop12(__builtin_huge_valf())) return x + x;
        if (x > 0x1.62e42ep6f) return __builtin_huge_valf();
        if (x < -0x1.9fe368p6f) return 0.f;
    }
    const double xd = x;
    // z = x 32/ln2 = k + r; both uses of the product are contracted (k via the 1.5 2^52 shift)
    double kd = fma(kInvLn2N, xd, kShift);
    const uint64_t ki = Bits64(kd);
    kd -= kShift;
    const double r = fma(kInvLn2N, xd, -kd);
    const double s = FromBits64(kExp2Tab[ki % 32] + (ki << 47));
    const double z = fma(C0, r, C1);
    const double r2 = r * r;
    double y = fma(C2, r, 1.0);
    y = fma(z, r2, y);
    return (float)(y * s);
}

// ---- log: log(c) + k ln2 from a 16-entry table plus a cubic in z/c - 1 (e_logf.c, e_logf_data.c)
struct LogEntry {
    double invc, logc;
};
constexpr LogEntry kLogTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
PHD float Log(float x) {
    constexpr double kLn2 = 0x1.62e42fefa39efp-1;
    constexpr double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = Bits(x);
    if (ix == 0x3f800000) return 0.f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -__builtin_huge_valf();
        if (ix == 0x7f800000) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);
        ix = Bits(x * 0x1p23f);  // subnormal: normalise
        ix -= 23u << 23;
    }
    // x = 2^k z, z in [0x3f330000, 2 * 0x3f330000); the interval's c is near z
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) % 16);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & (0x1ffu << 23));
    const double z = (double)FromBits(iz);
    const double r = fma(z, kLogTab[i].invc, -1.0);
    const double y0 = fma((double)k, kLn2, kLogTab[i].logc);
    const double r2 = r * r;
    double y = fma(A1, r, A2);
    y = fma(A0, r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}

// ---- asin / acos (e_asinf.c, e_acosf.c), float arithmetic, no fma -----------------------------
PHD float ASin(float x) {
    constexpr float kPio2Hi = 1.57079637050628662109375f, kPio2Lo = -4.37113900018624283e-8f,
                    kPio4Hi = 0.785398185253143310546875f;
    constexpr float p0 = 1.666675248e-1f, p1 = 7.495297643e-2f, p2 = 4.547037598e-2f, p3 = 2.417951451e-2f,
                    p4 = 4.216630880e-2f;
    const int32_t hx = (int32_t)Bits(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return x * kPio2Hi + x * kPio2Lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix < 0x32000000) return x;
        const float t = x * x;
        const float w = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
        return x + x * w;
    }
    float w = 1.f - std::fabs(x), t = w * 0.5f;
    float p = t * (p0 + t * (p1 + t * (p2 + t * (p3 + t * p4))));
    const float s = std::sqrt(t);
    if (ix >= 0x3F79999A) {
        t = kPio2Hi - (2.0f * (s + s * p) - kPio2Lo);
    } else {
        w = FromBits(Bits(s) & 0xfffff000u);
        const float c = (t - w * w) / (s + w);
        const float r = p;
        p = 2.0f * s * r - (kPio2Lo - 2.0f * c);
        const float q = kPio4Hi - 2.0f * w;
        t = kPio4Hi - (p - q);
    }
    return hx > 0 ? t : -t;
}
PHD float ACosP(float z) {
    const float pS0 = FromBits(0x3e2aaaab), pS1 = FromBits(0xbea6b090), pS2 = FromBits(0x3e4e0aa8),
                pS3 = FromBits(0xbd241146), pS4 = FromBits(0x3a4f7f04), pS5 = FromBits(0x3811ef08);
    return z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
}
PHD float ACosQ(float z) {
    const float qS1 = FromBits(0xc019d139), qS2 = FromBits(0x4001572d), qS3 = FromBits(0xbf303361),
                qS4 = FromBits(0x3d9dc62e);
    return 1.f + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
}
PHD float ACos(float x) {
    const float kPi = FromBits(0x40490fda), kPio2Hi = FromBits(0x3fc90fda), kPio2Lo = FromBits(0x33a22168);
    const int32_t hx = (int32_t)Bits(x), ix = hx & 0x7fffffff;
    if (ix == 0x3f800000) return hx > 0 ? 0.f : kPi + 2.0f * kPio2Lo;
    if (ix > 0x3f800000) return (x - x) / (x - x);
    if (ix < 0x3f000000) {
        if (ix <= 0x23000000) return kPio2Hi + kPio2Lo;
        const float z = x * x;
        const float r = ACosP(z) / ACosQ(z);
        return kPio2Hi - (x - (kPio2Lo - x * r));
    }
    if (hx < 0) {
        const float z = (1.f + x) * 0.5f;
        const float p = ACosP(z), q = ACosQ(z);
        const float s = std::sqrt(z);
        const float r = p / q;
        const float w = r * s - kPio2Lo;
        return kPi - 2.0f * (s + w);
    }
    const float z = (1.f - x) * 0.5f;
    const float s = std::sqrt(z);
    const float df = FromBits(Bits(s) & 0xfffff000u);
    const float c = (z - df * df) / (s + df);
    const float r = ACosP(z) / ACosQ(z);
    const float w = r * s + c;
    return 2.0f * (df + w);
}

// ---- atan / atan2 (s_atanf.c, e_atan2f.c) -----------------------------------------------------
PHD float ATan(float x) {
    const float atanhi[4] = {FromBits(0x3eed6338), FromBits(0x3f490fda), FromBits(0x3f7b985e), FromBits(0x3fc90fda)};
    const float atanlo[4] = {FromBits(0x31ac3769), FromBits(0x33222168), FromBits(0x33140fb4), FromBits(0x33a22168)};
    const int32_t hx = (int32_t)Bits(x), ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {  // |x| < 0.4375
        if (ix < 0x31000000) return x;
        id = -1;
    } else {
        x = std::fabs(x);
        if (ix < 0x3f980000) {
            if (ix < 0x3f300000) {
                id = 0;
                x = (2.0f * x - 1.f) / (2.0f + x);
            } else {
                id = 1;
                x = (x - 1.f) / (x + 1.f);
            }
        } else if (ix < 0x401c0000) {
            id = 2;
            x = (x - 1.5f) / (1.f + 1.5f * x);
        } else {
            id = 3;
            x = -1.0f / x;
        }
    }
    const float aT0 = FromBits(0x3eaaaaab), aT1 = FromBits(0xbe4ccccd), aT2 = FromBits(0x3e124925),
                aT3 = FromBits(0xbde38e38), aT4 = FromBits(0x3dba2e6e), aT5 = FromBits(0xbd9d8795),
                aT6 = FromBits(0x3d886b35), aT7 = FromBits(0xbd6ef16b), aT8 = FromBits(0x3d4bda59),
                aT9 = FromBits(0xbd15a221), aT10 = FromBits(0x3c8569d7);
    const float z = x * x, w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    float hi = 0, lo = 0;
    switch (id) {  // a switch, not an indexed local array (which would sit in scratch on the GPU)
    case 0: hi = atanhi[0], lo = atanlo[0]; break;
    case 1: hi = atanhi[1], lo = atanlo[1]; break;
    case 2: hi = atanhi[2], lo = atanlo[2]; break;
    default: hi = atanhi[3], lo = atanlo[3]; break;
    }
    const float r = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -r : r;
}
PHD float ATan2(float y, float x) {
    const float kPio4 = FromBits(0x3f490fdb), kPio2 = FromBits(0x3fc90fdb), kPi = FromBits(0x40490fdb),
                kPiLo = FromBits(0xb3bbbd2e);
    const int32_t hx = (int32_t)Bits(x), hy = (int32_t)Bits(y), ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return ATan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);  // 2 sign(x) + sign(y)
    if (iy == 0) return m <= 1 ? y : (m == 2 ? kPi : -kPi);
    if (ix == 0) return hy < 0 ? -kPio2 : kPio2;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            const float a = (m & 2) ? 3.0f * kPio4 : kPio4;
            return (m & 1) ? -a : a;
        }
        const float a = (m & 2) ? kPi : 0.f;
        return (m & 1) ? -a : a;
    }
    if (iy == 0x7f800000) return hy < 0 ? -kPio2 : kPio2;
    const int k = (iy - ix) >> 23;
    float z;
    if (k > 60)
        z = kPio2 + 0.5f * kPiLo;
    else if (hx < 0 && k < -60)
        z = 0.0f;
    else
        z = ATan(std::fabs(y / x));
    switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return kPi - (z - kPiLo);
    default: return (z - kPiLo) - kPi;
    }
}

// ---- tan (s_tanf.c over k_tanf.c; sinf's double reduction for |x| > pi/4) ----------------------
PHD float KernelTan(float x, float y, int iy) {
    const float kPio4 = FromBits(0x3f490fda), kPio4Lo = FromBits(0x33222168);
    const float T0 = FromBits(0x3eaaaaab), T1 = FromBits(0x3e088889), T2 = FromBits(0x3d5d0dd1),
                T3 = FromBits(0x3cb327a4), T4 = FromBits(0x3c11371f), T5 = FromBits(0x3b6b6916),
                T6 = FromBits(0x3abede48), T7 = FromBits(0x3a1a26c8), T8 = FromBits(0x398137b9),
                T9 = FromBits(0x38a3f445), T10 = FromBits(0x3895c07a), T11 = FromBits(0xb79bae5f),
                T12 = FromBits(0x37d95384);
    const int32_t hx = (int32_t)Bits(x), ix = hx & 0x7fffffff;
    if (ix < 0x39000000) {  // |x| < 2^-13
        if ((ix | (iy + 1)) == 0) return 1.f / std::fabs(x);
        return iy == 1 ? x : -1.f / x;
    }
    if (ix >= 0x3f2ca140) {  // |x| >= 0.6744: tan(pi/4 - x)
        if (hx < 0) {
            x = -x;
            y = -y;
        }
        const float z = kPio4 - x, w = kPio4Lo - y;
        x = z + w;
        y = 0.0f;
        if (std::fabs(x) < 0x1p-13f) return (float)((1 - ((hx >> 30) & 2)) * iy) * (1.0f - (float)(2 * iy) * x);
    }
    float z = x * x, w = z * z;
    float r = T1 + w * (T3 + w * (T5 + w * (T7 + w * (T9 + w * T11))));
    float v = z * (T2 + w * (T4 + w * (T6 + w * (T8 + w * (T10 + w * T12)))));
    float s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T0 * s;
    w = x + r;
    if (ix >= 0x3f2ca140) {
        v = (float)iy;
        return (float)(1 - ((hx >> 30) & 2)) * (v - 2.0f * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    // -1 / (x + r), accurately
    z = FromBits(Bits(w) & 0xfffff000u);
    v = r - (z - x);
    const float a = -1.0f / w;
    const float t = FromBits(Bits(a) & 0xfffff000u);
    s = 1.0f + t * z;
    return t + a * (s + t * v);
}
PHD float Tan(float x) {
    const int32_t ix = (int32_t)Bits(x) & 0x7fffffff;
    if (ix <= 0x3f490fda) return KernelTan(x, 0.0f, 1);
    if (ix >= 0x7f800000) return x - x;
    // __ieee754_rem_pio2f: the sinf reduction without fma (this file is not an -mfma variant)
    double dx = x;
    int n;
    if (AbsTop12(x) < AbsTop12(120.0f)) {
        dx = ReduceFast(dx, &n, false);
    } else {
        const uint32_t xi = Bits(x);
        dx = ReduceLarge(xi, &n);
        if (xi >> 31) {
            dx = -dx;
            n = -n;
        }
    }
    const float y0 = (float)dx, y1 = (float)(dx - (double)y0);
    return KernelTan(y0, y1, 1 - ((n & 1) << 1));
}

// ---- expm1 / sinh (s_expm1f.c, e_sinhf.c) ------------------------------------------------------
PHD float Expm1(float x) {
    const float kOThreshold = FromBits(0x42b17180), kLn2Hi = FromBits(0x3f317180), kLn2Lo = FromBits(0x3717f7d1),
                kInvLn2 = FromBits(0x3fb8aa3b);
    const float Q1 = FromBits(0xbd088889), Q2 = FromBits(0x3ad00d01), Q3 = FromBits(0xb8a670cd),
                Q4 = FromBits(0x36867e54), Q5 = FromBits(0xb457edbb);
    uint32_t hx = Bits(x);
    const uint32_t xsb = hx & 0x80000000u;
    hx &= 0x7fffffff;
    if (hx >= 0x4195b844) {  // |x| >= 27 ln2
        if (hx >= 0x42b17218) {
            if (hx > 0x7f800000) return x + x;
            if (hx == 0x7f800000) return xsb == 0 ? x : -1.0f;
            if (x > kOThreshold) return __builtin_huge_valf();
        }
        if (xsb != 0) return -1.0f;  // tiny - one
    }
    float hi, lo, c = 0.f, t;
    int32_t k;
    if (hx > 0x3eb17218) {  // |x| > ln2 / 2
        if (hx < 0x3F851592) {
            if (xsb == 0) {
                hi = x - kLn2Hi;
                lo = kLn2Lo;
                k = 1;
            } else {
                hi = x + kLn2Hi;
                lo = -kLn2Lo;
                k = -1;
            }
        } else {
            k = (int32_t)(kInvLn2 * x + (xsb == 0 ? 0.5f : -0.5f));
            t = (float)k;
            hi = x - t * kLn2Hi;
            lo = t * kLn2Lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x33000000) {
        return x;
    } else {
        k = 0;
    }
    const float hfx = 0.5f * x, hxs = x * hfx;
    const float r1 = 1.f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0f - r1 * hfx;
    float e = hxs * ((r1 - t) / (6.0f - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5f * (x - e) - 0.5f;
    if (k == 1) return x < -0.25f ? -2.0f * (e - (x + 0.5f)) : 1.f + 2.0f * (x - e);
    float y;
    if (k <= -2 || k > 56) {
        y = 1.f - (e - x);
        y = FromBits(Bits(y) + ((uint32_t)k << 23));
        return y - 1.f;
    }
    if (k < 23) {
        t = FromBits(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
        y = t - (e - x);
    } else {
        t = FromBits((uint32_t)(0x7f - k) << 23);  // 2^-k
        y = x - (e + t);
        y += 1.f;
    }
    return FromBits(Bits(y) + ((uint32_t)k << 23));
}
PHD float Sinh(float x) {
    const int32_t jx = (int32_t)Bits(x), ix = jx & 0x7fffffff;
    if (ix >= 0x7f800000) return x + x;
    const float h = jx < 0 ? -0.5f : 0.5f;
    if (ix < 0x41b00000) {  // |x| < 22
        if (ix < 0x31800000) return x;
        const float t = Expm1(std::fabs(x));
        if (ix < 0x3f800000) return h * (2.0f * t - t * t / (t + 1.f));
        return h * (t + t / (t + 1.f));
    }
    if (ix < 0x42b17180) return h * Exp(std::fabs(x));
    if (ix <= 0x42b2d4fc) {
        const float w = Exp(0.5f * std::fabs(x)), t = h * w;
        return t * w;
    }
    return x * 1.0e37f;
}

// one function by index, for the host / device self-checks (pbrt_debug_det_math): 0 sin, 1 cos,
// 2 asin, 3 acos (arguments clamped to [-1, 1] as SafeASin / SafeACos do), 4 atan2(a, b), 5 log,
// 6 / 7 sincos's sine / cosine, 8 exp, 9 sinh, 10 tan, 11 atan, 12 expm1
PHD float Eval(int fn, float a, float b) {
    float s, c;
    switch (fn) {
    case 0: return Sin(a);
    case 1: return Cos(a);
    case 2: return ASin(a < -1.f ? -1.f : (a > 1.f ? 1.f : a));  // pbrt's Clamp: NaN stays NaN
    case 3: return ACos(a < -1.f ? -1.f : (a > 1.f ? 1.f : a));
    case 4: return ATan2(a, b);
    case 5: return Log(a);
    case 6: SinCos(a, &s, &c); return s;
    case 7: SinCos(a, &s, &c); return c;
    case 8: return Exp(a);
    case 9: return Sinh(a);
    case 10: return Tan(a);
    case 11: return ATan(a);
    default: return Expm1(a);
    }
}
constexpr int kNumEvalFns = 13;

}  // namespace detm
}  // namespace pbrt_amd
