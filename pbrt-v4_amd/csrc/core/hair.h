// HairBxDF (bxdfs.h:1054-1152, bxdfs.cpp:279-573) and HairMaterial::GetBxDF (materials.h:
// 353-427): the d'Eon / Chiang longitudinal (Mp), attenuation (Ap) and azimuthal (Np) terms
// for pMax = 3, evaluated in pbrt's float operation order so a host restatement gives the same
// bits.  The constructor's constants (v, s, the scale-tilt sines) are computed per hit on the
// device, as GetBxDF constructs the BxDF per hit; its transcendentals are the portable ones of
// detmath.h (Sinf, Expf, Logf, Sinhf, ATan2f, ASinf).  Spectral quantities are kNSpectrumSamples
// arrays indexed by wavelength; the wavelength-independent factors (Mp, Np, the phases) are
// evaluated once and the per-wavelength loop only forms T and the Ap terms.
#pragma once

#include "core.h"

namespace pbrt_amd {

constexpr int kHairPMax = 3;

// util/math.h:294-309 Pow<n>: n2 * n2 * Pow<n & 1>
template <int n>
PHD float PowN(float v) {
    if constexpr (n == 0) {
        return 1.f;
    } else if constexpr (n == 1) {
        return v;
    } else {
        const float n2 = PowN<n / 2>(v);
        return n2 * n2 * PowN<n & 1>(v);
    }
}

// util/math.h:794-816 I0 / LogI0 (ten series terms; the denominators are int64 products
// converted to float, as the reference's float / int64 division does)
PHD float HairI0(float x) {
    float val = 0, x2i = 1;
    int64_t ifact = 1;
    int i4 = 1;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        if (i > 1) ifact *= i;
        val += x2i / (float)((int64_t)i4 * (ifact * ifact));
        x2i *= x * x;
        i4 *= 4;
    }
    return val;
}
PHD float HairLogI0(float x) {
    if (x > 12) return x + 0.5f * (-Logf(2 * kPi) + Logf(1 / x) + 1 / (8 * x));
    return Logf(HairI0(x));
}

// util/math.h:490-502, util/sampling.h:256-278 (logistic distribution on [-pi, pi])
PHD float Logistic(float x, float s) {
    x = std::fabs(x);
    return Expf(-x / s) / (s * Sqr(1 + Expf(-x / s)));
}
PHD float LogisticCDF(float x, float s) { return 1 / (1 + Expf(-x / s)); }
PHD float TrimmedLogistic(float x, float s, float a, float b) {
    return Logistic(x, s) / (LogisticCDF(b, s) - LogisticCDF(a, s));
}
PHD float SampleTrimmedLogistic(float u, float s, float a, float b) {
    const float pa = LogisticCDF(a, s), pb = LogisticCDF(b, s);
    u = (1 - u) * pa + u * pb;  // Lerp(u, P(a), P(b))
    const float x = -s * Logf(1 / u - 1);
    return Clampf(x, a, b);
}

// the BxDF's per-hit state (the constructor's fields but sigma_a, which the caller keeps as a
// kNSpectrumSamples array)
struct HairState {
    float h, eta, gamma_o;
    float v[kHairPMax + 1], s;
    float sin2k[kHairPMax], cos2k[kHairPMax];
};

// HairBxDF::HairBxDF (bxdfs.cpp:280-306)
PHD HairState MakeHair(float h, float eta, float beta_m, float beta_n, float alpha) {
    HairState H;
    H.h = h;
    H.eta = eta;
    H.gamma_o = SafeASin(h);
    H.v[0] = Sqr(0.726f * beta_m + 0.812f * Sqr(beta_m) + 3.7f * PowN<20>(beta_m));
    H.v[1] = (float)(.25 * (double)H.v[0]);
    H.v[2] = 4 * H.v[0];
    H.v[3] = H.v[2];
    const float SqrtPiOver8 = 0.626657069f;
    H.s = SqrtPiOver8 * (0.265f * beta_n + 1.194f * Sqr(beta_n) + 5.372f * PowN<22>(beta_n));
    H.sin2k[0] = Sinf((kPi / 180) * alpha);
    H.cos2k[0] = SafeSqrt(1 - Sqr(H.sin2k[0]));
    for (int i = 1; i < kHairPMax; ++i) {
        H.sin2k[i] = 2 * H.cos2k[i - 1] * H.sin2k[i - 1];
        H.cos2k[i] = Sqr(H.cos2k[i - 1]) - Sqr(H.sin2k[i - 1]);
    }
    return H;
}

// HairBxDF::SigmaAFromReflectance's denominator (bxdfs.cpp:564-573) for beta_n
PHD float HairReflectanceDenom(float beta_n) {
    return 5.969f - 0.215f * beta_n + 2.532f * Sqr(beta_n) - 10.73f * PowN<3>(beta_n) + 5.574f * PowN<4>(beta_n) +
           0.245f * PowN<5>(beta_n);
}
PHD float HairSigmaAFromReflectance(float c, float denom) { return Sqr(Logf(c) / denom); }

// bxdfs.h:1092-1100 Mp (the v <= .1 test is a double comparison in the reference)
PHD float HairMp(float cosTheta_i, float cosTheta_o, float sinTheta_i, float sinTheta_o, float v) {
    const float a = cosTheta_i * cosTheta_o / v, b = sinTheta_i * sinTheta_o / v;
    if ((double)v <= .1) return FastExp(HairLogI0(a) - b - 1 / v + 0.6931f + Logf(1 / (2 * v)));
    return (FastExp(-b) * HairI0(a)) / (Sinhf(1 / v) * 2 * v);
}
// bxdfs.h:1126-1140 Phi / Np
PHD float HairPhi(int p, float gamma_o, float gamma_t) { return (float)(2 * p) * gamma_t - 2 * gamma_o + (float)p * kPi; }
PHD float HairNp(float phi, int p, float s, float gamma_o, float gamma_t) {
    float dphi = phi - HairPhi(p, gamma_o, gamma_t);
    while (dphi > kPi) dphi -= 2 * kPi;
    while (dphi < -kPi) dphi += 2 * kPi;
    return TrimmedLogistic(dphi, s, -kPi, kPi);
}
// the scale-tilted sin / cos of theta_o for term p (bxdfs.cpp:338-358)
PHD void HairTilt(const HairState &H, int p, float sinTheta_o, float cosTheta_o, float *sp, float *cp) {
    float s, c;
    if (p == 0) {
        s = sinTheta_o * H.cos2k[1] - cosTheta_o * H.sin2k[1];
        c = cosTheta_o * H.cos2k[1] + sinTheta_o * H.sin2k[1];
    } else if (p == 1) {
        s = sinTheta_o * H.cos2k[0] + cosTheta_o * H.sin2k[0];
        c = cosTheta_o * H.cos2k[0] - sinTheta_o * H.sin2k[0];
    } else if (p == 2) {
        s = sinTheta_o * H.cos2k[2] + cosTheta_o * H.sin2k[2];
        c = cosTheta_o * H.cos2k[2] - sinTheta_o * H.sin2k[2];
    } else {
        s = sinTheta_o;
        c = cosTheta_o;
    }
    *sp = s;
    *cp = std::fabs(c);
}

// Ap (bxdfs.h:1102-1124) at one wavelength: f is FrDielectric(cosTheta_o cos(gamma_o), eta),
// T the single-path transmittance; ap[3] stays 0 when 1 - T f is zero at every wavelength
// (anyNz false), as the reference leaves it default-constructed
PHD void HairAp(float f, float T, bool anyNz, float ap[4]) {
    ap[0] = f;
    ap[1] = Sqr(1 - f) * T;
    ap[2] = ap[1] * T * f;
    ap[3] = anyNz ? ap[2] * f * T / (1 - T * f) : 0.f;
}

// the refracted ray's terms for sinTheta_o (bxdfs.cpp:320-331): the single-path transmittance
// exponent scale 2 cos(gamma_t) / cos(theta_t) and gamma_t
PHD void HairRefracted(const HairState &H, float sinTheta_o, float cosTheta_o, float *tScale, float *gamma_t) {
    const float sinTheta_t = sinTheta_o / H.eta;
    const float cosTheta_t = SafeSqrt(1 - Sqr(sinTheta_t));
    const float etap = SafeSqrt(Sqr(H.eta) - Sqr(sinTheta_o)) / cosTheta_o;
    const float sinGamma_t = H.h / etap;
    const float cosGamma_t = SafeSqrt(1 - Sqr(sinGamma_t));
    *gamma_t = SafeASin(sinGamma_t);
    *tScale = 2 * cosGamma_t / cosTheta_t;
}
// SampledSpectrum::operator bool of 1 - T f over the wavelengths
PHD bool HairAnyNz(const float *sigma_a, float tScale, float f) {
    bool nz = false;
#pragma unroll 1
    for (int i = 0; i < kNSpectrumSamples; ++i) nz |= 1 - Expf(-sigma_a[i] * tScale) * f != 0;
    return nz;
}

// HairBxDF::f (bxdfs.cpp:308-371) into out[kNSpectrumSamples]
PHD void HairF(const HairState &H, const float *sigma_a, V3 wo, V3 wi, float *out) {
    const float sinTheta_o = wo.x, cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
    const float phi_o = ATan2f(wo.z, wo.y);
    const float sinTheta_i = wi.x, cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
    const float phi_i = ATan2f(wi.z, wi.y);
    float tScale, gamma_t;
    HairRefracted(H, sinTheta_o, cosTheta_o, &tScale, &gamma_t);
    const float phi = phi_i - phi_o;
    float mnp[kHairPMax], mp3;
#pragma unroll
    for (int p = 0; p < kHairPMax; ++p) {
        float sp, cp;
        HairTilt(H, p, sinTheta_o, cosTheta_o, &sp, &cp);
        mnp[p] = HairMp(cosTheta_i, cp, sinTheta_i, sp, H.v[p]);
    }
    mp3 = HairMp(cosTheta_i, cosTheta_o, sinTheta_i, sinTheta_o, H.v[kHairPMax]);
    float np[kHairPMax];
#pragma unroll
    for (int p = 0; p < kHairPMax; ++p) np[p] = HairNp(phi, p, H.s, H.gamma_o, gamma_t);
    const float f = FrDielectric(cosTheta_o * SafeSqrt(1 - Sqr(H.h)), H.eta);
    const bool anyNz = HairAnyNz(sigma_a, tScale, f);
    const float absCos = std::fabs(wi.z);
#pragma unroll 1
    for (int i = 0; i < kNSpectrumSamples; ++i) {
        const float T = Expf(-sigma_a[i] * tScale);
        float ap[4];
        HairAp(f, T, anyNz, ap);
        float fs = 0;
#pragma unroll
        for (int p = 0; p < kHairPMax; ++p) fs += mnp[p] * ap[p] * np[p];
        fs += mp3 * ap[kHairPMax] / (2 * kPi);
        if (absCos > 0) fs /= absCos;
        out[i] = fs;
    }
}

// HairBxDF::ApPDF (bxdfs.cpp:373-400): note sinTheta_o is recomputed from cosTheta_o
PHD void HairApPDF(const HairState &H, const float *sigma_a, float cosTheta_o, float apPDF[4]) {
    const float sinTheta_o = SafeSqrt(1 - Sqr(cosTheta_o));
    float tScale, gamma_t;
    HairRefracted(H, sinTheta_o, cosTheta_o, &tScale, &gamma_t);
    const float f = FrDielectric(cosTheta_o * SafeSqrt(1 - Sqr(H.h)), H.eta);
    const bool anyNz = HairAnyNz(sigma_a, tScale, f);
    float sum[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int i = 0; i < kNSpectrumSamples; ++i) {
        const float T = Expf(-sigma_a[i] * tScale);
        float ap[4];
        HairAp(f, T, anyNz, ap);
#pragma unroll
        for (int p = 0; p < 4; ++p) sum[p] = i == 0 ? ap[p] : sum[p] + ap[p];
    }
    float sumY = 0, avg[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        avg[p] = sum[p] / kNSpectrumSamples;
        sumY += avg[p];
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) apPDF[p] = avg[p] / sumY;
}

// the PDF sum over the terms for a sampled / given azimuth difference (bxdfs.cpp:462-492, 520-549)
PHD float HairPdfSum(const HairState &H, const float apPDF[4], float sinTheta_o, float cosTheta_o, float sinTheta_i,
                     float cosTheta_i, float dphi, float gamma_t) {
    float pdf = 0;
#pragma unroll
    for (int p = 0; p < kHairPMax; ++p) {
        float sp, cp;
        HairTilt(H, p, sinTheta_o, cosTheta_o, &sp, &cp);
        pdf += HairMp(cosTheta_i, cp, sinTheta_i, sp, H.v[p]) * apPDF[p] * HairNp(dphi, p, H.s, H.gamma_o, gamma_t);
    }
    pdf += HairMp(cosTheta_i, cosTheta_o, sinTheta_i, sinTheta_o, H.v[kHairPMax]) * apPDF[kHairPMax] * (1 / (2 * kPi));
    return pdf;
}

// HairBxDF::PDF (bxdfs.cpp:497-551)
PHD float HairPDF(const HairState &H, const float *sigma_a, V3 wo, V3 wi) {
    const float sinTheta_o = wo.x, cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
    const float phi_o = ATan2f(wo.z, wo.y);
    const float sinTheta_i = wi.x, cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
    const float phi_i = ATan2f(wi.z, wi.y);
    const float etap = SafeSqrt(H.eta * H.eta - Sqr(sinTheta_o)) / cosTheta_o;
    const float gamma_t = SafeASin(H.h / etap);
    float apPDF[4];
    HairApPDF(H, sigma_a, cosTheta_o, apPDF);
    return HairPdfSum(H, apPDF, sinTheta_o, cosTheta_o, sinTheta_i, cosTheta_i, phi_i - phi_o, gamma_t);
}

// util/sampling.h:79-115 SampleDiscrete over the four Ap weights (uRemapped with std::min)
PHD int HairSampleTerm(const float w[4], float u, float *uRemapped) {
    float sumWeights = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) sumWeights += w[k];
    float up = u * sumWeights;
    if (up == sumWeights) up = NextFloatDown(up);
    int offset = 0;
    float sum = 0;
    while (offset < 3 && sum + w[offset] <= up) sum += w[offset++];
    const float r = (up - sum) / w[offset];
    *uRemapped = kOneMinusEpsilon < r ? kOneMinusEpsilon : r;
    return offset;
}

// HairBxDF::Sample_f (bxdfs.cpp:402-495); false when BSDF::Sample_f returns {} (f all zero,
// pdf 0 or wi.z 0), else wi, pdf and f in out[kNSpectrumSamples]
PHD bool HairSampleF(const HairState &H, const float *sigma_a, V3 wo, float uc, float u0, float u1, V3 *wiOut,
                     float *pdfOut, float *out) {
    const float sinTheta_o = wo.x, cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
    const float phi_o = ATan2f(wo.z, wo.y);
    float apPDF[4];
    HairApPDF(H, sigma_a, cosTheta_o, apPDF);
    const int p = HairSampleTerm(apPDF, uc, &uc);
    float sinThetap_o, cosThetap_o;
    HairTilt(H, p, sinTheta_o, cosTheta_o, &sinThetap_o, &cosThetap_o);
    const float vp = H.v[p];
    const float cosTheta = 1 + vp * Logf(std::fmax(u0, 1e-5f) + (1 - u0) * FastExp(-2 / vp));
    const float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    const float cosPhi = Cosf(2 * kPi * u1);
    const float sinTheta_i = -cosTheta * sinThetap_o + sinTheta * cosPhi * cosThetap_o;
    const float cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
    const float etap = SafeSqrt(Sqr(H.eta) - Sqr(sinTheta_o)) / cosTheta_o;
    const float sinGamma_t = H.h / etap;
    const float gamma_t = SafeASin(sinGamma_t);
    const float dphi = p < kHairPMax ? HairPhi(p, H.gamma_o, gamma_t) + SampleTrimmedLogistic(uc, H.s, -kPi, kPi)
                                     : 2 * kPi * uc;
    const float phi_i = phi_o + dphi;
    const V3 wi(sinTheta_i, cosTheta_i * Cosf(phi_i), cosTheta_i * Sinf(phi_i));
    const float pdf = HairPdfSum(H, apPDF, sinTheta_o, cosTheta_o, sinTheta_i, cosTheta_i, dphi, gamma_t);
    HairF(H, sigma_a, wo, wi, out);
    bool nz = false;
#pragma unroll 1
    for (int i = 0; i < kNSpectrumSamples; ++i) nz |= out[i] != 0;
    if (!nz || pdf == 0 || wi.z == 0) return false;
    *wiOut = wi;
    *pdfOut = pdf;
    return true;
}

// the debug entry pbrt_debug_hair's per-query evaluation (host and device): in[16] = {h, eta,
// beta_m, beta_n, alpha, sigma_a0, wo, wi, uc, u0, u1, sigma_a slope}, sigma_a[i] = sigma_a0 +
// slope i; out[kHairDebugOut] = {f(wo, wi)[NS], PDF(wo, wi), ok, wi', pdf', f'[NS]} (the
// BxDF constructed as GetBxDF does it, without its beta clamps)
constexpr int kHairDebugIn = 16, kHairDebugOut = 2 * kNSpectrumSamples + 6;
PHD void HairDebugEval(const float *in, float *out) {
    float sa[kNSpectrumSamples];
    for (int i = 0; i < kNSpectrumSamples; ++i) sa[i] = in[5] + in[15] * (float)i;
    const HairState H = MakeHair(in[0], in[1], in[2], in[3], in[4]);
    const V3 wo(in[6], in[7], in[8]), wi(in[9], in[10], in[11]);
    HairF(H, sa, wo, wi, out);
    out[kNSpectrumSamples] = HairPDF(H, sa, wo, wi);
    float *o = out + kNSpectrumSamples + 1;
    V3 ws(0, 0, 0);
    float pdf = 0;
    const bool ok = HairSampleF(H, sa, wo, in[12], in[13], in[14], &ws, &pdf, o + 5);
    o[0] = ok ? 1.f : 0.f;
    o[1] = ws.x;
    o[2] = ws.y;
    o[3] = ws.z;
    o[4] = pdf;
    if (!ok)
        for (int i = 0; i < kNSpectrumSamples; ++i) o[5 + i] = 0;
}

}  // namespace pbrt_amd
