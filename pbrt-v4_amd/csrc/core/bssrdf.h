// Subsurface scattering, shared by the host (loader, debug entries) and the device kernels:
// the Catmull-Rom spline utilities (util/math.cpp:157-290, util/sampling.cpp:424-488), the
// tabulated BSSRDF (bssrdf.h:112-318: Sr, SampleSr, PDF_Sr, SampleSp, PDF_Sp), the diffuse
// reflectance inversion (SubsurfaceFromDiffuse, bssrdf.h:322-333) and NormalizedFresnelBxDF
// (bxdfs.h:1206-1265).  Everything is float in pbrt's operation order (FMA only where pbrt's
// EvaluatePolynomial has one), so host and device results are identical.
//
// A BSSRDF table (BSSRDFTable, bssrdf.h:77-94) is one float block: rhoSamples[100],
// radiusSamples[64], profile[100][64], rhoEff[100], profileCDF[100][64] (SssTable views it).
#pragma once

#include "core.h"

namespace pbrt_amd {

constexpr int kSssRho = 100, kSssRadius = 64;
constexpr int kSssTableFloats = kSssRho + kSssRadius + 2 * kSssRho * kSssRadius + kSssRho;

struct SssTable {
    const float *rho, *radius, *profile, *rhoEff, *cdf;
    PHD static SssTable At(const float *t) {
        SssTable s;
        s.rho = t;
        s.radius = t + kSssRho;
        s.profile = s.radius + kSssRadius;
        s.rhoEff = s.profile + kSssRho * kSssRadius;
        s.cdf = s.rhoEff + kSssRho;
        return s;
    }
};

// FindInterval (util/math.h): the largest i in [0, sz - 2] with pred(i) (pred monotone)
template <typename Pred>
PHD int FindIntervalP(int sz, const Pred &pred) {
    int size = sz - 2, first = 1;
    while (size > 0) {
        const int half = size >> 1, middle = first + half;
        const bool r = pred(middle);
        first = r ? middle + 1 : first;
        size = r ? size - (half + 1) : half;
    }
    const int i = first - 1;
    return i < 0 ? 0 : (i > sz - 2 ? sz - 2 : i);
}

// CatmullRomWeights (util/math.cpp:157-203)
PHD bool CatmullRomWeights(const float *nodes, int n, float x, int *offset, float w[4]) {
    if (!(x >= nodes[0] && x <= nodes[n - 1])) return false;
    const int idx = FindIntervalP(n, [&](int i) { return nodes[i] <= x; });
    *offset = idx - 1;
    const float x0 = nodes[idx], x1 = nodes[idx + 1];
    const float t = (x - x0) / (x1 - x0), t2 = t * t, t3 = t2 * t;
    w[1] = 2 * t3 - 3 * t2 + 1;
    w[2] = -2 * t3 + 3 * t2;
    if (idx > 0) {
        const float w0 = (t3 - 2 * t2 + t) * (x1 - x0) / (x1 - nodes[idx - 1]);
        w[0] = -w0;
        w[2] += w0;
    } else {
        const float w0 = t3 - 2 * t2 + t;
        w[0] = 0;
        w[1] -= w0;
        w[2] += w0;
    }
    if (idx + 2 < n) {
        const float w3 = (t3 - t2) * (x1 - x0) / (nodes[idx + 2] - x0);
        w[1] -= w3;
        w[3] = w3;
    } else {
        const float w3 = t3 - t2;
        w[1] -= w3;
        w[2] += w3;
        w[3] = 0;
    }
    return true;
}

// NewtonBisection (util/math.h:662-696) with xEps = fEps = 1e-6; F(t) -> (value, derivative)
template <typename F>
PHD float NewtonBisection(float x0, float x1, const F &f) {
    const float xEps = 1e-6f, fEps = 1e-6f;
    float d;
    const float fx0 = f(x0, &d), fx1 = f(x1, &d);
    if (std::fabs(fx0) < fEps) return x0;
    if (std::fabs(fx1) < fEps) return x1;
    const bool startIsNegative = fx0 < 0;
    float xMid = x0 + (x1 - x0) * -fx0 / (fx1 - fx0);
    for (int it = 0; it < 1000; ++it) {  // pbrt loops until converged; a bound keeps waves finite
        if (!(x0 < xMid && xMid < x1)) xMid = (x0 + x1) / 2;
        float dMid;
        const float fMid = f(xMid, &dMid);
        if (startIsNegative == (fMid < 0)) x0 = xMid;
        else x1 = xMid;
        if ((x1 - x0) < xEps || std::fabs(fMid) < fEps) return xMid;
        xMid -= fMid / dMid;
    }
    return xMid;
}

// InvertCatmullRom (util/math.cpp:227-265)
PHD float InvertCatmullRom(const float *nodes, const float *f, int n, float u) {
    if (!(u > f[0])) return nodes[0];
    if (!(u < f[n - 1])) return nodes[n - 1];
    const int i = FindIntervalP(n, [&](int k) { return f[k] <= u; });
    const float x0 = nodes[i], x1 = nodes[i + 1];
    const float f0 = f[i], f1 = f[i + 1];
    const float width = x1 - x0;
    const float d0 = (i > 0) ? width * (f1 - f[i - 1]) / (x1 - nodes[i - 1]) : (f1 - f0);
    const float d1 = (i + 2 < n) ? width * (f[i + 2] - f0) / (nodes[i + 2] - x0) : (f1 - f0);
    const float t = NewtonBisection(0.f, 1.f, [&](float t, float *deriv) {
        const float t2 = t * t, t3 = t2 * t;
        const float Fhat = (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
        *deriv = (6 * t2 - 6 * t) * f0 + (-6 * t2 + 6 * t) * f1 + (3 * t2 - 4 * t + 1) * d0 + (3 * t2 - 2 * t) * d1;
        return Fhat - u;
    });
    return x0 + t * width;
}

// SampleCatmullRom2D (util/sampling.cpp:424-488) without fval / pdf
PHD float SampleCatmullRom2D(const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                             const float *cdf, float alpha, float u) {
    int offset;
    float w[4];
    if (!CatmullRomWeights(nodes1, n1, alpha, &offset, w)) return 0;
    auto interpolate = [&](const float *a, int idx) {
        float v = 0;
        for (int i = 0; i < 4; ++i)
            if (w[i] != 0) v += a[(offset + i) * n2 + idx] * w[i];
        return v;
    };
    const float maximum = interpolate(cdf, n2 - 1);
    u *= maximum;
    const int idx = FindIntervalP(n2, [&](int i) { return interpolate(cdf, i) <= u; });
    const float f0 = interpolate(values, idx), f1 = interpolate(values, idx + 1);
    const float x0 = nodes2[idx], x1 = nodes2[idx + 1];
    const float width = x1 - x0;
    float d0, d1;
    u = (u - interpolate(cdf, idx)) / width;
    if (idx > 0) d0 = width * (f1 - interpolate(values, idx - 1)) / (x1 - nodes2[idx - 1]);
    else d0 = f1 - f0;
    if (idx + 2 < n2) d1 = width * (interpolate(values, idx + 2) - f0) / (nodes2[idx + 2] - x0);
    else d1 = f1 - f0;
    const float t = NewtonBisection(0.f, 1.f, [&](float t, float *deriv) {
        // EvaluatePolynomial (FMA Horner) of the segment's integral and of the segment
        const float c3 = (1.f / 3.f) * (-2 * d0 - d1) + f1 - f0, c4 = 0.25f * (d0 + d1) + 0.5f * (f0 - f1);
        const float Fhat = fmaf(t, fmaf(t, fmaf(t, fmaf(t, c4, c3), 0.5f * d0), f0), 0.f);
        const float e2 = -2 * d0 - d1 + 3 * (f1 - f0), e3 = d0 + d1 + 2 * (f0 - f1);
        *deriv = fmaf(t, fmaf(t, fmaf(t, e3, e2), d0), f0);
        return Fhat - u;
    });
    return x0 + width * t;
}

// The per-wavelength scattering properties of a TabulatedBSSRDF (bssrdf.h:118-127)
struct SssCoeffs {
    float sigma_t, rho;
};
PHD SssCoeffs MakeSssCoeffs(float sigma_a, float sigma_s) {
    SssCoeffs c;
    c.sigma_t = sigma_a + sigma_s;
    c.rho = c.sigma_t != 0 ? sigma_s / c.sigma_t : 0.f;  // SafeDiv
    return c;
}

// TabulatedBSSRDF::Sr at one wavelength before the Sqr(sigma_t) scale (bssrdf.h:132-160)
PHD float SssSr(const SssTable &t, SssCoeffs c, float r) {
    const float rOptical = r * c.sigma_t;
    int rhoOffset, radiusOffset;
    float rhoW[4], radiusW[4];
    if (!CatmullRomWeights(t.rho, kSssRho, c.rho, &rhoOffset, rhoW) ||
        !CatmullRomWeights(t.radius, kSssRadius, rOptical, &radiusOffset, radiusW))
        return 0.f;
    float sr = 0;
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 4; ++k) {
            const float weight = rhoW[j] * radiusW[k];
            if (weight != 0) sr += weight * t.profile[(rhoOffset + j) * kSssRadius + radiusOffset + k];
        }
    if (rOptical != 0) sr /= 2 * kPi * rOptical;
    return sr;
}
// Sr(r)_i = ClampZero(SssSr * Sqr(sigma_t))
PHD float SssSrScaled(const SssTable &t, SssCoeffs c, float r) {
    const float v = SssSr(t, c, r) * (c.sigma_t * c.sigma_t);
    return v > 0 ? v : 0.f;
}
// TabulatedBSSRDF::PDF_Sr at one wavelength, ClampZero applied (bssrdf.h:172-206)
PHD float SssPdfSr(const SssTable &t, SssCoeffs c, float r) {
    const float rOptical = r * c.sigma_t;
    int rhoOffset, radiusOffset;
    float rhoW[4], radiusW[4];
    if (!CatmullRomWeights(t.rho, kSssRho, c.rho, &rhoOffset, rhoW) ||
        !CatmullRomWeights(t.radius, kSssRadius, rOptical, &radiusOffset, radiusW))
        return 0.f;
    float sr = 0, rhoEff = 0;
    for (int j = 0; j < 4; ++j)
        if (rhoW[j] != 0) {
            rhoEff += t.rhoEff[rhoOffset + j] * rhoW[j];
            for (int k = 0; k < 4; ++k)
                if (radiusW[k] != 0) sr += t.profile[(rhoOffset + j) * kSssRadius + radiusOffset + k] * rhoW[j] * radiusW[k];
        }
    if (rOptical != 0) sr /= 2 * kPi * rOptical;
    const float pdf = sr * (c.sigma_t * c.sigma_t) / rhoEff;
    return pdf > 0 ? pdf : 0.f;  // ClampZero (a NaN stays NaN in pbrt's max(0, v)... see below)
}
// TabulatedBSSRDF::SampleSr (bssrdf.h:162-170): false when sigma_t[0] == 0
PHD bool SssSampleSr(const SssTable &t, SssCoeffs c0, float u, float *r) {
    if (c0.sigma_t == 0) return false;
    *r = SampleCatmullRom2D(t.rho, kSssRho, t.radius, kSssRadius, t.profile, t.cdf, c0.rho, u) / c0.sigma_t;
    return true;
}

// Frame::FromX / FromY / FromZ of a normal (util/vecmath.h:1869-1904)
PHD Frame FrameFromAxis(int axis, V3 n) {
    V3 a, b;
    if (axis == 0) {
        CoordinateSystem(n, &a, &b);
        return Frame{n, a, b};
    }
    if (axis == 1) {
        CoordinateSystem(n, &b, &a);  // (z, x)
        return Frame{a, n, b};
    }
    CoordinateSystem(n, &a, &b);
    return Frame{a, b, n};
}

// TabulatedBSSRDF::SampleSp (bssrdf.h:208-236): the probe segment p0 -> p1, or false
PHD bool SssSampleSp(const SssTable &t, SssCoeffs c0, V3 po, V3 ns, float u1, float u20, float u21, V3 *p0, V3 *p1) {
    const Frame f = FrameFromAxis(u1 < 0.25f ? 0 : (u1 < 0.5f ? 1 : 2), ns);
    float r, rMax;
    if (!SssSampleSr(t, c0, u20, &r)) return false;
    const float phi = 2 * kPi * u21;
    if (!SssSampleSr(t, c0, 0.999f, &rMax) || r >= rMax) return false;
    const float l = 2 * std::sqrt(Sqr(rMax) - Sqr(r));
    float sp, cp;
    SinCosf(phi, &sp, &cp);
    const V3 pStart = po + r * (f.x * cp + f.y * sp) - l * f.z / 2;
    *p0 = pStart;
    *p1 = pStart + l * f.z;
    return true;
}

// PDF_Sp's projection radii and weights (bssrdf.h:238-258): pdf_i = sum over the three axes
// of PDF_Sr(rProj[a])_i * |nLocal[a]| * axisProb[a]
struct SssPdfGeom {
    float rProj[3], absN[3];
};
PHD SssPdfGeom MakeSssPdfGeom(V3 po, V3 ns, V3 pi, V3 ni) {
    const V3 d = pi - po;
    V3 x, y;
    CoordinateSystem(ns, &x, &y);  // Frame::FromZ(ns)
    const V3 dLocal(Dot(d, x), Dot(d, y), Dot(d, ns));
    const V3 nLocal(DotN(ni, x), DotN(ni, y), DotN(ni, ns));  // Frame::ToLocal(Normal3f)
    SssPdfGeom g;
    g.rProj[0] = std::sqrt(Sqr(dLocal.y) + Sqr(dLocal.z));
    g.rProj[1] = std::sqrt(Sqr(dLocal.z) + Sqr(dLocal.x));
    g.rProj[2] = std::sqrt(Sqr(dLocal.x) + Sqr(dLocal.y));
    g.absN[0] = std::fabs(nLocal.x);
    g.absN[1] = std::fabs(nLocal.y);
    g.absN[2] = std::fabs(nLocal.z);
    return g;
}
PHD float SssPdfSp(const SssTable &t, SssCoeffs c, const SssPdfGeom &g) {
    const float axisProb[3] = {.25f, .25f, .5f};
    float pdf = 0;
    for (int a = 0; a < 3; ++a) pdf = pdf + SssPdfSr(t, c, g.rProj[a]) * g.absN[a] * axisProb[a];
    return pdf;
}

// SubsurfaceFromDiffuse at one wavelength (bssrdf.h:322-333)
PHD void SssFromDiffuse(const SssTable &t, float rhoEff, float mfp, float *sigma_a, float *sigma_s) {
    const float rho = InvertCatmullRom(t.rho, t.rhoEff, kSssRho, rhoEff);
    *sigma_s = rho / mfp;
    *sigma_a = (1 - rho) / mfp;
}

// NormalizedFresnelBxDF::f (bxdfs.h:1249-1261) for radiance transport: c = 1 - 2
// FresnelMoment1(1 / eta) comes from the host (SubsurfaceDesc::fresnelC)
PHD float NormalizedFresnelF(float eta, float c, V3 wo, V3 wi) {
    if (!(wo.z * wi.z > 0)) return 0.f;  // SameHemisphere
    const float f = (1 - FrDielectric(wi.z, eta)) / (c * kPi);
    return f * Sqr(eta);
}

}  // namespace pbrt_amd
