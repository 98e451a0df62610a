// BSSRDF tables for SubsurfaceMaterial (materials.h:772-866): ComputeBeamDiffusionBSSRDF
// (bssrdf.cpp:124-155) over the photon beam diffusion profile, BeamDiffusionMS / SS
// (bssrdf.cpp:26-108), with FresnelMoment1 / 2 (util/scattering.cpp:10-31) and
// IntegrateCatmullRom (util/math.cpp:267-288).  Host float arithmetic in pbrt's operation
// order with libm's exp / log where pbrt calls them (std::exp through FastExp's CPU form,
// SampleExponential's std::log); the rows are independent, as in pbrt's ParallelFor.
#include "../core/bssrdf.h"
#include "scene.h"

namespace pbrt_amd {

// util/scattering.cpp:10-31; FresnelMoment1's eta^3 coefficient is a double literal in pbrt,
// so that term and the rest of its sum are evaluated in double
float FresnelMoment1(float eta) {
    const float eta2 = eta * eta, eta3 = eta2 * eta, eta4 = eta3 * eta, eta5 = eta4 * eta;
    if (eta < 1)
        return 0.45966f - 1.73965f * eta + 3.37668f * eta2 - 3.904945 * eta3 + 2.49277f * eta4 - 0.68441f * eta5;
    return -4.61686f + 11.1136f * eta - 10.4646f * eta2 + 5.11455f * eta3 - 1.27198f * eta4 + 0.12746f * eta5;
}
float FresnelMoment2(float eta) {
    const float eta2 = eta * eta, eta3 = eta2 * eta, eta4 = eta3 * eta, eta5 = eta4 * eta;
    if (eta < 1) return 0.27614f - 0.87350f * eta + 1.12077f * eta2 - 0.65095f * eta3 + 0.07883f * eta4 + 0.04860f * eta5;
    const float r_eta = 1 / eta, r_eta2 = r_eta * r_eta, r_eta3 = r_eta2 * r_eta;
    return -547.033f + 45.3087f * r_eta3 - 218.725f * r_eta2 + 458.843f * r_eta + 404.557f * eta - 189.519f * eta2 +
           54.9327f * eta3 - 9.00603f * eta4 + 0.63942f * eta5;
}

static float BeamDiffusionMS(float sigma_s, float sigma_a, float g, float eta, float r) {
    const int nSamples = 100;
    float Ed = 0;
    const float sigmap_s = sigma_s * (1 - g);
    const float sigmap_t = sigma_a + sigmap_s;
    const float rhop = sigmap_s / sigmap_t;
    const float D_g = (2 * sigma_a + sigmap_s) / (3 * sigmap_t * sigmap_t);
    const float sigma_tr = SafeSqrt(sigma_a / D_g);
    const float fm1 = FresnelMoment1(eta), fm2 = FresnelMoment2(eta);
    const float ze = -2 * D_g * (1 + 3 * fm2) / (1 - 2 * fm1);
    const float cPhi = 0.25f * (1 - 2 * fm1), cE = 0.5f * (1 - 3 * fm2);
    for (int i = 0; i < nSamples; ++i) {
        const float zr = SampleExponential((i + 0.5f) / nSamples, sigmap_t);
        const float zv = -zr + 2 * ze;
        const float dr = std::sqrt(Sqr(r) + Sqr(zr)), dv = std::sqrt(Sqr(r) + Sqr(zv));
        const float phiD = kInv4Pi / D_g * (FastExp(-sigma_tr * dr) / dr - FastExp(-sigma_tr * dv) / dv);
        const float EDn = kInv4Pi * (zr * (1 + sigma_tr * dr) * FastExp(-sigma_tr * dr) / (dr * dr * dr) -
                                     zv * (1 + sigma_tr * dv) * FastExp(-sigma_tr * dv) / (dv * dv * dv));
        const float E = phiD * cPhi + EDn * cE;
        const float kappa = 1 - FastExp(-2 * sigmap_t * (dr + zr));
        Ed += kappa * rhop * rhop * E;
    }
    return Ed / nSamples;
}

static float BeamDiffusionSS(float sigma_s, float sigma_a, float g, float eta, float r) {
    const float sigma_t = sigma_a + sigma_s, rho = sigma_s / sigma_t;
    const float tCrit = r * SafeSqrt(Sqr(eta) - 1);
    float Ess = 0;
    const int nSamples = 100;
    for (int i = 0; i < nSamples; ++i) {
        const float ti = tCrit + SampleExponential((i + 0.5f) / nSamples, sigma_t);
        const float d = std::sqrt(Sqr(r) + Sqr(ti));
        const float cosTheta_o = ti / d;
        Ess += rho * FastExp(-sigma_t * (d + tCrit)) / Sqr(d) * HenyeyGreenstein(cosTheta_o, g) *
               (1 - FrDielectric(-cosTheta_o, eta)) * std::fabs(cosTheta_o);
    }
    return Ess / nSamples;
}

static float IntegrateCatmullRom(const float *nodes, const float *f, int n, float *cdf) {
    float sum = 0;
    cdf[0] = 0;
    for (int i = 0; i < n - 1; ++i) {
        const float x0 = nodes[i], x1 = nodes[i + 1];
        const float f0 = f[i], f1 = f[i + 1];
        const float width = x1 - x0;
        const float d0 = (i > 0) ? width * (f1 - f[i - 1]) / (x1 - nodes[i - 1]) : (f1 - f0);
        const float d1 = (i + 2 < n) ? width * (f[i + 2] - f0) / (nodes[i + 2] - x0) : (f1 - f0);
        sum += width * ((f0 + f1) / 2 + (d0 - d1) / 12);
        cdf[i + 1] = sum;
    }
    return sum;
}

std::vector<float> ComputeBeamDiffusionTable(float g, float eta) {
    std::vector<float> out(kSssTableFloats, 0.f);
    float *rho = out.data(), *radius = rho + kSssRho, *profile = radius + kSssRadius;
    float *rhoEff = profile + kSssRho * kSssRadius, *cdf = rhoEff + kSssRho;
    radius[0] = 0;
    radius[1] = 2.5e-3f;
    for (int i = 2; i < kSssRadius; ++i) radius[i] = radius[i - 1] * 1.2f;
    for (int i = 0; i < kSssRho; ++i) rho[i] = (1 - FastExp(-8 * i / (float)(kSssRho - 1))) / (1 - FastExp(-8));
    for (int i = 0; i < kSssRho; ++i) {
        for (int j = 0; j < kSssRadius; ++j) {
            const float rh = rho[i], r = radius[j];
            profile[i * kSssRadius + j] =
                2 * kPi * r * (BeamDiffusionSS(rh, 1 - rh, g, eta, r) + BeamDiffusionMS(rh, 1 - rh, g, eta, r));
        }
        rhoEff[i] = IntegrateCatmullRom(radius, profile + i * kSssRadius, kSssRadius, cdf + i * kSssRadius);
    }
    return out;
}

}  // namespace pbrt_amd
