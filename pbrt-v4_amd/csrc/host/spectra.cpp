// Host spectral setup: CIE data, dense spectra, the sRGB colour space, and the RGB ->
// sigmoid-polynomial table of pbrt (util/color.cpp:36-75, util/colorspace.cpp:25-38,
// util/spectrum.cpp:37-51,133-163,2586-2610, cmd/rgb2spec_opt.cpp:248-570).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <thread>

#include "scene.h"

namespace pbrt_amd {

static std::string g_dataDir;
void SetDataDirectory(const std::string &dir) { g_dataDir = dir; }
std::string GetDataDirectory() {
    if (!g_dataDir.empty()) return g_dataDir;
    if (const char *e = std::getenv("PBRT_AMD_DATA")) return e;
    return "pbrt-v4_amd/data";
}

static float PiecewiseLinearEval(const std::vector<float> &lambdas, const std::vector<float> &values,
                                 float lambda) {
    // util/spectrum.cpp PiecewiseLinearSpectrum::operator()
    if (lambdas.empty() || lambda < lambdas.front() || lambda > lambdas.back()) return 0;
    // FindInterval(size, lambdas[i] <= lambda)
    int sz = (int)lambdas.size();
    int size = sz - 2, first = 1;
    while (size > 0) {
        int half = size >> 1, middle = first + half;
        bool pred = lambdas[middle] <= lambda;
        first = pred ? middle + 1 : first;
        size = pred ? size - (half + 1) : half;
    }
    int o = std::min(std::max(first - 1, 0), sz - 2);
    float t = (lambda - lambdas[o]) / (lambdas[o + 1] - lambdas[o]);
    return Lerpf(t, values[o], values[o + 1]);
}

static void Invert3(const double m[3][3], double r[3][3]) {
    double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                 m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                 m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    double id = 1.0 / det;
    r[0][0] = (m[1][1] * m[2][2] - m[1][2] * m[2][1]) * id;
    r[0][1] = (m[0][2] * m[2][1] - m[0][1] * m[2][2]) * id;
    r[0][2] = (m[0][1] * m[1][2] - m[0][2] * m[1][1]) * id;
    r[1][0] = (m[1][2] * m[2][0] - m[1][0] * m[2][2]) * id;
    r[1][1] = (m[0][0] * m[2][2] - m[0][2] * m[2][0]) * id;
    r[1][2] = (m[0][2] * m[1][0] - m[0][0] * m[1][2]) * id;
    r[2][0] = (m[1][0] * m[2][1] - m[1][1] * m[2][0]) * id;
    r[2][1] = (m[0][1] * m[2][0] - m[0][0] * m[2][1]) * id;
    r[2][2] = (m[0][0] * m[1][1] - m[0][1] * m[1][0]) * id;
}

// the four spaces RGBColorSpace::Init builds (util/colorspace.cpp:83-105): name, primaries
// r, g, b (xy) and the named illuminant
const ColorSpaceDef kColorSpaceDefs[kNumColorSpaces] = {
    {"srgb", {.64, .33, .3, .6, .15, .06}, "stdillum-D65"},
    {"dci-p3", {.68, .32, .265, .690, .15, .06}, "stdillum-D65"},
    {"rec2020", {.708, .292, .170, .797, .131, .046}, "stdillum-D65"},
    {"aces2065-1", {.7347, .2653, 0., 1., .0001, -.077}, "illum-acesD60"}};

// PiecewiseLinearSpectrum::FromInterleaved(samples, normalize = true) (util/spectrum.cpp:133-163):
// extended to Lambda_min - 1 / Lambda_max + 1, then scaled by CIE_Y_integral / InnerProduct(s, Y)
static void NormalizedIlluminant(const SpectralData &d, const std::vector<float> &iv, std::vector<float> *lam,
                                 std::vector<float> *val) {
    lam->clear();
    val->clear();
    for (size_t i = 0; i + 1 < iv.size(); i += 2) {
        lam->push_back(iv[i]);
        val->push_back(iv[i + 1]);
    }
    if (lam->front() > kLambdaMin) {
        lam->insert(lam->begin(), kLambdaMin - 1);
        val->insert(val->begin(), val->front());
    }
    if (lam->back() < kLambdaMax) {
        lam->push_back(kLambdaMax + 1);
        val->push_back(val->back());
    }
    // InnerProduct(spec, &Spectra::Y()) over lambda = 395..705 in Float steps
    float integral = 0;
    for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda)
        integral += PiecewiseLinearEval(*lam, *val, lambda) * d.denseY[DenseOffset(lambda)];
    const float CIE_Y_integral = 106.856895f;
    float s = CIE_Y_integral / integral;
    for (float &v : *val) v *= s;
}

// SpectrumToPhotometric(illuminant): sum over Float lambda of Y(l) * s(l)
static float PhotometricDense(const SpectralData &d, const std::array<float, 311> &s) {
    float y = 0;
    for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda)
        y += d.denseY[DenseOffset(lambda)] * s[DenseOffset(lambda)];
    return y;
}

// RGBColorSpace's constructor (util/colorspace.cpp:23-37) in double: W = SpectrumToXYZ(illuminant),
// the primaries' XYZ (Y = 1), C = inverse(rgb) * W, XYZFromRGB = rgb * diag(C), RGBFromXYZ its inverse
static void ColorSpaceMatrices(const SpectralData &d, const std::array<float, 311> &illum, const double prim[6],
                               double xyzFromRGBOut[3][3], double rgbFromXYZOut[3][3]) {
    double X = 0, Y = 0, Z = 0;
    for (int l = 395; l <= 705; ++l) {
        X += (double)d.denseX[l - 395] * illum[l - 395];
        Y += (double)d.denseY[l - 395] * illum[l - 395];
        Z += (double)d.denseZ[l - 395] * illum[l - 395];
    }
    const double CIE_Y_integral = 106.856895;
    X /= CIE_Y_integral;
    Y /= CIE_Y_integral;
    Z /= CIE_Y_integral;
    auto fromxyY = [](double x, double y, double out[3]) {
        if (y == 0) {  // XYZ::FromxyY: a primary on y = 0 is black
            out[0] = out[1] = out[2] = 0;
            return;
        }
        out[0] = x / y;
        out[1] = 1;
        out[2] = (1 - x - y) / y;
    };
    double R[3], G[3], B[3];
    fromxyY(prim[0], prim[1], R);
    fromxyY(prim[2], prim[3], G);
    fromxyY(prim[4], prim[5], B);
    const double W[3] = {X, Y, Z};
    double rgb[3][3] = {{R[0], G[0], B[0]}, {R[1], G[1], B[1]}, {R[2], G[2], B[2]}};
    double inv[3][3];
    Invert3(rgb, inv);
    double C[3];
    for (int i = 0; i < 3; ++i) C[i] = inv[i][0] * W[0] + inv[i][1] * W[1] + inv[i][2] * W[2];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) xyzFromRGBOut[i][j] = rgb[i][j] * C[j];
    Invert3(xyzFromRGBOut, rgbFromXYZOut);
}

static SpectralData LoadSpectralData() {
    SpectralData d;
    std::string path = GetDataDirectory() + "/spectral_data.txt";
    std::ifstream in(path);
    if (!in) throw Error("cannot open spectral data file " + path);
    std::string line;
    bool haveMipLUT = false, haveSrgbLUT = false;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string name;
        size_t n;
        ls >> name >> n;
        std::vector<double> v(n);
        for (size_t i = 0; i < n; ++i) ls >> v[i];
        auto tof = [&](std::vector<float> &dst) { dst.assign(v.begin(), v.end()); };
        if (name == "CIE_X") tof(d.cieX);
        else if (name == "CIE_Y") tof(d.cieY);
        else if (name == "CIE_Z") tof(d.cieZ);
        else if (name == "CIE_lambda") tof(d.cieLambda);
        else if (name == "CIE_Illum_D6500_interleaved") tof(d.d65Interleaved);
        else if (name == "opt_cie_x") d.optX = v;
        else if (name == "opt_cie_y") d.optY = v;
        else if (name == "opt_cie_z") d.optZ = v;
        else if (name == "opt_cie_d65_raw") d.optD65Raw = v;
        else if (name == "opt_cie_d65_divisor") d.optD65Divisor = v[0];
        else if (name == "opt_xyz_to_srgb") d.optXyzToSrgb = v;
        else if (name == "opt_srgb_to_xyz") d.optSrgbToXyz = v;
        else if (name == "opt_cie_d60_raw") d.optD60Raw = v;
        else if (name == "opt_cie_d60_divisor") d.optD60Divisor = v[0];
        else if (name == "opt_xyz_to_dcip3") d.optXyzToRgb[kColorSpaceDCIP3] = v;
        else if (name == "opt_dcip3_to_xyz") d.optRgbToXyz[kColorSpaceDCIP3] = v;
        else if (name == "opt_xyz_to_rec2020") d.optXyzToRgb[kColorSpaceRec2020] = v;
        else if (name == "opt_rec2020_to_xyz") d.optRgbToXyz[kColorSpaceRec2020] = v;
        else if (name == "opt_xyz_to_aces2065_1") d.optXyzToRgb[kColorSpaceACES] = v;
        else if (name == "opt_aces2065_1_to_xyz") d.optRgbToXyz[kColorSpaceACES] = v;
        else if (name == "MIPFilterLUT" && n == 128) {
            for (int i = 0; i < 128; ++i) d.mipFilterLUT[i] = (float)v[i];
            haveMipLUT = true;
        } else if (name == "SRGBToLinearLUT" && n == 256) {
            for (int i = 0; i < 256; ++i) d.srgbToLinear[i] = (float)v[i];
            haveSrgbLUT = true;
        }
        else if (name.rfind("named:", 0) == 0) tof(d.named[name.substr(6)]);
        else if (name.rfind("illum:", 0) == 0) tof(d.illuminants[name.substr(6)]);
        else if (name.rfind("sensor:", 0) == 0) tof(d.sensors[name.substr(7)]);
        else if (name.rfind("swatch:", 0) == 0) {
            d.swatches.emplace_back();
            tof(d.swatches.back());
        } else if (name == "CIE_S_lambda") tof(d.cieSLambda);
        else if (name == "CIE_S0") tof(d.cieS0);
        else if (name == "CIE_S1") tof(d.cieS1);
        else if (name == "CIE_S2") tof(d.cieS2);
        else if (name == "NoisePerm") tof(d.noisePerm);
        else if (name.rfind("mediumpreset:", 0) == 0) {
            std::vector<float> v;
            tof(v);
            if (v.size() != 6) throw Error("malformed medium preset " + name + " in " + path);
            std::string n = name.substr(13);
            std::replace(n.begin(), n.end(), '_', ' ');
            std::array<float, 6> a;
            std::copy(v.begin(), v.end(), a.begin());
            d.mediumPresets[n] = a;
        }
    }
    if (d.cieX.size() != 471 || d.optX.size() != 95) throw Error("malformed spectral data " + path);
    if (!haveMipLUT || !haveSrgbLUT)
        throw Error("malformed spectral data " + path + ": missing " +
                    (!haveMipLUT ? std::string("MIPFilterLUT") : std::string("SRGBToLinearLUT")));
    // Spectra::Init: dense X/Y/Z over Lambda_min..Lambda_max of PiecewiseLinear(CIE_lambda, CIE_*)
    for (int l = 395; l <= 705; ++l) {
        d.denseX[l - 395] = PiecewiseLinearEval(d.cieLambda, d.cieX, (float)l);
        d.denseY[l - 395] = PiecewiseLinearEval(d.cieLambda, d.cieY, (float)l);
        d.denseZ[l - 395] = PiecewiseLinearEval(d.cieLambda, d.cieZ, (float)l);
    }
    d.optXyzToRgb[kColorSpaceSRGB] = d.optXyzToSrgb;
    d.optRgbToXyz[kColorSpaceSRGB] = d.optSrgbToXyz;
    // stdillum-D65 = PiecewiseLinearSpectrum::FromInterleaved(CIE_Illum_D6500, normalize=true)
    std::vector<float> lam, val;
    NormalizedIlluminant(d, d.d65Interleaved, &lam, &val);
    // RGBColorSpace::illuminant = DenselySampledSpectrum(stdillum-D65)
    for (int l = 395; l <= 705; ++l) d.denseD65[l - 395] = PiecewiseLinearEval(lam, val, (float)l);
    d.photometricD65 = PhotometricDense(d, d.denseD65);
    // sRGB colour space matrices (colorspace.cpp:25-38), in double
    ColorSpaceMatrices(d, d.denseD65, kColorSpaceDefs[kColorSpaceSRGB].prim, d.xyzFromRGB, d.rgbFromXYZ);
    return d;
}

const SpectralData &GetSpectralData() {
    static std::once_flag once;
    static SpectralData *data = nullptr;
    std::call_once(once, [] { data = new SpectralData(LoadSpectralData()); });
    return *data;
}

// ------------------------------------------------------------------ rgb2spec restatement
namespace {
constexpr int kRes = 64;
constexpr int kCIESamples = 95;
constexpr double kCIEMin = 360.0, kCIEMax = 830.0;
constexpr int kFine = (kCIESamples - 1) * 3 + 1;

struct OptTables {
    double lambda_tbl[kFine], rgb_tbl[3][kFine], rgb_to_xyz[3][3], xyz_to_rgb[3][3], whitepoint[3];
};

double cie_interp(const double *data, double x) {  // rgb2spec_opt.cpp:248
    x -= kCIEMin;
    x *= (kCIESamples - 1) / (kCIEMax - kCIEMin);
    int offset = (int)x;
    if (offset < 0) offset = 0;
    if (offset > kCIESamples - 2) offset = kCIESamples - 2;
    double weight = x - offset;
    return (1.0 - weight) * data[offset] + weight * data[offset + 1];
}

// init_tables(gamut) (rgb2spec_opt.cpp:408-486) for one of the four colour spaces: ACES2065-1
// integrates against its D60 table, the others against D65
const OptTables &GetOptTables(int cs) {
    static std::once_flag once[kNumColorSpaces];
    static OptTables *tabs[kNumColorSpaces] = {};
    std::call_once(once[cs], [cs] {
        const SpectralData &d = GetSpectralData();
        OptTables *t = new OptTables();
        memset(t, 0, sizeof(*t));
        const bool d60 = cs == kColorSpaceACES;
        const std::vector<double> &raw = d60 ? d.optD60Raw : d.optD65Raw;
        const double div = d60 ? d.optD60Divisor : d.optD65Divisor;
        if (raw.size() != kCIESamples || d.optXyzToRgb[cs].size() != 9 || d.optRgbToXyz[cs].size() != 9)
            throw Error(std::string("spectral data has no rgb2spec tables for colour space ") + kColorSpaceDefs[cs].name);
        double ill[kCIESamples];
        for (int i = 0; i < kCIESamples; ++i) ill[i] = raw[i] / div;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                t->xyz_to_rgb[i][j] = d.optXyzToRgb[cs][3 * i + j];
                t->rgb_to_xyz[i][j] = d.optRgbToXyz[cs][3 * i + j];
            }
        double h = (kCIEMax - kCIEMin) / (kFine - 1);
        for (int i = 0; i < kFine; ++i) {
            double lambda = kCIEMin + i * h;
            double xyz[3] = {cie_interp(d.optX.data(), lambda), cie_interp(d.optY.data(), lambda),
                             cie_interp(d.optZ.data(), lambda)},
                   I = cie_interp(ill, lambda);
            double weight = 3.0 / 8.0 * h;
            if (i == 0 || i == kFine - 1)
                ;
            else if ((i - 1) % 3 == 2)
                weight *= 2.f;
            else
                weight *= 3.f;
            t->lambda_tbl[i] = lambda;
            for (int k = 0; k < 3; ++k)
                for (int j = 0; j < 3; ++j) t->rgb_tbl[k][i] += t->xyz_to_rgb[k][j] * xyz[j] * I * weight;
            for (int k = 0; k < 3; ++k) t->whitepoint[k] += xyz[k] * I * weight;
        }
        tabs[cs] = t;
    });
    return *tabs[cs];
}

void cie_lab(const OptTables &t, double *p) {
    double X = 0.0, Y = 0.0, Z = 0.0, Xw = t.whitepoint[0], Yw = t.whitepoint[1], Zw = t.whitepoint[2];
    for (int j = 0; j < 3; ++j) {
        X += p[j] * t.rgb_to_xyz[0][j];
        Y += p[j] * t.rgb_to_xyz[1][j];
        Z += p[j] * t.rgb_to_xyz[2][j];
    }
    auto f = [](double v) -> double {
        double delta = 6.0 / 29.0;
        if (v > delta * delta * delta) return cbrt(v);
        return v / (delta * delta * 3.0) + (4.0 / 29.0);
    };
    p[0] = 116.0 * f(Y / Yw) - 16.0;
    p[1] = 500.0 * (f(X / Xw) - f(Y / Yw));
    p[2] = 200.0 * (f(Y / Yw) - f(Z / Zw));
}

void eval_residual(const OptTables &t, const double *coeffs, const double *rgb, double *residual) {
    double out[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < kFine; ++i) {
        double lambda = (t.lambda_tbl[i] - kCIEMin) / (kCIEMax - kCIEMin);
        double x = 0.0;
        for (int k = 0; k < 3; ++k) x = x * lambda + coeffs[k];
        double s = 0.5 * x / std::sqrt(1.0 + x * x) + 0.5;
        for (int j = 0; j < 3; ++j) out[j] += t.rgb_tbl[j][i] * s;
    }
    cie_lab(t, out);
    memcpy(residual, rgb, sizeof(double) * 3);
    cie_lab(t, residual);
    for (int j = 0; j < 3; ++j) residual[j] -= out[j];
}

void eval_jacobian(const OptTables &t, const double *coeffs, const double *rgb, double **jac) {
    const double eps = 1e-4;
    double r0[3], r1[3], tmp[3];
    for (int i = 0; i < 3; ++i) {
        memcpy(tmp, coeffs, sizeof(double) * 3);
        tmp[i] -= eps;
        eval_residual(t, tmp, rgb, r0);
        memcpy(tmp, coeffs, sizeof(double) * 3);
        tmp[i] += eps;
        eval_residual(t, tmp, rgb, r1);
        for (int j = 0; j < 3; ++j) jac[j][i] = (r1[j] - r0[j]) * 1.0 / (2 * eps);
    }
}

bool LUPDecompose(double **A, int N, double Tol, int *P) {
    for (int i = 0; i <= N; i++) P[i] = i;
    for (int i = 0; i < N; i++) {
        double maxA = 0.0, absA;
        int imax = i;
        for (int k = i; k < N; k++)
            if ((absA = std::fabs(A[k][i])) > maxA) {
                maxA = absA;
                imax = k;
            }
        if (maxA < Tol) return false;
        if (imax != i) {
            int j = P[i];
            P[i] = P[imax];
            P[imax] = j;
            double *ptr = A[i];
            A[i] = A[imax];
            A[imax] = ptr;
            P[N]++;
        }
        for (int j = i + 1; j < N; j++) {
            A[j][i] /= A[i][i];
            for (int k = i + 1; k < N; k++) A[j][k] -= A[j][i] * A[i][k];
        }
    }
    return true;
}

void LUPSolve(double **const A, const int *P, const double *b, int N, double *x) {
    for (int i = 0; i < N; i++) {
        x[i] = b[P[i]];
        for (int k = 0; k < i; k++) x[i] -= A[i][k] * x[k];
    }
    for (int i = N - 1; i >= 0; i--) {
        for (int k = i + 1; k < N; k++) x[i] -= A[i][k] * x[k];
        x[i] = x[i] / A[i][i];
    }
}

void gauss_newton(const OptTables &t, const double rgb[3], double coeffs[3], int it = 15) {
    for (int i = 0; i < it; ++i) {
        double J0[3], J1[3], J2[3], *J[3] = {J0, J1, J2};
        double residual[3];
        eval_residual(t, coeffs, rgb, residual);
        eval_jacobian(t, coeffs, rgb, J);
        int P[4];
        if (!LUPDecompose(J, 3, 1e-15, P)) throw Error("rgb2spec: LU decomposition failed");
        double x[3];
        LUPSolve(J, P, residual, 3, x);
        double r = 0.0;
        for (int j = 0; j < 3; ++j) {
            coeffs[j] -= x[j];
            r += residual[j] * residual[j];
        }
        double mx = std::max(std::max(coeffs[0], coeffs[1]), coeffs[2]);
        if (mx > 200)
            for (int j = 0; j < 3; ++j) coeffs[j] *= 200 / mx;
        if (r < 1e-6) break;
    }
}

double smoothstep(double x) { return x * x * (3.0 - 2.0 * x); }
}  // namespace

float RGB2SpecZNode(int k) { return (float)smoothstep(smoothstep(k / double(kRes - 1))); }

std::vector<float> RGB2SpecColumn(int l, int j, int i, int cs) {
    // rgb2spec_opt.cpp:825-875 for one (l, j, i): two warm-started chains over k
    const OptTables &t = GetOptTables(cs);
    std::vector<float> out(kRes * 3);
    const double y = j / double(kRes - 1), x = i / double(kRes - 1);
    auto store = [&](int k, const double *coeffs) {
        double c0 = 360.0, c1 = 1.0 / (830.0 - 360.0);
        double A = coeffs[0], B = coeffs[1], C = coeffs[2];
        out[3 * k + 0] = float(A * (c1 * c1));
        out[3 * k + 1] = float(B * c1 - 2 * A * c0 * (c1 * c1));
        out[3 * k + 2] = float(C - B * c0 * c1 + A * ((c0 * c1) * (c0 * c1)));
    };
    double coeffs[3], rgb[3];
    int start = kRes / 5;
    memset(coeffs, 0, sizeof(coeffs));
    for (int k = start; k < kRes; ++k) {
        double b = (double)RGB2SpecZNode(k);
        rgb[l] = b;
        rgb[(l + 1) % 3] = x * b;
        rgb[(l + 2) % 3] = y * b;
        gauss_newton(t, rgb, coeffs);
        store(k, coeffs);
    }
    memset(coeffs, 0, sizeof(coeffs));
    for (int k = start; k >= 0; --k) {
        double b = (double)RGB2SpecZNode(k);
        rgb[l] = b;
        rgb[(l + 1) % 3] = x * b;
        rgb[(l + 2) % 3] = y * b;
        gauss_newton(t, rgb, coeffs);
        store(k, coeffs);
    }
    return out;
}

static const std::vector<float> &CachedColumn(int l, int j, int i, int cs) {
    static std::mutex mu;
    static std::map<int, std::vector<float>> cache;
    std::lock_guard<std::mutex> lock(mu);
    int key = ((cs * 3 + l) * kRes + j) * kRes + i;
    auto it = cache.find(key);
    if (it == cache.end()) it = cache.emplace(key, RGB2SpecColumn(l, j, i, cs)).first;
    return it->second;
}

const std::vector<float> &RGBToSpectrumTableData() {
    static std::once_flag once;
    static std::vector<float> table;
    std::call_once(once, [] {
        const size_t nData = (size_t)3 * kRes * kRes * kRes * 3;
        table.assign(kRes + nData, 0.f);
        const std::string path = GetDataDirectory() + "/rgbspec_srgb.bin";
        {
            std::ifstream in(path, std::ios::binary);
            if (in) {
                in.read(reinterpret_cast<char *>(table.data()), (std::streamsize)(table.size() * 4));
                // a cached table is trusted only when its size, its z nodes and three sampled
                // columns equal a fresh computation bit for bit; otherwise it is rebuilt
                bool ok = in.gcount() == (std::streamsize)(table.size() * 4) && in.peek() == EOF;
                for (int k = 0; ok && k < kRes; ++k) ok = table[k] == RGB2SpecZNode(k);
                const int probe[3][3] = {{0, 0, 0}, {1, kRes / 2, kRes / 3}, {2, kRes - 1, kRes - 2}};
                for (int p = 0; ok && p < 3; ++p) {
                    const int l = probe[p][0], j = probe[p][1], i = probe[p][2];
                    const std::vector<float> c = RGB2SpecColumn(l, j, i, kColorSpaceSRGB);
                    for (int k = 0; ok && k < kRes; ++k)
                        for (int ci = 0; ci < 3; ++ci)
                            ok = ok && table[kRes + ((((size_t)l * kRes + k) * kRes + j) * kRes + i) * 3 + ci] ==
                                           c[3 * k + ci];
                }
                if (ok) return;
            }
        }
        // rgb2spec_opt.cpp:800-880: every (maxc, y, x) column, independent of the others
        for (int k = 0; k < kRes; ++k) table[k] = RGB2SpecZNode(k);
        const int nCols = 3 * kRes * kRes;
        unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (int col = (int)t; col < nCols; col += (int)nt) {
                    const int l = col / (kRes * kRes), j = (col / kRes) % kRes, i = col % kRes;
                    const std::vector<float> c = RGB2SpecColumn(l, j, i, kColorSpaceSRGB);
                    for (int k = 0; k < kRes; ++k)
                        for (int ci = 0; ci < 3; ++ci)
                            table[kRes + ((((size_t)l * kRes + k) * kRes + j) * kRes + i) * 3 + ci] = c[3 * k + ci];
                }
            });
        for (auto &x : th) x.join();
        std::ofstream out(path, std::ios::binary);
        if (out) out.write(reinterpret_cast<const char *>(table.data()), (std::streamsize)(table.size() * 4));
    });
    return table;
}

std::array<float, 3> RGBToSigmoidCoeffs(float r, float g, float b, int cs) {
    // RGBColorSpace::ToRGBCoeffs -> RGBToSpectrumTable::operator() (util/color.cpp:36-75)
    float rgb[3] = {std::max(0.f, r), std::max(0.f, g), std::max(0.f, b)};
    if (rgb[0] == rgb[1] && rgb[1] == rgb[2])
        return {0.f, 0.f, (rgb[0] - .5f) / std::sqrt(rgb[0] * (1 - rgb[0]))};
    int maxc = (rgb[0] > rgb[1]) ? ((rgb[0] > rgb[2]) ? 0 : 2) : ((rgb[1] > rgb[2]) ? 1 : 2);
    float z = rgb[maxc];
    float x = rgb[(maxc + 1) % 3] * (kRes - 1) / z;
    float y = rgb[(maxc + 2) % 3] * (kRes - 1) / z;
    int xi = std::min((int)x, kRes - 2), yi = std::min((int)y, kRes - 2);
    float zNodes[kRes];
    for (int k = 0; k < kRes; ++k) zNodes[k] = RGB2SpecZNode(k);
    int zi;
    {
        int size = kRes - 2, first = 1;
        while (size > 0) {
            int half = size >> 1, middle = first + half;
            bool pred = zNodes[middle] < z;
            first = pred ? middle + 1 : first;
            size = pred ? size - (half + 1) : half;
        }
        zi = std::min(std::max(first - 1, 0), kRes - 2);
    }
    float dx = x - xi, dy = y - yi, dz = (z - zNodes[zi]) / (zNodes[zi + 1] - zNodes[zi]);
    std::array<float, 3> c;
    for (int ci = 0; ci < 3; ++ci) {
        auto co = [&](int ddx, int ddy, int ddz) {
            const std::vector<float> &col = CachedColumn(maxc, yi + ddy, xi + ddx, cs);
            return col[3 * (zi + ddz) + ci];
        };
        c[ci] = Lerpf(dz, Lerpf(dy, Lerpf(dx, co(0, 0, 0), co(1, 0, 0)), Lerpf(dx, co(0, 1, 0), co(1, 1, 0))),
                      Lerpf(dy, Lerpf(dx, co(0, 0, 1), co(1, 0, 1)), Lerpf(dx, co(0, 1, 1), co(1, 1, 1))));
    }
    return c;
}

std::array<float, 311> DenseRGBIlluminant(float r, float g, float b, int cs) {
    // DenselySampledSpectrum(RGBIlluminantSpectrum(cs, rgb)) (util/spectrum.cpp:246-251)
    const std::array<float, 311> &ill = GetColorSpace(cs).illuminant;
    float m = std::max({r, g, b});
    float scale = 2 * m;
    std::array<float, 3> c = scale ? RGBToSigmoidCoeffs(r / scale, g / scale, b / scale, cs)
                                   : RGBToSigmoidCoeffs(0, 0, 0, cs);
    std::array<float, 311> out;
    for (int l = 395; l <= 705; ++l) {
        float lambda = (float)l;
        out[l - 395] = scale * SigmoidPolynomial(c[0], c[1], c[2], lambda) * ill[DenseOffset(lambda)];
    }
    return out;
}

std::array<float, 311> DenseRGBUnbounded(float r, float g, float b, int cs) {
    // DenselySampledSpectrum(RGBUnboundedSpectrum(cs, rgb)) (util/spectrum.cpp:230-244)
    float m = std::max({r, g, b});
    float scale = 2 * m;
    std::array<float, 3> c = scale ? RGBToSigmoidCoeffs(r / scale, g / scale, b / scale, cs)
                                   : RGBToSigmoidCoeffs(0, 0, 0, cs);
    std::array<float, 311> out;
    for (int l = 395; l <= 705; ++l) out[l - 395] = scale * SigmoidPolynomial(c[0], c[1], c[2], (float)l);
    return out;
}

}  // namespace pbrt_amd

namespace pbrt_amd {
static void WhiteXY(const std::array<float, 311> &s, float *x, float *y);
static bool Invert3f(const float m[3][3], float r[3][3]);

// pbrt's InnerProduct(a, b, c, d, e, f) (util/math.h): TwoProd / TwoSum compensated, rounded once
static float CompInner3(float a0, float b0, float a1, float b1, float a2, float b2) {
    auto twoProd = [](float a, float b, float *err) {
        const float ab = a * b;
        *err = std::fma(a, b, -ab);
        return ab;
    };
    auto twoSum = [](float a, float b, float *err) {
        const float s = a + b, delta = s - a;
        *err = (a - (s - delta)) + (b - delta);
        return s;
    };
    float e2, e1, e0, es1, es0;
    const float p2 = twoProd(a2, b2, &e2);  // innermost term: InnerProduct(a2, b2)
    const float p1 = twoProd(a1, b1, &e1);
    const float s1 = twoSum(p1, p2, &es1);
    const float err1 = e1 + (e2 + es1);
    const float p0 = twoProd(a0, b0, &e0);
    const float s0 = twoSum(p0, s1, &es0);
    const float err0 = e0 + (err1 + es0);
    return s0 + err0;
}
void MulCompensated3(const float a[3][3], const float b[3][3], float r[3][3]) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[i][j] = CompInner3(a[i][0], b[0][j], a[i][1], b[1][j], a[i][2], b[2][j]);
}

// RGBColorSpace's constructor in pbrt's own float arithmetic (util/colorspace.cpp:23-37):
// W = SpectrumToXYZ(illuminant) (float InnerProducts / CIE_Y_integral), XYZ::FromxyY of the
// float primaries, C = Mul(Inverse(rgb), W), XYZFromRGB = rgb * Diag(C) (compensated products,
// one rounding each), RGBFromXYZ = Inverse(XYZFromRGB) (cofactors by DifferenceOfProducts)
static void ColorSpaceMatricesF(const SpectralData &d, const std::array<float, 311> &illum, const float prim[6],
                                float xyzFromRGB[3][3], float rgbFromXYZ[3][3]) {
    const float CIE_Y_integral = 106.856895f;
    float X = 0, Y = 0, Z = 0;
    for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda) {
        const int o = DenseOffset(lambda);
        X += d.denseX[o] * illum[o];
        Y += d.denseY[o] * illum[o];
        Z += d.denseZ[o] * illum[o];
    }
    const float W[3] = {X / CIE_Y_integral, Y / CIE_Y_integral, Z / CIE_Y_integral};
    auto fromxyY = [](float x, float y, float o[3]) {
        if (y == 0) {
            o[0] = o[1] = o[2] = 0;
            return;
        }
        o[0] = x * 1.f / y;
        o[1] = 1.f;
        o[2] = (1 - x - y) * 1.f / y;
    };
    float R[3], G[3], B[3];
    fromxyY(prim[0], prim[1], R);
    fromxyY(prim[2], prim[3], G);
    fromxyY(prim[4], prim[5], B);
    const float rgb[3][3] = {{R[0], G[0], B[0]}, {R[1], G[1], B[1]}, {R[2], G[2], B[2]}};
    float inv[3][3];
    if (!Invert3f(rgb, inv)) throw Error("colour space primaries are degenerate");
    float C[3];
    for (int i = 0; i < 3; ++i) {
        C[i] = 0;
        for (int j = 0; j < 3; ++j) C[i] += inv[i][j] * W[j];
    }
    const float diag[3][3] = {{C[0], 0, 0}, {0, C[1], 0}, {0, 0, C[2]}};
    MulCompensated3(rgb, diag, xyzFromRGB);
    if (!Invert3f(xyzFromRGB, rgbFromXYZ)) throw Error("colour space matrix is singular");
}

// RGBColorSpace::sRGB / DCI_P3 / Rec2020 / ACES2065_1 (util/colorspace.cpp:83-105): the
// densely sampled named illuminant, its photometric integral, white point and matrices
const ColorSpaceDesc &GetColorSpace(int cs) {
    if (cs < 0 || cs >= kNumColorSpaces) throw Error("colour space index out of range");
    static std::once_flag once;
    static ColorSpaceDesc *spaces = nullptr;
    std::call_once(once, [] {
        const SpectralData &d = GetSpectralData();
        spaces = new ColorSpaceDesc[kNumColorSpaces];
        for (int k = 0; k < kNumColorSpaces; ++k) {
            ColorSpaceDesc &c = spaces[k];
            const ColorSpaceDef &def = kColorSpaceDefs[k];
            c.name = def.name;
            for (int i = 0; i < 6; ++i) c.prim[i] = (float)def.prim[i];
            if (std::string(def.illuminant) == "stdillum-D65") {
                c.illuminant = d.denseD65;
            } else {
                auto it = d.illuminants.find(def.illuminant);
                if (it == d.illuminants.end())
                    throw Error(std::string("spectral data lacks the illuminant ") + def.illuminant);
                std::vector<float> lam, val;
                NormalizedIlluminant(d, it->second, &lam, &val);
                for (int l = 395; l <= 705; ++l) c.illuminant[l - 395] = PiecewiseLinearEval(lam, val, (float)l);
            }
            c.photometric = PhotometricDense(d, c.illuminant);
            ColorSpaceMatrices(d, c.illuminant, def.prim, c.xyzFromRGB, c.rgbFromXYZ);
            ColorSpaceMatricesF(d, c.illuminant, c.prim, c.xyzFromRGBf, c.rgbFromXYZf);
            WhiteXY(c.illuminant, &c.w[0], &c.w[1]);
        }
    });
    return spaces[cs];
}

int ColorSpaceByName(const std::string &n) {
    std::string name = n;
    std::transform(name.begin(), name.end(), name.begin(), ::tolower);  // RGBColorSpace::GetNamed
    for (int k = 0; k < kNumColorSpaces; ++k)
        if (name == kColorSpaceDefs[k].name) return k;
    return -1;
}

PLSpectrumDesc NamedPiecewiseLinear(const std::string &name) {
    const SpectralData &sd = GetSpectralData();
    const auto &named = sd.named;
    auto it = named.find(name);
    if (it == named.end()) {
        // the standard illuminants are registered normalised to luminance 1 (spectrum.cpp:2604-2650)
        auto il = sd.illuminants.find(name);
        if (il == sd.illuminants.end())
            throw Error("unknown named spectrum \"" + name + "\" (spectrum files are not supported)");
        PLSpectrumDesc d;
        NormalizedIlluminant(sd, il->second, &d.lambda, &d.value);
        return d;
    }
    const std::vector<float> &v = it->second;
    PLSpectrumDesc d;
    if (v[0] > kLambdaMin) {
        d.lambda.push_back(kLambdaMin - 1);
        d.value.push_back(v[1]);
    }
    for (size_t i = 0; i + 1 < v.size(); i += 2) {
        d.lambda.push_back(v[i]);
        d.value.push_back(v[i + 1]);
    }
    if (d.lambda.back() < kLambdaMax) {
        d.lambda.push_back(kLambdaMax + 1);
        d.value.push_back(d.value.back());
    }
    return d;
}
}  // namespace pbrt_amd

namespace pbrt_amd {
// BlackbodySpectrum (util/spectrum.h:530-560): Blackbody (core.h) over its value at Wien's peak
float BlackbodyNormalized(float lambda, float T) { return Blackbody(lambda, T) * BlackbodyNorm(T); }

// PiecewiseLinearSpectrum::FromInterleaved(samples, normalize = false) (util/spectrum.cpp:
// 133-163): split, then extended to Lambda_min - 1 / Lambda_max + 1 by the end values
static void SplitInterleaved(const std::vector<float> &iv, std::vector<float> *lam, std::vector<float> *val) {
    lam->clear();
    val->clear();
    for (size_t i = 0; i + 1 < iv.size(); i += 2) {
        lam->push_back(iv[i]);
        val->push_back(iv[i + 1]);
    }
    if (lam->front() > kLambdaMin) {
        lam->insert(lam->begin(), kLambdaMin - 1);
        val->insert(val->begin(), val->front());
    }
    if (lam->back() < kLambdaMax) {
        lam->push_back(kLambdaMax + 1);
        val->push_back(val->back());
    }
}
static std::array<float, 311> DenseOf(const std::vector<float> &lam, const std::vector<float> &val) {
    std::array<float, 311> d;
    for (int l = 395; l <= 705; ++l) d[l - 395] = PiecewiseLinearEval(lam, val, (float)l);
    return d;
}
// InnerProduct(f, g) over Float lambda = Lambda_min..Lambda_max (util/spectrum.h)
static float InnerDense(const std::array<float, 311> &f, const std::array<float, 311> &g) {
    float s = 0;
    for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda) s += f[DenseOffset(lambda)] * g[DenseOffset(lambda)];
    return s;
}
typedef std::array<std::array<float, 3>, 3> M3;
// SquareMatrix<3> * SquareMatrix<3> (util/math.h:1487-1495): one compensated InnerProduct per entry
static M3 Mul3(const M3 &a, const M3 &b) {
    M3 r{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r[i][j] = CompInner3(a[i][0], b[0][j], a[i][1], b[1][j], a[i][2], b[2][j]);
    return r;
}
// SpectrumToXYZ(s).xy() (util/color.cpp)
static void WhiteXY(const std::array<float, 311> &s, float *x, float *y) {
    const SpectralData &d = GetSpectralData();
    const float CIE_Y_integral = 106.856895f;
    const float X = InnerDense(d.denseX, s) / CIE_Y_integral, Y = InnerDense(d.denseY, s) / CIE_Y_integral,
                Z = InnerDense(d.denseZ, s) / CIE_Y_integral;
    *x = X / (X + Y + Z);
    *y = Y / (X + Y + Z);
}
// WhiteBalance(srcWhite, targetWhite) (util/color.h:551-560): Bradford
static M3 WhiteBalanceM(float sx, float sy, float tx, float ty) {
    const M3 LMSFromXYZ = {{{0.8951f, 0.2664f, -0.1614f}, {-0.7502f, 1.7135f, 0.0367f}, {0.0389f, -0.0685f, 1.0296f}}};
    const M3 XYZFromLMS = {{{0.986993f, -0.147054f, 0.159963f}, {0.432305f, 0.51836f, 0.0492912f},
                            {-0.00852866f, 0.0400428f, 0.968487f}}};
    auto fromxyY = [](float x, float y) { return std::array<float, 3>{x / y, 1.f, (1 - x - y) / y}; };
    const std::array<float, 3> src = fromxyY(sx, sy), dst = fromxyY(tx, ty);
    float srcL[3], dstL[3];
    for (int i = 0; i < 3; ++i) {
        srcL[i] = LMSFromXYZ[i][0] * src[0] + LMSFromXYZ[i][1] * src[1] + LMSFromXYZ[i][2] * src[2];
        dstL[i] = LMSFromXYZ[i][0] * dst[0] + LMSFromXYZ[i][1] * dst[1] + LMSFromXYZ[i][2] * dst[2];
    }
    M3 D{};
    for (int i = 0; i < 3; ++i) D[i][i] = dstL[i] / srcL[i];
    return Mul3(Mul3(XYZFromLMS, D), LMSFromXYZ);
}

// Inverse(SquareMatrix<3>) (util/math.h:1449-1469): cofactors by DifferenceOfProducts over the
// FMA-based Determinant (util/math.h:1420-1426), in float
static float DoP(float a, float b, float c, float d) {
    const float cd = c * d;
    return std::fma(a, b, -cd) + std::fma(-c, d, cd);
}
static bool Invert3f(const float m[3][3], float r[3][3]) {
    const float minor12 = DoP(m[1][1], m[2][2], m[1][2], m[2][1]);
    const float minor02 = DoP(m[1][0], m[2][2], m[1][2], m[2][0]);
    const float minor01 = DoP(m[1][0], m[2][1], m[1][1], m[2][0]);
    const float det = std::fma(m[0][2], minor01, DoP(m[0][0], minor12, m[0][1], minor02));
    if (det == 0) return false;
    const float invDet = 1 / det;
    r[0][0] = invDet * DoP(m[1][1], m[2][2], m[1][2], m[2][1]);
    r[1][0] = invDet * DoP(m[1][2], m[2][0], m[1][0], m[2][2]);
    r[2][0] = invDet * DoP(m[1][0], m[2][1], m[1][1], m[2][0]);
    r[0][1] = invDet * DoP(m[0][2], m[2][1], m[0][1], m[2][2]);
    r[1][1] = invDet * DoP(m[0][0], m[2][2], m[0][2], m[2][0]);
    r[2][1] = invDet * DoP(m[0][1], m[2][0], m[0][0], m[2][1]);
    r[0][2] = invDet * DoP(m[0][1], m[1][2], m[0][2], m[1][1]);
    r[1][2] = invDet * DoP(m[0][2], m[1][0], m[0][0], m[1][2]);
    r[2][2] = invDet * DoP(m[0][0], m[1][1], m[0][1], m[1][0]);
    return true;
}

std::array<float, 311> DenseCIEDaylight(float temperature) {
    const SpectralData &d = GetSpectralData();
    const float cct = temperature * 1.4388f / 1.4380f;
    std::array<float, 311> out;
    if (cct < 4000) {  // CIE D ill-defined: a normalised blackbody
        for (int l = 395; l <= 705; ++l) out[l - 395] = BlackbodyNormalized((float)l, cct);
        return out;
    }
    if (d.cieS0.size() != 107) throw Error("malformed spectral data: no CIE daylight basis");
    float x;
    if (cct <= 7000)
        x = -4.607f * 1e9f / (cct * cct * cct) + 2.9678f * 1e6f / (cct * cct) + 0.09911f * 1e3f / cct + 0.244063f;
    else
        x = -2.0064f * 1e9f / (cct * cct * cct) + 1.9018f * 1e6f / (cct * cct) + 0.24748f * 1e3f / cct + 0.23704f;
    const float y = -3 * x * x + 2.870f * x - 0.275f;
    const float M = 0.0241f + 0.2562f * x - 0.7341f * y;
    const float M1 = (-1.3515f - 1.7703f * x + 5.9114f * y) / M;
    const float M2 = (0.0300f - 31.4424f * x + 30.0717f * y) / M;
    std::vector<float> v(107);
    for (int i = 0; i < 107; ++i) v[i] = (float)((d.cieS0[i] + d.cieS1[i] * M1 + d.cieS2[i] * M2) * 0.01);
    return DenseOf(d.cieSLambda, v);
}

PixelSensorDesc BuildPixelSensor(const std::string &name, float whiteBalanceTemp, int csId) {
    const SpectralData &d = GetSpectralData();
    const ColorSpaceDesc &cs = GetColorSpace(csId);
    PixelSensorDesc s{};
    // PixelSensor::Create: named sensors white-balance to 6500 K unless told otherwise
    if (name != "cie1931" && whiteBalanceTemp == 0) whiteBalanceTemp = 6500;
    const bool haveIllum = whiteBalanceTemp != 0;
    s.illum.fill(0.f);
    if (haveIllum) s.illum = DenseCIEDaylight(whiteBalanceTemp);
    // the output colour space's white (RGBColorSpace ctor: SpectrumToXYZ(illuminant).xy())
    const float wx = cs.w[0], wy = cs.w[1];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) s.xyzFromSensorRGB[i][j] = i == j ? 1.f : 0.f;
    if (name == "cie1931") {
        s.r = d.denseX;
        s.g = d.denseY;
        s.b = d.denseZ;
        if (haveIllum) {
            float sx, sy;
            WhiteXY(s.illum, &sx, &sy);
            const M3 wb = WhiteBalanceM(sx, sy, wx, wy);
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) s.xyzFromSensorRGB[i][j] = wb[i][j];
        }
        return s;
    }
    auto curve = [&](const char *c) {
        auto it = d.sensors.find(name + c);
        if (it == d.sensors.end()) throw Error(name + ": unknown sensor type");
        std::vector<float> lam, val;
        SplitInterleaved(it->second, &lam, &val);
        return DenseOf(lam, val);
    };
    s.r = curve("_r");
    s.g = curve("_g");
    s.b = curve("_b");
    if (d.swatches.size() != 24) throw Error("malformed spectral data: no ColorChecker swatches");
    // ProjectReflectance (film.h:119-131) of the swatches: camera RGB under the white-balance
    // illuminant, XYZ under the colour space's illuminant scaled by sensorWhiteY / sensorWhiteG
    float rgbCamera[24][3], xyzOutput[24][3];
    const float sensorWhiteG = InnerDense(s.illum, s.g), sensorWhiteY = InnerDense(s.illum, d.denseY);
    for (int i = 0; i < 24; ++i) {
        std::vector<float> lam, val;
        SplitInterleaved(d.swatches[i], &lam, &val);
        float gi = 0, r3[3] = {0, 0, 0}, gx = 0, x3[3] = {0, 0, 0};
        for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda) {
            const int o = DenseOffset(lambda);
            const float rl = PiecewiseLinearEval(lam, val, lambda);
            gi += s.g[o] * s.illum[o];
            r3[0] += s.r[o] * rl * s.illum[o];
            r3[1] += s.g[o] * rl * s.illum[o];
            r3[2] += s.b[o] * rl * s.illum[o];
            gx += d.denseY[o] * cs.illuminant[o];
            x3[0] += d.denseX[o] * rl * cs.illuminant[o];
            x3[1] += d.denseY[o] * rl * cs.illuminant[o];
            x3[2] += d.denseZ[o] * rl * cs.illuminant[o];
        }
        for (int c = 0; c < 3; ++c) {
            rgbCamera[i][c] = r3[c] / gi;
            xyzOutput[i][c] = (x3[c] / gx) * (sensorWhiteY / sensorWhiteG);
        }
    }
    // LinearLeastSquares<3> (util/math.h:702-719): AtA and AtB accumulated in float,
    // Transpose(Inverse(AtA) * AtB) with pbrt's float 3x3 cofactor inverse and the compensated
    // SquareMatrix<3> product (InnerProduct: a correctly rounded float dot product)
    float AtA[3][3] = {}, AtB[3][3] = {};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int r = 0; r < 24; ++r) {
                AtA[i][j] += rgbCamera[r][i] * rgbCamera[r][j];
                AtB[i][j] += rgbCamera[r][i] * xyzOutput[r][j];
            }
    float inv[3][3];
    if (!Invert3f(AtA, inv)) throw Error("Sensor XYZ from RGB matrix could not be solved.");
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            s.xyzFromSensorRGB[j][i] = CompInner3(inv[i][0], AtB[0][j], inv[i][1], AtB[1][j], inv[i][2], AtB[2][j]);
    return s;
}
}  // namespace pbrt_amd
