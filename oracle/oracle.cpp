// oracle/oracle.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of pbrt-v4's wavefront
// path integrator (equivalently the CPU VolPathIntegrator for medium-free, non-specular
// paths: identical sample-dimension schedule, MIS and RR) for the scene
// subset the MI355X path supports.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg load this library, as the checker; the product never links it.
//
// It is written independently of pbrt-v4_amd/csrc: scalar, one path at a time, full
// 31-wavelength SampledSpectrum arithmetic for beta, r_u, r_l and L, spectral L converted
// to sensor RGB once per sample exactly as RGBFilm::AddSample does, its own BVH, its own
// Halton digit-permutation tables.  It consumes the loaded scene through the flat C view
// (pbrt_scene_flat) so that the scene description is identical on both sides.
//
// Reference functions restated (file:line in /root/reference/src/pbrt):
//   WavefrontPathIntegrator::Render / stages    wavefront/integrator.cpp:290-573,
//     wavefront/camera.cpp:31-80, samples.cpp:29-66, surfscatter.cpp:57-328,
//     intersect.h:16-156, film.cpp:13-39
//   HaltonSampler                              samplers.h:33-141, samplers.cpp:32-52,
//     util/lowdiscrepancy.h:25-140, util/hash.h:19-106, util/math.h:728-756
//   IntersectTriangle / InteractionFromIntersection / Sample / PDF
//                                              shapes.cpp:172-273, shapes.h:884-1174
//   sampling                                   util/sampling.h:79-420, util/sampling.cpp:28-175
//   BVHLightSampler::Sample / PMF, Importance  lightsamplers.h:130-403
//   DiffuseBxDF / BSDF                         bxdfs.h:30-82, bsdf.h:60-135
//   DiffuseAreaLight::L / SampleLi / PDF_Li    lights.h:443-480, lights.cpp:743-781
//   RGBFilm::AddSample / PixelSensor           film.h:95-100, 241-258
//   OffsetRayOrigin / SpawnRay(To)             ray.h:78-111
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../include/pbrt_amd.h"

namespace oracle {

typedef float Float;
static constexpr int NS = 31;
static constexpr Float Pi = 3.14159265358979323846f, InvPi = 0.31830988618379067154f;
static constexpr Float PiOver2 = 1.57079632679489661923f, PiOver4 = 0.78539816339744830961f;
static constexpr Float Infinity = std::numeric_limits<Float>::infinity();
static constexpr Float MachineEpsilon = std::numeric_limits<Float>::epsilon() * 0.5f;
static constexpr Float OneMinusEpsilon = 0x1.fffffep-1f;
static constexpr Float ShadowEpsilon = 0.0001f;
static constexpr Float LambdaMin = 395, LambdaMax = 705;

static inline constexpr Float gamma(int n) { return (n * MachineEpsilon) / (1 - n * MachineEpsilon); }
static inline Float Sqr(Float x) { return x * x; }
static inline Float Clamp(Float v, Float lo, Float hi) { return v < lo ? lo : (v > hi ? hi : v); }
static inline Float Lerp(Float t, Float a, Float b) { return (1 - t) * a + t * b; }
static inline Float SafeSqrt(Float x) { return std::sqrt(std::max<Float>(0.f, x)); }
// Transcendentals, in one of two modes (oracle_set_math_mode):
//   0 (default) libm's float functions, as the reference CPU build calls them.  This is also what
//     the GPU kernels compute: their core/detmath.h restates glibc's sinf, cosf, expf, logf, asinf,
//     acosf, atan2f, tanf and sinhf bit for bit (tools/detmath_exhaustive.cpp), so the GPU parity
//     tests compare against this mode and device decisions that hash or seed from a ray's bits
//     (medium RNG, wavefront/media.cpp:44; alpha tests, gpu/optix.cu:197-243; mix choices,
//     materials.h:285-294) follow the oracle's;
//   1 correctly rounded (double evaluation, one rounding), an ulp away from libm in a few per cent
//     of calls: the sensitivity check of tests/test_gpu_media.py.
// Mode 2 (round 5's restated device polynomials) is gone: it is mode 0 now.
static int g_mathMode = 0;
static inline Float CRSin(Float x) { return g_mathMode == 1 ? (Float)std::sin((double)x) : std::sin(x); }
static inline Float CRCos(Float x) { return g_mathMode == 1 ? (Float)std::cos((double)x) : std::cos(x); }
static inline Float CRExp(Float x) { return g_mathMode == 1 ? (Float)std::exp((double)x) : std::exp(x); }
static inline Float CRTan(Float x) { return g_mathMode == 1 ? (Float)std::tan((double)x) : std::tan(x); }
static inline Float CRSinh(Float x) { return g_mathMode == 1 ? (Float)std::sinh((double)x) : std::sinh(x); }
static inline Float CRLog(Float x) { return g_mathMode == 1 ? (Float)std::log((double)x) : std::log(x); }
static inline Float CRATan2(Float y, Float x) {
    return g_mathMode == 1 ? (Float)std::atan2((double)y, (double)x) : std::atan2(y, x);
}
static inline Float SafeASin(Float x) {
    return g_mathMode == 1 ? (Float)std::asin((double)Clamp(x, -1, 1)) : std::asin(Clamp(x, -1, 1));
}
static inline Float SafeACos(Float x) {
    return g_mathMode == 1 ? (Float)std::acos((double)Clamp(x, -1, 1)) : std::acos(Clamp(x, -1, 1));
}
static inline Float DifferenceOfProducts(Float a, Float b, Float c, Float d) {
    Float cd = c * d;
    return std::fma(a, b, -cd) + std::fma(-c, d, cd);
}
static inline Float SumOfProducts(Float a, Float b, Float c, Float d) {
    Float cd = c * d;
    return std::fma(a, b, cd) + std::fma(c, d, -cd);
}
static inline uint32_t FloatToBits(Float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}
static inline Float BitsToFloat(uint32_t u) {
    Float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static inline Float NextFloatUp(Float v) {
    if (std::isinf(v) && v > 0.f) return v;
    if (v == -0.f) v = 0.f;
    uint32_t ui = FloatToBits(v);
    if (v >= 0) ++ui;
    else --ui;
    return BitsToFloat(ui);
}
static inline Float NextFloatDown(Float v) {
    if (std::isinf(v) && v < 0.f) return v;
    if (v == 0.f) v = -0.f;
    uint32_t ui = FloatToBits(v);
    if (v > 0) --ui;
    else ++ui;
    return BitsToFloat(ui);
}

struct Vec {
    Float x = 0, y = 0, z = 0;
    Vec() = default;
    Vec(Float a, Float b, Float c) : x(a), y(b), z(c) {}
    Float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    Float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    Vec operator+(Vec o) const { return {x + o.x, y + o.y, z + o.z}; }
    Vec operator-(Vec o) const { return {x - o.x, y - o.y, z - o.z}; }
    Vec operator-() const { return {-x, -y, -z}; }
    Vec operator*(Float s) const { return {x * s, y * s, z * s}; }
    Vec operator/(Float s) const { return {x / s, y / s, z / s}; }
    bool operator==(Vec o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(Vec o) const { return !(*this == o); }
};
static inline Vec operator*(Float s, Vec v) { return {s * v.x, s * v.y, s * v.z}; }
static inline Float Dot(Vec a, Vec b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline Float AbsDot(Vec a, Vec b) { return std::abs(Dot(a, b)); }
// Normal3f dot products are FMA-compensated (util/vecmath.h:1059-1099)
static inline Float SumOfProducts(Float a, Float b, Float c, Float d);
static inline Float DotN(Vec n, Vec v) { return std::fma(n.x, v.x, SumOfProducts(n.y, v.y, n.z, v.z)); }
static inline Float AbsDotN(Vec n, Vec v) { return std::abs(DotN(n, v)); }
static inline Vec Cross(Vec v, Vec w) {
    return {DifferenceOfProducts(v.y, w.z, v.z, w.y), DifferenceOfProducts(v.z, w.x, v.x, w.z),
            DifferenceOfProducts(v.x, w.y, v.y, w.x)};
}
static inline Float LengthSquared(Vec v) { return Sqr(v.x) + Sqr(v.y) + Sqr(v.z); }
static inline Float Length(Vec v) { return std::sqrt(LengthSquared(v)); }
static inline Vec Normalize(Vec v) { return v / Length(v); }
static inline Vec Abs(Vec v) { return {std::abs(v.x), std::abs(v.y), std::abs(v.z)}; }
static inline Float DistanceSquared(Vec a, Vec b) { return LengthSquared(a - b); }
static inline Float MaxComp(Vec v) { return std::max(v.x, std::max(v.y, v.z)); }
static inline int MaxCompIndex(Vec v) { return (v.x > v.y) ? ((v.x > v.z) ? 0 : 2) : ((v.y > v.z) ? 1 : 2); }
static inline Vec GramSchmidt(Vec v, Vec w) { return v - Dot(v, w) * w; }
static inline Float AngleBetween(Vec v1, Vec v2) {
    if (Dot(v1, v2) < 0) return Pi - 2 * SafeASin(Length(v1 + v2) / 2);
    return 2 * SafeASin(Length(v2 - v1) / 2);
}
static inline void CoordinateSystem(Vec v1, Vec *v2, Vec *v3) {
    Float sign = std::copysign(Float(1), v1.z);
    Float a = -1 / (sign + v1.z);
    Float b = v1.x * v1.y * a;
    *v2 = Vec(1 + sign * Sqr(v1.x) * a, sign * b, -sign * v1.x);
    *v3 = Vec(b, sign + Sqr(v1.y) * a, -v1.y);
}

// ---------------------------------------------------------------- spectra
struct Spectrum {
    Float v[NS];
    Spectrum() { std::fill(v, v + NS, 0.f); }
    explicit Spectrum(Float c) { std::fill(v, v + NS, c); }
    Float &operator[](int i) { return v[i]; }
    Float operator[](int i) const { return v[i]; }
    Spectrum operator+(const Spectrum &o) const {
        Spectrum r = *this;
        for (int i = 0; i < NS; ++i) r.v[i] += o.v[i];
        return r;
    }
    Spectrum operator*(const Spectrum &o) const {
        Spectrum r = *this;
        for (int i = 0; i < NS; ++i) r.v[i] *= o.v[i];
        return r;
    }
    Spectrum operator*(Float a) const {
        Spectrum r = *this;
        for (int i = 0; i < NS; ++i) r.v[i] *= a;
        return r;
    }
    Spectrum operator/(Float a) const {
        Spectrum r = *this;
        for (int i = 0; i < NS; ++i) r.v[i] /= a;
        return r;
    }
    Spectrum operator/(const Spectrum &o) const {
        Spectrum r = *this;
        for (int i = 0; i < NS; ++i) r.v[i] /= o.v[i];
        return r;
    }
    explicit operator bool() const {
        for (int i = 0; i < NS; ++i)
            if (v[i] != 0) return true;
        return false;
    }
    Float Max() const {
        Float m = v[0];
        for (int i = 1; i < NS; ++i) m = std::max(m, v[i]);
        return m;
    }
    Float Average() const {
        Float s = v[0];
        for (int i = 1; i < NS; ++i) s += v[i];
        return s / NS;
    }
};

struct Wavelengths {
    Float lambda[NS], pdf[NS];
    static Wavelengths SampleUniform(Float u) {  // util/spectrum.h:318 (fork: uniform)
        Wavelengths w;
        w.lambda[0] = Lerp(u, LambdaMin, LambdaMax);
        Float delta = (LambdaMax - LambdaMin) / NS;
        for (int i = 1; i < NS; ++i) {
            w.lambda[i] = w.lambda[i - 1] + delta;
            if (w.lambda[i] > LambdaMax) w.lambda[i] = LambdaMin + (w.lambda[i] - LambdaMax);
        }
        for (int i = 0; i < NS; ++i) w.pdf[i] = 1 / (LambdaMax - LambdaMin);
        return w;
    }
};

static inline Spectrum SampleDense(const float *dense, const Wavelengths &w) {
    Spectrum s;
    for (int i = 0; i < NS; ++i) {
        long off = std::lround(w.lambda[i]) - 395;
        s[i] = (off < 0 || off >= 311) ? 0 : dense[off];
    }
    return s;
}

static inline Float Sigmoid(Float c0, Float c1, Float c2, Float lambda) {
    Float x = std::fma(lambda, std::fma(lambda, c0, c1), c2);
    if (std::isinf(x)) return x > 0 ? 1 : 0;
    return .5f + x / (2 * std::sqrt(1 + Sqr(x)));
}

// ---------------------------------------------------------------- Halton
static uint64_t Murmur64A(const unsigned char *key, size_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ (len * m);
    const unsigned char *end = key + 8 * (len / 8);
    while (key != end) {
        uint64_t k;
        std::memcpy(&k, key, 8);
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
    case 1: h ^= uint64_t(key[0]); h *= m;
    }
    h ^= h >> r;
    h *= m;
    h ^= h >> r;
    return h;
}
static int PermElem(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
    do {
        i ^= p; i *= 0xe170893d; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i *= 0x0929eb3f;
        i ^= p >> 23; i ^= (i & w) >> 1; i *= 1 | p >> 27; i *= 0x6935fa69; i ^= (i & w) >> 11;
        i *= 0x74dcb303; i ^= (i & w) >> 2; i *= 0x9e501cc3; i ^= (i & w) >> 2; i *= 0xc860a3df;
        i &= w; i ^= i >> 5;
    } while (i >= l);
    return (i + p) % l;
}

struct DigitPerm {
    int base = 0, nDigits = 0;
    std::vector<uint16_t> perm;
};

struct Halton {
    std::vector<DigitPerm> perms;
    int baseScales[2], baseExponents[2], multInverse[2];
    static void ExtGCD(uint64_t a, uint64_t b, int64_t *x, int64_t *y) {
        if (b == 0) { *x = 1; *y = 0; return; }
        int64_t d = a / b, xp, yp;
        ExtGCD(b, a % b, &xp, &yp);
        *x = yp;
        *y = xp - (d * yp);
    }
    static int MultInv(int64_t a, int64_t n) {
        int64_t x, y;
        ExtGCD(a, n, &x, &y);
        int64_t r = x % n;
        return (int)(r < 0 ? r + n : r);
    }
    void Init(int xres, int yres, uint32_t seed, int nDims) {
        std::vector<int> primes;
        for (int n = 2; (int)primes.size() < nDims; ++n) {
            bool ok = true;
            for (int q : primes) {
                if (q * q > n) break;
                if (n % q == 0) { ok = false; break; }
            }
            if (ok) primes.push_back(n);
        }
        perms.resize(nDims);
        for (int d = 0; d < nDims; ++d) {
            DigitPerm &p = perms[d];
            p.base = primes[d];
            volatile Float invBase = (Float)1 / (Float)p.base, invBaseM = 1;
            p.nDigits = 0;
            while (1 - (Float)(p.base - 1) * invBaseM < 1) { ++p.nDigits; invBaseM = invBaseM * invBase; }
            p.perm.resize(p.nDigits * p.base);
            for (int di = 0; di < p.nDigits; ++di) {
                unsigned char buf[12];
                int b = p.base, dd = di;
                std::memcpy(buf, &b, 4);
                std::memcpy(buf + 4, &dd, 4);
                std::memcpy(buf + 8, &seed, 4);
                uint64_t dseed = Murmur64A(buf, 12, 0);
                for (int v = 0; v < p.base; ++v) p.perm[di * p.base + v] = (uint16_t)PermElem(v, p.base, (uint32_t)dseed);
            }
        }
        int res[2] = {xres, yres};
        for (int i = 0; i < 2; ++i) {
            int base = i == 0 ? 2 : 3, scale = 1, exp = 0;
            while (scale < std::min(res[i], 128)) { scale *= base; ++exp; }
            baseScales[i] = scale;
            baseExponents[i] = exp;
        }
        multInverse[0] = MultInv(baseScales[1], baseScales[0]);
        multInverse[1] = MultInv(baseScales[0], baseScales[1]);
    }
};

struct HaltonState {
    const Halton *h;
    uint64_t index;
    int dimension;
    static uint64_t InvRadInv(uint64_t inverse, int base, int nDigits) {
        uint64_t index = 0;
        for (int i = 0; i < nDigits; ++i) {
            uint64_t digit = inverse % base;
            inverse /= base;
            index = index * base + digit;
        }
        return index;
    }
    void Start(int px, int py, int sampleIndex, int dim) {
        index = 0;
        int stride = h->baseScales[0] * h->baseScales[1];
        if (stride > 1) {
            int pm[2] = {((px % 128) + 128) % 128, ((py % 128) + 128) % 128};
            for (int i = 0; i < 2; ++i) {
                uint64_t off = InvRadInv(pm[i], i == 0 ? 2 : 3, h->baseExponents[i]);
                index += off * (stride / h->baseScales[i]) * h->multInverse[i];
            }
            index %= stride;
        }
        index += (uint64_t)sampleIndex * stride;
        dimension = std::max(2, dim);
    }
    Float Sample(int dim) const {
        const DigitPerm &p = h->perms[dim];
        uint64_t a = index;
        Float invBase = (Float)1 / (Float)p.base, invBaseM = 1;
        uint64_t rev = 0;
        for (int di = 0; di < p.nDigits; ++di) {
            uint64_t next = a / p.base;
            int dv = (int)(a - next * p.base);
            rev = rev * p.base + p.perm[di * p.base + dv];
            invBaseM *= invBase;
            a = next;
        }
        return std::min(invBaseM * rev, OneMinusEpsilon);
    }
    Float Get1D() {
        if (dimension >= (int)h->perms.size()) dimension = 2;
        return Sample(dimension++);
    }
    void Get2D(Float *a, Float *b) {
        if (dimension + 1 >= (int)h->perms.size()) dimension = 2;
        int d = dimension;
        dimension += 2;
        *a = Sample(d);
        *b = Sample(d + 1);
    }
    static Float RadInv(int base, uint64_t a) {
        uint64_t limit = ~0ull / base - base;
        Float invBase = (Float)1 / (Float)base, invBaseM = 1;
        uint64_t rev = 0;
        while (a && rev < limit) {
            uint64_t next = a / base;
            rev = rev * base + (a - next * base);
            invBaseM *= invBase;
            a = next;
        }
        return std::min(rev * invBaseM, OneMinusEpsilon);
    }
    void Pixel2D(Float *x, Float *y) const {
        *x = RadInv(2, index >> h->baseExponents[0]);
        *y = RadInv(3, index / h->baseScales[1]);
    }
};

// ---------------------------------------------------------------- ZSobol
// ZSobolSampler (samplers.h:225-370).  Sobol' dimension 0 is the van der Corput matrix; the
// rows of dimension 1 are Pascal's triangle mod 2 (bit r of row k set iff (r & k) == r by
// Lucas), top 32 bits of the 52-bit rows of util/sobolmatrices.
struct ZSobol {
    int log2Spp = 0, nBase4Digits = 0, seed = 0, randomize = 2;
    static const int perm4[24][4];
    void Init(int spp, int xres, int yres, int seed_, int randomize_) {
        seed = seed_;
        randomize = randomize_;
        log2Spp = 0;
        while ((2 << log2Spp) <= spp) ++log2Spp;  // Log2Int
        int res = 1;
        while (res < std::max(xres, yres)) res *= 2;  // RoundUpPow2
        int l = 0;
        while ((2 << l) <= res) ++l;
        nBase4Digits = l + (log2Spp + 1) / 2;
    }
};
const int ZSobol::perm4[24][4] = {{0, 1, 2, 3}, {0, 1, 3, 2}, {0, 2, 1, 3}, {0, 2, 3, 1}, {0, 3, 2, 1}, {0, 3, 1, 2},
                                  {1, 0, 2, 3}, {1, 0, 3, 2}, {1, 2, 0, 3}, {1, 2, 3, 0}, {1, 3, 2, 0}, {1, 3, 0, 2},
                                  {2, 1, 0, 3}, {2, 1, 3, 0}, {2, 0, 1, 3}, {2, 0, 3, 1}, {2, 3, 0, 1}, {2, 3, 1, 0},
                                  {3, 1, 2, 0}, {3, 1, 0, 2}, {3, 2, 1, 0}, {3, 2, 0, 1}, {3, 0, 2, 1}, {3, 0, 1, 2}};

static uint64_t Mix64(uint64_t v) {
    v = (v ^ (v >> 31)) * 0x7fb5d329728ea185ull;
    v = (v ^ (v >> 27)) * 0x81dadef4bc2dd44dull;
    return v ^ (v >> 33);
}
static uint32_t BitReverse(uint32_t v) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i) r |= ((v >> i) & 1u) << (31 - i);
    return r;
}
static uint32_t SobolRow(int dim, int k) {
    if (dim == 0) return k < 32 ? 0x80000000u >> k : 0u;
    uint32_t w = 0;
    for (int r = 0; r < 32; ++r)
        if ((r & k) == r) w |= 0x80000000u >> r;
    return w;
}

struct ZSobolState {
    const ZSobol *z;
    uint64_t morton = 0;
    int dimension = 0;
    void Start(int px, int py, int sampleIndex, int dim) {
        uint64_t m = 0;
        for (int b = 0; b < 32; ++b) m |= (uint64_t)((uint32_t)px >> b & 1) << (2 * b) | (uint64_t)((uint32_t)py >> b & 1) << (2 * b + 1);
        morton = (m << z->log2Spp) | (uint64_t)(uint32_t)sampleIndex;
        dimension = dim;
    }
    uint64_t Index() const {
        uint64_t idx = 0;
        const bool odd = z->log2Spp & 1;
        const uint64_t salt = (uint64_t)(uint32_t)(0x55555555u * (uint32_t)dimension);
        for (int i = z->nBase4Digits - 1; i >= (odd ? 1 : 0); --i) {
            int shift = 2 * i - (odd ? 1 : 0);
            int digit = (int)(morton >> shift) & 3;
            int p = (int)((Mix64((morton >> (shift + 2)) ^ salt) >> 24) % 24);
            idx |= (uint64_t)ZSobol::perm4[p][digit] << shift;
        }
        if (odd) idx |= ((morton & 1) ^ (Mix64((morton >> 1) ^ salt) & 1));
        return idx;
    }
    static uint64_t HashDimSeed(int d, int seed) {
        unsigned char buf[8];
        std::memcpy(buf, &d, 4);
        std::memcpy(buf + 4, &seed, 4);
        return Murmur64A(buf, 8, 0);
    }
    Float Sobol(uint64_t a, int dim, uint32_t h) const {
        uint32_t v = 0;
        for (int k = 0; a; a >>= 1, ++k)
            if (a & 1) v ^= SobolRow(dim, k);
        switch (z->randomize) {
        case 1: v ^= h; break;
        case 2: {  // FastOwenScrambler (lowdiscrepancy.h:221-237)
            v = BitReverse(v);
            v ^= v * 0x3d20adea;
            v += h;
            v *= (h >> 16) | 1;
            v ^= v * 0x05526c56;
            v ^= v * 0x53a22864;
            v = BitReverse(v);
            break;
        }
        case 3: {  // OwenScrambler (lowdiscrepancy.h:240-258)
            if (h & 1) v ^= 1u << 31;
            for (int b = 1; b < 32; ++b)
                if ((uint32_t)Mix64((v & (~0u << (32 - b))) ^ h) & (1u << b)) v ^= 1u << (31 - b);
            break;
        }
        default: break;
        }
        return std::min(v * 0x1p-32f, OneMinusEpsilon);
    }
    Float Get1D() {
        uint64_t idx = Index();
        ++dimension;
        return Sobol(idx, 0, (uint32_t)HashDimSeed(dimension, z->seed));
    }
    void Get2D(Float *a, Float *b) {
        uint64_t idx = Index();
        dimension += 2;
        uint64_t h = HashDimSeed(dimension, z->seed);
        *a = Sobol(idx, 0, (uint32_t)h);
        *b = Sobol(idx, 1, (uint32_t)(h >> 32));
    }
    void Pixel2D(Float *a, Float *b) { Get2D(a, b); }
};

// ---------------------------------------------------------------- independent / stratified /
// sobol / paddedsobol (samplers.h:144-224, 442-633).  The RNG is util/rng.h's PCG32 with its
// SetSequence / Advance (rng.h:119-150); Hash(args...) is MurmurHash64A over the packed
// arguments (util/hash.h:91-106); the Sobol' rows come from the scene's copy of
// util/sobolmatrices.cpp (pbrt_scene_flat::sobol_matrices32 / vdc_sobol / vdc_sobol_inv).
struct SeqRNG {
    uint64_t state = 0, inc = 1;
    uint32_t Next() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    void SetSequence(uint64_t seq) {
        state = 0u;
        inc = (seq << 1u) | 1u;
        Next();
        state += Mix64(seq);
        Next();
    }
    void Advance(uint64_t delta) {
        // delta steps of the LCG: x -> a x + c, composed by doubling (a^k, c (a^k - 1)/(a - 1))
        uint64_t a = 0x5851f42d4c957f2dULL, c = inc, A = 1, C = 0;
        for (; delta; delta >>= 1) {
            if (delta & 1) {
                A *= a;
                C = C * a + c;
            }
            c = (a + 1) * c;
            a *= a;
        }
        state = A * state + C;
    }
    Float Uniform() { return std::min<Float>(OneMinusEpsilon, Next() * 0x1p-32f); }
};
struct OtherSampler {
    int kind = 0;  // 2 independent, 3 stratified, 4 sobol, 5 paddedsobol (pbrt_scene_flat::sampler_type)
    int spp = 1, seed = 0, xs = 1, ys = 1, jitter = 1, randomize = 2, log2Scale = 0;
    const uint32_t *m32 = nullptr;
    const uint64_t *vdc = nullptr, *vdcInv = nullptr;
};
struct OtherState {
    const OtherSampler *o = nullptr;
    int px = 0, py = 0, si = 0, dimension = 0;
    uint64_t sobolIndex = 0;
    SeqRNG rng;
    static uint64_t HashInts(std::initializer_list<int> v) {
        unsigned char buf[16];
        size_t n = 0;
        for (int x : v) {
            std::memcpy(buf + n, &x, 4);
            n += 4;
        }
        return Murmur64A(buf, n, 0);
    }
    static uint32_t Scramble(uint32_t v, int randomize, uint32_t h) {
        switch (randomize) {
        case 1: return v ^ h;
        case 2:
            v = BitReverse(v);
            v ^= v * 0x3d20adea;
            v += h;
            v *= (h >> 16) | 1;
            v ^= v * 0x05526c56;
            v ^= v * 0x53a22864;
            return BitReverse(v);
        case 3:
            if (h & 1) v ^= 1u << 31;
            for (int b = 1; b < 32; ++b)
                if ((uint32_t)Mix64((v & (~0u << (32 - b))) ^ h) & (1u << b)) v ^= 1u << (31 - b);
            return v;
        default: return v;
        }
    }
    // SobolSample(a, dim, scrambler) over the full matrices
    Float Sobol(uint64_t a, int dim, int randomize, uint32_t h) const {
        uint32_t v = 0;
        for (int k = 0; a; a >>= 1, ++k)
            if (a & 1) v ^= o->m32[dim * 52 + k];
        return std::min(Scramble(v, randomize, h) * 0x1p-32f, OneMinusEpsilon);
    }
    // dimensions 0 / 1 (the padded sampler): van der Corput and Pascal's triangle mod 2
    static Float Sobol01(uint64_t a, int dim, int randomize, uint32_t h) {
        uint32_t v = 0;
        for (int k = 0; a; a >>= 1, ++k)
            if (a & 1) v ^= SobolRow(dim, k);
        return std::min(Scramble(v, randomize, h) * 0x1p-32f, OneMinusEpsilon);
    }
    void Start(int x, int y, int index, int dim) {
        px = x, py = y, si = index, dimension = dim;
        if (o->kind == 2 || o->kind == 3) {
            rng.SetSequence(HashInts({x, y, o->seed}));
            rng.Advance((uint64_t)index * 65536ull + (uint64_t)dim);
        }
        if (o->kind == 4) {
            dimension = std::max(2, dim);
            // SobolIntervalToIndex (lowdiscrepancy.h:266-287)
            const uint32_t m = (uint32_t)o->log2Scale;
            uint64_t frame = (uint64_t)index;
            if (m == 0) {
                sobolIndex = frame;
            } else {
                uint64_t idx = frame << (2 * m), delta = 0;
                for (int c = 0; frame; frame >>= 1, ++c)
                    if (frame & 1) delta ^= o->vdc[(m - 1) * 52 + c];
                uint64_t b = (((uint64_t)(uint32_t)x << m) | (uint32_t)y) ^ delta;
                for (int c = 0; b; b >>= 1, ++c)
                    if (b & 1) idx ^= o->vdcInv[(m - 1) * 52 + c];
                sobolIndex = idx;
            }
        }
    }
    Float SobolDimension(int d) const {
        return o->randomize == 0 ? Sobol(sobolIndex, d, 0, 0)
                                 : Sobol(sobolIndex, d, o->randomize, (uint32_t)HashInts({d, o->seed}));
    }
    int Permuted(uint64_t hash, int n) const { return PermElem((uint32_t)si, (uint32_t)n, (uint32_t)hash); }
    Float Get1D() {
        switch (o->kind) {
        case 2: return rng.Uniform();
        case 3: {
            const uint64_t hash = HashInts({px, py, dimension, o->seed});
            const int n = o->xs * o->ys, stratum = Permuted(hash, n);
            ++dimension;
            const Float delta = o->jitter ? rng.Uniform() : 0.5f;
            return (stratum + delta) / n;
        }
        case 4:
            if (dimension >= 1024) dimension = 2;
            return SobolDimension(dimension++);
        default: {
            const uint64_t hash = HashInts({px, py, dimension, o->seed});
            const int index = Permuted(hash, o->spp);
            ++dimension;
            return Sobol01((uint32_t)index, 0, o->randomize, (uint32_t)(hash >> 32));
        }
        }
    }
    void Get2D(Float *a, Float *b) {
        switch (o->kind) {
        case 2:
            *a = rng.Uniform();
            *b = rng.Uniform();
            return;
        case 3: {
            const uint64_t hash = HashInts({px, py, dimension, o->seed});
            const int stratum = Permuted(hash, o->xs * o->ys);
            dimension += 2;
            const int x = stratum % o->xs, y = stratum / o->xs;
            const Float dx = o->jitter ? rng.Uniform() : 0.5f;
            const Float dy = o->jitter ? rng.Uniform() : 0.5f;
            *a = (x + dx) / o->xs;
            *b = (y + dy) / o->ys;
            return;
        }
        case 4:
            if (dimension + 1 >= 1024) dimension = 2;
            *a = SobolDimension(dimension);
            *b = SobolDimension(dimension + 1);
            dimension += 2;
            return;
        default: {
            const uint64_t hash = HashInts({px, py, dimension, o->seed});
            const int index = Permuted(hash, o->spp);
            dimension += 2;
            *a = Sobol01((uint32_t)index, 0, o->randomize, (uint32_t)hash);
            *b = Sobol01((uint32_t)index, 1, o->randomize, (uint32_t)(hash >> 32));
            return;
        }
        }
    }
    void Pixel2D(Float *a, Float *b) {
        if (o->kind != 4) {
            Get2D(a, b);
            return;
        }
        const Float scale = (Float)(1 << o->log2Scale);
        Float u0 = Sobol(sobolIndex, 0, 0, 0), u1 = Sobol(sobolIndex, 1, 0, 0);
        *a = Clamp(u0 * scale - px, 0.f, OneMinusEpsilon);
        *b = Clamp(u1 * scale - py, 0.f, OneMinusEpsilon);
    }
};

// Any sampler behind pbrt's Sampler interface calls used by the wavefront
struct AnySampler {
    HaltonState h;
    ZSobolState z;
    bool zsobol;
    OtherState os;  // os.o set: one of the other four samplers
    void Start(int px, int py, int si, int dim) {
        if (os.o) os.Start(px, py, si, dim);
        else zsobol ? z.Start(px, py, si, dim) : h.Start(px, py, si, dim);
    }
    Float Get1D() { return os.o ? os.Get1D() : zsobol ? z.Get1D() : h.Get1D(); }
    void Get2D(Float *a, Float *b) { os.o ? os.Get2D(a, b) : zsobol ? z.Get2D(a, b) : h.Get2D(a, b); }
    void Pixel2D(Float *a, Float *b) { os.o ? os.Pixel2D(a, b) : zsobol ? z.Pixel2D(a, b) : h.Pixel2D(a, b); }
};

// ---------------------------------------------------------------- geometry
struct TriIsect {
    Float b0, b1, b2, t;
};
static bool IntersectTriangle(Vec o, Vec dir, Float tMax, Vec p0, Vec p1, Vec p2, TriIsect *out) {
    if (LengthSquared(Cross(p2 - p0, p1 - p0)) == 0) return false;
    Vec p0t = p0 - o, p1t = p1 - o, p2t = p2 - o;
    int kz = MaxCompIndex(Abs(dir));
    int kx = kz + 1 == 3 ? 0 : kz + 1;
    int ky = kx + 1 == 3 ? 0 : kx + 1;
    Vec d(dir[kx], dir[ky], dir[kz]);
    p0t = Vec(p0t[kx], p0t[ky], p0t[kz]);
    p1t = Vec(p1t[kx], p1t[ky], p1t[kz]);
    p2t = Vec(p2t[kx], p2t[ky], p2t[kz]);
    Float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1 / d.z;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    Float e0 = DifferenceOfProducts(p1t.x, p2t.y, p1t.y, p2t.x);
    Float e1 = DifferenceOfProducts(p2t.x, p0t.y, p2t.y, p0t.x);
    Float e2 = DifferenceOfProducts(p0t.x, p1t.y, p0t.y, p1t.x);
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        double a = (double)p2t.x * (double)p1t.y, b = (double)p2t.y * (double)p1t.x;
        e0 = (float)(b - a);
        double c = (double)p0t.x * (double)p2t.y, dd = (double)p0t.y * (double)p2t.x;
        e1 = (float)(dd - c);
        double e = (double)p1t.x * (double)p0t.y, f = (double)p1t.y * (double)p0t.x;
        e2 = (float)(f - e);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    Float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    Float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < tMax * det)) return false;
    if (det > 0 && (tScaled <= 0 || tScaled > tMax * det)) return false;
    Float invDet = 1 / det;
    Float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet, t = tScaled * invDet;
    Float maxZt = MaxComp(Abs(Vec(p0t.z, p1t.z, p2t.z)));
    Float deltaZ = gamma(3) * maxZt;
    Float maxXt = MaxComp(Abs(Vec(p0t.x, p1t.x, p2t.x)));
    Float maxYt = MaxComp(Abs(Vec(p0t.y, p1t.y, p2t.y)));
    Float deltaX = gamma(5) * (maxXt + maxZt), deltaY = gamma(5) * (maxYt + maxZt);
    Float deltaE = 2 * (gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    Float maxE = MaxComp(Abs(Vec(e0, e1, e2)));
    Float deltaT = 3 * (gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::abs(invDet);
    if (t <= deltaT) return false;
    *out = {b0, b1, b2, t};
    return true;
}

static Vec OffsetRayOrigin(Vec p, Vec err, Vec n, Vec w) {
    Float d = DotN(Abs(n), err);
    Vec offset = d * n;
    if (DotN(n, w) < 0) offset = -offset;
    Vec po = p + offset;
    for (int i = 0; i < 3; ++i) {
        if (offset[i] > 0) po[i] = NextFloatUp(po[i]);
        else if (offset[i] < 0) po[i] = NextFloatDown(po[i]);
    }
    return po;
}

struct Scene;

// Point3fi(p, e): interval [NextFloatDown(p - e), NextFloatUp(p + e)]; p() is its midpoint
// and Error() its half width (util/vecmath.h:753, util/math.h:829, util/float.h:201-229)
static void Point3fi(Vec v, Vec e, Vec *p, Vec *err) {
    for (int i = 0; i < 3; ++i) {
        Float lo = v[i], hi = v[i];
        if (e[i] != 0) {
            lo = NextFloatDown(v[i] + (-e[i]));
            hi = NextFloatUp(v[i] + e[i]);
        }
        (*p)[i] = (lo + hi) / 2;
        (*err)[i] = (hi - lo) / 2;
    }
}

struct Interaction {
    Vec p, err, n, ns, dpdu, dpdus, wo;
    Vec dpdv;        // geometric dpdv and uv: texture lookups (surfscatter.cpp:74-135)
    // shading dpdv and normal derivatives (bump mapping); a triangle without vertex normals or
    // a disk keeps the geometric dpdv and zero derivatives (hasShadingDiff false)
    Vec dpdvs, dndus, dndvs;
    bool hasShadingDiff = false;
    Float uv[2] = {0, 0};
    int prim = -1;
};

// a mesh triangle's optional vertex normals and uv (TriangleMesh n / uv, util/mesh.h:23-46)
struct TriAttr {
    bool hasN = false, hasUV = false, hasS = false;
    Vec n[3], s[3];
    Float uv[3][2] = {{0, 0}, {1, 0}, {1, 1}};
};

// Triangle::InteractionFromIntersection (shapes.h:884-1010) + SetShadingGeometry
// (interaction.h:194-214, orientationIsAuthoritative = true); dndu/dndv are not needed
static Interaction TriangleInteraction(Vec p0, Vec p1, Vec p2, bool flip, TriIsect ti, Vec rayD,
                                       const TriAttr &a = TriAttr()) {
    Interaction si;
    Float duv02[2] = {a.uv[0][0] - a.uv[2][0], a.uv[0][1] - a.uv[2][1]};
    Float duv12[2] = {a.uv[1][0] - a.uv[2][0], a.uv[1][1] - a.uv[2][1]};
    Vec dp02 = p0 - p2, dp12 = p1 - p2;
    Float determinant = DifferenceOfProducts(duv02[0], duv12[1], duv02[1], duv12[0]);
    Vec dpdu, dpdv;
    bool degenerate = std::abs(determinant) < 1e-9f;
    if (!degenerate) {
        Float invdet = 1 / determinant;
        for (int k = 0; k < 3; ++k) {
            dpdu[k] = DifferenceOfProducts(duv12[1], dp02[k], duv02[1], dp12[k]) * invdet;
            dpdv[k] = DifferenceOfProducts(duv02[0], dp12[k], duv12[0], dp02[k]) * invdet;
        }
    }
    if (degenerate || LengthSquared(Cross(dpdu, dpdv)) == 0) CoordinateSystem(Normalize(Cross(p2 - p0, p1 - p0)), &dpdu, &dpdv);
    Point3fi(ti.b0 * p0 + ti.b1 * p1 + ti.b2 * p2, gamma(7) * (Abs(ti.b0 * p0) + Abs(ti.b1 * p1) + Abs(ti.b2 * p2)),
             &si.p, &si.err);
    si.n = Normalize(Cross(dp02, dp12));
    if (flip) si.n = -si.n;
    si.ns = si.n;
    si.dpdu = si.dpdus = dpdu;
    si.dpdv = dpdv;
    // Point2f uvHit = b0 * uv[0] + b1 * uv[1] + b2 * uv[2] (shapes.h:920)
    for (int k = 0; k < 2; ++k) si.uv[k] = ti.b0 * a.uv[0][k] + ti.b1 * a.uv[1][k] + ti.b2 * a.uv[2][k];
    if (a.hasN || a.hasS) {
        Vec ns = si.n;
        if (a.hasN) {
            ns = ti.b0 * a.n[0] + ti.b1 * a.n[1] + ti.b2 * a.n[2];
            ns = LengthSquared(ns) > 0 ? Normalize(ns) : si.n;
        }
        Vec ss = si.dpdu;
        if (a.hasS) {  // shapes.h:951-957
            ss = ti.b0 * a.s[0] + ti.b1 * a.s[1] + ti.b2 * a.s[2];
            if (LengthSquared(ss) == 0) ss = si.dpdu;
        }
        Vec ts = Cross(ns, ss);
        if (LengthSquared(ts) > 0) ss = Cross(ts, ns);
        else CoordinateSystem(ns, &ss, &ts);
        si.ns = ns;
        if (DotN(si.n, ns) < 0) si.n = -si.n;  // FaceForward(n, shading.n)
        while (LengthSquared(ss) > 1e16f || LengthSquared(ts) > 1e16f) {
            ss = ss / 1e8f;
            ts = ts / 1e8f;
        }
        si.dpdus = ss;
        // shading bitangent and dndu, dndv from the vertex normals (shapes.h:961-1006)
        si.dpdvs = ts;
        si.hasShadingDiff = true;
        const Vec dn1 = a.n[0] - a.n[2], dn2 = a.n[1] - a.n[2];
        const Float det = DifferenceOfProducts(duv02[0], duv12[1], duv02[1], duv12[0]);
        if (!a.hasN) {
            // no vertex normals: dndu = dndv = 0
        } else if (std::abs(det) < 1e-9f) {
            const Vec dn = Cross(a.n[2] - a.n[0], a.n[1] - a.n[0]);
            if (LengthSquared(dn) != 0) CoordinateSystem(dn, &si.dndus, &si.dndvs);
        } else {
            const Float invDet = 1 / det;
            for (int k = 0; k < 3; ++k) {
                si.dndus[k] = DifferenceOfProducts(duv12[1], dn1[k], duv02[1], dn2[k]) * invDet;
                si.dndvs[k] = DifferenceOfProducts(duv02[0], dn2[k], duv12[0], dn1[k]) * invDet;
            }
        }
    }
    si.wo = Normalize(-rayD);
    return si;
}

// simple binned-SAH BVH2 over the scene triangles (oracle-side; any correct BVH gives the
// same closest hit up to exact-t ties)
struct OTextures;
struct BVHNode {
    Vec mn, mx;
    int left = -1, right = -1, first = 0, count = 0, axis = 0;
};

struct OShape;
struct Scene {
    const pbrt_scene_flat *f;
    const OTextures *tex = nullptr;  // alpha textures (f->prim_alpha)
    std::vector<OShape> shapes;  // spheres and disks: prim ids n_triangles + k
    std::vector<Vec> v;
    std::vector<int> tri;  // 3 per triangle
    std::vector<BVHNode> nodes;
    std::vector<int> order;
    Halton halton;
    ZSobol zsobol;
    bool useZSobol = false;
    OtherSampler other;  // other.kind >= 2: independent / stratified / sobol / paddedsobol
    AnySampler Sampler() const {
        AnySampler a{HaltonState{&halton, 0, 0}, ZSobolState{&zsobol}, useZSobol, OtherState{}};
        if (other.kind >= 2) a.os.o = &other;
        return a;
    }
    int xres, yres, px0, px1, py0, py1, maxDepth;
    Float frx, fry;
    Vec P(int t, int k) const { return v[tri[3 * t + k]]; }
    TriAttr Attr(int t) const {
        TriAttr a;
        const int bits = f->tri_shading ? f->tri_shading[t] : 0;
        for (int k = 0; k < 3; ++k) {
            const int vi = tri[3 * t + k];
            if (bits & 1) a.n[k] = Vec(f->vertex_normals[3 * vi], f->vertex_normals[3 * vi + 1], f->vertex_normals[3 * vi + 2]);
            if (bits & 2) {
                a.uv[k][0] = f->vertex_uv[2 * vi];
                a.uv[k][1] = f->vertex_uv[2 * vi + 1];
            }
            if ((bits & 4) && vi < f->n_vertex_s)
                a.s[k] = Vec(f->vertex_s[3 * vi], f->vertex_s[3 * vi + 1], f->vertex_s[3 * vi + 2]);
        }
        a.hasN = bits & 1;
        a.hasUV = bits & 2;
        a.hasS = bits & 4;
        return a;
    }

    int Build(int start, int end, std::vector<Vec> &cent) {
        BVHNode n;
        n.mn = Vec(Infinity, Infinity, Infinity);
        n.mx = Vec(-Infinity, -Infinity, -Infinity);
        Vec cmn = n.mn, cmx = n.mx;
        for (int i = start; i < end; ++i) {
            int t = order[i];
            for (int k = 0; k < 3; ++k) {
                Vec p = P(t, k);
                for (int a = 0; a < 3; ++a) {
                    n.mn[a] = std::min(n.mn[a], p[a]);
                    n.mx[a] = std::max(n.mx[a], p[a]);
                }
            }
            for (int a = 0; a < 3; ++a) {
                cmn[a] = std::min(cmn[a], cent[t][a]);
                cmx[a] = std::max(cmx[a], cent[t][a]);
            }
        }
        int idx = (int)nodes.size();
        nodes.push_back(n);
        if (end - start <= 4) {
            nodes[idx].first = start;
            nodes[idx].count = end - start;
            return idx;
        }
        int axis = MaxCompIndex(cmx - cmn);
        int mid = (start + end) / 2;
        std::nth_element(order.begin() + start, order.begin() + mid, order.begin() + end,
                         [&](int a, int b) { return cent[a][axis] < cent[b][axis]; });
        int l = Build(start, mid, cent), r = Build(mid, end, cent);
        nodes[idx].left = l;
        nodes[idx].right = r;
        nodes[idx].axis = axis;
        return idx;
    }

    void Init(const pbrt_scene_flat *flat, const pbrt_scene_info *info) {
        f = flat;
        for (int i = 0; i < f->n_vertices; ++i) v.push_back(Vec(f->vertices[3 * i], f->vertices[3 * i + 1], f->vertices[3 * i + 2]));
        tri.assign(f->triangles, f->triangles + 3 * f->n_triangles);
        std::vector<Vec> cent(f->n_triangles);
        order.resize(f->n_triangles);
        for (int t = 0; t < f->n_triangles; ++t) {
            order[t] = t;
            cent[t] = (P(t, 0) + P(t, 1) + P(t, 2)) / 3.f;
        }
        if (f->n_triangles) Build(0, f->n_triangles, cent);
        xres = info->xres;
        yres = info->yres;
        px0 = info->px0;
        px1 = info->px1;
        py0 = info->py0;
        py1 = info->py1;
        maxDepth = info->max_depth;
        frx = info->filter_radius_x;
        fry = info->filter_radius_y;
        InitShapes();
        halton.Init(xres, yres, (uint32_t)info->seed, std::max(f->n_dims, 7 * maxDepth + 7));
        useZSobol = f->sampler_type == 1;
        zsobol.Init(info->spp, xres, yres, info->seed, f->zs_randomize);
        if (f->sampler_type >= 2) {
            other.kind = f->sampler_type;
            other.spp = info->spp;
            other.seed = info->seed;
            other.xs = f->strat_xsamples;
            other.ys = f->strat_ysamples;
            other.jitter = f->strat_jitter;
            other.randomize = f->zs_randomize;
            other.log2Scale = f->sobol_log2_scale;
            other.m32 = f->sobol_matrices32;
            other.vdc = f->vdc_sobol;
            other.vdcInv = f->vdc_sobol_inv;
        }
    }

    void InitShapes();
    static bool BoxHit(const BVHNode &n, Vec o, Vec invDir, const int neg[3], Float rayTMax) {
        // util/vecmath.h:1576-1611
        Float b[2][3] = {{n.mn.x, n.mn.y, n.mn.z}, {n.mx.x, n.mx.y, n.mx.z}};
        Float tMin = (b[neg[0]][0] - o.x) * invDir.x;
        Float tMax = (b[1 - neg[0]][0] - o.x) * invDir.x;
        Float tyMin = (b[neg[1]][1] - o.y) * invDir.y;
        Float tyMax = (b[1 - neg[1]][1] - o.y) * invDir.y;
        tMax *= 1 + 2 * gamma(3);
        tyMax *= 1 + 2 * gamma(3);
        if (tMin > tyMax || tyMin > tMax) return false;
        if (tyMin > tMin) tMin = tyMin;
        if (tyMax < tMax) tMax = tyMax;
        Float tzMin = (b[neg[2]][2] - o.z) * invDir.z;
        Float tzMax = (b[1 - neg[2]][2] - o.z) * invDir.z;
        tzMax *= 1 + 2 * gamma(3);
        if (tMin > tzMax || tzMin > tMax) return false;
        if (tzMin > tMin) tMin = tzMin;
        if (tzMax < tMax) tMax = tzMax;
        return (tMin < rayTMax) && (tMax > 0);
    }

    int Intersect(Vec o, Vec d, Float tMax, TriIsect *hit, bool anyHit) const {
        int best = IntersectTris(o, d, tMax, hit, anyHit);
        if (anyHit && best >= 0) return best;
        return IntersectShapes(o, d, best >= 0 ? hit->t : tMax, hit, anyHit, best);
    }
    int IntersectShapes(Vec o, Vec d, Float tMax, TriIsect *hit, bool anyHit, int best) const;
    // GeometricPrimitive's alpha test as pbrt's GPU any-hit programs apply it (gpu/optix.cu:
    // 197-243): the candidate is ignored when its alpha texture is <= 0 at the hit, or < 1 and
    // below HashFloat(ray o, ray d)
    bool AlphaKilled(int prim, const TriIsect &ti, Vec o, Vec d) const;
    bool Alpha(int prim) const { return f->prim_alpha && f->prim_alpha[prim] >= 0; }
    // the per-primitive attributes of a triangle or a shape
    int Material(int prim) const;
    int Light(int prim) const;
    bool Medium(int prim, int *in, int *out) const;
    Interaction Interact(int prim, const TriIsect &ti, Vec rd) const;
    int IntersectTris(Vec o, Vec d, Float tMax, TriIsect *hit, bool anyHit) const {
        if (nodes.empty()) return -1;
        Vec invDir(1 / d.x, 1 / d.y, 1 / d.z);
        int neg[3] = {invDir.x < 0, invDir.y < 0, invDir.z < 0};
        int stack[128], sp = 0, best = -1;
        stack[sp++] = 0;
        while (sp) {
            const BVHNode &n = nodes[stack[--sp]];
            if (!BoxHit(n, o, invDir, neg, tMax)) continue;
            if (n.left < 0) {
                for (int i = n.first; i < n.first + n.count; ++i) {
                    int t = order[i];
                    TriIsect ti;
                    if (IntersectTriangle(o, d, tMax, P(t, 0), P(t, 1), P(t, 2), &ti)) {
                        if (Alpha(t) && AlphaKilled(t, ti, o, d)) continue;
                        if (anyHit) return t;
                        tMax = ti.t;
                        *hit = ti;
                        best = t;
                    }
                }
            } else if (neg[n.axis]) {  // near child first (cpu/aggregates.cpp:561-568)
                stack[sp++] = n.left;
                stack[sp++] = n.right;
            } else {
                stack[sp++] = n.right;
                stack[sp++] = n.left;
            }
        }
        return best;
    }
};

// ---------------------------------------------------------------- sampling
static void SampleUniformDiskConcentric(Float u0, Float u1, Float *x, Float *y) {
    Float ox = 2 * u0 - 1, oy = 2 * u1 - 1;
    if (ox == 0 && oy == 0) { *x = 0; *y = 0; return; }
    Float theta, r;
    if (std::abs(ox) > std::abs(oy)) { r = ox; theta = PiOver4 * (oy / ox); }
    else { r = oy; theta = PiOver2 - PiOver4 * (ox / oy); }
    *x = r * CRCos(theta);
    *y = r * CRSin(theta);
}
static Vec SampleCosineHemisphere(Float u0, Float u1) {
    Float x, y;
    SampleUniformDiskConcentric(u0, u1, &x, &y);
    return Vec(x, y, SafeSqrt(1 - Sqr(x) - Sqr(y)));
}
static Float SampleLinear(Float u, Float a, Float b) {
    if (u == 0 && a == 0) return 0;
    Float x = u * (a + b) / (a + std::sqrt(Lerp(u, Sqr(a), Sqr(b))));
    return std::min(x, OneMinusEpsilon);
}
static Float BilinearPDF(Float x, Float y, const Float w[4]) {
    if (x < 0 || x > 1 || y < 0 || y > 1) return 0;
    if (w[0] + w[1] + w[2] + w[3] == 0) return 1;
    return 4 * ((1 - x) * (1 - y) * w[0] + x * (1 - y) * w[1] + (1 - x) * y * w[2] + x * y * w[3]) /
           (w[0] + w[1] + w[2] + w[3]);
}
static void SampleBilinear(Float u0, Float u1, const Float w[4], Float *x, Float *y) {
    *y = SampleLinear(u1, w[0] + w[1], w[2] + w[3]);
    *x = SampleLinear(u0, Lerp(*y, w[0], w[2]), Lerp(*y, w[1], w[3]));
}
static void SampleUniformTriangle(Float u0, Float u1, Float b[3]) {
    if (u0 < u1) { b[0] = u0 / 2; b[1] = u1 - b[0]; }
    else { b[1] = u1 / 2; b[0] = u0 - b[1]; }
    b[2] = 1 - b[0] - b[1];
}
static Float SphericalTriangleArea(Vec a, Vec b, Vec c) {
    return std::abs(2 * CRATan2(Dot(a, Cross(b, c)), 1 + Dot(a, b) + Dot(a, c) + Dot(b, c)));
}
static bool SampleSphericalTriangle(Vec v0, Vec v1, Vec v2, Vec p, Float u0, Float u1, Float bary[3], Float *pdf) {
    *pdf = 0;
    Vec a = Normalize(v0 - p), b = Normalize(v1 - p), c = Normalize(v2 - p);
    Vec n_ab = Cross(a, b), n_bc = Cross(b, c), n_ca = Cross(c, a);
    if (LengthSquared(n_ab) == 0 || LengthSquared(n_bc) == 0 || LengthSquared(n_ca) == 0) {
        bary[0] = bary[1] = bary[2] = 0;
        return false;
    }
    n_ab = Normalize(n_ab); n_bc = Normalize(n_bc); n_ca = Normalize(n_ca);
    Float alpha = AngleBetween(n_ab, -n_ca), beta = AngleBetween(n_bc, -n_ab), gam = AngleBetween(n_ca, -n_bc);
    Float A_pi = alpha + beta + gam;
    Float Ap_pi = Lerp(u0, Pi, A_pi);
    Float A = A_pi - Pi;
    *pdf = (A <= 0) ? 0 : 1 / A;
    Float cosAlpha = CRCos(alpha), sinAlpha = CRSin(alpha);
    Float sinPhi = CRSin(Ap_pi) * cosAlpha - CRCos(Ap_pi) * sinAlpha;
    Float cosPhi = CRCos(Ap_pi) * cosAlpha + CRSin(Ap_pi) * sinAlpha;
    Float k1 = cosPhi + cosAlpha, k2 = sinPhi - sinAlpha * Dot(a, b);
    Float cosBp = (k2 + (DifferenceOfProducts(k2, cosPhi, k1, sinPhi)) * cosAlpha) /
                  ((SumOfProducts(k2, sinPhi, k1, cosPhi)) * sinAlpha);
    cosBp = Clamp(cosBp, -1, 1);
    Float sinBp = SafeSqrt(1 - Sqr(cosBp));
    Vec cp = cosBp * a + sinBp * Normalize(GramSchmidt(c, a));
    Float cosTheta = 1 - u1 * (1 - Dot(cp, b));
    Float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    Vec w = cosTheta * b + sinTheta * Normalize(GramSchmidt(cp, b));
    Vec e1 = v1 - v0, e2 = v2 - v0;
    Vec s1 = Cross(w, e2);
    Float divisor = Dot(s1, e1);
    if (divisor == 0) { bary[0] = bary[1] = bary[2] = 1.f / 3.f; return true; }
    Float inv = 1 / divisor;
    Vec s = p - v0;
    Float b1 = Dot(s, s1) * inv, b2 = Dot(w, Cross(s, e1)) * inv;
    b1 = Clamp(b1, 0, 1);
    b2 = Clamp(b2, 0, 1);
    if (b1 + b2 > 1) { b1 /= b1 + b2; b2 /= b1 + b2; }
    bary[0] = 1 - b1 - b2; bary[1] = b1; bary[2] = b2;
    return true;
}
static void InvertSphericalTriangleSample(Vec v0, Vec v1, Vec v2, Vec p, Vec w, Float *u0, Float *u1) {
    Vec a = Normalize(v0 - p), b = Normalize(v1 - p), c = Normalize(v2 - p);
    Vec n_ab = Cross(a, b), n_bc = Cross(b, c), n_ca = Cross(c, a);
    if (LengthSquared(n_ab) == 0 || LengthSquared(n_bc) == 0 || LengthSquared(n_ca) == 0) { *u0 = *u1 = 0; return; }
    n_ab = Normalize(n_ab); n_bc = Normalize(n_bc); n_ca = Normalize(n_ca);
    Float alpha = AngleBetween(n_ab, -n_ca), beta = AngleBetween(n_bc, -n_ab), gam = AngleBetween(n_ca, -n_bc);
    Vec cp = Normalize(Cross(Cross(b, w), Cross(c, a)));
    if (Dot(cp, a + c) < 0) cp = -cp;
    Float uu0;
    if (Dot(a, cp) > 0.99999847691f) uu0 = 0;
    else {
        Vec n_cpb = Cross(cp, b), n_acp = Cross(a, cp);
        if (LengthSquared(n_cpb) == 0 || LengthSquared(n_acp) == 0) { *u0 = *u1 = 0.5f; return; }
        n_cpb = Normalize(n_cpb);
        n_acp = Normalize(n_acp);
        Float Ap = alpha + AngleBetween(n_ab, n_cpb) + AngleBetween(n_acp, -n_cpb) - Pi;
        Float A = alpha + beta + gam - Pi;
        uu0 = Ap / A;
    }
    Float uu1 = (1 - Dot(w, b)) / (1 - Dot(cp, b));
    *u0 = Clamp(uu0, 0, 1);
    *u1 = Clamp(uu1, 0, 1);
}

// Triangle::Sample(ctx, u) -> false when pbrt returns {}
struct ShapeSample {
    Vec p, err, n;
    Float pdf;
    Float uv[2] = {0, 0};  // triangles: b0 uv0 + b1 uv1 + b2 uv2 (an image emitter's lookup)
};
static Float TriArea(Vec p0, Vec p1, Vec p2) { return 0.5f * Length(Cross(p1 - p0, p2 - p0)); }
// Triangle::Sample(u)'s normal (shapes.h:1023-1029)
static Vec SampledNormal(Vec p0, Vec p1, Vec p2, bool flip, const TriAttr &a, const Float b[3]) {
    Vec n = Normalize(Cross(p1 - p0, p2 - p0));
    if (a.hasN) {
        Vec ns = b[0] * a.n[0] + b[1] * a.n[1] + (1 - b[0] - b[1]) * a.n[2];
        if (DotN(n, ns) < 0) n = -n;
    } else if (flip) {
        n = n * -1.f;
    }
    return n;
}
static bool TriangleSample(Vec p0, Vec p1, Vec p2, bool flip, Vec ref, Vec ns, Float u0, Float u1, ShapeSample *ss,
                           const TriAttr &a = TriAttr()) {
    Float solidAngle = SphericalTriangleArea(Normalize(p0 - ref), Normalize(p1 - ref), Normalize(p2 - ref));
    if (solidAngle < 3e-4f || solidAngle > 6.22f) {
        Float b[3];
        SampleUniformTriangle(u0, u1, b);
        Vec p = b[0] * p0 + b[1] * p1 + b[2] * p2;
        Vec n = SampledNormal(p0, p1, p2, flip, a, b);
        Point3fi(p, gamma(6) * (Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2)), &p, &ss->err);
        Float pdf = 1 / TriArea(p0, p1, p2);
        Vec wi = p - ref;
        if (LengthSquared(wi) == 0) return false;
        wi = Normalize(wi);
        pdf /= AbsDotN(n, -wi) / DistanceSquared(ref, p);
        if (std::isinf(pdf)) return false;
        ss->p = p;
        ss->n = n;
        ss->pdf = pdf;
        for (int c = 0; c < 2; ++c) ss->uv[c] = b[0] * a.uv[0][c] + b[1] * a.uv[1][c] + b[2] * a.uv[2][c];
        return true;
    }
    Float pdf = 1;
    if (ns != Vec(0, 0, 0)) {
        Vec w0 = Normalize(p0 - ref), w1 = Normalize(p1 - ref), w2 = Normalize(p2 - ref);
        Float w[4] = {std::max<Float>(0.01, AbsDotN(ns, w1)), std::max<Float>(0.01, AbsDotN(ns, w1)),
                      std::max<Float>(0.01, AbsDotN(ns, w0)), std::max<Float>(0.01, AbsDotN(ns, w2))};
        Float x, y;
        SampleBilinear(u0, u1, w, &x, &y);
        u0 = x;
        u1 = y;
        pdf = BilinearPDF(u0, u1, w);
    }
    Float triPDF, b[3];
    SampleSphericalTriangle(p0, p1, p2, ref, u0, u1, b, &triPDF);
    if (triPDF == 0) return false;
    pdf *= triPDF;
    Point3fi(b[0] * p0 + b[1] * p1 + b[2] * p2, gamma(6) * (Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2)),
             &ss->p, &ss->err);
    ss->n = SampledNormal(p0, p1, p2, flip, a, b);
    ss->pdf = pdf;
    for (int c = 0; c < 2; ++c) ss->uv[c] = b[0] * a.uv[0][c] + b[1] * a.uv[1][c] + b[2] * a.uv[2][c];
    return true;
}
static Float TrianglePDF(Vec p0, Vec p1, Vec p2, bool flip, Vec ref, Vec refErr, Vec refN, Vec ns, Vec wi,
                         const TriAttr &a = TriAttr()) {
    Float solidAngle = SphericalTriangleArea(Normalize(p0 - ref), Normalize(p1 - ref), Normalize(p2 - ref));
    if (solidAngle < 3e-4f || solidAngle > 6.22f) {
        Vec o = OffsetRayOrigin(ref, refErr, refN, wi);
        TriIsect ti;
        if (!IntersectTriangle(o, wi, Infinity, p0, p1, p2, &ti)) return 0;
        Interaction si = TriangleInteraction(p0, p1, p2, flip, ti, wi, a);
        Float pdf = (1 / TriArea(p0, p1, p2)) / (AbsDotN(si.n, -wi) / DistanceSquared(ref, si.p));
        if (std::isinf(pdf)) pdf = 0;
        return pdf;
    }
    Float pdf = 1 / solidAngle;
    if (ns != Vec(0, 0, 0)) {
        Float u0, u1;
        InvertSphericalTriangleSample(p0, p1, p2, ref, wi, &u0, &u1);
        Vec w0 = Normalize(p0 - ref), w1 = Normalize(p1 - ref), w2 = Normalize(p2 - ref);
        Float w[4] = {std::max<Float>(0.01, AbsDotN(ns, w1)), std::max<Float>(0.01, AbsDotN(ns, w1)),
                      std::max<Float>(0.01, AbsDotN(ns, w0)), std::max<Float>(0.01, AbsDotN(ns, w2))};
        pdf *= BilinearPDF(u0, u1, w);
    }
    return pdf;
}

// ---------------------------------------------------------------- light sampler
// ---------------------------------------------------------------- spheres and disks
// Sphere / Disk (shapes.h:106-571, shapes.cpp:33-119) over the flat shape records, with pbrt's
// Interval (util/math.h:819-1076) under the CPU rounding helpers NextFloatUp/Down(a op b)
struct OInterval {
    Float lo = 0, hi = 0;
    OInterval() = default;
    explicit OInterval(Float v) : lo(v), hi(v) {}
    OInterval(Float a, Float b) : lo(std::min(a, b)), hi(std::max(a, b)) {}
    static OInterval VE(Float v, Float err) {
        OInterval i(v);
        if (err != 0) {
            i.lo = NextFloatDown(v - err);
            i.hi = NextFloatUp(v + err);
        }
        return i;
    }
    Float Mid() const { return (lo + hi) / 2; }
    Float Err() const { return (hi - lo) / 2; }
    OInterval operator+(OInterval b) const { return {NextFloatDown(lo + b.lo), NextFloatUp(hi + b.hi)}; }
    OInterval operator-(OInterval b) const { return {NextFloatDown(lo - b.hi), NextFloatUp(hi - b.lo)}; }
    OInterval operator*(OInterval b) const {
        return {std::min({NextFloatDown(lo * b.lo), NextFloatDown(hi * b.lo), NextFloatDown(lo * b.hi), NextFloatDown(hi * b.hi)}),
                std::max({NextFloatUp(lo * b.lo), NextFloatUp(hi * b.lo), NextFloatUp(lo * b.hi), NextFloatUp(hi * b.hi)})};
    }
    OInterval operator/(OInterval b) const {
        if (0 >= b.lo && 0 <= b.hi) return {-Infinity, Infinity};
        return {std::min({NextFloatDown(lo / b.lo), NextFloatDown(hi / b.lo), NextFloatDown(lo / b.hi), NextFloatDown(hi / b.hi)}),
                std::max({NextFloatUp(lo / b.lo), NextFloatUp(hi / b.lo), NextFloatUp(lo / b.hi), NextFloatUp(hi / b.hi)})};
    }
    bool operator==(OInterval b) const { return lo == b.lo && hi == b.hi; }
};
static OInterval operator*(Float f, OInterval i) {
    return f > 0 ? OInterval(NextFloatDown(f * i.lo), NextFloatUp(f * i.hi)) : OInterval(NextFloatDown(f * i.hi), NextFloatUp(f * i.lo));
}
static OInterval ISqr(OInterval i) {
    Float a = std::abs(i.lo), b = std::abs(i.hi);
    if (a > b) std::swap(a, b);
    if (0 >= i.lo && 0 <= i.hi) return {0, NextFloatUp(b * b)};
    return {NextFloatDown(a * a), NextFloatUp(b * b)};
}
static OInterval ISqrt(OInterval i) { return {std::max<Float>(0, NextFloatDown(std::sqrt(i.lo))), NextFloatUp(std::sqrt(i.hi))}; }

// Bilinear-patch helpers (util/math.h:614-637 Quadratic, :1420-1426 Determinant; util/vecmath.h
// InvertBilinear, SphericalQuadArea; util/sampling.cpp:163-345 spherical rectangles;
// util/transform.h:249-270 RotateFromTo)
static bool OQuadratic(Float a, Float b, Float c, Float *t0, Float *t1) {
    if (a == 0) {
        if (b == 0) return false;
        *t0 = *t1 = -c / b;
        return true;
    }
    Float disc = DifferenceOfProducts(b, b, 4 * a, c);
    if (disc < 0) return false;
    Float root = std::sqrt(disc);
    Float q = -0.5f * (b + std::copysign(root, b));
    *t0 = q / a;
    *t1 = c / q;
    if (*t0 > *t1) std::swap(*t0, *t1);
    return true;
}
static Float ODet3(const Float m[3][3]) {
    Float minor12 = DifferenceOfProducts(m[1][1], m[2][2], m[1][2], m[2][1]);
    Float minor02 = DifferenceOfProducts(m[1][0], m[2][2], m[1][2], m[2][0]);
    Float minor01 = DifferenceOfProducts(m[1][0], m[2][1], m[1][1], m[2][0]);
    return std::fma(m[0][2], minor01, DifferenceOfProducts(m[0][0], minor12, m[0][1], minor02));
}
static Vec OLerp(Float t, Vec a, Vec b) { return (1 - t) * a + t * b; }
static Float OSphericalQuadArea(Vec a, Vec b, Vec c, Vec d) {
    Vec axb = Cross(a, b), bxc = Cross(b, c), cxd = Cross(c, d), dxa = Cross(d, a);
    if (LengthSquared(axb) == 0 || LengthSquared(bxc) == 0 || LengthSquared(cxd) == 0 || LengthSquared(dxa) == 0) return 0;
    axb = Normalize(axb), bxc = Normalize(bxc), cxd = Normalize(cxd), dxa = Normalize(dxa);
    Float al = AngleBetween(dxa, -axb), be = AngleBetween(axb, -bxc), ga = AngleBetween(bxc, -cxd), de = AngleBetween(cxd, -dxa);
    return std::abs(al + be + ga + de - 2 * Pi);
}
struct ORectFrame {  // Frame::FromXY(ex / |ex|, ey / |ey|), z flipped toward the rectangle
    Vec x, y, z;
    Float x0, y0, z0, x1, y1, exl, eyl;
    ORectFrame(Vec pRef, Vec s, Vec ex, Vec ey) {
        exl = Length(ex), eyl = Length(ey);
        x = ex / exl;
        y = ey / eyl;
        z = Cross(x, y);
        Vec d = s - pRef;
        x0 = Dot(d, x);
        y0 = Dot(d, y);
        z0 = Dot(d, z);
        if (z0 > 0) {
            z = -z;
            z0 *= -1;
        }
        x1 = x0 + exl;
        y1 = y0 + eyl;
    }
    void Angles(Vec *n0, Vec *n2, Float g[4]) const {
        Vec v00(x0, y0, z0), v01(x0, y1, z0), v10(x1, y0, z0), v11(x1, y1, z0);
        Vec a = Normalize(Cross(v00, v10)), b = Normalize(Cross(v10, v11)), c = Normalize(Cross(v11, v01)),
            d = Normalize(Cross(v01, v00));
        g[0] = AngleBetween(-a, b);
        g[1] = AngleBetween(-b, c);
        g[2] = AngleBetween(-c, d);
        g[3] = AngleBetween(-d, a);
        *n0 = a;
        *n2 = c;
    }
};
static Vec OSampleSphericalRectangle(Vec pRef, Vec s, Vec ex, Vec ey, Float u0, Float u1, Float *pdf) {
    ORectFrame R(pRef, s, ex, ey);
    Vec n0, n2;
    Float g[4];
    R.Angles(&n0, &n2, g);
    Float solid = g[0] + g[1] + g[2] + g[3] - 2 * Pi;
    if (solid <= 0) {
        *pdf = 0;
        return s + u0 * ex + u1 * ey;
    }
    *pdf = std::max<Float>(0, 1 / solid);
    if (solid < 1e-3f) return s + u0 * ex + u1 * ey;
    Float b0 = n0.z, b1 = n2.z;
    Float au = u0 * (g[0] + g[1] - 2 * Pi) + (u0 - 1) * (g[2] + g[3]);
    Float fu = (CRCos(au) * b0 - b1) / CRSin(au);
    Float cu = std::copysign(1 / std::sqrt(Sqr(fu) + Sqr(b0)), fu);
    cu = Clamp(cu, -OneMinusEpsilon, OneMinusEpsilon);
    Float xu = Clamp(-(cu * R.z0) / SafeSqrt(1 - Sqr(cu)), R.x0, R.x1);
    Float dd = std::sqrt(Sqr(xu) + Sqr(R.z0));
    Float h0 = R.y0 / std::sqrt(Sqr(dd) + Sqr(R.y0)), h1 = R.y1 / std::sqrt(Sqr(dd) + Sqr(R.y1));
    Float hv = h0 + u1 * (h1 - h0), hvsq = Sqr(hv);
    Float yv = (hvsq < 1 - 1e-6f) ? (hv * dd) / std::sqrt(1 - hvsq) : R.y1;
    return pRef + (R.x * xu + R.y * yv + R.z * R.z0);
}
static void OInvertSphericalRectangle(Vec pRef, Vec s, Vec ex, Vec ey, Vec pRect, Float *ru0, Float *ru1) {
    ORectFrame R(pRef, s, ex, ey);
    Vec n0, n2;
    Float g[4];
    R.Angles(&n0, &n2, g);
    Float b0 = n0.z, b1 = n2.z, b0sq = Sqr(b0);
    Float solid = double(g[0]) + double(g[1]) + double(g[2]) + double(g[3]) - 2. * Pi;
    if (solid < 1e-3f) {
        Vec pq = pRect - s;
        *ru0 = Dot(pq, ex) / LengthSquared(ex);
        *ru1 = Dot(pq, ey) / LengthSquared(ey);
        return;
    }
    Vec v = pRect - pRef;
    Float xu = Clamp(Dot(v, R.x), R.x0, R.x1), yv = Dot(v, R.y);
    if (xu == 0) xu = 1e-10f;
    Float z0sq = Sqr(R.z0);
    Float fusq = (1 + z0sq / Sqr(xu)) - b0sq;
    Float fu = std::copysign(std::sqrt(fusq), xu);
    Float sq = SafeSqrt(DifferenceOfProducts(b0, b0, b1, b1) + fusq);
    Float au = CRATan2(-(b1 * fu) - std::copysign(b0 * sq, fu * b0), b0 * b1 - sq * std::abs(fu));
    if (au > 0) au -= 2 * Pi;
    if (fu == 0) au = Pi;
    Float u0 = (au + g[2] + g[3]) / solid;
    Float ddsq = Sqr(xu) + z0sq, dd = std::sqrt(ddsq);
    Float h0 = R.y0 / std::sqrt(ddsq + Sqr(R.y0)), h1 = R.y1 / std::sqrt(ddsq + Sqr(R.y1));
    Float yvsq = Sqr(yv);
    Float term = std::abs(h0 - h1) * std::sqrt(yvsq * (ddsq + yvsq)) / (ddsq + yvsq);
    Float ua = (DifferenceOfProducts(h0, h0, h0, h1) - term) / Sqr(h0 - h1);
    Float ub = (DifferenceOfProducts(h0, h0, h0, h1) + term) / Sqr(h0 - h1);
    Float ha = Lerp(ua, h0, h1), hb = Lerp(ub, h0, h1);
    Float ya = (ha * dd) / std::sqrt(1 - Sqr(ha)), yb = (hb * dd) / std::sqrt(1 - Sqr(hb));
    *ru0 = Clamp(u0, 0, 1);
    *ru1 = (std::abs(ya - yv) < std::abs(yb - yv)) ? ua : ub;
}
static Vec ORotateFromTo(Vec from, Vec to, Vec w) {
    Vec refl;
    if (std::abs(from.x) < 0.72f && std::abs(to.x) < 0.72f) refl = Vec(1, 0, 0);
    else if (std::abs(from.y) < 0.72f && std::abs(to.y) < 0.72f) refl = Vec(0, 1, 0);
    else refl = Vec(0, 0, 1);
    Vec u = refl - from, v = refl - to;
    Float m[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            m[i][j] = ((i == j) ? 1 : 0) - 2 / Dot(u, u) * u[i] * u[j] - 2 / Dot(v, v) * v[i] * v[j] +
                      4 * Dot(u, v) / (Dot(u, u) * Dot(v, v)) * v[i] * u[j];
    return Vec(m[0][0] * w.x + m[0][1] * w.y + m[0][2] * w.z, m[1][0] * w.x + m[1][1] * w.y + m[1][2] * w.z,
               m[2][0] * w.x + m[2][1] * w.y + m[2][2] * w.z);
}

struct OShape {
    int kind = 0, flags = 0;
    const float *r2o = nullptr, *o2r = nullptr;  // 3x4 row major
    Float a = 0, b = 0, c = 0, d = 0, e = 0, g = 0;
    // bilinear patch: corners, corner uvs, vertex normals; the oracle's own area / rectangle test
    Vec P[4], Nv[4];
    Float UV[4][2];
    bool rect = false;
    Float patchArea = 0;
    void Init(const pbrt_scene_flat *f, int k) {
        const int32_t *info = f->shape_info + 8 * k;
        const float *pp = f->shape_params + 32 * k;
        kind = info[0];
        flags = info[1];
        r2o = pp;
        o2r = pp + 12;
        a = pp[24], b = pp[25], c = pp[26], d = pp[27], e = pp[28], g = pp[29];
        if (kind == 3) {
            for (int i = 0; i < 4; ++i) {
                P[i] = Vec(pp[3 * i], pp[3 * i + 1], pp[3 * i + 2]);
                UV[i][0] = pp[12 + 2 * i];
                UV[i][1] = pp[12 + 2 * i + 1];
                const float *n = f->shape_normals + 12 * k + 3 * i;
                Nv[i] = Vec(n[0], n[1], n[2]);
            }
            InitPatch();
        }
    }
    bool sphere() const { return kind == 1; }
    bool cylinder() const { return kind == 4; }
    bool patch() const { return kind == 3; }
    bool flip() const { return ((flags & 1) != 0) != ((flags & 2) != 0); }
    // BilinearPatch ctor (shapes.cpp:1041-1071) with IsRectangle (shapes.h:1511-1532)
    void InitPatch() {
        const Vec p00 = P[0], p10 = P[1], p01 = P[2], p11 = P[3];
        rect = !(p00 == p01 || p01 == p11 || p11 == p10 || p10 == p00);
        if (rect && AbsDotN(Normalize(Cross(p10 - p00, p01 - p00)), Normalize(p11 - p00)) > 1e-5f) rect = false;
        if (rect) {
            Vec pc = (p00 + p01 + p10 + p11) / 4;
            Float d2[4] = {DistanceSquared(p00, pc), DistanceSquared(p01, pc), DistanceSquared(p10, pc), DistanceSquared(p11, pc)};
            for (int i = 1; i < 4; ++i)
                if (std::abs(d2[i] - d2[0]) / d2[0] > 1e-4f) rect = false;
        }
        if (rect) {
            patchArea = Length(p00 - p01) * Length(p00 - p10);
        } else {
            Vec q[4][4];
            for (int i = 0; i <= 3; ++i)
                for (int j = 0; j <= 3; ++j) q[i][j] = OLerp(Float(i) / Float(3), OLerp(Float(j) / Float(3), p00, p01), OLerp(Float(j) / Float(3), p10, p11));
            patchArea = 0;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) patchArea += 0.5f * Length(Cross(q[i + 1][j + 1] - q[i][j], q[i + 1][j] - q[i][j + 1]));
        }
    }
    Float Area() const {
        if (patch()) return patchArea;
        if (cylinder()) return (c - b) * a * d;  // Cylinder::Area (shapes.h:620)
        return sphere() ? d * a * (c - b) : d * Float(0.5) * (Sqr(b) - Sqr(c));
    }
    // IntersectBilinearPatch (shapes.h:1279-1347)
    bool PatchIntersect(Vec o, Vec dir, Float tMax, Float *tHit, Float *uo, Float *vo) const {
        const Vec p00 = P[0], p10 = P[1], p01 = P[2], p11 = P[3];
        Float qa = Dot(Cross(p10 - p00, p01 - p11), dir);
        Float qc = Dot(Cross(p00 - o, dir), p01 - p00);
        Float qb = Dot(Cross(p10 - o, dir), p11 - p10) - (qa + qc);
        Float u1, u2;
        if (!OQuadratic(qa, qb, qc, &u1, &u2)) return false;
        Float eps = gamma(10) * (MaxComp(Abs(o)) + MaxComp(Abs(dir)) + MaxComp(Abs(p00)) + MaxComp(Abs(p10)) +
                                 MaxComp(Abs(p01)) + MaxComp(Abs(p11)));
        Float t = tMax, u = 0, v = 0;
        auto solve = [&](Float uu, Float *vv, Float *tt, Float *p2) {
            Vec uo2 = OLerp(uu, p00, p10), ud = OLerp(uu, p01, p11) - uo2, deltao = uo2 - o, perp = Cross(dir, ud);
            *p2 = LengthSquared(perp);
            const Float mv[3][3] = {{deltao.x, dir.x, perp.x}, {deltao.y, dir.y, perp.y}, {deltao.z, dir.z, perp.z}};
            const Float mt[3][3] = {{deltao.x, ud.x, perp.x}, {deltao.y, ud.y, perp.y}, {deltao.z, ud.z, perp.z}};
            *vv = ODet3(mv);
            *tt = ODet3(mt);
        };
        if (0 <= u1 && u1 <= 1) {
            Float v1, t1, p2;
            solve(u1, &v1, &t1, &p2);
            if (t1 > p2 * eps && 0 <= v1 && v1 <= p2) {
                u = u1;
                v = v1 / p2;
                t = t1 / p2;
            }
        }
        if (0 <= u2 && u2 <= 1 && u2 != u1) {
            Float v2, t2, p2;
            solve(u2, &v2, &t2, &p2);
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
    // BilinearPatch::InteractionFromIntersection (shapes.h:1396-1497)
    Interaction PatchSurface(Float u, Float v) const {
        const Vec p00 = P[0], p10 = P[1], p01 = P[2], p11 = P[3];
        Vec p = OLerp(u, OLerp(v, p00, p01), OLerp(v, p10, p11));
        Vec dpdu = OLerp(v, p10, p11) - OLerp(v, p00, p01), dpdv = OLerp(u, p01, p11) - OLerp(u, p00, p10);
        Float st[2] = {u, v};
        if (flags & 4) {
            Float dstdu[2], dstdv[2];
            for (int j = 0; j < 2; ++j) {
                st[j] = Lerp(u, Lerp(v, UV[0][j], UV[2][j]), Lerp(v, UV[1][j], UV[3][j]));
                dstdu[j] = Lerp(v, UV[1][j], UV[3][j]) - Lerp(v, UV[0][j], UV[2][j]);
                dstdv[j] = Lerp(u, UV[2][j], UV[3][j]) - Lerp(u, UV[0][j], UV[1][j]);
            }
            Float duds = std::abs(dstdu[0]) < 1e-8f ? 0 : 1 / dstdu[0];
            Float dvds = std::abs(dstdv[0]) < 1e-8f ? 0 : 1 / dstdv[0];
            Float dudt = std::abs(dstdu[1]) < 1e-8f ? 0 : 1 / dstdu[1];
            Float dvdt = std::abs(dstdv[1]) < 1e-8f ? 0 : 1 / dstdv[1];
            Vec dpds = dpdu * duds + dpdv * dvds, dpdt = dpdu * dudt + dpdv * dvdt;
            if (Cross(dpds, dpdt) != Vec(0, 0, 0)) {
                if (Dot(Cross(dpdu, dpdv), Cross(dpds, dpdt)) < 0) dpdt = -dpdt;
                dpdu = dpds;
                dpdv = dpdt;
            }
        }
        Interaction si;
        Point3fi(p, gamma(6) * (Abs(p00) + Abs(p01) + Abs(p10) + Abs(p11)), &si.p, &si.err);
        Vec n = Normalize(Cross(dpdu, dpdv));
        if (flip()) n = -n;
        si.n = si.ns = n;
        si.dpdu = si.dpdus = dpdu;
        si.dpdv = dpdv;
        si.uv[0] = st[0];
        si.uv[1] = st[1];
        if (flags & 8) {
            Vec ns = OLerp(u, OLerp(v, Nv[0], Nv[2]), OLerp(v, Nv[1], Nv[3]));
            if (LengthSquared(ns) > 0) {
                ns = Normalize(ns);
                Vec sd = ORotateFromTo(Normalize(si.n), ns, dpdu), sv = ORotateFromTo(Normalize(si.n), ns, dpdv);
                si.ns = ns;
                if (DotN(si.n, ns) < 0) si.n = -si.n;  // SetShadingGeometry(..., true)
                while (LengthSquared(sd) > 1e16f || LengthSquared(sv) > 1e16f) {
                    sd = sd / 1e8f;
                    sv = sv / 1e8f;
                }
                si.dpdus = sd;
            }
        }
        return si;
    }
    Vec PatchNormalAt(Vec n, Float u, Float v) const {
        if (flags & 8) {
            Vec ns = OLerp(u, OLerp(v, Nv[0], Nv[2]), OLerp(v, Nv[1], Nv[3]));
            return DotN(n, ns) < 0 ? -n : n;
        }
        return flip() ? -n : n;
    }
    void PatchWeights(Float w[4]) const {
        const Vec p00 = P[0], p10 = P[1], p01 = P[2], p11 = P[3];
        w[0] = Length(Cross(p10 - p00, p01 - p00));
        w[1] = Length(Cross(p10 - p00, p11 - p10));
        w[2] = Length(Cross(p01 - p00, p11 - p01));
        w[3] = Length(Cross(p11 - p10, p11 - p01));
    }
    // a sample's (s, t): the mesh uv lerp at parametric (u, v) when the patch has uv
    void PatchST(Float u, Float v, Float st[2]) const {
        st[0] = u;
        st[1] = v;
        if (flags & 4)
            for (int j = 0; j < 2; ++j) st[j] = Lerp(u, Lerp(v, UV[0][j], UV[2][j]), Lerp(v, UV[1][j], UV[3][j]));
    }
    // BilinearPatch::Sample(u) (shapes.cpp:1158-1217)
    bool PatchSampleArea(Float u0, Float u1, ShapeSample *ss) const {
        Float pdf = 1, u = u0, v = u1;
        if (!rect) {
            Float w[4];
            PatchWeights(w);
            SampleBilinear(u0, u1, w, &u, &v);
            pdf = BilinearPDF(u, v, w);
        }
        Vec pu0 = OLerp(v, P[0], P[2]), pu1 = OLerp(v, P[1], P[3]);
        Vec p = OLerp(u, pu0, pu1), dpdu = pu1 - pu0, dpdv = OLerp(u, P[2], P[3]) - OLerp(u, P[0], P[1]);
        if (LengthSquared(dpdu) == 0 || LengthSquared(dpdv) == 0) return false;
        ss->n = PatchNormalAt(Normalize(Cross(dpdu, dpdv)), u, v);
        Point3fi(p, gamma(6) * (Abs(P[0]) + Abs(P[2]) + Abs(P[1]) + Abs(P[3])), &ss->p, &ss->err);
        ss->pdf = pdf / Length(Cross(dpdu, dpdv));
        PatchST(u, v, ss->uv);
        return true;
    }
    // BilinearPatch::Sample(ctx, u) and PDF(ctx, wi) (shapes.cpp:1257-1372)
    bool PatchSample(Vec cp, Vec cns, Float u0, Float u1, ShapeSample *out) const {
        Vec v00 = Normalize(P[0] - cp), v10 = Normalize(P[1] - cp), v01 = Normalize(P[2] - cp), v11 = Normalize(P[3] - cp);
        if (!rect || OSphericalQuadArea(v00, v10, v11, v01) <= 1e-4f) {
            ShapeSample ss;
            if (!PatchSampleArea(u0, u1, &ss)) return false;
            Vec wi = ss.p - cp;
            if (LengthSquared(wi) == 0) return false;
            wi = Normalize(wi);
            ss.pdf /= AbsDotN(ss.n, -wi) / DistanceSquared(cp, ss.p);
            if (std::isinf(ss.pdf)) return false;
            *out = ss;
            return true;
        }
        Float pdf = 1, uu = u0, vv = u1;
        if (cns != Vec(0, 0, 0)) {
            Float w[4] = {std::max<Float>(0.01f, AbsDotN(cns, v00)), std::max<Float>(0.01f, AbsDotN(cns, v10)),
                          std::max<Float>(0.01f, AbsDotN(cns, v01)), std::max<Float>(0.01f, AbsDotN(cns, v11))};
            SampleBilinear(u0, u1, w, &uu, &vv);
            pdf *= BilinearPDF(uu, vv, w);
        }
        Vec eu = P[1] - P[0], ev = P[2] - P[0];
        Float qpdf;
        Vec p = OSampleSphericalRectangle(cp, P[0], eu, ev, uu, vv, &qpdf);
        pdf *= qpdf;
        Float su = Dot(p - P[0], eu) / DistanceSquared(P[1], P[0]), sv = Dot(p - P[0], ev) / DistanceSquared(P[2], P[0]);
        out->n = PatchNormalAt(Normalize(Cross(eu, ev)), su, sv);
        out->p = p;
        out->err = Vec(0, 0, 0);
        out->pdf = pdf;
        PatchST(su, sv, out->uv);
        return true;
    }
    Float PatchPDF(Vec cp, Vec cpErr, Vec cn, Vec cns, Vec wi) const {
        Vec ro = OffsetRayOrigin(cp, cpErr, cn, wi);
        Float th, iu, iv;
        if (!PatchIntersect(ro, wi, Infinity, &th, &iu, &iv)) return 0;
        Interaction si = PatchSurface(iu, iv);
        Vec v00 = Normalize(P[0] - cp), v10 = Normalize(P[1] - cp), v01 = Normalize(P[2] - cp), v11 = Normalize(P[3] - cp);
        if (!rect || OSphericalQuadArea(v00, v10, v11, v01) <= 1e-4f) {
            Float u = si.uv[0], v = si.uv[1];
            if (flags & 4) {
                // InvertBilinear(uv, {uv00, uv10, uv01, uv11}): a = uv00, b = uv10, c = uv11, d = uv01
                const Float *A = UV[0], *B = UV[1], *C = UV[3], *D = UV[2];
                Float ee[2] = {B[0] - A[0], B[1] - A[1]}, ff[2] = {D[0] - A[0], D[1] - A[1]};
                Float gg[2] = {(A[0] - B[0]) + (C[0] - D[0]), (A[1] - B[1]) + (C[1] - D[1])}, hh[2] = {u - A[0], v - A[1]};
                auto cr = [](const Float *x, const Float *y) { return DifferenceOfProducts(x[0], y[1], x[1], y[0]); };
                Float k2 = cr(gg, ff), k1 = cr(ee, ff) + cr(hh, gg), k0 = cr(hh, ee);
                if (std::abs(k2) < 0.001f) {
                    u = std::abs(ee[0] * k1 - gg[0] * k0) < 1e-5f ? (hh[1] * k1 + ff[1] * k0) / (ee[1] * k1 - gg[1] * k0)
                                                                 : (hh[0] * k1 + ff[0] * k0) / (ee[0] * k1 - gg[0] * k0);
                    v = -k0 / k1;
                } else {
                    Float w0, w1;
                    if (!OQuadratic(k2, k1, k0, &w0, &w1)) {
                        u = v = 0;
                    } else {
                        Float uu = (hh[0] - ff[0] * w0) / (ee[0] + gg[0] * w0);
                        if (uu < 0 || uu > 1 || w0 < 0 || w0 > 1) {
                            u = (hh[0] - ff[0] * w1) / (ee[0] + gg[0] * w1);
                            v = w1;
                        } else {
                            u = uu;
                            v = w0;
                        }
                    }
                }
            }
            Float pdf = 1;
            if (!rect) {
                Float w[4];
                PatchWeights(w);
                pdf = BilinearPDF(u, v, w);
            }
            Vec pu0 = OLerp(v, P[0], P[2]), pu1 = OLerp(v, P[1], P[3]);
            Vec dpdu = pu1 - pu0, dpdv = OLerp(u, P[2], P[3]) - OLerp(u, P[0], P[1]);
            pdf = pdf / Length(Cross(dpdu, dpdv));
            pdf = pdf * (DistanceSquared(cp, si.p) / AbsDotN(si.n, -wi));
            return std::isinf(pdf) ? 0 : pdf;
        }
        Float pdf = 1 / OSphericalQuadArea(v00, v10, v11, v01);
        if (cns != Vec(0, 0, 0)) {
            Float w[4] = {std::max<Float>(0.01f, AbsDotN(cns, v00)), std::max<Float>(0.01f, AbsDotN(cns, v10)),
                          std::max<Float>(0.01f, AbsDotN(cns, v01)), std::max<Float>(0.01f, AbsDotN(cns, v11))};
            Float su, sv;
            OInvertSphericalRectangle(cp, P[0], P[1] - P[0], P[2] - P[0], si.p, &su, &sv);
            return BilinearPDF(su, sv, w) * pdf;
        }
        return pdf;
    }
    // Transform::operator() on points / vectors / normals (util/transform.h:133-176, 272-334)
    static void XPointI(const float *m, const OInterval in[3], OInterval out[3]) {
        const Float x = in[0].Mid(), y = in[1].Mid(), z = in[2].Mid();
        const Float ex = in[0].Err(), ey = in[1].Err(), ez = in[2].Err();
        const bool exact = ex == 0 && ey == 0 && ez == 0;
        for (int i = 0; i < 3; ++i) {
            const float *r = m + 4 * i;
            const Float v = (r[0] * x + r[1] * y) + (r[2] * z + r[3]);
            Float err = gamma(3) * (std::abs(r[0] * x) + std::abs(r[1] * y) + std::abs(r[2] * z) + std::abs(r[3]));
            if (!exact) err = (gamma(3) + 1) * (std::abs(r[0]) * ex + std::abs(r[1]) * ey + std::abs(r[2]) * ez) + err;
            out[i] = OInterval::VE(v, err);
        }
    }
    static void XVectorExact(const float *m, Vec v, OInterval out[3]) {
        for (int i = 0; i < 3; ++i) {
            const float *r = m + 4 * i;
            const Float err = gamma(3) * (std::abs(r[0] * v.x) + std::abs(r[1] * v.y) + std::abs(r[2] * v.z));
            out[i] = OInterval::VE(r[0] * v.x + r[1] * v.y + r[2] * v.z, err);
        }
    }
    static Vec XV(const float *m, Vec v) {
        return Vec(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z, m[8] * v.x + m[9] * v.y + m[10] * v.z);
    }
    static Vec XN(const float *mInv, Vec n) {
        return Vec(mInv[0] * n.x + mInv[4] * n.y + mInv[8] * n.z, mInv[1] * n.x + mInv[5] * n.y + mInv[9] * n.z,
                   mInv[2] * n.x + mInv[6] * n.y + mInv[10] * n.z);
    }
    static Vec XP(const float *m, Vec p) {
        return Vec(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
                   m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
    }
    static Float Phi(Vec p) {
        Float phi = CRATan2(p.y, p.x);
        if (phi < 0) phi += 2 * Pi;
        return phi;
    }
    // BasicIntersect -> tHit and the object-space hit
    bool Intersect(Vec ro, Vec rd, Float tMax, Float *tHit, Vec *pObj) const {
        if (patch()) {
            Float u, v;
            if (!PatchIntersect(ro, rd, tMax, tHit, &u, &v)) return false;
            *pObj = Vec(u, v, 0);
            return true;
        }
        OInterval oi[3], di[3];
        const OInterval ro3[3] = {OInterval(ro.x), OInterval(ro.y), OInterval(ro.z)};
        XPointI(r2o, ro3, oi);
        XVectorExact(r2o, rd, di);
        const Vec o(oi[0].Mid(), oi[1].Mid(), oi[2].Mid()), dd(di[0].Mid(), di[1].Mid(), di[2].Mid());
        if (cylinder()) {
            // Cylinder::BasicIntersect (shapes.h:628-722): x-y quadratic, hit reprojected to r
            const Float radius = a, zMin = b, zMax = c, phiMax = d;
            const OInterval A = ISqr(di[0]) + ISqr(di[1]);
            const OInterval B = 2.f * (di[0] * oi[0] + di[1] * oi[1]);
            const OInterval C = ISqr(oi[0]) + ISqr(oi[1]) - ISqr(OInterval(radius));
            const OInterval fct = B / (2.f * A);
            const OInterval vx = oi[0] - fct * di[0], vy = oi[1] - fct * di[1];
            const OInterval len = ISqrt(ISqr(vx) + ISqr(vy));
            const OInterval disc = 4.f * A * (OInterval(radius) + len) * (OInterval(radius) - len);
            if (disc.lo < 0) return false;
            const OInterval root = ISqrt(disc);
            const OInterval q = B.Mid() < 0 ? -.5f * (B - root) : -.5f * (B + root);
            OInterval t0 = q / A, t1 = C / q;
            if (t0.lo > t1.lo) std::swap(t0, t1);
            if (t0.hi > tMax || t1.lo <= 0) return false;
            OInterval ts = t0;
            if (ts.lo <= 0) {
                ts = t1;
                if (ts.hi > tMax) return false;
            }
            Vec p;
            Float phi;
            auto hitAt = [&](OInterval t) {
                p = o + t.Mid() * dd;
                const Float hitRad = std::sqrt(Sqr(p.x) + Sqr(p.y));
                p.x *= radius / hitRad;
                p.y *= radius / hitRad;
                phi = Phi(p);
            };
            hitAt(ts);
            if (p.z < zMin || p.z > zMax || phi > phiMax) {
                if (ts == t1) return false;
                ts = t1;
                if (t1.hi > tMax) return false;
                hitAt(ts);
                if (p.z < zMin || p.z > zMax || phi > phiMax) return false;
            }
            *tHit = ts.Mid();
            *pObj = p;
            return true;
        }
        if (!sphere()) {
            if (dd.z == 0) return false;
            const Float th = (a - o.z) / dd.z;
            if (th <= 0 || th >= tMax) return false;
            const Vec p = o + th * dd;
            const Float dist2 = Sqr(p.x) + Sqr(p.y);
            if (dist2 > Sqr(b) || dist2 < Sqr(c)) return false;
            if (Phi(p) > d) return false;
            *tHit = th;
            *pObj = p;
            return true;
        }
        const Float radius = a, zMin = b, zMax = c, phiMax = d;
        const OInterval A = ISqr(di[0]) + ISqr(di[1]) + ISqr(di[2]);
        const OInterval B = 2.f * (di[0] * oi[0] + di[1] * oi[1] + di[2] * oi[2]);
        const OInterval C = ISqr(oi[0]) + ISqr(oi[1]) + ISqr(oi[2]) - ISqr(OInterval(radius));
        const OInterval fct = B / (2.f * A);
        OInterval v[3];
        for (int i = 0; i < 3; ++i) v[i] = oi[i] - fct * di[i];
        const OInterval len = ISqrt(ISqr(v[0]) + ISqr(v[1]) + ISqr(v[2]));
        const OInterval disc = 4.f * A * (OInterval(radius) + len) * (OInterval(radius) - len);
        if (disc.lo < 0) return false;
        const OInterval root = ISqrt(disc);
        const OInterval q = B.Mid() < 0 ? -.5f * (B - root) : -.5f * (B + root);
        OInterval t0 = q / A, t1 = C / q;
        if (t0.lo > t1.lo) std::swap(t0, t1);
        if (t0.hi > tMax || t1.lo <= 0) return false;
        OInterval ts = t0;
        if (ts.lo <= 0) {
            ts = t1;
            if (ts.hi > tMax) return false;
        }
        auto hitAt = [&](OInterval t, Vec *p, Float *phi) {
            *p = o + t.Mid() * dd;
            *p = *p * (radius / Length(*p));
            if (p->x == 0 && p->y == 0) p->x = 1e-5f * radius;
            *phi = Phi(*p);
        };
        Vec p;
        Float phi;
        hitAt(ts, &p, &phi);
        auto clipped = [&]() { return (zMin > -radius && p.z < zMin) || (zMax < radius && p.z > zMax) || phi > phiMax; };
        if (clipped()) {
            if (ts == t1) return false;
            if (t1.hi > tMax) return false;
            ts = t1;
            hitAt(ts, &p, &phi);
            if (clipped()) return false;
        }
        *tHit = ts.Mid();
        *pObj = p;
        return true;
    }
    // InteractionFromIntersection + Transform::operator()(SurfaceInteraction)
    Interaction Surface(Vec pHit, Vec rd) const {
        if (patch()) {
            Interaction si = PatchSurface(pHit.x, pHit.y);
            si.wo = Normalize(-rd);
            return si;
        }
        const Float phi = Phi(pHit);
        Vec dpdu, dpdv, pErr;
        Float u, v;
        if (sphere()) {
            const Float radius = a, phiMax = d, tzMin = e, tzMax = g;
            u = phi / phiMax;
            const Float cosTheta = pHit.z / radius, theta = SafeACos(cosTheta);
            v = (theta - tzMin) / (tzMax - tzMin);
            const Float zr = std::sqrt(Sqr(pHit.x) + Sqr(pHit.y));
            const Float cp = pHit.x / zr, sp = pHit.y / zr;
            dpdu = Vec(-phiMax * pHit.y, phiMax * pHit.x, 0);
            const Float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
            dpdv = (tzMax - tzMin) * Vec(pHit.z * cp, pHit.z * sp, -radius * sinTheta);
            pErr = gamma(5) * Abs(pHit);
        } else if (cylinder()) {  // Cylinder::InteractionFromIntersection (shapes.h:725-760)
            u = phi / d;
            v = (pHit.z - b) / (c - b);
            dpdu = Vec(-d * pHit.y, d * pHit.x, 0);
            dpdv = Vec(0, 0, c - b);
            pErr = gamma(3) * Abs(Vec(pHit.x, pHit.y, 0));
        } else {
            const Float radius = b, inner = c, phiMax = d;
            u = phi / phiMax;
            const Float rHit = std::sqrt(Sqr(pHit.x) + Sqr(pHit.y));
            v = (radius - rHit) / (radius - inner);
            dpdu = Vec(-phiMax * pHit.y, phiMax * pHit.x, 0);
            dpdv = Vec(pHit.x, pHit.y, 0) * (inner - radius) / rHit;
            pHit.z = a;
            pErr = Vec(0, 0, 0);
        }
        Vec n = Normalize(Cross(dpdu, dpdv));
        if (((flags & 1) != 0) != ((flags & 2) != 0)) n = -n;
        const OInterval pi[3] = {OInterval::VE(pHit.x, pErr.x), OInterval::VE(pHit.y, pErr.y), OInterval::VE(pHit.z, pErr.z)};
        OInterval po[3];
        XPointI(o2r, pi, po);
        Interaction si;
        si.p = Vec(po[0].Mid(), po[1].Mid(), po[2].Mid());
        si.err = Vec(po[0].Err(), po[1].Err(), po[2].Err());
        si.n = Normalize(XN(r2o, n));
        si.dpdu = si.dpdus = XV(o2r, dpdu);
        si.dpdv = XV(o2r, dpdv);
        Vec ns = Normalize(XN(r2o, n));
        if (DotN(ns, si.n) < 0) ns = -ns;  // FaceForward(shading.n, n)
        si.ns = ns;
        si.uv[0] = u;
        si.uv[1] = v;
        si.wo = Normalize(-rd);
        return si;
    }
    // a sphere point's (phi / phiMax, (theta - thetaZMin) / (thetaZMax - thetaZMin)) (shapes.cpp:54-58)
    void SphereUV(Vec pObj, Float uv[2]) const {
        const Float theta = SafeACos(pObj.z / a);
        Float ph = CRATan2(pObj.y, pObj.x);
        if (ph < 0) ph += 2 * Pi;
        uv[0] = ph / d;
        uv[1] = (theta - e) / (g - e);
    }
    // Sphere::Sample(u) / Disk::Sample(u): area measure
    ShapeSample SampleArea(Float u0, Float u1) const {
        ShapeSample ss;
        if (sphere()) {
            const Float z = 1 - 2 * u0, r = SafeSqrt(1 - Sqr(z)), ph = 2 * Pi * u1;
            Vec pObj = Vec(0, 0, 0) + a * Vec(r * CRCos(ph), r * CRSin(ph), z);
            pObj = pObj * (a / Length(pObj));
            const Vec pErr = gamma(5) * Abs(pObj);
            Vec n = Normalize(XN(r2o, pObj));
            if (flags & 1) n = -n;
            const OInterval pi[3] = {OInterval::VE(pObj.x, pErr.x), OInterval::VE(pObj.y, pErr.y), OInterval::VE(pObj.z, pErr.z)};
            OInterval po[3];
            XPointI(o2r, pi, po);
            ss.p = Vec(po[0].Mid(), po[1].Mid(), po[2].Mid());
            ss.err = Vec(po[0].Err(), po[1].Err(), po[2].Err());
            ss.n = n;
            SphereUV(pObj, ss.uv);
        } else if (cylinder()) {  // Cylinder::Sample(u) (shapes.h:772-793)
            const Float z = Lerp(u0, b, c), ph = u1 * d;
            Vec pObj(a * CRCos(ph), a * CRSin(ph), z);
            const Float hitRad = std::sqrt(Sqr(pObj.x) + Sqr(pObj.y));
            pObj.x *= a / hitRad;
            pObj.y *= a / hitRad;
            const Vec pErr = gamma(3) * Abs(Vec(pObj.x, pObj.y, 0));
            const OInterval pi[3] = {OInterval::VE(pObj.x, pErr.x), OInterval::VE(pObj.y, pErr.y), OInterval::VE(pObj.z, pErr.z)};
            OInterval po[3];
            XPointI(o2r, pi, po);
            ss.p = Vec(po[0].Mid(), po[1].Mid(), po[2].Mid());
            ss.err = Vec(po[0].Err(), po[1].Err(), po[2].Err());
            Vec n = Normalize(XN(r2o, Vec(pObj.x, pObj.y, 0)));
            if (flags & 1) n = -n;
            ss.n = n;
            ss.uv[0] = ph / d;
            ss.uv[1] = (pObj.z - b) / (c - b);
        } else {
            Float dx, dy;
            SampleUniformDiskConcentric(u0, u1, &dx, &dy);
            // Disk::Sample(u)'s (u, v) (shapes.h:517-522)
            Float dphi = CRATan2(dy, dx);
            if (dphi < 0) dphi += 2 * Pi;
            const Float rs = std::sqrt(Sqr(dx * b) + Sqr(dy * b));
            ss.uv[0] = dphi / d;
            ss.uv[1] = (b - rs) / (b - c);
            const OInterval pi[3] = {OInterval(dx * b), OInterval(dy * b), OInterval(a)};
            OInterval po[3];
            XPointI(o2r, pi, po);
            ss.p = Vec(po[0].Mid(), po[1].Mid(), po[2].Mid());
            ss.err = Vec(po[0].Err(), po[1].Err(), po[2].Err());
            Vec n = Normalize(XN(r2o, Vec(0, 0, 1)));
            if (flags & 1) n = -n;
            ss.n = n;
        }
        ss.pdf = 1 / Area();
        return ss;
    }
    // Shape::Sample(ctx, u), solid angle (false: {})
    bool Sample(Vec cp, Vec cpErr, Vec cn, Float u0, Float u1, ShapeSample *out, Vec cns = Vec(0, 0, 0)) const {
        if (patch()) return PatchSample(cp, cns, u0, u1, out);
        if (sphere()) {
            const Vec pc = XP(o2r, Vec(0, 0, 0));
            const Vec po = OffsetRayOrigin(cp, cpErr, cn, pc - cp);
            if (DistanceSquared(po, pc) > Sqr(a)) {
                const Float sinMax = a / Length(cp - pc), sin2Max = Sqr(sinMax), cosMax = SafeSqrt(1 - sin2Max);
                Float omc = 1 - cosMax, cosT = (cosMax - 1) * u0 + 1, sin2T = 1 - Sqr(cosT);
                if (sin2Max < 0.00068523f) {
                    sin2T = sin2Max * u0;
                    cosT = std::sqrt(1 - sin2T);
                    omc = sin2Max / 2;
                }
                const Float cosA = sin2T / sinMax + cosT * SafeSqrt(1 - sin2T / Sqr(sinMax)), sinA = SafeSqrt(1 - Sqr(cosA));
                const Float ph = u1 * 2 * Pi;
                const Float st = Clamp(sinA, -1, 1);
                const Vec w(st * CRCos(ph), st * CRSin(ph), Clamp(cosA, -1, 1));
                const Vec fz = Normalize(pc - cp);
                Vec fx, fy;
                CoordinateSystem(fz, &fx, &fy);
                Vec n = fx * (-w.x) + fy * (-w.y) + fz * (-w.z);
                const Vec p = pc + a * n;
                if (flags & 1) n = -n;
                Point3fi(p, gamma(5) * Abs(p), &out->p, &out->err);
                out->n = n;
                out->pdf = 1 / (2 * Pi * omc);
                SphereUV(XP(r2o, p), out->uv);  // (*objectFromRender)(p)
                return true;
            }
        }
        ShapeSample ss = SampleArea(u0, u1);
        Vec wi = ss.p - cp;
        if (LengthSquared(wi) == 0) return false;
        wi = Normalize(wi);
        ss.pdf /= AbsDotN(ss.n, -wi) / DistanceSquared(cp, ss.p);
        if (std::isinf(ss.pdf)) return false;
        *out = ss;
        return true;
    }
    // Shape::PDF(ctx, wi)
    Float PDF(Vec cp, Vec cpErr, Vec cn, Vec wi, Vec cns = Vec(0, 0, 0)) const {
        if (patch()) return PatchPDF(cp, cpErr, cn, cns, wi);
        if (sphere()) {
            const Vec pc = XP(o2r, Vec(0, 0, 0));
            const Vec po = OffsetRayOrigin(cp, cpErr, cn, pc - cp);
            if (DistanceSquared(po, pc) > Sqr(a)) {
                const Float sin2Max = a * a / DistanceSquared(cp, pc), cosMax = SafeSqrt(1 - sin2Max);
                Float omc = 1 - cosMax;
                if (sin2Max < 0.00068523f) omc = sin2Max / 2;
                return 1 / (2 * Pi * omc);
            }
        }
        const Vec ro = OffsetRayOrigin(cp, cpErr, cn, wi);
        Float th;
        Vec pObj;
        if (!Intersect(ro, wi, Infinity, &th, &pObj)) return 0;
        const Interaction si = Surface(pObj, wi);
        Float pdf = (1 / Area()) / (AbsDotN(si.n, -wi) / DistanceSquared(cp, si.p));
        if (std::isinf(pdf)) pdf = 0;
        return pdf;
    }
    void Bounds(Vec *mn, Vec *mx) const {
        if (patch()) {
            *mn = Vec(std::min(std::min(P[0].x, P[2].x), std::min(P[1].x, P[3].x)), std::min(std::min(P[0].y, P[2].y), std::min(P[1].y, P[3].y)),
                      std::min(std::min(P[0].z, P[2].z), std::min(P[1].z, P[3].z)));
            *mx = Vec(std::max(std::max(P[0].x, P[2].x), std::max(P[1].x, P[3].x)), std::max(std::max(P[0].y, P[2].y), std::max(P[1].y, P[3].y)),
                      std::max(std::max(P[0].z, P[2].z), std::max(P[1].z, P[3].z)));
            return;
        }
        const bool rz = sphere() || cylinder();  // (-r, -r, zMin), (r, r, zMax)
        const Vec lo = rz ? Vec(-a, -a, b) : Vec(-b, -b, a), hi = rz ? Vec(a, a, c) : Vec(b, b, a);
        *mn = Vec(Infinity, Infinity, Infinity);
        *mx = -*mn;
        for (int i = 0; i < 8; ++i) {
            const Vec q = XP(o2r, Vec((i & 1) ? hi.x : lo.x, (i & 2) ? hi.y : lo.y, (i & 4) ? hi.z : lo.z));
            for (int k = 0; k < 3; ++k) {
                (*mn)[k] = std::min((*mn)[k], q[k]);
                (*mx)[k] = std::max((*mx)[k], q[k]);
            }
        }
    }
};

void Scene::InitShapes() {
    shapes.assign(f->n_shapes, OShape());
    for (int k = 0; k < f->n_shapes; ++k) shapes[k].Init(f, k);
}
int Scene::IntersectShapes(Vec o, Vec d, Float tMax, TriIsect *hit, bool anyHit, int best) const {
    for (size_t k = 0; k < shapes.size(); ++k) {
        Float th;
        Vec pObj;
        if (shapes[k].Intersect(o, d, tMax, &th, &pObj)) {
            const int prim = f->n_triangles + (int)k;
            if (Alpha(prim) && AlphaKilled(prim, TriIsect{pObj.x, pObj.y, pObj.z, th}, o, d)) continue;
            tMax = th;
            *hit = TriIsect{pObj.x, pObj.y, pObj.z, th};
            best = f->n_triangles + (int)k;
            if (anyHit) return best;
        }
    }
    return best;
}
int Scene::Material(int prim) const {
    return prim < f->n_triangles ? f->tri_material[prim] : f->shape_info[8 * (prim - f->n_triangles) + 2];
}
int Scene::Light(int prim) const {
    return prim < f->n_triangles ? f->tri_light[prim] : f->shape_info[8 * (prim - f->n_triangles) + 3];
}
bool Scene::Medium(int prim, int *in, int *out) const {
    if (prim >= f->n_triangles) {
        const int32_t *info = f->shape_info + 8 * (prim - f->n_triangles);
        *in = info[4];
        *out = info[5];
        return true;
    }
    if (!f->tri_medium) return false;
    *in = f->tri_medium[2 * prim];
    *out = f->tri_medium[2 * prim + 1];
    return true;
}
Interaction Scene::Interact(int prim, const TriIsect &ti, Vec rd) const {
    if (prim >= f->n_triangles) {
        Interaction si = shapes[prim - f->n_triangles].Surface(Vec(ti.b0, ti.b1, ti.b2), rd);
        si.prim = prim;
        return si;
    }
    return TriangleInteraction(P(prim, 0), P(prim, 1), P(prim, 2), f->tri_flip[prim], ti, rd, Attr(prim));
}

struct LightNode {
    Vec mn, mx, w;
    Float phi, cosO, cosE;
    int twoSided, childOrLight, isLeaf;
};
static Float CosSub(Float sa, Float ca, Float sb, Float cb) { return ca > cb ? 1 : ca * cb + sa * sb; }
static Float SinSub(Float sa, Float ca, Float sb, Float cb) { return ca > cb ? 0 : sa * cb - ca * sb; }
static Float Importance(const LightNode &b, Vec p, Vec n) {
    Vec pc = (b.mn + b.mx) / 2;
    Float d2 = DistanceSquared(p, pc);
    d2 = std::max(d2, Length(b.mx - b.mn) / 2);
    Vec wi = Normalize(p - pc);
    Float cosW = Dot(b.w, wi);
    if (b.twoSided) cosW = std::abs(cosW);
    Float sinW = SafeSqrt(1 - Sqr(cosW));
    // BoundSubtendedDirections
    Float cosB;
    {
        Vec c = (b.mn + b.mx) / 2;
        bool inside = c.x >= b.mn.x && c.x <= b.mx.x && c.y >= b.mn.y && c.y <= b.mx.y && c.z >= b.mn.z && c.z <= b.mx.z;
        Float radius = inside ? Length(c - b.mx) : 0;
        if (DistanceSquared(p, c) < Sqr(radius)) cosB = -1;
        else cosB = SafeSqrt(1 - Sqr(radius) / DistanceSquared(c, p));
    }
    Float sinB = SafeSqrt(1 - Sqr(cosB));
    Float sinO = SafeSqrt(1 - Sqr(b.cosO));
    Float cosX = CosSub(sinW, cosW, sinO, b.cosO), sinX = SinSub(sinW, cosW, sinO, b.cosO);
    Float cosThetap = CosSub(sinX, cosX, sinB, cosB);
    if (cosThetap <= b.cosE) return 0;
    Float imp = b.phi * cosThetap / d2;
    if (n != Vec(0, 0, 0)) {
        Float cosI = AbsDotN(n, wi), sinI = SafeSqrt(1 - Sqr(cosI));
        imp *= CosSub(sinI, cosI, sinB, cosB);
    }
    return std::max<Float>(imp, 0);
}

// ---------------------------------------------------------------- light BVH construction
// The oracle builds its own BVHLightSampler tree from the flat light list (it does not read the
// product's): LightBounds of each light (DiffuseAreaLight::Bounds lights.cpp:803-822 with
// Triangle::NormalBounds shapes.cpp:303-318; PointLight / SpotLight::Bounds lights.cpp:168-173,
// 1401-1411), their union (lights.h:137-150 over DirectionCone Union, util/vecmath.cpp:57-84,
// and Rotate, util/transform.h:220-247), the modified-SAH split (lightsamplers.cpp:135-238,
// EvaluateCost lightsamplers.h:383-396) and the CompactLightBounds quantisation with its
// decode (lightsamplers.h:95-180, OctahedralVector util/vecmath.h:1735-1785).
namespace lbvh {
struct Box {
    Vec mn{std::numeric_limits<Float>::max(), std::numeric_limits<Float>::max(), std::numeric_limits<Float>::max()};
    Vec mx{std::numeric_limits<Float>::lowest(), std::numeric_limits<Float>::lowest(), std::numeric_limits<Float>::lowest()};
    Box() = default;
    Box(Vec a, Vec b) {
        mn = Vec(std::min(a.x, b.x), std::min(a.y, b.y), std::min(a.z, b.z));
        mx = Vec(std::max(a.x, b.x), std::max(a.y, b.y), std::max(a.z, b.z));
    }
    Box Union(const Box &o) const {
        Box r;
        r.mn = Vec(std::min(mn.x, o.mn.x), std::min(mn.y, o.mn.y), std::min(mn.z, o.mn.z));
        r.mx = Vec(std::max(mx.x, o.mx.x), std::max(mx.y, o.mx.y), std::max(mx.z, o.mx.z));
        return r;
    }
    Box Union(Vec p) const { return Union(Box(p, p)); }
    Vec Diagonal() const { return mx - mn; }
    Float SurfaceArea() const {
        Vec d = Diagonal();
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
    Vec Offset(Vec p) const {
        Vec o = p - mn;
        for (int a = 0; a < 3; ++a)
            if (mx[a] > mn[a]) o[a] /= mx[a] - mn[a];
        return o;
    }
};
struct LB {  // LightBounds
    Box b;
    Vec w;
    Float phi = 0, cosO = 0, cosE = 0;
    bool two = false;
    LB() = default;
    LB(Box bb, Vec ww, Float p, Float co, Float ce, bool t) : b(bb), w(Normalize(ww)), phi(p), cosO(co), cosE(ce), two(t) {}
    Vec Centroid() const { return (b.mn + b.mx) / 2; }
};
struct Cone {
    Vec w;
    Float cosT = Infinity;
    Cone() = default;
    Cone(Vec ww, Float c) : w(Normalize(ww)), cosT(c) {}
    bool Empty() const { return cosT == Infinity; }
};
static Vec Rotated(Float thetaDeg, Vec axis, Vec v) {
    const Float rad = (Pi / 180) * thetaDeg;
    const Float st = std::sin(rad), ct = std::cos(rad);
    const Vec a = Normalize(axis);
    Float m[3][3];
    m[0][0] = a.x * a.x + (1 - a.x * a.x) * ct;
    m[0][1] = a.x * a.y * (1 - ct) - a.z * st;
    m[0][2] = a.x * a.z * (1 - ct) + a.y * st;
    m[1][0] = a.x * a.y * (1 - ct) + a.z * st;
    m[1][1] = a.y * a.y + (1 - a.y * a.y) * ct;
    m[1][2] = a.y * a.z * (1 - ct) - a.x * st;
    m[2][0] = a.x * a.z * (1 - ct) - a.y * st;
    m[2][1] = a.y * a.z * (1 - ct) + a.x * st;
    m[2][2] = a.z * a.z + (1 - a.z * a.z) * ct;
    return Vec(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z, m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
               m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z);
}
static Cone UnionCone(const Cone &a, const Cone &b) {
    if (a.Empty()) return b;
    if (b.Empty()) return a;
    const Float ta = SafeACos(a.cosT), tb = SafeACos(b.cosT), td = AngleBetween(a.w, b.w);
    if (std::min(td + tb, Pi) <= ta) return a;
    if (std::min(td + ta, Pi) <= tb) return b;
    const Float to = (ta + td + tb) / 2;
    if (to >= Pi) return Cone(Vec(0, 0, 1), -1);
    const Float tr = to - ta;
    const Vec wr = Cross(a.w, b.w);
    if (LengthSquared(wr) == 0) return Cone(Vec(0, 0, 1), -1);
    return Cone(Rotated((180 / Pi) * tr, wr, a.w), std::cos(to));
}
static LB Union(const LB &a, const LB &b) {
    if (a.phi == 0) return b;
    if (b.phi == 0) return a;
    const Cone c = UnionCone(Cone(a.w, a.cosO), Cone(b.w, b.cosO));
    return LB(a.b.Union(b.b), c.w, a.phi + b.phi, c.cosT, std::min(a.cosE, b.cosE), a.two || b.two);
}
static Float Cost(const LB &b, const Box &bounds, int dim) {
    const Float thO = std::acos(b.cosO), thE = std::acos(b.cosE);
    const Float thW = std::min(thO + thE, Pi);
    const Float sinO = SafeSqrt(1 - Sqr(b.cosO));
    const Float Mw = 2 * Pi * (1 - b.cosO) + Pi / 2 * (2 * thW * sinO - std::cos(thO - 2 * thW) - 2 * thO * sinO + b.cosO);
    const Vec d = bounds.Diagonal();
    const Float Kr = MaxComp(d) / d[dim];
    return b.phi * Mw * Kr * b.b.SurfaceArea();
}
// CompactLightBounds(lb, allb) and its decode
static LightNode Compact(const LB &lb, const Box &all) {
    LightNode n{};
    Vec v = Normalize(lb.w);
    v = v / (std::abs(v.x) + std::abs(v.y) + std::abs(v.z));
    auto enc = [](Float f) { return (uint16_t)std::round(std::min<Float>(std::max<Float>((f + 1) / 2, 0), 1) * 65535.f); };
    auto sgn = [](Float x) { return std::copysign(Float(1), x); };
    uint16_t ox, oy;
    if (v.z >= 0) ox = enc(v.x), oy = enc(v.y);
    else ox = enc((1 - std::abs(v.y)) * sgn(v.x)), oy = enc((1 - std::abs(v.x)) * sgn(v.y));
    Vec d(-1 + 2 * (ox / 65535.f), -1 + 2 * (oy / 65535.f), 0);
    d.z = 1 - (std::abs(d.x) + std::abs(d.y));
    if (d.z < 0) {
        const Float xo = d.x;
        d.x = (1 - std::abs(d.y)) * sgn(xo);
        d.y = (1 - std::abs(xo)) * sgn(d.y);
    }
    n.w = Normalize(d);
    n.phi = lb.phi;
    const unsigned qo = (unsigned)std::floor(32767.f * ((lb.cosO + 1) / 2)), qe = (unsigned)std::floor(32767.f * ((lb.cosE + 1) / 2));
    n.cosO = 2 * (qo / 32767.f) - 1;
    n.cosE = 2 * (qe / 32767.f) - 1;
    n.twoSided = lb.two;
    for (int c = 0; c < 3; ++c) {
        auto q = [&](Float x) { return all.mn[c] == all.mx[c] ? 0.f : 65535.f * Clamp((x - all.mn[c]) / (all.mx[c] - all.mn[c]), 0, 1); };
        const uint16_t q0 = (uint16_t)std::floor(q(lb.b.mn[c])), q1 = (uint16_t)std::ceil(q(lb.b.mx[c]));
        auto lerp = [&](Float t) { return (1 - t) * all.mn[c] + t * all.mx[c]; };
        n.mn[c] = lerp(q0 / 65535.f);
        n.mx[c] = lerp(q1 / 65535.f);
    }
    return n;
}
struct Builder {
    std::vector<LightNode> nodes;
    std::vector<uint32_t> trail;
    Box all;
    std::pair<int, LB> Build(std::vector<std::pair<int, LB>> &L, int start, int end, uint32_t bits, int depth) {
        if (end - start == 1) {
            const int idx = (int)nodes.size();
            LightNode n = Compact(L[start].second, all);
            n.childOrLight = L[start].first;
            n.isLeaf = 1;
            nodes.push_back(n);
            trail[L[start].first] = bits;
            return {idx, L[start].second};
        }
        Box bounds, cb;
        for (int i = start; i < end; ++i) {
            bounds = bounds.Union(L[i].second.b);
            cb = cb.Union(L[i].second.Centroid());
        }
        Float minCost = Infinity;
        int bestB = -1, bestDim = -1;
        constexpr int nb = 12;
        auto bucket = [&](const LB &lb, int dim) {
            int b = nb * cb.Offset(lb.Centroid())[dim];
            return b == nb ? nb - 1 : b;
        };
        for (int dim = 0; dim < 3; ++dim) {
            if (cb.mx[dim] == cb.mn[dim]) continue;
            LB bl[nb];
            for (int i = start; i < end; ++i) {
                const int b = bucket(L[i].second, dim);
                bl[b] = Union(bl[b], L[i].second);
            }
            Float cost[nb - 1];
            for (int i = 0; i < nb - 1; ++i) {
                LB b0, b1;
                for (int j = 0; j <= i; ++j) b0 = Union(b0, bl[j]);
                for (int j = i + 1; j < nb; ++j) b1 = Union(b1, bl[j]);
                cost[i] = Cost(b0, bounds, dim) + Cost(b1, bounds, dim);
            }
            for (int i = 1; i < nb - 1; ++i)
                if (cost[i] > 0 && cost[i] < minCost) minCost = cost[i], bestB = i, bestDim = dim;
        }
        int mid;
        if (bestDim == -1) mid = (start + end) / 2;
        else {
            auto it = std::partition(L.begin() + start, L.begin() + end,
                                     [&](const std::pair<int, LB> &l) { return bucket(l.second, bestDim) <= bestB; });
            mid = (int)(it - L.begin());
            if (mid == start || mid == end) mid = (start + end) / 2;
        }
        const int idx = (int)nodes.size();
        nodes.push_back(LightNode{});
        auto c0 = Build(L, start, mid, bits, depth + 1);
        auto c1 = Build(L, mid, end, bits | (1u << depth), depth + 1);
        const LB lb = Union(c0.second, c1.second);
        LightNode n = Compact(lb, all);
        n.childOrLight = c1.first;
        n.isLeaf = 0;
        nodes[idx] = n;
        return {idx, lb};
    }
    void Run(std::vector<std::pair<int, LB>> L, int nLights) {
        nodes.clear();
        trail.assign(nLights, 0xffffffffu);
        all = Box();
        std::vector<std::pair<int, LB>> in;
        for (auto &l : L)
            if (l.second.phi > 0) {  // lightsamplers.cpp:121-124
                in.push_back(l);
                all = all.Union(l.second.b);
            }
        if (!in.empty()) Build(in, 0, (int)in.size(), 0, 0);
    }
};
// LightBounds of the scene's bounded lights (area lights, then point / spot lights)
static std::vector<std::pair<int, LB>> SceneLightBounds(const pbrt_scene_flat *f) {
    std::vector<std::pair<int, LB>> L;
    auto denseMax = [&](int sp) {
        const float *d = f->dense_spectra + 311 * sp;
        return *std::max_element(d, d + 311);
    };
    for (int i = 0; i < f->n_area_lights; ++i) {
        const int t = f->light_prim[i];
        if (t >= f->n_triangles) {
            // a sphere or disk emitter: Shape::Bounds and NormalBounds (shapes.h:134, shapes.cpp:94-99)
            OShape sh;
            sh.Init(f, t - f->n_triangles);
            Vec mn, mx;
            sh.Bounds(&mn, &mx);
            Float phi = denseMax(f->light_spectrum[i]);
            phi *= f->light_scale[i] * sh.Area() * Pi;
            Cone nb(Vec(0, 0, 1), -1);  // DirectionCone::EntireSphere
            if (sh.patch()) {
                // BilinearPatch::NormalBounds (shapes.cpp:1083-1129)
                const Vec p00 = sh.P[0], p10 = sh.P[1], p01 = sh.P[2], p11 = sh.P[3];
                const bool hasN = (sh.flags & 8) != 0, flip = sh.flip();
                auto ff = [](Vec v, Vec n) { return DotN(v, n) < 0 ? -v : v; };
                if (p00 == p10 || p10 == p11 || p11 == p01 || p01 == p00) {
                    Vec du = OLerp(0.5f, p10, p11) - OLerp(0.5f, p00, p01), dv = OLerp(0.5f, p01, p11) - OLerp(0.5f, p00, p10);
                    Vec n = Normalize(Cross(du, dv));
                    if (hasN) n = ff(n, (sh.Nv[0] + sh.Nv[1] + sh.Nv[2] + sh.Nv[3]) / 4);
                    else if (flip) n = -n;
                    nb = Cone(n, 1);
                } else {
                    Vec n00 = Normalize(Cross(p10 - p00, p01 - p00)), n10 = Normalize(Cross(p11 - p10, p00 - p10));
                    Vec n01 = Normalize(Cross(p00 - p01, p11 - p01)), n11 = Normalize(Cross(p01 - p11, p10 - p11));
                    if (hasN) {
                        n00 = ff(n00, sh.Nv[0]), n10 = ff(n10, sh.Nv[1]), n01 = ff(n01, sh.Nv[2]), n11 = ff(n11, sh.Nv[3]);
                    } else if (flip) {
                        n00 = -n00, n10 = -n10, n01 = -n01, n11 = -n11;
                    }
                    Vec n = Normalize(n00 + n10 + n01 + n11);
                    Float ct = std::min(std::min(Dot(n, n00), Dot(n, n01)), std::min(Dot(n, n10), Dot(n, n11)));
                    nb = Cone(n, Clamp(ct, -1, 1));
                }
            } else if (!sh.sphere() && !sh.cylinder()) {
                Vec n = OShape::XN(sh.r2o, Vec(0, 0, 1));
                if (sh.flags & 1) n = -n;
                nb = Cone(n, 1);
            }
            L.push_back({i, LB(Box(mn, mx), nb.w, phi, nb.cosT, std::cos(Pi / 2), f->light_two_sided[i] != 0)});
            continue;
        }
        const int32_t *v = f->triangles + 3 * t;
        auto P = [&](int k) { return Vec(f->vertices[3 * v[k]], f->vertices[3 * v[k] + 1], f->vertices[3 * v[k] + 2]); };
        const Vec p0 = P(0), p1 = P(1), p2 = P(2);
        Float phi = denseMax(f->light_spectrum[i]);
        if (f->light_image && f->light_image[i] >= 0) {
            // DiffuseAreaLight::Bounds with an image (lights.cpp:806-813): the mean channel value
            const float *img = f->area_images + f->light_image[i];
            const int w = (int)img[0], h = (int)img[1];
            Float sum = 0;
            for (int k = 0; k < 3 * w * h; ++k) sum += img[2 + k];
            phi = sum / (3 * w * h);
        }
        phi *= f->light_scale[i] * TriArea(p0, p1, p2) * Pi;
        Vec n = Normalize(Cross(p1 - p0, p2 - p0));
        if (f->tri_shading && (f->tri_shading[t] & 1)) {
            auto N = [&](int k) { return Vec(f->vertex_normals[3 * v[k]], f->vertex_normals[3 * v[k] + 1], f->vertex_normals[3 * v[k] + 2]); };
            const Vec ns = N(0) + N(1) + N(2);
            if (DotN(n, ns) < 0) n = -n;  // FaceForward(Normal3f, Normal3f): FMA-compensated dot
        } else if (f->tri_flip[t]) {
            n = -n;
        }
        const Cone nb(n, 1);  // DirectionCone(Vector3f(n))
        L.push_back({i, LB(Box(p0, p1).Union(p2), nb.w, phi, nb.cosT, std::cos(Pi / 2), f->light_two_sided[i] != 0)});
    }
    for (int k = 0; k < f->n_point_spot; ++k) {
        const float *d = f->delta_lights + 24 * k;
        const Vec p(d[5], d[6], d[7]);
        const Float mx = denseMax((int)d[1]), scale = d[2];
        if ((int)d[0] >= 3) {  // goniometric / projection: the loader's LightBounds terms
            L.push_back({f->n_area_lights + k, LB(Box(p, p), Vec(d[8], d[9], d[10]), d[20], d[3], d[4], false)});
        } else if ((int)d[0] == 0) {
            L.push_back({f->n_area_lights + k, LB(Box(p, p), Vec(0, 0, 1), 4 * Pi * scale * mx, std::cos(Pi), std::cos(Pi / 2), false)});
        } else {
            const Float cosStart = d[3], cosEnd = d[4];
            Float cosE = std::cos(std::acos(cosEnd) - std::acos(cosStart));
            if (cosE == 1 && cosEnd != cosStart) cosE = 0.999f;
            L.push_back({f->n_area_lights + k, LB(Box(p, p), Vec(d[8], d[9], d[10]), scale * mx * 4 * Pi, cosStart, cosE, false)});
        }
    }
    return L;
}
}  // namespace lbvh

struct Lights {
    const pbrt_scene_flat *f;
    std::vector<LightNode> nodes;
    std::vector<uint32_t> bitTrail;  // per bounded light (area, then point / spot)
    void Init(const pbrt_scene_flat *flat) {
        f = flat;
        lbvh::Builder b;
        b.Run(lbvh::SceneLightBounds(f), f->n_area_lights + f->n_point_spot);
        nodes = b.nodes;
        bitTrail = b.trail;
    }
    // global light index: area lights, point / spot lights, then the infinite-light list
    int NumAll() const { return f->n_area_lights + f->n_point_spot + f->n_infinite_lights; }
    bool uniform() const {
        return f->n_light_nodes == 0 && f->n_infinite_lights + f->n_area_lights > 0 && uniformFlag;
    }
    bool uniformFlag = false;
    // returns light index (area first, then infinite) and pmf
    bool Sample(Vec p, Vec n, Float u, int *light, Float *pmf) const {
        if (uniformFlag) {
            int nAll = NumAll();
            if (!nAll) return false;
            *light = f->uniform_order[std::min<int>(u * nAll, nAll - 1)];  // pbrt's light order
            *pmf = 1.f / nAll;
            return true;
        }
        Float pInf = Float(f->n_infinite_lights) / Float(f->n_infinite_lights + (nodes.empty() ? 0 : 1));
        if (u < pInf) {
            u /= pInf;
            int index = std::min<int>(u * f->n_infinite_lights, f->n_infinite_lights - 1);
            *pmf = pInf / f->n_infinite_lights;
            *light = f->n_area_lights + f->n_point_spot + index;
            return true;
        }
        if (nodes.empty()) return false;
        u = std::min<Float>((u - pInf) / (1 - pInf), OneMinusEpsilon);
        int ni = 0;
        Float pm = 1 - pInf;
        while (true) {
            const LightNode &node = nodes[ni];
            if (!node.isLeaf) {
                Float ci[2] = {Importance(nodes[ni + 1], p, n), Importance(nodes[node.childOrLight], p, n)};
                if (ci[0] == 0 && ci[1] == 0) return false;
                // SampleDiscrete over two weights
                Float sum = 0;
                sum += ci[0];
                sum += ci[1];
                Float up = u * sum;
                if (up == sum) up = NextFloatDown(up);
                int off = 0;
                Float acc = 0;
                while (acc + ci[off] <= up) acc += ci[off++];
                pm *= ci[off] / sum;
                u = std::min((up - acc) / ci[off], OneMinusEpsilon);
                ni = off == 0 ? ni + 1 : node.childOrLight;
            } else {
                if (ni > 0 || Importance(node, p, n) > 0) {
                    *light = node.childOrLight;
                    *pmf = pm;
                    return true;
                }
                return false;
            }
        }
    }
    Float PMF(Vec p, Vec n, int light) const {
        if (uniformFlag) return NumAll() ? 1.f / NumAll() : 0.f;
        uint32_t trail = light < f->n_area_lights + f->n_point_spot ? bitTrail[light] : 0xffffffffu;
        bool inBVH = false;
        for (auto &nd : nodes)
            if (nd.isLeaf && nd.childOrLight == light) inBVH = true;
        if (!inBVH) return 1.f / (f->n_infinite_lights + (nodes.empty() ? 0 : 1));
        Float pInf = Float(f->n_infinite_lights) / Float(f->n_infinite_lights + (nodes.empty() ? 0 : 1));
        Float pm = 1 - pInf;
        int ni = 0;
        while (true) {
            const LightNode &node = nodes[ni];
            if (node.isLeaf) return pm;
            Float ci[2] = {Importance(nodes[ni + 1], p, n), Importance(nodes[node.childOrLight], p, n)};
            pm *= ci[trail & 1] / (ci[0] + ci[1]);
            ni = (trail & 1) ? node.childOrLight : ni + 1;
            trail >>= 1;
        }
    }
};

// ---------------------------------------------------------------- BxDFs
// DiffuseBxDF (bxdfs.h:30-82), DielectricBxDF (bxdfs.h:300-341, bxdfs.cpp:77-245),
// ConductorBxDF (bxdfs.h:413-517) with TrowbridgeReitzDistribution and the Fresnel terms of
// util/scattering.h:18-205 and pstd::complex (util/pstd.h:1066-1229).  The path integrator calls
// them with TransportMode::Radiance and BxDFReflTransFlags::All; the layered BxDFs below also
// use Importance mode (no 1/eta^2 on transmission) and single-lobe flags (sf: 1 R, 2 T).
enum { BxR = 1, BxT = 2, BxDiffuse = 4, BxGlossy = 8, BxSpecular = 16 };

struct BSDFSample {
    Spectrum f;
    Vec wi;
    Float pdf = 0;
    int flags = 0;
    Float eta = 1;
};

static inline Float Tan2Theta(Vec w) {
    Float sin2 = std::max<Float>(0, 1 - Sqr(w.z));
    return sin2 / Sqr(w.z);
}
static inline Float CosPhi(Vec w) {
    Float st = std::sqrt(std::max<Float>(0, 1 - Sqr(w.z)));
    return st == 0 ? 1 : Clamp(w.x / st, -1, 1);
}
static inline Float SinPhi(Vec w) {
    Float st = std::sqrt(std::max<Float>(0, 1 - Sqr(w.z)));
    return st == 0 ? 0 : Clamp(w.y / st, -1, 1);
}
static inline bool SameHemisphere(Vec a, Vec b) { return a.z * b.z > 0; }

struct TRDistribution {
    Float ax = 0, ay = 0;
    TRDistribution() = default;
    TRDistribution(Float x, Float y) : ax(x), ay(y) {
        if (!Smooth()) {
            ax = std::max<Float>(ax, 1e-4f);
            ay = std::max<Float>(ay, 1e-4f);
        }
    }
    bool Smooth() const { return std::max(ax, ay) < 1e-3f; }
    Float D(Vec wm) const {
        Float t2 = Tan2Theta(wm);
        if (std::isinf(t2)) return 0;
        Float c4 = Sqr(Sqr(wm.z));
        if (c4 < 1e-16f) return 0;
        Float e = t2 * (Sqr(CosPhi(wm) / ax) + Sqr(SinPhi(wm) / ay));
        return 1 / (Pi * ax * ay * c4 * Sqr(1 + e));
    }
    Float Lambda(Vec w) const {
        Float t2 = Tan2Theta(w);
        if (std::isinf(t2)) return 0;
        Float a2 = Sqr(CosPhi(w) * ax) + Sqr(SinPhi(w) * ay);
        return (std::sqrt(1 + a2 * t2) - 1) / 2;
    }
    Float G1(Vec w) const { return 1 / (1 + Lambda(w)); }
    Float G(Vec wo, Vec wi) const { return 1 / (1 + Lambda(wo) + Lambda(wi)); }
    Float PDF(Vec w, Vec wm) const { return G1(w) / std::abs(w.z) * D(wm) * AbsDot(w, wm); }
    Vec Sample_wm(Vec w, Float u0, Float u1) const {
        Vec wh = Normalize(Vec(ax * w.x, ay * w.y, w.z));
        if (wh.z < 0) wh = -wh;
        Vec T1 = (wh.z < 0.99999f) ? Normalize(Cross(Vec(0, 0, 1), wh)) : Vec(1, 0, 0);
        Vec T2 = Cross(wh, T1);
        Float r = std::sqrt(u0), th = 2 * Pi * u1;  // SampleUniformDiskPolar
        Float px = r * CRCos(th), py = r * CRSin(th);
        Float h = std::sqrt(1 - Sqr(px));
        py = Lerp((1 + wh.z) / 2, h, py);
        Float pz = std::sqrt(std::max<Float>(0, 1 - (Sqr(px) + Sqr(py))));
        Vec nh = px * T1 + py * T2 + pz * wh;
        return Normalize(Vec(ax * nh.x, ay * nh.y, std::max<Float>(1e-6f, nh.z)));
    }
    void Regularize() {
        if (ax < 0.3f) ax = Clamp(2 * ax, 0.1f, 0.3f);
        if (ay < 0.3f) ay = Clamp(2 * ay, 0.1f, 0.3f);
    }
};

static Float FrDielectric(Float cosI, Float eta) {
    cosI = Clamp(cosI, -1, 1);
    if (cosI < 0) {
        eta = 1 / eta;
        cosI = -cosI;
    }
    Float sin2T = (1 - Sqr(cosI)) / Sqr(eta);
    if (sin2T >= 1) return 1.f;
    Float cosT = SafeSqrt(1 - sin2T);
    Float rParl = (eta * cosI - cosT) / (eta * cosI + cosT);
    Float rPerp = (cosI - eta * cosT) / (cosI + eta * cosT);
    return (Sqr(rParl) + Sqr(rPerp)) / 2;
}

struct Complex {
    Float re, im;
    Complex(Float r, Float i = 0) : re(r), im(i) {}
    Complex operator+(Complex z) const { return {re + z.re, im + z.im}; }
    Complex operator-(Complex z) const { return {re - z.re, im - z.im}; }
    Complex operator*(Complex z) const { return {re * z.re - im * z.im, re * z.im + im * z.re}; }
    Complex operator/(Complex z) const {
        Float scale = 1 / (z.re * z.re + z.im * z.im);
        return {scale * (re * z.re + im * z.im), scale * (im * z.re - re * z.im)};
    }
};
static inline Float Norm(Complex z) { return z.re * z.re + z.im * z.im; }
static Complex Sqrt(Complex z) {
    Float n = std::sqrt(Norm(z)), t1 = std::sqrt(Float(.5) * (n + std::abs(z.re))), t2 = Float(.5) * z.im / t1;
    if (n == 0) return 0;
    if (z.re >= 0) return {t1, t2};
    return {std::abs(t2), std::copysign(t1, z.im)};
}
static Float FrComplex(Float cosI, Complex eta) {
    cosI = Clamp(cosI, 0, 1);
    Float sin2I = 1 - Sqr(cosI);
    Complex sin2T = Complex(sin2I) / (eta * eta);
    Complex cosT = Sqrt(Complex(1) - sin2T);
    Complex rParl = (eta * Complex(cosI) - cosT) / (eta * Complex(cosI) + cosT);
    Complex rPerp = (Complex(cosI) - eta * cosT) / (Complex(cosI) + eta * cosT);
    return (Norm(rParl) + Norm(rPerp)) / 2;
}
static bool Refract(Vec wi, Vec n, Float eta, Float *etap, Vec *wt) {
    Float cosI = DotN(n, wi);
    if (cosI < 0) {
        eta = 1 / eta;
        cosI = -cosI;
        n = -n;
    }
    Float sin2T = std::max<Float>(0, 1 - Sqr(cosI)) / Sqr(eta);
    if (sin2T >= 1) return false;
    Float cosT = std::sqrt(1 - sin2T);
    *wt = -wi / eta + (cosI / eta - cosT) * n;
    *etap = eta;
    return true;
}
static inline Vec Reflect(Vec wo, Vec n) { return -wo + 2 * Dot(wo, n) * n; }

static Float FastExp(Float x);
// HairBxDF (bxdfs.h:1054-1152, bxdfs.cpp:279-573) with the math helpers it calls (util/math.h:
// 294-309 Pow, :490-502 Logistic, :794-816 I0 / LogI0; util/sampling.h:79-115 SampleDiscrete,
// :256-278 SampleTrimmedLogistic), pMax = 3, every SampledSpectrum operation per wavelength.
namespace ohair {
constexpr int pMax = 3;
template <int n> static inline Float Pow(Float v) {
    if constexpr (n == 0) return 1;
    else if constexpr (n == 1) return v;
    else {
        Float n2 = Pow<n / 2>(v);
        return n2 * n2 * Pow<n & 1>(v);
    }
}
static inline Float I0(Float x) {
    Float val = 0, x2i = 1;
    int64_t ifact = 1;
    int i4 = 1;
    for (int i = 0; i < 10; ++i) {
        if (i > 1) ifact *= i;
        val += x2i / (i4 * (ifact * ifact));
        x2i *= x * x;
        i4 *= 4;
    }
    return val;
}
static inline Float LogI0(Float x) {
    if (x > 12) return x + 0.5f * (-CRLog(2 * Pi) + CRLog(1 / x) + 1 / (8 * x));
    return CRLog(I0(x));
}
static inline Float Logistic(Float x, Float s) {
    x = std::abs(x);
    return CRExp(-x / s) / (s * Sqr(1 + CRExp(-x / s)));
}
static inline Float LogisticCDF(Float x, Float s) { return 1 / (1 + CRExp(-x / s)); }
static inline Float TrimmedLogistic(Float x, Float s, Float a, Float b) {
    return Logistic(x, s) / (LogisticCDF(b, s) - LogisticCDF(a, s));
}
static inline Float SampleTrimmedLogistic(Float u, Float s, Float a, Float b) {
    auto P = [&](Float x) { return 1 / (1 + CRExp(-x / s)); };  // InvertLogisticSample
    u = Lerp(u, P(a), P(b));
    Float x = -s * CRLog(1 / u - 1);  // SampleLogistic
    return Clamp(x, a, b);
}
static inline Float Mp(Float cosTheta_i, Float cosTheta_o, Float sinTheta_i, Float sinTheta_o, Float v) {
    Float a = cosTheta_i * cosTheta_o / v, b = sinTheta_i * sinTheta_o / v;
    Float mp = (v <= .1) ? (FastExp(LogI0(a) - b - 1 / v + 0.6931f + CRLog(1 / (2 * v))))
                         : (FastExp(-b) * I0(a)) / (CRSinh(1 / v) * 2 * v);
    return mp;
}
static inline Float Phi(int p, Float gamma_o, Float gamma_t) { return 2 * p * gamma_t - 2 * gamma_o + p * Pi; }
static inline Float Np(Float phi, int p, Float s, Float gamma_o, Float gamma_t) {
    Float dphi = phi - Phi(p, gamma_o, gamma_t);
    while (dphi > Pi) dphi -= 2 * Pi;
    while (dphi < -Pi) dphi += 2 * Pi;
    return TrimmedLogistic(dphi, s, -Pi, Pi);
}
struct Hair {
    Float h = 0, eta = 1.55f;
    Spectrum sigma_a;
    Float v[pMax + 1] = {}, s = 0;
    Float sin2kAlpha[pMax] = {}, cos2kAlpha[pMax] = {};

    void Init(Float h_, Float eta_, const Spectrum &sa, Float beta_m, Float beta_n, Float alpha) {
        h = h_;
        eta = eta_;
        sigma_a = sa;
        v[0] = Sqr(0.726f * beta_m + 0.812f * Sqr(beta_m) + 3.7f * Pow<20>(beta_m));
        v[1] = .25 * v[0];
        v[2] = 4 * v[0];
        for (int p = 3; p <= pMax; ++p) v[p] = v[2];
        static const Float SqrtPiOver8 = 0.626657069f;
        s = SqrtPiOver8 * (0.265f * beta_n + 1.194f * Sqr(beta_n) + 5.372f * Pow<22>(beta_n));
        sin2kAlpha[0] = CRSin((Pi / 180) * alpha);
        cos2kAlpha[0] = SafeSqrt(1 - Sqr(sin2kAlpha[0]));
        for (int i = 1; i < pMax; ++i) {
            sin2kAlpha[i] = 2 * cos2kAlpha[i - 1] * sin2kAlpha[i - 1];
            cos2kAlpha[i] = Sqr(cos2kAlpha[i - 1]) - Sqr(sin2kAlpha[i - 1]);
        }
    }
    // Ap (bxdfs.h:1102-1124); ap[pMax] stays zero when 1 - T f is zero at every wavelength
    void Ap(Float cosTheta_o, const Spectrum &T, Spectrum ap[pMax + 1]) const {
        Float cosGamma_o = SafeSqrt(1 - Sqr(h));
        Float cosTheta = cosTheta_o * cosGamma_o;
        Float f = FrDielectric(cosTheta, eta);
        for (int i = 0; i < NS; ++i) ap[0][i] = f;
        for (int i = 0; i < NS; ++i) ap[1][i] = Sqr(1 - f) * T[i];
        for (int p = 2; p < pMax; ++p)
            for (int i = 0; i < NS; ++i) ap[p][i] = ap[p - 1][i] * T[i] * f;
        bool any = false;
        for (int i = 0; i < NS; ++i) any = any || (1 - T[i] * f) != 0;
        for (int i = 0; i < NS; ++i) ap[pMax][i] = any ? ap[pMax - 1][i] * f * T[i] / (1 - T[i] * f) : 0.f;
    }
    void Tilt(int p, Float sinTheta_o, Float cosTheta_o, Float *sinThetap_o, Float *cosThetap_o) const {
        if (p == 0) {
            *sinThetap_o = sinTheta_o * cos2kAlpha[1] - cosTheta_o * sin2kAlpha[1];
            *cosThetap_o = cosTheta_o * cos2kAlpha[1] + sinTheta_o * sin2kAlpha[1];
        } else if (p == 1) {
            *sinThetap_o = sinTheta_o * cos2kAlpha[0] + cosTheta_o * sin2kAlpha[0];
            *cosThetap_o = cosTheta_o * cos2kAlpha[0] - sinTheta_o * sin2kAlpha[0];
        } else if (p == 2) {
            *sinThetap_o = sinTheta_o * cos2kAlpha[2] + cosTheta_o * sin2kAlpha[2];
            *cosThetap_o = cosTheta_o * cos2kAlpha[2] - sinTheta_o * sin2kAlpha[2];
        } else {
            *sinThetap_o = sinTheta_o;
            *cosThetap_o = cosTheta_o;
        }
        *cosThetap_o = std::abs(*cosThetap_o);
    }
    Spectrum f(Vec wo, Vec wi) const {
        Float sinTheta_o = wo.x;
        Float cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
        Float phi_o = CRATan2(wo.z, wo.y);
        Float gamma_o = SafeASin(h);
        Float sinTheta_i = wi.x;
        Float cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
        Float phi_i = CRATan2(wi.z, wi.y);
        Float sinTheta_t = sinTheta_o / eta;
        Float cosTheta_t = SafeSqrt(1 - Sqr(sinTheta_t));
        Float etap = SafeSqrt(Sqr(eta) - Sqr(sinTheta_o)) / cosTheta_o;
        Float sinGamma_t = h / etap;
        Float cosGamma_t = SafeSqrt(1 - Sqr(sinGamma_t));
        Float gamma_t = SafeASin(sinGamma_t);
        Spectrum T;
        for (int i = 0; i < NS; ++i) T[i] = CRExp(-sigma_a[i] * (2 * cosGamma_t / cosTheta_t));
        Float phi = phi_i - phi_o;
        Spectrum ap[pMax + 1];
        Ap(cosTheta_o, T, ap);
        Spectrum fsum(0.f);
        for (int p = 0; p < pMax; ++p) {
            Float sinThetap_o, cosThetap_o;
            Tilt(p, sinTheta_o, cosTheta_o, &sinThetap_o, &cosThetap_o);
            Float m = Mp(cosTheta_i, cosThetap_o, sinTheta_i, sinThetap_o, v[p]);
            Float n = Np(phi, p, s, gamma_o, gamma_t);
            for (int i = 0; i < NS; ++i) fsum[i] += m * ap[p][i] * n;
        }
        Float m3 = Mp(cosTheta_i, cosTheta_o, sinTheta_i, sinTheta_o, v[pMax]);
        for (int i = 0; i < NS; ++i) fsum[i] += m3 * ap[pMax][i] / (2 * Pi);
        if (std::abs(wi.z) > 0)
            for (int i = 0; i < NS; ++i) fsum[i] /= std::abs(wi.z);
        return fsum;
    }
    void ApPDF(Float cosTheta_o, Float apPDF[pMax + 1]) const {
        Float sinTheta_o = SafeSqrt(1 - Sqr(cosTheta_o));
        Float sinTheta_t = sinTheta_o / eta;
        Float cosTheta_t = SafeSqrt(1 - Sqr(sinTheta_t));
        Float etap = SafeSqrt(Sqr(eta) - Sqr(sinTheta_o)) / cosTheta_o;
        Float sinGamma_t = h / etap;
        Float cosGamma_t = SafeSqrt(1 - Sqr(sinGamma_t));
        Spectrum T;
        for (int i = 0; i < NS; ++i) T[i] = CRExp(-sigma_a[i] * (2 * cosGamma_t / cosTheta_t));
        Spectrum ap[pMax + 1];
        Ap(cosTheta_o, T, ap);
        Float sumY = 0;
        for (int p = 0; p <= pMax; ++p) sumY += ap[p].Average();
        for (int p = 0; p <= pMax; ++p) apPDF[p] = ap[p].Average() / sumY;
    }
    Float PdfSum(const Float apPDF[pMax + 1], Float sinTheta_o, Float cosTheta_o, Float sinTheta_i, Float cosTheta_i,
                 Float dphi, Float gamma_o, Float gamma_t) const {
        Float pdf = 0;
        for (int p = 0; p < pMax; ++p) {
            Float sinThetap_o, cosThetap_o;
            Tilt(p, sinTheta_o, cosTheta_o, &sinThetap_o, &cosThetap_o);
            pdf += Mp(cosTheta_i, cosThetap_o, sinTheta_i, sinThetap_o, v[p]) * apPDF[p] * Np(dphi, p, s, gamma_o, gamma_t);
        }
        pdf += Mp(cosTheta_i, cosTheta_o, sinTheta_i, sinTheta_o, v[pMax]) * apPDF[pMax] * (1 / (2 * Pi));
        return pdf;
    }
    bool Sample_f(Vec wo, Float uc, Float u0, Float u1, BSDFSample *bs) const {
        Float sinTheta_o = wo.x;
        Float cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
        Float phi_o = CRATan2(wo.z, wo.y);
        Float gamma_o = SafeASin(h);
        Float apPDF[pMax + 1];
        ApPDF(cosTheta_o, apPDF);
        // SampleDiscrete(apPDF, uc, nullptr, &uc)
        Float sumWeights = 0;
        for (int k = 0; k <= pMax; ++k) sumWeights += apPDF[k];
        Float up = uc * sumWeights;
        if (up == sumWeights) up = NextFloatDown(up);
        int p = 0;
        Float sum = 0;
        while (p < pMax && sum + apPDF[p] <= up) sum += apPDF[p++];
        uc = std::min((up - sum) / apPDF[p], OneMinusEpsilon);
        Float sinThetap_o, cosThetap_o;
        Tilt(p, sinTheta_o, cosTheta_o, &sinThetap_o, &cosThetap_o);
        Float cosTheta = 1 + v[p] * CRLog(std::max<Float>(u0, 1e-5) + (1 - u0) * FastExp(-2 / v[p]));
        Float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
        Float cosPhi = CRCos(2 * Pi * u1);
        Float sinTheta_i = -cosTheta * sinThetap_o + sinTheta * cosPhi * cosThetap_o;
        Float cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
        Float etap = SafeSqrt(Sqr(eta) - Sqr(sinTheta_o)) / cosTheta_o;
        Float sinGamma_t = h / etap;
        Float gamma_t = SafeASin(sinGamma_t);
        Float dphi;
        if (p < pMax) dphi = Phi(p, gamma_o, gamma_t) + SampleTrimmedLogistic(uc, s, -Pi, Pi);
        else dphi = 2 * Pi * uc;
        Float phi_i = phi_o + dphi;
        Vec wi(sinTheta_i, cosTheta_i * CRCos(phi_i), cosTheta_i * CRSin(phi_i));
        Float pdf = PdfSum(apPDF, sinTheta_o, cosTheta_o, sinTheta_i, cosTheta_i, dphi, gamma_o, gamma_t);
        *bs = BSDFSample{f(wo, wi), wi, pdf, BxR | BxGlossy, 1};
        return true;
    }
    Float PDF(Vec wo, Vec wi) const {
        Float sinTheta_o = wo.x;
        Float cosTheta_o = SafeSqrt(1 - Sqr(sinTheta_o));
        Float phi_o = CRATan2(wo.z, wo.y);
        Float gamma_o = SafeASin(h);
        Float sinTheta_i = wi.x;
        Float cosTheta_i = SafeSqrt(1 - Sqr(sinTheta_i));
        Float phi_i = CRATan2(wi.z, wi.y);
        Float etap = SafeSqrt(eta * eta - Sqr(sinTheta_o)) / cosTheta_o;
        Float sinGamma_t = h / etap;
        Float gamma_t = SafeASin(sinGamma_t);
        Float apPDF[pMax + 1];
        ApPDF(cosTheta_o, apPDF);
        return PdfSum(apPDF, sinTheta_o, cosTheta_o, sinTheta_i, cosTheta_i, phi_i - phi_o, gamma_o, gamma_t);
    }
};
}  // namespace ohair

// ---- MeasuredBxDF (bxdfs.h:1154-1204, bxdfs.cpp:690-1124) and PiecewiseLinear2D
// (util/sampling.h:1264-1749), restated over the oracle's own reader of the RGL tensor file
namespace omeas {
// one PiecewiseLinear2D<D>: resolution, parameter grids, per-slice tables
struct Table {
    int nx = 0, ny = 0, D = 0;
    std::vector<float> params[3];
    uint32_t strides[3] = {0, 0, 0};
    std::vector<float> data, marginal, conditional;

    void Build(const float *in, int xSize, int ySize, int dims, const std::vector<float> *pv, bool normalize,
               bool cdf) {
        nx = xSize, ny = ySize, D = dims;
        uint32_t slices = 1;
        for (int i = D - 1; i >= 0; --i) {
            params[i] = pv[i];
            strides[i] = pv[i].size() > 1 ? slices : 0;
            slices *= (uint32_t)pv[i].size();
        }
        const size_t n = (size_t)nx * ny;
        data.resize(slices * n);
        if (cdf) {
            marginal.resize((size_t)slices * ny);
            conditional.resize(slices * n);
        }
        for (uint32_t s = 0; s < slices; ++s) {
            const float *d = in + s * n;
            float *o = data.data() + s * n;
            if (cdf) {
                float *cc = conditional.data() + s * n, *mc = marginal.data() + (size_t)s * ny;
                for (int y = 0; y < ny; ++y) {
                    double acc = 0;
                    cc[(size_t)y * nx] = 0;
                    for (int x = 0; x + 1 < nx; ++x) {
                        const size_t i = (size_t)y * nx + x;
                        acc += .5 * ((double)d[i] + (double)d[i + 1]);
                        cc[i + 1] = (float)acc;
                    }
                }
                double acc = 0;
                mc[0] = 0;
                for (int y = 0; y + 1 < ny; ++y) {
                    acc += .5 * ((double)cc[(size_t)(y + 1) * nx - 1] + (double)cc[(size_t)(y + 2) * nx - 1]);
                    mc[y + 1] = (float)acc;
                }
                const float norm = 1.f / mc[ny - 1];
                for (size_t i = 0; i < n; ++i) cc[i] *= norm;
                for (int i = 0; i < ny; ++i) mc[i] *= norm;
                for (size_t i = 0; i < n; ++i) o[i] = d[i] * norm;
            } else {
                float norm = 1.f / ((float)(nx - 1) * (float)(ny - 1));
                if (normalize) {
                    double acc = 0;
                    for (int y = 0; y + 1 < ny; ++y)
                        for (int x = 0; x + 1 < nx; ++x) {
                            const size_t i = (size_t)y * nx + x;
                            acc += (double)(.25f * (d[i] + d[i + 1] + d[i + nx] + d[i + 1 + nx]));
                        }
                    norm = float(1.0 / acc);
                }
                for (size_t i = 0; i < n; ++i) o[i] = d[i] * norm;
            }
        }
    }
    // parameter weights (the loop heading Sample / Invert / Evaluate)
    uint32_t Weights(const Float *param, Float *w) const {
        uint32_t slice = 0;
        for (int k = 0; k < D; ++k) {
            const int np = (int)params[k].size();
            if (np == 1) {
                w[2 * k] = 1, w[2 * k + 1] = 0;
                continue;
            }
            // FindInterval(np, params[k][i] <= param[k])
            int lo = 0, hi = np - 2;
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (params[k][mid] <= param[k]) lo = mid;
                else hi = mid - 1;
            }
            const Float p0 = params[k][lo], p1 = params[k][lo + 1];
            w[2 * k + 1] = Clamp((param[k] - p0) / (p1 - p0), 0, 1);
            w[2 * k] = 1 - w[2 * k + 1];
            slice += strides[k] * (uint32_t)lo;
        }
        return slice;
    }
    // lookup<Dim>: nested blend, the last parameter outermost
    Float At(const float *t, uint32_t i, uint32_t size, const Float *w, int dim) const {
        if (dim == 0) return t[i];
        const Float v0 = At(t, i, size, w, dim - 1), v1 = At(t, i + strides[dim - 1] * size, size, w, dim - 1);
        return std::fma(v0, w[2 * dim - 2], v1 * w[2 * dim - 1]);
    }
    Float Evaluate(Float x, Float y, const Float *param) const {
        Float w[6];
        const uint32_t slice = Weights(param, w);
        x *= (Float)(nx - 1);
        y *= (Float)(ny - 1);
        const int ix = std::min((int)x, nx - 2), iy = std::min((int)y, ny - 2);
        const Float fx = x - (Float)ix, fy = y - (Float)iy, gx = 1 - fx, gy = 1 - fy;
        const uint32_t size = (uint32_t)(nx * ny), i = (uint32_t)(ix + iy * nx) + (D ? slice * size : 0);
        const float *t = data.data();
        const Float v00 = At(t, i, size, w, D), v10 = At(t + 1, i, size, w, D), v01 = At(t + nx, i, size, w, D),
                    v11 = At(t + nx + 1, i, size, w, D);
        return std::fma(gy, std::fma(gx, v00, fx * v10), fy * std::fma(gx, v01, fx * v11)) *
               ((Float)(nx - 1) * (Float)(ny - 1));
    }
    void Invert(Float x, Float y, const Float *param, Float *ox, Float *oy, Float *pdf) const {
        Float w[6];
        const uint32_t slice = Weights(param, w);
        x *= (Float)(nx - 1);
        y *= (Float)(ny - 1);
        const int ix = std::min((int)x, nx - 2), iy = std::min((int)y, ny - 2);
        x -= (Float)ix;
        y -= (Float)iy;
        const uint32_t size = (uint32_t)(nx * ny), base = D ? slice * size : 0;
        uint32_t i = (uint32_t)(ix + iy * nx) + base;
        const float *t = data.data(), *c = conditional.data();
        const Float v00 = At(t, i, size, w, D), v10 = At(t + 1, i, size, w, D), v01 = At(t + nx, i, size, w, D),
                    v11 = At(t + nx + 1, i, size, w, D);
        const Float c0 = std::fma(1 - y, v00, y * v01), c1 = std::fma(1 - y, v10, y * v11);
        *pdf = std::fma(1 - x, c0, x * c1) * ((Float)(nx - 1) * (Float)(ny - 1));
        x *= c0 + .5f * x * (c1 - c0);
        x += (1.f - y) * At(c, i, size, w, D) + y * At(c + nx, i, size, w, D);
        i = (uint32_t)(iy * nx) + base;
        const Float r0 = At(c, i + nx - 1, size, w, D), r1 = At(c, i + (2 * nx - 1), size, w, D);
        x /= (1.f - y) * r0 + y * r1;
        y *= r0 + .5f * y * (r1 - r0);
        y += At(marginal.data(), (uint32_t)iy + (D ? slice * (uint32_t)ny : 0), (uint32_t)ny, w, D);
        *ox = x, *oy = y;
    }
    void Sample(Float x, Float y, const Float *param, Float *ox, Float *oy, Float *pdf) const {
        x = Clamp(x, 1 - OneMinusEpsilon, OneMinusEpsilon);
        y = Clamp(y, 1 - OneMinusEpsilon, OneMinusEpsilon);
        Float w[6];
        const uint32_t slice = Weights(param, w);
        const float *c = conditional.data(), *t = data.data();
        const uint32_t mbase = D ? slice * (uint32_t)ny : 0;
        // FindInterval over the marginal: last row whose CDF is below y
        int lo = 0, hi = ny - 2;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (At(marginal.data(), mbase + mid, (uint32_t)ny, w, D) < y) lo = mid;
            else hi = mid - 1;
        }
        const int row = lo;
        y -= At(marginal.data(), mbase + row, (uint32_t)ny, w, D);
        const uint32_t size = (uint32_t)(nx * ny);
        uint32_t off = (uint32_t)(row * nx) + (D ? slice * size : 0);
        const Float r0 = At(c, off + nx - 1, size, w, D), r1 = At(c, off + (2 * nx - 1), size, w, D);
        bool flat = std::abs(r0 - r1) < 1e-4f * (r0 + r1);
        y = flat ? (2.f * y) : (r0 - std::sqrt(std::max<Float>(0, r0 * r0 - 2.f * y * (r0 - r1))));
        y /= flat ? (r0 + r1) : (r0 - r1);
        x *= (1.f - y) * r0 + y * r1;
        auto cond = [&](int k) { return (1.f - y) * At(c, off + k, size, w, D) + y * At(c + nx, off + k, size, w, D); };
        lo = 0, hi = nx - 2;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (cond(mid) < x) lo = mid;
            else hi = mid - 1;
        }
        const int col = lo;
        x -= cond(col);
        off += (uint32_t)col;
        const Float v00 = At(t, off, size, w, D), v10 = At(t + 1, off, size, w, D), v01 = At(t + nx, off, size, w, D),
                    v11 = At(t + nx + 1, off, size, w, D);
        const Float c0 = std::fma(1.f - y, v00, y * v01), c1 = std::fma(1.f - y, v10, y * v11);
        flat = std::abs(c0 - c1) < 1e-4f * (c0 + c1);
        x = flat ? (2.f * x) : (c0 - std::sqrt(std::max<Float>(0, c0 * c0 - 2.f * x * (c0 - c1))));
        x /= flat ? (c0 + c1) : (c0 - c1);
        *ox = ((Float)col + x) * (1.f / (Float)(nx - 1));
        *oy = ((Float)row + y) * (1.f / (Float)(ny - 1));
        *pdf = ((1.f - x) * c0 + x * c1) * ((Float)(nx - 1) * (Float)(ny - 1));
    }
};

struct Brdf {
    bool isotropic = true;
    Table ndf, sigma, vndf, luminance, spectra;
};

// the tensor file (bxdfs.cpp:734-816): "tensor_file\0", version 1.0, fields {name, ndim, dtype,
// offset, shape}; only what MeasuredBxDFData::Create reads
static bool Load(const char *path, Brdf *b) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return false;
    std::vector<uint8_t> bytes;
    uint8_t buf[65536];
    size_t got;
    while ((got = std::fread(buf, 1, sizeof(buf), fp)) > 0) bytes.insert(bytes.end(), buf, buf + got);
    std::fclose(fp);
    if (bytes.size() < 18 || std::memcmp(bytes.data(), "tensor_file", 12) != 0) return false;
    size_t pos = 14;
    auto rd = [&](void *dst, size_t n) {
        std::memcpy(dst, bytes.data() + pos, n);
        pos += n;
    };
    uint32_t nf;
    rd(&nf, 4);
    struct F {
        std::vector<size_t> shape;
        const float *p;
    };
    std::map<std::string, F> fs;
    for (uint32_t k = 0; k < nf; ++k) {
        uint16_t len, nd;
        uint8_t dt;
        uint64_t off;
        rd(&len, 2);
        std::string name((const char *)bytes.data() + pos, len);
        pos += len;
        rd(&nd, 2);
        rd(&dt, 1);
        rd(&off, 8);
        F f;
        for (int j = 0; j < nd; ++j) {
            uint64_t v;
            rd(&v, 8);
            f.shape.push_back((size_t)v);
        }
        f.p = (const float *)(bytes.data() + off);
        fs[name] = f;
    }
    const F &phi = fs["phi_i"], &theta = fs["theta_i"], &wl = fs["wavelengths"];
    std::vector<float> pv[3] = {std::vector<float>(phi.p, phi.p + phi.shape[0]),
                                std::vector<float>(theta.p, theta.p + theta.shape[0]),
                                std::vector<float>(wl.p, wl.p + wl.shape[0])};
    b->isotropic = phi.shape[0] <= 2;
    const F &nd = fs["ndf"], &sg = fs["sigma"], &vn = fs["vndf"], &lu = fs["luminance"], &sp = fs["spectra"];
    b->ndf.Build(nd.p, (int)nd.shape[1], (int)nd.shape[0], 0, pv, false, false);
    b->sigma.Build(sg.p, (int)sg.shape[1], (int)sg.shape[0], 0, pv, false, false);
    b->vndf.Build(vn.p, (int)vn.shape[3], (int)vn.shape[2], 2, pv, true, true);
    b->luminance.Build(lu.p, (int)lu.shape[3], (int)lu.shape[2], 2, pv, true, true);
    b->spectra.Build(sp.p, (int)sp.shape[4], (int)sp.shape[3], 3, pv, false, false);
    return true;
}

static inline Float Theta2u(Float t) { return std::sqrt(t * (2 / Pi)); }
static inline Float Phi2u(Float p) { return p * (1 / (2 * Pi)) + .5f; }

struct Measured {
    const Brdf *b = nullptr;
    Spectrum lambda;

    Spectrum Fr(Float ux, Float uy, Float phi_o, Float theta_o) const {
        Spectrum fr;
        for (int i = 0; i < NS; ++i) {
            const Float par[3] = {phi_o, theta_o, lambda[i]};
            fr[i] = std::max<Float>(0, b->spectra.Evaluate(ux, uy, par));
        }
        return fr;
    }
    Spectrum f(Vec wo, Vec wi) const {
        if (!SameHemisphere(wo, wi)) return Spectrum(0.f);
        if (wo.z < 0) wo = -wo, wi = -wi;
        Vec wm = wi + wo;
        if (LengthSquared(wm) == 0) return Spectrum(0.f);
        wm = Normalize(wm);
        const Float theta_o = SafeACos(wo.z), phi_o = CRATan2(wo.y, wo.x);
        const Float theta_m = SafeACos(wm.z), phi_m = CRATan2(wm.y, wm.x);
        const Float uo[2] = {Theta2u(theta_o), Phi2u(phi_o)};
        Float um[2] = {Theta2u(theta_m), Phi2u(b->isotropic ? (phi_m - phi_o) : phi_m)};
        um[1] = um[1] - std::floor(um[1]);
        const Float par[2] = {phi_o, theta_o};
        Float ux, uy, unused;
        b->vndf.Invert(um[0], um[1], par, &ux, &uy, &unused);
        Spectrum fr = Fr(ux, uy, phi_o, theta_o);
        const Float n = b->ndf.Evaluate(um[0], um[1], nullptr);
        const Float den = 4 * b->sigma.Evaluate(uo[0], uo[1], nullptr) * wi.z;
        for (int i = 0; i < NS; ++i) fr[i] = fr[i] * n / den;
        return fr;
    }
    bool Sample_f(Vec wo, Float u0, Float u1, BSDFSample *bs) const {
        bool flip = false;
        if (wo.z <= 0) wo = -wo, flip = true;
        const Float theta_o = SafeACos(wo.z), phi_o = CRATan2(wo.y, wo.x);
        const Float par[2] = {phi_o, theta_o};
        Float ux, uy, lumPdf, mx, my, pdf;
        b->luminance.Sample(u0, u1, par, &ux, &uy, &lumPdf);
        b->vndf.Sample(ux, uy, par, &mx, &my, &pdf);
        Float phi_m = (2.f * my - 1.f) * Pi;
        const Float theta_m = Sqr(mx) * (Pi / 2.f);
        if (b->isotropic) phi_m += phi_o;
        const Float sinTheta_m = CRSin(theta_m), cosTheta_m = CRCos(theta_m);
        const Float st = Clamp(sinTheta_m, -1, 1);
        const Vec wm(st * CRCos(phi_m), st * CRSin(phi_m), Clamp(cosTheta_m, -1, 1));
        Vec wi = Reflect(wo, wm);
        if (wi.z <= 0) return false;
        Spectrum fr = Fr(ux, uy, phi_o, theta_o);
        const Float s = b->ndf.Evaluate(mx, my, nullptr) /
                        (4 * b->sigma.Evaluate(Theta2u(theta_o), Phi2u(phi_o), nullptr) * std::abs(wi.z));
        for (int i = 0; i < NS; ++i) fr[i] *= s;
        pdf /= 4 * Dot(wo, wm) * std::max<Float>(2 * Sqr(Pi) * mx * sinTheta_m, 1e-6f);
        if (flip) wi = -wi;
        *bs = BSDFSample{fr, wi, pdf * lumPdf, BxR | BxGlossy, 1};
        return true;
    }
    Float PDF(Vec wo, Vec wi) const {
        if (!SameHemisphere(wo, wi)) return 0;
        if (wo.z < 0) wo = -wo, wi = -wi;
        Vec wm = wi + wo;
        if (LengthSquared(wm) == 0) return 0;
        wm = Normalize(wm);
        const Float theta_o = SafeACos(wo.z), phi_o = CRATan2(wo.y, wo.x);
        const Float theta_m = SafeACos(wm.z), phi_m = CRATan2(wm.y, wm.x);
        Float um[2] = {Theta2u(theta_m), Phi2u(b->isotropic ? (phi_m - phi_o) : phi_m)};
        um[1] = um[1] - std::floor(um[1]);
        const Float par[2] = {phi_o, theta_o};
        Float sx, sy, vndfPdf;
        b->vndf.Invert(um[0], um[1], par, &sx, &sy, &vndfPdf);
        const Float pdf = b->luminance.Evaluate(sx, sy, par);
        const Float sinTheta_m = std::sqrt(Sqr(wm.x) + Sqr(wm.y));
        const Float jac = 4.f * Dot(wo, wm) * std::max<Float>(2 * Sqr(Pi) * um[0] * sinTheta_m, 1e-6f);
        return vndfPdf * pdf / jac;
    }
};
}  // namespace omeas

struct BxDF {
    int type = 0;  // 0 diffuse, 1 dielectric, 2 conductor, 6 thin dielectric, 7 diffuse transmission, 9 hair
    Spectrum R, Tt;  // Tt: DiffuseTransmissionBxDF's T
    Float eta = 1;
    TRDistribution mf;
    Spectrum etaS, kS;
    ohair::Hair hair;
    omeas::Measured meas;  // type 10

    int Flags() const {
        if (type == 9 || type == 10) return BxR | BxGlossy;  // MeasuredBxDF::Flags (bxdfs.h:1176)  // HairBxDF::Flags (bxdfs.h:1079)
        if (type == 0) return R ? (BxR | BxDiffuse) : 0;
        if (type == 6) return BxR | BxT | BxSpecular;  // ThinDielectricBxDF
        if (type == 7) return (R ? (BxR | BxDiffuse) : 0) | (Tt ? (BxT | BxDiffuse) : 0);
        int lobe = mf.Smooth() ? BxSpecular : BxGlossy;
        if (type == 1) return (eta == 1 ? BxT : (BxR | BxT)) | lobe;
        return BxR | lobe;
    }
    Spectrum FrC(Float cosI) const {
        Spectrum r;
        for (int i = 0; i < NS; ++i) r[i] = FrComplex(cosI, Complex(etaS[i], kS[i]));
        return r;
    }
    bool Sample_f(Vec wo, Float uc, Float u0, Float u1, BSDFSample *bs, bool radiance = true, int sf = 3) const {
        if (type == 9) return hair.Sample_f(wo, uc, u0, u1, bs);
        if (type == 10) return (sf & 1) && meas.Sample_f(wo, u0, u1, bs);
        if (type == 7) {
            // DiffuseTransmissionBxDF::Sample_f (bxdfs.h:231-260)
            Float pr = (sf & 1) ? R.Max() : 0, pt = (sf & 2) ? Tt.Max() : 0;
            if (pr == 0 && pt == 0) return false;
            Vec wi = SampleCosineHemisphere(u0, u1);
            if (uc < pr / (pr + pt)) {
                if (wo.z < 0) wi.z *= -1;
                *bs = BSDFSample{f(wo, wi), wi, std::abs(wi.z) * InvPi * pr / (pr + pt), BxR | BxDiffuse, 1};
            } else {
                if (wo.z > 0) wi.z *= -1;
                *bs = BSDFSample{f(wo, wi), wi, std::abs(wi.z) * InvPi * pt / (pr + pt), BxT | BxDiffuse, 1};
            }
            return true;
        }
        if (type == 6) {
            // ThinDielectricBxDF::Sample_f (bxdfs.h:355-386)
            Float R_ = FrDielectric(std::abs(wo.z), eta), T_ = 1 - R_;
            if (R_ < 1) {
                R_ += Sqr(T_) * R_ / (1 - Sqr(R_));
                T_ = 1 - R_;
            }
            Float pr = (sf & 1) ? R_ : 0, pt = (sf & 2) ? T_ : 0;
            if (pr == 0 && pt == 0) return false;
            if (uc < pr / (pr + pt)) {
                Vec wi(-wo.x, -wo.y, wo.z);
                *bs = BSDFSample{Spectrum(R_ / std::abs(wi.z)), wi, pr / (pr + pt), BxR | BxSpecular, 1};
            } else {
                Vec wi = -wo;
                *bs = BSDFSample{Spectrum(T_ / std::abs(wi.z)), wi, pt / (pr + pt), BxT | BxSpecular, 1};
            }
            return true;
        }
        if (type != 1 && !(sf & 1)) return false;
        if (type == 0) {
            Vec wi = SampleCosineHemisphere(u0, u1);
            if (wo.z < 0) wi.z *= -1;
            *bs = BSDFSample{R * InvPi, wi, std::abs(wi.z) * InvPi, BxR | BxDiffuse, 1};
            return true;
        }
        if (type == 11 && mf.Smooth()) {
            // RetroreflectiveBxDF::Sample_f (bxdfs.h:119-129): the smooth case sends wi = wo
            Vec wi = wo;
            *bs = BSDFSample{FrC(std::abs(wi.z)) / std::abs(wi.z), wi, 1, BxR | BxSpecular, 1};
            return true;
        }
        if (type == 2 || type == 11) {  // the rough retroreflective sample is the conductor's (bxdfs.h:130-152)
            if (mf.Smooth()) {
                Vec wi(-wo.x, -wo.y, wo.z);
                *bs = BSDFSample{FrC(std::abs(wi.z)) / std::abs(wi.z), wi, 1, BxR | BxSpecular, 1};
                return true;
            }
            if (wo.z == 0) return false;
            Vec wm = mf.Sample_wm(wo, u0, u1);
            Vec wi = Reflect(wo, wm);
            if (!SameHemisphere(wo, wi)) return false;
            Float pdf = mf.PDF(wo, wm) / (4 * AbsDot(wo, wm));
            Float co = std::abs(wo.z), ci = std::abs(wi.z);
            if (ci == 0 || co == 0) return false;
            Spectrum F = FrC(AbsDot(wo, wm));
            *bs = BSDFSample{F * mf.D(wm) * mf.G(wo, wi) / (4 * ci * co), wi, pdf, BxR | BxGlossy, 1};
            return true;
        }
        if (eta == 1 || mf.Smooth()) {
            Float R_ = FrDielectric(wo.z, eta), T_ = 1 - R_;
            Float pr = (sf & 1) ? R_ : 0, pt = (sf & 2) ? T_ : 0;
            if (pr == 0 && pt == 0) return false;
            if (uc < pr / (pr + pt)) {
                Vec wi(-wo.x, -wo.y, wo.z);
                *bs = BSDFSample{Spectrum(R_ / std::abs(wi.z)), wi, pr / (pr + pt), BxR | BxSpecular, 1};
                return true;
            }
            Vec wi;
            Float etap;
            if (!Refract(wo, Vec(0, 0, 1), eta, &etap, &wi)) return false;
            Spectrum ft(T_ / std::abs(wi.z));
            if (radiance) ft = ft / Sqr(etap);
            *bs = BSDFSample{ft, wi, pt / (pr + pt), BxT | BxSpecular, etap};
            return true;
        }
        Vec wm = mf.Sample_wm(wo, u0, u1);
        Float R_ = FrDielectric(Dot(wo, wm), eta), T_ = 1 - R_;
        Float pr = (sf & 1) ? R_ : 0, pt = (sf & 2) ? T_ : 0;
        if (pr == 0 && pt == 0) return false;
        if (uc < pr / (pr + pt)) {
            Vec wi = Reflect(wo, wm);
            if (!SameHemisphere(wo, wi)) return false;
            Float pdf = mf.PDF(wo, wm) / (4 * AbsDot(wo, wm)) * pr / (pr + pt);
            Spectrum f(mf.D(wm) * mf.G(wo, wi) * R_ / (4 * wi.z * wo.z));
            *bs = BSDFSample{f, wi, pdf, BxR | BxGlossy, 1};
            return true;
        }
        Float etap;
        Vec wi;
        bool tir = !Refract(wo, wm, eta, &etap, &wi);
        if (SameHemisphere(wo, wi) || wi.z == 0 || tir) return false;
        Float denom = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap);
        Float dwm_dwi = AbsDot(wi, wm) / denom;
        Float pdf = mf.PDF(wo, wm) * dwm_dwi * pt / (pr + pt);
        Spectrum ft(T_ * mf.D(wm) * mf.G(wo, wi) * std::abs(Dot(wi, wm) * Dot(wo, wm) / (wi.z * wo.z * denom)));
        if (radiance) ft = ft / Sqr(etap);
        *bs = BSDFSample{ft, wi, pdf, BxT | BxGlossy, etap};
        return true;
    }
    // the generalized half vector of a dielectric pair, or false (f = pdf = 0)
    bool DielectricHalf(Vec wo, Vec wi, Vec *wm, Float *etap, bool *reflect) const {
        Float co = wo.z, ci = wi.z;
        *reflect = ci * co > 0;
        *etap = 1;
        if (!*reflect) *etap = co > 0 ? eta : (1 / eta);
        Vec h = wi * *etap + wo;
        if (ci == 0 || co == 0 || LengthSquared(h) == 0) return false;
        h = Normalize(h);
        if (h.z < 0) h = -h;  // FaceForward(wm, (0,0,1))
        if (Dot(h, wi) * ci < 0 || Dot(h, wo) * co < 0) return false;
        *wm = h;
        return true;
    }
    Spectrum f(Vec wo, Vec wi, bool radiance = true) const {
        if (type == 9) return hair.f(wo, wi);
        if (type == 10) return meas.f(wo, wi);
        if (type == 6) return Spectrum(0.f);
        if (type == 7) return SameHemisphere(wo, wi) ? R * InvPi : Tt * InvPi;
        if (type == 0) return SameHemisphere(wo, wi) ? R * InvPi : Spectrum(0.f);
        if (type == 11) {
            // RetroreflectiveBxDF::f (bxdfs.h:155-178): a retro lobe about wo plus the conductor
            // lobe, both scaled by 1 - (R_i - R_o)
            if (!SameHemisphere(wo, wi) || mf.Smooth()) return Spectrum(0.f);
            Float co = std::abs(wo.z), ci = std::abs(wi.z);
            if (ci == 0 || co == 0) return Spectrum(0.f);
            Vec wm = wo + wi, wmRetro = wo;
            if (LengthSquared(wm) == 0) return Spectrum(0.f);
            wm = Normalize(wm);
            Float R_o = FrDielectric(Dot(wo, wm), 1.59f), R_i = FrDielectric(Dot(wi, wmRetro), 1.59f);
            Spectrum F = FrC(AbsDot(wo, wm)), Fr = FrC(AbsDot(wi, wmRetro));
            Spectrum retro = Fr * mf.D(wmRetro) * mf.G(wo, wi) / (4 * ci * co);
            Float w = 1 - (R_i - R_o);
            return retro * w + (F * mf.D(wm) * mf.G(wo, wi) / (4 * ci * co)) * w;
        }
        if (type == 2) {
            if (!SameHemisphere(wo, wi) || mf.Smooth()) return Spectrum(0.f);
            Float co = std::abs(wo.z), ci = std::abs(wi.z);
            if (ci == 0 || co == 0) return Spectrum(0.f);
            Vec wm = wi + wo;
            if (LengthSquared(wm) == 0) return Spectrum(0.f);
            wm = Normalize(wm);
            Spectrum F = FrC(AbsDot(wo, wm));
            return F * mf.D(wm) * mf.G(wo, wi) / (4 * ci * co);
        }
        if (eta == 1 || mf.Smooth()) return Spectrum(0.f);
        Vec wm;
        Float etap;
        bool reflect;
        if (!DielectricHalf(wo, wi, &wm, &etap, &reflect)) return Spectrum(0.f);
        Float F = FrDielectric(Dot(wo, wm), eta);
        if (reflect) return Spectrum(mf.D(wm) * mf.G(wo, wi) * F / std::abs(4 * wi.z * wo.z));
        Float denom = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap) * wi.z * wo.z;
        Float ft = mf.D(wm) * (1 - F) * mf.G(wo, wi) * std::abs(Dot(wi, wm) * Dot(wo, wm) / denom);
        if (radiance) ft /= Sqr(etap);
        return Spectrum(ft);
    }
    Float PDF(Vec wo, Vec wi, int sf = 3) const {
        if (type == 9) return hair.PDF(wo, wi);
        if (type == 10) return (sf & 1) ? meas.PDF(wo, wi) : 0;
        if (type == 6) return 0;
        if (type == 7) {
            Float pr = (sf & 1) ? R.Max() : 0, pt = (sf & 2) ? Tt.Max() : 0;
            if (pr == 0 && pt == 0) return 0;
            return (SameHemisphere(wo, wi) ? pr : pt) / (pr + pt) * (std::abs(wi.z) * InvPi);
        }
        if (type != 1 && !(sf & 1)) return 0;
        if (type == 0) return SameHemisphere(wo, wi) ? std::abs(wi.z) * InvPi : 0;
        if (type == 2 || type == 11) {  // RetroreflectiveBxDF::PDF is the conductor's (bxdfs.h:181-201)
            if (!SameHemisphere(wo, wi) || mf.Smooth()) return 0;
            Vec wm = wo + wi;
            if (LengthSquared(wm) == 0) return 0;
            wm = Normalize(wm);
            if (wm.z < 0) wm = -wm;
            return mf.PDF(wo, wm) / (4 * AbsDot(wo, wm));
        }
        if (eta == 1 || mf.Smooth()) return 0;
        Vec wm;
        Float etap;
        bool reflect;
        if (!DielectricHalf(wo, wi, &wm, &etap, &reflect)) return 0;
        Float R_ = FrDielectric(Dot(wo, wm), eta), T_ = 1 - R_;
        Float pr = (sf & 1) ? R_ : 0, pt = (sf & 2) ? T_ : 0;
        if (pr == 0 && pt == 0) return 0;
        if (reflect) return mf.PDF(wo, wm) / (4 * AbsDot(wo, wm)) * pr / (pr + pt);
        Float denom = Sqr(Dot(wi, wm) + Dot(wo, wm) / etap);
        return mf.PDF(wo, wm) * (AbsDot(wi, wm) / denom) * pt / (pr + pt);
    }
};

// PiecewiseLinearSpectrum::operator() (util/spectrum.cpp:68-78)
static Float PLEval(const float *lam, const float *val, int n, Float l) {
    if (n == 0 || l < lam[0] || l > lam[n - 1]) return 0;
    // FindInterval (util/math.h:509-520): binary search for the last lam[i] <= l, i <= n-2
    int size = n - 2, first = 1;
    while (size > 0) {
        int half = size >> 1, middle = first + half;
        bool pr = lam[middle] <= l;
        first = pr ? middle + 1 : first;
        size = pr ? size - (half + 1) : half;
    }
    int o = std::min(std::max(first - 1, 0), n - 2);
    Float t = (l - lam[o]) / (lam[o + 1] - lam[o]);
    return Lerp(t, val[o], val[o + 1]);
}

// ---------------------------------------------------------------- media
// HomogeneousMedium / GridMedium (media.h:209-350), HGPhaseFunction (media.h:43-70,
// util/scattering.h:49-58, util/sampling.cpp:347-373), SampleT_maj (media.h:725-800) with
// the majorant iterators (media.h:79-205), PCG32 RNG (util/rng.h:30-140) seeded from ray
// hashes (util/hash.h), FastExp's CPU polynomial (util/math.h:450-475).
struct PCG32 {
    uint64_t state = 0, inc = 1;
    PCG32(uint64_t seqIndex, uint64_t offset) {
        state = 0u;
        inc = (seqIndex << 1u) | 1u;
        NextU32();
        state += offset;
        NextU32();
    }
    uint32_t NextU32() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    Float Uniform() { return std::min<Float>(OneMinusEpsilon, NextU32() * 0x1p-32f); }
};
template <typename... T>
static uint64_t HashFloats(T... v) {
    const float a[] = {float(v)...};
    return Murmur64A((const unsigned char *)a, sizeof(a), 0);
}

static Float FastExp(Float x) {
    Float xp = x * 1.442695041f;
    if (!(xp > -256.f)) return 0;  // far below the float range (and NaN): the exponent test's 0
    if (xp > 256.f) return Infinity;
    Float fxp = std::floor(xp), f = xp - fxp;
    int i = (int)fxp;
    // EvaluatePolynomial(f, 1, 0.695556856, 0.226173572, 0.0781455737) with FMA
    Float twoToF = std::fma(f, std::fma(f, std::fma(f, 0.0781455737f, 0.226173572f), 0.695556856f), 1.f);
    int exponent = (int)((FloatToBits(twoToF) >> 23) & 0xff) - 127 + i;
    if (exponent < -126) return 0;
    if (exponent > 127) return Infinity;
    uint32_t bits = FloatToBits(twoToF);
    bits &= 0b10000000011111111111111111111111u;
    bits |= (uint32_t)(exponent + 127) << 23;
    return BitsToFloat(bits);
}

// Blackbody (util/spectrum.h:69-80) and BlackbodySpectrum::Sample (util/spectrum.h:530-560):
// Planck's law over its value at Wien's peak lambda_max = 2.8977721e-3 / T
static Float Blackbody(Float lambda, Float T) {
    if (T <= 0) return 0;
    const Float c = 299792458.f, h = 6.62606957e-34f, kb = 1.3806488e-23f;
    const Float l = lambda * 1e-9f;
    const Float l5 = (l * l) * (l * l) * l;  // Pow<5>
    return (2 * h * c * c) / (l5 * (FastExp((h * c) / (l * kb * T)) - 1));
}
static Float BlackbodySample(Float lambda, Float T) {
    const Float lambdaMax = 2.8977721e-3f / T;
    const Float normalizationFactor = 1 / Blackbody(lambdaMax * 1e9f, T);
    return Blackbody(lambda, T) * normalizationFactor;
}

static Float HenyeyGreenstein(Float cosTheta, Float g) {
    g = Clamp(g, -.99f, .99f);
    Float denom = 1 + Sqr(g) + 2 * g * cosTheta;
    return (1 / (4 * Pi)) * (1 - Sqr(g)) / (denom * SafeSqrt(denom));
}
static Vec SampleHG(Vec wo, Float g, Float u0, Float u1, Float *pdf) {
    g = Clamp(g, -.99f, .99f);
    Float cosTheta;
    if (std::abs(g) < 1e-3f) cosTheta = 1 - 2 * u0;
    else cosTheta = -1 / (2 * g) * (1 + Sqr(g) - Sqr((1 - Sqr(g)) / (1 + g - 2 * g * u0)));
    Float sinTheta = SafeSqrt(1 - Sqr(cosTheta));
    Float phi = 2 * Pi * u1;
    // Frame::FromZ(wo).FromLocal(SphericalDirection(sinTheta, cosTheta, phi))
    Vec z = wo, x, y;
    CoordinateSystem(z, &x, &y);
    Vec l(Clamp(sinTheta, -1, 1) * CRCos(phi), Clamp(sinTheta, -1, 1) * CRSin(phi), Clamp(cosTheta, -1, 1));
    *pdf = HenyeyGreenstein(cosTheta, g);
    return x * l.x + y * l.y + z * l.z;
}

// ---------------------------------------------------------------- layered BxDFs
// LayeredBxDF<DielectricBxDF, DiffuseBxDF | ConductorBxDF, twoSided = true> (bxdfs.h:565-1052),
// i.e. CoatedDiffuseBxDF and CoatedConductorBxDF.  Written over the BxDF above with pbrt's
// SampledSpectrum arithmetic.  The RNG streams follow the reference: RNG(Hash(seed, wo), Hash(wi))
// for f, RNG(Hash(seed, wo), Hash(uc, u)) for Sample_f, RNG(Hash(seed, wi), Hash(wo)) for PDF,
// seed = GetOptions().seed (0, pbrt's default).  Where the reference draws a sample as
// `Sample_f(w, r(), {r(), r()})` / `Point2f(r(), r())` (argument order unspecified in C++), the
// draws are taken left to right; that choice is shared with core.h and is why parity with a
// pbrt binary is unpinned for these materials.
static uint64_t HashIntVec(int a, Vec v) {
    unsigned char b[16];
    float f[3] = {v.x, v.y, v.z};
    std::memcpy(b, &a, 4);
    std::memcpy(b + 4, f, 12);
    return Murmur64A(b, 16, 0);
}
static Float PowerHeuristic(Float nf, Float fPdf, Float ng, Float gPdf) {
    Float f = nf * fPdf, g = ng * gPdf;
    if (std::isinf(Sqr(f))) return 1;
    return Sqr(f) / (Sqr(f) + Sqr(g));
}
struct LayeredBxDF {
    BxDF top, bottom;  // top: type 1; bottom: type 0 or 2
    Float thickness = .01f, g = 0;
    Spectrum albedo;
    int maxDepth = 10, nSamples = 1;
    int seed = 0;

    static Float Tr(Float dz, Vec w) {
        if (std::abs(dz) <= std::numeric_limits<Float>::min()) return 1;
        return FastExp(-std::abs(dz / w.z));
    }
    // a sampled lobe that the reference keeps: exists, f != 0, pdf > 0 (wi.z tested by callers)
    static bool Good(bool ok, const BSDFSample &bs) { return ok && bs.f && bs.pdf > 0; }
    const BxDF &Iface(bool isTop) const { return isTop ? top : bottom; }

    int Flags() const {
        int tf = top.Flags(), bf = bottom.Flags();
        int fl = BxR;
        if (tf & BxSpecular) fl |= BxSpecular;
        if ((tf & BxDiffuse) || (bf & BxDiffuse) || albedo) fl |= BxDiffuse;
        else if ((tf & BxGlossy) || (bf & BxGlossy)) fl |= BxGlossy;
        if ((tf & BxT) && (bf & BxT)) fl |= BxT;
        return fl;
    }

    Spectrum f(Vec wo, Vec wi, bool radiance) const {
        Spectrum fr(0.f);
        if (wo.z < 0) {
            wo = -wo;
            wi = -wi;
        }
        // entered through the top; the exit is the bottom when wo and wi are on opposite sides
        const bool exitBottom = !SameHemisphere(wo, wi);
        const BxDF &exitI = Iface(!exitBottom), &nonExitI = Iface(exitBottom);
        const Float exitZ = exitBottom ? 0 : thickness;
        if (SameHemisphere(wo, wi)) fr = top.f(wo, wi, radiance) * Float(nSamples);
        PCG32 rng(HashIntVec(seed, wo), HashFloats(wi.x, wi.y, wi.z));
        auto r = [&]() { return rng.Uniform(); };
        for (int s = 0; s < nSamples; ++s) {
            BSDFSample wos, wis;
            Float uc = r(), a = r(), b = r();
            bool ok = top.Sample_f(wo, uc, a, b, &wos, radiance, 2);
            if (!Good(ok, wos) || wos.wi.z == 0) continue;
            uc = r();
            a = r();
            b = r();
            ok = exitI.Sample_f(wi, uc, a, b, &wis, !radiance, 2);
            if (!Good(ok, wis) || wis.wi.z == 0) continue;
            Spectrum beta = wos.f * std::abs(wos.wi.z) / wos.pdf;
            Float z = thickness;
            Vec w = wos.wi;
            for (int depth = 0; depth < maxDepth; ++depth) {
                if (depth > 3 && beta.Max() < 0.25f) {
                    Float q = std::max<Float>(0, 1 - beta.Max());
                    if (r() < q) break;
                    beta = beta / (1 - q);
                }
                if (!albedo) {
                    z = (z == thickness) ? 0 : thickness;
                    beta = beta * Tr(thickness, w);
                } else {
                    Float dz = -CRLog(1 - r()) / (1 / std::abs(w.z));  // SampleExponential, sigma_t = 1
                    Float zp = w.z > 0 ? (z + dz) : (z - dz);
                    if (z == zp) continue;
                    if (0 < zp && zp < thickness) {
                        Float wt = 1;
                        if (!(exitI.Flags() & BxSpecular))
                            wt = PowerHeuristic(1, wis.pdf, 1, HenyeyGreenstein(Dot(-w, -wis.wi), g));
                        fr = fr + beta * albedo * HenyeyGreenstein(Dot(-w, -wis.wi), g) * wt * Tr(zp - exitZ, wis.wi) *
                                      wis.f / wis.pdf;
                        Float u0 = r(), u1 = r(), ppdf;
                        Vec pwi = SampleHG(-w, g, u0, u1, &ppdf);
                        if (ppdf == 0 || pwi.z == 0) continue;
                        beta = beta * (albedo * ppdf / ppdf);
                        w = pwi;
                        z = zp;
                        if (((z < exitZ && w.z > 0) || (z > exitZ && w.z < 0)) && !(exitI.Flags() & BxSpecular)) {
                            Spectrum fExit = exitI.f(-w, wi, radiance);
                            if (fExit) {
                                Float exitPDF = exitI.PDF(-w, wi, 2);
                                Float wt2 = PowerHeuristic(1, ppdf, 1, exitPDF);
                                fr = fr + beta * Tr(zp - exitZ, pwi) * fExit * wt2;
                            }
                        }
                        continue;
                    }
                    z = Clamp(zp, 0, thickness);
                }
                if (z == exitZ) {
                    BSDFSample bs;
                    Float c = r(), a2 = r(), b2 = r();
                    bool ok2 = exitI.Sample_f(-w, c, a2, b2, &bs, radiance, 1);
                    if (!Good(ok2, bs) || bs.wi.z == 0) break;
                    beta = beta * (bs.f * std::abs(bs.wi.z) / bs.pdf);
                    w = bs.wi;
                } else {
                    if (!(nonExitI.Flags() & BxSpecular)) {
                        Float wt = 1;
                        if (!(exitI.Flags() & BxSpecular)) wt = PowerHeuristic(1, wis.pdf, 1, nonExitI.PDF(-w, -wis.wi));
                        fr = fr + beta * nonExitI.f(-w, -wis.wi, radiance) * std::abs(wis.wi.z) * wt *
                                      Tr(thickness, wis.wi) * wis.f / wis.pdf;
                    }
                    BSDFSample bs;
                    Float c = r(), a2 = r(), b2 = r();
                    bool ok2 = nonExitI.Sample_f(-w, c, a2, b2, &bs, radiance, 1);
                    if (!Good(ok2, bs) || bs.wi.z == 0) break;
                    beta = beta * (bs.f * std::abs(bs.wi.z) / bs.pdf);
                    w = bs.wi;
                    if (!(exitI.Flags() & BxSpecular)) {
                        Spectrum fExit = exitI.f(-w, wi, radiance);
                        if (fExit) {
                            Float wt = 1;
                            if (!(nonExitI.Flags() & BxSpecular)) wt = PowerHeuristic(1, bs.pdf, 1, exitI.PDF(-w, wi, 2));
                            fr = fr + beta * Tr(thickness, bs.wi) * fExit * wt;
                        }
                    }
                }
            }
        }
        return fr / Float(nSamples);
    }

    // BSDFSample with pdfIsProportional = true
    bool Sample_f(Vec wo, Float uc, Float u0, Float u1, BSDFSample *out, bool radiance) const {
        bool flipWi = false;
        if (wo.z < 0) {
            wo = -wo;
            flipWi = true;
        }
        BSDFSample bs;
        bool ok = top.Sample_f(wo, uc, u0, u1, &bs, radiance, 3);
        if (!Good(ok, bs) || bs.wi.z == 0) return false;
        if (bs.flags & BxR) {
            if (flipWi) bs.wi = -bs.wi;
            *out = bs;
            return true;
        }
        Vec w = bs.wi;
        bool specularPath = bs.flags & BxSpecular;
        PCG32 rng(HashIntVec(seed, wo), HashFloats(uc, u0, u1));
        auto r = [&]() { return rng.Uniform(); };
        Spectrum fr = bs.f * std::abs(bs.wi.z);
        Float pdf = bs.pdf;
        Float z = thickness;
        for (int depth = 0; depth < maxDepth; ++depth) {
            Float rrBeta = fr.Max() / pdf;
            if (depth > 3 && rrBeta < 0.25f) {
                Float q = std::max<Float>(0, 1 - rrBeta);
                if (r() < q) return false;
                pdf *= 1 - q;
            }
            if (w.z == 0) return false;
            if (albedo) {
                Float dz = -CRLog(1 - r()) / (1 / std::abs(w.z));
                Float zp = w.z > 0 ? (z + dz) : (z - dz);
                if (zp == z) return false;
                if (0 < zp && zp < thickness) {
                    Float a = r(), b = r(), ppdf;
                    Vec pwi = SampleHG(-w, g, a, b, &ppdf);
                    if (ppdf == 0 || pwi.z == 0) return false;
                    fr = fr * (albedo * ppdf);
                    pdf *= ppdf;
                    specularPath = false;
                    w = pwi;
                    z = zp;
                    continue;
                }
                z = Clamp(zp, 0, thickness);
            } else {
                z = (z == thickness) ? 0 : thickness;
                fr = fr * Tr(thickness, w);
            }
            const BxDF &in = Iface(z != 0);
            Float c = r(), a = r(), b = r();
            BSDFSample is;
            bool ok2 = in.Sample_f(-w, c, a, b, &is, radiance, 3);
            if (!Good(ok2, is) || is.wi.z == 0) return false;
            fr = fr * is.f;
            pdf *= is.pdf;
            specularPath &= (is.flags & BxSpecular) != 0;
            w = is.wi;
            if (is.flags & BxT) {
                int fl = SameHemisphere(wo, w) ? BxR : BxT;
                fl |= specularPath ? BxSpecular : BxGlossy;
                if (flipWi) w = -w;
                *out = BSDFSample{fr, w, pdf, fl, 1};
                return true;
            }
            fr = fr * std::abs(is.wi.z);
        }
        return false;
    }

    Float PDF(Vec wo, Vec wi, bool radiance) const {
        if (wo.z < 0) {
            wo = -wo;
            wi = -wi;
        }
        PCG32 rng(HashIntVec(seed, wi), HashFloats(wo.x, wo.y, wo.z));
        auto r = [&]() { return rng.Uniform(); };
        Float pdfSum = 0;
        if (SameHemisphere(wo, wi)) pdfSum += nSamples * top.PDF(wo, wi, 1);
        for (int s = 0; s < nSamples; ++s) {
            if (SameHemisphere(wo, wi)) {
                // TRT: transmit through the top, reflect off the bottom, transmit back out
                BSDFSample wos, wis;
                Float c = r(), a = r(), b = r();
                bool okO = Good(top.Sample_f(wo, c, a, b, &wos, radiance, 2), wos);
                c = r();
                a = r();
                b = r();
                bool okI = Good(top.Sample_f(wi, c, a, b, &wis, !radiance, 2), wis);
                if (okO && okI) {
                    if (!(top.Flags() & (BxDiffuse | BxGlossy))) {
                        pdfSum += bottom.PDF(-wos.wi, -wis.wi);
                    } else {
                        BSDFSample rs;
                        c = r();
                        a = r();
                        b = r();
                        if (Good(bottom.Sample_f(-wos.wi, c, a, b, &rs, radiance, 3), rs)) {
                            if (!(bottom.Flags() & (BxDiffuse | BxGlossy))) {
                                pdfSum += top.PDF(-rs.wi, wi);
                            } else {
                                Float rPDF = bottom.PDF(-wos.wi, -wis.wi);
                                pdfSum += PowerHeuristic(1, wis.pdf, 1, rPDF) * rPDF;
                                Float tPDF = top.PDF(-rs.wi, wi);
                                pdfSum += PowerHeuristic(1, rs.pdf, 1, tPDF) * tPDF;
                            }
                        }
                    }
                }
            } else {
                // TT: through the top and out of the bottom; the opaque bottom never transmits
                BSDFSample wos, wis;
                Float c = r(), a = r(), b = r();
                bool ok = top.Sample_f(wo, c, a, b, &wos, radiance, 3);
                if (!Good(ok, wos) || wos.wi.z == 0 || (wos.flags & BxR)) continue;
                c = r();
                a = r();
                b = r();
                ok = bottom.Sample_f(wi, c, a, b, &wis, !radiance, 3);
                if (!Good(ok, wis) || wis.wi.z == 0 || (wis.flags & BxR)) continue;
                if (top.Flags() & BxSpecular) pdfSum += bottom.PDF(-wos.wi, wi);
                else if (bottom.Flags() & BxSpecular) pdfSum += top.PDF(wo, -wis.wi);
                else pdfSum += (top.PDF(wo, -wis.wi) + bottom.PDF(-wos.wi, wi)) / 2;
            }
        }
        return Lerp(0.9f, 1 / (4 * Pi), pdfSum / nSamples);
    }
};

struct MediumProps {
    Spectrum sigma_a, sigma_s, Le;
};
struct MajorantSeg {
    Float tMin, tMax;
    Spectrum sigma_maj;
};

struct Media {
    const pbrt_scene_flat *f = nullptr;
    int n = 0;
    const int32_t *Info(int m) const { return f->medium_info + 16 * m; }
    const float *Params(int m) const { return f->medium_params + 24 * m; }
    Spectrum Dense(int idx, const Wavelengths &lambda) const { return SampleDense(f->dense_spectra + 311 * idx, lambda); }
    // Transform::ApplyInverse(Point3f) (util/transform.h:387-398)
    Vec ToMedium(int m, Vec p) const {
        const float *M = Params(m) + 8;
        Float x = (M[0] * p.x + M[1] * p.y) + (M[2] * p.z + M[3]);
        Float y = (M[4] * p.x + M[5] * p.y) + (M[6] * p.z + M[7]);
        Float z = (M[8] * p.x + M[9] * p.y) + (M[10] * p.z + M[11]);
        Float w = (M[12] * p.x + M[13] * p.y) + (M[14] * p.z + M[15]);
        return w == 1 ? Vec(x, y, z) : Vec(x, y, z) / w;
    }
    // SampledGrid<Float>::Lookup(Point3f) (util/containers.h:804-835)
    static Float GridLookup(const float *v, int nx, int ny, int nz, Vec p) {
        auto at = [&](int x, int y, int z) -> Float {
            if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return 0;
            return v[((size_t)z * ny + y) * nx + x];
        };
        Float sx = p.x * nx - .5f, sy = p.y * ny - .5f, sz = p.z * nz - .5f;
        int ix = (int)std::floor(sx), iy = (int)std::floor(sy), iz = (int)std::floor(sz);
        Float dx = sx - ix, dy = sy - iy, dz = sz - iz;
        Float d00 = Lerp(dx, at(ix, iy, iz), at(ix + 1, iy, iz));
        Float d10 = Lerp(dx, at(ix, iy + 1, iz), at(ix + 1, iy + 1, iz));
        Float d01 = Lerp(dx, at(ix, iy, iz + 1), at(ix + 1, iy, iz + 1));
        Float d11 = Lerp(dx, at(ix, iy + 1, iz + 1), at(ix + 1, iy + 1, iz + 1));
        return Lerp(dz, Lerp(dy, d00, d10), Lerp(dy, d01, d11));
    }
    // Bounds3::Offset (util/vecmath.h:1325-1334)
    Vec Offset(int m, Vec p) const {
        const float *P = Params(m);
        Vec o(p.x - P[1], p.y - P[2], p.z - P[3]);
        if (P[4] > P[1]) o.x /= P[4] - P[1];
        if (P[5] > P[2]) o.y /= P[5] - P[2];
        if (P[6] > P[3]) o.z /= P[6] - P[3];
        return o;
    }
    // util/noise.cpp Noise(x, y, z) / Grad / NoiseWeight (:53-118) over NoisePerm
    static Float NoiseAt(const float *perm, Float x, Float y, Float z) {
        auto grad = [&](int xi, int yi, int zi, Float dx, Float dy, Float dz) {
            int h = (int)perm[(int)perm[(int)perm[xi] + yi] + zi] & 15;
            Float u = h < 8 || h == 12 || h == 13 ? dx : dy;
            Float v = h < 4 || h == 12 || h == 13 ? dy : dz;
            return ((h & 1) ? -u : u) + ((h & 2) ? -v : v);
        };
        auto weight = [](Float t) {
            Float t2 = t * t;  // Pow<5> = t2 t2 t, Pow<4> = t2 t2 1, Pow<3> = t t t
            return 6 * (t2 * t2 * t) - 15 * (t2 * t2 * 1) + 10 * (t * t * t);
        };
        x = std::fmod(x, Float(1 << 30));
        y = std::fmod(y, Float(1 << 30));
        z = std::fmod(z, Float(1 << 30));
        int ix = (int)std::floor(x), iy = (int)std::floor(y), iz = (int)std::floor(z);
        Float dx = x - ix, dy = y - iy, dz = z - iz;
        ix &= 255, iy &= 255, iz &= 255;
        Float w000 = grad(ix, iy, iz, dx, dy, dz), w100 = grad(ix + 1, iy, iz, dx - 1, dy, dz);
        Float w010 = grad(ix, iy + 1, iz, dx, dy - 1, dz), w110 = grad(ix + 1, iy + 1, iz, dx - 1, dy - 1, dz);
        Float w001 = grad(ix, iy, iz + 1, dx, dy, dz - 1), w101 = grad(ix + 1, iy, iz + 1, dx - 1, dy, dz - 1);
        Float w011 = grad(ix, iy + 1, iz + 1, dx, dy - 1, dz - 1);
        Float w111 = grad(ix + 1, iy + 1, iz + 1, dx - 1, dy - 1, dz - 1);
        Float wx = weight(dx), wy = weight(dy), wz = weight(dz);
        Float y0 = Lerp(wy, Lerp(wx, w000, w100), Lerp(wx, w010, w110));
        Float y1 = Lerp(wy, Lerp(wx, w001, w101), Lerp(wx, w011, w111));
        return Lerp(wz, y0, y1);
    }
    // CloudMedium::Density (media.h:493-517); c = {density, wispiness, frequency, perm[512]}
    static Float CloudDensity(const float *c, Vec p) {
        const float *perm = c + 3;
        Vec pp = p * c[2];
        if (c[1] > 0) {
            Float vomega = 0.05f * c[1], vlambda = 10.f;
            for (int i = 0; i < 2; ++i) {
                Vec q = pp * vlambda;
                const Float delta = .01f;
                Float n = NoiseAt(perm, q.x, q.y, q.z);
                Vec dn((NoiseAt(perm, q.x + delta, q.y + 0.f, q.z + 0.f) - n) / delta,
                       (NoiseAt(perm, q.x + 0.f, q.y + delta, q.z + 0.f) - n) / delta,
                       (NoiseAt(perm, q.x + 0.f, q.y + 0.f, q.z + delta) - n) / delta);
                pp = pp + dn * vomega;
                vomega *= 0.5f;
                vlambda *= 1.99f;
            }
        }
        Float d = 0, omega = 0.5f, lambda = 1.f;
        for (int i = 0; i < 5; ++i) {
            Vec q = pp * lambda;
            d += omega * NoiseAt(perm, q.x, q.y, q.z);
            omega *= 0.5f;
            lambda *= 1.99f;
        }
        d = Clamp((1 - p.y) * 4.5f * c[0] * d, 0, 1);
        d += 2 * std::max<Float>(0, 0.5f - p.y);
        return Clamp(d, 0, 1);
    }
    MediumProps SamplePoint(int m, Vec p, const Wavelengths &lambda) const {
        const int32_t *I = Info(m);
        MediumProps mp{Dense(I[1], lambda), Dense(I[2], lambda), Spectrum(0.f)};
        if (I[0] == 0) {
            mp.Le = Dense(I[3], lambda);
            return mp;
        }
        if (I[0] == 2) {  // CloudMedium::SamplePoint: density * sigma (no emission)
            const Float d = CloudDensity(f->medium_values + I[11], ToMedium(m, p));
            mp.sigma_a = mp.sigma_a * d;
            mp.sigma_s = mp.sigma_s * d;
            return mp;
        }
        Vec q = Offset(m, ToMedium(m, p));
        if (I[0] == 3) {
            // RGBGridMedium::SamplePoint (media.h:377-400): per-wavelength trilinear lookups of
            // the voxels' RGBUnboundedSpectrum / RGBIlluminantSpectrum samples; voxel k of
            // block b is {c0, c1, c2, scale} at medium_values[I[11] + 4 (b n + k)]
            const int nx = I[5], ny = I[6], nz = I[7];
            const size_t n = (size_t)nx * ny * nz;
            const Spectrum illum = Dense(I[3], lambda);
            auto lookup = [&](int b) {
                const float *g = f->medium_values + I[11] + 4 * b * n;
                auto at = [&](int x, int y, int z) {
                    Spectrum s(0.f);
                    if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return s;
                    const float *c = g + 4 * (((size_t)z * ny + y) * nx + x);
                    for (int i = 0; i < NS; ++i) s[i] = c[3] * Sigmoid(c[0], c[1], c[2], lambda.lambda[i]);
                    return b == 2 ? s * illum : s;
                };
                Float sx = q.x * nx - .5f, sy = q.y * ny - .5f, sz = q.z * nz - .5f;
                int ix = (int)std::floor(sx), iy = (int)std::floor(sy), iz = (int)std::floor(sz);
                Float dx = sx - ix, dy = sy - iy, dz = sz - iz;
                auto SLerp = [](Float t, const Spectrum &a, const Spectrum &b) {
                    Spectrum r;
                    for (int i = 0; i < NS; ++i) r[i] = Lerp(t, a[i], b[i]);
                    return r;
                };
                Spectrum d00 = SLerp(dx, at(ix, iy, iz), at(ix + 1, iy, iz));
                Spectrum d10 = SLerp(dx, at(ix, iy + 1, iz), at(ix + 1, iy + 1, iz));
                Spectrum d01 = SLerp(dx, at(ix, iy, iz + 1), at(ix + 1, iy, iz + 1));
                Spectrum d11 = SLerp(dx, at(ix, iy + 1, iz + 1), at(ix + 1, iy + 1, iz + 1));
                return SLerp(dz, SLerp(dy, d00, d10), SLerp(dy, d01, d11));
            };
            const Float sigmaScale = Params(m)[7];
            mp.sigma_a = ((I[15] & 1) ? lookup(0) : Spectrum(1.f)) * sigmaScale;
            mp.sigma_s = ((I[15] & 2) ? lookup(1) : Spectrum(1.f)) * sigmaScale;
            const Float LeScale = f->medium_values[I[12]];
            if ((I[15] & 4) && LeScale > 0) mp.Le = lookup(2) * LeScale;
            return mp;
        }
        Float d = GridLookup(f->medium_values + I[11], I[5], I[6], I[7], q);
        mp.sigma_a = mp.sigma_a * d;
        mp.sigma_s = mp.sigma_s * d;
        if (I[4]) {
            Float scale = GridLookup(f->medium_values + I[12], I[8], I[9], I[10], q);
            if (scale > 0) {
                if (I[15] >= 0) {
                    // temperature grid (media.h:303-311): values[I[15]] = {offset, scale}, then
                    // the [nz][ny][nx] temperatures
                    const float *tg = f->medium_values + I[15];
                    Float temp = GridLookup(tg + 2, I[5], I[6], I[7], q);
                    temp = (temp - tg[0]) * tg[1];
                    if (temp > 100.f)
                        for (int i = 0; i < NS; ++i) mp.Le[i] = scale * BlackbodySample(lambda.lambda[i], temp);
                } else
                    mp.Le = Dense(I[3], lambda) * scale;
            }
        }
        return mp;
    }
};

// Majorant segments of a ray in medium m (HomogeneousMajorantIterator / DDAMajorantIterator)
struct MajorantIter {
    bool homogeneous = true, called = false, empty = false;
    MajorantSeg seg;
    // DDA state
    const float *grid = nullptr;
    Spectrum sigma_t;
    Float tMin = Infinity, tMax = -Infinity, nextCrossingT[3], deltaT[3];
    int step[3], voxelLimit[3], voxel[3];

    bool Next(MajorantSeg *out) {
        if (homogeneous) {
            if (called || empty) return false;
            called = true;
            *out = seg;
            return true;
        }
        if (empty || tMin >= tMax) return false;
        int bits = ((nextCrossingT[0] < nextCrossingT[1]) << 2) + ((nextCrossingT[0] < nextCrossingT[2]) << 1) +
                   ((nextCrossingT[1] < nextCrossingT[2]));
        const int cmpToAxis[8] = {2, 1, 2, 1, 2, 2, 0, 0};
        int stepAxis = cmpToAxis[bits];
        Float tVoxelExit = std::min(tMax, nextCrossingT[stepAxis]);
        Float mx = grid[voxel[0] + 16 * (voxel[1] + 16 * voxel[2])];
        *out = MajorantSeg{tMin, tVoxelExit, sigma_t * mx};
        tMin = tVoxelExit;
        if (nextCrossingT[stepAxis] > tMax) tMin = tMax;
        voxel[stepAxis] += step[stepAxis];
        if (voxel[stepAxis] == voxelLimit[stepAxis]) tMin = tMax;
        nextCrossingT[stepAxis] += deltaT[stepAxis];
        return true;
    }
};

static MajorantIter SampleRay(const Media &M, int m, Vec o, Vec d, Float raytMax, const Wavelengths &lambda) {
    MajorantIter it;
    const int32_t *I = M.Info(m);
    Spectrum sa = M.Dense(I[1], lambda), ss = M.Dense(I[2], lambda);
    if (I[0] == 0) {
        it.seg = MajorantSeg{0, raytMax, sa + ss};
        return it;
    }
    it.homogeneous = false;
    // Transform::ApplyInverse(Ray, &tMax) (util/transform.h:416-429): exact origin -> Point3fi
    const float *Mx = M.Params(m) + 8;
    Float x = o.x, y = o.y, z = o.z;
    Float xp = (Mx[0] * x + Mx[1] * y) + (Mx[2] * z + Mx[3]);
    Float yp = (Mx[4] * x + Mx[5] * y) + (Mx[6] * z + Mx[7]);
    Float zp = (Mx[8] * x + Mx[9] * y) + (Mx[10] * z + Mx[11]);
    Vec err(gamma(3) * (std::abs(Mx[0] * x) + std::abs(Mx[1] * y) + std::abs(Mx[2] * z)),
            gamma(3) * (std::abs(Mx[4] * x) + std::abs(Mx[5] * y) + std::abs(Mx[6] * z)),
            gamma(3) * (std::abs(Mx[8] * x) + std::abs(Mx[9] * y) + std::abs(Mx[10] * z)));
    Vec lo, hi;
    Vec pc(xp, yp, zp);
    for (int a = 0; a < 3; ++a) {
        lo[a] = err[a] == 0 ? pc[a] : NextFloatDown(pc[a] - err[a]);
        hi[a] = err[a] == 0 ? pc[a] : NextFloatUp(pc[a] + err[a]);
    }
    Vec dm(Mx[0] * d.x + Mx[1] * d.y + Mx[2] * d.z, Mx[4] * d.x + Mx[5] * d.y + Mx[6] * d.z,
           Mx[8] * d.x + Mx[9] * d.y + Mx[10] * d.z);
    Float l2 = LengthSquared(dm);
    if (l2 > 0) {
        Vec oErr((hi.x - lo.x) / 2, (hi.y - lo.y) / 2, (hi.z - lo.z) / 2);
        Float dt = Dot(Abs(dm), oErr) / l2;
        for (int a = 0; a < 3; ++a) {
            Float v = dm[a] * dt;
            lo[a] = NextFloatDown(lo[a] + v);
            hi[a] = NextFloatUp(hi[a] + v);
        }
        raytMax -= dt;
    }
    Vec om((lo.x + hi.x) / 2, (lo.y + hi.y) / 2, (lo.z + hi.z) / 2);
    // Bounds3::IntersectP(o, d, tMax, &t0, &t1) (util/vecmath.h:1549-1573)
    const float *P = M.Params(m);
    Float t0 = 0, t1 = raytMax;
    for (int a = 0; a < 3; ++a) {
        Float inv = 1 / dm[a];
        Float tNear = (P[1 + a] - om[a]) * inv, tFar = (P[4 + a] - om[a]) * inv;
        if (tNear > tFar) std::swap(tNear, tFar);
        tFar *= 1 + 2 * gamma(3);
        t0 = tNear > t0 ? tNear : t0;
        t1 = tFar < t1 ? tFar : t1;
        if (t0 > t1) {
            it.empty = true;
            return it;
        }
    }
    if (I[0] == 2) {  // CloudMedium: HomogeneousMajorantIterator(tMin, tMax, sigma_t)
        it.homogeneous = true;
        it.seg = MajorantSeg{t0, t1, sa + ss};
        return it;
    }
    // DDAMajorantIterator (media.h:168-205) over the medium's 16^3 majorant grid
    it.grid = M.f->medium_values + I[13];
    it.sigma_t = sa + ss;
    it.tMin = t0;
    it.tMax = t1;
    Vec diag(P[4] - P[1], P[5] - P[2], P[6] - P[3]);
    Vec og = M.Offset(m, om);
    Vec dg(dm.x / diag.x, dm.y / diag.y, dm.z / diag.z);
    Vec gi = og + dg * t0;
    for (int a = 0; a < 3; ++a) {
        it.voxel[a] = (int)Clamp(gi[a] * 16, 0, 15);
        it.deltaT[a] = 1 / (std::abs(dg[a]) * 16);
        if (dg[a] == -0.f) dg[a] = 0.f;
        if (dg[a] >= 0) {
            Float next = Float(it.voxel[a] + 1) / 16;
            it.nextCrossingT[a] = t0 + (next - gi[a]) / dg[a];
            it.step[a] = 1;
            it.voxelLimit[a] = 16;
        } else {
            Float next = Float(it.voxel[a]) / 16;
            it.nextCrossingT[a] = t0 + (next - gi[a]) / dg[a];
            it.step[a] = -1;
            it.voxelLimit[a] = -1;
        }
    }
    return it;
}

static Spectrum FastExpS(const Spectrum &s) {
    Spectrum r;
    for (int i = 0; i < NS; ++i) r[i] = FastExp(s[i]);
    return r;
}
static Spectrum ClampZero(const Spectrum &s) {
    Spectrum r;
    for (int i = 0; i < NS; ++i) r[i] = std::max<Float>(0, s[i]);
    return r;
}
static Spectrum operator-(const Spectrum &a, const Spectrum &b) {
    Spectrum r;
    for (int i = 0; i < NS; ++i) r[i] = a[i] - b[i];
    return r;
}

// SampleT_maj<ConcreteMedium>(ray, tMax, u, rng, lambda, callback) (media.h:737-800)
template <typename F>
static Spectrum SampleTmaj(const Media &M, int m, Vec o, Vec d, Float tMax, Float u, PCG32 &rng,
                           const Wavelengths &lambda, F callback) {
    tMax *= Length(d);
    d = Normalize(d);
    MajorantIter iter = SampleRay(M, m, o, d, tMax, lambda);
    Spectrum T_maj(1.f);
    MajorantSeg seg;
    while (true) {
        if (!iter.Next(&seg)) return T_maj;
        if (seg.sigma_maj[0] == 0) {
            Float dt = seg.tMax - seg.tMin;
            if (std::isinf(dt)) dt = std::numeric_limits<Float>::max();
            T_maj = T_maj * FastExpS(seg.sigma_maj * -dt);
            continue;
        }
        Float tMin = seg.tMin;
        while (true) {
            Float t = tMin + (-CRLog(1 - u) / seg.sigma_maj[0]);  // SampleExponential
            u = rng.Uniform();
            if (t < seg.tMax) {
                T_maj = T_maj * FastExpS(seg.sigma_maj * -(t - tMin));
                Vec p = o + d * t;
                MediumProps mp = M.SamplePoint(m, p, lambda);
                if (!callback(p, mp, seg.sigma_maj, T_maj)) return Spectrum(1.f);
                T_maj = Spectrum(1.f);
                tMin = t;
            } else {
                Float dt = seg.tMax - tMin;
                if (std::isinf(dt)) dt = std::numeric_limits<Float>::max();
                T_maj = T_maj * FastExpS(seg.sigma_maj * -dt);
                break;
            }
        }
    }
}

static int SampleDiscrete3(Float w0, Float w1, Float w2, Float u) {
    const Float w[3] = {w0, w1, w2};
    Float sum = 0;
    for (Float x : w) sum += x;
    Float up = u * sum;
    if (up == sum) up = NextFloatDown(up);
    int offset = 0;
    Float acc = 0;
    while (acc + w[offset] <= up) acc += w[offset++];
    return offset;
}

// ---------------------------------------------------------------- pixel filters
// Filters (filters.h, filters.cpp): Box, Gaussian, Mitchell, LanczosSinc, Triangle.  The
// tabulated ones sample through FilterSampler (filters.cpp:133-147) = PiecewiseConstant2D
// (util/sampling.h:603-790) over |f| at 32 samples per unit radius; weight = f / pdf.
struct Distribution1D {
    std::vector<Float> func, cdf;
    Float lo = 0, hi = 1, integral = 0;
    void Init(const Float *f, int n, Float mn, Float mx) {
        lo = mn;
        hi = mx;
        func.assign(f, f + n);
        for (Float &x : func) x = std::abs(x);
        cdf.assign(n + 1, 0);
        for (int i = 1; i <= n; ++i) cdf[i] = cdf[i - 1] + func[i - 1] * (mx - mn) / n;
        integral = cdf[n];
        for (int i = 1; i <= n; ++i) cdf[i] = integral == 0 ? Float(i) / Float(n) : cdf[i] / integral;
    }
    Float Sample(Float u, Float *pdf, int *off) const {
        // FindInterval over cdf: last i in [0, n - 1] with cdf[i] <= u
        int n = (int)func.size();
        int lo_ = 0, hi_ = n - 1;  // invariant: cdf[lo_] <= u or lo_ == 0
        int size = n + 1 - 2, first = 1;
        while (size > 0) {
            int half = size >> 1, middle = first + half;
            bool pr = cdf[middle] <= u;
            first = pr ? middle + 1 : first;
            size = pr ? size - (half + 1) : half;
        }
        (void)lo_;
        (void)hi_;
        int o = std::min(std::max(first - 1, 0), n - 1);
        *off = o;
        Float du = u - cdf[o];
        if (cdf[o + 1] - cdf[o] > 0) du /= cdf[o + 1] - cdf[o];
        *pdf = integral > 0 ? func[o] / integral : 0;
        return Lerp((o + du) / n, lo, hi);
    }
};

struct PixelFilter {
    int type = 0;  // 0 box, 1 gaussian, 2 mitchell, 3 sinc, 4 triangle
    Float rx = 0.5f, ry = 0.5f, a = 0, b = 0, expX = 0, expY = 0;
    int nx = 0, ny = 0;
    std::vector<Float> f;
    std::vector<Distribution1D> rows;
    Distribution1D marginal;

    static Float Gauss(Float x, Float sigma) {  // util/math.h:478, mu = 0
        return 1 / std::sqrt(2 * Pi * sigma * sigma) * FastExp(-Sqr(x - 0) / (2 * sigma * sigma));
    }
    static Float Mitchell(Float x, Float B, Float C) {
        x = std::abs(x);
        if (x <= 1) return ((12 - 9 * B - 6 * C) * x * x * x + (-18 + 12 * B + 6 * C) * x * x + (6 - 2 * B)) * (1.f / 6.f);
        if (x <= 2)
            return ((-B - 6 * C) * x * x * x + (6 * B + 30 * C) * x * x + (-12 * B - 48 * C) * x + (8 * B + 24 * C)) *
                   (1.f / 6.f);
        return 0;
    }
    static Float SinXOverX(Float x) { return 1 - x * x == 1 ? 1 : CRSin(x) / x; }
    static Float Lanczos(Float x, Float r, Float tau) {
        if (std::abs(x) > r) return 0;
        return SinXOverX(Pi * x) * SinXOverX(Pi * (x / tau));
    }
    Float Evaluate(Float x, Float y) const {
        switch (type) {
        case 1: return std::max<Float>(0, Gauss(x, a) - expX) * std::max<Float>(0, Gauss(y, a) - expY);
        case 2: return Mitchell(2 * x / rx, a, b) * Mitchell(2 * y / ry, a, b);
        case 3: return Lanczos(x, rx, a) * Lanczos(y, ry, a);
        case 4: return std::max<Float>(0, rx - std::abs(x)) * std::max<Float>(0, ry - std::abs(y));
        default: return (std::abs(x) <= rx && std::abs(y) <= ry) ? 1 : 0;
        }
    }
    void Init(int t, Float rx_, Float ry_, Float a_, Float b_) {
        type = t;
        rx = rx_;
        ry = ry_;
        a = a_;
        b = b_;
        if (type == 1) {
            expX = Gauss(rx, a);
            expY = Gauss(ry, a);
        }
        if (type == 0 || type == 4) return;
        nx = int(32 * rx);
        ny = int(32 * ry);
        f.resize((size_t)nx * ny);
        for (int y = 0; y < ny; ++y)
            for (int x = 0; x < nx; ++x)
                f[(size_t)y * nx + x] = Evaluate(Lerp((x + 0.5f) / nx, -rx, rx), Lerp((y + 0.5f) / ny, -ry, ry));
        rows.resize(ny);
        std::vector<Float> m(ny);
        for (int y = 0; y < ny; ++y) {
            rows[y].Init(&f[(size_t)y * nx], nx, -rx, rx);
            m[y] = rows[y].integral;
        }
        marginal.Init(m.data(), ny, -ry, ry);
    }
    static Float Tent(Float u, Float r) {  // SampleTent (util/sampling.h:196-201)
        // SampleDiscrete({0.5, 0.5}, u, nullptr, &u)
        Float sum = 0.5f + 0.5f, up = u * sum;
        if (up == sum) up = NextFloatDown(up);
        int k = (0 + 0.5f <= up) ? 1 : 0;
        Float base = k ? 0.5f : 0.f;
        u = std::min((up - base) / 0.5f, OneMinusEpsilon);
        if (k == 0) return -r + r * SampleLinear(u, 0, 1);
        return r * SampleLinear(u, 1, 0);
    }
    void Sample(Float u0, Float u1, Float *px, Float *py, Float *w) const {
        if (type == 0) {
            *px = Lerp(u0, -rx, rx);
            *py = Lerp(u1, -ry, ry);
            *w = 1;
            return;
        }
        if (type == 4) {
            *px = Tent(u0, rx);
            *py = Tent(u1, ry);
            *w = 1;
            return;
        }
        Float p1, p0;
        int iy, ix;
        *py = marginal.Sample(u1, &p1, &iy);
        *px = rows[iy].Sample(u0, &p0, &ix);
        *w = f[(size_t)iy * nx + ix] / (p0 * p1);
    }
};

// ---------------------------------------------------------------- textures
// Image textures and texture expressions, restated independently of the product:
//   Image::GeneratePyramid / FloatResizeUp / ResampleWeights   util/image.cpp:208-383
//   ColorEncoding FromLinear / ToLinear, LinearToSRGB           util/color.h:420-538, color.cpp
//   Half(float) round to nearest even                           util/float.h:419-470
//   Image::GetChannel / BilerpChannel, RemapPixelCoords          util/image.h:96-146, 255-292
//   MIPMap::Filter / Bilerp / Texel / EWA                        util/mipmap.cpp:208-375
//   textures and mappings                                        textures.h:86-1175, textures.cpp
//   RGBToSpectrumTable::operator(), RGB*Spectrum                 util/color.cpp:36-75, spectrum.cpp
//   CameraBase::FindMinimumDifferentials / Approximate_dp_dxy    cameras.cpp:170-216, cameras.h:167
//   the (u,v) derivatives of the material stage                  wavefront/surfscatter.cpp:74-104
// The oracle builds its own MIPMap pyramid from the decoded image files the loader hands over
// (pbrt_scene_flat image_raw_*) and evaluates each texture tree recursively with full
// SampledSpectrum arithmetic, as pbrt's UniversalTextureEvaluator does.  The only tables it
// shares with the product are reference data: the 8-bit sRGB decode table (the literals of
// util/color.cpp), the EWA weight table (util/mipmap.cpp) and the rgb2spec_opt coefficient
// table (set through oracle_set_rgb_table).
static const float *g_rgbTable = nullptr;  // zNodes[64], then coefficients [3][64][64][64][3]
static const float *g_ewaLut = nullptr;    // MIPFilterLUT[128]

static uint16_t OFloatToHalf(float ff) {
    uint32_t f = FloatToBits(ff);
    const uint32_t sign = f & 0x80000000u;
    f ^= sign;
    uint16_t o;
    if (f >= (uint32_t)(127 + 16) << 23) {
        o = (f > (255u << 23)) ? 0x7e00 : 0x7c00;
    } else if (f < (113u << 23)) {
        const uint32_t magic = ((127 - 15) + (23 - 10) + 1) << 23;
        float v = BitsToFloat(f) + BitsToFloat(magic);
        o = (uint16_t)(FloatToBits(v) - magic);
    } else {
        const uint32_t mantOdd = (f >> 13) & 1;
        f += ((uint32_t)(15 - 127) << 23) + 0xfff;
        f += mantOdd;
        o = (uint16_t)(f >> 13);
    }
    return (uint16_t)(o | (sign >> 16));
}
static float OHalfToFloat(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    float v;
    if (e == 0) v = std::ldexp((float)m, -24);
    else if (e == 31) v = m ? std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::infinity();
    else v = std::ldexp((float)(m | 1024), e - 25);
    return (h & 0x8000) ? -v : v;
}
static Float OEvalPoly(Float t, const Float *c, int n) {
    Float r = c[n - 1];
    for (int i = n - 2; i >= 0; --i) r = std::fma(t, r, c[i]);
    return r;
}
static Float OLinearToSRGB(Float value) {
    if (value <= 0.0031308f) return 12.92f * value;
    const Float sq = SafeSqrt(value);
    static const Float P[6] = {-0.0016829072605308378f, 0.03453868659826638f, 0.7642611304733891f,
                               2.0041169284241644f, 0.7551545191665577f, -0.016202083165206348f};
    static const Float Q[6] = {4.178892964897981e-7f, -0.00004375359692957097f, 0.03467195408529984f,
                               0.6085338522168684f, 1.8970238036421054f, 1.f};
    return OEvalPoly(sq, P, 6) / OEvalPoly(sq, Q, 6) * value;
}

struct OEncoding {
    int kind = 1;  // 0 linear, 1 sRGB, 2 gamma
    Float gamma = 1;
    const float *srgbLut = nullptr;
    Float apply[256], inverse[1024];
    void Init(int k, Float g, const float *lut) {
        kind = k;
        gamma = g;
        srgbLut = lut;
        if (kind == 2) {
            for (int i = 0; i < 256; ++i) apply[i] = std::pow(Float(i) / 255.f, gamma);
            for (int i = 0; i < 1024; ++i) inverse[i] = Clamp(255.f * std::pow(Float(i) / Float(1023), 1.f / gamma) + .5f, 0, 255);
        }
    }
    Float ToLinear(uint8_t v) const { return kind == 0 ? v / 255.f : (kind == 1 ? srgbLut[v] : apply[v]); }
    uint8_t FromLinear(Float v) const {
        if (kind == 0) return (uint8_t)Clamp(v * 255.f + 0.5f, 0, 255);
        if (kind == 1) {
            if (v <= 0) return 0;
            if (v >= 1) return 255;
            return (uint8_t)Clamp(std::round(255.f * OLinearToSRGB(v)), 0, 255);
        }
        return (uint8_t)inverse[(size_t)Clamp(v * Float(1023), 0, 1023)];
    }
};

struct OImage {
    int format = 0, nc = 0, wrap = 0, nLevels = 0;
    OEncoding enc;
    std::vector<int> w, h;
    std::vector<std::vector<uint8_t>> l8;
    std::vector<std::vector<uint16_t>> l16;
    std::vector<std::vector<float>> l32;

    static bool Remap(int *px, int *py, int W, int H, int wrap) {
        int x = *px, y = *py;
        if (wrap == 3) {
            if (x < 0) { x = -x; y = H - 1 - y; }
            else if (x >= W) { x = 2 * W - 1 - x; y = H - 1 - y; }
            if (y < 0) { x = W - 1 - x; y = -y; }
            else if (y >= H) { x = W - 1 - x; y = 2 * H - 1 - y; }
            if (W == 1) x = 0;
            if (H == 1) y = 0;
        } else {
            int *c[2] = {&x, &y};
            const int res[2] = {W, H};
            for (int k = 0; k < 2; ++k) {
                if (*c[k] >= 0 && *c[k] < res[k]) continue;
                if (wrap == 0) { int r = *c[k] % res[k]; *c[k] = r < 0 ? r + res[k] : r; }
                else if (wrap == 2) *c[k] = Clamp(*c[k], 0, res[k] - 1);
                else return false;
            }
        }
        *px = x;
        *py = y;
        return true;
    }
    Float Get(int level, int x, int y, int c) const {
        if (!Remap(&x, &y, w[level], h[level], wrap)) return 0;
        const size_t i = ((size_t)y * w[level] + x) * nc + c;
        if (format == 0) return enc.ToLinear(l8[level][i]);
        if (format == 1) return OHalfToFloat(l16[level][i]);
        return l32[level][i];
    }
    void Store(const std::vector<float> &f, int W, int H) {
        w.push_back(W);
        h.push_back(H);
        l8.emplace_back();
        l16.emplace_back();
        l32.emplace_back();
        if (format == 0) for (float v : f) l8.back().push_back(enc.FromLinear(v));
        else if (format == 1) for (float v : f) l16.back().push_back(OFloatToHalf(v));
        else l32.back() = f;
    }
    // Image::GeneratePyramid
    void Build(const uint8_t *raw, int W, int H) {
        std::vector<float> f((size_t)W * H * nc);
        for (size_t i = 0; i < f.size(); ++i) {
            if (format == 0) f[i] = enc.ToLinear(raw[i]);
            else if (format == 1) { uint16_t hv; std::memcpy(&hv, raw + 2 * i, 2); f[i] = OHalfToFloat(hv); }
            else std::memcpy(&f[i], raw + 4 * i, 4);
        }
        auto pow2 = [](int v) { return v > 0 && !(v & (v - 1)); };
        auto up2 = [](int v) { int r = 1; while (r < v) r <<= 1; return r; };
        if (!pow2(W) || !pow2(H)) {
            const int nw = up2(W), nh = up2(H);
            f = ResizeUp(f, W, H, nw, nh);
            W = nw;
            H = nh;
        }
        int lv = 1, m = std::max(W, H);
        while (m > 1) { m >>= 1; ++lv; }
        nLevels = lv;
        for (int i = 0; i < nLevels - 1; ++i) {
            Store(f, W, H);
            const int nw = std::max(1, W / 2), nh = std::max(1, H / 2);
            std::vector<float> next((size_t)nw * nh * nc);
            for (int y = 0; y < nh; ++y)
                for (int x = 0; x < nw; ++x)
                    for (int c = 0; c < nc; ++c) {
                        const int x0 = 2 * x, y0 = 2 * y, x1 = W == 1 ? x0 : x0 + 1, y1 = H == 1 ? y0 : y0 + 1;
                        auto at = [&](int xx, int yy) { return f[((size_t)yy * W + xx) * nc + c]; };
                        next[((size_t)y * nw + x) * nc + c] = (at(x0, y0) + at(x1, y0) + at(x0, y1) + at(x1, y1)) / 4;
                    }
            f.swap(next);
            W = nw;
            H = nh;
        }
        Store(f, W, H);
    }
    static Float WSinc(Float x) {
        // WindowedSinc(x, 2, 2): SinXOverX(Pi x) * SinXOverX(Pi x / 2)
        if (std::abs(x) > 2) return 0;
        auto sxx = [](Float v) { return (1 - v * v == 1) ? Float(1) : std::sin(v) / v; };
        return sxx(Pi * x) * sxx(Pi * (x / 2));
    }
    std::vector<float> ResizeUp(const std::vector<float> &src, int W, int H, int nw, int nh) const {
        struct RW { int first; Float wt[4]; };
        auto weights = [](int oldRes, int newRes) {
            std::vector<RW> r(newRes);
            for (int i = 0; i < newRes; ++i) {
                Float center = (i + .5f) * oldRes / newRes;
                r[i].first = (int)std::floor((center - 2) + 0.5f);
                for (int j = 0; j < 4; ++j) r[i].wt[j] = WSinc(r[i].first + j + .5f - center);
                Float inv = 1 / (r[i].wt[0] + r[i].wt[1] + r[i].wt[2] + r[i].wt[3]);
                for (int j = 0; j < 4; ++j) r[i].wt[j] *= inv;
            }
            return r;
        };
        std::vector<RW> xw = weights(W, nw), yw = weights(H, nh);
        auto in = [&](int x, int y, int c) {
            Remap(&x, &y, W, H, wrap);
            return src[((size_t)y * W + x) * nc + c];
        };
        auto xpass = [&](int x, int y, int c) {
            const RW &r = xw[x];
            return r.wt[0] * in(r.first, y, c) + r.wt[1] * in(r.first + 1, y, c) + r.wt[2] * in(r.first + 2, y, c) +
                   r.wt[3] * in(r.first + 3, y, c);
        };
        std::vector<float> out((size_t)nw * nh * nc);
        for (int y = 0; y < nh; ++y)
            for (int x = 0; x < nw; ++x)
                for (int c = 0; c < nc; ++c) {
                    const RW &r = yw[y];
                    out[((size_t)y * nw + x) * nc + c] =
                        std::max<Float>(0, (r.wt[0] * xpass(x, r.first, c) + r.wt[1] * xpass(x, r.first + 1, c) +
                                            r.wt[2] * xpass(x, r.first + 2, c) + r.wt[3] * xpass(x, r.first + 3, c)));
                }
        return out;
    }
    // MIPMap::Bilerp / Texel for RGB (channels 0-2, or the single channel) and Float
    Float BilerpC(int level, Float s, Float t, int c) const {
        Float x = s * w[level] - 0.5f, y = t * h[level] - 0.5f;
        int xi = (int)std::floor(x), yi = (int)std::floor(y);
        Float dx = x - xi, dy = y - yi;
        return ((1 - dx) * (1 - dy) * Get(level, xi, yi, c) + dx * (1 - dy) * Get(level, xi + 1, yi, c) +
                (1 - dx) * dy * Get(level, xi, yi + 1, c) + dx * dy * Get(level, xi + 1, yi + 1, c));
    }
    void BilerpRGB(int level, Float s, Float t, Float *rgb) const {
        for (int c = 0; c < 3; ++c) rgb[c] = BilerpC(level, s, t, nc == 1 ? 0 : c);
    }
    Float BilerpF(int level, Float s, Float t) const {
        if (nc == 1) return BilerpC(level, s, t, 0);
        if (nc == 3) {
            Float sum = 0;
            for (int c = 0; c < 3; ++c) sum += BilerpC(level, s, t, c);
            return sum / 3;
        }
        return BilerpC(level, s, t, 3);
    }
    void TexelRGB(int level, int x, int y, Float *rgb) const {
        for (int c = 0; c < 3; ++c) rgb[c] = Get(level, x, y, nc == 1 ? 0 : c);
    }
    // MIPMap::Filter; nOut = 3 (RGB) or 1 (Float)
    void Filter(int filter, Float maxAniso, Float s, Float t, Float d0s, Float d0t, Float d1s, Float d1t, int nOut,
                Float *out) const {
        auto bil = [&](int level, Float *o) {
            if (nOut == 3) BilerpRGB(level, s, t, o);
            else o[0] = BilerpF(level, s, t);
        };
        auto texel = [&](int level, int x, int y, Float *o) {
            if (nOut == 3) TexelRGB(level, x, y, o);
            else o[0] = Get(level, x, y, 0);
        };
        const Float invLog2 = 1.442695040888963387004650940071f;
        if (filter != 3) {
            Float width = 2 * std::max({std::abs(d0s), std::abs(d0t), std::abs(d1s), std::abs(d1t)});
            Float level = nLevels - 1 + CRLog(std::max<Float>(width, 1e-8f)) * invLog2;
            if (level >= nLevels - 1) return texel(nLevels - 1, 0, 0, out);
            int iLevel = std::max(0, (int)std::floor(level));
            if (filter == 0)
                return texel(iLevel, (int)std::round(s * w[iLevel] - 0.5f), (int)std::round(t * h[iLevel] - 0.5f), out);
            if (filter == 1 || iLevel == 0) return bil(iLevel, out);
            Float a[3], b[3];
            bil(iLevel, a);
            bil(iLevel + 1, b);
            for (int k = 0; k < nOut; ++k) out[k] = Lerp(level - iLevel, a[k], b[k]);
            return;
        }
        if (Sqr(d0s) + Sqr(d0t) < Sqr(d1s) + Sqr(d1t)) {
            std::swap(d0s, d1s);
            std::swap(d0t, d1t);
        }
        Float longer = std::sqrt(Sqr(d0s) + Sqr(d0t)), shorter = std::sqrt(Sqr(d1s) + Sqr(d1t));
        if (shorter * maxAniso < longer && shorter > 0) {
            Float sc = longer / (shorter * maxAniso);
            d1s *= sc;
            d1t *= sc;
            shorter *= sc;
        }
        if (shorter == 0) return bil(0, out);
        Float lod = std::max<Float>(0, nLevels - 1 + CRLog(shorter) * invLog2);
        int ilod = (int)std::floor(lod);
        Float a[3], b[3];
        EWA(ilod, s, t, d0s, d0t, d1s, d1t, nOut, a);
        EWA(ilod + 1, s, t, d0s, d0t, d1s, d1t, nOut, b);
        for (int k = 0; k < nOut; ++k) out[k] = Lerp(lod - ilod, a[k], b[k]);
    }
    void EWA(int level, Float s, Float t, Float d0s, Float d0t, Float d1s, Float d1t, int nOut, Float *out) const {
        if (level >= nLevels) {
            if (nOut == 3) TexelRGB(nLevels - 1, 0, 0, out);
            else out[0] = Get(nLevels - 1, 0, 0, 0);
            return;
        }
        s = s * w[level] - 0.5f;
        t = t * h[level] - 0.5f;
        d0s *= w[level];
        d0t *= h[level];
        d1s *= w[level];
        d1t *= h[level];
        Float A = Sqr(d0t) + Sqr(d1t) + 1, B = -2 * (d0s * d0t + d1s * d1t), C = Sqr(d0s) + Sqr(d1s) + 1;
        Float invF = 1 / (A * C - Sqr(B) * 0.25f);
        A *= invF;
        B *= invF;
        C *= invF;
        Float det = -Sqr(B) + 4 * A * C, invDet = 1 / det;
        Float uSqrt = SafeSqrt(det * C), vSqrt = SafeSqrt(A * det);
        int s0 = (int)std::ceil(s - 2 * invDet * uSqrt), s1 = (int)std::floor(s + 2 * invDet * uSqrt);
        int t0 = (int)std::ceil(t - 2 * invDet * vSqrt), t1 = (int)std::floor(t + 2 * invDet * vSqrt);
        Float sum[3] = {0, 0, 0}, sumW = 0;
        for (int it = t0; it <= t1; ++it) {
            Float tt = it - t;
            for (int is = s0; is <= s1; ++is) {
                Float ss = is - s;
                Float r2 = A * Sqr(ss) + B * ss * tt + C * Sqr(tt);
                if (r2 < 1) {
                    int index = std::min<int>((int)(r2 * 128), 127);
                    Float wt = g_ewaLut[index], v[3];
                    if (nOut == 3) TexelRGB(level, is, it, v);
                    else v[0] = Get(level, is, it, 0);
                    for (int k = 0; k < nOut; ++k) sum[k] = sum[k] + wt * v[k];
                    sumW += wt;
                }
            }
        }
        for (int k = 0; k < nOut; ++k) out[k] = sum[k] / sumW;
    }
};

// RGBToSpectrumTable::operator() (util/color.cpp:36-75)
static void ORGBCoeffs(Float r, Float g, Float b, Float c[3]) {
    if (r == g && g == b) {
        c[0] = c[1] = 0;
        c[2] = (r - .5f) / std::sqrt(r * (1 - r));
        return;
    }
    const Float rgb[3] = {r, g, b};
    const int res = 64;
    const float *zn = g_rgbTable, *data = g_rgbTable + 64;
    int maxc = (r > g) ? ((r > b) ? 0 : 2) : ((g > b) ? 1 : 2);
    Float z = rgb[maxc], x = rgb[(maxc + 1) % 3] * (res - 1) / z, y = rgb[(maxc + 2) % 3] * (res - 1) / z;
    int xi = std::min((int)x, res - 2), yi = std::min((int)y, res - 2);
    int zi = 0;
    while (zi < res - 2 && zn[zi + 1] < z) ++zi;  // FindInterval over the monotone z nodes
    Float dx = x - xi, dy = y - yi, dz = (z - zn[zi]) / (zn[zi + 1] - zn[zi]);
    for (int i = 0; i < 3; ++i) {
        auto co = [&](int a, int bb, int cc) {
            return data[((((size_t)maxc * res + (zi + cc)) * res + (yi + bb)) * res + (xi + a)) * 3 + i];
        };
        c[i] = Lerp(dz, Lerp(dy, Lerp(dx, co(0, 0, 0), co(1, 0, 0)), Lerp(dx, co(0, 1, 0), co(1, 1, 0))),
                    Lerp(dy, Lerp(dx, co(0, 0, 1), co(1, 0, 1)), Lerp(dx, co(0, 1, 1), co(1, 1, 1))));
    }
}

// ImageInfiniteLight (lights.h:557-641, lights.cpp:1038-1083) over the flat view's linear
// R, G, B pixels: compensated PiecewiseConstant2D, equal-area octahedral mapping
// (util/math.cpp:292-361), nearest-pixel RGBIlluminantSpectrum radiance
struct OEnvLight {
    int n = 0;
    const float *rgb = nullptr;
    const float *m = nullptr, *mi = nullptr;  // renderFromLight, its inverse (3x3 row major)
    std::vector<Distribution1D> rows;
    Distribution1D marginal;
    void Init(const pbrt_scene_flat *f, int k) {
        n = f->env_info[4 * k];
        rgb = f->env_rgb + 3 * f->env_offset[k];
        m = f->env_xform + 18 * k;
        mi = m + 9;
        std::vector<Float> d((size_t)n * n);
        for (size_t p = 0; p < d.size(); ++p) {
            Float sum = 0;
            for (int c = 0; c < 3; ++c) sum += rgb[3 * p + c];
            d[p] = sum / 3;  // ImageChannelValues::Average
        }
        double avg = 0.;
        for (Float v : d) avg += v;
        avg /= d.size();
        for (Float &v : d) v = std::max<Float>(v - avg, 0);
        if (std::all_of(d.begin(), d.end(), [](Float v) { return v == 0; })) std::fill(d.begin(), d.end(), Float(1));
        rows.assign(n, Distribution1D());
        std::vector<Float> mf(n);
        for (int v = 0; v < n; ++v) {
            rows[v].Init(&d[(size_t)v * n], n, 0, 1);
            mf[v] = rows[v].integral;
        }
        marginal.Init(mf.data(), n, 0, 1);
        if (f->env_info[4 * k + 1]) InitPortal(f, k);
    }
    static Vec Mul(const float *a, Vec v) {
        return Vec(a[0] * v.x + a[1] * v.y + a[2] * v.z, a[3] * v.x + a[4] * v.y + a[5] * v.z,
                   a[6] * v.x + a[7] * v.y + a[8] * v.z);
    }
    static Vec SquareToSphere(Float px, Float py) {
        Float u = 2 * px - 1, v = 2 * py - 1, up = std::abs(u), vp = std::abs(v);
        Float sd = 1 - (up + vp), dd = std::abs(sd), r = 1 - dd;
        Float phi = (r == 0 ? 1 : (vp - up) / r + 1) * Pi / 4;
        Float z = std::copysign(1 - Sqr(r), sd);
        Float cp = std::copysign(CRCos(phi), u), sp = std::copysign(CRSin(phi), v);
        return Vec(cp * r * SafeSqrt(2 - Sqr(r)), sp * r * SafeSqrt(2 - Sqr(r)), z);
    }
    static void SphereToSquare(Vec d, Float *uo, Float *vo) {
        Float x = std::abs(d.x), y = std::abs(d.y), z = std::abs(d.z);
        Float r = SafeSqrt(1 - z);
        Float a = std::max(x, y), b = std::min(x, y);
        b = a == 0 ? 0 : b / a;
        // EvaluatePolynomial(b, t1..t7) = FMA(b, EvaluatePolynomial(b, t2..t7), t1)
        static const Float t[7] = {0.406758566246788489601959989e-5f, 0.636226545274016134946890922156f,
                                   0.61572017898280213493197203466e-2f, -0.247333733281268944196501420480f,
                                   0.881770664775316294736387951347e-1f, 0.419038818029165735901852432784e-1f,
                                   -0.251390972343483509333252996350e-1f};
        Float phi = t[6];
        for (int i = 5; i >= 0; --i) phi = std::fma(b, phi, t[i]);
        if (x < y) phi = 1 - phi;
        Float v = phi * r, u = r - v;
        if (d.z < 0) {
            std::swap(u, v);
            u = 1 - u;
            v = 1 - v;
        }
        u = std::copysign(u, d.x);
        v = std::copysign(v, d.y);
        *uo = 0.5f * (u + 1);
        *vo = 0.5f * (v + 1);
    }
    // Image::LookupNearestChannel with WrapMode::OctahedralSphere, then RGBIlluminantSpectrum
    // of ClampZero(rgb) (util/spectrum.cpp:246-251) times the light scale
    Spectrum Le(Float u, Float v, const Wavelengths &lambda, const float *illum, Float lightScale) const {
        int x = (int)(u * n), y = (int)(v * n);
        if (x < 0) x = -x, y = n - 1 - y;
        else if (x >= n) x = 2 * n - 1 - x, y = n - 1 - y;
        if (y < 0) x = n - 1 - x, y = -y;
        else if (y >= n) x = n - 1 - x, y = 2 * n - 1 - y;
        if (n == 1) x = y = 0;
        const float *px = rgb + 3 * ((size_t)y * n + x);
        Float c3[3] = {std::max<Float>(0, px[0]), std::max<Float>(0, px[1]), std::max<Float>(0, px[2])};
        Float mx = std::max({c3[0], c3[1], c3[2]}), scale = 2 * mx, co[3];
        if (scale) ORGBCoeffs(c3[0] / scale, c3[1] / scale, c3[2] / scale, co);
        else ORGBCoeffs(0, 0, 0, co);
        Spectrum s;
        for (int i = 0; i < NS; ++i) s[i] = scale * Sigmoid(co[0], co[1], co[2], lambda.lambda[i]);
        return (s * SampleDense(illum, lambda)) * lightScale;
    }
    // compensatedDistribution.Sample / PDF (util/sampling.h:760-779)
    bool Sample(Float u0, Float u1, Float *uo, Float *vo, Float *mapPDF) const {
        Float p1, p0;
        int iv, iu;
        *vo = marginal.Sample(u1, &p1, &iv);
        *uo = rows[iv].Sample(u0, &p0, &iu);
        *mapPDF = p0 * p1;
        return *mapPDF != 0;
    }
    Float PDF(Float u, Float v) const {
        int iu = std::clamp((int)(u * n), 0, n - 1), iv = std::clamp((int)(v * n), 0, n - 1);
        return rows[iv].func[iu] / marginal.integral;
    }

    // ---- PortalImageInfiniteLight (lights.h:644-744, lights.cpp:1140-1297)
    bool portal = false;
    Vec pc[4], fx, fy, fz;    // corners (render space), portalFrame = Frame::FromXY(p03, p01)
    std::vector<float> prgb;  // the rectified image [n][n][3]
    std::vector<Float> pfunc; // WindowedPiecewiseConstant2D's function
    std::vector<double> psat; // ... and its SummedAreaTable
    bool ImageFromRender(Vec wr, Float *u, Float *v, Float *duv_dw) const {
        Vec w(Dot(wr, fx), Dot(wr, fy), Dot(wr, fz));
        if (w.z <= 0) return false;
        if (duv_dw) *duv_dw = Sqr(Pi) * (1 - Sqr(w.x)) * (1 - Sqr(w.y)) / w.z;
        Float alpha = CRATan2(w.x, w.z), beta = CRATan2(w.y, w.z);
        *u = Clamp((alpha + Pi / 2) / Pi, 0, 1);
        *v = Clamp((beta + Pi / 2) / Pi, 0, 1);
        return true;
    }
    Vec RenderFromImage(Float u, Float v, Float *duv_dw) const {
        Float alpha = -Pi / 2 + u * Pi, beta = -Pi / 2 + v * Pi;
        Float x = CRTan(alpha), y = CRTan(beta);
        Vec w = Normalize(Vec(x, y, 1));
        if (duv_dw) *duv_dw = Sqr(Pi) * (1 - Sqr(w.x)) * (1 - Sqr(w.y)) / w.z;
        return fx * w.x + fy * w.y + fz * w.z;
    }
    bool ImageBounds(Vec p, Float b[4]) const {
        Float u0, v0, u1, v1;
        if (!ImageFromRender(Normalize(pc[0] - p), &u0, &v0, nullptr)) return false;
        if (!ImageFromRender(Normalize(pc[2] - p), &u1, &v1, nullptr)) return false;
        b[0] = std::min(u0, u1), b[1] = std::min(v0, v1), b[2] = std::max(u0, u1), b[3] = std::max(v0, v1);
        return true;
    }
    Float SatInt(int x, int y) const {
        if (x == 0 || y == 0) return 0;
        x = std::min(x - 1, n - 1);
        y = std::min(y - 1, n - 1);
        return (Float)psat[(size_t)y * n + x];
    }
    Float SatLookup(Float x, Float y) const {
        x *= n;
        y *= n;
        int x0 = (int)x, y0 = (int)y;
        Float v00 = SatInt(x0, y0), v10 = SatInt(x0 + 1, y0), v01 = SatInt(x0, y0 + 1), v11 = SatInt(x0 + 1, y0 + 1);
        Float dx = x - int(x), dy = y - int(y);
        return (1 - dx) * (1 - dy) * v00 + (1 - dx) * dy * v01 + dx * (1 - dy) * v10 + dx * dy * v11;
    }
    Float Integral(Float x0, Float y0, Float x1, Float y1) const {
        double s = (((double)SatLookup(x1, y1) - (double)SatLookup(x0, y1)) +
                    ((double)SatLookup(x0, y0) - (double)SatLookup(x1, y0)));
        return std::max<Float>(s / (n * n), 0);
    }
    Float FuncEval(Float u, Float v) const {
        return pfunc[(size_t)std::min<int>(v * n, n - 1) * n + std::min<int>(u * n, n - 1)];
    }
    // SampleBisection (util/sampling.h:956-972), capped at 128 halvings as the product's
    template <typename CDF>
    Float Bisect(CDF P, Float u, Float mn, Float mx) const {
        for (int it = 0; it < 128 && std::ceil(n * mx) - std::floor(n * mn) > 1; ++it) {
            Float mid = (mn + mx) / 2;
            if (P(mid) > u) mx = mid;
            else mn = mid;
        }
        Float t = (u - P(mn)) / (P(mx) - P(mn));
        return Clamp(Lerp(t, mn, mx), mn, mx);
    }
    bool WindowedSample(Float u0, Float u1, const Float b[4], Float *px, Float *py, Float *pdf) const {
        if (Integral(b[0], b[1], b[2], b[3]) == 0) return false;
        Float bInt = Integral(b[0], b[1], b[2], b[3]);
        Float x = Bisect([&](Float t) { return Integral(b[0], b[1], t, b[3]) / bInt; }, u0, b[0], b[2]);
        Float c0 = std::floor(x * n) / n, c1 = std::ceil(x * n) / n;
        if (c0 == c1) c1 += 1.f / n;
        if (Integral(c0, b[1], c1, b[3]) == 0) return false;
        Float cInt = Integral(c0, b[1], c1, b[3]);
        Float y = Bisect([&](Float t) { return Integral(c0, b[1], c1, t) / cInt; }, u1, b[1], b[3]);
        *px = x;
        *py = y;
        *pdf = FuncEval(x, y) / bInt;
        return true;
    }
    // ImageLookup: LookupNearestChannel (clamp wrap) of the rectified image, RGBIlluminantSpectrum
    Spectrum RectLe(Float u, Float v, const Wavelengths &lambda, const float *illum, Float lightScale) const {
        int x = std::clamp((int)(u * n), 0, n - 1), y = std::clamp((int)(v * n), 0, n - 1);
        const float *px = prgb.data() + 3 * ((size_t)y * n + x);
        Float c3[3] = {std::max<Float>(0, px[0]), std::max<Float>(0, px[1]), std::max<Float>(0, px[2])};
        Float mx = std::max({c3[0], c3[1], c3[2]}), scale = 2 * mx, co[3];
        if (scale) ORGBCoeffs(c3[0] / scale, c3[1] / scale, c3[2] / scale, co);
        else ORGBCoeffs(0, 0, 0, co);
        Spectrum s;
        for (int i = 0; i < NS; ++i) s[i] = scale * Sigmoid(co[0], co[1], co[2], lambda.lambda[i]);
        return (s * SampleDense(illum, lambda)) * lightScale;
    }
    // the rectification, sampling distribution and SAT (lights.cpp:1164-1211); Init runs it in
    // the host's libm mode
    void InitPortal(const pbrt_scene_flat *f, int k) {
        portal = true;
        const float *c = f->env_portal + 12 * k;
        for (int i = 0; i < 4; ++i) pc[i] = Vec(c[3 * i], c[3 * i + 1], c[3 * i + 2]);
        Vec p01 = Normalize(pc[1] - pc[0]), p03 = Normalize(pc[3] - pc[0]);
        fx = p03;
        fy = p01;
        fz = Cross(p03, p01);
        prgb.assign((size_t)n * n * 3, 0.f);
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                Vec w = RenderFromImage((x + 0.5f) / n, (y + 0.5f) / n, nullptr);
                w = Normalize(Mul(mi, w));
                Float ue, ve;
                SphereToSquare(w, &ue, &ve);
                // Image::BilerpChannel with WrapMode::OctahedralSphere
                Float fxp = ue * n - 0.5f, fyp = ve * n - 0.5f;
                int xi = (int)std::floor(fxp), yi = (int)std::floor(fyp);
                Float dx = fxp - xi, dy = fyp - yi;
                auto get = [&](int px, int py, int ch) {
                    if (px < 0) px = -px, py = n - 1 - py;
                    else if (px >= n) px = 2 * n - 1 - px, py = n - 1 - py;
                    if (py < 0) px = n - 1 - px, py = -py;
                    else if (py >= n) px = n - 1 - px, py = 2 * n - 1 - py;
                    if (n == 1) px = py = 0;
                    return rgb[3 * ((size_t)py * n + px) + ch];
                };
                for (int ch = 0; ch < 3; ++ch)
                    prgb[3 * ((size_t)y * n + x) + ch] =
                        ((1 - dx) * (1 - dy) * get(xi, yi, ch) + dx * (1 - dy) * get(xi + 1, yi, ch) +
                         (1 - dx) * dy * get(xi, yi + 1, ch) + dx * dy * get(xi + 1, yi + 1, ch));
            }
        pfunc.assign((size_t)n * n, 0);
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                Float sum = 0;
                for (int ch = 0; ch < 3; ++ch) sum += prgb[3 * ((size_t)y * n + x) + ch];
                Float d;
                (void)RenderFromImage((x + .5f) / n, (y + .5f) / n, &d);
                pfunc[(size_t)y * n + x] = sum / 3 * d;
            }
        psat.assign((size_t)n * n, 0.);
        auto S = [&](int x, int y) -> double & { return psat[(size_t)y * n + x]; };
        auto F = [&](int x, int y) { return pfunc[(size_t)y * n + x]; };
        S(0, 0) = F(0, 0);
        for (int x = 1; x < n; ++x) S(x, 0) = F(x, 0) + S(x - 1, 0);
        for (int y = 1; y < n; ++y) S(0, y) = F(0, y) + S(0, y - 1);
        for (int y = 1; y < n; ++y)
            for (int x = 1; x < n; ++x) S(x, y) = (F(x, y) + S(x - 1, y) + S(x, y - 1) - S(x - 1, y - 1));
    }

    // Light::SampleLi for either kind from the reference point p: direction, solid-angle pdf
    // (mapPDF / (4 pi) for an ImageInfiniteLight) and radiance; false for {} or pdf 0
    bool SampleLi(Vec p, Float u0, Float u1, const Wavelengths &lambda, const float *illum, Float scale, Vec *wi,
                  Float *pdf, Spectrum *Le) const {
        if (portal) {
            Float b[4], uu, vv, mapPDF, duv_dw;
            if (!ImageBounds(p, b) || !WindowedSample(u0, u1, b, &uu, &vv, &mapPDF)) return false;
            *wi = RenderFromImage(uu, vv, &duv_dw);
            if (duv_dw == 0) return false;
            *pdf = mapPDF / duv_dw;
            *Le = RectLe(uu, vv, lambda, illum, scale);
            return *pdf != 0;
        }
        Float eu, ev, emap;
        if (!Sample(u0, u1, &eu, &ev, &emap)) return false;
        *wi = Mul(m, SquareToSphere(eu, ev));
        *pdf = emap / (4 * Pi);
        *Le = this->Le(eu, ev, lambda, illum, scale);
        return true;
    }
    // Light::Le(ray) of an escaped ray (origin o, direction d)
    Spectrum LeRay(Vec o, Vec d, const Wavelengths &lambda, const float *illum, Float scale) const {
        if (portal) {
            Float u, v, b[4];
            if (!ImageFromRender(Normalize(d), &u, &v, nullptr) || !ImageBounds(o, b) || !(u >= b[0] && u <= b[2] && v >= b[1] && v <= b[3]))
                return Spectrum(0.f);
            return RectLe(u, v, lambda, illum, scale);
        }
        Float u, v;
        SphereToSquare(Normalize(Mul(mi, d)), &u, &v);
        return Le(u, v, lambda, illum, scale);
    }
    // Light::PDF_Li(ctx, w, allowIncompletePDF) from the previous vertex p
    Float PdfLi(Vec p, Vec w) const {
        if (portal) {
            Float u, v, duv_dw, b[4];
            if (!ImageFromRender(w, &u, &v, &duv_dw) || duv_dw == 0) return 0;
            if (!ImageBounds(p, b)) return 0;
            Float fi = Integral(b[0], b[1], b[2], b[3]);
            if (fi == 0) return 0;
            return (FuncEval(u, v) / fi) / duv_dw;
        }
        Float u, v;
        SphereToSquare(Mul(mi, w), &u, &v);
        return PDF(u, v) / (4 * Pi);
    }
};

struct OTexCtx {
    Vec p, n;
    Float u = 0, v = 0, dudx = 0, dudy = 0, dvdx = 0, dvdy = 0;
};

// ---------------------------------------------------------------- procedural textures
// FBm / Turbulence (util/noise.cpp:114-152), WindyTexture (textures.h:1125-1130),
// InsidePolkaDot (textures.cpp:287-303), MarbleTexture's RGB (textures.cpp:524-549 with
// EvaluateCubicBezier, util/splines.h:18-28) over Perlin's Noise (Media::NoiseAt).
namespace proc {
static Float Octaves(Vec dpdx, Vec dpdy, int maxOct) {
    const Float len2 = std::max(LengthSquared(dpdx), LengthSquared(dpdy));
    const Float invLog2 = 1.442695040888963387004650940071;
    return Clamp(-1 - (CRLog(len2) * invLog2) / 2, 0, (Float)maxOct);
}
static Float SmoothStep(Float x, Float a, Float b) {
    if (a == b) return x < a ? 0 : 1;
    const Float t = Clamp((x - a) / (b - a), 0, 1);
    return t * t * (3 - 2 * t);
}
static Float FBm(const float *perm, Vec p, Vec dpdx, Vec dpdy, Float omega, int maxOct) {
    const Float n = Octaves(dpdx, dpdy, maxOct);
    const int nInt = (int)std::floor(n);
    Float sum = 0, lambda = 1, o = 1;
    for (int i = 0; i < nInt; ++i) {
        sum += o * Media::NoiseAt(perm, lambda * p.x, lambda * p.y, lambda * p.z);
        lambda *= 1.99f;
        o *= omega;
    }
    sum += o * SmoothStep(n - nInt, .3f, .7f) * Media::NoiseAt(perm, lambda * p.x, lambda * p.y, lambda * p.z);
    return sum;
}
static Float Turbulence(const float *perm, Vec p, Vec dpdx, Vec dpdy, Float omega, int maxOct) {
    const Float n = Octaves(dpdx, dpdy, maxOct);
    const int nInt = (int)std::floor(n);
    Float sum = 0, lambda = 1, o = 1;
    for (int i = 0; i < nInt; ++i) {
        sum += o * std::abs(Media::NoiseAt(perm, lambda * p.x, lambda * p.y, lambda * p.z));
        lambda *= 1.99f;
        o *= omega;
    }
    sum += o * Lerp(SmoothStep(n - nInt, .3f, .7f), 0.2f, std::abs(Media::NoiseAt(perm, lambda * p.x, lambda * p.y, lambda * p.z)));
    for (int i = nInt; i < maxOct; ++i) {
        sum += o * 0.2f;
        o *= omega;
    }
    return sum;
}
static Float Windy(const float *perm, Vec p, Vec dpdx, Vec dpdy) {
    return std::abs(FBm(perm, p * .1f, dpdx * .1f, dpdy * .1f, .5f, 3)) * FBm(perm, p, dpdx, dpdy, .5f, 6);
}
static bool PolkaDot(const float *perm, Float s, Float t) {
    const int sc = (int)std::floor(s + .5f), tc = (int)std::floor(t + .5f);
    if (!(Media::NoiseAt(perm, sc + .5f, tc + .5f, .5f) > 0)) return false;
    const Float r = .35f, shift = .5f - r;
    const Float cs = sc + shift * Media::NoiseAt(perm, sc + 1.5f, tc + 2.8f, .5f);
    const Float ct = tc + shift * Media::NoiseAt(perm, sc + 4.5f, tc + 9.8f, .5f);
    return Sqr(s - cs) + Sqr(t - ct) < Sqr(r);
}
static void Marble(const float *perm, Vec p, Vec dpdx, Vec dpdy, int oct, Float omega, Float scale, Float variation,
                   Float rgb[3]) {
    static const Float col[9][3] = {{.58f, .58f, .6f}, {.58f, .58f, .6f}, {.58f, .58f, .6f}, {.5f, .5f, .5f},  {.6f, .59f, .58f},
                                    {.58f, .58f, .6f}, {.58f, .58f, .6f}, {.2f, .2f, .33f},  {.58f, .58f, .6f}};
    p = p * scale;
    const Float m = p.y + variation * FBm(perm, p, dpdx * scale, dpdy * scale, omega, oct);
    Float t = .5f + .5f * CRSin(m);
    const int first = std::min((int)std::floor(t * 6), 5);
    t = t * 6 - first;
    for (int c = 0; c < 3; ++c) {
        Float a[3], b[2];
        for (int k = 0; k < 3; ++k) a[k] = Lerp(t, col[first + k][c], col[first + k + 1][c]);
        for (int k = 0; k < 2; ++k) b[k] = Lerp(t, a[k], a[k + 1]);
        rgb[c] = 1.5f * Lerp(t, b[0], b[1]);
    }
}
}  // namespace proc

struct OTextures {
    const pbrt_scene_flat *f = nullptr;
    std::vector<OImage> images;
    // camera differentials (own FindMinimumDifferentials) and CameraFromRender
    Vec minPosDx, minPosDy, minDirDx, minDirDy;
    Float sppScale = 1;
    int n = 0;

    void Init(const pbrt_scene_flat *flat, int spp, int xres, int yres) {
        f = flat;
        fullRes[0] = xres;
        fullRes[1] = yres;
        n = flat->n_tex_nodes;
        if (!n && !flat->n_images) return;  // normal maps are images without a texture node
        sppScale = (flat->options & 1) ? 1.f : std::max<Float>(.125f, 1 / std::sqrt((Float)spp));
        images.resize(flat->n_images);
        for (int i = 0; i < flat->n_images; ++i) {
            const int32_t *ri = flat->image_raw_info + 8 * i;
            const int32_t *ii = flat->image_info + 8 * i;
            OImage &im = images[i];
            im.format = ri[2];
            im.nc = ri[3];
            im.wrap = ii[3];
            im.enc.Init(ri[4], flat->image_raw_gamma[i], flat->image_luts + 256 * i);
            im.Build(flat->image_raw_data + flat->image_raw_offset[i], ri[0], ri[1]);
        }
        FindMinimumDifferentials();
    }
    const int32_t *Info(int node) const { return f->tex_node_info + 8 * node; }
    // PointTransformMapping (textures.h:229-246): textureFromRender (params [0..11]) of a point / vector
    static Vec P3(const float *q, Vec p) {
        return Vec(q[0] * p.x + q[1] * p.y + q[2] * p.z + q[3], q[4] * p.x + q[5] * p.y + q[6] * p.z + q[7],
                   q[8] * p.x + q[9] * p.y + q[10] * p.z + q[11]);
    }
    static Vec V3x(const float *q, Vec v) {
        return Vec(q[0] * v.x + q[1] * v.y + q[2] * v.z, q[4] * v.x + q[5] * v.y + q[6] * v.z, q[8] * v.x + q[9] * v.y + q[10] * v.z);
    }
    const float *Par(int node) const { return f->tex_node_params + 28 * node; }
    const float *Spec(int node, int k) const { return f->tex_node_spec + 32 * node + 8 * k; }

    // PerspectiveCamera::GenerateRayDifferential (cameras.cpp:458-520) + RenderFromCamera, then
    // CameraBase::FindMinimumDifferentials (cameras.cpp:170-216)
    static Vec XP(const float *m, Vec p) {
        Float x = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], y = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
        Float z = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11], w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
        return w == 1 ? Vec(x, y, z) : Vec(x, y, z) / w;
    }
    static Vec XV(const float *m, Vec v) {
        return Vec(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z, m[8] * v.x + m[9] * v.y + m[10] * v.z);
    }
    Vec CameraFromRenderV(Vec v) const {
        const float *c = f->camera_from_render;
        return Vec(c[0] * v.x + c[1] * v.y + c[2] * v.z, c[4] * v.x + c[5] * v.y + c[6] * v.z, c[8] * v.x + c[9] * v.y + c[10] * v.z);
    }
    void FindMinimumDifferentials() {
        const float *cfr = f->camera_from_raster, *rfc = f->render_from_camera;
        const Vec dxCam = XP(cfr, Vec(1, 0, 0)) - XP(cfr, Vec(0, 0, 0)), dyCam = XP(cfr, Vec(0, 1, 0)) - XP(cfr, Vec(0, 0, 0));
        const Float inf = Infinity;
        minPosDx = minPosDy = minDirDx = minDirDy = Vec(inf, inf, inf);
        // the film's full resolution: camera_from_raster maps raster (xres, yres) corners
        const int xres = fullRes[0], yres = fullRes[1];
        for (int i = 0; i < 512; ++i) {
            Vec pCam = XP(cfr, Vec(Float(i) / 511 * xres, Float(i) / 511 * yres, 0));
            Vec d = Normalize(pCam), o(0, 0, 0), rxd, ryd;
            if (f->lens_radius > 0) {
                Float ft = f->focal_distance / d.z;
                d = Normalize((o + d * ft) - o);
                Vec dx = Normalize(pCam + dxCam), dy = Normalize(pCam + dyCam);
                rxd = Normalize((Vec(0, 0, 0) + (f->focal_distance / dx.z) * dx) - o);
                ryd = Normalize((Vec(0, 0, 0) + (f->focal_distance / dy.z) * dy) - o);
            } else {
                rxd = Normalize(pCam + dxCam);
                ryd = Normalize(pCam + dyCam);
            }
            // Transform::operator()(Ray): the origin moves to the edge of its error bound
            Vec oo = XP(rfc, o), dd = XV(rfc, d);
            Vec err = gamma(3) * Abs(Vec(rfc[3], rfc[7], rfc[11]));
            if (LengthSquared(dd) > 0) oo = oo + dd * (Dot(Abs(dd), err) / LengthSquared(dd));
            Vec rxo = XP(rfc, o), ryo = rxo;
            Vec dox = CameraFromRenderV(rxo - oo), doy = CameraFromRenderV(ryo - oo);
            if (Length(dox) < Length(minPosDx)) minPosDx = dox;
            if (Length(doy) < Length(minPosDy)) minPosDy = doy;
            Vec rd = Normalize(dd), rx = Normalize(XV(rfc, rxd)), ry = Normalize(XV(rfc, ryd));
            Vec fx, fy;
            CoordinateSystem(rd, &fx, &fy);
            auto local = [&](Vec v) { return Vec(Dot(v, fx), Dot(v, fy), Dot(v, rd)); };
            Vec df = local(rd), dxf = Normalize(local(rx)), dyf = Normalize(local(ry));
            if (Length(dxf - df) < Length(minDirDx)) minDirDx = dxf - df;
            if (Length(dyf - df) < Length(minDirDy)) minDirDy = dyf - df;
        }
    }
    int fullRes[2] = {1, 1};

    // CameraBase::Approximate_dp_dxy (cameras.h:167-195)
    void DpDxy(Vec p, Vec n, Vec *dpdx, Vec *dpdy) const {
        const float *ci = f->camera_from_render, *m = f->render_from_camera;
        Vec pc((ci[0] * p.x + ci[1] * p.y) + (ci[2] * p.z + ci[3]), (ci[4] * p.x + ci[5] * p.y) + (ci[6] * p.z + ci[7]),
               (ci[8] * p.x + ci[9] * p.y) + (ci[10] * p.z + ci[11]));
        Vec nc(m[0] * n.x + m[4] * n.y + m[8] * n.z, m[1] * n.x + m[5] * n.y + m[9] * n.z, m[2] * n.x + m[6] * n.y + m[10] * n.z);
        // RotateFromTo(Normalize(pc), (0, 0, 1)) (util/transform.h:249-270)
        Vec from = Normalize(pc), to(0, 0, 1), refl;
        if (std::abs(from.x) < 0.72f && std::abs(to.x) < 0.72f) refl = Vec(1, 0, 0);
        else if (std::abs(from.y) < 0.72f && std::abs(to.y) < 0.72f) refl = Vec(0, 1, 0);
        else refl = Vec(0, 0, 1);
        Vec u = refl - from, v = refl - to;
        Float r[3][3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                r[i][j] = ((i == j) ? 1 : 0) - 2 / Dot(u, u) * u[i] * u[j] - 2 / Dot(v, v) * v[i] * v[j] +
                          4 * Dot(u, v) / (Dot(u, u) * Dot(v, v)) * v[i] * u[j];
        auto R = [&](Vec a, bool transpose) {
            Vec o;
            for (int i = 0; i < 3; ++i)
                o[i] = transpose ? r[0][i] * a.x + r[1][i] * a.y + r[2][i] * a.z : r[i][0] * a.x + r[i][1] * a.y + r[i][2] * a.z;
            return o;
        };
        Vec pz = R(pc, false);
        pz = Vec(pz.x + 0, pz.y + 0, pz.z + 0);
        Vec nz = R(nc, false);
        Float d = nz.z * pz.z;
        Vec xo = Vec(0, 0, 0) + minPosDx, xd = Vec(0, 0, 1) + minDirDx;
        Vec yo = Vec(0, 0, 0) + minPosDy, yd = Vec(0, 0, 1) + minDirDy;
        Float tx = -(DotN(nz, xo) - d) / DotN(nz, xd), ty = -(DotN(nz, yo) - d) / DotN(nz, yd);
        Vec px = xo + xd * tx, py = yo + yd * ty;
        auto toRender = [&](Vec a) {
            return Vec(m[0] * a.x + m[1] * a.y + m[2] * a.z, m[4] * a.x + m[5] * a.y + m[6] * a.z, m[8] * a.x + m[9] * a.y + m[10] * a.z);
        };
        *dpdx = sppScale * toRender(R(px - pz, true));
        *dpdy = sppScale * toRender(R(py - pz, true));
    }
    // wavefront/surfscatter.cpp:74-104
    OTexCtx Ctx(const Interaction &si) const {
        OTexCtx c;
        c.p = si.p;
        c.n = si.n;
        c.u = si.uv[0];
        c.v = si.uv[1];
        if (f->options & 4) {  // Option "disabletexturefiltering" (surfscatter.cpp:76-77)
            c.dudx = c.dudy = c.dvdx = c.dvdy = 0;
            return c;
        }
        Vec dpdx, dpdy;
        DpDxy(si.p, si.n, &dpdx, &dpdy);
        Float ata00 = Dot(si.dpdu, si.dpdu), ata01 = Dot(si.dpdu, si.dpdv), ata11 = Dot(si.dpdv, si.dpdv);
        Float invDet = 1 / DifferenceOfProducts(ata00, ata11, ata01, ata01);
        invDet = std::isfinite(invDet) ? invDet : 0.f;
        Float atb0x = Dot(si.dpdu, dpdx), atb1x = Dot(si.dpdv, dpdx), atb0y = Dot(si.dpdu, dpdy), atb1y = Dot(si.dpdv, dpdy);
        Float v[4] = {DifferenceOfProducts(ata11, atb0x, ata01, atb1x) * invDet, DifferenceOfProducts(ata11, atb0y, ata01, atb1y) * invDet,
                      DifferenceOfProducts(ata00, atb1x, ata01, atb0x) * invDet, DifferenceOfProducts(ata00, atb1y, ata01, atb0y) * invDet};
        for (Float &x : v) x = std::isfinite(x) ? Clamp(x, -1e8f, 1e8f) : 0.f;
        c.dudx = v[0];
        c.dudy = v[1];
        c.dvdx = v[2];
        c.dvdy = v[3];
        return c;
    }

    // NormalMap / BumpMap (materials.h:86-140) and the caller's ns = FaceForward(Normalize(
    // Cross(dpdu, dpdv)), n) (surfscatter.cpp:109-127) on the oracle's own texture evaluation
    void Bump(int dispNode, int normalImage, Interaction *si) const {
        const OTexCtx c = Ctx(*si);
        const Vec sdpdv = si->hasShadingDiff ? si->dpdvs : si->dpdv;
        const Vec sdndu = si->hasShadingDiff ? si->dndus : Vec(0, 0, 0);
        const Vec sdndv = si->hasShadingDiff ? si->dndvs : Vec(0, 0, 0);
        Vec dpdu, dpdv;
        if (normalImage >= 0) {
            // Image::BilerpChannel at (u, 1 - v), repeat wrap, linear encoding
            const OImage &im = images[normalImage];
            const Float sx = c.u * im.w[0] - 0.5f, sy = (1 - c.v) * im.h[0] - 0.5f;
            const int xi = (int)std::floor(sx), yi = (int)std::floor(sy);
            const Float dx = sx - xi, dy = sy - yi;
            Vec ns;
            for (int ch = 0; ch < 3; ++ch) {
                const Float v = ((1 - dx) * (1 - dy) * im.Get(0, xi, yi, ch) + dx * (1 - dy) * im.Get(0, xi + 1, yi, ch) +
                                 (1 - dx) * dy * im.Get(0, xi, yi + 1, ch) + dx * dy * im.Get(0, xi + 1, yi + 1, ch));
                ns[ch] = 2 * v - 1;
            }
            ns = Normalize(ns);
            const Vec fx = Normalize(si->dpdus), fz = si->ns, fy = Cross(fz, fx);
            ns = fx * ns.x + fy * ns.y + fz * ns.z;
            const Float ulen = Length(si->dpdus), vlen = Length(sdpdv);
            dpdu = Normalize(si->dpdus - Dot(si->dpdus, ns) * ns) * ulen;
            dpdv = Normalize(Cross(ns, dpdu)) * vlen;
        } else {
            OTexCtx sc = c;
            Float du = .5f * (std::abs(c.dudx) + std::abs(c.dudy));
            if (du == 0) du = .0005f;
            sc.p = c.p + du * si->dpdus;
            sc.u = c.u + du;
            sc.v = c.v + 0.f;
            const Float uDisplace = EvalF(dispNode, sc);
            Float dv = .5f * (std::abs(c.dvdx) + std::abs(c.dvdy));
            if (dv == 0) dv = .0005f;
            sc.p = c.p + dv * sdpdv;
            sc.u = c.u + 0.f;
            sc.v = c.v + dv;
            const Float vDisplace = EvalF(dispNode, sc);
            const Float displace = EvalF(dispNode, c);
            dpdu = si->dpdus + (uDisplace - displace) / du * si->ns + displace * sdndu;
            dpdv = sdpdv + (vDisplace - displace) / dv * si->ns + displace * sdndv;
        }
        Vec ns = Normalize(Cross(dpdu, dpdv));
        if (DotN(ns, si->n) < 0) ns = -ns;  // FaceForward(ns, n)
        si->ns = ns;
        si->dpdus = dpdu;
    }

    // TextureMapping2D::Map (textures.h:86-202); the wavefront's dpdx = dpdy = 0
    void Map2D(int node, const OTexCtx &c, Float st[2], Float dst[4]) const {
        const int mapping = Info(node)[6];
        const float *q = Par(node);
        if (mapping == 0) {
            dst[0] = q[18] * c.dudx;
            dst[1] = q[18] * c.dudy;
            dst[2] = q[19] * c.dvdx;
            dst[3] = q[19] * c.dvdy;
            st[0] = q[18] * c.u + q[20];
            st[1] = q[19] * c.v + q[21];
            return;
        }
        Vec pt(q[0] * c.p.x + q[1] * c.p.y + q[2] * c.p.z + q[3], q[4] * c.p.x + q[5] * c.p.y + q[6] * c.p.z + q[7],
               q[8] * c.p.x + q[9] * c.p.y + q[10] * c.p.z + q[11]);
        const Vec zero(0, 0, 0);
        if (mapping == 1) {
            Float x2y2 = Sqr(pt.x) + Sqr(pt.y), sq = std::sqrt(x2y2);
            Vec dsdp = Vec(-pt.y, pt.x, 0) / (2 * Pi * x2y2);
            Vec dtdp = 1 / (Pi * (x2y2 + Sqr(pt.z))) * Vec(pt.x * pt.z / sq, pt.y * pt.z / sq, -sq);
            dst[0] = Dot(dsdp, zero);
            dst[1] = Dot(dsdp, zero);
            dst[2] = Dot(dtdp, zero);
            dst[3] = Dot(dtdp, zero);
            Vec vec = Normalize(pt - Vec(0, 0, 0));
            Float phi = CRATan2(vec.y, vec.x);
            st[0] = SafeACos(vec.z) * InvPi;
            st[1] = (phi < 0 ? phi + 2 * Pi : phi) * 0.15915494309189533577f;
        } else if (mapping == 2) {
            Float x2y2 = Sqr(pt.x) + Sqr(pt.y);
            Vec dsdp = Vec(-pt.y, pt.x, 0) / (2 * Pi * x2y2), dtdp(0, 0, 1);
            dst[0] = Dot(dsdp, zero);
            dst[1] = Dot(dsdp, zero);
            dst[2] = Dot(dtdp, zero);
            dst[3] = Dot(dtdp, zero);
            st[0] = (Pi + CRATan2(pt.y, pt.x)) * 0.15915494309189533577f;
            st[1] = pt.z;
        } else {
            Vec vs(q[12], q[13], q[14]), vt(q[15], q[16], q[17]);
            dst[0] = Dot(vs, zero);
            dst[1] = Dot(vs, zero);
            dst[2] = Dot(vt, zero);
            dst[3] = Dot(vt, zero);
            st[0] = q[18] + Dot(pt, vs);
            st[1] = q[19] + Dot(pt, vt);
        }
    }
    // Checkerboard (textures.cpp:183-217)
    Float Checker(int node, const OTexCtx &c) const {
        auto d = [](Float x) {
            Float y = x / 2 - std::floor(x / 2) - 0.5f;
            return x / 2 + y * (1 - 2 * std::abs(y));
        };
        auto bf = [&](Float x, Float r) -> Float {
            if (std::floor(x - r) == std::floor(x + r)) return 1 - 2 * ((int)std::floor(x) & 1);
            return (d(x + r) - 2 * d(x) + d(x - r)) / Sqr(r);
        };
        if (!(Info(node)[1] & 16)) {
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            Float ds = std::max(std::abs(dst[0]), std::abs(dst[1])), dt = std::max(std::abs(dst[2]), std::abs(dst[3]));
            ds *= 1.5f;
            dt *= 1.5f;
            return 0.5f - bf(st[0], ds) * bf(st[1], dt) / 2;
        }
        const float *q = Par(node);
        Vec p(q[0] * c.p.x + q[1] * c.p.y + q[2] * c.p.z + q[3], q[4] * c.p.x + q[5] * c.p.y + q[6] * c.p.z + q[7],
              q[8] * c.p.x + q[9] * c.p.y + q[10] * c.p.z + q[11]);
        Float dx = 1.5f * std::max(std::abs(0.f), std::abs(0.f));
        return 0.5f - 0.5f * bf(p.x, dx) * bf(p.y, dx) * bf(p.z, dx);
    }
    Float EvalF(int node, const OTexCtx &c) const {
        const int32_t *in = Info(node);
        const float *q = Par(node);
        switch (in[0]) {
        case 0: return q[22];
        case 1: {  // FloatScaledTexture
            Float sc = EvalF(in[3], c);
            if (sc == 0) return 0;
            return EvalF(in[2], c) * sc;
        }
        case 2: {  // FloatMixTexture
            Float amt = EvalF(in[4], c), t1 = 0, t2 = 0;
            if (amt != 1) t1 = EvalF(in[2], c);
            if (amt != 0) t2 = EvalF(in[3], c);
            return (1 - amt) * t1 + amt * t2;
        }
        case 3: {  // FloatDirectionMixTexture
            Float amt = AbsDotN(c.n, Vec(q[22], q[23], q[24])), t1 = 0, t2 = 0;
            if (amt != 0) t1 = EvalF(in[2], c);
            if (amt != 1) t2 = EvalF(in[3], c);
            return amt * t1 + (1 - amt) * t2;
        }
        case 4: {  // FloatCheckerboardTexture
            Float w = Checker(node, c), t0 = 0, t1 = 0;
            if (w != 1) t0 = EvalF(in[2], c);
            if (w != 0) t1 = EvalF(in[3], c);
            return (1 - w) * t0 + w * t1;
        }
        case 5: {  // FloatBilerpTexture
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            return (1 - st[0]) * (1 - st[1]) * q[22] + st[0] * (1 - st[1]) * q[24] + (1 - st[0]) * st[1] * q[23] +
                   st[0] * st[1] * q[25];
        }
        case 7: {  // FloatDotsTexture
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            return proc::PolkaDot(f->noise_perm, st[0], st[1]) ? EvalF(in[2], c) : EvalF(in[3], c);
        }
        case 8:
        case 9:
        case 10: {  // FBmTexture / WrinkledTexture / WindyTexture over the point mapping
            const Vec p = P3(q, c.p), d0 = V3x(q, Vec(0, 0, 0));
            if (in[0] == 8) return proc::FBm(f->noise_perm, p, d0, d0, q[23], (int)q[22]);
            if (in[0] == 9) return proc::Turbulence(f->noise_perm, p, d0, d0, q[23], (int)q[22]);
            return proc::Windy(f->noise_perm, p, d0, d0);
        }
        default: {  // FloatImageTexture
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            st[1] = 1 - st[1];
            Float v;
            images[in[5]].Filter(in[7], q[27], st[0], st[1], dst[0], dst[2], dst[1], dst[3], 1, &v);
            v = q[26] * v;
            return (in[1] & 8) ? std::max<Float>(0, 1 - v) : v;
        }
        }
    }
    Spectrum ConstS(int node, int k, const Wavelengths &L) const {
        const float *s = Spec(node, k);
        Spectrum r;
        for (int i = 0; i < NS; ++i) r[i] = s[0] != 0 ? s[5] * Sigmoid(s[2], s[3], s[4], L.lambda[i]) : s[1];
        return r;
    }
    Spectrum EvalS(int node, const OTexCtx &c, const Wavelengths &L) const {
        const int32_t *in = Info(node);
        const float *q = Par(node);
        switch (in[0]) {
        case 0: return ConstS(node, 0, L);
        case 1: {
            Float sc = EvalF(in[3], c);
            if (sc == 0) return Spectrum(0.f);
            return EvalS(in[2], c, L) * sc;
        }
        case 2: {
            Float amt = EvalF(in[4], c);
            Spectrum t1, t2;
            if (amt != 1) t1 = EvalS(in[2], c, L);
            if (amt != 0) t2 = EvalS(in[3], c, L);
            return t1 * (1 - amt) + t2 * amt;
        }
        case 3: {
            Float amt = AbsDotN(c.n, Vec(q[22], q[23], q[24]));
            Spectrum t1, t2;
            if (amt != 0) t1 = EvalS(in[2], c, L);
            if (amt != 1) t2 = EvalS(in[3], c, L);
            return t1 * amt + t2 * (1 - amt);
        }
        case 4: {
            Float w = Checker(node, c);
            Spectrum t0, t1;
            if (w != 1) t0 = EvalS(in[2], c, L);
            if (w != 0) t1 = EvalS(in[3], c, L);
            return t0 * (1 - w) + t1 * w;
        }
        case 7: {  // SpectrumDotsTexture
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            return proc::PolkaDot(f->noise_perm, st[0], st[1]) ? EvalS(in[2], c, L) : EvalS(in[3], c, L);
        }
        case 11: {  // MarbleTexture: RGBAlbedoSpectrum(sRGB, rgb)
            const Vec p = P3(q, c.p), d0 = V3x(q, Vec(0, 0, 0));
            Float rgb[3], co[3];
            proc::Marble(f->noise_perm, p, d0, d0, (int)q[22], q[23], q[26], q[24], rgb);
            ORGBCoeffs(rgb[0], rgb[1], rgb[2], co);
            Spectrum r;
            for (int i = 0; i < NS; ++i) r[i] = Sigmoid(co[0], co[1], co[2], L.lambda[i]);
            return r;
        }
        case 5: {  // Bilerp({s, t}, {v00, v10, v01, v11}) (util/spectrum.h:734-738)
            Float st[2], dst[4];
            Map2D(node, c, st, dst);
            return ConstS(node, 0, L) * ((1 - st[0]) * (1 - st[1])) + ConstS(node, 1, L) * (st[0] * (1 - st[1])) +
                   ConstS(node, 2, L) * ((1 - st[0]) * st[1]) + ConstS(node, 3, L) * (st[0] * st[1]);
        }
        default: {  // SpectrumImageTexture (textures.cpp:359-405)
            Float st[2], dst[4], rgb[3];
            Map2D(node, c, st, dst);
            st[1] = 1 - st[1];
            images[in[5]].Filter(in[7], q[27], st[0], st[1], dst[0], dst[2], dst[1], dst[3], 3, rgb);
            if (in[1] & 32) {
                // GPUSpectrumImageTexture::Evaluate, the fork's multispectral basis branch
                // (textures.h:655-679): sum_c basis[3 + i + c NS] (texel_c - int offset), the basis
                // indexed by the wavelength sample i (clamped to the table), the texel unscaled
                const float *tab = f->tex_basis + (int)q[22];
                const int width = (int)q[24], nCh = (int)tab[0], off = (int)tab[2];
                Spectrum s(0.f);
                for (int ch = 0; ch < nCh; ++ch) {
                    Spectrum b;
                    for (int i = 0; i < NS; ++i) b[i] = tab[std::min(3 + i + ch * NS, width - 1)];
                    s = b * (rgb[ch] - off) + s;
                }
                return s;
            }
            for (int k = 0; k < 3; ++k) {
                rgb[k] = q[26] * rgb[k];
                rgb[k] = std::max<Float>(0, (in[1] & 8) ? 1 - rgb[k] : rgb[k]);
            }
            Float co[3], scale = 1;
            if (((in[1] >> 1) & 3) == 0) {  // RGBAlbedoSpectrum(Clamp(rgb, 0, 1))
                ORGBCoeffs(Clamp(rgb[0], 0, 1), Clamp(rgb[1], 0, 1), Clamp(rgb[2], 0, 1), co);
                Spectrum r;
                for (int i = 0; i < NS; ++i) r[i] = Sigmoid(co[0], co[1], co[2], L.lambda[i]);
                return r;
            }
            Float m = std::max({rgb[0], rgb[1], rgb[2]});  // RGBUnboundedSpectrum
            scale = 2 * m;
            if (scale != 0) ORGBCoeffs(rgb[0] / scale, rgb[1] / scale, rgb[2] / scale, co);
            else ORGBCoeffs(0, 0, 0, co);
            Spectrum r;
            for (int i = 0; i < NS; ++i) r[i] = scale * Sigmoid(co[0], co[1], co[2], L.lambda[i]);
            return r;
        }
        }
    }
};

// ---------------------------------------------------------------- integrator
bool Scene::AlphaKilled(int prim, const TriIsect &ti, Vec o, Vec d) const {
    const Interaction si = Interact(prim, ti, d);
    OTexCtx c;
    c.p = si.p;
    c.n = si.n;
    c.u = si.uv[0];
    c.v = si.uv[1];
    const Float a = tex->EvalF(f->prim_alpha[prim], c);
    if (a >= 1) return false;
    if (a <= 0) return true;
    const float od[6] = {o.x, o.y, o.z, d.x, d.y, d.z};
    unsigned char buf[24];
    std::memcpy(buf, od, 24);
    return (Float)(uint32_t)Murmur64A(buf, 24, 0) * 0x1p-32f > a;
}

// ---------------------------------------------------------------- subsurface scattering
// SubsurfaceMaterial's TabulatedBSSRDF and the wavefront's SampleSubsurface
// (wavefront/subsurface.cpp:18-206), restated: the BSSRDF table (ComputeBeamDiffusionBSSRDF,
// bssrdf.cpp:26-155, with FresnelMoment1/2 util/scattering.cpp:10-31 and IntegrateCatmullRom
// util/math.cpp:267-288), the spline utilities (CatmullRomWeights / InvertCatmullRom
// util/math.cpp:157-265, SampleCatmullRom2D util/sampling.cpp:424-488, NewtonBisection
// util/math.h:662-696) and TabulatedBSSRDF's Sr / PDF_Sr / SampleSr / SampleSp / PDF_Sp
// (bssrdf.h:118-258).  The table is built here from (g, eta), independently of the product.
namespace osss {
constexpr int NRho = 100, NRad = 64, TableFloats = NRho + NRad + 2 * NRho * NRad + NRho;
static Float FresnelMoment1(Float eta) {
    Float eta2 = eta * eta, eta3 = eta2 * eta, eta4 = eta3 * eta, eta5 = eta4 * eta;
    if (eta < 1) return 0.45966f - 1.73965f * eta + 3.37668f * eta2 - 3.904945 * eta3 + 2.49277f * eta4 - 0.68441f * eta5;
    return -4.61686f + 11.1136f * eta - 10.4646f * eta2 + 5.11455f * eta3 - 1.27198f * eta4 + 0.12746f * eta5;
}
static Float FresnelMoment2(Float eta) {
    Float eta2 = eta * eta, eta3 = eta2 * eta, eta4 = eta3 * eta, eta5 = eta4 * eta;
    if (eta < 1) return 0.27614f - 0.87350f * eta + 1.12077f * eta2 - 0.65095f * eta3 + 0.07883f * eta4 + 0.04860f * eta5;
    Float r_eta = 1 / eta, r_eta2 = r_eta * r_eta, r_eta3 = r_eta2 * r_eta;
    return -547.033f + 45.3087f * r_eta3 - 218.725f * r_eta2 + 458.843f * r_eta + 404.557f * eta - 189.519f * eta2 +
           54.9327f * eta3 - 9.00603f * eta4 + 0.63942f * eta5;
}
static Float SampleExp(Float u, Float a) { return -CRLog(1 - u) / a; }
static Float BeamDiffusionMS(Float sigma_s, Float sigma_a, Float g, Float eta, Float r) {
    const int nSamples = 100;
    Float Ed = 0;
    Float sigmap_s = sigma_s * (1 - g), sigmap_t = sigma_a + sigmap_s, rhop = sigmap_s / sigmap_t;
    Float D_g = (2 * sigma_a + sigmap_s) / (3 * sigmap_t * sigmap_t);
    Float sigma_tr = SafeSqrt(sigma_a / D_g);
    Float fm1 = FresnelMoment1(eta), fm2 = FresnelMoment2(eta);
    Float ze = -2 * D_g * (1 + 3 * fm2) / (1 - 2 * fm1);
    Float cPhi = 0.25f * (1 - 2 * fm1), cE = 0.5f * (1 - 3 * fm2);
    const Float Inv4Pi = 0.07957747154594766788f;
    for (int i = 0; i < nSamples; ++i) {
        Float zr = SampleExp((i + 0.5f) / nSamples, sigmap_t);
        Float zv = -zr + 2 * ze;
        Float dr = std::sqrt(Sqr(r) + Sqr(zr)), dv = std::sqrt(Sqr(r) + Sqr(zv));
        Float phiD = Inv4Pi / D_g * (FastExp(-sigma_tr * dr) / dr - FastExp(-sigma_tr * dv) / dv);
        Float EDn = Inv4Pi * (zr * (1 + sigma_tr * dr) * FastExp(-sigma_tr * dr) / (dr * dr * dr) -
                              zv * (1 + sigma_tr * dv) * FastExp(-sigma_tr * dv) / (dv * dv * dv));
        Float E = phiD * cPhi + EDn * cE;
        Float kappa = 1 - FastExp(-2 * sigmap_t * (dr + zr));
        Ed += kappa * rhop * rhop * E;
    }
    return Ed / nSamples;
}
static Float BeamDiffusionSS(Float sigma_s, Float sigma_a, Float g, Float eta, Float r) {
    Float sigma_t = sigma_a + sigma_s, rho = sigma_s / sigma_t;
    Float tCrit = r * SafeSqrt(Sqr(eta) - 1);
    Float Ess = 0;
    const int nSamples = 100;
    for (int i = 0; i < nSamples; ++i) {
        Float ti = tCrit + SampleExp((i + 0.5f) / nSamples, sigma_t);
        Float d = std::sqrt(Sqr(r) + Sqr(ti));
        Float cosTheta_o = ti / d;
        Ess += rho * FastExp(-sigma_t * (d + tCrit)) / Sqr(d) * HenyeyGreenstein(cosTheta_o, g) *
               (1 - FrDielectric(-cosTheta_o, eta)) * std::abs(cosTheta_o);
    }
    return Ess / nSamples;
}
static std::vector<float> Table(Float g, Float eta) {
    std::vector<float> t(TableFloats, 0.f);
    float *rho = t.data(), *rad = rho + NRho, *prof = rad + NRad, *rhoEff = prof + NRho * NRad, *cdf = rhoEff + NRho;
    rad[0] = 0;
    rad[1] = 2.5e-3f;
    for (int i = 2; i < NRad; ++i) rad[i] = rad[i - 1] * 1.2f;
    for (int i = 0; i < NRho; ++i) rho[i] = (1 - FastExp(-8 * i / (Float)(NRho - 1))) / (1 - FastExp(-8));
    for (int i = 0; i < NRho; ++i) {
        for (int j = 0; j < NRad; ++j)
            prof[i * NRad + j] = 2 * Pi * rad[j] *
                                 (BeamDiffusionSS(rho[i], 1 - rho[i], g, eta, rad[j]) + BeamDiffusionMS(rho[i], 1 - rho[i], g, eta, rad[j]));
        // IntegrateCatmullRom
        const float *f = prof + i * NRad;
        float *c = cdf + i * NRad;
        Float sum = 0;
        c[0] = 0;
        for (int k = 0; k < NRad - 1; ++k) {
            Float x0 = rad[k], x1 = rad[k + 1], f0 = f[k], f1 = f[k + 1], width = x1 - x0;
            Float d0 = k > 0 ? width * (f1 - f[k - 1]) / (x1 - rad[k - 1]) : f1 - f0;
            Float d1 = k + 2 < NRad ? width * (f[k + 2] - f0) / (rad[k + 2] - x0) : f1 - f0;
            sum += width * ((f0 + f1) / 2 + (d0 - d1) / 12);
            c[k + 1] = sum;
        }
        rhoEff[i] = sum;
    }
    return t;
}
template <typename Pred>
static int FindInterval(int sz, const Pred &pred) {
    int size = sz - 2, first = 1;
    while (size > 0) {
        int half = size >> 1, middle = first + half;
        bool r = pred(middle);
        first = r ? middle + 1 : first;
        size = r ? size - (half + 1) : half;
    }
    return std::max(0, std::min(first - 1, sz - 2));
}
static bool Weights(const float *nodes, int n, Float x, int *offset, Float w[4]) {
    if (!(x >= nodes[0] && x <= nodes[n - 1])) return false;
    int idx = FindInterval(n, [&](int i) { return nodes[i] <= x; });
    *offset = idx - 1;
    Float x0 = nodes[idx], x1 = nodes[idx + 1];
    Float t = (x - x0) / (x1 - x0), t2 = t * t, t3 = t2 * t;
    w[1] = 2 * t3 - 3 * t2 + 1;
    w[2] = -2 * t3 + 3 * t2;
    if (idx > 0) {
        Float w0 = (t3 - 2 * t2 + t) * (x1 - x0) / (x1 - nodes[idx - 1]);
        w[0] = -w0;
        w[2] += w0;
    } else {
        Float w0 = t3 - 2 * t2 + t;
        w[0] = 0;
        w[1] -= w0;
        w[2] += w0;
    }
    if (idx + 2 < n) {
        Float w3 = (t3 - t2) * (x1 - x0) / (nodes[idx + 2] - x0);
        w[1] -= w3;
        w[3] = w3;
    } else {
        Float w3 = t3 - t2;
        w[1] -= w3;
        w[2] += w3;
        w[3] = 0;
    }
    return true;
}
template <typename F>
static Float Newton(F f) {
    Float x0 = 0, x1 = 1;
    const Float eps = 1e-6f;
    std::pair<Float, Float> a = f(x0), b = f(x1);
    if (std::abs(a.first) < eps) return x0;
    if (std::abs(b.first) < eps) return x1;
    bool startIsNegative = a.first < 0;
    Float xMid = x0 + (x1 - x0) * -a.first / (b.first - a.first);
    while (true) {
        if (!(x0 < xMid && xMid < x1)) xMid = (x0 + x1) / 2;
        std::pair<Float, Float> m = f(xMid);
        if (startIsNegative == (m.first < 0)) x0 = xMid;
        else x1 = xMid;
        if ((x1 - x0) < eps || std::abs(m.first) < eps) return xMid;
        xMid -= m.first / m.second;
    }
}
static Float InvertCatmullRom(const float *x, const float *f, int n, Float u) {
    if (!(u > f[0])) return x[0];
    if (!(u < f[n - 1])) return x[n - 1];
    int i = FindInterval(n, [&](int k) { return f[k] <= u; });
    Float x0 = x[i], x1 = x[i + 1], f0 = f[i], f1 = f[i + 1], width = x1 - x0;
    Float d0 = i > 0 ? width * (f1 - f[i - 1]) / (x1 - x[i - 1]) : f1 - f0;
    Float d1 = i + 2 < n ? width * (f[i + 2] - f0) / (x[i + 2] - x0) : f1 - f0;
    Float t = Newton([&](Float t) {
        Float t2 = t * t, t3 = t2 * t;
        Float Fhat = (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
        Float fhat = (6 * t2 - 6 * t) * f0 + (-6 * t2 + 6 * t) * f1 + (3 * t2 - 4 * t + 1) * d0 + (3 * t2 - 2 * t) * d1;
        return std::make_pair(Fhat - u, fhat);
    });
    return x0 + t * width;
}
static Float SampleCatmullRom2D(const float *n1, int s1, const float *n2, int s2, const float *values, const float *cdf,
                                Float alpha, Float u) {
    int offset;
    Float w[4];
    if (!Weights(n1, s1, alpha, &offset, w)) return 0;
    auto interp = [&](const float *a, int idx) {
        Float v = 0;
        for (int i = 0; i < 4; ++i)
            if (w[i] != 0) v += a[(offset + i) * s2 + idx] * w[i];
        return v;
    };
    Float maximum = interp(cdf, s2 - 1);
    u *= maximum;
    int idx = FindInterval(s2, [&](int i) { return interp(cdf, i) <= u; });
    Float f0 = interp(values, idx), f1 = interp(values, idx + 1);
    Float x0 = n2[idx], x1 = n2[idx + 1], width = x1 - x0, d0, d1;
    u = (u - interp(cdf, idx)) / width;
    d0 = idx > 0 ? width * (f1 - interp(values, idx - 1)) / (x1 - n2[idx - 1]) : f1 - f0;
    d1 = idx + 2 < s2 ? width * (interp(values, idx + 2) - f0) / (n2[idx + 2] - x0) : f1 - f0;
    Float t = Newton([&](Float t) {
        // EvaluatePolynomial: FMA Horner
        Float c3 = (1.f / 3.f) * (-2 * d0 - d1) + f1 - f0, c4 = 0.25f * (d0 + d1) + 0.5f * (f0 - f1);
        Float Fhat = std::fma(t, std::fma(t, std::fma(t, std::fma(t, c4, c3), 0.5f * d0), f0), 0.f);
        Float fhat = std::fma(t, std::fma(t, std::fma(t, d0 + d1 + 2 * (f0 - f1), -2 * d0 - d1 + 3 * (f1 - f0)), d0), f0);
        return std::make_pair(Fhat - u, fhat);
    });
    return x0 + width * t;
}
struct BSSRDF {
    const float *rho, *rad, *prof, *rhoEff, *cdf;
    Vec po, ns;
    Spectrum sigma_t, rhoS;
    Spectrum Sr(Float r) const {
        Spectrum out(0.f);
        for (int i = 0; i < NS; ++i) {
            Float rOptical = r * sigma_t[i];
            int ro, rr;
            Float rw[4], dw[4];
            if (!Weights(rho, NRho, rhoS[i], &ro, rw) || !Weights(rad, NRad, rOptical, &rr, dw)) continue;
            Float sr = 0;
            for (int j = 0; j < 4; ++j)
                for (int k = 0; k < 4; ++k)
                    if (Float weight = rw[j] * dw[k]; weight != 0) sr += weight * prof[(ro + j) * NRad + rr + k];
            if (rOptical != 0) sr /= 2 * Pi * rOptical;
            out[i] = sr;
        }
        for (int i = 0; i < NS; ++i) out[i] = std::max<Float>(0, out[i] * (sigma_t[i] * sigma_t[i]));
        return out;
    }
    Spectrum PdfSr(Float r) const {
        Spectrum pdf(0.f);
        for (int i = 0; i < NS; ++i) {
            Float rOptical = r * sigma_t[i];
            int ro, rr;
            Float rw[4], dw[4];
            if (!Weights(rho, NRho, rhoS[i], &ro, rw) || !Weights(rad, NRad, rOptical, &rr, dw)) continue;
            Float sr = 0, re = 0;
            for (int j = 0; j < 4; ++j)
                if (rw[j] != 0) {
                    re += rhoEff[ro + j] * rw[j];
                    for (int k = 0; k < 4; ++k)
                        if (dw[k] != 0) sr += prof[(ro + j) * NRad + rr + k] * rw[j] * dw[k];
                }
            if (rOptical != 0) sr /= 2 * Pi * rOptical;
            pdf[i] = sr * (sigma_t[i] * sigma_t[i]) / re;
        }
        for (int i = 0; i < NS; ++i) pdf[i] = std::max<Float>(0, pdf[i]);
        return pdf;
    }
    bool SampleSr(Float u, Float *r) const {
        if (sigma_t[0] == 0) return false;
        *r = SampleCatmullRom2D(rho, NRho, rad, NRad, prof, cdf, rhoS[0], u) / sigma_t[0];
        return true;
    }
    bool SampleSp(Float u1, Float u20, Float u21, Vec *p0, Vec *p1) const {
        Vec fx, fy, fz;
        if (u1 < 0.25f) {
            fx = ns;
            CoordinateSystem(ns, &fy, &fz);
        } else if (u1 < 0.5f) {
            fy = ns;
            CoordinateSystem(ns, &fz, &fx);
        } else {
            fz = ns;
            CoordinateSystem(ns, &fx, &fy);
        }
        Float r, rMax;
        if (!SampleSr(u20, &r)) return false;
        Float phi = 2 * Pi * u21;
        if (!SampleSr(0.999f, &rMax) || r >= rMax) return false;
        Float l = 2 * std::sqrt(Sqr(rMax) - Sqr(r));
        Vec pStart = po + (fx * CRCos(phi) + fy * CRSin(phi)) * r - fz * l / 2;
        *p0 = pStart;
        *p1 = pStart + fz * l;
        return true;
    }
    Spectrum PdfSp(Vec pi, Vec ni) const {
        Vec d = pi - po, x, y;
        CoordinateSystem(ns, &x, &y);
        Vec dl(Dot(d, x), Dot(d, y), Dot(d, ns)), nl(DotN(ni, x), DotN(ni, y), DotN(ni, ns));
        Float rProj[3] = {std::sqrt(Sqr(dl.y) + Sqr(dl.z)), std::sqrt(Sqr(dl.z) + Sqr(dl.x)), std::sqrt(Sqr(dl.x) + Sqr(dl.y))};
        Float axisProb[3] = {.25f, .25f, .5f};
        Spectrum pdf(0.f);
        for (int a = 0; a < 3; ++a) pdf = pdf + PdfSr(rProj[a]) * std::abs(nl[a]) * axisProb[a];
        return pdf;
    }
};
}  // namespace osss

// IntersectOneRandom (optix.cu:478-518): closest hits from p0 towards p1 (tMax 1), each
// continued by SpawnRayTo(p1) up to 99 traces, reservoir-sampling the hits on material `mat`
// (weight 1, RNG seeded with Hash(p0, p1)); -1 when none
int ProbeOneRandom(const Scene &S, Vec p0, Vec p1, int mat, TriIsect *cti, Vec *cdir, Float *resPdf) {
    const uint64_t hseed = HashFloats(p0.x, p0.y, p0.z, p1.x, p1.y, p1.z);
    PCG32 wrs(hseed, Mix64(hseed));  // WeightedReservoirSampler::Seed: RNG::SetSequence
    Float wsum = 0;
    int chosen = -1;
    Vec po = p0, pd = p1 - p0;
    for (int it = 1; LengthSquared(pd) > 0 && it < 100; ++it) {
        TriIsect t2;
        const int hp = S.Intersect(po, pd, 1, &t2, false);
        if (hp < 0) break;
        const Interaction hi = S.Interact(hp, t2, pd);
        if (S.Material(hp) == mat) {
            wsum += 1;
            if (wrs.Uniform() < 1 / wsum) chosen = hp, *cti = t2, *cdir = pd;
        }
        pd = p1 - hi.p;
        po = OffsetRayOrigin(hi.p, hi.err, hi.n, pd);
    }
    *resPdf = chosen >= 0 && wsum > 0 ? 1 / wsum : 0;
    return chosen >= 0 && wsum > 0 ? chosen : -1;
}

struct Renderer {
    std::vector<OEnvLight> envs;  // ImageInfiniteLights (flat inf_image)
    // the image light behind global light index li, or null
    const OEnvLight *EnvOf(int li) const {
        const int j = li - f->n_area_lights - f->n_point_spot;
        if (f->n_env == 0 || j < 0 || f->inf_image[j] < 0) return nullptr;
        return &envs[f->inf_image[j]];
    }
    Scene S;
    OTextures tex;
    Lights lights;
    Media M;
    PixelFilter filt;
    const pbrt_scene_flat *f;
    std::vector<std::vector<float>> sssTables;  // osss::Table(g, eta) per subsurface material
    std::vector<omeas::Brdf> measured;          // flat measured_files, read by the oracle itself

    // TraceTransmittance (wavefront/intersect.h:164-274) up to the light point o + tMax d:
    // closest hits; a non-interface surface blocks (T_ray = 0); interfaces are crossed with
    // SpawnRayTo(pLight); ratio tracking with RR in every medium.  RNG(Hash(o), Hash(d)).
    void TraceTransmittance(Vec o, Vec d, Float tMax, int med, const Wavelengths &lambda, Spectrum *Tout,
                            Spectrum *tuOut, Spectrum *tlOut) const {
        const Vec pLight = o + d * tMax;
        PCG32 rng(HashFloats(o.x, o.y, o.z), HashFloats(d.x, d.y, d.z));
        Spectrum T_ray(1.f), tu(1.f), tl(1.f);
        while (d != Vec(0, 0, 0)) {
            TriIsect ti;
            int hp = S.Intersect(o, d, tMax, &ti, false);
            if (hp >= 0 && f->material_type[S.Material(hp)] != 3) {
                T_ray = Spectrum(0.f);
                break;
            }
            Interaction hsi;
            if (hp >= 0) hsi = S.Interact(hp, ti, d);
            if (med >= 0) {
                Float tEnd = hp < 0 ? tMax : (Length(o - hsi.p) / Length(d));
                Spectrum T_maj = SampleTmaj(M, med, o, d, tEnd, rng.Uniform(), rng, lambda,
                                            [&](Vec, const MediumProps &mp, const Spectrum &sigma_maj, const Spectrum &Tm) {
                    Spectrum sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
                    Float pr = Tm[0] * sigma_maj[0];
                    T_ray = T_ray * (Tm * sigma_n / pr);
                    tl = tl * (Tm * sigma_maj / pr);
                    tu = tu * (Tm * sigma_n / pr);
                    Spectrum Tr = T_ray / (tl + tu).Average();
                    if (Tr.Max() < 0.05f) {
                        Float q = 0.75f;
                        if (rng.Uniform() < q) T_ray = Spectrum(0.f);
                        else T_ray = T_ray / (1 - q);
                    }
                    return bool(T_ray);
                });
                T_ray = T_ray * (T_maj / T_maj[0]);
                tl = tl * (T_maj / T_maj[0]);
                tu = tu * (T_maj / T_maj[0]);
            }
            if (hp < 0 || !T_ray) break;
            // SurfaceInteraction::SpawnRayTo(pLight) (interaction.h, ray.h:98-104)
            int mi = med, mo = med, pin, pout;
            if (f->n_media > 0 && S.Medium(hp, &pin, &pout) && pin != pout) {
                mi = pin;
                mo = pout;
            }
            Vec dd = pLight - hsi.p;
            o = OffsetRayOrigin(hsi.p, hsi.err, hsi.n, dd);
            d = pLight - hsi.p;
            med = DotN(hsi.n, d) > 0 ? mo : mi;
        }
        *Tout = T_ray;
        *tuOut = tu;
        *tlOut = tl;
    }

    Vec Xf(const float *m, Vec p, bool point) const {
        Float x = m[0] * p.x + m[1] * p.y + m[2] * p.z, y = m[4] * p.x + m[5] * p.y + m[6] * p.z,
              z = m[8] * p.x + m[9] * p.y + m[10] * p.z;
        if (!point) return Vec(x, y, z);
        x = x + m[3];
        y = y + m[7];
        z = z + m[11];
        Float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
        if (w == 1) return Vec(x, y, z);
        return Vec(x, y, z) / w;
    }

    Spectrum LightL(int li, const Wavelengths &lambda, const Float *uv = nullptr) const {
        const float *dense = f->dense_spectra + 311 * f->light_spectrum[li];
        if (uv && f->light_image && f->light_image[li] >= 0) {
            // an image emitter (lights.h:460-467): Image::BilerpChannel at (u, 1 - v), clamp
            // wrap, RGBIlluminantSpectrum of ClampZero(rgb) times the light scale
            const float *img = f->area_images + f->light_image[li];
            const int w = (int)img[0], h = (int)img[1];
            const float *rgb = img + 2;
            const Float x = uv[0] * w - 0.5f, y = (1 - uv[1]) * h - 0.5f;
            const int xi = (int)std::floor(x), yi = (int)std::floor(y);
            const Float dx = x - xi, dy = y - yi;
            auto at = [&](int px, int py, int c) {
                px = std::clamp(px, 0, w - 1), py = std::clamp(py, 0, h - 1);
                return rgb[((size_t)py * w + px) * 3 + c];
            };
            Float c3[3];
            for (int c = 0; c < 3; ++c)
                c3[c] = std::max<Float>(0, (1 - dx) * (1 - dy) * at(xi, yi, c) + dx * (1 - dy) * at(xi + 1, yi, c) +
                                               (1 - dx) * dy * at(xi, yi + 1, c) + dx * dy * at(xi + 1, yi + 1, c));
            Float mx = std::max({c3[0], c3[1], c3[2]}), rs = 2 * mx, co[3];
            if (rs) ORGBCoeffs(c3[0] / rs, c3[1] / rs, c3[2] / rs, co);
            else ORGBCoeffs(0, 0, 0, co);
            Spectrum sp;
            for (int i = 0; i < NS; ++i) sp[i] = rs * Sigmoid(co[0], co[1], co[2], lambda.lambda[i]);
            return (sp * SampleDense(dense, lambda)) * f->light_scale[li];
        }
        return SampleDense(dense, lambda) * f->light_scale[li];
    }
    // DiffuseAreaLight::L (lights.h:443-470) leaving along w at a point with normal n: zero on the
    // back of a one-sided emitter and, with this fork's spread, outside the cone
    // AbsDot(w, n) >= cosFalloffEnd
    Spectrum AreaL(int li, Vec n, Vec w, const Wavelengths &lambda, const Float *uv = nullptr) const {
        if (!(f->light_two_sided[li] || DotN(n, w) >= 0)) return Spectrum(0.f);
        const float cosE = f->light_spread ? f->light_spread[3 * li] : -1;
        if (cosE > 0 && std::abs(DotN(n, w)) < cosE) return Spectrum(0.f);
        return LightL(li, lambda, uv);
    }
    // DiffuseAreaLight::SampleLi's spread attenuation (lights.cpp:763-771) toward wi
    Spectrum SampledAreaL(int li, Vec n, Vec wi, const Wavelengths &lambda, const Float *uv = nullptr) const {
        Spectrum Le = AreaL(li, n, -wi, lambda, uv);
        const float *sp = f->light_spread ? f->light_spread + 3 * li : nullptr;
        if (sp && sp[0] > 0) {
            const Float cos_a = -DotN(n, wi);
            const Float sin_a = SafeSqrt(1 - Sqr(cos_a));
            const Float tan_a = sin_a / cos_a;
            Le = Le * std::max((1.0f - (sp[1] * tan_a)) * sp[2], 0.0f);
        }
        return Le;
    }
    // PointLight / SpotLight / DistantLight::SampleLi (lights.h:221-228, 282-289, 784-798) for a
    // global light index past the area lights; false for a UniformInfiniteLight (SampleLi with
    // allowIncompletePDF returns nothing) and for a spot light whose Li vanishes.
    struct DeltaSample {
        Vec wi, p;
        Spectrum L;
    };
    static Float SmoothStep(Float x, Float a, Float b) {
        if (a == b) return (x < a) ? 0 : 1;
        Float t = std::min<Float>(std::max<Float>((x - a) / (b - a), 0), 1);
        return t * t * (3 - 2 * t);
    }
    bool DeltaLi(int li, Vec ref, const Wavelengths &lambda, DeltaSample *ds) const {
        const int k = li - f->n_area_lights;
        int di = k;
        if (k >= f->n_point_spot) {
            di = f->inf_distant[k - f->n_point_spot];
            if (di < 0) return false;
        }
        const float *d = f->delta_lights + 24 * di;
        const int type = (int)d[0];
        const Spectrum I = SampleDense(f->dense_spectra + 311 * (int)d[1], lambda);
        const Float scale = d[2];
        if (type == 2) {
            ds->wi = Normalize(Vec(d[8], d[9], d[10]));
            ds->p = ref + ds->wi * (2 * f->scene_radius);
            ds->L = I * scale;
            return true;
        }
        const Vec p(d[5], d[6], d[7]);
        ds->wi = Normalize(p - ref);
        ds->p = p;
        Float sc = scale;
        if (type >= 3) {
            // GoniometricLight / ProjectionLight::SampleLi (lights.cpp:320-331, 538-547): I at
            // renderFromLight.ApplyInverse(-wi), divided by the squared distance
            const Vec v = -ds->wi;
            const Vec wl(d[11] * v.x + d[12] * v.y + d[13] * v.z, d[14] * v.x + d[15] * v.y + d[16] * v.z,
                         d[17] * v.x + d[18] * v.y + d[19] * v.z);
            const float *img = f->delta_images + (int)d[21];
            const int w = (int)d[22], h = (int)d[23];
            auto nearest = [&](Float u, Float vv) {  // Image::LookupNearestChannel, WrapMode::Clamp
                const int x = std::clamp((int)(u * w), 0, w - 1), y = std::clamp((int)(vv * h), 0, h - 1);
                return (size_t)y * w + x;
            };
            if (type == 3) {
                Float u, vv;
                OEnvLight::SphereToSquare(wl, &u, &vv);
                ds->L = (I * scale * img[4 + nearest(u, vv)]) / DistanceSquared(p, ref);
                return (bool)ds->L;
            }
            // ProjectionLight::I (lights.cpp:343-360)
            if (wl.z < 1e-3f) return false;
            const Float s = img[0], aspect = Float(w) / Float(h);
            const Float bx = aspect > 1 ? aspect : 1, by = aspect > 1 ? 1 : 1 / aspect;
            const Float psx = (s * wl.x) / wl.z, psy = (s * wl.y) / wl.z;
            if (!(psx >= -bx && psx <= bx && psy >= -by && psy <= by)) return false;
            const float *px = img + 4 + 3 * nearest((psx - -bx) / (bx - -bx), (psy - -by) / (by - -by));
            Float c3[3] = {std::max<Float>(0, px[0]), std::max<Float>(0, px[1]), std::max<Float>(0, px[2])};
            Float mx = std::max({c3[0], c3[1], c3[2]}), rs = 2 * mx, co[3];
            if (rs) ORGBCoeffs(c3[0] / rs, c3[1] / rs, c3[2] / rs, co);
            else ORGBCoeffs(0, 0, 0, co);
            Spectrum sp;
            for (int i = 0; i < NS; ++i) sp[i] = rs * Sigmoid(co[0], co[1], co[2], lambda.lambda[i]);
            ds->L = ((sp * I) * scale) / DistanceSquared(p, ref);  // scale * RGBIlluminantSpectrum
            return (bool)ds->L;
        }
        if (type == 1) {
            const Vec v = -ds->wi;
            const Vec wl = Normalize(Vec(d[11] * v.x + d[12] * v.y + d[13] * v.z, d[14] * v.x + d[15] * v.y + d[16] * v.z,
                                         d[17] * v.x + d[18] * v.y + d[19] * v.z));
            sc = SmoothStep(wl.z, d[4], d[3]) * scale;
        }
        ds->L = (I * sc) / DistanceSquared(p, ref);
        return (bool)ds->L;
    }

    // MixMaterial resolution of a hit's material (see the loop's comment)
    int ResolveMix(int mat, const Interaction &si) const {
        // MixMaterial::ChooseMaterial at the closest hit (wavefront/intersect.h:90-97,
        // materials.h:285-294): amount texture without (u,v) derivatives, HashFloat(p, wo,
        // m0, m1) with the material indices standing in for pbrt's material pointers
        while (f->material_mix && f->material_type[mat] == 8) {
            const int32_t *mm = f->material_mix + 4 * mat;
            OTexCtx c0;
            c0.p = si.p;
            c0.n = si.n;
            c0.u = si.uv[0];
            c0.v = si.uv[1];
            const Float amt = tex.EvalF(mm[2], c0);
            if (amt <= 0) mat = mm[0];
            else if (amt >= 1) mat = mm[1];
            else {
                unsigned char buf[40];
                const Float pv[6] = {si.p.x, si.p.y, si.p.z, si.wo.x, si.wo.y, si.wo.z};
                const uint64_t m0 = (uint32_t)mm[0], m1 = (uint32_t)mm[1];
                std::memcpy(buf, pv, 24);
                std::memcpy(buf + 24, &m0, 8);
                std::memcpy(buf + 32, &m1, 8);
                const Float u = (Float)(uint32_t)Murmur64A(buf, 40, 0) * 0x1p-32f;
                mat = (amt < u) ? mm[0] : mm[1];
            }
        }
        return mat;
    }
    // Material::GetBxDF (materials.h:466-471 diffuse, :182-204 dielectric, :491-511 conductor,
    // materials.cpp:301-329 / 391-437 coated) with bump / normal mapping applied to si first;
    // lambda's secondary wavelengths may be terminated.  Returns whether the BSDF is layered.
    bool MakeBSDF(int mat, Wavelengths &lambda, bool anyNonSpecular, Interaction &si, BxDF &bx,
                  LayeredBxDF &lay) const {
        const float *mc = f->material_coeffs + 4 * mat;
        // bump / normal mapping (surfscatter.cpp:109-127, materials.h:86-140): the shading
        // normal and dpdu the BSDF, the light sample and the next vertex's MIS context use
        if (f->material_bump && (f->material_bump[2 * mat] >= 0 || f->material_bump[2 * mat + 1] >= 0))
            tex.Bump(f->material_bump[2 * mat], f->material_bump[2 * mat + 1], &si);
        bx.type = f->material_type[mat];
        const bool layered = bx.type == 4 || bx.type == 5;
        if (layered) {
            // CoatedDiffuseMaterial / CoatedConductorMaterial::GetBxDF (materials.cpp:301-329, :391-437)
            const float *mp = f->material_params + 4 * mat, *ml = f->material_layer + 12 * mat;
            Float ieta = mp[2] == 0 ? 1.f : mp[2];
            if (ml[11] >= 0) {  // spectral interface eta: eta(lambda_0) and TerminateSecondary
                const int es = (int)ml[11], a = f->pl_offsets[es];
                Float e = PLEval(f->pl_lambda + a, f->pl_value + a, f->pl_offsets[es + 1] - a, lambda.lambda[0]);
                ieta = e == 0 ? 1.f : e;
                if (lambda.pdf[1] != 0) {
                    for (int i = 1; i < NS; ++i) lambda.pdf[i] = 0;
                    lambda.pdf[0] /= NS;
                }
            }
            lay.top.type = 1;
            lay.top.eta = ieta;
            lay.top.mf.ax = mp[0];
            lay.top.mf.ay = mp[1];
            lay.bottom.type = bx.type == 4 ? 0 : 2;
            lay.bottom.mf.ax = ml[9];
            lay.bottom.mf.ay = ml[10];
            const int es = f->material_spectra[2 * mat], ks = f->material_spectra[2 * mat + 1];
            for (int i = 0; i < NS; ++i) {
                Float l = lambda.lambda[i];
                if (bx.type == 4) {
                    Float r = f->material_constant[mat] ? mc[3] : Sigmoid(mc[0], mc[1], mc[2], l);
                    lay.bottom.R[i] = Clamp(r, 0, 1);
                } else {
                    Float e, k;
                    if (es >= 0) {
                        const int a = f->pl_offsets[es], b = f->pl_offsets[ks];
                        e = PLEval(f->pl_lambda + a, f->pl_value + a, f->pl_offsets[es + 1] - a, l);
                        k = PLEval(f->pl_lambda + b, f->pl_value + b, f->pl_offsets[ks + 1] - b, l);
                    } else {
                        Float r = Clamp(Sigmoid(mc[0], mc[1], mc[2], l), 0, .9999f);
                        e = 1;
                        k = 2 * std::sqrt(r) / std::sqrt(std::max<Float>(0, 1 - r));
                    }
                    lay.bottom.etaS[i] = e / ieta;
                    lay.bottom.kS[i] = k / ieta;
                }
                Float av = ml[8] != 0 ? ml[7] : Sigmoid(ml[4], ml[5], ml[6], l);
                lay.albedo[i] = Clamp(av, 0, 1);
            }
            lay.thickness = std::max<Float>(ml[0], std::numeric_limits<Float>::min());
            lay.g = Clamp(ml[1], -1, 1);
            lay.maxDepth = (int)ml[2];
            lay.nSamples = (int)ml[3];
            if (f->regularize && anyNonSpecular) {
                lay.top.mf.Regularize();
                lay.bottom.mf.Regularize();
            }
        } else if (bx.type == 9) {
            // HairMaterial::GetBxDF (materials.h:380-404) of constant parameters; material_layer
            // holds {mode, sigma_a | color: kind value c0 c1 c2 scale pl, eta, beta_m, beta_n, alpha}
            const float *ml = f->material_layer + 12 * mat;
            // textured eta / beta_m / beta_n / alpha, and eumelanin / pheomelanin as a pair
            // (SigmaAFromConcentration, bxdfs.cpp:553-562: RGBUnboundedSpectrum of the RGB sum)
            Float e = ml[8], bmIn = ml[9], bnIn = ml[10], a = ml[11];
            const int32_t *hn = f->material_hair_tex ? f->material_hair_tex + 6 * mat : nullptr;
            bool conc = false;
            Float cScale = 0, cCo[3] = {0, 0, 0};
            if (hn && (hn[0] >= 0 || hn[1] >= 0 || hn[2] >= 0 || hn[3] >= 0 || hn[4] >= 0)) {
                const OTexCtx hc = tex.Ctx(si);
                if (hn[0] >= 0) e = tex.EvalF(hn[0], hc);
                if (hn[1] >= 0) bmIn = tex.EvalF(hn[1], hc);
                if (hn[2] >= 0) bnIn = tex.EvalF(hn[2], hc);
                if (hn[3] >= 0) a = tex.EvalF(hn[3], hc);
                if (hn[4] >= 0) {
                    const Float ce = std::max<Float>(0, tex.EvalF(hn[4], hc)), cp = std::max<Float>(0, tex.EvalF(hn[5], hc));
                    const Float r = ce * 0.419f + cp * 0.187f, g = ce * 0.697f + cp * 0.4f, b = ce * 1.37f + cp * 1.05f;
                    cScale = 2 * std::max({r, g, b});
                    if (cScale != 0) ORGBCoeffs(r / cScale, g / cScale, b / cScale, cCo);
                    else ORGBCoeffs(0, 0, 0, cCo);
                    conc = true;
                }
            }
            Float bm = std::max<Float>(1e-2, std::min<Float>(1.0, bmIn));
            Float bn = std::max<Float>(1e-2, std::min<Float>(1.0, bnIn));
            Spectrum sig;
            // a textured sigma_a / reflectance (texEval at the hit)
            const int ht = f->material_tex ? f->material_tex[4 * mat] : -1;
            Spectrum hq{};
            if (ht >= 0) hq = tex.EvalS(ht, tex.Ctx(si), lambda);
            for (int i = 0; i < NS; ++i) {
                const Float l = lambda.lambda[i];
                const int kind = (int)ml[1];
                Float q;
                if (conc) q = cScale * Sigmoid(cCo[0], cCo[1], cCo[2], l);
                else if (ht >= 0) q = hq[i];
                else if (kind == 0) q = ml[2];
                else if (kind == 1) q = ml[6] * Sigmoid(ml[3], ml[4], ml[5], l);
                else {
                    const int pl = (int)ml[7], o = f->pl_offsets[pl];
                    q = PLEval(f->pl_lambda + o, f->pl_value + o, f->pl_offsets[pl + 1] - o, l);
                }
                if (ml[0] == 0) {
                    sig[i] = std::max<Float>(0, q);  // ClampZero(sigma_a)
                } else {
                    // HairBxDF::SigmaAFromReflectance (bxdfs.cpp:564-573) of Clamp(color, 0, 1)
                    Float c = Clamp(q, 0, 1);
                    sig[i] = Sqr(CRLog(c) / (5.969f - 0.215f * bn + 2.532f * Sqr(bn) - 10.73f * ohair::Pow<3>(bn) +
                                             5.574f * ohair::Pow<4>(bn) + 0.245f * ohair::Pow<5>(bn)));
                }
            }
            bx.hair.Init(-1 + 2 * si.uv[1], e, sig, bm, bn, a);
        } else if (bx.type == 10) {
            // MeasuredMaterial::GetBxDF (materials.h:931-934): material_layer[0] = the BRDF
            bx.meas.b = &measured[(int)f->material_layer[12 * mat]];
            for (int i = 0; i < NS; ++i) bx.meas.lambda[i] = lambda.lambda[i];
        } else if (bx.type == 7) {
            // DiffuseTransmissionMaterial::GetBxDF (materials.h): Clamp(scale * R | T, 0, 1)
            const float *ml = f->material_layer + 12 * mat;
            const Float scale = f->material_params[4 * mat + 3];
            for (int i = 0; i < NS; ++i) {
                Float l = lambda.lambda[i];
                Float r = f->material_constant[mat] ? mc[3] : Sigmoid(mc[0], mc[1], mc[2], l);
                Float t = ml[8] != 0 ? ml[7] : Sigmoid(ml[4], ml[5], ml[6], l);
                bx.R[i] = Clamp(scale * r, 0, 1);
                bx.Tt[i] = Clamp(scale * t, 0, 1);
            }
        } else if (bx.type == 0) {
            // DiffuseMaterial::GetBxDF: Clamp(texEval(reflectance), 0, 1)
            const int rt = f->material_tex ? f->material_tex[4 * mat] : -1;
            if (rt >= 0) {
                const Spectrum R = tex.EvalS(rt, tex.Ctx(si), lambda);
                for (int i = 0; i < NS; ++i) bx.R[i] = Clamp(R[i], 0, 1);
            } else {
                for (int i = 0; i < NS; ++i) {
                    Float r = f->material_constant[mat] ? mc[3] : Sigmoid(mc[0], mc[1], mc[2], lambda.lambda[i]);
                    bx.R[i] = Clamp(r, 0, 1);
                }
            }
        } else {
            const float *mp = f->material_params + 4 * mat;
            bx.mf.ax = mp[0];  // alphas arrive remapped and clamped (TrowbridgeReitz ctor)
            bx.mf.ay = mp[1];
            const int32_t *mt = f->material_tex ? f->material_tex + 4 * mat : nullptr;
            OTexCtx tctx;
            if (mt && (mt[0] >= 0 || mt[1] >= 0)) tctx = tex.Ctx(si);
            if (mt && mt[1] >= 0) {
                // texEval(uRoughness), texEval(vRoughness), RoughnessToAlpha if remapped,
                // TrowbridgeReitzDistribution(urough, vrough) (materials.h:182-204, :491-511)
                Float ur = tex.EvalF(mt[1], tctx), vr = tex.EvalF(mt[2], tctx);
                if (mt[3]) {
                    ur = std::sqrt(ur);
                    vr = std::sqrt(vr);
                }
                bx.mf = TRDistribution(ur, vr);
            }
            bx.eta = mp[2] == 0 ? 1.f : mp[2];
            if ((bx.type == 1 || bx.type == 6) && f->material_spectra[2 * mat] >= 0) {
                // DielectricMaterial::GetBxDF (materials.cpp:25-49): a spectral eta is taken at
                // lambda_0 and the secondary wavelengths are terminated
                // (SampledWavelengths::TerminateSecondary: pdf = (pdf_0 / n, 0, ..., 0))
                const int es = f->material_spectra[2 * mat], a = f->pl_offsets[es];
                Float e = PLEval(f->pl_lambda + a, f->pl_value + a, f->pl_offsets[es + 1] - a, lambda.lambda[0]);
                bx.eta = e == 0 ? 1.f : e;
                if (lambda.pdf[1] != 0) {
                    for (int i = 1; i < NS; ++i) lambda.pdf[i] = 0;
                    lambda.pdf[0] /= NS;
                }
            }
            if (bx.type == 2 || bx.type == 11) {  // conductor; retroreflective reads the same parameters
                int es = f->material_spectra[2 * mat], ks = f->material_spectra[2 * mat + 1];
                for (int i = 0; i < NS; ++i) {
                    Float l = lambda.lambda[i];
                    if (es >= 0) {
                        const int a = f->pl_offsets[es], b = f->pl_offsets[ks];
                        bx.etaS[i] = PLEval(f->pl_lambda + a, f->pl_value + a, f->pl_offsets[es + 1] - a, l);
                        bx.kS[i] = PLEval(f->pl_lambda + b, f->pl_value + b, f->pl_offsets[ks + 1] - b, l);
                    } else {
                        Float r = Clamp(Sigmoid(mc[0], mc[1], mc[2], l), 0, .9999f);
                        bx.etaS[i] = 1;
                        bx.kS[i] = 2 * std::sqrt(r) / std::sqrt(std::max<Float>(0, 1 - r));
                    }
                }
                if (mt && mt[0] >= 0) {
                    // ConductorMaterial::GetBxDF: r = Clamp(texEval(reflectance), 0, .9999)
                    const Spectrum R = tex.EvalS(mt[0], tctx, lambda);
                    for (int i = 0; i < NS; ++i) {
                        Float r = Clamp(R[i], 0, .9999f);
                        bx.etaS[i] = 1;
                        bx.kS[i] = 2 * std::sqrt(r) / std::sqrt(std::max<Float>(0, 1 - r));
                    }
                }
            }
            if (f->regularize && anyNonSpecular && bx.type != 6) bx.mf.Regularize();  // thin: no-op
        }
        return layered;
    }
    // The camera sample and ray of EvaluatePixelSample (cpu/integrators.cpp:228-242; the wavefront's
    // camera.cpp:31-80 draws the same dimensions): wavelengths, filter, time, lens, render-space ray
    // Option "disablewavelengthjitter" (camera.cpp:55) and "disablepixeljitter" (GetCameraSample,
    // samplers.h:807-812): the draws happen, their values are replaced
    void CameraRay(int px, int py, AnySampler &hs, Wavelengths &lambda, float *weight, Vec &ro, Vec &rd) const {
        Float lu = hs.Get1D();
        if (f->options & 2) lu = 0.5f;
        lambda = Wavelengths::SampleUniform(lu);
        Float fx, fy;
        hs.Pixel2D(&fx, &fy);
        Float ox, oy, fw;
        filt.Sample(fx, fy, &ox, &oy, &fw);  // Filter::Sample(GetPixel2D())
        Float pFilmX = px + ox + 0.5f, pFilmY = py + oy + 0.5f;
        hs.Get1D();  // time
        Float l0, l1;
        hs.Get2D(&l0, &l1);
        if (f->options & 1) {
            pFilmX = px + 0.5f;
            pFilmY = py + 0.5f;
            l0 = l1 = 0.5f;
            fw = 1;
        }
        *weight = fw;
        Vec pCam = Xf(f->camera_from_raster, Vec(pFilmX, pFilmY, 0), true);
        ro = Vec(0, 0, 0);
        rd = Normalize(pCam);
        if (f->lens_radius > 0) {
            Float lx, ly;
            SampleUniformDiskConcentric(l0, l1, &lx, &ly);
            lx *= f->lens_radius;
            ly *= f->lens_radius;
            Float ft = f->focal_distance / rd.z;
            Vec pFocus = ro + rd * ft;
            ro = Vec(lx, ly, 0);
            rd = Normalize(pFocus - ro);
        }
        {
            const float *m = f->render_from_camera;
            Vec oo = Xf(m, ro, true);
            Vec err = gamma(3) * (Abs(Vec(m[0] * ro.x, m[4] * ro.x, m[8] * ro.x)) + Abs(Vec(m[1] * ro.y, m[5] * ro.y, m[9] * ro.y)) +
                                  Abs(Vec(m[2] * ro.z, m[6] * ro.z, m[10] * ro.z)) + Abs(Vec(m[3], m[7], m[11])));
            Vec dd = Xf(m, rd, false);
            Float l2 = LengthSquared(dd);
            if (l2 > 0) oo = oo + dd * (Dot(Abs(dd), err) / l2);
            ro = oo;
            rd = dd;
        }
    }
    // one pixel sample -> sensor RGB and filter weight (film.h:95-100)
    void Li(int px, int py, int sampleIndex, float rgb[3], float *weight) const {
        AnySampler hs = S.Sampler();
        hs.Start(px, py, sampleIndex, 0);
        Wavelengths lambda;
        Vec ro, rd;
        CameraRay(px, py, hs, lambda, weight, ro, rd);
        Spectrum L(0.f), beta(1.f), r_u(1.f), r_l(1.f);
        bool specularBounce = false, anyNonSpecular = false;
        Float etaScale = 1;
        Vec prevP, prevErr, prevN, prevNs;
        // WavefrontPathIntegrator::Render (integrator.cpp:374-432) for one path: iteration wf of
        // the wavefront loop processes this path's ray of path depth `depth`.  Interface
        // crossings continue in the next iteration at the same path depth; the loop ends at
        // wf == maxDepth after emission (so a path may stop before depth reaches maxDepth).
        // WavefrontPathIntegrator's haveMedia (wavefront/integrator.cpp:49-110): media, or any
        // "interface" material (a null Material) -- shadow rays then pass interfaces
        // (IntersectShadowTr) instead of stopping at them
        bool haveMedia = f->n_media > 0;
        for (int m = 0; m < f->n_materials && !haveMedia; ++m) haveMedia = f->material_type[m] == 3;
        int medium = haveMedia ? f->camera_medium : -1;
        int depth = 0;
        auto mediaOf = [&](int prim, int rayMedium, int *in, int *out) {
            *in = *out = rayMedium;
            int pin, pout;
            if (haveMedia && f->n_media > 0 && S.Medium(prim, &pin, &pout) && pin != pout) {
                *in = pin;
                *out = pout;
            }
        };
        auto isInterface = [&](int prim) { return f->material_type[S.Material(prim)] == 3; };
        // Shape::Sample(ctx, u) / PDF(ctx, wi) of area light li (a triangle, sphere or disk)
        auto sampleArea = [&](int li, Vec ref, Vec refErr, Vec refN, Vec refNs, Float u0, Float u1, ShapeSample *ss) {
            const int lp = f->light_prim[li];
            if (lp >= f->n_triangles) return S.shapes[lp - f->n_triangles].Sample(ref, refErr, refN, u0, u1, ss, refNs);
            return TriangleSample(S.P(lp, 0), S.P(lp, 1), S.P(lp, 2), f->tri_flip[lp], ref, refNs, u0, u1, ss, S.Attr(lp));
        };
        auto pdfArea = [&](int li, Vec ref, Vec refErr, Vec refN, Vec refNs, Vec wi) {
            const int lp = f->light_prim[li];
            if (lp >= f->n_triangles) return S.shapes[lp - f->n_triangles].PDF(ref, refErr, refN, wi, refNs);
            return TrianglePDF(S.P(lp, 0), S.P(lp, 1), S.P(lp, 2), f->tri_flip[lp], ref, refErr, refN, refNs, wi, S.Attr(lp));
        };
        // shadow rays: plain occlusion, or TraceTransmittance (wavefront/intersect.h:164-274)
        // whenever the scene has media (interface surfaces are then transparent to them)
        auto shadow = [&](Vec o, Vec d, int med, const Spectrum &Ld, const Spectrum &ru, const Spectrum &rl) {
            TriIsect dummy;
            if (!haveMedia) {
                if (S.Intersect(o, d, 1 - ShadowEpsilon, &dummy, true) < 0) L = L + Ld / (ru + rl).Average();
                return;
            }
            Spectrum T_ray, tu, tl;
            TraceTransmittance(o, d, 1 - ShadowEpsilon, med, lambda, &T_ray, &tu, &tl);
            if (T_ray) L = L + Ld * T_ray / (ru * tu + rl * tl).Average();
        };
        for (int wf = 0;; ++wf) {
            TriIsect ti;
            int prim = S.Intersect(ro, rd, Infinity, &ti, false);
            Interaction si;
            if (prim >= 0) si = S.Interact(prim, ti, rd);
            // GenerateRaySamples: dims 6 + 7 depth (path depth), 6 + 10 depth with subsurface
            // materials, whose three subsurface dimensions follow (samples.cpp:29-66)
            AnySampler h2 = S.Sampler();
            h2.Start(px, py, sampleIndex, 6 + f->dims_per_depth * depth);
            Float dUc = h2.Get1D(), dU0, dU1;
            h2.Get2D(&dU0, &dU1);
            Float iUc = h2.Get1D(), iU0, iU1;
            h2.Get2D(&iU0, &iU1);
            Float rr = h2.Get1D();
            Float sUc = 0, sU0 = 0, sU1 = 0;
            if (f->n_sss > 0) {
                sUc = h2.Get1D();
                h2.Get2D(&sU0, &sU1);
            }
            if (haveMedia && medium >= 0) {
                // SampleMediumInteraction (wavefront/media.cpp:22-247)
                const Float tHit = prim >= 0 ? ti.t : Infinity;
                PCG32 rng(HashFloats(ro.x, ro.y, ro.z, tHit), HashFloats(rd.x, rd.y, rd.z));
                Float uDist = rng.Uniform(), uMode = rng.Uniform();
                bool scattered = false, pushScatter = false;
                Vec pS;
                Spectrum Lm(0.f);
                Spectrum T_maj = SampleTmaj(M, medium, ro, rd, tHit, uDist, rng, lambda,
                                            [&](Vec p, const MediumProps &mp, const Spectrum &sigma_maj, const Spectrum &Tm) {
                    if (depth < S.maxDepth && mp.Le) {
                        Float pr = sigma_maj[0] * Tm[0];
                        Spectrum r_e = r_u * sigma_maj * Tm / pr;
                        if (r_e) Lm = Lm + beta * mp.sigma_a * Tm * mp.Le / (pr * r_e.Average());
                    }
                    Float pAbsorb = mp.sigma_a[0] / sigma_maj[0], pScatter = mp.sigma_s[0] / sigma_maj[0];
                    Float pNull = std::max<Float>(0, 1 - pAbsorb - pScatter);
                    int mode = SampleDiscrete3(pAbsorb, pScatter, pNull, uMode);
                    if (mode == 0) {
                        beta = Spectrum(0.f);
                        return false;
                    }
                    if (mode == 1) {
                        Float pr = Tm[0] * mp.sigma_s[0];
                        beta = beta * (Tm * mp.sigma_s / pr);
                        r_u = r_u * (Tm * mp.sigma_s / pr);
                        pushScatter = bool(beta) && bool(r_u);
                        pS = p;
                        scattered = true;
                        return false;
                    }
                    Spectrum sigma_n = ClampZero(sigma_maj - mp.sigma_a - mp.sigma_s);
                    Float pr = Tm[0] * sigma_n[0];
                    beta = beta * (Tm * sigma_n / pr);
                    if (pr == 0) beta = Spectrum(0.f);
                    r_u = r_u * (Tm * sigma_n / pr);
                    r_l = r_l * (Tm * sigma_maj / pr);
                    uMode = rng.Uniform();
                    return bool(beta) && bool(r_u);
                });
                if (!scattered && beta) {
                    beta = beta * (T_maj / T_maj[0]);
                    r_u = r_u * (T_maj / T_maj[0]);
                    r_l = r_l * (T_maj / T_maj[0]);
                }
                L = L + Lm;
                if (scattered) {
                    if (!pushScatter || wf == S.maxDepth) break;
                    // SampleMediumScattering<HGPhaseFunction> (wavefront/media.cpp:259-352)
                    const Float g = M.Params(medium)[0];
                    const Vec wo = -rd;
                    int li;
                    Float lpmf;
                    DeltaSample ds;
                    const bool sampledL = lights.Sample(pS, Vec(0, 0, 0), dUc, &li, &lpmf);
                    const OEnvLight *E = sampledL ? EnvOf(li) : nullptr;
                    if (E) {
                        // ImageInfiniteLight / PortalImageInfiniteLight::SampleLi from the medium
                        // point (media.cpp:280-305)
                        const int k = li - f->n_area_lights - f->n_point_spot;
                        Vec wi;
                        Float epdf;
                        Spectrum Le;
                        if (E->SampleLi(pS, dU0, dU1, lambda, f->dense_spectra + 311 * f->inf_spectrum[k], f->inf_scale[k],
                                        &wi, &epdf, &Le)) {
                            Vec lp = pS + wi * (2 * f->scene_radius);
                            if (Le) {
                                Float ph = HenyeyGreenstein(Dot(wo, wi), g);
                                Float lightPDF = epdf * lpmf;
                                Spectrum ru = r_u * ph, rl = r_u * lightPDF;
                                shadow(pS, lp - pS, medium, beta * ph * Le, ru, rl);
                            }
                        }
                    } else if (sampledL && li >= f->n_area_lights && DeltaLi(li, pS, lambda, &ds)) {
                        Float ph = HenyeyGreenstein(Dot(wo, ds.wi), g);
                        Spectrum ru = r_u * 0.f, rl = r_u * (1 * lpmf);
                        shadow(pS, ds.p - pS, medium, beta * ph * ds.L, ru, rl);
                    } else if (sampledL && li < f->n_area_lights) {
                        ShapeSample ss;
                        if (sampleArea(li, pS, Vec(0, 0, 0), Vec(0, 0, 0), Vec(0, 0, 0), dU0, dU1, &ss) &&
                            ss.pdf != 0 && LengthSquared(ss.p - pS) != 0) {
                            Vec wi = Normalize(ss.p - pS);
                            const Spectrum Le = SampledAreaL(li, ss.n, wi, lambda, ss.uv);
                            if (Le) {
                                Float ph = HenyeyGreenstein(Dot(wo, wi), g);
                                Spectrum b2 = beta * ph;
                                Float lightPDF = ss.pdf * lpmf;
                                Spectrum ru = r_u * ph, rl = r_u * lightPDF;
                                shadow(pS, ss.p - pS, medium, b2 * Le, ru, rl);
                            }
                        }
                    }
                    Float pdf;
                    Vec wi = SampleHG(wo, g, iU0, iU1, &pdf);
                    if (pdf == 0) break;
                    beta = beta * pdf / pdf;
                    r_l = r_u / pdf;
                    Spectrum rrBeta = beta * etaScale / r_u.Average();
                    if (rrBeta.Max() < 1 && depth >= 1) {
                        Float q = std::max<Float>(0, 1 - rrBeta.Max());
                        if (rr < q) break;
                        beta = beta / (1 - q);
                    }
                    ro = pS;
                    rd = wi;
                    ++depth;
                    specularBounce = false;
                    anyNonSpecular = true;
                    prevP = pS;
                    prevErr = prevN = prevNs = Vec(0, 0, 0);
                    continue;
                }
                if (!beta || !r_u || depth == S.maxDepth) break;
            }
            if (prim < 0) {
                // HandleEscapedRays (integrator.cpp:495-537): uniform infinite lights, whose
                // PDF_Li(allowIncomplete) is 0, and image infinite lights
                for (int k = 0; k < f->n_infinite_lights; ++k) {
                    if (f->inf_distant[k] >= 0) continue;  // DistantLight: not an Infinite-type light
                    const int gi = f->n_area_lights + f->n_point_spot + k;
                    const OEnvLight *E = EnvOf(gi);
                    const float *illum = f->dense_spectra + 311 * f->inf_spectrum[k];
                    Spectrum Le;
                    if (E) {
                        Le = E->LeRay(ro, rd, lambda, illum, f->inf_scale[k]);
                    } else {
                        Le = SampleDense(illum, lambda) * f->inf_scale[k];
                    }
                    if (!Le) continue;
                    if (depth == 0 || specularBounce) L = L + beta * Le / r_u.Average();
                    else {
                        Float pdfLi = 0;
                        if (E) pdfLi = E->PdfLi(prevP, rd);
                        Spectrum rl = r_l * lights.PMF(prevP, prevNs, gi) * pdfLi;
                        L = L + beta * Le / (r_u + rl).Average();
                    }
                }
                break;
            }
            int mIn, mOut;
            mediaOf(prim, medium, &mIn, &mOut);
            if (isInterface(prim)) {
                // Material "interface": SpawnRay(ray.d) into the next wavefront iteration, same depth
                if (wf == S.maxDepth) break;
                ro = OffsetRayOrigin(si.p, si.err, si.n, rd);
                medium = DotN(si.n, rd) > 0 ? mOut : mIn;
                continue;
            }
            // HandleEmissiveIntersection
            int light = S.Light(prim);
            if (light >= 0) {
                const Spectrum Le = AreaL(light, si.n, si.wo, lambda, si.uv);
                if (Le) {
                    if (depth == 0 || specularBounce) L = L + beta * Le / r_u.Average();
                    else {
                        Float lightChoicePDF = lights.PMF(prevP, prevNs, light);
                        Float lightPDF = lightChoicePDF * pdfArea(light, prevP, prevErr, prevN, prevNs, -si.wo);
                        Spectrum rl = r_l * lightPDF;
                        L = L + beta * Le / (r_u + rl).Average();
                    }
                }
            }
            if (wf == S.maxDepth) break;
            // Material::GetBxDF (materials.h:466-471 diffuse, :182-204 dielectric, :491-511 conductor)
            const int mat = ResolveMix(S.Material(prim), si);
            BxDF bx;
            LayeredBxDF lay;
            const bool layered = MakeBSDF(mat, lambda, anyNonSpecular, si, bx, lay);
            Vec fx_ = Normalize(si.dpdus), fz = si.ns, fy_ = Cross(fz, fx_);
            auto toLocal = [&](Vec v) { return Vec(Dot(v, fx_), Dot(v, fy_), Dot(v, fz)); };
            auto fromLocal = [&](Vec v) { return fx_ * v.x + fy_ * v.y + fz * v.z; };
            Vec woL = toLocal(si.wo);
            const int flags = layered ? lay.Flags() : bx.Flags();
            Spectrum oldBeta = beta;
            bool haveNext = false, nextSpecular = false, toSss = false;
            Vec nextO, nextD;
            Spectrum nb;
            Spectrum nrl;
            Float nextEtaScale = etaScale;
            // BSDF::Sample_f (bsdf.h:89-116), then surfscatter.cpp:183-250
            BSDFSample bs;
            const bool sampled = layered ? lay.Sample_f(woL, iUc, iU0, iU1, &bs, true) : bx.Sample_f(woL, iUc, iU0, iU1, &bs);
            if (woL.z != 0 && flags && sampled && bs.f && bs.pdf != 0 && bs.wi.z != 0) {
                Vec wi = fromLocal(bs.wi);
                nb = beta * bs.f * AbsDotN(si.ns, wi) / bs.pdf;
                // pdfIsProportional (layered): r_l = r_u / BSDF::PDF(wo, wi), wi back in the local frame
                nrl = layered ? r_u / lay.PDF(woL, toLocal(wi), true) : r_u / bs.pdf;
                if (bs.flags & BxT) nextEtaScale *= Sqr(bs.eta);
                Spectrum rrBeta = nb * nextEtaScale / r_u.Average();
                if (rrBeta.Max() < 1 && depth >= 1) {
                    Float q = std::max<Float>(0, 1 - rrBeta.Max());
                    if (rr < q) nb = Spectrum(0.f);
                    else nb = nb / (1 - q);
                }
                if (nb) {
                    haveNext = true;
                    // a subsurface material's transmitted sample enters the BSSRDF stage
                    toSss = (bs.flags & BxT) && f->material_sss && f->material_sss[mat] >= 0;
                    nextSpecular = bs.flags & BxSpecular;
                    nextO = OffsetRayOrigin(si.p, si.err, si.n, wi);
                    nextD = wi;
                }
            }
            // light sampling + shadow ray (surfscatter.cpp:252-326), IsNonSpecular(flags)
            if (flags & (BxDiffuse | BxGlossy)) {
                Vec cp = si.p, cpErr = si.err;  // LightSampleContext: the offset point is exact
                bool refl = flags & BxR, trans = flags & BxT;
                if (refl && !trans) cp = OffsetRayOrigin(si.p, si.err, si.n, si.wo), cpErr = Vec(0, 0, 0);
                else if (trans && refl) cp = OffsetRayOrigin(si.p, si.err, si.n, -si.wo), cpErr = Vec(0, 0, 0);
                int li;
                Float lpmf;
                DeltaSample ds;
                const bool sampledL = lights.Sample(cp, si.ns, dUc, &li, &lpmf);
                const OEnvLight *E = sampledL ? EnvOf(li) : nullptr;
                if (E) {
                    // ImageInfiniteLight::SampleLi(allowIncompletePDF) (lights.h:594-618), or the
                    // portal light's (lights.cpp:1257-1281): a light point 2 sceneRadius away
                    // without error bounds or normal
                    const int k = li - f->n_area_lights - f->n_point_spot;
                    Vec wi;
                    Float epdf;
                    Spectrum Le;
                    if (E->SampleLi(cp, dU0, dU1, lambda, f->dense_spectra + 311 * f->inf_spectrum[k], f->inf_scale[k], &wi,
                                    &epdf, &Le)) {
                        Vec lp = cp + wi * (2 * f->scene_radius);
                        Vec wiL = toLocal(wi);
                        Spectrum fv = woL.z == 0 ? Spectrum(0.f) : layered ? lay.f(woL, wiL, true) : bx.f(woL, wiL);
                        if (Le && fv) {
                            Spectrum b2 = oldBeta * fv * AbsDotN(si.ns, wi);
                            Float lightPDF = epdf * lpmf;
                            Float bsdfPDF = woL.z == 0 ? 0 : layered ? lay.PDF(woL, wiL, true) : bx.PDF(woL, wiL);
                            Spectrum ru = r_u * bsdfPDF, rl = r_u * lightPDF;
                            Vec pf = OffsetRayOrigin(si.p, si.err, si.n, lp - si.p);
                            shadow(pf, lp - pf, DotN(si.n, lp - pf) > 0 ? mOut : mIn, b2 * Le, ru, rl);
                        }
                    }
                } else if (sampledL && li >= f->n_area_lights && DeltaLi(li, cp, lambda, &ds)) {
                    // a delta light: pdf 1, no BSDF MIS weight (IsDeltaLight), the light point
                    // has no error bounds and no normal (SpawnRayTo leaves it where it is)
                    Vec wi = ds.wi, wiL = toLocal(wi);
                    Spectrum fv = woL.z == 0 ? Spectrum(0.f) : layered ? lay.f(woL, wiL, true) : bx.f(woL, wiL);
                    if (fv) {
                        Spectrum b2 = oldBeta * fv * AbsDotN(si.ns, wi);
                        Float lightPDF = 1 * lpmf;
                        Spectrum ru = r_u * 0.f, rl = r_u * lightPDF;
                        Vec pf = OffsetRayOrigin(si.p, si.err, si.n, ds.p - si.p);
                        shadow(pf, ds.p - pf, DotN(si.n, ds.p - pf) > 0 ? mOut : mIn, b2 * ds.L, ru, rl);
                    }
                } else if (sampledL && li < f->n_area_lights) {
                    ShapeSample ss;
                    if (sampleArea(li, cp, cpErr, si.n, si.ns, dU0, dU1, &ss) && ss.pdf != 0 &&
                        LengthSquared(ss.p - cp) != 0) {
                        Vec wi = Normalize(ss.p - cp);
                        const Spectrum Le = SampledAreaL(li, ss.n, wi, lambda, ss.uv);
                        if (Le) {
                            Vec wiL = toLocal(wi);
                            Spectrum fv = woL.z == 0 ? Spectrum(0.f)  // BSDF::f (bsdf.h:60-70)
                                          : layered ? lay.f(woL, wiL, true) : bx.f(woL, wiL);
                            if (fv) {
                                Spectrum b2 = oldBeta * fv * AbsDotN(si.ns, wi);
                                Float lightPDF = ss.pdf * lpmf;
                                Float bsdfPDF = woL.z == 0 ? 0 : layered ? lay.PDF(woL, wiL, true) : bx.PDF(woL, wiL);
                                Spectrum ru = r_u * bsdfPDF, rl = r_u * lightPDF;
                                Spectrum Ld = b2 * Le;
                                // SpawnRayTo(pi, n, time, pLight.pi, pLight.n) (ray.h:106-111)
                                Vec pf = OffsetRayOrigin(si.p, si.err, si.n, ss.p - si.p);
                                Vec pt = OffsetRayOrigin(ss.p, ss.err, ss.n, pf - ss.p);
                                shadow(pf, pt - pf, DotN(si.n, pt - pf) > 0 ? mOut : mIn, Ld, ru, rl);
                            }
                        }
                    }
                }
            }
            if (haveNext && toSss) {
                // SampleSubsurface (wavefront/subsurface.cpp:18-206): GetBSSRDF, SampleSp with
                // the subsurface samples, IntersectOneRandom over the probe segment, then the
                // exit vertex's NormalizedFresnelBxDF: indirect ray and light sample
                const int k = f->material_sss[mat];
                const float *P = f->sss_params + 20 * k;
                const float *T = sssTables[k].data();
                osss::BSSRDF bd;
                bd.rho = T;
                bd.rad = T + osss::NRho;
                bd.prof = bd.rad + osss::NRad;
                bd.rhoEff = bd.prof + osss::NRho * osss::NRad;
                bd.cdf = bd.rhoEff + osss::NRho;
                bd.po = si.p;
                bd.ns = si.ns;
                auto specAt = [&](const float *q, Float lam) -> Float {
                    const int kind = (int)q[0];
                    if (kind == 0) return q[1];
                    if (kind == 1) return q[5] * Sigmoid(q[2], q[3], q[4], lam);
                    const int pl = (int)q[6], a = f->pl_offsets[pl];
                    return PLEval(f->pl_lambda + a, f->pl_value + a, f->pl_offsets[pl + 1] - a, lam);
                };
                // a textured reflectance: texEval at the entry (materials.h:823-841)
                const int rt = f->material_tex ? f->material_tex[4 * mat] : -1;
                Spectrum rTex{};
                if (rt >= 0 && P[0] != 0) rTex = tex.EvalS(rt, tex.Ctx(si), lambda);
                // textured sigma_a, and sigma_s | mfp (Unbounded), the same way
                const int sat = f->material_sss_tex ? f->material_sss_tex[2 * mat] : -1;
                const int sbt = f->material_sss_tex ? f->material_sss_tex[2 * mat + 1] : -1;
                Spectrum aTex{}, bTex{};
                if (sat >= 0) aTex = tex.EvalS(sat, tex.Ctx(si), lambda);
                if (sbt >= 0) bTex = tex.EvalS(sbt, tex.Ctx(si), lambda);
                for (int i = 0; i < NS; ++i) {
                    const Float lam = lambda.lambda[i];
                    Float sa, ss;
                    if (P[0] == 0) {
                        sa = std::max<Float>(0, P[1] * (sat >= 0 ? aTex[i] : specAt(P + 4, lam)));
                        ss = std::max<Float>(0, P[1] * (sbt >= 0 ? bTex[i] : specAt(P + 11, lam)));
                    } else {
                        const Float mfree = std::max<Float>(0, P[1] * (sbt >= 0 ? bTex[i] : specAt(P + 11, lam)));
                        const Float refl = rt >= 0 ? rTex[i] : specAt(P + 4, lam);
                        const Float rh = osss::InvertCatmullRom(bd.rho, bd.rhoEff, osss::NRho, Clamp(refl, 0, 1));
                        ss = rh / mfree;
                        sa = (1 - rh) / mfree;
                    }
                    bd.sigma_t[i] = sa + ss;
                    bd.rhoS[i] = bd.sigma_t[i] != 0 ? ss / bd.sigma_t[i] : 0;
                }
                Vec p0, p1;
                if (!bd.SampleSp(sUc, sU0, sU1, &p0, &p1)) break;
                TriIsect cti{};
                Vec cdir;
                Float resPdf;
                const int chosen = ProbeOneRandom(S, p0, p1, mat, &cti, &cdir, &resPdf);
                if (chosen < 0) break;
                const Interaction ex = S.Interact(chosen, cti, cdir);
                const Spectrum Sp = bd.Sr(Length(bd.po - ex.p)), pdfSp = bd.PdfSp(ex.p, ex.n);
                if (!Sp || !pdfSp) break;
                const Float pr = resPdf * pdfSp[0];
                const Spectrum betap = nb * Sp / pr;
                const Spectrum ru2 = r_u * pdfSp / pdfSp[0];
                const Float eta = P[2], fc = P[3];
                Vec ex_ = Normalize(ex.dpdus), ez_ = ex.ns, ey_ = Cross(ez_, ex_);
                auto toL = [&](Vec v) { return Vec(Dot(v, ex_), Dot(v, ey_), Dot(v, ez_)); };
                const Vec woS = toL(ex.ns);
                auto nfF = [&](Vec wiL) -> Float {  // NormalizedFresnelBxDF::f (bxdfs.h:1249-1261)
                    if (!(woS.z * wiL.z > 0)) return 0;
                    const Float fv = (1 - FrDielectric(wiL.z, eta)) / (fc * Pi);
                    return fv * Sqr(eta);
                };
                auto nfPdf = [&](Vec wiL) -> Float { return woS.z * wiL.z > 0 ? std::abs(wiL.z) * InvPi : 0; };
                bool haveNext2 = false;
                Spectrum nb2, nrl2;
                Vec nO, nD;
                if (woS.z != 0) {
                    Vec wiL = SampleCosineHemisphere(iU0, iU1);
                    if (woS.z < 0) wiL.z *= -1;
                    const Float fv = nfF(wiL), pv = nfPdf(wiL);
                    if (fv != 0 && pv != 0 && wiL.z != 0) {
                        const Vec wi = ex_ * wiL.x + ey_ * wiL.y + ez_ * wiL.z;
                        Spectrum b = betap * fv * AbsDotN(ex.ns, wi) / pv;
                        const Spectrum rl = ru2 / pv;
                        const Spectrum rrBeta = b * nextEtaScale / ru2.Average();
                        if (rrBeta.Max() < 1 && depth > 1) {
                            const Float q = std::max<Float>(0, 1 - rrBeta.Max());
                            if (rr < q) b = Spectrum(0.f);
                            else b = b / (1 - q);
                        }
                        if (b) {
                            haveNext2 = true;
                            nb2 = b;
                            nrl2 = rl;
                            nO = OffsetRayOrigin(ex.p, ex.err, ex.n, wi);
                            nD = wi;
                        }
                    }
                }
                // direct lighting from the exit point (LightSampleContext(pi, n, ns), no offset)
                int li;
                Float lpmf;
                DeltaSample ds;
                const bool sampledL = woS.z != 0 && lights.Sample(ex.p, ex.ns, dUc, &li, &lpmf);
                const OEnvLight *E = sampledL ? EnvOf(li) : nullptr;
                if (E) {
                    const int kk = li - f->n_area_lights - f->n_point_spot;
                    Vec wi;
                    Float epdf;
                    Spectrum Le;
                    if (E->SampleLi(ex.p, dU0, dU1, lambda, f->dense_spectra + 311 * f->inf_spectrum[kk], f->inf_scale[kk],
                                    &wi, &epdf, &Le)) {
                        Vec lp = ex.p + wi * (2 * f->scene_radius);
                        const Float fv = nfF(toL(wi));
                        if (Le && fv != 0) {
                            Spectrum b2 = betap * fv * AbsDotN(ex.ns, wi);
                            Float lightPDF = epdf * lpmf;
                            Spectrum ru = ru2 * nfPdf(toL(wi)), rl = ru2 * lightPDF;
                            Vec pf = OffsetRayOrigin(ex.p, ex.err, ex.n, lp - ex.p);
                            shadow(pf, lp - pf, DotN(ex.n, lp - pf) > 0 ? mOut : mIn, b2 * Le, ru, rl);
                        }
                    }
                } else if (sampledL && li >= f->n_area_lights && DeltaLi(li, ex.p, lambda, &ds)) {
                    const Float fv = nfF(toL(ds.wi));
                    if (fv != 0) {
                        Spectrum b2 = betap * fv * AbsDotN(ex.ns, ds.wi);
                        Spectrum ru = ru2 * 0.f, rl = ru2 * (1 * lpmf);
                        Vec pf = OffsetRayOrigin(ex.p, ex.err, ex.n, ds.p - ex.p);
                        shadow(pf, ds.p - pf, DotN(ex.n, ds.p - pf) > 0 ? mOut : mIn, b2 * ds.L, ru, rl);
                    }
                } else if (sampledL && li < f->n_area_lights) {
                    ShapeSample ss;
                    if (sampleArea(li, ex.p, ex.err, ex.n, ex.ns, dU0, dU1, &ss) && ss.pdf != 0 &&
                        LengthSquared(ss.p - ex.p) != 0) {
                        Vec wi = Normalize(ss.p - ex.p);
                        const Spectrum Le = SampledAreaL(li, ss.n, wi, lambda, ss.uv);
                        if (Le) {
                            const Float fv = nfF(toL(wi));
                            if (fv != 0) {
                                Spectrum b2 = betap * fv * AbsDotN(ex.ns, wi);
                                Float lightPDF = ss.pdf * lpmf;
                                Spectrum ru = ru2 * nfPdf(toL(wi)), rl = ru2 * lightPDF;
                                Vec pf = OffsetRayOrigin(ex.p, ex.err, ex.n, ss.p - ex.p);
                                Vec pt = OffsetRayOrigin(ss.p, ss.err, ss.n, pf - ss.p);
                                shadow(pf, pt - pf, DotN(ex.n, pt - pf) > 0 ? mOut : mIn, b2 * Le, ru, rl);
                            }
                        }
                    }
                }
                if (!haveNext2) break;
                beta = nb2;
                r_u = ru2;
                r_l = nrl2;
                specularBounce = false;
                anyNonSpecular = true;
                etaScale = nextEtaScale;
                prevP = ex.p;
                prevErr = ex.err;
                prevN = ex.n;
                prevNs = ex.ns;
                medium = DotN(ex.n, nD) > 0 ? mOut : mIn;
                ro = nO;
                rd = nD;
                ++depth;
                continue;
            }
            if (!haveNext) break;
            beta = nb;
            r_l = nrl;
            specularBounce = nextSpecular;
            anyNonSpecular = anyNonSpecular || !nextSpecular;
            etaScale = nextEtaScale;
            prevP = si.p;
            prevErr = si.err;
            prevN = si.n;
            prevNs = si.ns;
            medium = DotN(si.n, nextD) > 0 ? mOut : mIn;
            ro = nextO;
            rd = nextD;
            ++depth;
        }
        // PixelSensor::ToSensorRGB (cie1931): L / pdf, averaged against X/Y/Z bars
        Spectrum Lp;
        for (int i = 0; i < NS; ++i) Lp[i] = lambda.pdf[i] != 0 ? L[i] / lambda.pdf[i] : 0;
        Spectrum xb = SampleDense(f->sensor_xyz, lambda), yb = SampleDense(f->sensor_xyz + 311, lambda),
                 zb = SampleDense(f->sensor_xyz + 622, lambda);
        rgb[0] = f->imaging_ratio * (xb * Lp).Average();
        rgb[1] = f->imaging_ratio * (yb * Lp).Average();
        rgb[2] = f->imaging_ratio * (zb * Lp).Average();
    }

    // PathIntegrator::Li (cpu/integrators.cpp:629-762) with SampleLd (:764-805) for one pixel
    // sample -- configs[0]'s CPU integrator, a different estimator of the same image as the
    // wavefront volpath above: power-heuristic MIS, Russian roulette after the second bounce, and
    // the CPU sampler's sequential dimensions (light choice 1D + light point 2D only when the
    // BSDF is non-specular, BSDF 1D + 2D, the roulette 1D only when it is tested).  Surfaces only
    // (a scene with media returns false).
    bool PathLi(int px, int py, int sampleIndex, float rgb[3], float *weight) const {
        if (f->n_media > 0) return false;
        AnySampler hs = S.Sampler();
        hs.Start(px, py, sampleIndex, 0);
        Wavelengths lambda;
        Vec ro, rd;
        CameraRay(px, py, hs, lambda, weight, ro, rd);
        Spectrum L(0.f), beta(1.f);
        int depth = 0;
        Float p_b = 0, etaScale = 1;
        bool specularBounce = false, anyNonSpecular = false;
        Vec prevP, prevErr, prevN, prevNs;
        TriIsect dummy;
        auto unoccluded = [&](Vec pf, Vec pt) { return S.Intersect(pf, pt - pf, 1 - ShadowEpsilon, &dummy, true) < 0; };
        while (true) {
            TriIsect ti;
            const int prim = S.Intersect(ro, rd, Infinity, &ti, false);
            if (prim < 0) {
                // escaped: every infinite light's Le, MIS-weighted against the BSDF sample
                for (int k = 0; k < f->n_infinite_lights; ++k) {
                    if (f->inf_distant[k] >= 0) continue;  // DistantLight is not in infiniteLights
                    const int gi = f->n_area_lights + f->n_point_spot + k;
                    const OEnvLight *E = EnvOf(gi);
                    const float *illum = f->dense_spectra + 311 * f->inf_spectrum[k];
                    Spectrum Le;
                    Float pdfLi = 0;
                    if (E) {
                        Le = E->LeRay(ro, rd, lambda, illum, f->inf_scale[k]);
                        pdfLi = E->PdfLi(prevP, rd);
                    } else {
                        Le = SampleDense(illum, lambda) * f->inf_scale[k];
                    }
                    if (depth == 0 || specularBounce) L = L + beta * Le;
                    else {
                        const Float p_l = lights.PMF(prevP, prevNs, gi) * pdfLi;
                        L = L + beta * PowerHeuristic(1, p_b, 1, p_l) * Le;
                    }
                }
                break;
            }
            Interaction si = S.Interact(prim, ti, rd);
            // emission at the hit (SurfaceInteraction::Le -> DiffuseAreaLight::L)
            const int light = S.Light(prim);
            if (light >= 0) {
                const Spectrum Le = AreaL(light, si.n, si.wo, lambda, si.uv);
                if (Le) {
                    if (depth == 0 || specularBounce) L = L + beta * Le;
                    else {
                        const int lp = f->light_prim[light];
                        const Float pdfA = lp >= f->n_triangles
                            ? S.shapes[lp - f->n_triangles].PDF(prevP, prevErr, prevN, -si.wo, prevNs)
                            : TrianglePDF(S.P(lp, 0), S.P(lp, 1), S.P(lp, 2), f->tri_flip[lp], prevP, prevErr, prevN,
                                          prevNs, -si.wo, S.Attr(lp));
                        const Float p_l = lights.PMF(prevP, prevNs, light) * pdfA;
                        L = L + beta * PowerHeuristic(1, p_b, 1, p_l) * Le;
                    }
                }
            }
            // GetBSDF; an interface (no BSDF) is skipped at the same depth
            const int mat0 = S.Material(prim);
            if (f->material_type[mat0] == 3) {
                specularBounce = true;
                ro = OffsetRayOrigin(si.p, si.err, si.n, rd);
                continue;
            }
            const int mat = ResolveMix(mat0, si);
            BxDF bx;
            LayeredBxDF lay;
            const bool layered = MakeBSDF(mat, lambda, anyNonSpecular, si, bx, lay);
            if (depth++ == S.maxDepth) break;
            Vec fx_ = Normalize(si.dpdus), fz = si.ns, fy_ = Cross(fz, fx_);
            auto toLocal = [&](Vec v) { return Vec(Dot(v, fx_), Dot(v, fy_), Dot(v, fz)); };
            auto fromLocal = [&](Vec v) { return fx_ * v.x + fy_ * v.y + fz * v.z; };
            const Vec woL = toLocal(si.wo);
            const int flags = layered ? lay.Flags() : bx.Flags();
            auto bsdfF = [&](Vec wi) {
                const Vec wiL = toLocal(wi);
                return woL.z == 0 ? Spectrum(0.f) : layered ? lay.f(woL, wiL, true) : bx.f(woL, wiL);
            };
            auto bsdfPDF = [&](Vec wi) {
                const Vec wiL = toLocal(wi);
                return woL.z == 0 ? Float(0) : layered ? lay.PDF(woL, wiL, true) : bx.PDF(woL, wiL);
            };
            // SampleLd: light choice, light point, BSDF * |cos|, visibility, MIS
            if (flags & (BxDiffuse | BxGlossy)) {
                Vec cp = si.p, cpErr = si.err;
                const bool refl = flags & BxR, trans = flags & BxT;
                if (refl && !trans) cp = OffsetRayOrigin(si.p, si.err, si.n, si.wo), cpErr = Vec(0, 0, 0);
                else if (trans && !refl) cp = OffsetRayOrigin(si.p, si.err, si.n, -si.wo), cpErr = Vec(0, 0, 0);
                const Float uc = hs.Get1D();
                Float u0, u1;
                hs.Get2D(&u0, &u1);
                int li;
                Float lpmf;
                if (lights.Sample(cp, si.ns, uc, &li, &lpmf)) {
                    Spectrum Le(0.f);
                    Vec wi, pf, pt;
                    Float pdf = 0;
                    bool delta = false;
                    DeltaSample ds;
                    const OEnvLight *E = EnvOf(li);
                    if (E) {
                        const int k = li - f->n_area_lights - f->n_point_spot;
                        if (E->SampleLi(cp, u0, u1, lambda, f->dense_spectra + 311 * f->inf_spectrum[k], f->inf_scale[k], &wi,
                                        &pdf, &Le)) {
                            pt = cp + wi * (2 * f->scene_radius);
                            pf = OffsetRayOrigin(si.p, si.err, si.n, pt - si.p);
                        }
                    } else if (li >= f->n_area_lights) {
                        if (DeltaLi(li, cp, lambda, &ds)) {
                            wi = ds.wi;
                            Le = ds.L;
                            pdf = 1;
                            delta = true;
                            pf = OffsetRayOrigin(si.p, si.err, si.n, ds.p - si.p);
                            pt = ds.p;
                        }
                    } else {
                        ShapeSample ss;
                        const int lp = f->light_prim[li];
                        const bool ok = lp >= f->n_triangles
                            ? S.shapes[lp - f->n_triangles].Sample(cp, cpErr, si.n, u0, u1, &ss, si.ns)
                            : TriangleSample(S.P(lp, 0), S.P(lp, 1), S.P(lp, 2), f->tri_flip[lp], cp, si.ns, u0, u1, &ss,
                                             S.Attr(lp));
                        if (ok && ss.pdf != 0 && LengthSquared(ss.p - cp) != 0) {
                            wi = Normalize(ss.p - cp);
                            Le = SampledAreaL(li, ss.n, wi, lambda, ss.uv);
                            pdf = ss.pdf;
                            pf = OffsetRayOrigin(si.p, si.err, si.n, ss.p - si.p);
                            pt = OffsetRayOrigin(ss.p, ss.err, ss.n, pf - ss.p);
                        }
                    }
                    if (Le && pdf != 0) {
                        const Spectrum fv = bsdfF(wi) * AbsDotN(si.ns, wi);
                        if (fv && unoccluded(pf, pt)) {
                            const Float p_l = lpmf * pdf;
                            if (delta) L = L + beta * (Le * fv / p_l);
                            else {
                                const Float w_l = PowerHeuristic(1, p_l, 1, bsdfPDF(wi));
                                L = L + beta * (Le * w_l * fv / p_l);  // w_l * L[i]: one product, same bits
                            }
                        }
                    }
                }
            }
            // BSDF sample -> next ray, then Russian roulette
            const Float ucB = hs.Get1D();
            Float b0, b1;
            hs.Get2D(&b0, &b1);
            BSDFSample bs;
            const bool sampled = woL.z != 0 && flags &&
                                 (layered ? lay.Sample_f(woL, ucB, b0, b1, &bs, true) : bx.Sample_f(woL, ucB, b0, b1, &bs));
            if (!sampled || !bs.f || bs.pdf == 0 || bs.wi.z == 0) break;
            const Vec wi = fromLocal(bs.wi);
            beta = beta * bs.f * AbsDotN(si.ns, wi) / bs.pdf;
            p_b = layered ? bsdfPDF(wi) : bs.pdf;  // pdfIsProportional: BSDF::PDF
            specularBounce = bs.flags & BxSpecular;
            anyNonSpecular = anyNonSpecular || !specularBounce;
            if (bs.flags & BxT) etaScale *= Sqr(bs.eta);
            prevP = si.p;
            prevErr = si.err;
            prevN = si.n;
            prevNs = si.ns;
            ro = OffsetRayOrigin(si.p, si.err, si.n, wi);
            rd = wi;
            const Spectrum rrBeta = beta * etaScale;
            if (rrBeta.Max() < 1 && depth > 1) {
                const Float q = std::max<Float>(0, 1 - rrBeta.Max());
                if (hs.Get1D() < q) break;
                beta = beta / (1 - q);
            }
        }
        Spectrum Lp;
        for (int i = 0; i < NS; ++i) Lp[i] = lambda.pdf[i] != 0 ? L[i] / lambda.pdf[i] : 0;
        Spectrum xb = SampleDense(f->sensor_xyz, lambda), yb = SampleDense(f->sensor_xyz + 311, lambda),
                 zb = SampleDense(f->sensor_xyz + 622, lambda);
        rgb[0] = f->imaging_ratio * (xb * Lp).Average();
        rgb[1] = f->imaging_ratio * (yb * Lp).Average();
        rgb[2] = f->imaging_ratio * (zb * Lp).Average();
        return true;
    }
};

}  // namespace oracle

using namespace oracle;

extern "C" {
// the oracle's Catmull-Rom restatements (tests against tests/golden "catmull_rom"): op 0
// CatmullRomWeights over nodes1 -> [n][6] ok offset w0..w3; 1 InvertCatmullRom(nodes1, values)
// -> [n]; 2 IntegrateCatmullRom-free (unused); 3 SampleCatmullRom2D(x[2i] alpha, x[2i+1] u) -> [n]
void oracle_catmull_rom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                        const float *cdf, const float *x, int n, float *out) {
    for (int i = 0; i < n; ++i) {
        if (op == 0) {
            int off = 0;
            Float w[4] = {0, 0, 0, 0};
            const bool ok = osss::Weights(nodes1, n1, x[i], &off, w);
            const float r[6] = {ok ? 1.f : 0.f, (float)(ok ? off : 0), w[0], w[1], w[2], w[3]};
            std::copy(r, r + 6, out + 6 * i);
        } else if (op == 1) {
            out[i] = osss::InvertCatmullRom(nodes1, values, n1, x[i]);
        } else if (op == 3) {
            out[i] = osss::SampleCatmullRom2D(nodes1, n1, nodes2, n2, values, cdf, x[2 * i], x[2 * i + 1]);
        }
    }
}
// the oracle's HairBxDF (ohair::Hair) on queries laid out as pbrt_debug_hair's: in[16] {h, eta,
// beta_m, beta_n, alpha, sigma_a0, wo, wi, uc, u0, u1, slope} -> out[68] {f[NS], PDF, ok, wi,
// pdf, f[NS]}, in the current math mode
void oracle_hair_eval(const float *in, int n, float *out) {
    for (int k = 0; k < n; ++k) {
        const float *q = in + 16 * k;
        float *o = out + (2 * NS + 6) * k;
        Spectrum sa;
        for (int i = 0; i < NS; ++i) sa[i] = q[5] + q[15] * (float)i;
        ohair::Hair h;
        h.Init(q[0], q[1], sa, q[2], q[3], q[4]);
        const Vec wo(q[6], q[7], q[8]), wi(q[9], q[10], q[11]);
        const Spectrum fv = h.f(wo, wi);
        for (int i = 0; i < NS; ++i) o[i] = fv[i];
        o[NS] = h.PDF(wo, wi);
        float *s = o + NS + 1;
        std::fill(s, s + 5 + NS, 0.f);
        BSDFSample bs;
        // BSDF::Sample_f's checks (bsdf.h:89-116)
        if (h.Sample_f(wo, q[12], q[13], q[14], &bs) && bs.f && bs.pdf != 0 && bs.wi.z != 0) {
            s[0] = 1;
            s[1] = bs.wi.x, s[2] = bs.wi.y, s[3] = bs.wi.z;
            s[4] = bs.pdf;
            for (int i = 0; i < NS; ++i) s[5 + i] = bs.f[i];
        }
    }
}
// PiecewiseLinear2D<dim> (util/sampling.h:1299-1749) alone, as pbrt_debug_pl2d: the table over
// data [pr0][pr1][ys][xs] (dim 2; normalised, CDF iff cdf) and per query q[6] {u0, u1, px, py, p0, p1}
// -> out[7] {Sample x, y, pdf, Invert x, y, pdf, Evaluate} (Sample / Invert zero without a CDF)
int oracle_pl2d(int dim, int cdf, const float *data, int xs, int ys, const int *pr, const float *pv0,
                const float *pv1, const float *q, int n, float *out) {
    if ((dim != 0 && dim != 2) || xs < 2 || ys < 2) return -1;
    std::vector<float> pv[3];
    if (dim == 2) {
        pv[0].assign(pv0, pv0 + pr[0]);
        pv[1].assign(pv1, pv1 + pr[1]);
    }
    omeas::Table t;
    t.Build(data, xs, ys, dim, pv, true, cdf != 0);
    for (int k = 0; k < n; ++k) {
        const float *x = q + 6 * k;
        float *o = out + 7 * k;
        std::fill(o, o + 7, 0.f);
        const Float par[2] = {x[4], x[5]};
        if (cdf) {
            t.Sample(x[0], x[1], par, &o[0], &o[1], &o[2]);
            t.Invert(x[2], x[3], par, &o[3], &o[4], &o[5]);
        }
        o[6] = t.Evaluate(x[2], x[3], par);
    }
    return 0;
}
// WindowedPiecewiseConstant2D (util/sampling.h:890-980) alone, as pbrt_debug_windowed2d: the
// function f [n][n] with its SummedAreaTable; per query q[8] {u0, u1, b0, b1, b2, b3, qx, qy}
// -> out[5] {ok, x, y, pdf, PDF(q, b)}
int oracle_windowed2d(const float *f, int n, const float *q, int k, float *out) {
    if (n < 1) return -1;
    OEnvLight E;
    E.n = n;
    E.pfunc.assign(f, f + (size_t)n * n);
    E.psat.assign((size_t)n * n, 0.);
    auto S = [&](int x, int y) -> double & { return E.psat[(size_t)y * n + x]; };
    auto F = [&](int x, int y) { return E.pfunc[(size_t)y * n + x]; };
    S(0, 0) = F(0, 0);
    for (int x = 1; x < n; ++x) S(x, 0) = F(x, 0) + S(x - 1, 0);
    for (int y = 1; y < n; ++y) S(0, y) = F(0, y) + S(0, y - 1);
    for (int y = 1; y < n; ++y)
        for (int x = 1; x < n; ++x) S(x, y) = (F(x, y) + S(x - 1, y) + S(x, y - 1) - S(x - 1, y - 1));
    for (int i = 0; i < k; ++i) {
        const float *x = q + 8 * i;
        float *o = out + 5 * i;
        std::fill(o, o + 5, 0.f);
        const Float b[4] = {x[2], x[3], x[4], x[5]};
        Float px, py, pdf;
        if (E.WindowedSample(x[0], x[1], b, &px, &py, &pdf)) o[0] = 1, o[1] = px, o[2] = py, o[3] = pdf;
        const Float bi = E.Integral(b[0], b[1], b[2], b[3]);
        o[4] = bi == 0 ? 0.f : E.FuncEval(x[6], x[7]) / bi;
    }
    return 0;
}
// the oracle's MeasuredBxDF (omeas) read from `path`, on queries laid out as pbrt_debug_measured's:
// in[8] {wo, wi, u0, u1} at the wavelengths lambda[NS] -> out[68] {f[NS], PDF, ok, wi, pdf, f[NS]}
int oracle_measured_eval(const char *path, const float *in, int n, const float *lambda, float *out) {
    omeas::Brdf b;
    if (!omeas::Load(path, &b)) return -1;
    omeas::Measured m;
    m.b = &b;
    for (int i = 0; i < NS; ++i) m.lambda[i] = lambda[i];
    for (int k = 0; k < n; ++k) {
        const float *q = in + 8 * k;
        float *o = out + (2 * NS + 6) * k;
        const Vec wo(q[0], q[1], q[2]), wi(q[3], q[4], q[5]);
        const Spectrum fv = m.f(wo, wi);
        for (int i = 0; i < NS; ++i) o[i] = fv[i];
        o[NS] = m.PDF(wo, wi);
        float *s = o + NS + 1;
        std::fill(s, s + 5 + NS, 0.f);
        BSDFSample bs;
        if (m.Sample_f(wo, q[6], q[7], &bs)) {
            s[0] = 1;
            s[1] = bs.wi.x, s[2] = bs.wi.y, s[3] = bs.wi.z;
            s[4] = bs.pdf;
            for (int i = 0; i < NS; ++i) s[5 + i] = bs.f[i];
        }
    }
    return 0;
}
// the oracle's own BSSRDF table for (g, eta) (osss::Table), kSssTableFloats floats
void oracle_sss_table(float g, float eta, float *out) {
    const std::vector<float> t = osss::Table(g, eta);
    std::copy(t.begin(), t.end(), out);
}

// Transcendental mode of every later call (see CRSin): 0 = libm float (reference), 1 = CR
void oracle_set_cr_math(int on) { g_mathMode = on ? 1 : 0; }
void oracle_set_math_mode(int mode) { g_mathMode = mode; }
int oracle_get_math_mode(void) { return g_mathMode; }
// the oracle's transcendentals in its current mode: fn 0 sin, 1 cos, 2 asin, 3 acos, 4 atan2(a, b), 5 log,
// 6 exp, 7 sinh, 8 tan, 9 atan, 10 expm1
void oracle_math_eval(int fn, const float *a, const float *b, int n, float *out) {
    for (int i = 0; i < n; ++i) {
        switch (fn) {
        case 0: out[i] = CRSin(a[i]); break;
        case 1: out[i] = CRCos(a[i]); break;
        case 2: out[i] = SafeASin(a[i]); break;
        case 3: out[i] = SafeACos(a[i]); break;
        case 4: out[i] = CRATan2(a[i], b[i]); break;
        case 6: out[i] = CRExp(a[i]); break;
        case 7: out[i] = CRSinh(a[i]); break;
        case 8: out[i] = CRTan(a[i]); break;
        case 9: out[i] = g_mathMode == 1 ? (Float)std::atan((double)a[i]) : std::atan(a[i]); break;
        case 10: out[i] = g_mathMode == 1 ? (Float)std::expm1((double)a[i]) : std::expm1(a[i]); break;
        default: out[i] = CRLog(a[i]); break;
        }
    }
}

// Filter::Sample(u) of a filter (type as pbrt_scene_flat::filter_type): out3 = p.x p.y weight;
// out_eval = Filter::Evaluate(px, py)
void oracle_filter_sample(int type, float rx, float ry, float a, float b, float u0, float u1, float px, float py,
                          float *out4) {
    PixelFilter f;
    f.Init(type, rx, ry, a, b);
    f.Sample(u0, u1, &out4[0], &out4[1], &out4[2]);
    out4[3] = f.Evaluate(px, py);
}

// IntersectShadowTr over a batch (the counterpart of pbrt_intersect_tr): rays [7][n], medium
// [n] (-1 vacuum), lambda0 [n] -> out [3][31][n] T_ray, r_u, r_l
int oracle_intersect_tr(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const float *rays,
                        const int32_t *medium, const float *lambda0, int n, float *out) {
    Renderer r;
    r.f = flat;
    // Scene setup is host work in the product (BVH, light BVH cones, filter tables, pyramids,
    // environment distributions: libm on the host), so in device-math mode it runs with libm
    // and only the per-sample work uses the device's polynomials.
    struct HostMath {
        int mode = g_mathMode;
        HostMath() { if (mode != 0) g_mathMode = 0; }
        void Done() { g_mathMode = mode; }
        ~HostMath() { Done(); }
    } hostMath;
    r.S.Init(flat, info);
    if (flat->n_tex_nodes > 0 && (!g_rgbTable || !g_ewaLut)) return -2;  // oracle_set_rgb_table first
    r.tex.Init(flat, info->spp, info->xres, info->yres);
    r.S.tex = &r.tex;
    r.M.f = flat;
    r.M.n = flat->n_media;
    const int nt = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int w = 0; w < nt; ++w)
        pool.emplace_back([&, w] {
            for (int i = w; i < n; i += nt) {
                Wavelengths lam = Wavelengths::SampleUniform(0.f);
                lam.lambda[0] = lambda0[i];
                for (int k = 1; k < NS; ++k) {
                    lam.lambda[k] = lam.lambda[k - 1] + (LambdaMax - LambdaMin) / NS;
                    if (lam.lambda[k] > LambdaMax) lam.lambda[k] = LambdaMin + (lam.lambda[k] - LambdaMax);
                }
                Spectrum T, tu, tl;
                const int med = medium && medium[i] >= 0 && medium[i] < flat->n_media ? medium[i] : -1;
                r.TraceTransmittance(Vec(rays[i], rays[n + i], rays[2 * n + i]),
                                     Vec(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]), rays[6 * n + i], med, lam,
                                     &T, &tu, &tl);
                for (int k = 0; k < NS; ++k) {
                    out[(size_t)k * n + i] = T[k];
                    out[(size_t)(NS + k) * n + i] = tu[k];
                    out[(size_t)(2 * NS + k) * n + i] = tl[k];
                }
            }
        });
    for (auto &t : pool) t.join();
    return 0;
}

// Renders rows x [first_sample, first_sample + n_samples) into film[4][yres*xres]
// (sensor RGB sums + weight sums, RGBFilm::Pixel layout) with `threads` host threads.
static int RenderRows(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const int32_t *rows, int nRows,
                      int firstSample, int nSamples, int uniformLightSampler, int threads, double *film, bool path) {
    Renderer r;
    r.f = flat;
    // Scene setup is host work in the product (BVH, light BVH cones, filter tables, pyramids,
    // environment distributions: libm on the host), so in device-math mode it runs with libm
    // and only the per-sample work uses the device's polynomials.
    struct HostMath {
        int mode = g_mathMode;
        HostMath() { if (mode != 0) g_mathMode = 0; }
        void Done() { g_mathMode = mode; }
        ~HostMath() { Done(); }
    } hostMath;
    r.S.Init(flat, info);
    if (flat->n_tex_nodes > 0 && (!g_rgbTable || !g_ewaLut)) return -2;  // oracle_set_rgb_table first
    r.tex.Init(flat, info->spp, info->xres, info->yres);
    r.S.tex = &r.tex;
    if ((flat->n_env > 0 || flat->n_tex_nodes > 0) && !g_rgbTable) return -2;
    r.envs.resize(flat->n_env);
    for (int k = 0; k < flat->n_env; ++k) r.envs[k].Init(flat, k);
    r.lights.Init(flat);
    r.lights.uniformFlag = uniformLightSampler != 0;
    r.M.f = flat;
    r.M.n = flat->n_media;
    r.filt.Init(flat->filter_type, info->filter_radius_x, info->filter_radius_y, flat->filter_a, flat->filter_b);
    r.measured.resize(flat->n_measured);
    for (int k = 0; k < flat->n_measured; ++k)
        if (!omeas::Load(flat->measured_files[k], &r.measured[k])) std::fprintf(stderr, "oracle: cannot read %s\n", flat->measured_files[k]);
    for (int k = 0; k < flat->n_sss; ++k) r.sssTables.push_back(osss::Table(flat->sss_params[20 * k + 18], flat->sss_params[20 * k + 2]));
    hostMath.Done();
    size_t npix = (size_t)info->xres * info->yres;
    std::atomic<int> next(0);
    auto work = [&]() {
        while (true) {
            int ri = next.fetch_add(1);
            if (ri >= nRows) break;
            int y = rows[ri];
            for (int x = info->px0; x < info->px1; ++x) {
                size_t pix = (size_t)y * info->xres + x;
                for (int s = firstSample; s < firstSample + nSamples; ++s) {
                    float rgb[3], w;
                    if (path) {
                        if (!r.PathLi(x, y, s, rgb, &w)) return;
                    } else {
                        r.Li(x, y, s, rgb, &w);
                    }
                    // RGBFilm::AddSample's clamp (film.h:247-249)
                    const float m = std::max({rgb[0], rgb[1], rgb[2]});
                    if (m > flat->max_component_value) {
                        const float sc = flat->max_component_value / m;
                        for (int c = 0; c < 3; ++c) rgb[c] *= sc;
                    }
                    film[pix] += w * rgb[0];
                    film[npix + pix] += w * rgb[1];
                    film[2 * npix + pix] += w * rgb[2];
                    film[3 * npix + pix] += w;
                }
            }
        }
    };
    threads = std::max(1, threads);
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; ++t) pool.emplace_back(work);
    work();
    for (auto &t : pool) t.join();
    return path && flat->n_media > 0 ? -3 : 0;
}

// WavefrontPathIntegrator semantics (the product's): film[4][yres][xres] += w * rgb, w
int oracle_render(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const int32_t *rows, int nRows,
                  int firstSample, int nSamples, int uniformLightSampler, int threads, double *film) {
    return RenderRows(flat, info, rows, nRows, firstSample, nSamples, uniformLightSampler, threads, film, false);
}
// PathIntegrator (cpu/integrators.cpp:629-805) on the same film; -3 for a scene with media
int oracle_render_path(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const int32_t *rows, int nRows,
                       int firstSample, int nSamples, int uniformLightSampler, int threads, double *film) {
    return RenderRows(flat, info, rows, nRows, firstSample, nSamples, uniformLightSampler, threads, film, true);
}

// closest / any hit for an SoA ray batch rays[7][n] (o, d, tMax); prim = original triangle
int oracle_intersect_batch(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const float *rays, int n,
                           int anyHit, int32_t *prim, float *hit) {
    Scene S;
    S.Init(flat, info);
    if (flat->n_tex_nodes > 0 && (!g_rgbTable || !g_ewaLut)) return -2;  // oracle_set_rgb_table first
    OTextures tex;
    tex.Init(flat, info->spp, info->xres, info->yres);
    S.tex = &tex;
    // independent rays: split over host threads (large scenes, 10^5+ rays in the tests)
    const int nt = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (int w = 0; w < nt; ++w)
        pool.emplace_back([&, w] {
            for (int i = w; i < n; i += nt) {
                Vec o(rays[i], rays[n + i], rays[2 * n + i]), d(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
                TriIsect ti{0, 0, 0, 0};
                prim[i] = S.Intersect(o, d, rays[6 * n + i], &ti, anyHit != 0);
                hit[i] = ti.b0;
                hit[n + i] = ti.b1;
                hit[2 * n + i] = ti.b2;
                hit[3 * n + i] = ti.t;
            }
        });
    for (auto &t : pool) t.join();
    return 0;
}

// IntersectOneRandom per segment segs[6][n] (p0, p1) with materials[n]: prim (original
// numbering, -1), hit[3][n] (b0 b1 b2), pdf[n]
int oracle_intersect_one_random(const pbrt_scene_flat *flat, const pbrt_scene_info *info, const float *segs,
                                const int32_t *mats, int n, int32_t *prim, float *hit, float *pdf) {
    Scene S;
    S.Init(flat, info);
    if (flat->n_tex_nodes > 0 && (!g_rgbTable || !g_ewaLut)) return -2;
    OTextures tex;
    tex.Init(flat, info->spp, info->xres, info->yres);
    S.tex = &tex;
    for (int i = 0; i < n; ++i) {
        const Vec p0(segs[i], segs[n + i], segs[2 * n + i]), p1(segs[3 * n + i], segs[4 * n + i], segs[5 * n + i]);
        TriIsect ti{0, 0, 0, 0};
        Vec d;
        Float pr = 0;
        prim[i] = ProbeOneRandom(S, p0, p1, mats[i], &ti, &d, &pr);
        hit[i] = prim[i] >= 0 ? ti.b0 : 0;
        hit[n + i] = prim[i] >= 0 ? ti.b1 : 0;
        hit[2 * n + i] = prim[i] >= 0 ? ti.b2 : 0;
        pdf[i] = pr;
    }
    return 0;
}

// The oracle's own light BVH: over given LightBounds rows ([n][13] pMin3 pMax3 w3 phi cosO cosE
// twoSided) when lights13 != NULL, else over the scene's lights.  Same output layout as
// pbrt_debug_light_bvh.  Returns the node count.
int oracle_light_bvh(const pbrt_scene_flat *flat, const float *lights13, int n, float *nodes12, int32_t *info3,
                     uint32_t *trails, int maxNodes) {
    std::vector<std::pair<int, lbvh::LB>> L;
    int nLights = n;
    if (lights13) {
        for (int i = 0; i < n; ++i) {
            const float *v = lights13 + 13 * i;
            lbvh::LB lb;
            lb.b = lbvh::Box(Vec(v[0], v[1], v[2]), Vec(v[3], v[4], v[5]));
            lb.w = Vec(v[6], v[7], v[8]);  // as stored by the LightBounds constructor
            lb.phi = v[9];
            lb.cosO = v[10];
            lb.cosE = v[11];
            lb.two = v[12] != 0;
            L.push_back({i, lb});
        }
    } else {
        L = lbvh::SceneLightBounds(flat);
        nLights = flat->n_area_lights + flat->n_point_spot;
    }
    lbvh::Builder b;
    b.Run(L, nLights);
    for (int i = 0; i < std::min((int)b.nodes.size(), maxNodes); ++i) {
        const LightNode &d = b.nodes[i];
        const float v[12] = {d.mn.x, d.mn.y, d.mn.z, d.mx.x, d.mx.y, d.mx.z, d.w.x, d.w.y, d.w.z, d.phi, d.cosO, d.cosE};
        if (nodes12) std::memcpy(nodes12 + 12 * i, v, sizeof v);
        if (info3) info3[3 * i] = d.childOrLight, info3[3 * i + 1] = d.isLeaf, info3[3 * i + 2] = d.twoSided;
    }
    if (trails) std::copy(b.trail.begin(), b.trail.end(), trails);
    return (int)b.nodes.size();
}

// ---- textures
void oracle_set_rgb_table(const float *table, const float *ewaLut) {
    g_rgbTable = table;
    g_ewaLut = ewaLut;
}
// the oracle's texture evaluation at a hit (p, n, dpdu, dpdv, uv): out[0..3] uv derivatives,
// then the spectrum at each of the n wavelengths (slot 0) or the float texture (slots 1, 2)
int oracle_texture_eval(const pbrt_scene_flat *flat, const pbrt_scene_info *info, int material, int slot,
                        const float *hit, const float *lambda, int n, float *out) {
    if (!g_rgbTable || !g_ewaLut) return -2;
    OTextures t;
    t.Init(flat, info->spp, info->xres, info->yres);
    const int node = flat->material_tex[4 * material + slot];
    if (node < 0) return -1;
    Interaction si;
    si.p = Vec(hit[0], hit[1], hit[2]);
    si.n = Vec(hit[3], hit[4], hit[5]);
    si.dpdu = Vec(hit[6], hit[7], hit[8]);
    si.dpdv = Vec(hit[9], hit[10], hit[11]);
    si.uv[0] = hit[12];
    si.uv[1] = hit[13];
    const OTexCtx c = t.Ctx(si);
    out[0] = c.dudx;
    out[1] = c.dudy;
    out[2] = c.dvdx;
    out[3] = c.dvdy;
    if (slot != 0) {
        out[4] = t.EvalF(node, c);
        return 0;
    }
    // the wavelengths in groups of NS, lambda[i] at sample index i % NS (a multispectral basis
    // is indexed by the sample index)
    for (int i0 = 0; i0 < n; i0 += NS) {
        Wavelengths L = Wavelengths::SampleUniform(0.f);
        for (int k = 0; k < NS; ++k) L.lambda[k] = lambda[std::min(i0 + k, n - 1)];
        const Spectrum v = t.EvalS(node, c, L);
        for (int k = 0; k < NS && i0 + k < n; ++k) out[4 + i0 + k] = v[k];
    }
    return 0;
}
// the oracle's sphere / disk evaluation, laid out as pbrt_debug_shape_eval's rows
int oracle_shape_eval(const pbrt_scene_flat *flat, int shape, const float *rays, const float *u, int n, float *out) {
    if (shape < 0 || shape >= flat->n_shapes) return -1;
    OShape sh;
    sh.Init(flat, shape);
    for (int i = 0; i < n; ++i) {
        float *o = out + 40 * (size_t)i;
        std::fill(o, o + 40, 0.f);
        const Vec ro(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]), rd(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        const Vec cns = (i & 1) ? Normalize(-rd) : Vec(0, 0, 0);
        Float th;
        Vec pObj;
        if (sh.Intersect(ro, rd, Infinity, &th, &pObj)) {
            const Interaction si = sh.Surface(pObj, rd);
            const Vec v[8] = {pObj, si.p, si.err, si.n, si.ns, si.dpdu, si.dpdv, Vec(si.uv[0], si.uv[1], 0)};
            o[0] = 1;
            o[1] = th;
            for (int k = 0; k < 8; ++k)
                for (int j = 0; j < (k == 7 ? 2 : 3); ++j) o[2 + 3 * k + j] = v[k][j];
        }
        ShapeSample ss;
        if (sh.Sample(ro, Vec(0, 0, 0), Vec(0, 0, 0), u[2 * i], u[2 * i + 1], &ss, cns)) {
            o[26] = 1;
            for (int j = 0; j < 3; ++j) {
                o[27 + j] = ss.p[j];
                o[30 + j] = ss.err[j];
                o[33 + j] = ss.n[j];
            }
            o[36] = ss.pdf;
        }
        o[37] = sh.PDF(ro, Vec(0, 0, 0), Vec(0, 0, 0), rd, cns);
    }
    return 0;
}
// the oracle's ImageInfiniteLight lookups, laid out as pbrt_debug_env_eval's rows
int oracle_env_eval(const pbrt_scene_flat *flat, int env, const float *dirs, const float *u, int n, float *out) {
    if (!g_rgbTable) return -2;
    if (env < 0 || env >= flat->n_env) return -1;
    OEnvLight E;
    E.Init(flat, env);
    static const float kLam[4] = {400.f, 500.f, 600.f, 700.f};
    float one[311];
    std::fill(one, one + 311, 1.f);
    for (int i = 0; i < n; ++i) {
        float *o = out + 16 * (size_t)i;
        const Vec d(dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2]);
        Float uu, vv, pu, pv;
        OEnvLight::SphereToSquare(Normalize(OEnvLight::Mul(E.mi, d)), &uu, &vv);
        o[0] = uu;
        o[1] = vv;
        OEnvLight::SphereToSquare(OEnvLight::Mul(E.mi, d), &pu, &pv);
        o[2] = E.PDF(pu, pv) / (4 * Pi);
        for (int k = 0; k < 4; ++k) {
            Wavelengths L = Wavelengths::SampleUniform(0.f);
            for (int j = 0; j < NS; ++j) L.lambda[j] = kLam[k];
            o[3 + k] = E.Le(uu, vv, L, one, 1.f)[0];
        }
        Float su, sv, mp;
        E.Sample(u[2 * i], u[2 * i + 1], &su, &sv, &mp);
        o[7] = su;
        o[8] = sv;
        o[9] = mp;
        const Vec wi = OEnvLight::Mul(E.m, OEnvLight::SquareToSphere(su, sv));
        o[10] = wi.x;
        o[11] = wi.y;
        o[12] = wi.z;
        o[13] = E.PDF(su, sv);                // PiecewiseConstant2D::PDF at the sample
        o[14] = E.PDF(u[2 * i], u[2 * i + 1]);  // ... and at u taken as a point of [0,1]^2
        o[15] = 0;
    }
    return 0;
}
// PortalImageInfiniteLight queries laid out as pbrt_debug_portal_eval's: q[8] = {p, d, u0, u1}
// -> out[16] = {Le(ray p, d) at 400/500/600/700 nm (light scale 1, illuminant 1), PDF_Li(p, d),
// SampleLi ok, wi, pdf, sample Le at the four wavelengths, ImageBounds ok, 0}; img (optional):
// the rectified image [res][res][3] then the distribution's function [res][res]
int oracle_portal_eval(const pbrt_scene_flat *flat, int env, const float *q, int n, float *out, float *img) {
    if (!g_rgbTable) return -2;
    if (env < 0 || env >= flat->n_env || !flat->env_portal || !flat->env_info[4 * env + 1]) return -1;
    OEnvLight E;
    {
        const int mode = g_mathMode;
        if (mode != 0) g_mathMode = 0;  // construction is host work (libm)
        E.Init(flat, env);
        g_mathMode = mode;
    }
    static const float kLam[4] = {400.f, 500.f, 600.f, 700.f};
    float one[311];
    std::fill(one, one + 311, 1.f);
    auto at4 = [&](auto &&fn, float *o) {
        for (int k = 0; k < 4; ++k) {
            Wavelengths L = Wavelengths::SampleUniform(0.f);
            for (int j = 0; j < NS; ++j) L.lambda[j] = kLam[k];
            o[k] = fn(L)[0];
        }
    };
    for (int i = 0; i < n; ++i) {
        const float *x = q + 8 * (size_t)i;
        float *o = out + 16 * (size_t)i;
        std::fill(o, o + 16, 0.f);
        const Vec p(x[0], x[1], x[2]), d(x[3], x[4], x[5]);
        at4([&](const Wavelengths &L) { return E.LeRay(p, d, L, one, 1.f); }, o);
        o[4] = E.PdfLi(p, d);
        Vec wi;
        Float pdf;
        Spectrum Le;
        Wavelengths L0 = Wavelengths::SampleUniform(0.f);
        if (E.SampleLi(p, x[6], x[7], L0, one, 1.f, &wi, &pdf, &Le)) {
            o[5] = 1;
            o[6] = wi.x, o[7] = wi.y, o[8] = wi.z;
            o[9] = pdf;
            Float b[4], uu, vv, mp;
            E.ImageBounds(p, b);
            E.WindowedSample(x[6], x[7], b, &uu, &vv, &mp);
            at4([&](const Wavelengths &L) { return E.RectLe(uu, vv, L, one, 1.f); }, o + 10);
        }
        Float b[4];
        o[14] = E.ImageBounds(p, b) ? 1.f : 0.f;
    }
    if (img) {
        const size_t np = (size_t)E.n * E.n;
        std::copy(E.prgb.begin(), E.prgb.end(), img);
        for (size_t k = 0; k < np; ++k) img[3 * np + k] = E.pfunc[k];
    }
    return 0;
}
// EqualAreaSquareToSphere (toSphere: in[n][2] -> out[n][3]) or EqualAreaSphereToSquare
// (in[n][3] -> out[n][2]) of the oracle (util/math.cpp:292-361)
// util/noise.cpp Noise / DNoise and CloudMedium::Density: c = {density, wispiness, frequency,
// NoisePerm[512]}; out5 per point = Noise, DNoise xyz, Density
int oracle_cloud_density(const float *c, const float *pts, int n, float *out) {
    const float *perm = c + 3;
    for (int i = 0; i < n; ++i) {
        const Vec p(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
        const Float nz = Media::NoiseAt(perm, p.x, p.y, p.z), d = .01f;
        out[5 * i] = nz;
        out[5 * i + 1] = (Media::NoiseAt(perm, p.x + d, p.y + 0.f, p.z + 0.f) - nz) / d;
        out[5 * i + 2] = (Media::NoiseAt(perm, p.x + 0.f, p.y + d, p.z + 0.f) - nz) / d;
        out[5 * i + 3] = (Media::NoiseAt(perm, p.x + 0.f, p.y + 0.f, p.z + d) - nz) / d;
        out[5 * i + 4] = Media::CloudDensity(c, p);
    }
    return 0;
}

// Medium::SamplePoint of medium `medium` at render-space points and the given wavelengths
// (lambdas [n][31]) -> out [n][3][31]: sigma_a, sigma_s, Le
int oracle_medium_point(const pbrt_scene_flat *flat, int medium, const float *pts, const float *lambdas, int n,
                        float *out) {
    if (medium < 0 || medium >= flat->n_media) return -1;
    Media M;
    M.f = flat;
    M.n = flat->n_media;
    for (int i = 0; i < n; ++i) {
        Wavelengths lam = Wavelengths::SampleUniform(0.f);
        for (int k = 0; k < NS; ++k) lam.lambda[k] = lambdas[NS * i + k];
        const MediumProps mp = M.SamplePoint(medium, Vec(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]), lam);
        for (int k = 0; k < NS; ++k) {
            out[(3 * i) * NS + k] = mp.sigma_a[k];
            out[(3 * i + 1) * NS + k] = mp.sigma_s[k];
            out[(3 * i + 2) * NS + k] = mp.Le[k];
        }
    }
    return 0;
}

int oracle_equal_area(int toSphere, const float *in, int n, float *out) {
    for (int i = 0; i < n; ++i) {
        if (toSphere) {
            const Vec w = OEnvLight::SquareToSphere(in[2 * i], in[2 * i + 1]);
            out[3 * i] = w.x;
            out[3 * i + 1] = w.y;
            out[3 * i + 2] = w.z;
        } else {
            Float uu, vv;
            OEnvLight::SphereToSquare(Vec(in[3 * i], in[3 * i + 1], in[3 * i + 2]), &uu, &vv);
            out[2 * i] = uu;
            out[2 * i + 1] = vv;
        }
    }
    return 0;
}
// the oracle's FindMinimumDifferentials: pos dx, pos dy, dir dx, dir dy
int oracle_camera_min_diff(const pbrt_scene_flat *flat, const pbrt_scene_info *info, float *out12) {
    OTextures t;
    t.f = flat;
    t.fullRes[0] = info->xres;
    t.fullRes[1] = info->yres;
    t.FindMinimumDifferentials();
    const Vec v[4] = {t.minPosDx, t.minPosDy, t.minDirDx, t.minDirDy};
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 3; ++j) out12[3 * k + j] = v[k][j];
    return 0;
}
// one level of the oracle's own MIPMap pyramid of image `image`, in its stored format:
// returns the byte count (writes at most cap bytes to out), w / h of the level
int64_t oracle_image_level(const pbrt_scene_flat *flat, int image, int level, uint8_t *out, int64_t cap, int *w, int *h) {
    OImage im;
    const int32_t *ri = flat->image_raw_info + 8 * image;
    im.format = ri[2];
    im.nc = ri[3];
    im.wrap = flat->image_info[8 * image + 3];
    im.enc.Init(ri[4], flat->image_raw_gamma[image], flat->image_luts + 256 * image);
    im.Build(flat->image_raw_data + flat->image_raw_offset[image], ri[0], ri[1]);
    if (level < 0 || level >= im.nLevels) return -1;
    *w = im.w[level];
    *h = im.h[level];
    const uint8_t *src;
    int64_t bytes;
    if (im.format == 0) src = im.l8[level].data(), bytes = (int64_t)im.l8[level].size();
    else if (im.format == 1) src = (const uint8_t *)im.l16[level].data(), bytes = 2 * (int64_t)im.l16[level].size();
    else src = (const uint8_t *)im.l32[level].data(), bytes = 4 * (int64_t)im.l32[level].size();
    std::memcpy(out, src, (size_t)std::min(bytes, cap));
    return bytes;
}

// ---- component entry points checked against tests/golden/reference_components.json
int oracle_intersect_triangle(const float *p9, const float *o3, const float *d3, float tMax, int flip, float *out) {
    // out: b0 b1 b2 t | p3 err3 n3 dpdu3 wo3
    TriIsect ti;
    Vec p0(p9[0], p9[1], p9[2]), p1(p9[3], p9[4], p9[5]), p2(p9[6], p9[7], p9[8]);
    Vec d(d3[0], d3[1], d3[2]);
    if (!IntersectTriangle(Vec(o3[0], o3[1], o3[2]), d, tMax, p0, p1, p2, &ti)) return 0;
    Interaction si = TriangleInteraction(p0, p1, p2, flip != 0, ti, d);
    float v[19] = {ti.b0, ti.b1, ti.b2, ti.t, si.p.x, si.p.y, si.p.z, si.err.x, si.err.y, si.err.z, si.n.x,
                   si.n.y, si.n.z, si.dpdu.x, si.dpdu.y, si.dpdu.z, si.wo.x, si.wo.y, si.wo.z};
    std::memcpy(out, v, sizeof v);
    return 1;
}

void oracle_warps(const float *u2, const float *w4, float *out) {
    // out: disk2 cos3 tri3 bilinear2 bilinear_pdf1
    Float x, y;
    SampleUniformDiskConcentric(u2[0], u2[1], &x, &y);
    Vec c = SampleCosineHemisphere(u2[0], u2[1]);
    Float b[3];
    SampleUniformTriangle(u2[0], u2[1], b);
    Float bx, by;
    SampleBilinear(u2[0], u2[1], w4, &bx, &by);
    float v[11] = {x, y, c.x, c.y, c.z, b[0], b[1], b[2], bx, by, BilinearPDF(bx, by, w4)};
    std::memcpy(out, v, sizeof v);
}

void oracle_spherical_triangle(const float *v9, const float *p3, const float *u2, float *out) {
    // out: b3 pdf1 w3 inv2 area1
    Vec v0(v9[0], v9[1], v9[2]), v1(v9[3], v9[4], v9[5]), v2(v9[6], v9[7], v9[8]), p(p3[0], p3[1], p3[2]);
    Float b[3], pdf;
    SampleSphericalTriangle(v0, v1, v2, p, u2[0], u2[1], b, &pdf);
    Vec ps = b[0] * v0 + b[1] * v1 + b[2] * v2;
    Vec w = Normalize(ps - p);
    Float i0, i1;
    InvertSphericalTriangleSample(v0, v1, v2, p, w, &i0, &i1);
    Float area = SphericalTriangleArea(Normalize(v0 - p), Normalize(v1 - p), Normalize(v2 - p));
    float v[10] = {b[0], b[1], b[2], pdf, w.x, w.y, w.z, i0, i1, area};
    std::memcpy(out, v, sizeof v);
}

int oracle_triangle_sample(const float *v9, int flip, const float *ref3, const float *n3, const float *ns3,
                           const float *u2, float *out) {
    // out: p3 err3 n3 pdf1 pdf_wi1 solid_angle1
    Vec p0(v9[0], v9[1], v9[2]), p1(v9[3], v9[4], v9[5]), p2(v9[6], v9[7], v9[8]);
    Vec ref(ref3[0], ref3[1], ref3[2]), n(n3[0], n3[1], n3[2]), ns(ns3[0], ns3[1], ns3[2]);
    ShapeSample ss;
    if (!TriangleSample(p0, p1, p2, flip != 0, ref, ns, u2[0], u2[1], &ss)) return 0;
    Vec wi = Normalize(ss.p - ref);
    Float pdf2 = TrianglePDF(p0, p1, p2, flip != 0, ref, Vec(0, 0, 0), n, ns, wi);
    Float sa = SphericalTriangleArea(Normalize(p0 - ref), Normalize(p1 - ref), Normalize(p2 - ref));
    float v[12] = {ss.p.x, ss.p.y, ss.p.z, ss.err.x, ss.err.y, ss.err.z, ss.n.x, ss.n.y, ss.n.z, ss.pdf, pdf2, sa};
    std::memcpy(out, v, sizeof v);
    return 1;
}

float oracle_light_importance(const float *decoded11, float phi, int twoSided, const float *p3, const float *n3) {
    LightNode b{Vec(decoded11[0], decoded11[1], decoded11[2]), Vec(decoded11[3], decoded11[4], decoded11[5]),
                Vec(decoded11[6], decoded11[7], decoded11[8]), phi, decoded11[9], decoded11[10], twoSided, 0, 1};
    return Importance(b, Vec(p3[0], p3[1], p3[2]), Vec(n3[0], n3[1], n3[2]));
}

void oracle_offset_ray_origin(const float *p3, const float *e3, const float *n3, const float *w3, float *out) {
    Vec pm, em;  // the reference call site passes Point3fi(p, e)
    Point3fi(Vec(p3[0], p3[1], p3[2]), Vec(e3[0], e3[1], e3[2]), &pm, &em);
    Vec po = OffsetRayOrigin(pm, em, Vec(n3[0], n3[1], n3[2]), Vec(w3[0], w3[1], w3[2]));
    out[0] = po.x;
    out[1] = po.y;
    out[2] = po.z;
}

void oracle_sample_wavelengths(float u, float *lambda31, float *pdf) {
    Wavelengths w = Wavelengths::SampleUniform(u);
    std::memcpy(lambda31, w.lambda, sizeof w.lambda);
    *pdf = w.pdf[0];
}

void oracle_zsobol(int spp, int xres, int yres, int seed, int randomize, int px, int py, int sampleIndex, int dim,
                   float *out7) {
    ZSobol z;
    z.Init(spp, xres, yres, seed, randomize);
    ZSobolState s{&z};
    s.Start(px, py, sampleIndex, dim);
    out7[0] = s.Get1D();
    s.Get2D(&out7[1], &out7[2]);
    out7[3] = s.Get1D();
    s.Get2D(&out7[4], &out7[5]);
    out7[6] = s.Get1D();
}

// IndependentSampler / StratifiedSampler / SobolSampler / PaddedSobolSampler (kind 2..5) from
// StartPixelSample((px, py), sampleIndex, dim) in the wavefront's call order: dimension 0 the
// camera's Get1D, GetPixel2D, Get1D, Get2D, Get1D; otherwise Get1D, Get2D, Get1D, Get2D, Get1D
void oracle_sampler(int kind, int spp, int seed, int xs, int ys, int jitter, int randomize, int xres, int yres,
                    const uint32_t *m32, const uint64_t *vdc, const uint64_t *vdcInv, int px, int py,
                    int sampleIndex, int dim, float *out7) {
    OtherSampler o;
    o.kind = kind;
    o.spp = spp;
    o.seed = seed;
    o.xs = xs;
    o.ys = ys;
    o.jitter = jitter;
    o.randomize = randomize;
    int res = 1;
    while (res < std::max(xres, yres)) res *= 2;  // SobolSampler: scale = RoundUpPow2(max res)
    while ((2 << o.log2Scale) <= res) ++o.log2Scale;
    o.m32 = m32;
    o.vdc = vdc;
    o.vdcInv = vdcInv;
    OtherState st;
    st.o = &o;
    st.Start(px, py, sampleIndex, dim);
    out7[0] = st.Get1D();
    if (dim == 0) st.Pixel2D(&out7[1], &out7[2]);
    else st.Get2D(&out7[1], &out7[2]);
    out7[3] = st.Get1D();
    st.Get2D(&out7[4], &out7[5]);
    out7[6] = st.Get1D();
}
// the oracle's procedural textures: kind 0 fbm, 1 turbulence, 2 windy, 3 polka dot (in9[0..1]),
// 4 marble (out: RGB, then its sigmoid coefficients); params4 = octaves, roughness, scale, variation
void oracle_procedural(int kind, const float *perm, const float *params4, const float *in9, int n, float *out6) {
    for (int i = 0; i < n; ++i) {
        const float *q = in9 + 9 * i;
        float *o = out6 + 6 * i;
        const Vec p(q[0], q[1], q[2]), dx(q[3], q[4], q[5]), dy(q[6], q[7], q[8]);
        for (int k = 0; k < 6; ++k) o[k] = 0;
        if (kind == 0) o[0] = proc::FBm(perm, p, dx, dy, params4[1], (int)params4[0]);
        else if (kind == 1) o[0] = proc::Turbulence(perm, p, dx, dy, params4[1], (int)params4[0]);
        else if (kind == 2) o[0] = proc::Windy(perm, p, dx, dy);
        else if (kind == 3) o[0] = proc::PolkaDot(perm, q[0], q[1]) ? 1.f : 0.f;
        else {
            proc::Marble(perm, p, dx, dy, (int)params4[0], params4[1], params4[2], params4[3], o);
            ORGBCoeffs(o[0], o[1], o[2], o + 3);
        }
    }
}
void oracle_rng(uint64_t seq, uint64_t advance, uint32_t *out2) {
    SeqRNG r;
    r.SetSequence(seq);
    r.Advance(advance);
    out2[0] = r.Next();
    out2[1] = r.Next();
}

float oracle_halton(int xres, int yres, int seed, int px, int py, int sampleIndex, int dim) {
    static thread_local Halton h;
    static thread_local int key[3] = {-1, -1, -1};
    if (key[0] != xres || key[1] != yres || key[2] != seed) {
        h = Halton();
        h.Init(xres, yres, (uint32_t)seed, 60);
        key[0] = xres;
        key[1] = yres;
        key[2] = seed;
    }
    HaltonState s{&h, 0, 0};
    s.Start(px, py, sampleIndex, dim < 0 ? 0 : dim);
    Float a, b;
    s.Pixel2D(&a, &b);
    if (dim == -1) return a;
    if (dim == -2) return b;
    return s.Sample(std::max(2, dim));
}

void oracle_triangle_shading(const float *p9, const float *n9, const float *uv6, int flip, const float *b3,
                             const float *u2, float *out) {
    Vec p0(p9[0], p9[1], p9[2]), p1(p9[3], p9[4], p9[5]), p2(p9[6], p9[7], p9[8]);
    TriAttr a;
    if (n9) {
        a.hasN = true;
        for (int k = 0; k < 3; ++k) a.n[k] = Vec(n9[3 * k], n9[3 * k + 1], n9[3 * k + 2]);
    }
    if (uv6) {
        a.hasUV = true;
        for (int k = 0; k < 3; ++k) a.uv[k][0] = uv6[2 * k], a.uv[k][1] = uv6[2 * k + 1];
    }
    TriIsect ti{b3[0], b3[1], b3[2], 1};
    Interaction si = TriangleInteraction(p0, p1, p2, flip != 0, ti, Vec(0, 0, 1), a);
    Float b[3];
    SampleUniformTriangle(u2[0], u2[1], b);
    Vec sn = SampledNormal(p0, p1, p2, flip != 0, a, b);
    float v[15] = {si.n.x, si.n.y, si.n.z, si.ns.x, si.ns.y, si.ns.z, si.dpdu.x, si.dpdu.y, si.dpdu.z,
                   si.dpdus.x, si.dpdus.y, si.dpdus.z, sn.x, sn.y, sn.z};
    std::memcpy(out, v, sizeof v);
}

void oracle_trowbridge(const float *in, float *out) {
    TRDistribution d(in[0], in[1]);
    Vec wo(in[2], in[3], in[4]), wi(in[5], in[6], in[7]), wm(in[8], in[9], in[10]);
    Vec sw = d.Sample_wm(wo, in[11], in[12]);
    TRDistribution r = d;
    r.Regularize();
    Float dwm = d.G1(wo) / std::abs(wo.z) * d.D(wm) * AbsDot(wo, wm);  // D(w, wm)
    float v[14] = {d.ax, d.ay, (float)d.Smooth(), d.D(wm), dwm, d.Lambda(wo), d.G1(wo), d.G(wo, wi), d.PDF(wo, wm),
                   sw.x, sw.y, sw.z, r.ax, r.ay};
    std::memcpy(out, v, sizeof v);
}

void oracle_fresnel(const float *in, float *out) {
    Vec wi(in[4], in[5], in[6]), n(in[7], in[8], in[9]);
    Float etap = 0;
    Vec wt(0, 0, 0);
    bool ok = Refract(wi, n, in[1], &etap, &wt);
    Vec rf = Reflect(wi, n);
    float v[10] = {FrDielectric(in[0], in[1]), FrComplex(in[0], Complex(in[2], in[3])), (float)ok, etap, wt.x, wt.y,
                   wt.z, rf.x, rf.y, rf.z};
    std::memcpy(out, v, sizeof v);
}

// PiecewiseLinearSpectrum::FromInterleaved(samples, false) (util/spectrum.cpp:133-163) then
// operator() at each lambda
void oracle_named_spectrum(const float *interleaved, int nValues, const float *lambda, int n, float *out) {
    std::vector<float> lam, val;
    if (interleaved[0] > LambdaMin) {
        lam.push_back(LambdaMin - 1);
        val.push_back(interleaved[1]);
    }
    for (int i = 0; i + 1 < nValues; i += 2) {
        lam.push_back(interleaved[i]);
        val.push_back(interleaved[i + 1]);
    }
    if (lam.back() < LambdaMax) {
        lam.push_back(LambdaMax + 1);
        val.push_back(val.back());
    }
    for (int i = 0; i < n; ++i) out[i] = PLEval(lam.data(), val.data(), (int)lam.size(), lambda[i]);
}

void oracle_bxdf(int type, const float *params, const float *eta31, const float *k31, const float *wo3,
                 const float *wi3, const float *u3, float *out) {
    BxDF bx;
    bx.type = type;
    bx.mf.ax = params[0];
    bx.mf.ay = params[1];
    bx.eta = params[2];
    for (int i = 0; i < NS; ++i) {
        bx.etaS[i] = eta31[i];
        bx.kS[i] = k31[i];
    }
    Vec wo(wo3[0], wo3[1], wo3[2]), wi(wi3[0], wi3[1], wi3[2]);
    std::fill(out, out + 70, 0.f);
    BSDFSample bs;
    if (bx.Sample_f(wo, u3[0], u3[1], u3[2], &bs)) {
        float v[7] = {1, bs.wi.x, bs.wi.y, bs.wi.z, bs.pdf, (float)bs.flags, bs.eta};
        std::memcpy(out, v, sizeof v);
        for (int i = 0; i < NS; ++i) out[7 + i] = bs.f[i];
    }
    Spectrum f = bx.f(wo, wi);
    for (int i = 0; i < NS; ++i) out[38 + i] = f[i];
    out[69] = bx.PDF(wo, wi);
}

// LayeredBxDF (coated diffuse: params[3] = 0, coated conductor: 2) in the shading frame, as
// pbrt_debug_layered: params12 = top ax ay eta, bottom type ax ay, thickness g maxdepth
// nsamples radiance 0; a31 = R or conductor eta, b31 = k, alb31 = albedo; out72 = sample_ok
// wi3 pdf flags f_sample[31] f(wo,wi)[31] PDF(wo,wi) Flags() 0 0
void oracle_layered(const float *params, const float *a31, const float *b31, const float *alb31, const float *wo3,
                    const float *wi3, const float *u3, float *out) {
    LayeredBxDF L;
    L.top.type = 1;
    L.top.mf.ax = params[0];
    L.top.mf.ay = params[1];
    L.top.eta = params[2];
    L.bottom.type = (int)params[3];
    L.bottom.mf.ax = params[4];
    L.bottom.mf.ay = params[5];
    for (int i = 0; i < NS; ++i) {
        L.bottom.R[i] = a31[i];
        L.bottom.etaS[i] = a31[i];
        L.bottom.kS[i] = b31[i];
        L.albedo[i] = alb31[i];
    }
    L.thickness = std::max<Float>(params[6], std::numeric_limits<Float>::min());
    L.g = params[7];
    L.maxDepth = (int)params[8];
    L.nSamples = (int)params[9];
    const bool radiance = params[10] != 0;
    Vec wo(wo3[0], wo3[1], wo3[2]), wi(wi3[0], wi3[1], wi3[2]);
    std::fill(out, out + 72, 0.f);
    BSDFSample bs;
    if (L.Sample_f(wo, u3[0], u3[1], u3[2], &bs, radiance)) {
        float v[6] = {1, bs.wi.x, bs.wi.y, bs.wi.z, bs.pdf, (float)bs.flags};
        std::memcpy(out, v, sizeof v);
        for (int i = 0; i < NS; ++i) out[6 + i] = bs.f[i];
    }
    Spectrum f = L.f(wo, wi, radiance);
    for (int i = 0; i < NS; ++i) out[37 + i] = f[i];
    out[68] = L.PDF(wo, wi, radiance);
    out[69] = (float)L.Flags();
}

}  // extern "C"
