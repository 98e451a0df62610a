// Image textures on the host: file readers (PNG through zlib, PFM), pbrt's colour encodings and
// the MIPMap pyramid, restated from the reference:
//   Image::Read / ReadPNG / ReadPFM               util/image.cpp:877-921, 1260-1367, 1614-1695
//   MIPMap::CreateFromFile (channel selection)    util/mipmap.cpp:377-417
//   Image::GeneratePyramid, FloatResizeUp,        util/image.cpp:208-383
//     ResampleWeights, CopyRectIn / CopyRectOut   util/image.cpp:657-752
//   ColorEncoding (linear, sRGB, gamma)           util/color.h:420-538, util/color.cpp:190-286
//   Half (round to nearest even)                  util/float.h:419-470
// Each pyramid level keeps the image's original pixel format (the reference re-quantises every
// level into it), so the device decodes exactly the texel values pbrt's GetChannel returns.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <limits>
#include <thread>

#include "texture.h"
#include "image.h"

namespace pbrt_amd {

// ---------------------------------------------------------------- half
uint16_t FloatToHalf(float ff) {
    uint32_t u;
    std::memcpy(&u, &ff, 4);
    const uint32_t sign = (u >> 16) & 0x8000u;
    u &= 0x7fffffffu;
    uint16_t o;
    if (u >= 0x47800000u) {  // >= 65536: Inf or NaN (and overflow)
        o = (u > 0x7f800000u) ? 0x7e00 : 0x7c00;
    } else if (u < 0x38800000u) {  // below the smallest normal half: subnormal or zero
        float f;
        std::memcpy(&f, &u, 4);
        const float magic = 0.5f;  // 2^-1: aligns the 10 subnormal mantissa bits, RNE by the add
        float s = f + magic;
        uint32_t su;
        std::memcpy(&su, &s, 4);
        o = (uint16_t)(su - 0x3f000000u);
    } else {
        const uint32_t mantOdd = (u >> 13) & 1;
        u += 0xc8000fffu;  // rebias exponent (-112 << 23) and add the rounding bias 0xfff
        u += mantOdd;
        o = (uint16_t)(u >> 13);
    }
    return (uint16_t)(o | sign);
}

float HalfToFloat(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1f, mant = h & 0x3ffu;
    uint32_t u;
    if (exp == 0) {
        if (mant == 0) u = sign;
        else {  // subnormal: normalise
            int e = -1;
            do {
                ++e;
                mant <<= 1;
            } while (!(mant & 0x400u));
            mant &= 0x3ffu;
            u = sign | ((uint32_t)(127 - 15 - e) << 23) | (mant << 13);
        }
    } else if (exp == 31) {
        u = sign | 0x7f800000u | (mant << 13);
    } else {
        u = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    }
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// ---------------------------------------------------------------- colour encodings
static float EvalPoly(float t, std::initializer_list<float> c) {
    // EvaluatePolynomial (util/math.h): c0 + t (c1 + t (c2 + ...)), one FMA per coefficient
    const float *a = c.begin();
    int n = (int)c.size();
    float r = a[n - 1];
    for (int i = n - 2; i >= 0; --i) r = std::fma(t, r, a[i]);
    return r;
}
float LinearToSRGB(float value) {
    if (value <= 0.0031308f) return 12.92f * value;
    float sqrtValue = std::sqrt(std::max(0.f, value));
    float p = EvalPoly(sqrtValue, {-0.0016829072605308378f, 0.03453868659826638f, 0.7642611304733891f,
                                   2.0041169284241644f, 0.7551545191665577f, -0.016202083165206348f});
    float q = EvalPoly(sqrtValue, {4.178892964897981e-7f, -0.00004375359692957097f, 0.03467195408529984f,
                                   0.6085338522168684f, 1.8970238036421054f, 1.f});
    return p / q * value;
}
float SRGBToLinear(float value) {
    if (value <= 0.04045f) return value * (1 / 12.92f);
    float p = EvalPoly(value, {-0.0163933279112946f, -0.7386328024653209f, -11.199318357635072f,
                               -47.46726633009393f, -36.04572663838034f});
    float q = EvalPoly(value, {-0.004261480793199332f, -19.140923959601675f, -59.096406619244426f,
                               -18.225745396846637f, 1.f});
    return p / q * value;
}
uint8_t LinearToSRGB8(float value) {
    if (value <= 0) return 0;
    if (value >= 1) return 255;
    float v = std::round(255.f * LinearToSRGB(value));
    return (uint8_t)std::min(255.f, std::max(0.f, v));
}

Encoding Encoding::Get(const std::string &name, const std::string &loc) {
    Encoding e;
    if (name == "linear") {
        e.kind = kEncLinear;
    } else if (name == "sRGB") {
        e.kind = kEncSRGB;
    } else {
        std::istringstream is(name);
        std::string g;
        float gamma = 0;
        is >> g >> gamma;
        std::string rest;
        if (g != "gamma" || (is >> rest)) throw Error(loc + ": " + name + ": expected \"gamma <value>\" for color encoding");
        if (gamma == 0) throw Error(loc + ": " + name + ": unable to parse gamma value");
        e.kind = kEncGamma;
        e.gamma = gamma;
        // GammaColorEncoding::GammaColorEncoding (util/color.cpp:252-261)
        for (int i = 0; i < 256; ++i) e.applyLUT[i] = std::pow(float(i) / 255.f, gamma);
        for (int i = 0; i < 1024; ++i) {
            float v = float(i) / float(1023);
            e.inverseLUT[i] = std::min(255.f, std::max(0.f, 255.f * std::pow(v, 1.f / gamma) + .5f));
        }
    }
    return e;
}
float Encoding::ToLinear(uint8_t v) const {
    switch (kind) {
    case kEncLinear: return v / 255.f;
    case kEncSRGB: return GetSpectralData().srgbToLinear[v];
    default: return applyLUT[v];
    }
}
float Encoding::ToFloatLinear(float v) const {
    switch (kind) {
    case kEncLinear: return v;
    case kEncSRGB: return SRGBToLinear(v);
    default: return std::pow(v, gamma);
    }
}
uint8_t Encoding::FromLinear(float v) const {
    switch (kind) {
    case kEncLinear: {
        float x = v * 255.f + 0.5f;
        x = x < 0 ? 0.f : (x > 255 ? 255.f : x);
        return (uint8_t)x;
    }
    case kEncSRGB: return LinearToSRGB8(v);
    default: {
        float x = v * float(1023);
        x = x < 0 ? 0.f : (x > 1023 ? 1023.f : x);
        return (uint8_t)inverseLUT[(size_t)x];
    }
    }
}

// ---------------------------------------------------------------- decoded images
// A decoded image in one of pbrt's three pixel formats (Image, util/image.h:216-479)
struct RawImage {
    int w = 0, h = 0, nc = 0;
    int format = kImgU8;
    std::vector<uint8_t> p8;
    std::vector<uint16_t> p16;
    std::vector<float> p32;
    float Get(size_t i, const Encoding &enc) const {
        switch (format) {
        case kImgU8: return enc.ToLinear(p8[i]);
        case kImgHalf: return HalfToFloat(p16[i]);
        default: return p32[i];
        }
    }
};

static std::string ReadFile(const std::string &fn) {
    std::ifstream in(fn, std::ios::binary);
    if (!in) throw Error(fn + ": unable to open image file");
    std::stringstream ss;
    ss << in.rdbuf();
    return ss.str();
}

static uint32_t BE32(const uint8_t *p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }

// ReadPNG (util/image.cpp:1260-1367): grey / grey-alpha decode to one "Y" channel, everything
// else to RGB, or RGBA when the colour type is RGBA; 16-bit samples become Half through
// ColorEncoding::ToFloatLinear, 8-bit ones stay bytes with the encoding
static RawImage ReadPNG(const std::string &fn, const Encoding &enc) {
    const std::string s = ReadFile(fn);
    const uint8_t *d = (const uint8_t *)s.data();
    const size_t n = s.size();
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) throw Error(fn + ": not a PNG file");
    uint32_t w = 0, h = 0;
    int bitDepth = 0, colorType = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t pos = 8;
    bool end = false;
    while (pos + 12 <= n && !end) {
        uint32_t len = BE32(d + pos);
        std::string type((const char *)d + pos + 4, 4);
        if (pos + 12 + len > n) throw Error(fn + ": truncated PNG chunk " + type);
        const uint8_t *c = d + pos + 8;
        if (type == "IHDR") {
            if (len != 13) throw Error(fn + ": bad IHDR");
            w = BE32(c);
            h = BE32(c + 4);
            bitDepth = c[8];
            colorType = c[9];
            interlace = c[12];
        } else if (type == "PLTE") {
            plte.assign(c, c + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), c, c + len);
        } else if (type == "IEND") {
            end = true;
        }
        pos += 12 + len;
    }
    if (w == 0 || h == 0 || colorType < 0) throw Error(fn + ": PNG without an image header");
    if (interlace) throw Error(fn + ": interlaced PNG files are not supported");
    int samples;
    switch (colorType) {
    case 0: samples = 1; break;
    case 2: samples = 3; break;
    case 3: samples = 1; break;
    case 4: samples = 2; break;
    case 6: samples = 4; break;
    default: throw Error(fn + ": bad PNG colour type");
    }
    // the PNG specification's bit depths per colour type (grey 1/2/4/8/16, palette 1/2/4/8,
    // RGB, grey-alpha and RGBA 8/16); anything else would size rows wrongly
    const bool depthOk = colorType == 0   ? (bitDepth == 1 || bitDepth == 2 || bitDepth == 4 || bitDepth == 8 ||
                                           bitDepth == 16)
                         : colorType == 3 ? (bitDepth == 1 || bitDepth == 2 || bitDepth == 4 || bitDepth == 8)
                                          : (bitDepth == 8 || bitDepth == 16);
    if (!depthOk)
        throw Error(fn + ": bad PNG bit depth " + std::to_string(bitDepth) + " for colour type " +
                    std::to_string(colorType));
    if ((uint64_t)w * h > (1ull << 31)) throw Error(fn + ": PNG image too large");
    if (colorType == 3 && plte.empty()) throw Error(fn + ": paletted PNG without a palette");
    const size_t bitsPerPixel = (size_t)samples * bitDepth;
    const size_t rowBytes = (w * bitsPerPixel + 7) / 8;
    const size_t bpp = std::max<size_t>(1, bitsPerPixel / 8);
    std::vector<uint8_t> raw((rowBytes + 1) * h);
    uLongf rawLen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawLen, idat.data(), (uLong)idat.size()) != Z_OK || rawLen != raw.size())
        throw Error(fn + ": corrupt PNG image data");
    // unfilter (PNG spec 9): None, Sub, Up, Average, Paeth
    std::vector<uint8_t> px(rowBytes * h);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t *in = raw.data() + y * (rowBytes + 1);
        uint8_t *out = px.data() + y * rowBytes;
        const uint8_t *prev = y ? px.data() + (y - 1) * rowBytes : nullptr;
        const int ft = in[0];
        ++in;
        for (size_t i = 0; i < rowBytes; ++i) {
            const int a = i >= bpp ? out[i - bpp] : 0, b = prev ? prev[i] : 0, cc = (prev && i >= bpp) ? prev[i - bpp] : 0;
            int v = in[i];
            switch (ft) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: {
                const int p = a + b - cc, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - cc);
                v += (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : cc);
                break;
            }
            default: throw Error(fn + ": bad PNG filter type");
            }
            out[i] = (uint8_t)v;
        }
    }
    // sample s of pixel x in row y, as an integer of bitDepth bits
    auto sample = [&](uint32_t x, uint32_t y, int sIdx) -> uint32_t {
        const uint8_t *row = px.data() + y * rowBytes;
        if (bitDepth == 16) {
            const uint8_t *p = row + ((size_t)x * samples + sIdx) * 2;
            return (uint32_t(p[0]) << 8) | p[1];
        }
        if (bitDepth == 8) return row[(size_t)x * samples + sIdx];
        const size_t bit = ((size_t)x * samples + sIdx) * bitDepth;
        return (row[bit / 8] >> (8 - bitDepth - bit % 8)) & ((1u << bitDepth) - 1);
    };
    RawImage img;
    img.w = (int)w;
    img.h = (int)h;
    const bool grey = colorType == 0 || colorType == 4;
    const bool hasAlpha = colorType == 6;
    img.nc = grey ? 1 : (hasAlpha ? 4 : 3);
    const bool wide = bitDepth == 16;
    img.format = wide ? kImgHalf : kImgU8;
    const size_t total = (size_t)w * h * img.nc;
    if (wide) img.p16.resize(total);
    else img.p8.resize(total);
    for (uint32_t y = 0; y < h; ++y)
        for (uint32_t x = 0; x < w; ++x) {
            uint32_t v[4] = {0, 0, 0, 0};
            if (colorType == 3) {
                const uint32_t idx = sample(x, y, 0);
                if (3 * idx + 2 >= plte.size()) throw Error(fn + ": PNG palette index out of range");
                for (int c = 0; c < 3; ++c) v[c] = plte[3 * idx + c];
            } else if (grey) {
                v[0] = sample(x, y, 0);
                // lodepng's grey conversion to 8 bits scales 1/2/4-bit samples to 0..255
                if (bitDepth < 8) v[0] = v[0] * 255 / ((1u << bitDepth) - 1);
            } else {
                for (int c = 0; c < img.nc; ++c) v[c] = sample(x, y, c);
            }
            const size_t o = ((size_t)y * w + x) * img.nc;
            for (int c = 0; c < img.nc; ++c) {
                if (wide) img.p16[o + c] = FloatToHalf(enc.ToFloatLinear(v[c] / 65535.f));
                else img.p8[o + c] = (uint8_t)v[c];
            }
        }
    return img;
}

// ReadPFM (util/image.cpp:1614-1695): rows bottom to top, |scale| applied, sign = endianness
static RawImage ReadPFM(const std::string &fn) {
    const std::string s = ReadFile(fn);
    size_t pos = 0;
    auto word = [&]() {
        while (pos < s.size() && std::isspace((unsigned char)s[pos])) ++pos;
        size_t b = pos;
        while (pos < s.size() && !std::isspace((unsigned char)s[pos])) ++pos;
        std::string r = s.substr(b, pos - b);
        if (pos < s.size()) ++pos;  // the single whitespace after the word
        return r;
    };
    std::string magic = word();
    RawImage img;
    if (magic == "Pf") img.nc = 1;
    else if (magic == "PF") img.nc = 3;
    else throw Error(fn + ": unable to decode PFM file type");
    img.w = std::atoi(word().c_str());
    img.h = std::atoi(word().c_str());
    float scale = (float)std::atof(word().c_str());
    if (img.w <= 0 || img.h <= 0) throw Error(fn + ": bad PFM resolution");
    img.format = kImgFloat;
    const size_t nf = (size_t)img.nc * img.w * img.h;
    if (s.size() < pos + nf * 4) throw Error(fn + ": premature end of file in PFM file");
    img.p32.resize(nf);
    const bool fileLittle = scale < 0.f;
    for (int y = img.h - 1; y >= 0; --y) {
        std::memcpy(&img.p32[(size_t)img.nc * y * img.w], s.data() + pos, 4 * img.nc * img.w);
        pos += 4 * img.nc * img.w;
    }
    if (!fileLittle)
        for (float &f : img.p32) {
            uint8_t b[4];
            std::memcpy(b, &f, 4);
            std::swap(b[0], b[3]);
            std::swap(b[1], b[2]);
            std::memcpy(&f, b, 4);
        }
    if (std::abs(scale) != 1.f)
        for (float &f : img.p32) f *= std::abs(scale);
    return img;
}

static bool HasExt(const std::string &fn, const std::string &ext) {
    if (fn.size() <= ext.size()) return false;
    std::string e = fn.substr(fn.size() - ext.size());
    std::transform(e.begin(), e.end(), e.begin(), ::tolower);
    return fn[fn.size() - ext.size() - 1] == '.' && e == ext;
}

// ---------------------------------------------------------------- pyramid
static bool RemapPixel(int *x, int *y, int w, int h, int wrap) {
    // RemapPixelCoords (util/image.h:96-146)
    int p[2] = {*x, *y}, res[2] = {w, h};
    if (wrap == kWrapOctahedral) {
        if (p[0] < 0) {
            p[0] = -p[0];
            p[1] = res[1] - 1 - p[1];
        } else if (p[0] >= res[0]) {
            p[0] = 2 * res[0] - 1 - p[0];
            p[1] = res[1] - 1 - p[1];
        }
        if (p[1] < 0) {
            p[0] = res[0] - 1 - p[0];
            p[1] = -p[1];
        } else if (p[1] >= res[1]) {
            p[0] = res[0] - 1 - p[0];
            p[1] = 2 * res[1] - 1 - p[1];
        }
        if (res[0] == 1) p[0] = 0;
        if (res[1] == 1) p[1] = 0;
    } else {
        for (int c = 0; c < 2; ++c) {
            if (p[c] >= 0 && p[c] < res[c]) continue;
            if (wrap == kWrapRepeat) p[c] = ((p[c] % res[c]) + res[c]) % res[c];
            else if (wrap == kWrapClamp) p[c] = std::min(std::max(p[c], 0), res[c] - 1);
            else return false;
        }
    }
    *x = p[0];
    *y = p[1];
    return true;
}

struct ResampleWeight {
    int firstPixel;
    float weight[4];
};
static std::vector<ResampleWeight> ResampleWeights(int oldRes, int newRes) {
    std::vector<ResampleWeight> wt(newRes);
    const float filterRadius = 2, tau = 2;
    for (int i = 0; i < newRes; ++i) {
        float center = (i + .5f) * oldRes / newRes;
        wt[i].firstPixel = (int)std::floor((center - filterRadius) + 0.5f);
        for (int j = 0; j < 4; ++j) {
            float pos = wt[i].firstPixel + j + .5f;
            wt[i].weight[j] = WindowedSinc(pos - center, filterRadius, tau);
        }
        float invSumWts = 1 / (wt[i].weight[0] + wt[i].weight[1] + wt[i].weight[2] + wt[i].weight[3]);
        for (int j = 0; j < 4; ++j) wt[i].weight[j] *= invSumWts;
    }
    return wt;
}

// Image::FloatResizeUp (util/image.cpp:230-311): separable 4-tap windowed-sinc upsampling, the
// x pass over every needed source row, then the y pass, clamped at zero
static std::vector<float> FloatResizeUp(const std::vector<float> &src, int w, int h, int nc, int nw, int nh, int wrap) {
    if (wrap == kWrapBlack) throw Error("black wrap mode on a non power-of-two image (pbrt's FloatResizeUp CHECK fails)");
    std::vector<ResampleWeight> xw = ResampleWeights(w, nw), yw = ResampleWeights(h, nh);
    auto in = [&](int x, int y, int c) {
        RemapPixel(&x, &y, w, h, wrap);
        return src[((size_t)y * w + x) * nc + c];
    };
    // x pass: rows yIn in [yw[0].firstPixel, yw[nh-1].firstPixel + 4)
    const int y0 = yw[0].firstPixel, y1 = yw[nh - 1].firstPixel + 4;
    std::vector<float> xb((size_t)(y1 - y0) * nw * nc);
    for (int y = y0; y < y1; ++y)
        for (int x = 0; x < nw; ++x) {
            const ResampleWeight &r = xw[x];
            for (int c = 0; c < nc; ++c)
                xb[((size_t)(y - y0) * nw + x) * nc + c] =
                    r.weight[0] * in(r.firstPixel, y, c) + r.weight[1] * in(r.firstPixel + 1, y, c) +
                    r.weight[2] * in(r.firstPixel + 2, y, c) + r.weight[3] * in(r.firstPixel + 3, y, c);
        }
    std::vector<float> out((size_t)nw * nh * nc);
    for (int y = 0; y < nh; ++y) {
        const ResampleWeight &r = yw[y];
        for (int x = 0; x < nw; ++x)
            for (int c = 0; c < nc; ++c) {
                auto b = [&](int k) { return xb[((size_t)(r.firstPixel + k - y0) * nw + x) * nc + c]; };
                out[((size_t)y * nw + x) * nc + c] =
                    std::max<float>(0, (r.weight[0] * b(0) + r.weight[1] * b(1) + r.weight[2] * b(2) + r.weight[3] * b(3)));
            }
    }
    return out;
}

static int RoundUpPow2(int v) {
    v--;
    v |= v >> 1;
    v |= v >> 2;
    v |= v >> 4;
    v |= v >> 8;
    v |= v >> 16;
    return v + 1;
}
static bool IsPow2(int v) { return v && !(v & (v - 1)); }
static int Log2Int(uint32_t v) { return 31 - __builtin_clz(v); }

// store one float level in the original format (CopyRectIn, util/image.cpp:710-752)
static void StoreLevel(ImageDesc &img, const std::vector<float> &f, const Encoding &enc) {
    const size_t n = f.size();
    const size_t off = img.data.size();
    img.levelOffset.push_back(off);
    if (img.format == kImgU8) {
        img.data.resize(off + n);
        for (size_t i = 0; i < n; ++i) img.data[off + i] = enc.FromLinear(f[i]);
    } else if (img.format == kImgHalf) {
        img.data.resize(off + 2 * n);
        for (size_t i = 0; i < n; ++i) {
            uint16_t hv = FloatToHalf(f[i]);
            std::memcpy(&img.data[off + 2 * i], &hv, 2);
        }
    } else {
        img.data.resize(off + 4 * n);
        std::memcpy(&img.data[off], f.data(), 4 * n);
    }
    // keep every level 16-byte aligned
    img.data.resize((img.data.size() + 15) & ~size_t(15));
}

ImageDesc LoadImageTexture(const std::string &filename, const std::string &encodingName, int wrap, const std::string &loc) {
    const Encoding enc = Encoding::Get(encodingName, loc);
    RawImage raw;
    if (HasExt(filename, "png")) raw = ReadPNG(filename, enc);
    else if (HasExt(filename, "pfm")) raw = ReadPFM(filename);
    else throw Error(loc + ": " + filename + ": only PNG and PFM image textures are supported");
    // MIPMap::CreateFromFile: RGBA whose alpha is 1 everywhere drops to RGB
    if (raw.nc == 4) {
        bool allOne = true;
        for (size_t i = 3; i < (size_t)raw.w * raw.h * 4 && allOne; i += 4) allOne = raw.Get(i, enc) == 1;
        if (allOne) {
            RawImage rgb = raw;
            rgb.nc = 3;
            const size_t np = (size_t)raw.w * raw.h;
            if (raw.format == kImgU8) {
                rgb.p8.resize(np * 3);
                for (size_t p = 0; p < np; ++p)
                    for (int c = 0; c < 3; ++c) rgb.p8[3 * p + c] = raw.p8[4 * p + c];
            } else {
                rgb.p16.resize(np * 3);
                for (size_t p = 0; p < np; ++p)
                    for (int c = 0; c < 3; ++c) rgb.p16[3 * p + c] = raw.p16[4 * p + c];
            }
            raw = std::move(rgb);
        }
    }
    ImageDesc img;
    img.filename = filename;
    img.format = raw.format;
    img.nc = raw.nc;
    img.wrap = wrap;
    for (int i = 0; i < 256; ++i) img.toLinear[i] = enc.ToLinear((uint8_t)i);
    img.rawW = raw.w;
    img.rawH = raw.h;
    img.encoding = enc.kind;
    img.gamma = enc.gamma;
    if (raw.format == kImgU8) img.raw = raw.p8;
    else if (raw.format == kImgHalf) img.raw.assign((const uint8_t *)raw.p16.data(), (const uint8_t *)raw.p16.data() + 2 * raw.p16.size());
    else img.raw.assign((const uint8_t *)raw.p32.data(), (const uint8_t *)raw.p32.data() + 4 * raw.p32.size());
    // GeneratePyramid: float image at a power-of-two resolution
    int w = raw.w, h = raw.h;
    const int nc = raw.nc;
    std::vector<float> f((size_t)w * h * nc);
    for (size_t i = 0; i < f.size(); ++i) f[i] = raw.Get(i, enc);
    if (!IsPow2(w) || !IsPow2(h)) {
        const int nw = RoundUpPow2(w), nh = RoundUpPow2(h);
        f = FloatResizeUp(f, w, h, nc, nw, nh, wrap);
        w = nw;
        h = nh;
    }
    const int nLevels = 1 + Log2Int((uint32_t)std::max(w, h));
    for (int i = 0; i < nLevels - 1; ++i) {
        img.levelRes.push_back({w, h});
        StoreLevel(img, f, enc);
        const int nw = std::max(1, w / 2), nh = std::max(1, h / 2);
        int d1 = nc, d2 = nc * w, d3 = nc * (w + 1);
        if (w == 1) {
            d1 = 0;
            d3 -= nc;
        }
        if (h == 1) {
            d2 = 0;
            d3 -= nc * w;
        }
        std::vector<float> next((size_t)nw * nh * nc);
        for (int y = 0; y < nh; ++y) {
            size_t so = (size_t)nc * (2 * y) * w, no = (size_t)nc * y * nw;
            for (int x = 0; x < nw; ++x, so += nc)
                for (int c = 0; c < nc; ++c, ++so, ++no)
                    next[no] = (f[so] + f[so + d1] + f[so + d2] + f[so + d3]) / 4;
        }
        f.swap(next);
        w = nw;
        h = nh;
    }
    img.levelRes.push_back({w, h});
    StoreLevel(img, f, enc);
    return img;
}

LightImage LoadLightImage(const std::string &filename, const std::string &loc) {
    LightImage li;
    if (HasExt(filename, "exr")) {
        Image im;
        try {
            im = ReadImage(filename);
        } catch (const std::exception &e) {
            throw Error(loc + ": " + e.what());
        }
        li.w = im.width;
        li.h = im.height;
        li.nc = 3;
        li.exr = true;
        li.v = std::move(im.rgb);
        return li;
    }
    const Encoding enc = Encoding::Get("sRGB", loc);
    RawImage raw;
    if (HasExt(filename, "png")) raw = ReadPNG(filename, enc);
    else if (HasExt(filename, "pfm")) raw = ReadPFM(filename);
    else throw Error(loc + ": " + filename + ": only PNG, PFM and EXR light images are supported");
    li.w = raw.w;
    li.h = raw.h;
    li.nc = raw.nc;
    li.format = raw.format;
    li.v.resize((size_t)raw.w * raw.h * raw.nc);
    for (size_t i = 0; i < li.v.size(); ++i) li.v[i] = raw.Get(i, enc);
    return li;
}
float LightImage::Restore(float v) const {
    static const Encoding enc = Encoding::Get("sRGB", "");
    switch (format) {
    case kImgU8: return enc.ToLinear(enc.FromLinear(v));
    case kImgHalf: return HalfToFloat(FloatToHalf(v));
    default: return v;
    }
}

EnvLightDesc LoadEnvironmentImage(const std::string &filename, const std::string &loc) {
    EnvLightDesc env;
    int w = 0, h = 0;
    if (HasExt(filename, "exr")) {
        Image im;
        try {
            im = ReadImage(filename);
        } catch (const std::exception &e) {
            throw Error(loc + ": " + e.what());
        }
        w = im.width;
        h = im.height;
        env.rgb = std::move(im.rgb);
    } else {
        const Encoding enc = Encoding::Get("sRGB", loc);
        RawImage raw;
        if (HasExt(filename, "png")) raw = ReadPNG(filename, enc);
        else if (HasExt(filename, "pfm")) raw = ReadPFM(filename);
        else throw Error(loc + ": " + filename + ": only PNG, PFM and EXR environment images are supported");
        if (raw.nc < 3)
            throw Error(loc + ": " + filename + ": image provided to \"infinite\" light must have R, G, and B channels.");
        w = raw.w;
        h = raw.h;
        env.rgb.resize((size_t)3 * w * h);
        for (size_t p = 0; p < (size_t)w * h; ++p)
            for (int c = 0; c < 3; ++c) env.rgb[3 * p + c] = raw.Get(p * raw.nc + c, enc);
    }
    if (w != h)
        throw Error(loc + ": " + filename + ": image resolution (" + std::to_string(w) + ", " + std::to_string(h) +
                    ") is non-square. It's unlikely this is an equal area environment map.");
    env.res = w;
    return env;
}

// Decoded texel value (GetChannel, util/image.h:255-276) of a stored level
float ImageTexel(const ImageDesc &img, int level, int x, int y, int c) {
    const auto &r = img.levelRes[level];
    if (!RemapPixel(&x, &y, r[0], r[1], img.wrap)) return 0;
    const size_t i = ((size_t)y * r[0] + x) * img.nc + c;
    const uint8_t *base = img.data.data() + img.levelOffset[level];
    switch (img.format) {
    case kImgU8: return img.toLinear[base[i]];
    case kImgHalf: {
        uint16_t hv;
        std::memcpy(&hv, base + 2 * i, 2);
        return HalfToFloat(hv);
    }
    default: {
        float v;
        std::memcpy(&v, base + 4 * i, 4);
        return v;
    }
    }
}

}  // namespace pbrt_amd

namespace pbrt_amd {

// ---------------------------------------------------------------- expression compiler
// Lowers a texture tree to the two-phase program core/texture_eval.h runs (see scene.h
// TexProgram).  Phase 1 evaluates every float sub-texture, image lookup and weight once per
// hit; phase 2 replays the spectrum arithmetic of the tree per wavelength in pbrt's order.
namespace {
constexpr int kMaxRegs = kTexMaxRegs, kMaxStack = kTexMaxStack;
struct TexCompiler {
    SceneDesc &s;
    std::vector<TexInstr> p1, p2;
    int nRegs = 0, depth = 0;
    int NewReg(int n = 1) {
        const int r = nRegs;
        nRegs += n;
        if (nRegs > kMaxRegs) throw Error("texture expression too large (more than 16 scalar registers)");
        return r;
    }
    void Emit1(int op, int a, int b, int c, int node) { p1.push_back(TexInstr{op, a, b, c, node}); }
    void Emit2(int op, int a, int b, int node, int pushes) {
        p2.push_back(TexInstr{op, a, b, 0, node});
        depth += pushes;
        if (depth > kMaxStack) throw Error("texture expression too deep (more than 8 pending spectra)");
    }
    int F(int node) {
        const TextureDesc &t = s.textures[node];
        if (t.spectrum) throw Error("internal: spectrum texture where a float texture is needed");
        int r;
        switch (t.kind) {
        case kTexConstant: r = NewReg(); Emit1(kT1FConst, r, 0, 0, node); return r;
        case kTexImage: r = NewReg(); Emit1(kT1FImage, r, 0, 0, node); return r;
        case kTexBilerp: r = NewReg(); Emit1(kT1FBilerp, r, 0, 0, node); return r;
        case kTexCheckerboard: {
            const int w = NewReg();
            Emit1(kT1CheckW, w, 0, 0, node);
            const int a = F(t.child[0]), b = F(t.child[1]);
            r = NewReg();
            Emit1(kT1FMix, r, a, b, w);
            return r;
        }
        case kTexMix: {
            const int amt = F(t.child[2]), a = F(t.child[0]), b = F(t.child[1]);
            r = NewReg();
            Emit1(kT1FMix, r, a, b, amt);
            return r;
        }
        case kTexDirectionMix: {
            const int amt = NewReg();
            Emit1(kT1DirAmt, amt, 0, 0, node);
            const int a = F(t.child[0]), b = F(t.child[1]);
            r = NewReg();
            Emit1(kT1FDMix, r, a, b, amt);
            return r;
        }
        case kTexScale: {
            const int a = F(t.child[0]), b = F(t.child[1]);
            r = NewReg();
            Emit1(kT1FScale, r, a, b, -1);
            return r;
        }
        case kTexFBm: r = NewReg(); Emit1(kT1FBm, r, 0, 0, node); return r;
        case kTexWrinkled: r = NewReg(); Emit1(kT1Wrinkled, r, 0, 0, node); return r;
        case kTexWindy: r = NewReg(); Emit1(kT1Windy, r, 0, 0, node); return r;
        case kTexDots: {
            const int w = NewReg();
            Emit1(kT1DotsW, w, 0, 0, node);
            const int a = F(t.child[0]), b = F(t.child[1]);
            r = NewReg();
            Emit1(kT1FSel, r, a, b, w);
            return r;
        }
        }
        throw Error("internal: unknown texture kind");
    }
    void S(int node) {
        const TextureDesc &t = s.textures[node];
        if (!t.spectrum) throw Error("internal: float texture where a spectrum texture is needed");
        switch (t.kind) {
        case kTexConstant: Emit2(kT2Const, 0, 0, node, 1); return;
        case kTexImage: {
            if (t.basis >= 0) {  // multispectral basis: the raw RGB, then the per-sample basis sum
                const int r = NewReg(3);
                Emit1(kT1SBasisRGB, r, 0, 0, node);
                Emit2(kT2Basis, r, 0, node, 1);
                return;
            }
            const int r = NewReg(4);
            Emit1(kT1SImage, r, 0, 0, node);
            Emit2(kT2RGBReg, r, t.specType == kSpecUnbounded ? 1 : 0, -1, 1);
            return;
        }
        case kTexScale: {
            S(t.child[0]);
            const int sc = F(t.child[1]);
            Emit2(kT2Scale, sc, 0, -1, 0);
            return;
        }
        case kTexMix: {
            const int amt = F(t.child[2]);
            S(t.child[0]);
            S(t.child[1]);
            Emit2(kT2Mix, amt, 0, -1, -1);
            return;
        }
        case kTexCheckerboard: {
            const int w = NewReg();
            Emit1(kT1CheckW, w, 0, 0, node);
            S(t.child[0]);
            S(t.child[1]);
            Emit2(kT2Mix, w, 0, -1, -1);
            return;
        }
        case kTexDirectionMix: {
            const int amt = NewReg();
            Emit1(kT1DirAmt, amt, 0, 0, node);
            S(t.child[0]);
            S(t.child[1]);
            Emit2(kT2DMix, amt, 0, -1, -1);
            return;
        }
        case kTexBilerp: {
            const int w = NewReg(4);
            Emit1(kT1BilerpW, w, 0, 0, node);
            for (int k = 0; k < 4; ++k) Emit2(kT2Const, k, 0, node, 1);
            Emit2(kT2Bilerp, w, 0, -1, -3);
            return;
        }
        case kTexDots: {
            const int w = NewReg();
            Emit1(kT1DotsW, w, 0, 0, node);
            S(t.child[0]);
            S(t.child[1]);
            Emit2(kT2Sel, w, 0, -1, -1);
            return;
        }
        case kTexMarble: {
            const int r = NewReg(4);
            Emit1(kT1Marble, r, 0, 0, node);
            Emit2(kT2RGBReg, r, 0, -1, 1);
            return;
        }
        }
        throw Error("internal: unknown texture kind");
    }
};
}  // namespace

int CompileTexProgram(SceneDesc &s, int node, bool spectrum) {
    TexCompiler c{s};
    TexProgram pg;
    pg.spectrum = spectrum;
    pg.root = node;
    if (spectrum) c.S(node);
    else pg.result = c.F(node);
    pg.p1 = (int)s.texInstrs.size();
    pg.n1 = (int)c.p1.size();
    s.texInstrs.insert(s.texInstrs.end(), c.p1.begin(), c.p1.end());
    pg.p2 = (int)s.texInstrs.size();
    pg.n2 = (int)c.p2.size();
    s.texInstrs.insert(s.texInstrs.end(), c.p2.begin(), c.p2.end());
    pg.nRegs = c.nRegs;
    s.texPrograms.push_back(pg);
    return (int)s.texPrograms.size() - 1;
}

// ---------------------------------------------------------------- camera differentials
static V3 XfP(const float *m, V3 p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1) return V3(xp, yp, zp);
    return V3(xp, yp, zp) / wp;
}
static V3 XfV(const float *m, V3 v) {
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}

// CameraBase::FindMinimumDifferentials (cameras.cpp:170-216) over
// PerspectiveCamera::GenerateRayDifferential (cameras.cpp:458-520), in float on the device's
// camera matrices; also CameraFromRender for Approximate_dp_dxy
void ComputeCameraDifferentials(SceneDesc &s) {
    float cfr[16], rfc[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            cfr[4 * i + j] = (float)s.camera.cameraFromRaster[i][j];
            rfc[4 * i + j] = (float)s.camera.renderFromCamera[i][j];
        }
    const Mat4 inv = Inverse4(s.camera.renderFromCamera);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 4; ++j) s.cameraFromRender[4 * i + j] = (float)inv[i][j];
    const float *ci = s.cameraFromRender;
    auto cameraFromRenderV = [&](V3 v) {
        return V3(ci[0] * v.x + ci[1] * v.y + ci[2] * v.z, ci[4] * v.x + ci[5] * v.y + ci[6] * v.z,
                  ci[8] * v.x + ci[9] * v.y + ci[10] * v.z);
    };
    const V3 dxCamera = XfP(cfr, V3(1, 0, 0)) - XfP(cfr, V3(0, 0, 0));
    const V3 dyCamera = XfP(cfr, V3(0, 1, 0)) - XfP(cfr, V3(0, 0, 0));
    const float inf = std::numeric_limits<float>::infinity();
    V3 mpx(inf, inf, inf), mpy = mpx, mdx = mpx, mdy = mpx;
    const int n = 512;
    for (int i = 0; i < n; ++i) {
        const float fx = float(i) / (n - 1) * s.xres, fy = float(i) / (n - 1) * s.yres;
        const V3 pCamera = XfP(cfr, V3(fx, fy, 0));
        V3 o(0, 0, 0), d = Normalize(pCamera), rxo = o, ryo = o, rxd, ryd;
        if (s.camera.lensRadius > 0) {
            // pLens = lensRadius * SampleUniformDiskConcentric(0.5, 0.5) = (0, 0)
            const float fd = s.camera.focalDistance;
            const float ft = fd / d.z;
            const V3 pFocus = o + d * ft;
            d = Normalize(pFocus - o);
            const V3 dx = Normalize(pCamera + dxCamera);
            const float ftx = fd / dx.z;
            rxd = Normalize((V3(0, 0, 0) + ftx * dx) - rxo);
            const V3 dy = Normalize(pCamera + dyCamera);
            const float fty = fd / dy.z;
            ryd = Normalize((V3(0, 0, 0) + fty * dy) - ryo);
        } else {
            rxd = Normalize(pCamera + dxCamera);
            ryd = Normalize(pCamera + dyCamera);
        }
        // RenderFromCamera(RayDifferential): origin offset to its error bound (as k_camera)
        V3 oo = XfP(rfc, o);
        const V3 err = gamma(3) * Abs(V3(rfc[3], rfc[7], rfc[11]));
        const V3 dd = XfV(rfc, d);
        const float l2 = LengthSquared(dd);
        if (l2 > 0) oo = oo + dd * (Dot(Abs(dd), err) / l2);
        const V3 rxO = XfP(rfc, rxo), ryO = XfP(rfc, ryo);
        const V3 rxD = XfV(rfc, rxd), ryD = XfV(rfc, ryd);
        const V3 dox = cameraFromRenderV(rxO - oo), doy = cameraFromRenderV(ryO - oo);
        if (Length(dox) < Length(mpx)) mpx = dox;
        if (Length(doy) < Length(mpy)) mpy = doy;
        const V3 rd = Normalize(dd), rdx = Normalize(rxD), rdy = Normalize(ryD);
        V3 fxv, fyv;
        CoordinateSystem(rd, &fxv, &fyv);  // Frame::FromZ
        auto toLocal = [&](V3 v) { return V3(Dot(v, fxv), Dot(v, fyv), Dot(v, rd)); };
        const V3 df = toLocal(rd), dxf = Normalize(toLocal(rdx)), dyf = Normalize(toLocal(rdy));
        if (Length(dxf - df) < Length(mdx)) mdx = dxf - df;
        if (Length(dyf - df) < Length(mdy)) mdy = dyf - df;
    }
    for (int k = 0; k < 3; ++k) {
        s.minPosDx[k] = mpx[k];
        s.minPosDy[k] = mpy[k];
        s.minDirDx[k] = mdx[k];
        s.minDirDy[k] = mdy[k];
    }
}

void BuildTexTables(const SceneDesc &s, TexTables *t) {
    *t = TexTables{};
    t->basis = s.texBasis;
    t->basis.push_back(0.f);
    for (size_t i = 0; i < s.textures.size(); ++i) {
        const TextureDesc &d = s.textures[i];
        DeviceTexNode n{};
        n.kind = d.kind;
        n.flags = (d.spectrum ? 1 : 0) | (d.specType << 1) | (d.invert ? 8 : 0) | (d.mapping == kMap3D ? 16 : 0) |
                  (d.basis >= 0 ? kTexNodeBasis : 0);
        n.child0 = d.child[0];
        n.child1 = d.child[1];
        n.child2 = d.child[2];
        n.image = d.image;
        n.mapping = d.mapping == kMap3D ? 0 : d.mapping;
        n.filter = d.filter;
        for (int k = 0; k < 12; ++k) n.p[k] = d.textureFromRender[k];
        for (int k = 0; k < 3; ++k) n.p[12 + k] = d.vs[k], n.p[15 + k] = d.vt[k];
        for (int k = 0; k < 4; ++k) n.p[18 + k] = d.map[k];
        for (int k = 0; k < 4; ++k) n.p[22 + k] = d.fvalue[k];
        if (d.kind == kTexDirectionMix)
            for (int k = 0; k < 3; ++k) n.p[22 + k] = d.dir[k];
        n.p[26] = d.scale;
        n.p[27] = d.maxAniso;
        if (d.basis >= 0) {  // the multispectral basis table: start in texBasis, length
            n.p[22] = (float)d.basis;
            n.p[24] = (float)d.basisWidth;
        }
        if (d.kind >= kTexDots) {  // procedural: octaves, omega, variation (core/texture_eval.h)
            n.p[22] = (float)d.octaves;
            n.p[23] = d.omega;
            n.p[24] = d.variation;
        }
        t->nodes.push_back(n);
        for (int k = 0; k < 4; ++k) {
            const TexSpectrumConst &c = d.svalue[k];
            t->spec.push_back(DeviceTexSpec{c.rgb ? 1.f : 0.f, c.value, c.c[0], c.c[1], c.c[2], c.scale, 0.f, 0.f});
        }
        t->nodeInfo.insert(t->nodeInfo.end(), {n.kind, n.flags, n.child0, n.child1, n.child2, n.image, n.mapping, n.filter});
        t->nodeParams.insert(t->nodeParams.end(), n.p, n.p + 28);
        for (int k = 0; k < 4; ++k) {
            const DeviceTexSpec &q = t->spec[4 * i + k];
            t->specFlat.insert(t->specFlat.end(), {q.rgb, q.value, q.c0, q.c1, q.c2, q.scale, 0.f, 0.f});
        }
    }
    for (size_t i = 0; i < s.images.size(); ++i) {
        const ImageDesc &im = s.images[i];
        DeviceImage di{};
        di.format = im.format;
        di.nc = im.nc;
        di.nLevels = (int)im.levelRes.size();
        di.wrap = im.wrap;
        di.levelBase = (int)t->levels.size();
        di.lutBase = (int)(256 * i);
        const uint64_t base = t->data.size();
        t->data.insert(t->data.end(), im.data.begin(), im.data.end());
        t->data.resize((t->data.size() + 15) & ~size_t(15));
        for (size_t l = 0; l < im.levelRes.size(); ++l) {
            const uint64_t off = base + im.levelOffset[l];
            t->levels.push_back(DeviceImageLevel{im.levelRes[l][0], im.levelRes[l][1], (uint32_t)off, (uint32_t)(off >> 32)});
            t->levelInfo.insert(t->levelInfo.end(), {im.levelRes[l][0], im.levelRes[l][1], (int32_t)(uint32_t)off,
                                                     (int32_t)(uint32_t)(off >> 32)});
        }
        t->luts.insert(t->luts.end(), im.toLinear.begin(), im.toLinear.end());
        t->images.push_back(di);
        t->imageInfo.insert(t->imageInfo.end(), {di.format, di.nc, di.nLevels, di.wrap, di.levelBase, di.lutBase, 0, 0});
        t->rawInfo.insert(t->rawInfo.end(), {im.rawW, im.rawH, im.format, im.nc, im.encoding, 0, 0, 0});
        t->rawGamma.push_back(im.gamma);
        t->rawOffset.push_back(t->rawData.size());
        t->rawData.insert(t->rawData.end(), im.raw.begin(), im.raw.end());
    }
    for (const TexInstr &in : s.texInstrs)
        t->instrs.push_back(DeviceTexInstr{in.op | (in.a << 8) | (in.b << 16) | (in.c << 24), in.node});
    for (const TexProgram &pg : s.texPrograms) {
        int simple = 0;
        if (pg.spectrum && pg.n1 == 1 && pg.n2 == 1) {
            const TexInstr &a = s.texInstrs[pg.p1], &b = s.texInstrs[pg.p2];
            simple = a.op == kT1SImage && a.a == 0 && b.op == kT2RGBReg && b.a == 0 && b.b == 0;
        }
        t->progs.push_back(DeviceTexProgram{pg.p1, pg.n1, pg.p2, pg.n2, pg.result, pg.nRegs, simple, 0});
    }
    for (const MaterialDesc &m : s.materials) {
        t->matTex.insert(t->matTex.end(), {m.texReflectance, m.texURough, m.texVRough, m.remapRoughness ? 1 : 0});
        auto root = [&](int p) { return p >= 0 ? s.texPrograms[p].root : -1; };
        t->matTexNode.insert(t->matTexNode.end(),
                             {root(m.texReflectance), root(m.texURough), root(m.texVRough), m.remapRoughness ? 1 : 0});
        t->matMixNode.insert(t->matMixNode.end(), {m.mixMat[0], m.mixMat[1], root(m.texAmount), 0});
        t->matBumpNode.insert(t->matBumpNode.end(), {root(m.texDisp), m.normalMap});
        for (int k = 0; k < 6; ++k) {
            t->matHairNode.push_back(root(m.texHair[k]));
            t->anyHairTex = t->anyHairTex || m.texHair[k] >= 0;
        }
        for (int k = 0; k < 2; ++k) {
            t->matSssNode.push_back(root(m.texSss[k]));
            t->anySssTex = t->anySssTex || m.texSss[k] >= 0;
        }
    }
}
// a TexView over host copies (debug entry points; the device view points at DevBufs)
TexView HostTexView(const TexTables &t) {
    const std::vector<float> &rgb = RGBToSpectrumTableData();
    TexView v{};
    v.nodes = t.nodes.data();
    v.spec = t.spec.data();
    v.images = t.images.data();
    v.levels = t.levels.data();
    v.data = t.data.data();
    v.luts = t.luts.data();
    v.instrs = t.instrs.data();
    v.progs = t.progs.data();
    v.rgbZNodes = rgb.data();
    v.rgbCoeffs = rgb.data() + 64;
    v.ewaLut = GetSpectralData().mipFilterLUT.data();
    v.noisePerm = GetSpectralData().noisePerm.data();
    v.basis = t.basis.data();
    v.nProgs = (int)t.progs.size();
    v.nLuts = (int)t.images.size();
    return v;
}

float HostTexFloat(const TexView &T, int prog, const TexEvalCtx &c) {
    float R[kTexMaxRegs];
    const DeviceTexProgram pg = T.progs[prog];
    TexPhase1(T, pg, c, R);
    return R[pg.result];
}

}  // namespace pbrt_amd
