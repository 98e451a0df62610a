// Image output and comparison: the formats pbrt-v4 writes a film to
// and the error metrics of its imgtool, restated without the image libraries the reference
// links (OpenEXR, lodepng), which this image does not have.
//
//   PFM  Image::WritePFM / ReadPFM (util/image.cpp:1614-1800): "PF", width height, scale -1
//        (little endian), rows bottom to top, 3 floats per pixel.
//   EXR  OpenEXR single-part scanline file, NO_COMPRESSION, channels B G R (the file format
//        sorts them), HALF (pbrt's RGBFilm default, writefp16 = true, film.cpp) or FLOAT.
//        The reader accepts exactly what the writer emits (uncompressed scanline, HALF/FLOAT
//        R G B [A]); anything else is rejected loudly.
//   PNG  8-bit sRGB-encoded RGB (Image::WritePNG converts to U256 with the sRGB curve), zlib
//        stream of stored (uncompressed) deflate blocks.
//   metrics  Image::MAE / MSE / MRSE (util/image.cpp:543-639) as imgtool diff/error call them
//        (cmd/imgtool.cpp:960-1105): per channel, double sums over pixels / (x res * y res);
//        MAE is pbrt's signed mean difference; infinite terms are skipped.
#include "image.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace pbrt_amd {

static std::string Ext(const std::string &path) {
    size_t dot = path.rfind('.');
    if (dot == std::string::npos) return "";
    std::string e = path.substr(dot + 1);
    for (char &c : e) c = (char)std::tolower((unsigned char)c);
    return e;
}

struct File {
    FILE *f;
    File(const std::string &p, const char *mode) : f(std::fopen(p.c_str(), mode)) {
        if (!f) throw std::runtime_error(p + ": unable to open");
    }
    ~File() {
        if (f) std::fclose(f);
    }
};

// ---------------------------------------------------------------- PFM
static void WritePFM(const std::string &path, const float *rgb, int w, int h) {
    File fp(path, "wb");
    std::fprintf(fp.f, "PF\n%d %d\n%f\n", w, h, -1.f);  // negative scale: little endian
    for (int y = h - 1; y >= 0; --y)
        if (std::fwrite(rgb + (size_t)3 * w * y, sizeof(float), (size_t)3 * w, fp.f) != (size_t)3 * w)
            throw std::runtime_error(path + ": write failed");
}

static std::string ReadWord(FILE *f) {
    std::string s;
    int c;
    while ((c = std::fgetc(f)) != EOF && std::isspace(c)) {
    }
    while (c != EOF && !std::isspace(c)) {
        s.push_back((char)c);
        c = std::fgetc(f);
    }
    return s;
}

static Image ReadPFM(const std::string &path) {
    File fp(path, "rb");
    const std::string magic = ReadWord(fp.f);
    int nc = magic == "PF" ? 3 : (magic == "Pf" ? 1 : 0);
    if (!nc) throw std::runtime_error(path + ": not a PFM file");
    Image im;
    im.width = std::stoi(ReadWord(fp.f));
    im.height = std::stoi(ReadWord(fp.f));
    const float scale = std::stof(ReadWord(fp.f));
    const size_t n = (size_t)nc * im.width * im.height;
    std::vector<float> raw(n);
    for (int y = im.height - 1; y >= 0; --y)
        if (std::fread(&raw[(size_t)nc * im.width * y], sizeof(float), (size_t)nc * im.width, fp.f) !=
            (size_t)nc * im.width)
            throw std::runtime_error(path + ": premature end of PFM file");
    if (scale > 0)  // big-endian file on this little-endian host
        for (float &v : raw) {
            uint32_t u;
            std::memcpy(&u, &v, 4);
            u = __builtin_bswap32(u);
            std::memcpy(&v, &u, 4);
        }
    if (std::fabs(scale) != 1.f)
        for (float &v : raw) v *= std::fabs(scale);
    im.rgb.resize((size_t)3 * im.width * im.height);
    for (size_t i = 0; i < (size_t)im.width * im.height; ++i)
        for (int c = 0; c < 3; ++c) im.rgb[3 * i + c] = raw[nc * i + (nc == 3 ? c : 0)];
    return im;
}

// ---------------------------------------------------------------- half floats
static uint16_t FloatToHalf(float f) {  // round to nearest even, inf / nan kept
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t exp = (x >> 23) & 0xffu;
    uint32_t mant = x & 0x7fffffu;
    if (exp == 0xff) return (uint16_t)(sign | 0x7c00u | (mant ? 0x200u : 0u));
    int e = (int)exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);  // overflow -> inf
    if (e <= 0) {                                     // subnormal half (or zero)
        if (e < -10) return (uint16_t)sign;
        mant |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = mant >> shift;
        const uint32_t rem = mant & ((1u << shift) - 1), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) ++h;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (mant >> 13);
    const uint32_t rem = mant & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;  // may carry into the exponent: fine
    return (uint16_t)(sign | h);
}
static float HalfToFloat(uint16_t h) {
    const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
    uint32_t exp = (h >> 10) & 0x1fu, mant = h & 0x3ffu, x;
    if (exp == 0) {
        if (mant == 0) {
            x = sign;
        } else {
            exp = 1;
            while (!(mant & 0x400u)) {
                mant <<= 1;
                --exp;
            }
            mant &= 0x3ffu;
            x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
        }
    } else if (exp == 31) {
        x = sign | 0x7f800000u | (mant << 13);
    } else {
        x = sign | ((exp + 127 - 15) << 23) | (mant << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

// ---------------------------------------------------------------- EXR
struct Bytes {
    std::vector<uint8_t> b;
    void u8(uint8_t v) { b.push_back(v); }
    void u32(uint32_t v) {
        for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(v >> (8 * i)));
    }
    void i32(int32_t v) { u32((uint32_t)v); }
    void u64(uint64_t v) {
        for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(v >> (8 * i)));
    }
    void f32(float v) {
        uint32_t u;
        std::memcpy(&u, &v, 4);
        u32(u);
    }
    void str(const char *s) {
        while (*s) b.push_back((uint8_t)*s++);
        b.push_back(0);
    }
    void attr(const char *name, const char *type, const Bytes &value) {
        str(name);
        str(type);
        u32((uint32_t)value.b.size());
        b.insert(b.end(), value.b.begin(), value.b.end());
    }
};

// win = {x0, y0, fullW, fullH}: the image covers the film's pixelBounds starting at (x0, y0) of a
// fullW x fullH frame (Image::WriteEXR, util/image.cpp:1179-1200: displayWindow = full resolution,
// dataWindow = pixelBounds; scanline y coordinates are absolute).
static void WriteEXR(const std::string &path, const float *rgb, int w, int h, bool half, const int win[4]) {
    const int pt = half ? 1 : 2, bpc = half ? 2 : 4;  // pixel type HALF / FLOAT
    Bytes hdr;
    hdr.u32(20000630u);  // magic
    hdr.u32(2u);         // version 2, single-part scanline
    {
        Bytes ch;
        for (const char *name : {"B", "G", "R"}) {  // channel list sorted by name
            ch.str(name);
            ch.i32(pt);
            ch.u8(0);  // pLinear
            ch.u8(0), ch.u8(0), ch.u8(0);
            ch.i32(1), ch.i32(1);  // x / y sampling
        }
        ch.u8(0);
        hdr.attr("channels", "chlist", ch);
    }
    {
        Bytes v;
        v.u8(0);  // NO_COMPRESSION
        hdr.attr("compression", "compression", v);
    }
    {
        Bytes data, disp;
        data.i32(win[0]), data.i32(win[1]), data.i32(win[0] + w - 1), data.i32(win[1] + h - 1);
        disp.i32(0), disp.i32(0), disp.i32(win[2] - 1), disp.i32(win[3] - 1);
        hdr.attr("dataWindow", "box2i", data);
        hdr.attr("displayWindow", "box2i", disp);
    }
    {
        Bytes v;
        v.u8(0);  // INCREASING_Y
        hdr.attr("lineOrder", "lineOrder", v);
    }
    {
        Bytes v;
        v.f32(1.f);
        hdr.attr("pixelAspectRatio", "float", v);
    }
    {
        Bytes v;
        v.f32(0.f), v.f32(0.f);
        hdr.attr("screenWindowCenter", "v2f", v);
    }
    {
        Bytes v;
        v.f32(1.f);
        hdr.attr("screenWindowWidth", "float", v);
    }
    hdr.u8(0);  // end of header
    const size_t lineBytes = (size_t)3 * w * bpc;
    const uint64_t tableEnd = hdr.b.size() + (uint64_t)8 * h;
    for (int y = 0; y < h; ++y) hdr.u64(tableEnd + (uint64_t)y * (8 + lineBytes));
    File fp(path, "wb");
    std::fwrite(hdr.b.data(), 1, hdr.b.size(), fp.f);
    std::vector<uint8_t> line(8 + lineBytes);
    for (int y = 0; y < h; ++y) {
        int32_t yy = win[1] + y, sz = (int32_t)lineBytes;
        std::memcpy(&line[0], &yy, 4);
        std::memcpy(&line[4], &sz, 4);
        uint8_t *p = &line[8];
        for (int c : {2, 1, 0})  // B, G, R planes of the scanline
            for (int x = 0; x < w; ++x) {
                const float v = rgb[((size_t)y * w + x) * 3 + c];
                if (half) {
                    const uint16_t hv = FloatToHalf(v);
                    std::memcpy(p, &hv, 2);
                } else {
                    std::memcpy(p, &v, 4);
                }
                p += bpc;
            }
        std::fwrite(line.data(), 1, line.size(), fp.f);
    }
}

static Image ReadEXR(const std::string &path) {
    File fp(path, "rb");
    std::vector<uint8_t> d;
    {
        uint8_t buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), fp.f)) > 0) d.insert(d.end(), buf, buf + n);
    }
    size_t pos = 0;
    auto need = [&](size_t n) {
        if (pos + n > d.size()) throw std::runtime_error(path + ": truncated EXR file");
    };
    auto rd32 = [&]() {
        need(4);
        uint32_t v;
        std::memcpy(&v, &d[pos], 4);
        pos += 4;
        return v;
    };
    auto rdstr = [&]() {
        std::string s;
        while (true) {
            need(1);
            char c = (char)d[pos++];
            if (!c) break;
            s.push_back(c);
        }
        return s;
    };
    if (rd32() != 20000630u) throw std::runtime_error(path + ": not an OpenEXR file");
    if ((rd32() & 0xffu) != 2u) throw std::runtime_error(path + ": unsupported EXR version");
    struct Ch {
        std::string name;
        int type;
    };
    std::vector<Ch> chans;
    int compression = -1, x0 = 0, y0 = 0, x1 = -1, y1 = -1;
    while (true) {
        std::string name = rdstr();
        if (name.empty()) break;
        std::string type = rdstr();
        const uint32_t size = rd32();
        need(size);
        const size_t end = pos + size;
        if (name == "channels") {
            while (pos < end && d[pos] != 0) {
                std::string cn = rdstr();
                int32_t t;
                std::memcpy(&t, &d[pos], 4);
                chans.push_back({cn, t});
                pos += 16;
            }
        } else if (name == "compression") {
            compression = d[pos];
        } else if (name == "dataWindow") {
            std::memcpy(&x0, &d[pos], 4);
            std::memcpy(&y0, &d[pos + 4], 4);
            std::memcpy(&x1, &d[pos + 8], 4);
            std::memcpy(&y1, &d[pos + 12], 4);
        }
        pos = end;
    }
    if (compression != 0) throw std::runtime_error(path + ": only uncompressed EXR files are supported");
    Image im;
    im.width = x1 - x0 + 1;
    im.height = y1 - y0 + 1;
    if (im.width <= 0 || im.height <= 0) throw std::runtime_error(path + ": bad EXR data window");
    int idx[3] = {-1, -1, -1};
    size_t lineBytes = 0;
    std::vector<size_t> chOff;
    for (size_t i = 0; i < chans.size(); ++i) {
        if (chans[i].type != 1 && chans[i].type != 2) throw std::runtime_error(path + ": unsupported EXR pixel type");
        chOff.push_back(lineBytes);
        lineBytes += (size_t)im.width * (chans[i].type == 1 ? 2 : 4);
        if (chans[i].name == "R") idx[0] = (int)i;
        if (chans[i].name == "G") idx[1] = (int)i;
        if (chans[i].name == "B") idx[2] = (int)i;
    }
    if (idx[0] < 0 || idx[1] < 0 || idx[2] < 0) throw std::runtime_error(path + ": EXR file has no R, G, B channels");
    pos += (size_t)8 * im.height;  // offset table (lines are read in order)
    im.rgb.assign((size_t)3 * im.width * im.height, 0.f);
    for (int l = 0; l < im.height; ++l) {
        need(8);
        int32_t y, sz;
        std::memcpy(&y, &d[pos], 4);
        std::memcpy(&sz, &d[pos + 4], 4);
        pos += 8;
        need((size_t)sz);
        if ((size_t)sz != lineBytes || y - y0 < 0 || y - y0 >= im.height)
            throw std::runtime_error(path + ": bad EXR scanline");
        for (int c = 0; c < 3; ++c) {
            const Ch &ch = chans[idx[c]];
            const uint8_t *p = &d[pos + chOff[idx[c]]];
            for (int x = 0; x < im.width; ++x) {
                float v;
                if (ch.type == 1) {
                    uint16_t hv;
                    std::memcpy(&hv, p + 2 * x, 2);
                    v = HalfToFloat(hv);
                } else {
                    std::memcpy(&v, p + 4 * x, 4);
                }
                im.rgb[((size_t)(y - y0) * im.width + x) * 3 + c] = v;
            }
        }
        pos += sz;
    }
    return im;
}

// ---------------------------------------------------------------- PNG
static uint32_t Crc32(const uint8_t *p, size_t n, uint32_t crc = 0) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xffu] ^ (crc >> 8);
    return ~crc;
}

// sRGB encoding of a linear value, 8 bits (ColorEncoding sRGB, util/color.h LinearToSRGB)
static uint8_t LinearToSRGB8(float v) {
    if (!(v > 0)) return 0;
    float s = v <= 0.0031308f ? 12.92f * v : 1.055f * std::pow(v, 1.f / 2.4f) - 0.055f;
    s = std::fmin(std::fmax(s, 0.f), 1.f);
    return (uint8_t)std::lround(s * 255.f);
}

static void WritePNG(const std::string &path, const float *rgb, int w, int h) {
    std::vector<uint8_t> raw;
    raw.reserve((size_t)h * (1 + 3 * (size_t)w));
    for (int y = 0; y < h; ++y) {
        raw.push_back(0);  // filter: none
        for (int x = 0; x < w * 3; ++x) raw.push_back(LinearToSRGB8(rgb[(size_t)y * w * 3 + x]));
    }
    // zlib stream of stored deflate blocks
    std::vector<uint8_t> z{0x78, 0x01};
    uint32_t a = 1, b = 0;
    for (uint8_t v : raw) {
        a = (a + v) % 65521u;
        b = (b + a) % 65521u;
    }
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
        const size_t n = std::min<size_t>(65535, raw.size() - off);
        z.push_back(off + n >= raw.size() ? 1 : 0);
        z.push_back((uint8_t)n), z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n), z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + off, raw.begin() + off + n);
        if (raw.empty()) break;
    }
    const uint32_t adler = (b << 16) | a;
    for (int i = 3; i >= 0; --i) z.push_back((uint8_t)(adler >> (8 * i)));
    File fp(path, "wb");
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::fwrite(sig, 1, 8, fp.f);
    auto chunk = [&](const char *type, const std::vector<uint8_t> &data) {
        uint8_t len[4] = {(uint8_t)(data.size() >> 24), (uint8_t)(data.size() >> 16), (uint8_t)(data.size() >> 8),
                          (uint8_t)data.size()};
        std::fwrite(len, 1, 4, fp.f);
        std::vector<uint8_t> td(type, type + 4);
        td.insert(td.end(), data.begin(), data.end());
        std::fwrite(td.data(), 1, td.size(), fp.f);
        const uint32_t crc = Crc32(td.data(), td.size());
        uint8_t c[4] = {(uint8_t)(crc >> 24), (uint8_t)(crc >> 16), (uint8_t)(crc >> 8), (uint8_t)crc};
        std::fwrite(c, 1, 4, fp.f);
    };
    std::vector<uint8_t> ihdr = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8), (uint8_t)w,
                                 (uint8_t)(h >> 24), (uint8_t)(h >> 16), (uint8_t)(h >> 8), (uint8_t)h,
                                 8, 2, 0, 0, 0};  // 8-bit RGB
    chunk("IHDR", ihdr);
    chunk("sRGB", {0});
    chunk("IDAT", z);
    chunk("IEND", {});
}

// ---------------------------------------------------------------- public
void WriteImage(const std::string &path, const float *rgb, int w, int h, bool exrHalf, const int *window) {
    const std::string e = Ext(path);
    const int full[4] = {0, 0, w, h};
    if (e == "pfm") WritePFM(path, rgb, w, h);
    else if (e == "exr") WriteEXR(path, rgb, w, h, exrHalf, window ? window : full);
    else if (e == "png") WritePNG(path, rgb, w, h);
    else throw std::runtime_error(path + ": unsupported image format \"" + e + "\" (pfm, exr, png)");
}

Image ReadImage(const std::string &path) {
    const std::string e = Ext(path);
    if (e == "pfm") return ReadPFM(path);
    if (e == "exr") return ReadEXR(path);
    throw std::runtime_error(path + ": unsupported image format \"" + e + "\" for reading (pfm, exr)");
}

std::array<double, 3> ImageError(const float *img, const float *ref, int w, int h, ErrorMetric metric) {
    double sum[3] = {0, 0, 0};
    for (size_t i = 0; i < (size_t)w * h; ++i)
        for (int c = 0; c < 3; ++c) {
            const double v = img[3 * i + c], r = ref[3 * i + c];
            double e;
            if (metric == ErrorMetric::MAE) e = v - r;  // pbrt's MAE: the signed difference
            else if (metric == ErrorMetric::MSE) e = (v - r) * (v - r);
            else e = (v - r) * (v - r) / ((r + 0.01) * (r + 0.01));
            if (std::isinf(e)) continue;
            sum[c] += e;
        }
    const float denom = float(w) * float(h);
    return {sum[0] / denom, sum[1] / denom, sum[2] / denom};
}

}  // namespace pbrt_amd
