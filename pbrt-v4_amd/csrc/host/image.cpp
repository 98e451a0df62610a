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
#include <algorithm>
#include "image.h"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include <zlib.h>

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
static void WriteEXR(const std::string &path, const float *rgb, int w, int h, bool half, const int win[4],
                     const float *chroma8) {
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
    if (chroma8) {
        Bytes v;
        for (int i = 0; i < 8; ++i) v.f32(chroma8[i]);
        hdr.attr("chromaticities", "chromaticities", v);
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

// OpenEXR's RLE / ZIP(S) decoders: byte predictor, then the two half-streams interleaved
// (the file format's documented reorder of a block's bytes)
static void ExrUnpredict(std::vector<uint8_t> &t, std::vector<uint8_t> *out) {
    for (size_t i = 1; i < t.size(); ++i) t[i] = (uint8_t)(int(t[i - 1]) + int(t[i]) - 128);
    out->resize(t.size());
    const size_t half = (t.size() + 1) / 2;
    for (size_t i = 0, a = 0, b = half; i < t.size(); ++i) (*out)[i] = (i & 1) ? t[b++] : t[a++];
}
static bool ExrRle(const uint8_t *in, size_t n, size_t outSize, std::vector<uint8_t> *t) {
    t->clear();
    size_t i = 0;
    while (i < n) {
        const int c = (int8_t)in[i++];
        if (c < 0) {
            if (i + (size_t)-c > n) return false;
            t->insert(t->end(), in + i, in + i + (size_t)-c);
            i += (size_t)-c;
        } else {
            if (i >= n) return false;
            t->insert(t->end(), (size_t)c + 1, in[i++]);
        }
        if (t->size() > outSize) return false;
    }
    return t->size() == outSize;
}

// Scanline OpenEXR with NONE / RLE / ZIPS / ZIP compression and HALF or FLOAT channels (what
// Image::Read, util/image.cpp:1055-1180, takes through the OpenEXR library; PIZ and the lossy
// codecs, tiled and deep files are refused).  chromaticities must be sRGB's
// (RGBColorSpace::Lookup's 1e-3 relative match).
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
    const uint32_t version = rd32();
    if ((version & 0xffu) != 2u) throw std::runtime_error(path + ": unsupported EXR version");
    if (version & 0x1a00u) throw std::runtime_error(path + ": tiled, multi-part and deep EXR files are not supported");
    struct Ch {
        std::string name;
        int type;
    };
    std::vector<Ch> chans;
    int compression = -1, x0 = 0, y0 = 0, x1 = -1, y1 = -1;
    float chroma[8];
    bool hasChroma = false, haveWindow = false;
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
                int32_t t, xs, ys;
                need(16);
                std::memcpy(&t, &d[pos], 4);
                std::memcpy(&xs, &d[pos + 8], 4);
                std::memcpy(&ys, &d[pos + 12], 4);
                if (xs != 1 || ys != 1) throw std::runtime_error(path + ": subsampled EXR channels are not supported");
                chans.push_back({cn, t});
                pos += 16;
            }
        } else if (name == "compression") {
            compression = d[pos];
        } else if (name == "dataWindow") {
            if (size < 16) throw std::runtime_error(path + ": bad EXR data window");
            haveWindow = true;
            std::memcpy(&x0, &d[pos], 4);
            std::memcpy(&y0, &d[pos + 4], 4);
            std::memcpy(&x1, &d[pos + 8], 4);
            std::memcpy(&y1, &d[pos + 12], 4);
        } else if (name == "chromaticities" && size == 32) {
            std::memcpy(chroma, &d[pos], 32);
            hasChroma = true;
        }
        pos = end;
    }
    static const char *kCodec[] = {"NONE", "RLE", "ZIPS", "ZIP", "PIZ", "PXR24", "B44", "B44A", "DWAA", "DWAB"};
    if (compression < 0 || compression > 3)
        throw std::runtime_error(path + ": EXR compression " +
                                 (compression >= 0 && compression < 10 ? kCodec[compression] : std::string("?")) +
                                 " is not supported (NONE, RLE, ZIPS and ZIP are)");
    if (hasChroma) {
        // sRGB primaries and the D65 white point
        const float srgb[8] = {.64f, .33f, .3f, .6f, .15f, .06f, .3127f, .329f};
        for (int i = 0; i < 8; ++i)
            if (!(chroma[i] == srgb[i] || std::abs((chroma[i] - srgb[i]) / srgb[i]) < 1e-3f))
                throw std::runtime_error(path + ": EXR chromaticities are not sRGB's; only sRGB images are supported");
    }
    // dataWindow must exist and span a sane, non-empty box (64-bit extents: no int overflow)
    const int64_t wExt = (int64_t)x1 - x0 + 1, hExt = (int64_t)y1 - y0 + 1;
    if (!haveWindow || wExt <= 0 || hExt <= 0 || wExt > 65536 || hExt > 65536 || wExt * hExt > (int64_t(1) << 28))
        throw std::runtime_error(path + ": bad EXR data window");
    if (chans.empty()) throw std::runtime_error(path + ": EXR file without channels");
    Image im;
    im.width = (int)wExt;
    im.height = (int)hExt;
    int idx[3] = {-1, -1, -1};
    size_t lineBytes = 0;
    std::vector<size_t> chOff;
    for (size_t i = 0; i < chans.size(); ++i) {
        if (chans[i].type != 1 && chans[i].type != 2) throw std::runtime_error(path + ": unsupported EXR pixel type");
        if (chans[i].type != chans[0].type)
            throw std::runtime_error(path + ": EXR images with multiple channel types are not supported");
        chOff.push_back(lineBytes);
        lineBytes += (size_t)im.width * (chans[i].type == 1 ? 2 : 4);
        if (chans[i].name == "R") idx[0] = (int)i;
        if (chans[i].name == "G") idx[1] = (int)i;
        if (chans[i].name == "B") idx[2] = (int)i;
    }
    if (idx[0] < 0 || idx[1] < 0 || idx[2] < 0) throw std::runtime_error(path + ": EXR file has no R, G, B channels");
    const int linesPerBlock = compression == 3 ? 16 : 1;
    const int nBlocks = (im.height + linesPerBlock - 1) / linesPerBlock;
    std::vector<uint64_t> table(nBlocks);
    need((size_t)8 * nBlocks);
    std::memcpy(table.data(), &d[pos], (size_t)8 * nBlocks);
    im.rgb.assign((size_t)3 * im.width * im.height, 0.f);
    std::vector<uint8_t> tmp, raw;
    for (int blk = 0; blk < nBlocks; ++blk) {
        pos = (size_t)table[blk];
        need(8);
        int32_t y, sz;
        std::memcpy(&y, &d[pos], 4);
        std::memcpy(&sz, &d[pos + 4], 4);
        pos += 8;
        if (sz < 0) throw std::runtime_error(path + ": bad EXR block");
        need((size_t)sz);
        const int ly = y - y0;
        const int nl = std::min(linesPerBlock, im.height - ly);
        if (ly < 0 || ly >= im.height || ly % linesPerBlock) throw std::runtime_error(path + ": bad EXR block");
        const size_t rawSize = lineBytes * nl;
        const uint8_t *src = &d[pos];
        if ((size_t)sz == rawSize) {
            raw.assign(src, src + rawSize);  // stored: the codec did not shrink it
        } else if (compression == 1) {
            if (!ExrRle(src, (size_t)sz, rawSize, &tmp)) throw std::runtime_error(path + ": corrupt RLE block");
            ExrUnpredict(tmp, &raw);
        } else if (compression == 2 || compression == 3) {
            tmp.resize(rawSize);
            uLongf outLen = (uLongf)rawSize;
            if (uncompress(tmp.data(), &outLen, src, (uLong)sz) != Z_OK || outLen != rawSize)
                throw std::runtime_error(path + ": corrupt ZIP block");
            ExrUnpredict(tmp, &raw);
        } else {
            throw std::runtime_error(path + ": bad EXR scanline");
        }
        for (int l = 0; l < nl; ++l)
            for (int c = 0; c < 3; ++c) {
                const Ch &ch = chans[idx[c]];
                const uint8_t *p = raw.data() + l * lineBytes + chOff[idx[c]];
                for (int x = 0; x < im.width; ++x) {
                    float v;
                    if (ch.type == 1) {
                        uint16_t hv;
                        std::memcpy(&hv, p + 2 * x, 2);
                        v = HalfToFloat(hv);
                    } else {
                        std::memcpy(&v, p + 4 * x, 4);
                    }
                    im.rgb[((size_t)(ly + l) * im.width + x) * 3 + c] = v;
                }
            }
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
void WriteImage(const std::string &path, const float *rgb, int w, int h, bool exrHalf, const int *window,
                const float *chroma8) {
    const std::string e = Ext(path);
    const int full[4] = {0, 0, w, h};
    if (e == "pfm") WritePFM(path, rgb, w, h);
    else if (e == "exr") WriteEXR(path, rgb, w, h, exrHalf, window ? window : full, chroma8);
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
    if (metric == ErrorMetric::FLIP) {
        // imgtool.cpp:1248-1255: every channel reports the map's mean
        const std::vector<float> m = FlipErrorMap(img, ref, w, h);
        float s = 0;
        for (float v : m) s += v;
        const double e = s / (w * h);
        return {e, e, e};
    }
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

// ---------------------------------------------------------------- FLIP
// FLIP (Andersson, Nilsson, Akenine-Moller, Oskarsson, Astrom, Fairchild, "FLIP: A Difference
// Evaluator for Alternating Images", HPG 2020), the LDR evaluator as pbrt's imgtool runs it
// (cmd/imgtool.cpp:1224-1255: inputs clamped to [0, 1] and read as sRGB-encoded, FLIP's default
// viewing conditions -- 0.7 m from a 0.7 m wide 3840-pixel monitor).  Colour pipeline: YCxCz
// opponent space, contrast-sensitivity filters (sums of Gaussians per channel), back to linear
// RGB clamped to the gamut, CIELab with the Hunt adjustment, HyAB distance redistributed into
// [0, 1].  Feature pipeline: first / second Gaussian-derivative edge and point detectors on the
// achromatic channel.  Per pixel: colour^(1 - feature).  Float arithmetic throughout, as the
// published evaluator (pinned by tests/golden "flip", ComputeFLIPError of src/ext/flip).
namespace {
struct C3 {
    float a = 0, b = 0, c = 0;
};
constexpr float kWhiteX = 0.950428545377181f, kWhiteY = 1.0f, kWhiteZ = 1.088900370798128f;
C3 SrgbToXyz(C3 v) {
    auto lin = [](float x) { return x <= 0.04045f ? x / 12.92f : powf((x + 0.055f) / 1.055f, 2.4f); };
    v = {lin(v.a), lin(v.b), lin(v.c)};
    return {(10135552.0f / 24577794.0f) * v.a + (8788810.0f / 24577794.0f) * v.b + (4435075.0f / 24577794.0f) * v.c,
            (2613072.0f / 12288897.0f) * v.a + (8788810.0f / 12288897.0f) * v.b + (887015.0f / 12288897.0f) * v.c,
            (1425312.0f / 73733382.0f) * v.a + (8788810.0f / 73733382.0f) * v.b + (70074185.0f / 73733382.0f) * v.c};
}
C3 LinearToXyz(C3 v) {
    return {(10135552.0f / 24577794.0f) * v.a + (8788810.0f / 24577794.0f) * v.b + (4435075.0f / 24577794.0f) * v.c,
            (2613072.0f / 12288897.0f) * v.a + (8788810.0f / 12288897.0f) * v.b + (887015.0f / 12288897.0f) * v.c,
            (1425312.0f / 73733382.0f) * v.a + (8788810.0f / 73733382.0f) * v.b + (70074185.0f / 73733382.0f) * v.c};
}
C3 XyzToLinear(C3 v) {
    return {3.241003232976358f * v.a + -1.537398969488785f * v.b + -0.498615881996363f * v.c,
            -0.969224252202516f * v.a + 1.875929983695176f * v.b + 0.041554226340085f * v.c,
            0.055639419851975f * v.a + -0.204011206123910f * v.b + 1.057148977187533f * v.c};
}
C3 XyzToYCxCz(C3 v) {
    const float x = v.a / kWhiteX, y = v.b / kWhiteY, z = v.c / kWhiteZ;
    return {116.0f * y - 16.0f, 500.0f * (x - y), 200.0f * (y - z)};
}
C3 YCxCzToXyz(C3 v) {
    const float yy = (v.a + 16.0f) / 116.0f, cx = v.b / 500.0f, cz = v.c / 200.0f;
    return {(yy + cx) * kWhiteX, yy * kWhiteY, (yy - cz) * kWhiteZ};
}
C3 XyzToLab(C3 v) {
    auto f = [](float t) { return t > 0.008856 ? powf(t, 1.0f / 3.0f) : 7.787f * t + 16.0f / 116.0f; };
    const float x = f(fabsf(v.a) / kWhiteX), y = f(fabsf(v.b) / kWhiteY), z = f(fabsf(v.c) / kWhiteZ);
    return {116.0f * y - 16.0f, 500.0f * (x - y), 200.0f * (y - z)};
}
float HyABDist(C3 p, C3 q) { return fabsf(p.a - q.a) + sqrtf((p.b - q.b) * (p.b - q.b) + (p.c - q.c) * (p.c - q.c)); }
C3 HuntAdjust(C3 lab) { return {lab.a, 0.01f * lab.a * lab.b, 0.01f * lab.a * lab.c}; }
// 2D convolution with clamp-to-edge borders; kernel [k][k] (odd), three channels
std::vector<C3> Convolve(const std::vector<C3> &img, int w, int h, const std::vector<C3> &ker, int k) {
    std::vector<C3> out(img.size());
    const int r = k / 2;
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) {
            C3 acc;
            for (int dy = -r; dy <= r; ++dy) {
                const int yy = std::min(std::max(0, y + dy), h - 1);
                for (int dx = -r; dx <= r; ++dx) {
                    const int xx = std::min(std::max(0, x + dx), w - 1);
                    const C3 &kv = ker[(dy + r) * k + dx + r], &v = img[yy * w + xx];
                    acc = {acc.a + kv.a * v.a, acc.b + kv.b * v.b, acc.c + kv.c * v.c};
                }
            }
            out[y * w + x] = acc;
        }
    return out;
}
}  // namespace

std::vector<float> FlipErrorMap(const float *test, const float *ref, int w, int h) {
    const float pi = 3.14159265358979323846f;
    const float ppd = 0.7f * (3840.0f / 0.7f) * (pi / 180.0f);
    const size_t n = (size_t)w * h;
    std::vector<C3> T(n), R(n);
    for (size_t i = 0; i < n; ++i) {
        auto cl = [](float v) { return std::min(std::max(v, 0.f), 1.f); };
        T[i] = XyzToYCxCz(SrgbToXyz({cl(test[3 * i]), cl(test[3 * i + 1]), cl(test[3 * i + 2])}));
        R[i] = XyzToYCxCz(SrgbToXyz({cl(ref[3 * i]), cl(ref[3 * i + 1]), cl(ref[3 * i + 2])}));
    }
    // contrast sensitivity: per channel a1 sqrt(pi/b1) exp(-pi^2 r^2 / b1) + a2 sqrt(pi/b2) exp(-pi^2 r^2 / b2)
    const C3 A1{1.0f, 1.0f, 34.1f}, B1{0.0047f, 0.0053f, 0.04f}, A2{0.0f, 0.0f, 13.5f}, B2{1.0e-5f, 1.0e-5f, 0.025f};
    const float pi2 = float(M_PI * M_PI);
    const float bmax = std::max({B1.a, B1.b, B1.c, B2.a, B2.b, B2.c});
    const int rad = int(std::ceil(3.0f * sqrtf(bmax / (2.0f * pi2)) * ppd)), kw = 2 * rad + 1;
    std::vector<C3> csf(kw * kw);
    C3 sum;
    auto gs = [&](float r2, float a1, float b1, float a2, float b2) {
        return a1 * sqrtf(pi / b1) * expf(-pi2 * r2 / b1) + a2 * sqrtf(pi / b2) * expf(-pi2 * r2 / b2);
    };
    for (int y = 0; y < kw; ++y)
        for (int x = 0; x < kw; ++x) {
            const float fx = (x - rad) * (1.0f / ppd), fy = (y - rad) * (1.0f / ppd), r2 = fx * fx + fy * fy;
            const C3 v{gs(r2, A1.a, B1.a, A2.a, B2.a), gs(r2, A1.b, B1.b, A2.b, B2.b), gs(r2, A1.c, B1.c, A2.c, B2.c)};
            csf[y * kw + x] = v;
            sum = {sum.a + v.a, sum.b + v.b, sum.c + v.c};
        }
    for (C3 &v : csf) v = {v.a / sum.a, v.b / sum.b, v.c / sum.c};
    auto toLab = [&](const std::vector<C3> &img) {
        std::vector<C3> f = Convolve(img, w, h, csf, kw);
        for (C3 &p : f) {
            C3 l = XyzToLinear(YCxCzToXyz(p));
            auto g = [](float v) { return std::max(std::min(v, 1.0f), 0.0f); };
            p = HuntAdjust(XyzToLab(LinearToXyz({g(l.a), g(l.b), g(l.c)})));
        }
        return f;
    };
    const std::vector<C3> LT = toLab(T), LR = toLab(R);
    const float qc = 0.7f, pc = 0.4f, pt = 0.95f;
    const float cmax = powf(HyABDist(HuntAdjust(XyzToLab(LinearToXyz({0, 1, 0}))), HuntAdjust(XyzToLab(LinearToXyz({0, 0, 1})))), qc);
    // feature detectors: Gaussian (std 0.5 w ppd, w = 0.082 deg) first derivative (edges) and
    // second derivative (points), positive and negative weights each normalized to sum 1
    const float sd = 0.5f * 0.082f * ppd;
    const int fr = int(std::ceil(3.0f * sd)), fw = 2 * fr + 1;
    auto detector = [&](bool point) {
        std::vector<C3> k(fw * fw);
        float px = 0, nx = 0, py = 0, ny = 0;
        for (int y = 0; y < fw; ++y)
            for (int x = 0; x < fw; ++x) {
                const float xx = float(x - fr), yy = float(y - fr);
                const float G = expf(-(xx * xx + yy * yy) / (2.0f * sd * sd));
                const float wx = point ? (xx * xx / (sd * sd) - 1.0f) * G : -xx * G;
                const float wy = point ? (yy * yy / (sd * sd) - 1.0f) * G : -yy * G;
                k[y * fw + x] = {wx, wy, 0.f};
                (wx > 0 ? px : nx) += wx > 0 ? wx : -wx;
                (wy > 0 ? py : ny) += wy > 0 ? wy : -wy;
            }
        for (C3 &v : k) v = {v.a / (v.a > 0 ? px : nx), v.b / (v.b > 0 ? py : ny), 0.f};
        return k;
    };
    const std::vector<C3> edgeK = detector(false), pointK = detector(true);
    auto gray = [&](const std::vector<C3> &img) {
        std::vector<C3> g(img.size());
        for (size_t i = 0; i < img.size(); ++i) {
            const float c = (img[i].a + 16.0f) / 116.0f;
            g[i] = {c, c, 0.f};
        }
        return g;
    };
    const std::vector<C3> gT = gray(T), gR = gray(R);
    const std::vector<C3> eT = Convolve(gT, w, h, edgeK, fw), eR = Convolve(gR, w, h, edgeK, fw);
    const std::vector<C3> pT = Convolve(gT, w, h, pointK, fw), pR = Convolve(gR, w, h, pointK, fw);
    std::vector<float> out(n);
    for (size_t i = 0; i < n; ++i) {
        float e = powf(HyABDist(LR[i], LT[i]), qc);
        e = e < pc * cmax ? e * (pt / (pc * cmax)) : pt + ((e - pc * cmax) / (cmax - pc * cmax)) * (1.0f - pt);
        auto mag = [](C3 v) { return sqrtf(v.a * v.a + v.b * v.b); };
        const float de = std::abs(mag(eR[i]) - mag(eT[i])), dp = std::abs(mag(pR[i]) - mag(pT[i]));
        const float feat = std::pow((1.0f / sqrtf(2.0f)) * std::max(de, dp), 0.5f);
        out[i] = std::pow(e, 1.0f - feat);
    }
    return out;
}

}  // namespace pbrt_amd
