// PLY mesh reader for Shape "plymesh": the subset TriQuadMesh::ReadPLY (util/mesh.cpp:322-420)
// extracts through rply -- vertex x/y/z, optional nx/ny/nz and u/v (or s/t, texture_u/v,
// texture_s/t), face vertex_indices (triangles and quads; other polygon sizes are skipped
// with a warning, as rply_face_callback does, mesh.cpp:274-312) and optional face_indices.
// ascii, binary_little_endian and binary_big_endian files; every scalar is read at its
// declared type and converted through double, as rply's ply_get_argument_value does.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "ply.h"

namespace pbrt_amd {

namespace {

enum class PType { I8, U8, I16, U16, I32, U32, F32, F64, Invalid };

PType ParseType(const std::string &t) {
    if (t == "char" || t == "int8") return PType::I8;
    if (t == "uchar" || t == "uint8") return PType::U8;
    if (t == "short" || t == "int16") return PType::I16;
    if (t == "ushort" || t == "uint16") return PType::U16;
    if (t == "int" || t == "int32") return PType::I32;
    if (t == "uint" || t == "uint32") return PType::U32;
    if (t == "float" || t == "float32") return PType::F32;
    if (t == "double" || t == "float64") return PType::F64;
    return PType::Invalid;
}
int TypeSize(PType t) {
    switch (t) {
    case PType::I8: case PType::U8: return 1;
    case PType::I16: case PType::U16: return 2;
    case PType::I32: case PType::U32: case PType::F32: return 4;
    case PType::F64: return 8;
    default: return 0;
    }
}

struct Property {
    std::string name;
    bool isList = false;
    PType type = PType::Invalid, countType = PType::Invalid;
};
struct Element {
    std::string name;
    size_t count = 0;
    std::vector<Property> props;
};

struct Reader {
    std::string file;
    std::vector<char> data;
    size_t pos = 0;
    int format = 0;  // 0 ascii, 1 little endian, 2 big endian

    [[noreturn]] void Fail(const std::string &m) const { throw Error(file + ": " + m); }

    double Binary(PType t) {
        const int n = TypeSize(t);
        if (pos + n > data.size()) Fail("unexpected end of PLY data");
        unsigned char b[8];
        memcpy(b, &data[pos], n);
        pos += n;
        if (format == 2) std::reverse(b, b + n);  // this host is little endian
        switch (t) {
        case PType::I8: { int8_t v; memcpy(&v, b, 1); return v; }
        case PType::U8: { uint8_t v; memcpy(&v, b, 1); return v; }
        case PType::I16: { int16_t v; memcpy(&v, b, 2); return v; }
        case PType::U16: { uint16_t v; memcpy(&v, b, 2); return v; }
        case PType::I32: { int32_t v; memcpy(&v, b, 4); return v; }
        case PType::U32: { uint32_t v; memcpy(&v, b, 4); return v; }
        case PType::F32: { float v; memcpy(&v, b, 4); return v; }
        case PType::F64: { double v; memcpy(&v, b, 8); return v; }
        default: Fail("bad property type");
        }
    }
    double Ascii() {
        while (pos < data.size() && isspace((unsigned char)data[pos])) ++pos;
        if (pos >= data.size()) Fail("unexpected end of PLY data");
        const char *s = &data[pos];
        char *end = nullptr;
        double v = strtod(s, &end);
        if (end == s) Fail("malformed number in PLY data");
        pos += end - s;
        return v;
    }
    double Value(PType t) { return format == 0 ? Ascii() : Binary(t); }
};

}  // namespace

PlyMesh ReadPly(const std::string &filename) {
    Reader r;
    r.file = filename;
    {
        std::ifstream in(filename, std::ios::binary);
        if (!in) throw Error("Couldn't open PLY file \"" + filename + "\"");
        r.data.assign(std::istreambuf_iterator<char>(in), std::istreambuf_iterator<char>());
    }
    // ---- header
    std::vector<Element> elements;
    auto line = [&]() {
        size_t e = r.pos;
        while (e < r.data.size() && r.data[e] != '\n') ++e;
        if (e >= r.data.size()) r.Fail("unterminated PLY header");
        std::string l(&r.data[r.pos], e - r.pos);
        r.pos = e + 1;
        if (!l.empty() && l.back() == '\r') l.pop_back();
        return l;
    };
    if (line() != "ply") r.Fail("not a PLY file");
    bool sawFormat = false;
    while (true) {
        std::string l = line();
        std::istringstream ls(l);
        std::string kw;
        ls >> kw;
        if (kw == "end_header") break;
        if (kw == "comment" || kw == "obj_info" || kw.empty()) continue;
        if (kw == "format") {
            std::string f, ver;
            ls >> f >> ver;
            if (f == "ascii") r.format = 0;
            else if (f == "binary_little_endian") r.format = 1;
            else if (f == "binary_big_endian") r.format = 2;
            else r.Fail("unknown PLY format \"" + f + "\"");
            sawFormat = true;
        } else if (kw == "element") {
            Element e;
            ls >> e.name >> e.count;
            elements.push_back(e);
        } else if (kw == "property") {
            if (elements.empty()) r.Fail("property before element");
            Property p;
            std::string t;
            ls >> t;
            if (t == "list") {
                std::string ct, it;
                ls >> ct >> it >> p.name;
                p.isList = true;
                p.countType = ParseType(ct);
                p.type = ParseType(it);
                if (p.countType == PType::Invalid || p.type == PType::Invalid) r.Fail("bad list property types");
            } else {
                p.type = ParseType(t);
                ls >> p.name;
                if (p.type == PType::Invalid) r.Fail("bad property type \"" + t + "\"");
            }
            elements.back().props.push_back(p);
        } else {
            r.Fail("unknown PLY header keyword \"" + kw + "\"");
        }
    }
    if (!sawFormat) r.Fail("PLY header has no format line");

    PlyMesh m;
    size_t vertexCount = 0, faceCount = 0;
    for (auto &e : elements) {
        if (e.name == "vertex") vertexCount = e.count;
        if (e.name == "face") faceCount = e.count;
    }
    if (vertexCount == 0 || faceCount == 0) r.Fail("PLY file is invalid! No face/vertex elements found!");

    // ---- body
    for (const Element &e : elements) {
        if (e.name == "vertex") {
            auto find = [&](const char *n) {
                for (size_t i = 0; i < e.props.size(); ++i)
                    if (e.props[i].name == n && !e.props[i].isList) return (int)i;
                return -1;
            };
            int px = find("x"), py = find("y"), pz = find("z");
            if (px < 0 || py < 0 || pz < 0) r.Fail("Vertex coordinate property not found!");
            int nx = find("nx"), ny = find("ny"), nz = find("nz");
            const bool hasN = nx >= 0 && ny >= 0 && nz >= 0;
            int tu = -1, tv = -1;
            const char *uvNames[4][2] = {{"u", "v"}, {"s", "t"}, {"texture_u", "texture_v"}, {"texture_s", "texture_t"}};
            for (auto &pr : uvNames)
                if (tu < 0 && find(pr[0]) >= 0 && find(pr[1]) >= 0) {
                    tu = find(pr[0]);
                    tv = find(pr[1]);
                }
            m.p.resize(e.count);
            if (hasN) m.n.resize(e.count);
            if (tu >= 0) m.uv.resize(e.count);
            std::vector<double> vals(e.props.size());
            for (size_t i = 0; i < e.count; ++i) {
                for (size_t k = 0; k < e.props.size(); ++k) {
                    const Property &p = e.props[k];
                    if (p.isList) {
                        size_t c = (size_t)r.Value(p.countType);
                        for (size_t j = 0; j < c; ++j) r.Value(p.type);
                        vals[k] = 0;
                    } else {
                        vals[k] = r.Value(p.type);
                    }
                }
                m.p[i] = V3((float)vals[px], (float)vals[py], (float)vals[pz]);
                if (hasN) m.n[i] = V3((float)vals[nx], (float)vals[ny], (float)vals[nz]);
                if (tu >= 0) m.uv[i] = {(float)vals[tu], (float)vals[tv]};
            }
        } else if (e.name == "face") {
            int vi = -1, fi = -1;
            for (size_t k = 0; k < e.props.size(); ++k) {
                if (e.props[k].name == "vertex_indices" && e.props[k].isList) vi = (int)k;
                if (e.props[k].name == "face_indices" && !e.props[k].isList) fi = (int)k;
            }
            if (vi < 0) r.Fail("vertex indices not found in PLY file");
            m.triIndices.reserve(e.count * 3);
            for (size_t i = 0; i < e.count; ++i) {
                for (size_t k = 0; k < e.props.size(); ++k) {
                    const Property &p = e.props[k];
                    if (!p.isList) {
                        double v = r.Value(p.type);
                        if ((int)k == fi) m.faceIndices.push_back((int)v);
                        continue;
                    }
                    size_t c = (size_t)r.Value(p.countType);
                    int f[4] = {0, 0, 0, 0};
                    for (size_t j = 0; j < c; ++j) {
                        double v = r.Value(p.type);
                        if (j < 4) f[j] = (int)v;
                    }
                    if ((int)k != vi) continue;
                    if (c == 3) {
                        m.triIndices.insert(m.triIndices.end(), {f[0], f[1], f[2]});
                    } else if (c == 4) {
                        // rply_face_callback's bilinear-patch order 0 1 3 2
                        m.quadIndices.insert(m.quadIndices.end(), {f[0], f[1], f[3], f[2]});
                    } else {
                        ++m.skippedFaces;
                    }
                }
            }
        } else {
            // other elements are skipped
            for (size_t i = 0; i < e.count; ++i)
                for (const Property &p : e.props) {
                    if (p.isList) {
                        size_t c = (size_t)r.Value(p.countType);
                        for (size_t j = 0; j < c; ++j) r.Value(p.type);
                    } else {
                        r.Value(p.type);
                    }
                }
        }
    }
    for (int idx : m.triIndices)
        if (idx < 0 || idx >= (int)m.p.size())
            r.Fail("plymesh: Vertex index " + std::to_string(idx) + " is out of bounds! Valid range is [0.." +
                   std::to_string(m.p.size()) + ")");
    for (int idx : m.quadIndices)
        if (idx < 0 || idx >= (int)m.p.size())
            r.Fail("plymesh: Vertex index " + std::to_string(idx) + " is out of bounds! Valid range is [0.." +
                   std::to_string(m.p.size()) + ")");
    return m;
}

}  // namespace pbrt_amd
