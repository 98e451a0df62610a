// .pbrt scene-description subset loader (the drop-in boundary on the scene side).
// Mirrors the directive semantics of the reference parser and BasicSceneBuilder
// (parser.cpp, scene.cpp:92-98 fork defaults, scene.cpp CreateAggregate/CreateLights)
// for the statements the wavefront hot path needs; anything else fails loudly with the
// file location, as pbrt's ErrorExit does.
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <map>
#include <functional>
#include <memory>
#include <set>
#include <sstream>

#include "displace.h"
#include "ply.h"
#include "scene.h"
#include "texture.h"

namespace pbrt_amd {
// multispectral basis files (below, beside the texture instantiation)
void ReadBasisFile(const std::string &path, const std::string &loc, std::vector<float> *out);
// host/subdiv.cpp
void LoopSubdivideMesh(int nLevels, const std::vector<int> &indices, const std::vector<V3> &p, std::vector<V3> *P,
                       std::vector<int> *tris, std::vector<V3> *N);

// ------------------------------------------------------------------ matrices (double)
Mat4 Identity4() {
    Mat4 m{};
    for (int i = 0; i < 4; ++i) m[i][i] = 1;
    return m;
}
Mat4 Mul(const Mat4 &a, const Mat4 &b) {
    Mat4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += a[i][k] * b[k][j];
            r[i][j] = s;
        }
    return r;
}
Mat4 Inverse4(const Mat4 &m) {
    // Gauss-Jordan with full pivoting (util/math.cpp InvertOrExit semantics)
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    Mat4 minv = m;
    for (int i = 0; i < 4; i++) {
        int irow = 0, icol = 0;
        double big = 0.;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (std::fabs(minv[j][k]) >= big) {
                            big = std::fabs(minv[j][k]);
                            irow = j;
                            icol = k;
                        }
                    } else if (ipiv[k] > 1)
                        throw Error("singular matrix");
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(minv[irow][k], minv[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (minv[icol][icol] == 0.) throw Error("singular matrix");
        double pivinv = 1. / minv[icol][icol];
        minv[icol][icol] = 1.;
        for (int j = 0; j < 4; j++) minv[icol][j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                double save = minv[j][icol];
                minv[j][icol] = 0;
                for (int k = 0; k < 4; k++) minv[j][k] -= minv[icol][k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--) {
        if (indxr[j] != indxc[j]) {
            for (int k = 0; k < 4; k++) std::swap(minv[k][indxr[j]], minv[k][indxc[j]]);
        }
    }
    return minv;
}
V3 XformPoint(const Mat4 &m, V3 p) {
    double x = p.x, y = p.y, z = p.z;
    double xp = m[0][0] * x + m[0][1] * y + m[0][2] * z + m[0][3];
    double yp = m[1][0] * x + m[1][1] * y + m[1][2] * z + m[1][3];
    double zp = m[2][0] * x + m[2][1] * y + m[2][2] * z + m[2][3];
    double wp = m[3][0] * x + m[3][1] * y + m[3][2] * z + m[3][3];
    if (wp == 1) return V3((float)xp, (float)yp, (float)zp);
    return V3((float)(xp / wp), (float)(yp / wp), (float)(zp / wp));
}
V3 XformVector(const Mat4 &m, V3 v) {
    double x = v.x, y = v.y, z = v.z;
    return V3((float)(m[0][0] * x + m[0][1] * y + m[0][2] * z), (float)(m[1][0] * x + m[1][1] * y + m[1][2] * z),
              (float)(m[2][0] * x + m[2][1] * y + m[2][2] * z));
}
V3 XformNormal(const Mat4 &mi, V3 n) {
    double x = n.x, y = n.y, z = n.z;
    return V3((float)(mi[0][0] * x + mi[1][0] * y + mi[2][0] * z), (float)(mi[0][1] * x + mi[1][1] * y + mi[2][1] * z),
              (float)(mi[0][2] * x + mi[1][2] * y + mi[2][2] * z));
}
bool SwapsHandedness(const Mat4 &m) {
    double det = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]) -
                 m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]) +
                 m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    return det < 0;
}
static Mat4 TranslateM(double x, double y, double z) {
    Mat4 m = Identity4();
    m[0][3] = x;
    m[1][3] = y;
    m[2][3] = z;
    return m;
}
static Mat4 ScaleM(double x, double y, double z) {
    Mat4 m = Identity4();
    m[0][0] = x;
    m[1][1] = y;
    m[2][2] = z;
    return m;
}
static Mat4 RotateM(double theta, double ax, double ay, double az) {
    // util/transform.h Rotate(theta, axis)
    double len = std::sqrt(ax * ax + ay * ay + az * az);
    ax /= len;
    ay /= len;
    az /= len;
    double s = std::sin(theta * M_PI / 180.0), c = std::cos(theta * M_PI / 180.0);
    Mat4 m = Identity4();
    m[0][0] = ax * ax + (1 - ax * ax) * c;
    m[0][1] = ax * ay * (1 - c) - az * s;
    m[0][2] = ax * az * (1 - c) + ay * s;
    m[1][0] = ax * ay * (1 - c) + az * s;
    m[1][1] = ay * ay + (1 - ay * ay) * c;
    m[1][2] = ay * az * (1 - c) - ax * s;
    m[2][0] = ax * az * (1 - c) - ay * s;
    m[2][1] = ay * az * (1 - c) + ax * s;
    m[2][2] = az * az + (1 - az * az) * c;
    return m;
}
static Mat4 LookAtM(V3 pos, V3 look, V3 up) {
    // util/transform.cpp:81-117: cameraFromWorld = Inverse(worldFromCamera)
    auto nrm = [](double v[3]) {
        double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        v[0] /= l;
        v[1] /= l;
        v[2] /= l;
    };
    auto cross = [](const double a[3], const double b[3], double r[3]) {
        r[0] = a[1] * b[2] - a[2] * b[1];
        r[1] = a[2] * b[0] - a[0] * b[2];
        r[2] = a[0] * b[1] - a[1] * b[0];
    };
    double dir[3] = {(double)look.x - pos.x, (double)look.y - pos.y, (double)look.z - pos.z};
    nrm(dir);
    double u[3] = {up.x, up.y, up.z};
    nrm(u);
    double right[3];
    cross(u, dir, right);
    double rl = std::sqrt(right[0] * right[0] + right[1] * right[1] + right[2] * right[2]);
    if (rl == 0) throw Error("LookAt: up vector and viewing direction are parallel");
    nrm(right);
    double newUp[3];
    cross(dir, right, newUp);
    Mat4 w = Identity4();
    for (int i = 0; i < 3; ++i) {
        w[i][0] = right[i];
        w[i][1] = newUp[i];
        w[i][2] = dir[i];
    }
    w[0][3] = pos.x;
    w[1][3] = pos.y;
    w[2][3] = pos.z;
    return Inverse4(w);
}
static Mat4 PerspectiveM(double fov, double n, double f) {
    Mat4 persp{};
    persp[0][0] = 1;
    persp[1][1] = 1;
    persp[2][2] = f / (f - n);
    persp[2][3] = -f * n / (f - n);
    persp[3][2] = 1;
    double invTanAng = 1 / std::tan(fov * M_PI / 180.0 / 2);
    return Mul(ScaleM(invTanAng, invTanAng, 1), persp);
}

// ------------------------------------------------------------------ tokenizer
struct Token {
    std::string text;
    bool isString = false;
    std::string file;
    int line = 0;
};

static std::vector<Token> Tokenize(const std::string &src, const std::string &file) {
    std::vector<Token> toks;
    size_t i = 0, n = src.size();
    int line = 1;
    while (i < n) {
        char c = src[i];
        if (c == '\n') {
            ++line;
            ++i;
        } else if (std::isspace((unsigned char)c)) {
            ++i;
        } else if (c == '#') {
            while (i < n && src[i] != '\n') ++i;
        } else if (c == '"') {
            size_t j = i + 1;
            std::string s;
            while (j < n && src[j] != '"') {
                if (src[j] == '\n') throw Error(file + ":" + std::to_string(line) + ": unterminated string");
                if (src[j] == '\\' && j + 1 < n) {
                    ++j;
                    char e = src[j];
                    s += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
                } else
                    s += src[j];
                ++j;
            }
            toks.push_back({s, true, file, line});
            i = j + 1;
        } else if (c == '[' || c == ']') {
            toks.push_back({std::string(1, c), false, file, line});
            ++i;
        } else {
            size_t j = i;
            while (j < n && !std::isspace((unsigned char)src[j]) && src[j] != '"' && src[j] != '[' &&
                   src[j] != ']' && src[j] != '#')
                ++j;
            toks.push_back({src.substr(i, j - i), false, file, line});
            i = j;
        }
    }
    return toks;
}

// ------------------------------------------------------------------ parameters
struct Param {
    std::string type, name;
    std::vector<double> nums;
    std::vector<std::string> strs;
    std::vector<bool> bools;
    bool used = false;
    bool attribute = false;  // from an Attribute directive: may go unused (scene.cpp:209-213)
    int colorSpace = kColorSpaceSRGB;  // the graphics state's at parse time (ParsedParameter::colorSpace)
};
struct ParamSet {
    std::vector<Param> params;
    std::string loc;
    int colorSpace = kColorSpaceSRGB;  // ParameterDictionary::ColorSpace(): the directive's graphics state
    Param *Find(const std::string &name, const std::string &type = "") {
        for (auto &p : params)
            if (p.name == name && (type.empty() || p.type == type)) {
                p.used = true;
                return &p;
            }
        return nullptr;
    }
    double GetFloat(const std::string &name, double def) {
        Param *p = Find(name, "float");
        return (p && !p->nums.empty()) ? p->nums[0] : def;
    }
    int GetInt(const std::string &name, int def) {
        Param *p = Find(name, "integer");
        return (p && !p->nums.empty()) ? (int)p->nums[0] : def;
    }
    bool GetBool(const std::string &name, bool def) {
        Param *p = Find(name, "bool");
        return (p && !p->bools.empty()) ? (bool)p->bools[0] : def;
    }
    std::string GetString(const std::string &name, const std::string &def) {
        Param *p = Find(name, "string");
        return (p && !p->strs.empty()) ? p->strs[0] : def;
    }
    void CheckUnused() const {
        for (auto &p : params)
            if (!p.used && !p.attribute)
                throw Error(loc + ": parameter \"" + p.type + " " + p.name + "\" is not supported");
    }
};
// ParameterDictionary(params, attributes) (paramdict.cpp:150-159): a directive's own parameters
// first, then the graphics state's Attribute parameters of its target, latest first, so a lookup
// finds the directive's value, else the most recent attribute
static ParamSet WithAttributes(ParamSet own, const std::vector<Param> &attributes) {
    for (auto it = attributes.rbegin(); it != attributes.rend(); ++it) own.params.push_back(*it);
    return own;
}

struct GraphicsState {
    Mat4 ctm = Identity4();
    // Attribute "shape" / "light" / "material" / "medium" / "texture" parameters (scene.cpp:189-215),
    // scoped by AttributeBegin / AttributeEnd like the rest of the graphics state
    std::vector<Param> shapeAttributes, lightAttributes, materialAttributes, mediumAttributes, textureAttributes;
    bool reverseOrientation = false;
    int material = -1;  // index into materials (-1 -> default diffuse)
    std::string areaLightName;
    ParamSet areaLightParams;
    std::string insideMedium, outsideMedium;  // MediumInterface ("" = vacuum)
    int colorSpace = kColorSpaceSRGB;         // ColorSpace directive (scene.cpp:108-115)
};

class Parser {
  public:
    Parser(SceneDesc &s, const std::map<std::string, std::string> &ov) : scene(s), overrides(ov) {}

    void ParseFile(const std::string &path) {
        std::ifstream in(path);
        if (!in) throw Error("cannot open scene file " + path);
        std::stringstream ss;
        ss << in.rdbuf();
        std::string dir = path.substr(0, path.find_last_of('/') == std::string::npos ? 0 : path.find_last_of('/'));
        ParseString(ss.str(), path, dir);
    }

    void ParseString(const std::string &text, const std::string &file, const std::string &dir) {
        std::vector<Token> toks = Tokenize(text, file);
        size_t pos = 0;
        while (pos < toks.size()) Directive(toks, pos, dir);
    }

    void Finish();

  private:
    SceneDesc &scene;
    std::map<std::string, std::string> overrides;
    GraphicsState gs;
    std::vector<GraphicsState> stack;
    std::map<std::string, int> namedMaterials;
    std::map<std::string, Mat4> namedCoordSys;
    bool haveCamera = false;
    Mat4 cameraFromWorld = Identity4();
    ParamSet cameraParams, filmParams, samplerParams, integratorParams, filterParams;
    std::string cameraType = "perspective", filmType = "rgb";
    bool inWorld = false;
    float curImageKe = 1;  // the current shape's image-emitter k_e factor (power normalisation)
    struct PendingShape {
        int kind = 0;                 // 0 triangle mesh, kShapeSphereT, kShapeDiskT, kShapeBilinearT
        std::vector<int> quadIdx;     // bilinear patches: 4 vertex indices each (p00 p10 p01 p11)
        float sp[4] = {0, 0, 0, 0};   // sphere: radius zmin zmax phimax; disk: height radius innerradius phimax
        std::vector<V3> P;
        std::vector<int> idx;
        std::vector<float> uv;  // per vertex, 2 floats
        std::vector<V3> N;      // per vertex (object space)
        std::vector<V3> S;      // per-vertex shading tangents (object space; trianglemesh "S")
        std::string insideMedium, outsideMedium;
        Mat4 renderFromObject;
        bool flip;
        int material;
        std::string areaLight;
        ParamSet areaParams;
        std::string loc;
        std::string dir;  // directory of the declaring file (an area light's "filename")
        bool hasAlpha = false;  // "float alpha" < 1 or "texture alpha" (scene.cpp:1369-1384)
        Param alpha;
        bool hasDisp = false;  // plymesh "texture displacement", applied once textures resolve
        Param disp;
        float edgeLength = 1;
    };
    std::vector<PendingShape> shapes;
    void DisplacePlyMeshes();
    std::map<std::string, int> alphaIds;  // alpha parameter -> SceneDesc::alphaTex entry
    int AlphaId(const PendingShape &s);
    // object instancing (scene.cpp:309-395): shapes of each ObjectBegin/End definition, and the
    // ObjectInstance uses, resolved after parsing (a use may precede its definition)
    std::map<std::string, std::vector<PendingShape>> instanceDefs;
    std::string activeInstance;
    struct InstanceUse {
        std::string name, loc;
        Mat4 worldFromInstance;
    };
    std::vector<InstanceUse> instanceUses;
    struct PendingLight {
        std::string type;
        ParamSet params;
        Mat4 worldFromLight;
        std::string dir;  // directory of the file that declared it (relative "filename")
    };
    std::vector<PendingLight> lights;
    InfiniteLightDesc InfiniteLight(PendingLight &l);
    void ImageLight(PendingLight &l, const Mat4 &rfl, float sc, DeltaLightDesc *d);
    AreaLightDesc curSpread;  // the current AreaLightSource's spread terms
    void SetSpread(AreaLightDesc *l) const {
        l->image = curSpread.image;
        l->cosFalloffEnd = curSpread.cosFalloffEnd;
        l->tanFalloffEnd = curSpread.tanFalloffEnd;
        l->normFalloffEnd = curSpread.normFalloffEnd;
    }
    void DeltaLight(PendingLight &l, std::vector<DeltaLightDesc> &pointSpot, std::vector<DeltaLightDesc> &distants,
                    std::vector<int> &distantEntry, std::vector<std::pair<int, int>> &lsOrder);
    struct PendingMedium {
        std::string name, type;
        ParamSet params;
        Mat4 worldFromMedium;
    };
    std::vector<PendingMedium> pendingMedia;
    std::string cameraMediumName;
    // Texture directives (scene.cpp BasicSceneBuilder::Texture): kept by (name, is spectrum) and
    // instantiated per SpectrumType when a material uses them (scene.cpp CreateTextures)
    struct PendingTexture {
        std::string name, cls, dir;
        bool spectrum = false;
        ParamSet params;
        Mat4 worldFromTexture;
    };
    std::map<std::pair<std::string, bool>, PendingTexture> pendingTextures;
    std::map<std::tuple<std::string, bool, int>, int> texInstances;
    std::set<std::pair<std::string, bool>> texInProgress;
    // textured material parameters, resolved at Finish once the camera (render space) is known
    struct MatTexPending {
        int mat = -1;
        std::string loc;
        bool hasRefl = false;
        Param refl;
        int reflSpec = 0;  // kSpecAlbedo, or kSpecUnbounded (hair "sigma_a")
        bool hasRough = false;
        Param ur, vr;  // type "" = constant 0 (no parameter)
        bool remap = true;
        bool hasAmount = false;  // mix: "amount" (default 0.5)
        Param amount;
        bool hasDisp = false;   // "displacement" (a float texture or constant)
        Param disp;
        std::string normalMap;  // "normalmap" image file
        bool hasHair = false;   // hair: textured eta, beta_m, beta_n, alpha, eumelanin, pheomelanin
        Param hair[6];          // type "" = not textured
        bool hasSss = false;    // subsurface: textured sigma_a, and sigma_s or mfp (Unbounded)
        Param sss[2];
    };
    std::vector<MatTexPending> matTexPending;
    void ResolveTextures();
    int InstTex(const std::string &name, bool spectrum, int specType, const std::string &loc);
    int FloatTexParam(ParamSet &ps, const std::string &name, float def);
    int SpectrumTexParam(ParamSet &ps, const std::string &name, int specType, float def);
    int FloatParamNode(const Param *p, float def, const std::string &loc);
    int SpectrumParamNode(const Param *p, int specType, float def, const std::string &loc);
    int NewTexNode(const TextureDesc &t) {
        scene.textures.push_back(t);
        return (int)scene.textures.size() - 1;
    }
    TexSpectrumConst RGBConst(const Param *p, int specType, const std::string &loc);
    void TexMapping(ParamSet &ps, const Mat4 &renderFromTexture, TextureDesc *t, bool allow3D);

    static std::string Loc(const Token &t) { return t.file + ":" + std::to_string(t.line); }

    // BasicSceneBuilder::Option (scene.cpp:492-560) with the wavefront integrator's refusals
    // (wavefront/integrator.cpp:202-212)
    enum { kRenderCamera = 0, kRenderCameraWorld = 1, kRenderWorld = 2 };
    int renderSpace = kRenderCameraWorld;
    bool optionSeedSet = false;
    int optionSeed = 0;
    void Option(const std::string &name, const Token &v, const std::string &loc) {
        std::string n;  // normalizeArg (util/args.h:23-30)
        for (unsigned char c : name)
            if (c != '_' && c != '-') n += (char)std::tolower(c);
        const std::string raw = v.isString ? "\"" + v.text + "\"" : v.text;  // the token as pbrt sees it
        auto boolean = [&]() {
            if (raw == "true") return true;
            if (raw == "false") return false;
            throw Error(loc + ": " + raw + ": expected \"true\" or \"false\" for option value");
        };
        auto quoted = [&]() {
            if (!v.isString || v.text.empty()) throw Error(loc + ": " + raw + ": expected quoted string for option value");
            return v.text;
        };
        if (n == "disablepixeljitter") {
            scene.options = boolean() ? (scene.options | kOptNoPixelJitter) : (scene.options & ~kOptNoPixelJitter);
        } else if (n == "disabletexturefiltering") {
            scene.options = boolean() ? (scene.options | kOptNoTextureFiltering) : (scene.options & ~kOptNoTextureFiltering);
        } else if (n == "disablewavelengthjitter") {
            scene.options = boolean() ? (scene.options | kOptNoWavelengthJitter) : (scene.options & ~kOptNoWavelengthJitter);
        } else if (n == "displacementedgescale") {
            char *end = nullptr;
            const double e = std::strtod(raw.c_str(), &end);
            if (v.isString || end == raw.c_str() || *end) throw Error(loc + ": " + raw + ": expected floating-point option value");
            scene.displacementEdgeScale = (float)e;  // only displaced meshes use it: refused at their Shape
        } else if (n == "msereferenceimage") {
            quoted();
            throw Error(loc + ": The wavefront integrator does not support --mse-reference-image.");
        } else if (n == "msereferenceout") {
            quoted();  // the MSE output of a reference image, which the wavefront refuses anyway
        } else if (n == "rendercoordsys") {
            const std::string cs = quoted();
            if (cs == "camera") renderSpace = kRenderCamera;
            else if (cs == "cameraworld") renderSpace = kRenderCameraWorld;
            else if (cs == "world") renderSpace = kRenderWorld;
            else throw Error(loc + ": " + cs + ": unknown rendering coordinate system.");
        } else if (n == "seed") {
            optionSeedSet = true;
            optionSeed = std::atoi(raw.c_str());
        } else if (n == "forcediffuse") {
            if (boolean()) throw Error(loc + ": The wavefront integrator does not support --force-diffuse.");
        } else if (n == "pixelstats") {
            if (boolean()) throw Error(loc + ": The wavefront integrator does not support --pixelstats.");
        } else if (n == "wavefront") {
            boolean();  // this library is the wavefront integrator either way
        } else {
            throw Error(loc + ": " + name + ": unknown option");
        }
    }

    double Num(const std::vector<Token> &toks, size_t &pos) {
        if (pos >= toks.size()) throw Error("unexpected end of file");
        const Token &t = toks[pos++];
        char *end = nullptr;
        double v = std::strtod(t.text.c_str(), &end);
        if (t.isString || end == t.text.c_str() || *end) throw Error(Loc(t) + ": expected a number, got '" + t.text + "'");
        return v;
    }
    std::string Str(const std::vector<Token> &toks, size_t &pos) {
        if (pos >= toks.size() || !toks[pos].isString)
            throw Error((pos < toks.size() ? Loc(toks[pos]) : std::string("EOF")) + ": expected a quoted string");
        return toks[pos++].text;
    }
    ParamSet Params(const std::vector<Token> &toks, size_t &pos) {
        ParamSet ps;
        ps.loc = pos > 0 ? Loc(toks[pos - 1]) : "";
        ps.colorSpace = gs.colorSpace;
        while (pos < toks.size() && toks[pos].isString) {
            std::string decl = toks[pos].text;
            std::istringstream ds(decl);
            Param p;
            p.colorSpace = gs.colorSpace;
            ds >> p.type >> p.name;
            if (p.name.empty()) break;  // a bare string: not a parameter declaration
            ++pos;
            if (p.type == "point") p.type = "point3";
            if (p.type == "vector") p.type = "vector3";
            if (p.type == "color") p.type = "rgb";
            if (p.type == "normal3") p.type = "normal";
            auto value = [&](const Token &t) {
                if (p.type == "string" || p.type == "texture" || (p.type == "spectrum" && t.isString)) {
                    if (!t.isString) throw Error(Loc(t) + ": expected string value for " + p.name);
                    p.strs.push_back(t.text);
                } else if (p.type == "bool") {
                    std::string v = t.text;
                    if (v != "true" && v != "false") throw Error(Loc(t) + ": bad bool value");
                    p.bools.push_back(v == "true");
                } else {
                    char *end = nullptr;
                    double v = std::strtod(t.text.c_str(), &end);
                    if (t.isString || *end) throw Error(Loc(t) + ": bad numeric value '" + t.text + "'");
                    p.nums.push_back(v);
                }
            };
            if (pos < toks.size() && toks[pos].text == "[" && !toks[pos].isString) {
                ++pos;
                while (pos < toks.size() && !(toks[pos].text == "]" && !toks[pos].isString)) value(toks[pos++]);
                if (pos >= toks.size()) throw Error(ps.loc + ": unterminated [");
                ++pos;
            } else if (pos < toks.size()) {
                value(toks[pos++]);
            }
            ps.params.push_back(std::move(p));
        }
        return ps;
    }

    void Directive(const std::vector<Token> &toks, size_t &pos, const std::string &dir) {
        const Token &t = toks[pos++];
        const std::string &d = t.text;
        std::string loc = Loc(t);
        if (d == "LookAt") {
            double v[9];
            for (double &x : v) x = Num(toks, pos);
            gs.ctm = Mul(gs.ctm, LookAtM(V3(v[0], v[1], v[2]), V3(v[3], v[4], v[5]), V3(v[6], v[7], v[8])));
        } else if (d == "Translate") {
            double x = Num(toks, pos), y = Num(toks, pos), z = Num(toks, pos);
            gs.ctm = Mul(gs.ctm, TranslateM(x, y, z));
        } else if (d == "Scale") {
            double x = Num(toks, pos), y = Num(toks, pos), z = Num(toks, pos);
            gs.ctm = Mul(gs.ctm, ScaleM(x, y, z));
        } else if (d == "Rotate") {
            double a = Num(toks, pos), x = Num(toks, pos), y = Num(toks, pos), z = Num(toks, pos);
            gs.ctm = Mul(gs.ctm, RotateM(a, x, y, z));
        } else if (d == "Identity") {
            gs.ctm = Identity4();
        } else if (d == "Transform" || d == "ConcatTransform") {
            bool br = pos < toks.size() && toks[pos].text == "[";
            if (br) ++pos;
            double v[16];
            for (double &x : v) x = Num(toks, pos);
            if (br) {
                if (toks[pos].text != "]") throw Error(loc + ": expected ]");
                ++pos;
            }
            Mat4 m;
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) m[i][j] = v[j * 4 + i];  // Transpose(m)
            gs.ctm = (d == "Transform") ? m : Mul(gs.ctm, m);
        } else if (d == "CoordinateSystem") {
            namedCoordSys[Str(toks, pos)] = gs.ctm;
        } else if (d == "CoordSysTransform") {
            std::string n = Str(toks, pos);
            if (!namedCoordSys.count(n)) throw Error(loc + ": unknown coordinate system " + n);
            gs.ctm = namedCoordSys[n];
        } else if (d == "ReverseOrientation") {
            gs.reverseOrientation = !gs.reverseOrientation;
        } else if (d == "Camera") {
            cameraType = Str(toks, pos);
            cameraParams = Params(toks, pos);
            cameraParams.loc = loc;
            cameraFromWorld = gs.ctm;
            namedCoordSys["camera"] = Inverse4(gs.ctm);
            haveCamera = true;
            cameraMediumName = gs.outsideMedium;  // CameraSceneEntity's medium
        } else if (d == "Film") {
            filmType = Str(toks, pos);
            filmParams = Params(toks, pos);
            filmParams.loc = loc;
        } else if (d == "Sampler") {
            scene.samplerName = Str(toks, pos);
            samplerParams = Params(toks, pos);
            samplerParams.loc = loc;
        } else if (d == "PixelFilter") {
            scene.filterName = Str(toks, pos);
            filterParams = Params(toks, pos);
            filterParams.loc = loc;
        } else if (d == "Integrator") {
            scene.integratorName = Str(toks, pos);
            integratorParams = Params(toks, pos);
            integratorParams.loc = loc;
        } else if (d == "Accelerator") {
            Str(toks, pos);
            Params(toks, pos);  // the BVH8 build is the aggregate whatever is asked (gpu/aggregate.cpp)
        } else if (d == "ColorSpace") {
            // BasicSceneBuilder::ColorSpace (scene.cpp:108-115): RGBColorSpace::GetNamed
            const std::string name = Str(toks, pos);
            const int cs = ColorSpaceByName(name);
            if (cs < 0) throw Error(loc + ": " + name + ": color space unknown");
            gs.colorSpace = cs;
        } else if (d == "Option") {
            // parser.cpp:877-880: a quoted name, then one raw value token
            std::string name = Str(toks, pos);
            if (pos >= toks.size()) throw Error(loc + ": Option needs a value");
            Option(name, toks[pos], loc);
            ++pos;
        } else if (d == "Attribute") {
            // BasicSceneBuilder::Attribute (scene.cpp:189-215)
            std::string target = Str(toks, pos);
            ParamSet ps = Params(toks, pos);
            std::vector<Param> *attrs = target == "shape"      ? &gs.shapeAttributes
                                        : target == "light"    ? &gs.lightAttributes
                                        : target == "material" ? &gs.materialAttributes
                                        : target == "medium"   ? &gs.mediumAttributes
                                        : target == "texture"  ? &gs.textureAttributes
                                                               : nullptr;
            if (!attrs)
                throw Error(loc + ": Unknown attribute target \"" + target +
                            "\". Must be \"shape\", \"light\", \"material\", \"medium\", or \"texture\".");
            for (Param &p : ps.params) {
                p.attribute = true;
                attrs->push_back(p);
            }
        } else if (d == "WorldBegin") {
            inWorld = true;
            gs.ctm = Identity4();
            namedCoordSys["world"] = gs.ctm;
        } else if (d == "WorldEnd") {
        } else if (d == "AttributeBegin" || d == "TransformBegin") {
            stack.push_back(gs);
        } else if (d == "AttributeEnd" || d == "TransformEnd") {
            if (stack.empty()) throw Error(loc + ": unmatched " + d);
            if (d == "TransformEnd") {
                Mat4 m = stack.back().ctm;
                stack.pop_back();
                gs.ctm = m;
            } else {
                gs = stack.back();
                stack.pop_back();
            }
        } else if (d == "Material") {
            std::string type = Str(toks, pos);
            ParamSet ps = WithAttributes(Params(toks, pos), gs.materialAttributes);
            ps.loc = loc;
            gs.material = MakeMaterial(type, ps, "", dir);
        } else if (d == "MakeNamedMaterial") {
            std::string name = Str(toks, pos);
            ParamSet ps = WithAttributes(Params(toks, pos), gs.materialAttributes);
            ps.loc = loc;
            std::string type = ps.GetString("type", "");
            if (type.empty()) throw Error(loc + ": MakeNamedMaterial needs \"string type\"");
            namedMaterials[name] = MakeMaterial(type, ps, name, dir);
        } else if (d == "NamedMaterial") {
            std::string name = Str(toks, pos);
            if (!namedMaterials.count(name)) throw Error(loc + ": named material \"" + name + "\" undefined");
            gs.material = namedMaterials[name];
        } else if (d == "AreaLightSource") {
            gs.areaLightName = Str(toks, pos);
            gs.areaLightParams = WithAttributes(Params(toks, pos), gs.lightAttributes);
            gs.areaLightParams.loc = loc;
            if (gs.areaLightName != "diffuse") throw Error(loc + ": unsupported area light " + gs.areaLightName);
        } else if (d == "LightSource") {
            PendingLight l;
            l.type = Str(toks, pos);
            l.params = WithAttributes(Params(toks, pos), gs.lightAttributes);
            l.params.loc = loc;
            l.worldFromLight = gs.ctm;
            l.dir = dir;
            lights.push_back(std::move(l));
        } else if (d == "Shape") {
            std::string type = Str(toks, pos);
            ParamSet ps = WithAttributes(Params(toks, pos), gs.shapeAttributes);
            ps.loc = loc;
            Shape(type, ps, dir);
        } else if (d == "Include" || d == "Import") {
            std::string f = Str(toks, pos);
            std::string path = (f.size() && f[0] == '/') ? f : (dir.empty() ? f : dir + "/" + f);
            ParseFile(path);
        } else if (d == "MakeNamedMedium") {
            PendingMedium m;
            m.name = Str(toks, pos);
            m.params = WithAttributes(Params(toks, pos), gs.mediumAttributes);
            m.params.loc = loc;
            m.type = m.params.GetString("type", "");
            if (m.type.empty()) throw Error(loc + ": MakeNamedMedium needs \"string type\"");
            m.worldFromMedium = gs.ctm;
            for (auto &o : pendingMedia)
                if (o.name == m.name) throw Error(loc + ": medium \"" + m.name + "\" redefined");
            pendingMedia.push_back(std::move(m));
        } else if (d == "MediumInterface") {
            // one name: inside = outside; two: inside, outside (parser.cpp MediumInterface)
            std::string a = Str(toks, pos), b = a;
            if (pos < toks.size() && toks[pos].isString) b = Str(toks, pos);
            gs.insideMedium = a;
            gs.outsideMedium = b;
        } else if (d == "ObjectBegin") {
            std::string name = Str(toks, pos);
            if (!activeInstance.empty()) throw Error(loc + ": ObjectBegin called inside of instance definition");
            if (instanceDefs.count(name)) throw Error(loc + ": " + name + ": trying to redefine an object instance");
            stack.push_back(gs);  // as AttributeBegin
            instanceDefs[name];
            activeInstance = name;
        } else if (d == "ObjectEnd") {
            if (activeInstance.empty()) throw Error(loc + ": ObjectEnd called outside of instance definition");
            if (stack.empty()) throw Error(loc + ": unmatched ObjectEnd");
            gs = stack.back();
            stack.pop_back();
            activeInstance.clear();
        } else if (d == "ObjectInstance") {
            std::string name = Str(toks, pos);
            if (!activeInstance.empty()) throw Error(loc + ": ObjectInstance can't be called inside instance definition");
            instanceUses.push_back(InstanceUse{name, loc, gs.ctm});
        } else if (d == "Texture") {
            PendingTexture t;
            t.name = Str(toks, pos);
            std::string type = Str(toks, pos);
            t.cls = Str(toks, pos);
            t.params = WithAttributes(Params(toks, pos), gs.textureAttributes);
            t.params.loc = loc;
            if (type != "float" && type != "spectrum")
                throw Error(loc + ": " + type + ": texture type unknown. Must be \"float\" or \"spectrum\".");
            t.spectrum = type == "spectrum";
            t.worldFromTexture = gs.ctm;
            t.dir = dir;
            auto key = std::make_pair(t.name, t.spectrum);
            if (pendingTextures.count(key)) throw Error(loc + ": Redefining texture \"" + t.name + "\".");
            pendingTextures[key] = std::move(t);
        } else if (d == "ActiveTransform" || d == "TransformTimes") {
            throw Error(loc + ": directive " + d + " is not supported by the wavefront hot path yet");
        } else {
            throw Error(loc + ": unknown directive '" + d + "'");
        }
    }

    // RGBUnboundedSpectrum(cs, rgb) (util/spectrum.cpp:230-244) as a SssSpectrumDesc
    static SssSpectrumDesc UnboundedRGB(float r, float g, float b, int cs = kColorSpaceSRGB) {
        SssSpectrumDesc q;
        const float mx = std::max({r, g, b});
        q.kind = 1;
        q.scale = 2 * mx;
        const auto c = q.scale ? RGBToSigmoidCoeffs(r / q.scale, g / q.scale, b / q.scale, cs)
                               : RGBToSigmoidCoeffs(0, 0, 0, cs);
        q.c0 = c[0], q.c1 = c[1], q.c2 = c[2];
        return q;
    }
    // GetSpectrumTexture(name, SpectrumType::Albedo | Unbounded) of a constant "rgb" or
    // "spectrum" parameter (textured forms are refused)
    SssSpectrumDesc ConstSpectrum(Param *p, bool albedo, const std::string &loc, const char *mat) {
        if (p->type == "texture")
            throw Error(loc + ": textured \"" + p->name + "\" for the " + mat + " material is not supported yet");
        if (p->type == "rgb") {
            if (p->nums.size() != 3) throw Error(loc + ": " + p->name + " needs 3 values");
            const float r = (float)p->nums[0], g = (float)p->nums[1], b = (float)p->nums[2];
            if (albedo) {
                if (r < 0 || r > 1 || g < 0 || g > 1 || b < 0 || b > 1)
                    throw Error(loc + ": RGB parameter \"" + p->name + "\" used as an albedo has > 1 component.");
                SssSpectrumDesc q;
                q.kind = 1;
                q.scale = 1;
                const auto c = RGBToSigmoidCoeffs(r, g, b, p->colorSpace);
                q.c0 = c[0], q.c1 = c[1], q.c2 = c[2];
                return q;
            }
            if (r < 0 || g < 0 || b < 0) throw Error(loc + ": RGB parameter \"" + p->name + "\" has negative component.");
            return UnboundedRGB(r, g, b, p->colorSpace);
        }
        if (p->type == "spectrum") {
            SssSpectrumDesc q;
            q.kind = 2;
            q.pl = SpectrumParam(p, loc);
            return q;
        }
        throw Error(loc + ": \"" + p->type + " " + p->name + "\" is not supported for the " + mat + " material yet");
    }

    int MakeMaterial(const std::string &type, ParamSet &ps, const std::string &name, const std::string &dir) {
        MaterialDesc m;
        m.name = name;
        // shading-normal perturbation (materials.cpp: GetFloatTextureOrNull("displacement"),
        // scene.cpp normal map cache: Image::Read(normalmap, ColorEncoding::Linear)): every
        // material Create but hair's, interface's and mix's reads them (materials.cpp:51-664)
        if (type == "diffuse" || type == "dielectric" || type == "conductor" || type == "subsurface" ||
            type == "coateddiffuse" || type == "coatedconductor" || type == "diffusetransmission" ||
            type == "measured" || type == "retroreflective" || type == "thindielectric") {
            if (Param *d = ps.Find("displacement")) {
                MatTexPending &mp = PendingTex(ps.loc);
                mp.hasDisp = true;
                mp.disp = *d;
            }
            std::string nm = ps.GetString("normalmap", "");
            if (!nm.empty()) {
                if (nm[0] != '/' && !dir.empty()) nm = dir + "/" + nm;
                MatTexPending &mp = PendingTex(ps.loc);
                mp.normalMap = nm;
            }
        }
        if (type == "diffuse") {
            m.type = kMatDiffuse;
            Param *r = ps.Find("reflectance");
            if (!r) {
                m.constant = true;
                m.constantValue = 0.5f;
            } else if (r->type == "rgb") {
                if (r->nums.size() != 3) throw Error(ps.loc + ": reflectance needs 3 values");
                float rgb[3] = {(float)r->nums[0], (float)r->nums[1], (float)r->nums[2]};
                for (float v : rgb)
                    if (v < 0 || v > 1) throw Error(ps.loc + ": RGB reflectance must be in [0,1]");
                auto c = RGBToSigmoidCoeffs(rgb[0], rgb[1], rgb[2], r->colorSpace);
                m.c0 = c[0];
                m.c1 = c[1];
                m.c2 = c[2];
            } else if (r->type == "float") {
                m.constant = true;
                m.constantValue = (float)r->nums[0];
            } else if (r->type == "texture") {
                // GetSpectrumTexture("reflectance", ..., SpectrumType::Albedo) (materials.cpp)
                MatTexPending &mp = PendingTex(ps.loc);
                mp.hasRefl = true;
                mp.refl = *r;
            } else {
                throw Error(ps.loc + ": reflectance of type " + r->type + " not supported");
            }
        } else if (type == "mix") {
            // MixMaterial::Create (materials.cpp:105-125, scene.cpp CreateMaterials): two named
            // materials and a float "amount" texture the closest-hit stage can evaluate
            m.type = kMatMix;
            Param *ms = ps.Find("materials", "string");
            if (!ms || ms->strs.size() != 2) throw Error(ps.loc + ": Must provide two values for \"string materials\" for mix material.");
            for (int k = 0; k < 2; ++k) {
                auto it = namedMaterials.find(ms->strs[k]);
                if (it == namedMaterials.end()) throw Error(ps.loc + ": " + ms->strs[k] + ": named material not found.");
                m.mixMat[k] = it->second;
            }
            MatTexPending &mp = PendingTex(ps.loc);
            mp.hasAmount = true;
            if (Param *a = ps.Find("amount")) mp.amount = *a;
        } else if (type == "interface") {
            // a null material: the surface only bounds media (scene.cpp: "interface")
            m.type = kMatInterface;
        } else if (type == "dielectric") {
            // DielectricMaterial::Create (materials.cpp:51-74)
            m.type = kMatDielectric;
            if (Param *e = ps.Find("eta", "float")) {
                if (e->nums.empty()) throw Error(ps.loc + ": \"float eta\" needs a value");
                m.eta = (float)e->nums[0];
            } else if (Param *es = ps.Find("eta", "spectrum")) {
                // a non-constant eta: GetBxDF takes eta(lambda_0) and calls
                // SampledWavelengths::TerminateSecondary (materials.cpp:25-49)
                m.etaSpec = SpectrumParam(es, ps.loc);
            }
            Roughness(ps, &m);
        } else if (type == "subsurface") {
            // SubsurfaceMaterial::Create (materials.cpp:544-613): a DielectricBxDF(eta, roughness)
            // at the surface and a TabulatedBSSRDF below it
            m.type = kMatDielectric;
            SubsurfaceDesc d;
            d.g = (float)ps.GetFloat("g", 0.0f);
            const std::string nm = ps.GetString("name", "");
            auto unbounded = [](float r, float g, float b) { return UnboundedRGB(r, g, b); };
            auto param = [&](Param *p, bool albedo) { return ConstSpectrum(p, albedo, ps.loc, "subsurface"); };
            if (!nm.empty()) {
                // GetMediumScatteringProperties (media.cpp:74-151, 160-165): measured sigma'_s and
                // sigma_a in mm^-1 as RGBUnboundedSpectrum; g forced to 0
                auto it = GetSpectralData().mediumPresets.find(nm);
                if (it == GetSpectralData().mediumPresets.end()) throw Error(ps.loc + ": " + nm + ": named medium not found.");
                if (d.g != 0) std::fprintf(stderr, "%s: Warning: Non-zero \"g\" ignored with named scattering coefficients.\n", ps.loc.c_str());
                d.g = 0;
                const auto &pv = it->second;
                d.a = unbounded(pv[3], pv[4], pv[5]);
                d.b = unbounded(pv[0], pv[1], pv[2]);
            } else {
                Param *sa = ps.Find("sigma_a"), *ss = ps.Find("sigma_s");
                if (sa && !ss) throw Error(ps.loc + ": Provided \"sigma_a\" parameter without \"sigma_s\".");
                if (ss && !sa) throw Error(ps.loc + ": Provided \"sigma_s\" parameter without \"sigma_a\".");
                // a textured sigma_a / sigma_s / mfp (GetSpectrumTextureOrNull, Unbounded) is
                // evaluated per hit by the texture stage; k_vsss_* read it at the entry record
                auto sssTex = [&](Param *q, int k) {
                    MatTexPending &mp = PendingTex(ps.loc);
                    mp.hasSss = true;
                    mp.sss[k] = *q;
                };
                if (sa) {
                    if (sa->type == "texture") sssTex(sa, 0);
                    else d.a = param(sa, false);
                    if (ss->type == "texture") sssTex(ss, 1);
                    else d.b = param(ss, false);
                } else if (Param *refl = ps.Find("reflectance")) {
                    d.mode = 1;
                    if (refl->type == "texture") {
                        // evaluated per hit by the texture stage; k_vsss_* read it at the entry
                        MatTexPending &mp = PendingTex(ps.loc);
                        mp.hasRefl = true;
                        mp.refl = *refl;
                        mp.reflSpec = kSpecAlbedo;
                    } else {
                        d.a = param(refl, true);
                    }
                    if (Param *mfp = ps.Find("mfp")) {
                        if (mfp->type == "texture") sssTex(mfp, 1);
                        else d.b = param(mfp, false);
                    } else {
                        d.b.kind = 0, d.b.value = 1;  // ConstantSpectrum(1)
                    }
                } else {
                    d.a = unbounded(.0011f, .0024f, .014f);
                    d.b = unbounded(2.55f, 3.21f, 3.77f);
                }
            }
            d.scale = (float)ps.GetFloat("scale", 1.f);
            d.eta = (float)ps.GetFloat("eta", 1.33f);
            m.eta = d.eta;
            Roughness(ps, &m);
            d.fresnelC = 1 - 2 * FresnelMoment1(1 / d.eta);
            d.table = ComputeBeamDiffusionTable(d.g, d.eta);
            m.sss = (int)scene.sss.size();
            scene.sss.push_back(std::move(d));
        } else if (type == "hair") {
            // HairMaterial::Create (materials.cpp:135-184): sigma_a, else reflectance / color,
            // else eumelanin / pheomelanin (SigmaAFromConcentration, bxdfs.cpp:553-562), else
            // eumelanin 1.3; eta 1.55, beta_m .3, beta_n .3, alpha 2.  Constant parameters only.
            m.type = kMatHair;
            Param *sa = ps.Find("sigma_a"), *refl = ps.Find("reflectance");
            if (!refl) refl = ps.Find("color");
            Param *eu = ps.Find("eumelanin"), *ph = ps.Find("pheomelanin");
            auto warn = [&](const char *what) { std::fprintf(stderr, "%s: Warning: %s\n", ps.loc.c_str(), what); };
            auto constFloat = [&](Param *p) {
                if (p->type != "float" || p->nums.empty())
                    throw Error(ps.loc + ": \"" + p->type + " " + p->name + "\" is not a float parameter of the hair material");
                return (float)p->nums[0];
            };
            // a textured sigma_a (Unbounded) or reflectance (Albedo) is evaluated per hit by the
            // texture stage (GetSpectrumTexture, materials.cpp:135-160)
            auto textured = [&](Param *p, int spec) {
                MatTexPending &mp = PendingTex(ps.loc);
                mp.hasRefl = true;
                mp.refl = *p;
                mp.reflSpec = spec;
            };
            if (sa) {
                if (refl) warn("Ignoring \"reflectance\" parameter since \"sigma_a\" was provided.");
                if (eu) warn("Ignoring \"eumelanin\" parameter since \"sigma_a\" was provided.");
                if (ph) warn("Ignoring \"pheomelanin\" parameter since \"sigma_a\" was provided.");
                m.hairMode = 0;
                if (sa->type == "texture") textured(sa, kSpecUnbounded);
                else m.hairSpec = ConstSpectrum(sa, false, ps.loc, "hair");
            } else if (refl) {
                if (eu) warn("Ignoring \"eumelanin\" parameter since \"reflectance\" was provided.");
                if (ph) warn("Ignoring \"pheomelanin\" parameter since \"reflectance\" was provided.");
                m.hairMode = 1;
                if (refl->type == "texture") textured(refl, kSpecAlbedo);
                else m.hairSpec = ConstSpectrum(refl, true, ps.loc, "hair");
            } else if ((eu && eu->type == "texture") || (ph && ph->type == "texture")) {
                // textured concentrations: sigma_a = SigmaAFromConcentration(ce, cp) per hit
                // (materials.h:396-399), a missing concentration is 0
                MatTexPending &mp = PendingTex(ps.loc);
                mp.hasHair = true;
                if (eu) mp.hair[4] = *eu;
                if (ph) mp.hair[5] = *ph;
                m.hairMode = 0;
            } else {
                // the concentrations' RGB sigma_a (ce, cp clamped at 0 by GetBxDF)
                const float ce = eu ? std::max(0.f, constFloat(eu)) : (ph ? 0.f : 1.3f);
                const float cp = ph ? std::max(0.f, constFloat(ph)) : 0.f;
                m.hairMode = 0;
                m.hairSpec = UnboundedRGB(ce * 0.419f + cp * 0.187f, ce * 0.697f + cp * 0.4f, ce * 1.37f + cp * 1.05f);
            }
            m.eta = 1.55f;
            // eta, beta_m, beta_n, alpha: constants, or float textures evaluated per hit
            auto hairFloat = [&](const char *name, int k, float *dst) {
                Param *q = ps.Find(name);
                if (!q) return;
                if (q->type == "texture") {
                    MatTexPending &mp = PendingTex(ps.loc);
                    mp.hasHair = true;
                    mp.hair[k] = *q;
                } else {
                    *dst = constFloat(q);
                }
            };
            hairFloat("eta", 0, &m.eta);
            hairFloat("beta_m", 1, &m.hairBetaM);
            hairFloat("beta_n", 2, &m.hairBetaN);
            hairFloat("alpha", 3, &m.hairAlpha);
        } else if (type == "measured") {
            // MeasuredMaterial::Create (materials.cpp:644-667): the resolved "filename", each
            // file read once (MeasuredBxDF::BRDFDataFromFile's cache, bxdfs.cpp:995-1001)
            m.type = kMatMeasured;
            const std::string f = ps.GetString("filename", "");
            if (f.empty()) throw Error(ps.loc + ": Filename must be provided for MeasuredMaterial");
            const std::string path = (f[0] == '/') ? f : (dir.empty() ? f : dir + "/" + f);
            for (size_t k = 0; k < scene.measured.size() && m.measured < 0; ++k)
                if (scene.measured[k].path == path) m.measured = (int)k;
            if (m.measured < 0) {
                try {
                    scene.measured.push_back(LoadMeasuredBRDF(path));
                } catch (const std::exception &e) {
                    throw Error(ps.loc + ": " + e.what());
                }
                m.measured = (int)scene.measured.size() - 1;
            }
        } else if (type == "diffusetransmission") {
            // DiffuseTransmissionMaterial::Create (materials.cpp:620-645): reflectance and
            // transmittance default 0.25, scale 1; the transmittance rides in the albedo fields
            m.type = kMatDiffuseTransmission;
            m.constant = true;
            m.constantValue = 0.25f;
            if (Param *r = ps.Find("reflectance")) AlbedoParam(r, ps.loc, &m.constant, &m.constantValue, &m.c0, &m.c1, &m.c2);
            m.albedoConstant = true;
            m.albedoValue = 0.25f;
            if (Param *t = ps.Find("transmittance"))
                AlbedoParam(t, ps.loc, &m.albedoConstant, &m.albedoValue, &m.a0, &m.a1, &m.a2);
            m.scale = ps.GetFloat("scale", 1.f);
        } else if (type == "thindielectric") {
            // ThinDielectricMaterial::Create (materials.cpp:83-97): eta only, always specular
            m.type = kMatThinDielectric;
            if (Param *e = ps.Find("eta", "float")) {
                if (e->nums.empty()) throw Error(ps.loc + ": \"float eta\" needs a value");
                m.eta = (float)e->nums[0];
            } else if (Param *es = ps.Find("eta", "spectrum")) {
                m.etaSpec = SpectrumParam(es, ps.loc);  // eta(lambda_0) + TerminateSecondary
            }
        } else if (type == "conductor" || type == "retroreflective") {
            // ConductorMaterial::Create (materials.cpp:217-251); RetroreflectiveMaterial::Create
            // (materials.cpp:263-297) reads the same parameters for its RetroreflectiveBxDF
            m.type = type == "conductor" ? kMatConductor : kMatRetroreflective;
            if (m.type == kMatRetroreflective)
                for (const Param &q : ps.params)
                    if (q.type == "texture" && !q.attribute && q.name != "displacement")
                        throw Error(ps.loc + ": textured parameters of the retroreflective material are not supported yet");
            Param *eta = ps.Find("eta"), *k = ps.Find("k"), *refl = ps.Find("reflectance");
            if (refl && (eta || k))
                throw Error(ps.loc + ": For the conductor material, both \"reflectance\" and \"eta\" and \"k\" can't be provided.");
            if (refl && refl->type == "texture") {
                MatTexPending &mp = PendingTex(ps.loc);
                mp.hasRefl = true;
                mp.refl = *refl;
            } else if (refl) {
                if (refl->type != "rgb" || refl->nums.size() != 3)
                    throw Error(ps.loc + ": conductor reflectance must be \"rgb\" (3 values)");
                float rgb[3] = {(float)refl->nums[0], (float)refl->nums[1], (float)refl->nums[2]};
                for (float v : rgb)
                    if (v < 0 || v > 1) throw Error(ps.loc + ": RGB parameter \"reflectance\" used as an albedo has > 1 component.");
                auto c = RGBToSigmoidCoeffs(rgb[0], rgb[1], rgb[2], refl->colorSpace);
                m.c0 = c[0];
                m.c1 = c[1];
                m.c2 = c[2];
            } else {
                m.etaSpec = eta ? SpectrumParam(eta, ps.loc) : NamedPLSpectrum("metal-Cu-eta", ps.loc);
                m.kSpec = k ? SpectrumParam(k, ps.loc) : NamedPLSpectrum("metal-Cu-k", ps.loc);
            }
            Roughness(ps, &m);
        } else if (type == "coateddiffuse") {
            // CoatedDiffuseMaterial::Create (materials.cpp:347-389)
            m.type = kMatCoatedDiffuse;
            Param *r = ps.Find("reflectance");
            if (!r) {
                m.constant = true;
                m.constantValue = 0.5f;
            } else {
                AlbedoParam(r, ps.loc, &m.constant, &m.constantValue, &m.c0, &m.c1, &m.c2);
            }
            Roughness(ps, &m);
            LayerParams(ps, &m, "eta");
        } else if (type == "coatedconductor") {
            // CoatedConductorMaterial::Create (materials.cpp:460-540)
            m.type = kMatCoatedConductor;
            MaterialDesc c;
            Roughness(ps, &m, "interface.");
            Roughness(ps, &c, "conductor.");
            m.cAlphaX = c.alphaX;
            m.cAlphaY = c.alphaY;
            Param *eta = ps.Find("conductor.eta"), *k = ps.Find("conductor.k"), *refl = ps.Find("reflectance");
            if (refl && (eta || k))
                throw Error(ps.loc + ": For the coated conductor material, both \"reflectance\" and \"eta\" and \"k\" can't be provided.");
            if (refl) {
                if (refl->type != "rgb" || refl->nums.size() != 3)
                    throw Error(ps.loc + ": coated conductor reflectance must be \"rgb\" (3 values)");
                float rgb[3] = {(float)refl->nums[0], (float)refl->nums[1], (float)refl->nums[2]};
                for (float v : rgb)
                    if (v < 0 || v > 1) throw Error(ps.loc + ": RGB parameter \"reflectance\" used as an albedo has > 1 component.");
                auto cf = RGBToSigmoidCoeffs(rgb[0], rgb[1], rgb[2], refl->colorSpace);
                m.c0 = cf[0];
                m.c1 = cf[1];
                m.c2 = cf[2];
            } else {
                m.etaSpec = eta ? SpectrumParam(eta, ps.loc) : NamedPLSpectrum("metal-Cu-eta", ps.loc);
                m.kSpec = k ? SpectrumParam(k, ps.loc) : NamedPLSpectrum("metal-Cu-k", ps.loc);
            }
            LayerParams(ps, &m, "interface.eta");
        } else {
            throw Error(ps.loc + ": material \"" + type + "\" is not supported yet");
        }
        ps.Find("type");
        ps.CheckUnused();
        scene.materials.push_back(m);
        return (int)scene.materials.size() - 1;
    }

    // an Albedo-type spectrum parameter: "rgb" in [0,1] (RGBAlbedoSpectrum sigmoid) or "float"
    void AlbedoParam(Param *r, const std::string &loc, bool *constant, float *value, float *c0, float *c1, float *c2) {
        if (r->type == "rgb") {
            if (r->nums.size() != 3) throw Error(loc + ": " + r->name + " needs 3 values");
            float rgb[3] = {(float)r->nums[0], (float)r->nums[1], (float)r->nums[2]};
            for (float v : rgb)
                if (v < 0 || v > 1) throw Error(loc + ": RGB " + r->name + " must be in [0,1]");
            auto c = RGBToSigmoidCoeffs(rgb[0], rgb[1], rgb[2], r->colorSpace);
            *constant = false;
            *c0 = c[0];
            *c1 = c[1];
            *c2 = c[2];
        } else if (r->type == "float" && !r->nums.empty()) {
            *constant = true;
            *value = (float)r->nums[0];
        } else {
            throw Error(loc + ": " + r->name + " of type " + r->type + " not supported");
        }
    }
    // the LayeredBxDF parameters common to both coated materials; etaName: the interface IOR
    void LayerParams(ParamSet &ps, MaterialDesc *m, const std::string &etaName) {
        if (Param *e = ps.Find(etaName, "float")) {
            if (e->nums.empty()) throw Error(ps.loc + ": \"float " + etaName + "\" needs a value");
            m->eta = (float)e->nums[0];
        } else if (Param *es = ps.Find(etaName, "spectrum")) {
            m->ifaceEtaSpec = SpectrumParam(es, ps.loc);  // eta(lambda_0) + TerminateSecondary
        }
        if (m->eta == 0) m->eta = 1;
        m->thickness = ps.GetFloat("thickness", .01f);
        m->g = ps.GetFloat("g", 0.f);
        m->maxDepth = ps.GetInt("maxdepth", 10);
        m->nSamples = ps.GetInt("nsamples", 1);
        if (Param *a = ps.Find("albedo")) AlbedoParam(a, ps.loc, &m->albedoConstant, &m->albedoValue, &m->a0, &m->a1, &m->a2);
    }

    // uroughness / vroughness / roughness + remaproughness -> TrowbridgeReitzDistribution alphas
    // (materials.cpp:62-70, materials.h:194-199 / :494-509, util/scattering.h:109-118, 192);
    // prefix "interface." / "conductor." for the coated conductor's two distributions
    // the MatTexPending record of the material MakeMaterial is building
    MatTexPending &PendingTex(const std::string &loc) {
        const int idx = (int)scene.materials.size();
        if (matTexPending.empty() || matTexPending.back().mat != idx) {
            matTexPending.emplace_back();
            matTexPending.back().mat = idx;
            matTexPending.back().loc = loc;
        }
        return matTexPending.back();
    }
    void Roughness(ParamSet &ps, MaterialDesc *m, const std::string &prefix = "") {
        // GetFloatTextureOrNull("uroughness" / "vroughness"), else GetFloatTexture("roughness", 0)
        // (materials.cpp:51-74, 217-251): a textured roughness is evaluated per hit
        auto findTex = [&](const std::string &n) -> Param * {
            for (auto &p : ps.params)
                if (p.name == n && p.type == "texture") return &p;
            return nullptr;
        };
        Param *ut = findTex(prefix + "uroughness"), *vt = findTex(prefix + "vroughness"), *rt = findTex(prefix + "roughness");
        if (ut || vt || rt) {
            if (!prefix.empty()) throw Error(ps.loc + ": textured " + prefix + "roughness is not supported yet");
            Param *uf = ut ? ut : ps.Find("uroughness", "float"), *vf = vt ? vt : ps.Find("vroughness", "float");
            Param *rf = rt ? rt : ps.Find("roughness", "float");
            MatTexPending &mp = PendingTex(ps.loc);
            mp.hasRough = true;
            if (uf) mp.ur = *uf;
            else if (rf) mp.ur = *rf;
            if (vf) mp.vr = *vf;
            else if (rf) mp.vr = *rf;
            for (Param *q : {ut, vt, rt, uf, vf, rf})
                if (q) q->used = true;
            mp.remap = ps.GetBool("remaproughness", true);
            m->remapRoughness = mp.remap;
            return;
        }
        Param *u = ps.Find(prefix + "uroughness", "float"), *v = ps.Find(prefix + "vroughness", "float");
        float ur = 0, vr = 0;
        if (!u || !v) {
            Param *r = ps.Find(prefix + "roughness", "float");
            float rv = (r && !r->nums.empty()) ? (float)r->nums[0] : 0.f;
            ur = vr = rv;
        }
        if (u) ur = u->nums.empty() ? 0.f : (float)u->nums[0];
        if (v) vr = v->nums.empty() ? 0.f : (float)v->nums[0];
        if (ps.GetBool("remaproughness", true)) {
            ur = RoughnessToAlpha(ur);
            vr = RoughnessToAlpha(vr);
        }
        TrowbridgeReitz t = TrowbridgeReitz::Make(ur, vr);
        m->alphaX = t.ax;
        m->alphaY = t.ay;
    }

    // named spectrum -> PiecewiseLinearSpectrum::FromInterleaved(samples, normalize = false)
    // (util/spectrum.cpp:133-163, 2636-2662): extended to cover Lambda_min..Lambda_max
    int NamedPLSpectrum(const std::string &name, const std::string &loc) {
        try {
            scene.plSpectra.push_back(NamedPiecewiseLinear(name));
        } catch (const Error &e) {
            throw Error(loc + ": " + e.what());
        }
        return (int)scene.plSpectra.size() - 1;
    }

    // "spectrum" parameter of an Unbounded spectrum texture (paramdict.cpp:384-450, :817-875)
    int SpectrumParam(Param *p, const std::string &loc) {
        if (p->type == "spectrum" && !p->strs.empty()) return NamedPLSpectrum(p->strs[0], loc);
        if (p->type == "spectrum" && !p->nums.empty()) {
            if (p->nums.size() % 2) throw Error(loc + ": Found odd number of values for \"" + p->name + "\"");
            PLSpectrumDesc d;
            for (size_t i = 0; i < p->nums.size(); i += 2) {
                if (i > 0 && (float)p->nums[i] <= d.lambda.back())
                    throw Error(loc + ": Spectrum description invalid: wavelengths aren't increasing");
                d.lambda.push_back((float)p->nums[i]);
                d.value.push_back((float)p->nums[i + 1]);
            }
            if (d.lambda.size() < 2) throw Error(loc + ": spectrum \"" + p->name + "\" needs at least two samples");
            scene.plSpectra.push_back(std::move(d));
            return (int)scene.plSpectra.size() - 1;
        }
        throw Error(loc + ": \"" + p->type + " " + p->name + "\" is not supported for conductors yet (use \"spectrum\")");
    }

    // Curve parameters as Curve::Create reads them (shapes.cpp:1004-1105), then the dicing of
    // OptiXAggregate::diceCurveToBLP: nDiceU + 1 rings along the curve's global u (each in the
    // cubic Bezier segment u falls in: degree 2 elevated, b-splines converted, util/splines.h),
    // a ribbon's two edges across the slerped normal, or a tube of nDiceV + 1 vertices around
    // flat and cylinder curves (with per-vertex normals), all in float as the reference has them.
    static void DiceCurve(ParamSet &ps, PendingShape *s, int nDiceU, int nDiceV) {
        const float width = (float)ps.GetFloat("width", 1.f);
        const float width0 = (float)ps.GetFloat("width0", width), width1 = (float)ps.GetFloat("width1", width);
        const int degree = ps.GetInt("degree", 3);
        if (degree != 2 && degree != 3)
            throw Error(ps.loc + ": Invalid degree " + std::to_string(degree) + ": only degree 2 and 3 curves are supported.");
        const std::string basis = ps.GetString("basis", "bezier");
        if (basis != "bezier" && basis != "bspline")
            throw Error(ps.loc + ": Invalid basis \"" + basis + "\": only \"bezier\" and \"bspline\" are supported.");
        std::vector<V3> cp;
        Param *P = ps.Find("P", "point3");
        if (!P) P = ps.Find("P", "point");
        if (P)
            for (size_t i = 0; i + 2 < P->nums.size(); i += 3) cp.push_back(V3((float)P->nums[i], (float)P->nums[i + 1], (float)P->nums[i + 2]));
        const bool bezier = basis == "bezier";
        int nSegments;
        if (bezier) {
            if (cp.size() < (size_t)degree + 1 || (cp.size() - 1 - degree) % degree != 0)
                throw Error(ps.loc + ": Invalid number of control points " + std::to_string(cp.size()) + ": for the degree " +
                            std::to_string(degree) + " Bezier basis " + std::to_string(degree + 1) + " + n * " +
                            std::to_string(degree) + " are required, for n >= 0.");
            nSegments = (int)(cp.size() - 1) / degree;
        } else {
            if (cp.size() < (size_t)degree + 1)
                throw Error(ps.loc + ": Invalid number of control points " + std::to_string(cp.size()) + ": for the degree " +
                            std::to_string(degree) + " b-spline basis, must have >= " + std::to_string(degree + 1) + ".");
            nSegments = (int)cp.size() - degree;
        }
        enum { kFlat, kCylinder, kRibbon } ctype = kFlat;
        const std::string ct = ps.GetString("type", "flat");
        if (ct == "ribbon")
            ctype = kRibbon;
        else if (ct == "cylinder")
            ctype = kCylinder;
        else if (ct != "flat") {
            std::fprintf(stderr, "%s: Error: Unknown curve type \"%s\".  Using \"cylinder\".\n", ps.loc.c_str(), ct.c_str());
            ctype = kCylinder;
        }
        std::vector<V3> n;
        Param *N = ps.Find("N", "normal");
        if (!N) N = ps.Find("N", "normal3");
        if (N)
            for (size_t i = 0; i + 2 < N->nums.size(); i += 3) n.push_back(V3((float)N->nums[i], (float)N->nums[i + 1], (float)N->nums[i + 2]));
        if (!n.empty()) {
            if (ctype != kRibbon) {
                std::fprintf(stderr, "%s: Warning: Curve normals are only used with \"ribbon\" type curves.\n", ps.loc.c_str());
                n.clear();
            } else if ((int)n.size() != nSegments + 1) {
                throw Error(ps.loc + ": Invalid number of normals " + std::to_string(n.size()) + ": must provide " +
                            std::to_string(nSegments + 1) + " normals for ribbon curves with " + std::to_string(nSegments) +
                            " segments.");
            }
            for (V3 &v : n) v = Normalize(v);
        } else if (ctype == kRibbon) {
            throw Error(ps.loc + ": Must provide normals \"N\" at curve endpoints with ribbon curves.");
        }
        ps.GetInt("splitdepth", 3);  // Curve::Create's subdivision; the diced mesh has none
        auto lerp = [](float t, V3 a, V3 b) { return (1 - t) * a + t * b; };
        int lastOffset = -1;
        V3 seg[4];
        for (int i = 0; i <= nDiceU; ++i) {
            const float u = float(i) / float(nDiceU);
            const float w = (1 - u) * width0 + u * width1;
            int segmentIndex = int(u * nSegments);
            if (segmentIndex == nSegments) --segmentIndex;
            const int off = bezier ? segmentIndex * degree : segmentIndex;
            if (off != lastOffset) {
                const V3 *c = &cp[off];
                if (bezier && degree == 3) {
                    for (int k = 0; k < 4; ++k) seg[k] = c[k];
                } else if (degree == 2) {
                    // QuadraticBSplineToBezier, then ElevateQuadraticBezierToCubic
                    V3 q[3] = {c[0], c[1], c[2]};
                    if (!bezier) q[0] = lerp(0.5f, c[0], c[1]), q[2] = lerp(0.5f, c[1], c[2]);
                    seg[0] = q[0];
                    seg[1] = lerp(2.f / 3.f, q[0], q[1]);
                    seg[2] = lerp(1.f / 3.f, q[1], q[2]);
                    seg[3] = q[2];
                } else {
                    // CubicBSplineToBezier (blossoming)
                    const V3 p122 = lerp(2.f / 3.f, c[0], c[1]), p223 = lerp(1.f / 3.f, c[1], c[2]);
                    const V3 p233 = lerp(2.f / 3.f, c[1], c[2]), p334 = lerp(1.f / 3.f, c[2], c[3]);
                    seg[0] = lerp(0.5f, p122, p223);
                    seg[1] = p223;
                    seg[2] = p233;
                    seg[3] = lerp(0.5f, p233, p334);
                }
                lastOffset = off;
            }
            const float uSeg = (u * nSegments) - segmentIndex;
            // EvaluateCubicBezier with its derivative (util/splines.h:30-43)
            const V3 c1[3] = {lerp(uSeg, seg[0], seg[1]), lerp(uSeg, seg[1], seg[2]), lerp(uSeg, seg[2], seg[3])};
            const V3 c2[2] = {lerp(uSeg, c1[0], c1[1]), lerp(uSeg, c1[1], c1[2])};
            const V3 dpdu = LengthSquared(c2[1] - c2[0]) > 0 ? 3 * (c2[1] - c2[0]) : seg[3] - seg[0];
            const V3 p = lerp(uSeg, c2[0], c2[1]);
            const int base = (int)s->P.size();
            if (ctype == kRibbon) {
                const V3 n0 = n[segmentIndex], n1 = n[segmentIndex + 1];
                const float normalAngle =
                    DotN(n0, n1) < 0 ? kPi - 2 * SafeASin(Length(n0 + n1) / 2) : 2 * SafeASin(Length(n1 - n0) / 2);
                const float invSinNormalAngle = 1 / std::sin(normalAngle);
                V3 nu;
                if (normalAngle == 0) {
                    nu = n0;
                } else {
                    const float sin0 = std::sin((1 - uSeg) * normalAngle) * invSinNormalAngle;
                    const float sin1 = std::sin(uSeg * normalAngle) * invSinNormalAngle;
                    nu = sin0 * n0 + sin1 * n1;
                }
                const V3 dpdv = Normalize(Cross(nu, dpdu)) * w;
                s->P.push_back(p - dpdv / 2);
                s->P.push_back(p + dpdv / 2);
                s->uv.insert(s->uv.end(), {u, 0.f, u, 1.f});
                if (i > 0) s->quadIdx.insert(s->quadIdx.end(), {base - 2, base - 1, base, base + 1});
            } else {
                V3 o0, o1;
                CoordinateSystem(Normalize(dpdu), &o0, &o1);
                o0 = o0 * (w / 2);
                o1 = o1 * (w / 2);
                for (int v = 0; v <= nDiceV; ++v) {
                    const float angle = float(v) / nDiceV * 2 * kPi;
                    const V3 q = p + o0 * std::cos(angle) + o1 * std::sin(angle);
                    s->P.push_back(q);
                    s->N.push_back(Normalize(q - p));
                    s->uv.insert(s->uv.end(), {u, float(v) / nDiceV});
                }
                if (i > 0)
                    for (int v = 0; v < nDiceV; ++v) {
                        const int r0 = (nDiceV + 1) * (i - 1), r1 = (nDiceV + 1) * i;
                        s->quadIdx.insert(s->quadIdx.end(), {r0 + v, r0 + v + 1, r1 + v, r1 + v + 1});
                    }
            }
        }
    }

    // Shape "trianglemesh" (Triangle::CreateMesh, shapes.cpp:1380-1417) and "plymesh"
    // (shapes.cpp:1418-1478; TriQuadMesh::ReadPLY, util/mesh.cpp:322-420)
    void Shape(const std::string &type, ParamSet &ps, const std::string &dir) {
        PendingShape s;
        if (type == "trianglemesh") {
            Param *P = ps.Find("P", "point3");
            if (!P || P->nums.size() % 3) throw Error(ps.loc + ": trianglemesh needs \"point3 P\"");
            for (size_t i = 0; i < P->nums.size(); i += 3) s.P.push_back(V3(P->nums[i], P->nums[i + 1], P->nums[i + 2]));
            Param *I = ps.Find("indices", "integer");
            if (I)
                for (double v : I->nums) s.idx.push_back((int)v);
            else if (s.P.size() == 3)
                s.idx = {0, 1, 2};
            else
                throw Error(ps.loc + ": trianglemesh needs \"integer indices\"");
            if (s.idx.size() % 3) throw Error(ps.loc + ": indices not a multiple of 3");
            for (int v : s.idx)
                if (v < 0 || v >= (int)s.P.size()) throw Error(ps.loc + ": vertex index out of range");
            Param *uv = ps.Find("uv", "point2");
            if (uv) {
                if (uv->nums.size() != 2 * s.P.size()) throw Error(ps.loc + ": uv count mismatch");
                for (double v : uv->nums) s.uv.push_back((float)v);
            }
            Param *N = ps.Find("N", "normal");
            if (!N) N = ps.Find("N", "normal3");
            if (N) {
                if (N->nums.size() != 3 * s.P.size()) throw Error(ps.loc + ": N count mismatch");
                for (size_t i = 0; i < N->nums.size(); i += 3) s.N.push_back(V3(N->nums[i], N->nums[i + 1], N->nums[i + 2]));
            }
            // per-vertex shading tangents (shapes.cpp:408-413): a count mismatch is reported and
            // the tangents discarded, as pbrt's Error() does
            Param *Sp = ps.Find("S", "vector3");
            if (!Sp) Sp = ps.Find("S", "vector");
            if (Sp) {
                if (Sp->nums.size() != 3 * s.P.size()) {
                    std::fprintf(stderr, "%s: Error: Number of \"S\"s for triangle mesh must match \"P\"s. Discarding \"S\"s.\n",
                                 ps.loc.c_str());
                } else {
                    for (size_t i = 0; i < Sp->nums.size(); i += 3)
                        s.S.push_back(V3(Sp->nums[i], Sp->nums[i + 1], Sp->nums[i + 2]));
                }
            }
            ps.Find("faceIndices");
        } else if (type == "plymesh") {
            std::string f = ps.GetString("filename", "");
            if (f.empty()) throw Error(ps.loc + ": plymesh needs \"string filename\"");
            std::string path = (f[0] == '/') ? f : (dir.empty() ? f : dir + "/" + f);
            // shapes.cpp:1422-1458: a displacement texture refines and displaces the mesh
            // (DisplacePlyMeshes, once the textures are resolved)
            s.edgeLength = (float)ps.GetFloat("edgelength", 1);
            if (Param *dp = ps.Find("displacement")) {
                if (dp->type != "texture")
                    throw Error(ps.loc + ": \"" + dp->type + " displacement\": plymesh displacement must be a float texture");
                s.hasDisp = true;
                s.disp = *dp;
            }
            PlyMesh m;
            try {
                m = ReadPly(path);
            } catch (const Error &e) {
                throw Error(ps.loc + ": " + e.what());
            }
            // triangles become a TriangleMesh, quads a BilinearPatchMesh (scene.cpp plymesh)
            if (m.triIndices.empty() && m.quadIndices.empty()) throw Error(ps.loc + ": " + f + " has no faces");
            s.P = std::move(m.p);
            s.idx = std::move(m.triIndices);
            s.quadIdx = std::move(m.quadIndices);
            s.N = std::move(m.n);
            for (auto &t : m.uv) s.uv.insert(s.uv.end(), {t[0], t[1]});
        } else if (type == "bilinearmesh") {
            // BilinearPatch::CreateMesh (shapes.cpp:914-1003)
            s.kind = kShapeBilinearT;
            Param *P = ps.Find("P", "point3");
            if (!P) P = ps.Find("P", "point");
            if (!P || P->nums.empty() || P->nums.size() % 3)
                throw Error(ps.loc + ": Vertex positions \"P\" must be provided with bilinear patch mesh shape.");
            for (size_t i = 0; i < P->nums.size(); i += 3) s.P.push_back(V3(P->nums[i], P->nums[i + 1], P->nums[i + 2]));
            if (Param *I = ps.Find("indices", "integer")) {
                for (double v : I->nums) s.quadIdx.push_back((int)v);
                while (s.quadIdx.size() % 4) s.quadIdx.pop_back();  // "Discarding excess"
            } else if (s.P.size() == 4) {
                s.quadIdx = {0, 1, 2, 3};
            } else {
                throw Error(ps.loc + ": Vertex indices \"indices\" must be provided with bilinear patch mesh shape.");
            }
            for (int v : s.quadIdx)
                if (v < 0 || v >= (int)s.P.size())
                    throw Error(ps.loc + ": Bilinear patch mesh has out of-bounds vertex index " + std::to_string(v));
            if (Param *uv = ps.Find("uv", "point2")) {
                if (uv->nums.size() == 2 * s.P.size())
                    for (double v : uv->nums) s.uv.push_back((float)v);
            }
            Param *N = ps.Find("N", "normal");
            if (!N) N = ps.Find("N", "normal3");
            if (N && N->nums.size() == 3 * s.P.size())
                for (size_t i = 0; i < N->nums.size(); i += 3) s.N.push_back(V3(N->nums[i], N->nums[i + 1], N->nums[i + 2]));
            if (ps.Find("emissionfilename")) throw Error(ps.loc + ": \"emissionfilename\" is not supported yet");
            ps.Find("faceIndices");
        } else if (type == "sphere") {
            // Sphere::Create (shapes.cpp:75-85)
            s.kind = kShapeSphereT;
            const float radius = (float)ps.GetFloat("radius", 1.f);
            s.sp[0] = radius;
            s.sp[1] = (float)ps.GetFloat("zmin", -radius);
            s.sp[2] = (float)ps.GetFloat("zmax", radius);
            s.sp[3] = (float)ps.GetFloat("phimax", 360.f);
        } else if (type == "disk") {
            // Disk::Create (shapes.cpp:110-119)
            s.kind = kShapeDiskT;
            s.sp[0] = (float)ps.GetFloat("height", 0.);
            s.sp[1] = (float)ps.GetFloat("radius", 1);
            s.sp[2] = (float)ps.GetFloat("innerradius", 0);
            s.sp[3] = (float)ps.GetFloat("phimax", 360);
        } else if (type == "cylinder") {
            // Cylinder::Create (shapes.cpp:136-146)
            s.kind = kShapeCylinderT;
            s.sp[0] = (float)ps.GetFloat("radius", 1);
            s.sp[1] = (float)ps.GetFloat("zmin", -1);
            s.sp[2] = (float)ps.GetFloat("zmax", 1);
            s.sp[3] = (float)ps.GetFloat("phimax", 360);
        } else if (type == "loopsubdiv") {
            // Shape "loopsubdiv" (shapes.cpp:1476-1493): LoopSubdivide's limit-surface triangle
            // mesh with its vertex normals (host/subdiv.cpp)
            const int levels = ps.GetInt("levels", 3);
            Param *I = ps.Find("indices", "integer");
            if (!I || I->nums.empty()) throw Error(ps.loc + ": Vertex indices \"indices\" not provided for LoopSubdiv shape.");
            Param *P = ps.Find("P", "point3");
            if (!P) P = ps.Find("P", "point");
            if (!P || P->nums.size() < 3) throw Error(ps.loc + ": Vertex positions \"P\" not provided for LoopSubdiv shape.");
            ps.GetString("scheme", "loop");  // "don't actually use this for now"
            std::vector<int> ctrl;
            for (double v : I->nums) ctrl.push_back((int)v);
            std::vector<V3> cp;
            for (size_t i = 0; i + 2 < P->nums.size(); i += 3) cp.push_back(V3((float)P->nums[i], (float)P->nums[i + 1], (float)P->nums[i + 2]));
            try {
                LoopSubdivideMesh(levels, ctrl, cp, &s.P, &s.idx, &s.N);
            } catch (const Error &e) {
                throw Error(ps.loc + ": " + e.what());
            }
        } else if (type == "curve") {
            // the wavefront's curves: diced into a bilinear patch mesh on the host
            // (OptiXAggregate::diceCurveToBLP, gpu/aggregate.cpp:547-760, called with 5 steps
            // along the curve and 5 around it: gpu/aggregate.cpp:800-806)
            s.kind = kShapeBilinearT;
            // the reference pairs a curve's area lights (one per split Curve segment) with its
            // diced patches by index, which do not correspond: refused rather than guessed
            if (!gs.areaLightName.empty()) throw Error(ps.loc + ": area lights on curves are not supported");
            DiceCurve(ps, &s, 5, 5);
        } else {
            throw Error(ps.loc + ": shape \"" + type + "\" is not supported yet");
        }
        if (Param *a = ps.Find("alpha")) {
            if (a->type != "float" && a->type != "texture")
                throw Error(ps.loc + ": \"" + a->type + " alpha\" must be a float or a texture");
            s.alpha = *a;
            s.hasAlpha = true;
        }
        ps.CheckUnused();
        s.renderFromObject = gs.ctm;  // renderFromWorld applied at Finish
        s.flip = gs.reverseOrientation;
        s.material = gs.material;
        s.areaLight = gs.areaLightName;
        s.areaParams = gs.areaLightParams;
        s.dir = dir;
        s.insideMedium = gs.insideMedium;
        s.outsideMedium = gs.outsideMedium;
        s.loc = ps.loc;
        if (!activeInstance.empty()) {
            // BasicSceneBuilder::Shape: "Area lights not supported with object instancing"
            // (a warning; the shape is kept without emission)
            if (!s.areaLight.empty()) {
                std::fprintf(stderr, "%s: Warning: Area lights not supported with object instancing\n", ps.loc.c_str());
                s.areaLight.clear();
            }
            instanceDefs[activeInstance].push_back(std::move(s));
            return;
        }
        shapes.push_back(std::move(s));
    }

    // Sphere / Disk constructors (shapes.h:117-128, 407-417) in render space: affine
    // renderFromObject and its inverse as float matrices; the shape's area light (its own
    // DiffuseAreaLight, lights.cpp:941-966 with Shape::Area) in shape order
    template <typename MediumOf>
    void AnalyticShape(const PendingShape &s, const Mat4 &rfo, int mat, int lightSpectrum, float lightScale,
                       bool twoSided, float power, const MediumOf &mediumOf) {
        if (rfo[3][0] != 0 || rfo[3][1] != 0 || rfo[3][2] != 0 || rfo[3][3] != 1)
            throw Error(s.loc + ": projective transforms of spheres and disks are not supported");
        const Mat4 ofr = Inverse4(rfo);
        AnalyticShapeDesc a;
        DeviceShape &d = a.dev;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 4; ++j) {
                d.o2r[4 * i + j] = (float)rfo[i][j];
                d.r2o[4 * i + j] = (float)ofr[i][j];
            }
        d.kind = s.kind;
        d.flags = (s.flip ? 1 : 0) | (SwapsHandedness(rfo) ? 2 : 0);
        auto radians = [](float deg) { return (kPi / 180) * deg; };
        if (s.kind == kShapeSphereT) {
            const float radius = s.sp[0], zMin = s.sp[1], zMax = s.sp[2], phiMax = s.sp[3];
            d.a = radius;
            d.b = Clampf(std::min(zMin, zMax), -radius, radius);
            d.c = Clampf(std::max(zMin, zMax), -radius, radius);
            d.e = std::acos(Clampf(std::min(zMin, zMax) / radius, -1, 1));
            d.f = std::acos(Clampf(std::max(zMin, zMax) / radius, -1, 1));
            d.d = radians(Clampf(phiMax, 0, 360));
        } else if (s.kind == kShapeCylinderT) {  // Cylinder ctor (shapes.h:580-590)
            d.a = s.sp[0];
            d.b = std::min(s.sp[1], s.sp[2]);
            d.c = std::max(s.sp[1], s.sp[2]);
            d.d = radians(Clampf(s.sp[3], 0, 360));
        } else {
            d.a = s.sp[0];
            d.b = s.sp[1];
            d.c = s.sp[2];
            d.d = radians(Clampf(s.sp[3], 0, 360));
        }
        a.material = mat;
        a.alpha = AlphaId(s);
        if (!scene.media.empty()) {
            a.medium[0] = (int16_t)mediumOf(s.insideMedium, s.loc);
            a.medium[1] = (int16_t)mediumOf(s.outsideMedium, s.loc);
        }
        if (lightSpectrum >= 0) {
            AreaLightDesc l;
                SetSpread(&l);
            l.shape = (int)scene.shapes.size();
            l.spectrum = lightSpectrum;
            l.scale = lightScale;
            l.twoSided = twoSided;
            l.area = ShapeArea(d);
            if (power > 0) {
                float k_e = curImageKe;  // an image emitter's mean luminance, else 1
                k_e *= (twoSided ? 2 : 1) * l.area * kPi;
                l.scale *= power / k_e;
            }
            a.light = (int)scene.areaLights.size();
            scene.areaLights.push_back(l);
        }
        scene.shapes.push_back(a);
    }

    // BilinearPatchMesh ctor (util/mesh.cpp: render-space P, N through renderFromObject and
    // negated under ReverseOrientation) and one BilinearPatch per quad (shapes.cpp:1041-1071:
    // IsRectangle, area); each emissive patch is its own DiffuseAreaLight
    template <typename MediumOf>
    void BilinearPatches(const PendingShape &s, const Mat4 &rfo, int mat, int lightSpectrum, float lightScale,
                         bool twoSided, float power, const MediumOf &mediumOf, int base) {
        const Mat4 inv = Inverse4(rfo);
        const bool swaps = SwapsHandedness(rfo);
        for (size_t q = 0; q + 3 < s.quadIdx.size(); q += 4) {
            AnalyticShapeDesc a;
            DeviceShape &d = a.dev;
            d.kind = kShapeBilinearT;
            d.flags = (s.flip ? 1 : 0) | (swaps ? 2 : 0) | (s.uv.empty() ? 0 : 4) | (s.N.empty() ? 0 : 8);
            V3 pv[4];
            for (int k = 0; k < 4; ++k) {
                const int vi = s.quadIdx[q + k];
                pv[k] = scene.verts[base + vi];  // render space (pushed by the mesh pass)
                for (int j = 0; j < 3; ++j) d.r2o[3 * k + j] = pv[k][j];
                if (!s.uv.empty()) {
                    d.o2r[2 * k] = s.uv[2 * vi];
                    d.o2r[2 * k + 1] = s.uv[2 * vi + 1];
                }
                if (!s.N.empty()) {
                    V3 nn = XformNormal(inv, s.N[vi]);
                    if (s.flip) nn = -nn;
                    for (int j = 0; j < 3; ++j) a.normals[3 * k + j] = nn[j];
                }
            }
            const V3 p00 = pv[0], p10 = pv[1], p01 = pv[2], p11 = pv[3];
            bool rect = !(p00 == p01 || p01 == p11 || p11 == p10 || p10 == p00);
            if (rect) {
                const V3 n = Normalize(Cross(p10 - p00, p01 - p00));
                if (AbsDotN(n, Normalize(p11 - p00)) > 1e-5f) rect = false;
            }
            if (rect) {
                const V3 pCenter = (p00 + p01 + p10 + p11) / 4;
                const float d2[4] = {DistanceSquared(p00, pCenter), DistanceSquared(p01, pCenter),
                                     DistanceSquared(p10, pCenter), DistanceSquared(p11, pCenter)};
                for (int i = 1; i < 4; ++i)
                    if (std::abs(d2[i] - d2[0]) / d2[0] > 1e-4f) rect = false;
            }
            float area = 0;
            if (rect) {
                area = Distance(p00, p01) * Distance(p00, p10);
            } else {
                V3 g[4][4];
                for (int i = 0; i <= 3; ++i)
                    for (int j = 0; j <= 3; ++j) {
                        const float u = float(i) / float(3), v = float(j) / float(3);
                        g[i][j] = LerpV(u, LerpV(v, p00, p01), LerpV(v, p10, p11));
                    }
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j)
                        area += 0.5f * Length(Cross(g[i + 1][j + 1] - g[i][j], g[i + 1][j] - g[i][j + 1]));
            }
            d.a = area;
            d.b = rect ? 1.f : 0.f;
            a.material = mat;
            a.alpha = AlphaId(s);
            if (!scene.media.empty()) {
                a.medium[0] = (int16_t)mediumOf(s.insideMedium, s.loc);
                a.medium[1] = (int16_t)mediumOf(s.outsideMedium, s.loc);
            }
            if (lightSpectrum >= 0) {
                AreaLightDesc l;
                SetSpread(&l);
                l.shape = (int)scene.shapes.size();
                l.spectrum = lightSpectrum;
                l.scale = lightScale;
                l.twoSided = twoSided;
                l.area = area;
                if (power > 0) {
                    float k_e = curImageKe;  // an image emitter's mean luminance, else 1
                    k_e *= (twoSided ? 2 : 1) * l.area * kPi;
                    l.scale *= power / k_e;
                }
                a.light = (int)scene.areaLights.size();
                scene.areaLights.push_back(l);
            }
            scene.shapes.push_back(a);
        }
    }

    // ObjectInstance: renderFromInstance = RenderFromObject() * worldFromRender (scene.cpp:392),
    // applied to each definition shape's renderFromObject, i.e. the shape's world-from-object
    // becomes worldFromInstance * worldFromObject.  The instances are flattened into the
    // triangle list (one BVH over every instance's triangles).
    void ResolveInstances() {
        if (!activeInstance.empty()) throw Error("End of files inside ObjectBegin \"" + activeInstance + "\"");
        for (const InstanceUse &u : instanceUses) {
            auto it = instanceDefs.find(u.name);
            if (it == instanceDefs.end()) throw Error(u.loc + ": " + u.name + ": object instance not defined");
            for (const PendingShape &d : it->second) {
                PendingShape c = d;
                c.renderFromObject = Mul(u.worldFromInstance, d.renderFromObject);
                shapes.push_back(std::move(c));
            }
        }
    }
};

static std::array<float, 311> DensePiecewiseLinear(const std::vector<double> &nums, const std::string &loc) {
    if (nums.size() % 2) throw Error(loc + ": odd number of values in spectrum");
    std::vector<float> lam, val;
    for (size_t i = 0; i < nums.size(); i += 2) {
        if (!lam.empty() && (float)nums[i] <= lam.back()) throw Error(loc + ": spectrum wavelengths not increasing");
        lam.push_back((float)nums[i]);
        val.push_back((float)nums[i + 1]);
    }
    std::array<float, 311> out;
    for (int l = 395; l <= 705; ++l) {
        float lambda = (float)l;
        float v = 0;
        if (!(lambda < lam.front() || lambda > lam.back())) {
            size_t o = 0;
            while (o + 2 < lam.size() && lam[o + 1] <= lambda) ++o;
            if (lam.size() == 1)
                v = val[0];
            else {
                float t = (lambda - lam[o]) / (lam[o + 1] - lam[o]);
                v = Lerpf(t, val[o], val[o + 1]);
            }
        }
        out[l - 395] = v;
    }
    return out;
}

static float PhotometricOf(const std::array<float, 311> &dense) {
    // SpectrumToPhotometric (util/spectrum.cpp:37-51) over the dense samples
    const SpectralData &d = GetSpectralData();
    float y = 0;
    for (float lambda = kLambdaMin; lambda <= kLambdaMax; ++lambda)
        y += d.denseY[DenseOffset(lambda)] * dense[DenseOffset(lambda)];
    return y;
}

// A spectrum parameter as a DenselySampledSpectrum (395..705 nm), scaled.  Unbounded: rgb ->
// RGBUnboundedSpectrum; Illuminant: rgb -> RGBIlluminantSpectrum; either: "spectrum" as
// inline lambda/value pairs (PiecewiseLinearSpectrum).  *photometric gets SpectrumToPhotometric
// of the unscaled spectrum (illuminant part for rgb, util/spectrum.cpp:37-51).
// GridMedium's MajorantGrid (media.h:124-160, media.cpp:239-246): per 16^3 voxel of the
// medium's [0,1]^3, SampledGrid::MaxValue of the density (util/containers.h:838-854)
static void BuildMajorantGrid(MediumDesc &m) {
    const int R = 16;
    m.majorant.assign(R * R * R, 0.f);
    auto lookup = [&](int x, int y, int z) -> float {
        if (x < 0 || x >= m.nx || y < 0 || y >= m.ny || z < 0 || z >= m.nz) return 0.f;
        return m.density[((size_t)z * m.ny + y) * m.nx + x];
    };
    for (int z = 0; z < R; ++z)
        for (int y = 0; y < R; ++y)
            for (int x = 0; x < R; ++x) {
                const float b0[3] = {float(x) / R, float(y) / R, float(z) / R};
                const float b1[3] = {float(x + 1) / R, float(y + 1) / R, float(z + 1) / R};
                const int n[3] = {m.nx, m.ny, m.nz};
                int lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::max((int)std::floor(b0[a] * n[a] - .5f), 0);
                    hi[a] = std::min((int)std::floor(b1[a] * n[a] - .5f) + 1, n[a] - 1);
                }
                float v = lookup(lo[0], lo[1], lo[2]);
                for (int zz = lo[2]; zz <= hi[2]; ++zz)
                    for (int yy = lo[1]; yy <= hi[1]; ++yy)
                        for (int xx = lo[0]; xx <= hi[0]; ++xx) v = std::max(v, lookup(xx, yy, zz));
                m.majorant[x + R * (y + R * z)] = v;
            }
}

// RGBGridMedium::Create (media.cpp:382-452) and its constructor's majorant grid (:339-380):
// per voxel RGBUnboundedSpectrum / RGBIlluminantSpectrum(sRGB, rgb) as {c0, c1, c2, scale}
// (scale = 2 max(r, g, b), coefficients of rgb / scale); majorant voxel = sigmaScale *
// (max of sigma_a's MaxValue, or 1 without sigma_a) + (the same for sigma_s).
static void BuildRGBGridMedium(ParamSet &ps, MediumDesc &m) {
    m.type = kMediumRGBGrid;
    auto rgbArray = [&](const char *name) {
        std::vector<float> v;
        if (Param *p = ps.Find(name)) {
            if (p->type != "rgb" || p->nums.size() % 3)
                throw Error(ps.loc + ": \"" + name + "\" of an RGB grid medium must be \"rgb\" values");
            for (double x : p->nums) v.push_back((float)x);
        }
        return v;
    };
    const std::vector<float> grids[3] = {rgbArray("sigma_a"), rgbArray("sigma_s"), rgbArray("Le")};
    const std::vector<float> &a = grids[0], &s = grids[1], &le = grids[2];
    if (a.empty() && s.empty())
        throw Error(ps.loc + ": RGB grid requires \"sigma_a\" and/or \"sigma_s\" parameter values.");
    const size_t n = (a.empty() ? s.size() : a.size()) / 3;
    if (!a.empty() && !s.empty() && a.size() != s.size())
        throw Error(ps.loc + ": Different number of samples (" + std::to_string(n) + " vs " +
                    std::to_string(s.size() / 3) + ") provided for \"sigma_a\" and \"sigma_s\".");
    if (!le.empty() && a.empty()) throw Error(ps.loc + ": RGB grid requires \"sigma_a\" if \"Le\" value provided.");
    if (!le.empty() && le.size() / 3 != n)
        throw Error(ps.loc + ": Expected " + std::to_string(n) + " values for \"Le\" parameter but were given " +
                    std::to_string(le.size() / 3) + ".");
    m.nx = ps.GetInt("nx", 1);
    m.ny = ps.GetInt("ny", 1);
    m.nz = ps.GetInt("nz", 1);
    if ((long)n != (long)m.nx * m.ny * m.nz)
        throw Error(ps.loc + ": RGB grid medium has " + std::to_string(n) + " density values; expected nx*ny*nz = " +
                    std::to_string((long)m.nx * m.ny * m.nz));
    m.density.assign(12 * n, 0.f);
    m.rgbGrids = 0;
    for (int k = 0; k < 3; ++k) {
        if (grids[k].empty()) continue;
        m.rgbGrids |= 1 << k;
        for (size_t i = 0; i < n; ++i) {
            const float r = grids[k][3 * i], g = grids[k][3 * i + 1], b = grids[k][3 * i + 2];
            if (r < 0 || g < 0 || b < 0) throw Error(ps.loc + ": RGB grid medium value has a negative component.");
            const float scale = 2 * std::max({r, g, b});
            const std::array<float, 3> c = scale ? RGBToSigmoidCoeffs(r / scale, g / scale, b / scale, ps.colorSpace)
                                                 : RGBToSigmoidCoeffs(0, 0, 0, ps.colorSpace);
            float *d = &m.density[(size_t)k * 4 * n + 4 * i];
            d[0] = c[0], d[1] = c[1], d[2] = c[2], d[3] = scale;
        }
    }
    if (Param *p0 = ps.Find("p0", "point3")) m.p0 = V3((float)p0->nums[0], (float)p0->nums[1], (float)p0->nums[2]);
    if (Param *p1 = ps.Find("p1", "point3")) m.p1 = V3((float)p1->nums[0], (float)p1->nums[1], (float)p1->nums[2]);
    const float LeScale = (float)ps.GetFloat("Lescale", 1);
    m.g = (float)ps.GetFloat("g", 0);
    m.sigmaScale = (float)ps.GetFloat("scale", 1);
    m.LeScale = {LeScale};
    m.emissive = !le.empty() && LeScale > 0;  // IsEmissive
    // RGBSigmoidPolynomial::MaxValue (util/color.h:346-352) times the voxel's scale
    auto maxOf = [&](int k, size_t i) {
        const float *c = &m.density[(size_t)k * 4 * n + 4 * i];
        auto f = [&](float l) { return SigmoidPolynomial(c[0], c[1], c[2], l); };
        float r = std::max(f(360), f(830));
        const float lambda = -c[1] / (2 * c[0]);
        if (lambda >= 360 && lambda <= 830) r = std::max(r, f(lambda));
        return c[3] * r;
    };
    const int R = 16, nn[3] = {m.nx, m.ny, m.nz};  // MajorantGrid res {16, 16, 16}
    m.majorant.assign(R * R * R, 0.f);
    for (int z = 0; z < R; ++z)
        for (int y = 0; y < R; ++y)
            for (int x = 0; x < R; ++x) {
                const float b0[3] = {float(x) / R, float(y) / R, float(z) / R};
                const float b1[3] = {float(x + 1) / R, float(y + 1) / R, float(z + 1) / R};
                int lo[3], hi[3];
                for (int ax = 0; ax < 3; ++ax) {
                    lo[ax] = std::max((int)std::floor(b0[ax] * nn[ax] - .5f), 0);
                    hi[ax] = std::min((int)std::floor(b1[ax] * nn[ax] - .5f) + 1, nn[ax] - 1);
                }
                // SampledGrid::MaxValue (util/containers.h:838-854)
                auto gridMax = [&](int k) {
                    float v = maxOf(k, ((size_t)lo[2] * m.ny + lo[1]) * m.nx + lo[0]);
                    for (int zz = lo[2]; zz <= hi[2]; ++zz)
                        for (int yy = lo[1]; yy <= hi[1]; ++yy)
                            for (int xx = lo[0]; xx <= hi[0]; ++xx)
                                v = std::max(v, maxOf(k, ((size_t)zz * m.ny + yy) * m.nx + xx));
                    return v;
                };
                const float maxSigmaT = (a.empty() ? 1.f : gridMax(0)) + (s.empty() ? 1.f : gridMax(1));
                m.majorant[x + R * (y + R * z)] = m.sigmaScale * maxSigmaT;
            }
}

static std::array<float, 311> MediumSpectrum(ParamSet &ps, const char *name, bool illuminant, float defaultValue,
                                             bool *given, float *photometric) {
    Param *p = ps.Find(name);
    std::array<float, 311> d;
    *given = p != nullptr;
    if (photometric) *photometric = 1;
    if (!p) {
        d.fill(defaultValue);
        return d;
    }
    if (p->type == "rgb" && p->nums.size() == 3) {
        float r = (float)p->nums[0], g = (float)p->nums[1], b = (float)p->nums[2];
        if (r < 0 || g < 0 || b < 0) throw Error(ps.loc + ": RGB parameter \"" + std::string(name) + "\" has negative component.");
        if (illuminant) {
            d = DenseRGBIlluminant(r, g, b, p->colorSpace);
            if (photometric) *photometric = GetColorSpace(p->colorSpace).photometric;
        } else {
            d = DenseRGBUnbounded(r, g, b, p->colorSpace);
        }
        return d;
    }
    if (p->type == "spectrum" && !p->nums.empty()) {
        d = DensePiecewiseLinear(p->nums, ps.loc);
        if (photometric) *photometric = PhotometricOf(d);
        return d;
    }
    if (p->type == "blackbody" && p->nums.size() == 1) {
        // BlackbodySpectrum(T), normalised to 1 at its peak (util/spectrum.h:530-560)
        const float T = (float)p->nums[0];
        for (int i = 0; i < 311; ++i) d[i] = BlackbodyNormalized(395.f + i, T);
        if (photometric) *photometric = PhotometricOf(d);
        return d;
    }
    throw Error(ps.loc + ": \"" + p->type + " " + name + "\" is not supported for media yet (use rgb, spectrum or blackbody)");
}

void Parser::Finish() {
    if (!haveCamera) {
        cameraFromWorld = Identity4();
    }
    // ---- film (film.cpp FilmBaseParameters)
    if (filmType != "rgb") throw Error(filmParams.loc + ": film \"" + filmType + "\" not supported (rgb only)");
    scene.xres = filmParams.GetInt("xresolution", 1280);
    scene.yres = filmParams.GetInt("yresolution", 720);
    if (overrides.count("xresolution")) scene.xres = std::stoi(overrides.at("xresolution"));
    if (overrides.count("yresolution")) scene.yres = std::stoi(overrides.at("yresolution"));
    scene.outFile = filmParams.GetString("filename", "pbrt.exr");
    {
        Param *pb = filmParams.Find("pixelbounds", "integer");
        Param *cw = filmParams.Find("cropwindow", "float");
        scene.px0 = 0;
        scene.px1 = scene.xres;
        scene.py0 = 0;
        scene.py1 = scene.yres;
        if (pb && pb->nums.size() == 4) {
            scene.px0 = (int)pb->nums[0];
            scene.px1 = (int)pb->nums[1];
            scene.py0 = (int)pb->nums[2];
            scene.py1 = (int)pb->nums[3];
        } else if (cw && cw->nums.size() == 4) {
            scene.px0 = (int)std::ceil(scene.xres * cw->nums[0]);
            scene.px1 = (int)std::ceil(scene.xres * cw->nums[1]);
            scene.py0 = (int)std::ceil(scene.yres * cw->nums[2]);
            scene.py1 = (int)std::ceil(scene.yres * cw->nums[3]);
        }
        if (overrides.count("pixelbounds")) {
            int v[4];
            std::istringstream is(overrides.at("pixelbounds"));
            char c;
            is >> v[0] >> c >> v[1] >> c >> v[2] >> c >> v[3];
            scene.px0 = v[0];
            scene.px1 = v[1];
            scene.py0 = v[2];
            scene.py1 = v[3];
        }
        double iso = filmParams.GetFloat("iso", 100.);
        // PixelSensor::Create (film.cpp:222-262) and RGBFilm's clamp (film.cpp:585)
        scene.sensorName = filmParams.GetString("sensor", "cie1931");
        scene.whiteBalance = (float)filmParams.GetFloat("whitebalance", 0);
        scene.maxComponentValue = (float)filmParams.GetFloat("maxcomponentvalue", kInfinity);
        filmParams.Find("savefp16");
        filmParams.Find("diagonal");
        double exposure = cameraParams.GetFloat("shutterclose", 1.0) - cameraParams.GetFloat("shutteropen", 0.0);
        scene.imagingRatio = (float)(exposure * iso / 100);
        filmParams.CheckUnused();
    }
    // ---- sampler
    scene.spp = samplerParams.GetInt("pixelsamples", 16);
    // the sampler's "seed" defaults to Options->seed (samplers.cpp:73 etc.): --seed (the "seed"
    // override), replaced by a scene's Option "seed" (scene.cpp:543-544), which is parsed later
    {
        int optionsSeed = overrides.count("seed") ? std::stoi(overrides.at("seed")) : 0;
        if (optionSeedSet) optionsSeed = optionSeed;
        scene.seed = samplerParams.GetInt("seed", optionsSeed);
    }
    if (overrides.count("spp")) scene.spp = std::stoi(overrides.at("spp"));
    if (scene.samplerName == "halton") {
        scene.samplerType = 0;
        if (samplerParams.GetString("randomization", "permutedigits") != "permutedigits")
            throw Error(samplerParams.loc + ": halton: only permutedigits randomization is supported");
    } else if (scene.samplerName == "zsobol" || scene.samplerName == "sobol" || scene.samplerName == "paddedsobol") {
        // samplers.cpp:108-130, 146-170, 258-295 (PaddedSobol / ZSobol / SobolSampler::Create):
        // default randomization fastowen
        scene.samplerType = scene.samplerName == "zsobol" ? kSamplerZSobol
                            : scene.samplerName == "sobol" ? kSamplerSobol : kSamplerPaddedSobol;
        std::string r = samplerParams.GetString("randomization", "fastowen");
        if (r == "none") scene.zsRandomize = 0;
        else if (r == "permutedigits") scene.zsRandomize = 1;
        else if (r == "fastowen") scene.zsRandomize = 2;
        else if (r == "owen") scene.zsRandomize = 3;
        else {
            const char *cls = scene.samplerType == kSamplerZSobol ? "ZSobolSampler"
                              : scene.samplerType == kSamplerSobol ? "SobolSampler" : "PaddedSobolSampler";
            throw Error(samplerParams.loc + ": unknown randomization strategy \"" + r + "\" given to " + cls);
        }
    } else if (scene.samplerName == "independent") {
        // samplers.cpp:240-247 (IndependentSampler::Create): 4 pixel samples by default
        scene.samplerType = kSamplerIndependent;
        scene.spp = samplerParams.GetInt("pixelsamples", 4);
        if (overrides.count("spp")) scene.spp = std::stoi(overrides.at("spp"));
    } else if (scene.samplerName == "stratified") {
        // samplers.cpp:297-320 (StratifiedSampler::Create): xsamples x ysamples strata, jittered
        // by default; a pixel-sample override is factored into the two counts
        scene.samplerType = kSamplerStratified;
        scene.stratJitter = samplerParams.GetBool("jitter", true) ? 1 : 0;
        scene.stratXs = samplerParams.GetInt("xsamples", 4);
        scene.stratYs = samplerParams.GetInt("ysamples", 4);
        if (overrides.count("spp")) {
            const int n = std::stoi(overrides.at("spp"));
            int div = (int)std::sqrt((double)n);
            while (div > 0 && n % div) --div;
            if (div <= 0) throw Error("stratified: cannot factor " + std::to_string(n) + " pixel samples");
            scene.stratXs = n / div;
            scene.stratYs = n / scene.stratXs;
        }
        if (scene.stratXs <= 0 || scene.stratYs <= 0)
            throw Error(samplerParams.loc + ": stratified: xsamples and ysamples must be positive");
        scene.spp = scene.stratXs * scene.stratYs;
    } else if (scene.samplerName == "pmj02bn") {
        throw Error(samplerParams.loc + ": sampler \"pmj02bn\" not supported (its PMJ02BN tables are not part of "
                                        "this build); use halton, zsobol, sobol, paddedsobol, independent or stratified");
    } else {
        throw Error(samplerParams.loc + ": unknown sampler \"" + scene.samplerName + "\"");
    }
    samplerParams.CheckUnused();
    // ---- integrator
    scene.maxDepth = integratorParams.GetInt("maxdepth", 5);
    if (overrides.count("maxdepth")) scene.maxDepth = std::stoi(overrides.at("maxdepth"));
    scene.regularize = integratorParams.GetBool("regularize", false);
    std::string ls = integratorParams.GetString("lightsampler", "bvh");
    if (ls != "bvh" && ls != "uniform") throw Error(integratorParams.loc + ": lightsampler " + ls + " not supported");
    if (ls == "uniform") scene.uniformLightSampler = true;
    // ---- filter
    // Filter::Create (filters.cpp:26-130): box 0.5, gaussian 1.5 / sigma 0.5, mitchell 2 / B = C
    // = 1/3, sinc 4 / tau 3, triangle 2
    {
        const std::string &fn = scene.filterName;
        float r = 0.5f;
        if (fn == "box") scene.filterType = kFilterBox, r = 0.5f;
        else if (fn == "gaussian") scene.filterType = kFilterGaussian, r = 1.5f;
        else if (fn == "mitchell") scene.filterType = kFilterMitchell, r = 2.f;
        else if (fn == "sinc") scene.filterType = kFilterSinc, r = 4.f;
        else if (fn == "triangle") scene.filterType = kFilterTriangle, r = 2.f;
        else throw Error(filterParams.loc + ": " + fn + ": filter type unknown.");
        scene.filterRadiusX = (float)filterParams.GetFloat("xradius", r);
        scene.filterRadiusY = (float)filterParams.GetFloat("yradius", r);
        if (fn == "gaussian") scene.filterA = (float)filterParams.GetFloat("sigma", 0.5);
        if (fn == "mitchell") {
            scene.filterA = (float)filterParams.GetFloat("B", 1. / 3.);
            scene.filterB = (float)filterParams.GetFloat("C", 1. / 3.);
        }
        if (fn == "sinc") scene.filterA = (float)filterParams.GetFloat("tau", 3.);
        filterParams.CheckUnused();
        BuildFilterTable(scene);
    }

    // ---- camera (cameras.cpp:43-73, 266-285, 543-600) in cameraworld rendering space
    if (cameraType != "perspective") throw Error(cameraParams.loc + ": camera \"" + cameraType + "\" not supported");
    {
        Mat4 worldFromCamera = Inverse4(cameraFromWorld);
        V3 pCam = XformPoint(worldFromCamera, V3(0, 0, 0));
        // CameraTransform (cameras.cpp:43-73): Option "rendercoordsys" picks the rendering space
        Mat4 renderFromWorld = renderSpace == kRenderCamera  ? cameraFromWorld
                               : renderSpace == kRenderWorld ? Identity4()
                                                             : TranslateM(-(double)pCam.x, -(double)pCam.y, -(double)pCam.z);
        scene.camera.renderFromWorld = renderFromWorld;
        scene.camera.renderFromCamera = Mul(renderFromWorld, worldFromCamera);
        double frame = cameraParams.GetFloat("frameaspectratio", double((float)scene.xres / (float)scene.yres));
        double sx0, sx1, sy0, sy1;
        if (frame > 1.) {
            sx0 = -frame;
            sx1 = frame;
            sy0 = -1;
            sy1 = 1;
        } else {
            sx0 = -1;
            sx1 = 1;
            sy0 = -1 / frame;
            sy1 = 1 / frame;
        }
        if (Param *sw = cameraParams.Find("screenwindow", "float")) {
            if (sw->nums.size() != 4) throw Error(cameraParams.loc + ": screenwindow needs 4 values");
            sx0 = sw->nums[0];
            sx1 = sw->nums[1];
            sy0 = sw->nums[2];
            sy1 = sw->nums[3];
        }
        double fov = cameraParams.GetFloat("fov", 90.);
        scene.camera.fov = (float)fov;
        scene.camera.lensRadius = (float)cameraParams.GetFloat("lensradius", 0.);
        scene.camera.focalDistance = (float)cameraParams.GetFloat("focaldistance", 1e6);
        scene.camera.shutterOpen = (float)cameraParams.GetFloat("shutteropen", 0.);
        scene.camera.shutterClose = (float)cameraParams.GetFloat("shutterclose", 1.);
        Mat4 screenFromCamera = PerspectiveM(fov, 1e-2, 1000.);
        Mat4 NDCFromScreen = Mul(ScaleM(1 / (sx1 - sx0), 1 / (sy1 - sy0), 1), TranslateM(-sx0, -sy1, 0));
        Mat4 rasterFromNDC = ScaleM(scene.xres, -scene.yres, 1);
        Mat4 rasterFromScreen = Mul(rasterFromNDC, NDCFromScreen);
        scene.camera.cameraFromRaster = Mul(Inverse4(screenFromCamera), Inverse4(rasterFromScreen));
        cameraParams.CheckUnused();
    }
    // ---- textures of the materials (render space is known now)
    ResolveTextures();
    // ---- sensor / output colour space
    {
        // RGBFilm: outputRGBFromSensorRGB = colorSpace->RGBFromXYZ * sensor->XYZFromSensorRGB
        const ColorSpaceDesc &sd = GetColorSpace(filmParams.colorSpace);
        scene.filmColorSpace = filmParams.colorSpace;
        PixelSensorDesc ps;
        try {
            ps = BuildPixelSensor(scene.sensorName, scene.whiteBalance, filmParams.colorSpace);
        } catch (const Error &e) {
            throw Error(filmParams.loc + ": " + e.what());
        }
        scene.sensorX = ps.r;
        scene.sensorY = ps.g;
        scene.sensorZ = ps.b;
        // film.cpp:505: the float SquareMatrix<3> product, one compensated dot per entry
        float out[3][3];
        MulCompensated3(sd.rgbFromXYZf, ps.xyzFromSensorRGB, out);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                scene.xyzFromSensorRGB[i][j] = ps.xyzFromSensorRGB[i][j];
                scene.outputRGBFromSensorRGB[i][j] = out[i][j];
            }
    }
    // ---- media (MakeNamedMedium -> HomogeneousMedium / GridMedium, media.cpp:167-330)
    std::map<std::string, int> mediumIndex;
    for (PendingMedium &pm : pendingMedia) {
        ParamSet &ps = pm.params;
        MediumDesc m;
        m.name = pm.name;
        // HomogeneousMedium::Create's "preset" (media.cpp:170-186, GetMediumScatteringProperties):
        // sigma_a and sigma_s from the named measurement (RGBUnboundedSpectrum of sRGB), else a
        // warning and the parameters; the other media have no "preset" parameter
        const std::string preset = ps.GetString("preset", "");
        const std::array<float, 6> *presetVals = nullptr;
        if (!preset.empty()) {
            if (pm.type != "homogeneous")
                throw Error(ps.loc + ": \"string preset\": unused parameter (only homogeneous media take a preset)");
            auto it = GetSpectralData().mediumPresets.find(preset);
            if (it == GetSpectralData().mediumPresets.end())
                std::fprintf(stderr, "%s: Warning: Material preset \"%s\" not found.\n", ps.loc.c_str(), preset.c_str());
            else
                presetVals = &it->second;
        }
        if (pm.type == "cloud") {
            // CloudMedium::Create (media.cpp:462-484): no scale or Le; sigma_a / sigma_s default 1
            m.type = kMediumCloud;
            bool given;
            auto addDense = [&](const std::array<float, 311> &d) {
                scene.denseSpectra.push_back(d);
                return (int)scene.denseSpectra.size() - 1;
            };
            m.sigmaA = addDense(MediumSpectrum(ps, "sigma_a", false, 1.f, &given, nullptr));
            m.sigmaS = addDense(MediumSpectrum(ps, "sigma_s", false, 1.f, &given, nullptr));
            std::array<float, 311> zero{};
            m.Le = addDense(zero);
            m.g = (float)ps.GetFloat("g", 0);
            m.density = {(float)ps.GetFloat("density", 1), (float)ps.GetFloat("wispiness", 1),
                         (float)ps.GetFloat("frequency", 5)};
            const auto &perm = GetSpectralData().noisePerm;
            if (perm.size() != 512) throw Error("spectral data lacks the noise permutation (NoisePerm)");
            m.density.insert(m.density.end(), perm.begin(), perm.end());
            Param *p0 = ps.Find("p0", "point3"), *p1 = ps.Find("p1", "point3");
            if (p0) m.p0 = V3((float)p0->nums[0], (float)p0->nums[1], (float)p0->nums[2]);
            if (p1) m.p1 = V3((float)p1->nums[0], (float)p1->nums[1], (float)p1->nums[2]);
            m.renderFromMedium = Mul(scene.camera.renderFromWorld, pm.worldFromMedium);
            ps.Find("type");
            ps.CheckUnused();
            mediumIndex[pm.name] = (int)scene.media.size();
            scene.media.push_back(std::move(m));
            continue;
        }
        if (pm.type == "rgbgrid") {
            BuildRGBGridMedium(ps, m);
            m.renderFromMedium = Mul(scene.camera.renderFromWorld, pm.worldFromMedium);
            // SampleT_maj's sigma_t is SampledSpectrum(1) (media.h:411-414): sigma_a "ones",
            // sigma_s zero; Le is the colour space's illuminant (RGBIlluminantSpectrum)
            std::array<float, 311> ones, zero{};
            ones.fill(1.f);
            scene.denseSpectra.push_back(ones);
            m.sigmaA = (int)scene.denseSpectra.size() - 1;
            scene.denseSpectra.push_back(zero);
            m.sigmaS = (int)scene.denseSpectra.size() - 1;
            scene.denseSpectra.push_back(GetColorSpace(ps.colorSpace).illuminant);
            m.Le = (int)scene.denseSpectra.size() - 1;
            ps.Find("type");
            ps.CheckUnused();
            mediumIndex[pm.name] = (int)scene.media.size();
            scene.media.push_back(std::move(m));
            continue;
        }
        bool given;
        float scale = (float)ps.GetFloat("scale", 1);
        auto addDense = [&](std::array<float, 311> d, float k) {
            for (float &v : d) v *= k;  // DenselySampledSpectrum::Scale
            scene.denseSpectra.push_back(d);
            return (int)scene.denseSpectra.size() - 1;
        };
        if (presetVals) {
            const std::array<float, 6> &pv = *presetVals;
            m.sigmaA = addDense(DenseRGBUnbounded(pv[3], pv[4], pv[5]), scale);
            m.sigmaS = addDense(DenseRGBUnbounded(pv[0], pv[1], pv[2]), scale);
        } else {
            m.sigmaA = addDense(MediumSpectrum(ps, "sigma_a", false, 1.f, &given, nullptr), scale);
            m.sigmaS = addDense(MediumSpectrum(ps, "sigma_s", false, 1.f, &given, nullptr), scale);
        }
        m.g = (float)ps.GetFloat("g", 0);
        float photometric = 1;
        std::array<float, 311> Le = MediumSpectrum(ps, "Le", true, 0.f, &given, &photometric);
        const bool LeZero = !given || *std::max_element(Le.begin(), Le.end()) == 0;
        if (LeZero) Le.fill(0.f);
        if (pm.type == "homogeneous") {
            m.type = kMediumHomogeneous;
            float LeScale = (float)ps.GetFloat("Lescale", 1);
            if (!LeZero) LeScale /= photometric;
            m.Le = addDense(Le, LeScale);
            const auto &LeD = scene.denseSpectra[m.Le];
            m.emissive = *std::max_element(LeD.begin(), LeD.end()) > 0;  // IsEmissive
        } else if (pm.type == "uniformgrid") {
            m.type = kMediumGrid;
            Param *dens = ps.Find("density", "float");
            if (!dens || dens->nums.empty()) throw Error(ps.loc + ": No \"density\" value provided for grid medium.");
            Param *temp = ps.Find("temperature", "float");
            if (temp && !temp->nums.empty()) {
                if (temp->nums.size() != dens->nums.size())
                    throw Error(ps.loc + ": Different number of samples (" + std::to_string(dens->nums.size()) + " vs " +
                                std::to_string(temp->nums.size()) + ") provided for \"density\" and \"temperature\".");
                if (ps.Find("Le")) throw Error(ps.loc + ": Both \"Le\" and \"temperature\" values were provided.");
                for (double v : temp->nums) m.temperature.push_back((float)v);
            }
            // "temperatureoffset" defaults to "temperaturecutoff" (media.cpp:320-322)
            m.temperatureOffset = (float)ps.GetFloat("temperatureoffset", ps.GetFloat("temperaturecutoff", 0));
            m.temperatureScale = (float)ps.GetFloat("temperaturescale", 1);
            m.nx = ps.GetInt("nx", 1);
            m.ny = ps.GetInt("ny", 1);
            m.nz = ps.GetInt("nz", 1);
            if ((long)dens->nums.size() != (long)m.nx * m.ny * m.nz)
                throw Error(ps.loc + ": Grid medium has " + std::to_string(dens->nums.size()) +
                            " density values; expected nx*ny*nz = " + std::to_string(m.nx * m.ny * m.nz));
            for (double v : dens->nums) m.density.push_back((float)v);
            const float LeNorm = LeZero ? 1.f : 1 / photometric;
            Param *ls = ps.Find("Lescale", "float");
            if (!ls) {
                m.LeScale = {LeNorm};
            } else {
                if ((long)ls->nums.size() != (long)m.nx * m.ny * m.nz)
                    throw Error(ps.loc + ": \"Lescale\" needs nx*ny*nz values");
                for (double v : ls->nums) m.LeScale.push_back((float)v * LeNorm);
                m.lnx = m.nx, m.lny = m.ny, m.lnz = m.nz;
            }
            m.Le = addDense(Le, 1.f);
            m.emissive = !m.temperature.empty() || !LeZero;  // isEmissive (media.h:263)
            Param *p0 = ps.Find("p0", "point3"), *p1 = ps.Find("p1", "point3");
            if (p0) m.p0 = V3((float)p0->nums[0], (float)p0->nums[1], (float)p0->nums[2]);
            if (p1) m.p1 = V3((float)p1->nums[0], (float)p1->nums[1], (float)p1->nums[2]);
            m.renderFromMedium = Mul(scene.camera.renderFromWorld, pm.worldFromMedium);
            BuildMajorantGrid(m);
        } else {
            throw Error(ps.loc + ": medium type \"" + pm.type + "\" is not supported yet");
        }
        ps.Find("type");
        ps.CheckUnused();
        mediumIndex[pm.name] = (int)scene.media.size();
        scene.media.push_back(std::move(m));
    }
    auto mediumOf = [&](const std::string &n, const std::string &loc) -> int {
        if (n.empty()) return -1;
        auto it = mediumIndex.find(n);
        if (it == mediumIndex.end()) throw Error(loc + ": named medium \"" + n + "\" undefined");
        return it->second;
    };
    scene.cameraMedium = mediumOf(cameraMediumName, "Camera");

    // ---- displaced plymeshes, object instances (flattened), then shapes -> render-space
    // triangles; area lights in shape order
    DisplacePlyMeshes();
    ResolveInstances();
    const Mat4 &renderFromWorld = scene.camera.renderFromWorld;
    std::map<std::string, int> spectrumCache;
    for (PendingShape &s : shapes) {
        Mat4 rfo = Mul(renderFromWorld, s.renderFromObject);
        bool flip = s.flip ^ SwapsHandedness(rfo);
        int base = (int)scene.verts.size();
        for (V3 p : s.P) scene.verts.push_back(XformPoint(rfo, p));
        // normals: renderFromObject(n) (inverse transpose), negated under ReverseOrientation
        // (TriangleMesh ctor, util/mesh.cpp:49-57); uv as given
        const uint8_t shadeBits = (s.N.empty() ? 0 : 1) | (s.uv.empty() ? 0 : 2) | (s.S.empty() ? 0 : 4);
        // shading tangents: renderFromObject(s) as a vector, not flipped (util/mesh.cpp:58-63)
        if (!s.S.empty() || !scene.vertS.empty()) {
            scene.vertS.resize(base, V3(0, 0, 0));
            for (size_t i = 0; i < s.P.size(); ++i) scene.vertS.push_back(s.S.empty() ? V3(0, 0, 0) : XformVector(rfo, s.S[i]));
        }
        if (shadeBits || !scene.vertN.empty()) {
            scene.vertN.resize(base, V3(0, 0, 0));
            scene.vertUV.resize(base, {0.f, 0.f});
            Mat4 inv = Inverse4(rfo);
            for (size_t i = 0; i < s.P.size(); ++i) {
                V3 nn(0, 0, 0);
                if (!s.N.empty()) {
                    nn = XformNormal(inv, s.N[i]);
                    if (s.flip) nn = -nn;
                }
                scene.vertN.push_back(nn);
                scene.vertUV.push_back(s.uv.empty() ? std::array<float, 2>{0.f, 0.f}
                                                    : std::array<float, 2>{s.uv[2 * i], s.uv[2 * i + 1]});
            }
        }
        int mat = s.material;
        if (mat < 0) {
            // pbrt's default material is "diffuse" with reflectance 0.5
            MaterialDesc m;
            m.constant = true;
            m.constantValue = 0.5f;
            m.name = "__default";
            scene.materials.push_back(m);
            mat = (int)scene.materials.size() - 1;
            for (PendingShape &o : shapes)
                if (o.material < 0) o.material = mat;
        }
        int lightSpectrum = -1;
        float lightScale = 1;
        bool twoSided = false;
        float power = -1;
        float imageKe = 1;  // an image emitter's mean luminance (k_e before the area term)
        if (!s.areaLight.empty()) {
            ParamSet &ap = s.areaParams;
            Param *L = ap.Find("L");
            float rgb[3] = {0, 0, 0};
            std::array<float, 311> dense;
            // DiffuseAreaLight::Create (lights.cpp:901-941): L defaults to the parameters' colour
            // space illuminant, and scale /= its photometric integral (an image emitter's too;
            // its pixels are RGBIlluminantSpectrum of the image's own colour space, sRGB here)
            const ColorSpaceDesc &acs = GetColorSpace(L ? L->colorSpace : ap.colorSpace);
            float photometric = acs.photometric;
            std::string spectrumKey;
            bool image = false;
            for (const Param &q : ap.params) image |= q.name == "filename" && q.type == "string";
            if (!L) {
                dense = image ? GetSpectralData().denseD65 : acs.illuminant;  // colorSpace->illuminant
            } else if (L->type == "rgb") {
                if (L->nums.size() != 3) throw Error(ap.loc + ": L needs 3 values");
                for (int i = 0; i < 3; ++i) rgb[i] = (float)L->nums[i];
                dense = DenseRGBIlluminant(rgb[0], rgb[1], rgb[2], L->colorSpace);
            } else if (L->type == "spectrum" && !L->nums.empty()) {
                // PiecewiseLinearSpectrum from (lambda, value) pairs (paramdict.cpp:415-439)
                dense = DensePiecewiseLinear(L->nums, ap.loc);
                photometric = PhotometricOf(dense);
                rgb[0] = -1;
                spectrumKey = "pl:" + std::to_string(scene.denseSpectra.size());
            } else if (L->type == "blackbody") {
                // BlackbodySpectrum(T) (util/spectrum.h), densely sampled; photometric over it
                if (L->nums.size() != 1) throw Error(ap.loc + ": blackbody L needs one temperature");
                const float T = (float)L->nums[0];
                for (int i = 0; i < 311; ++i) dense[i] = BlackbodyNormalized(395.f + i, T);
                photometric = PhotometricOf(dense);
                rgb[0] = -1;
                spectrumKey = "bb:" + std::to_string(T);
            } else {
                throw Error(ap.loc + ": L of type " + L->type + " not supported");
            }
            std::string key = spectrumKey.empty() ? std::to_string(rgb[0]) + "," + std::to_string(rgb[1]) + "," +
                                                        std::to_string(rgb[2]) + (L ? "" : image ? "D65" : "illum") +
                                                        "@" + acs.name
                                                  : spectrumKey;
            if (!spectrumCache.count(key)) {
                scene.denseSpectra.push_back(dense);
                spectrumCache[key] = (int)scene.denseSpectra.size() - 1;
            }
            lightSpectrum = spectrumCache[key];
            lightScale = (float)ap.GetFloat("scale", 1);
            twoSided = ap.GetBool("twosided", false);
            // lights.cpp:941: scale /= SpectrumToPhotometric(L) (illuminant part only)
            lightScale /= photometric;
            power = (float)ap.GetFloat("power", -1);  // applied per triangle below
            // DiffuseAreaLight's spread angle (lights.cpp:715-717): emission only within the
            // cone about the normal, SampleLi attenuated by the falloff (lights.cpp:763-771)
            {
                const float spread = (float)ap.GetFloat("spread", 90);
                const float rad = (kPi / 180) * spread;
                curSpread.cosFalloffEnd = std::cos(rad);
                curSpread.tanFalloffEnd = std::tan((kPi / 2 - rad));
                curSpread.normFalloffEnd = 2.0f / (2.0f + (2.0f * (kPi / 2 - rad) - kPi) * curSpread.tanFalloffEnd);
            }
            // lights.cpp:909-939: an image-textured emitter ("filename") emits the image and
            // folds its average luminance into k_e; neither is on this path, so it is refused
            // rather than rendered with the default illuminant.
            curSpread.image = -1;
            if (Param *fnp = ap.Find("filename", "string")) {
                if (L) throw Error(ap.loc + ": Both \"L\" and \"filename\" specified for DiffuseAreaLight.");
                // an image emitter: R, G, B bilerped at the hit's (u, 1 - v) as an
                // RGBIlluminantSpectrum; scale already divided by the colour space illuminant's
                // photometric integral (no "L": the default above)
                std::string fn = fnp->strs.empty() ? std::string() : fnp->strs[0];
                if (!fn.empty() && fn[0] != '/' && !s.dir.empty()) fn = s.dir + "/" + fn;
                LightImage im = LoadLightImage(fn, ap.loc);
                for (float v : im.v) {
                    if (std::isinf(v)) throw Error(ap.loc + ": " + fn + ": image has infinite pixel values and so is not suitable as a light.");
                    if (std::isnan(v)) throw Error(ap.loc + ": " + fn + ": image has not-a-number pixel values and so is not suitable as a light.");
                }
                if (im.nc < 3) throw Error(ap.loc + ": " + fn + ": Image provided to \"diffuse\" area light must have R, G, and B channels.");
                AreaLightImage ai;
                ai.w = im.w;
                ai.h = im.h;
                ai.rgb.resize((size_t)3 * im.w * im.h);
                for (size_t q = 0; q < (size_t)im.w * im.h; ++q)
                    for (int c = 0; c < 3; ++c) ai.rgb[3 * q + c] = im.v[q * im.nc + c];
                if (power > 0) {
                    // k_e of an image emitter: its mean luminance (the image colour space's
                    // LuminanceVector, lights.cpp:945-957); the area and pi follow per shape
                    const float(*xr)[3] = GetColorSpace(kColorSpaceSRGB).xyzFromRGBf;  // the image's (sRGB) LuminanceVector
                    const float lum[3] = {(float)xr[1][0], (float)xr[1][1], (float)xr[1][2]};
                    float k = 0;
                    for (int y = 0; y < im.h; ++y)
                        for (int x = 0; x < im.w; ++x)
                            for (int c = 0; c < 3; ++c) k += ai.rgb[3 * ((size_t)y * im.w + x) + c] * lum[c];
                    k /= im.w * im.h;
                    imageKe = k;
                }
                curSpread.image = (int)scene.areaLightImages.size();
                scene.areaLightImages.push_back(std::move(ai));
            }
            ap.CheckUnused();
            // DiffuseAreaLight::AlphaMasked (lights.h) masks the emission of an alpha-tested
            // emitter by HashFloat(p); not on this path yet
            if (AlphaId(s) >= 0) throw Error(s.loc + ": \"alpha\" on area lights is not supported yet");
        }
        {
            // bump / normal mapping needs the shading normal's derivatives dndu, dndv, which only
            // triangles (vertex normals) and disks (zero) provide here
            const MaterialDesc &md = scene.materials[mat];
            if ((md.texDisp >= 0 || md.normalMap >= 0) &&
                (s.kind == kShapeSphereT || s.kind == kShapeCylinderT || !s.quadIdx.empty()))
                throw Error(s.loc + ": bump and normal mapping on spheres, cylinders and bilinear patches are not supported yet");
        }
        curImageKe = imageKe;
        if (s.kind == kShapeSphereT || s.kind == kShapeDiskT || s.kind == kShapeCylinderT) {
            AnalyticShape(s, rfo, mat, lightSpectrum, lightScale, twoSided, power, mediumOf);
            continue;
        }
        if (!s.quadIdx.empty())
            BilinearPatches(s, rfo, mat, lightSpectrum, lightScale, twoSided, power, mediumOf, base);
        const int alphaId = AlphaId(s);
        for (size_t t = 0; t < s.idx.size(); t += 3) {
            scene.triAlpha.push_back(alphaId);
            std::array<int, 3> tri = {base + s.idx[t], base + s.idx[t + 1], base + s.idx[t + 2]};
            int triIndex = (int)scene.tris.size();
            scene.tris.push_back(tri);
            scene.triMaterial.push_back(s.material < 0 ? mat : s.material);
            scene.triFlip.push_back(flip ? 1 : 0);
            scene.triShade.push_back(shadeBits);
            if (!scene.media.empty())
                scene.triMedium.push_back({(int16_t)mediumOf(s.insideMedium, s.loc), (int16_t)mediumOf(s.outsideMedium, s.loc)});
            if (lightSpectrum >= 0) {
                AreaLightDesc l;
                SetSpread(&l);
                l.prim = triIndex;
                l.spectrum = lightSpectrum;
                l.scale = lightScale;
                l.twoSided = twoSided;
                V3 p0 = scene.verts[tri[0]], p1 = scene.verts[tri[1]], p2 = scene.verts[tri[2]];
                l.area = 0.5f * Length(Cross(p1 - p0, p2 - p0));  // Triangle::Area (shapes.h)
                if (power > 0) {
                    // lights.cpp:943-965: each triangle is its own DiffuseAreaLight, scaled so that
                    // it emits phi_v: k_e = (twoSided ? 2 : 1) * Area * Pi (times an image's mean
                    // luminance)
                    float k_e = imageKe;
                    k_e *= (twoSided ? 2 : 1) * l.area * kPi;
                    l.scale *= power / k_e;
                }
                scene.triLight.push_back((int)scene.areaLights.size());
                scene.areaLights.push_back(l);
            } else {
                scene.triLight.push_back(-1);
            }
        }
    }
    // LightSource lights in the order written (pbrt appends them after the area lights,
    // scene.cpp:1288-1348); point and spot lights join the light BVH, distant and uniform
    // infinite lights the infinite-light list (lightsamplers.cpp BVHLightSampler ctor)
    std::vector<std::pair<int, int>> lsOrder;  // (0: delta light j, 1: infinite-list entry j)
    std::vector<DeltaLightDesc> pointSpot, distants;
    std::vector<int> distantEntry;  // infinite-list entry of each distant light
    for (PendingLight &l : lights) {
        if (l.type == "point" || l.type == "spot" || l.type == "distant" || l.type == "goniometric" ||
            l.type == "projection") {
            DeltaLight(l, pointSpot, distants, distantEntry, lsOrder);
            continue;
        }
        if (l.type != "infinite") throw Error(l.params.loc + ": light \"" + l.type + "\" not supported yet");
        lsOrder.push_back({1, (int)scene.infiniteLights.size()});
        scene.infiniteLights.push_back(InfiniteLight(l));
    }
    scene.nPointSpot = (int)pointSpot.size();
    scene.deltaLights = pointSpot;
    for (size_t j = 0; j < distants.size(); ++j) {
        scene.infiniteLights[distantEntry[j]].distant = (int)scene.deltaLights.size();
        scene.deltaLights.push_back(distants[j]);
    }
    const int nA = (int)scene.areaLights.size(), nPS = scene.nPointSpot;
    scene.uniformOrder.clear();
    for (int i = 0; i < nA; ++i) scene.uniformOrder.push_back(i);
    for (auto &o : lsOrder) scene.uniformOrder.push_back(o.first == 0 ? nA + o.second : nA + nPS + o.second);
    // Bounds3f::BoundingSphere of the aggregate's bounds (every triangle), DistantLight::Preprocess
    {
        V3 mn(kInfinity, kInfinity, kInfinity), mx(-kInfinity, -kInfinity, -kInfinity);
        for (auto &t : scene.tris)
            for (int k = 0; k < 3; ++k) {
                const V3 v = scene.verts[t[k]];
                mn = V3(std::fmin(mn.x, v.x), std::fmin(mn.y, v.y), std::fmin(mn.z, v.z));
                mx = V3(std::fmax(mx.x, v.x), std::fmax(mx.y, v.y), std::fmax(mx.z, v.z));
            }
        for (const AnalyticShapeDesc &a : scene.shapes) {
            V3 lo, hi;
            ShapeBounds(a.dev, &lo, &hi);
            mn = V3(std::fmin(mn.x, lo.x), std::fmin(mn.y, lo.y), std::fmin(mn.z, lo.z));
            mx = V3(std::fmax(mx.x, hi.x), std::fmax(mx.y, hi.y), std::fmax(mx.z, hi.z));
        }
        const V3 c = (mn + mx) / 2;
        const bool inside = c.x >= mn.x && c.x <= mx.x && c.y >= mn.y && c.y <= mx.y && c.z >= mn.z && c.z <= mx.z;
        scene.sceneRadius = inside ? Distance(c, mx) : 0;
    }
    const size_t nLights = scene.areaLights.size() + scene.deltaLights.size() +
                           (scene.infiniteLights.size() - distants.size());
    if (nLights == 0) throw Error("No light sources specified");

    if (nLights == 1) scene.uniformLightSampler = true;
}

// Light::Create "infinite" (lights.cpp:1558-1694): no "L" and no "filename" -> the colour
// space's illuminant; "L" -> UniformInfiniteLight of it; "filename" -> ImageInfiniteLight of the
// image's R, G, B channels (square, finite, sRGB).  scale /= SpectrumToPhotometric of the
// spectrum (the colour space's illuminant for images); "illuminance" E_v scales a uniform
// light by E_v / pi.
InfiniteLightDesc Parser::InfiniteLight(PendingLight &l) {
    ParamSet &ps = l.params;
    Param *L = ps.Find("L");
    InfiniteLightDesc il;
    float scale = (float)ps.GetFloat("scale", 1);
    const float E_v = (float)ps.GetFloat("illuminance", -1);
    Param *portal = ps.Find("portal", "point3");
    if (!portal) portal = ps.Find("portal", "point");
    std::string fn = ps.GetString("filename", "");
    if (L && !fn.empty()) throw Error(ps.loc + ": Can't specify both emission \"L\" and \"filename\" with ImageInfiniteLight");
    if (portal && fn.empty()) throw Error(ps.loc + ": a portal infinite light with \"L\" (no \"filename\") is not supported yet");
    if (portal && portal->nums.size() != 12)
        throw Error(ps.loc + ": Expected 4 vertices for infinite light portal but given " + std::to_string(portal->nums.size() / 3));
    if (fn.empty()) {
        // UniformInfiniteLight (lights.cpp:1559-1580): L defaults to the parameters' colour space
        // illuminant; scale /= SpectrumToPhotometric(L)
        const ColorSpaceDesc &lcs = GetColorSpace(L ? L->colorSpace : ps.colorSpace);
        std::array<float, 311> dense = lcs.illuminant;
        float photometric = lcs.photometric;
        if (L && L->type == "rgb" && L->nums.size() == 3)
            dense = DenseRGBIlluminant((float)L->nums[0], (float)L->nums[1], (float)L->nums[2], L->colorSpace);
        else if (L && L->type == "spectrum" && !L->nums.empty()) {
            dense = DensePiecewiseLinear(L->nums, ps.loc);
            photometric = PhotometricOf(dense);
        } else if (L && L->type == "blackbody" && L->nums.size() == 1) {
            const float T = (float)L->nums[0];
            for (int i = 0; i < 311; ++i) dense[i] = BlackbodyNormalized(395.f + i, T);
            photometric = PhotometricOf(dense);
        } else if (L)
            throw Error(ps.loc + ": infinite light L must be rgb, spectrum or blackbody");
        scene.denseSpectra.push_back(dense);
        il.spectrum = (int)scene.denseSpectra.size() - 1;
        scale /= photometric;
        if (E_v > 0) scale *= E_v / kPi;
        il.scale = scale;
        ps.CheckUnused();
        return il;
    }
    if (fn[0] != '/' && !l.dir.empty()) fn = l.dir + "/" + fn;
    EnvLightDesc env = LoadEnvironmentImage(fn, ps.loc);
    for (float v : env.rgb) {
        if (std::isinf(v)) throw Error(ps.loc + ": " + fn + ": image has infinite pixel values and so is not suitable as a light.");
        if (std::isnan(v)) throw Error(ps.loc + ": " + fn + ": image has not-a-number pixel values and so is not suitable as a light.");
    }
    // the sRGB colour space's illuminant (std illuminant D65)
    scene.denseSpectra.push_back(GetSpectralData().denseD65);
    il.spectrum = (int)scene.denseSpectra.size() - 1;
    scale /= GetSpectralData().photometricD65;
    if (E_v > 0) {
        // the upper hemisphere's illuminance of the map (lights.cpp:1651-1679): pixel centres
        // through EqualAreaSquareToSphere, luminance-weighted, cosine-weighted; scale *= E_v / it
        const float(*xr)[3] = GetColorSpace(kColorSpaceSRGB).xyzFromRGBf;  // the image's (sRGB) LuminanceVector
        const float lum[3] = {(float)xr[1][0], (float)xr[1][1], (float)xr[1][2]};
        float illuminance = 0;
        for (int y = 0; y < env.res; ++y) {
            const float v = (float(y) + 0.5f) / float(env.res);
            for (int x = 0; x < env.res; ++x) {
                const float u = (x + 0.5f) / env.res;
                const V3 w = EqualAreaSquareToSphere(u, v);
                if (w.z <= 0) continue;
                const float *c = &env.rgb[((size_t)y * env.res + x) * 3];
                for (int k = 0; k < 3; ++k) illuminance += c[k] * lum[k] * w.z;
            }
        }
        illuminance *= 2 * kPi / (env.res * env.res);
        scale *= E_v / illuminance;
    }
    il.scale = scale;
    const Mat4 rfl = Mul(scene.camera.renderFromWorld, l.worldFromLight);
    const Mat4 lfr = Inverse4(rfl);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            env.renderFromLight[3 * i + j] = (float)rfl[i][j];
            env.lightFromRender[3 * i + j] = (float)lfr[i][j];
        }
    env.filename = fn;
    if (portal) {
        // the portal's corners through RenderFromWorld only (lights.cpp:1683-1685)
        for (int k = 0; k < 4; ++k) {
            const V3 p = XformPoint(scene.camera.renderFromWorld,
                                    V3((float)portal->nums[3 * k], (float)portal->nums[3 * k + 1], (float)portal->nums[3 * k + 2]));
            env.portalP[k][0] = p.x, env.portalP[k][1] = p.y, env.portalP[k][2] = p.z;
        }
        env.portal = true;
        BuildPortal(env, ps.loc);
    }
    il.image = (int)scene.envLights.size();
    scene.envLights.push_back(std::move(env));
    ps.CheckUnused();
    return il;
}

// GoniometricLight::Create / ProjectionLight::Create (lights.cpp:448-518, 603-680) after the
// photometric normalisation (sc): the image, "power", the render-space position and the
// inverse of renderFromLight * swapYZ (goniometric) or * Scale(1, -1, 1) (projection), and
// the LightBounds terms (lights.cpp:384-399, 563-575) the light BVH needs.
void Parser::ImageLight(PendingLight &l, const Mat4 &rfl, float sc, DeltaLightDesc *d) {
    ParamSet &ps = l.params;
    const bool gonio = l.type == "goniometric";
    std::string fn = ps.GetString("filename", "");
    if (fn.empty())
        throw Error(ps.loc + (gonio ? ": goniometric light without \"filename\" is not supported"
                                    : ": Must provide \"filename\" to \"projection\" light source"));
    if (fn[0] != '/' && !l.dir.empty()) fn = l.dir + "/" + fn;
    LightImage im = LoadLightImage(fn, ps.loc);
    for (float v : im.v) {
        if (std::isinf(v)) throw Error(ps.loc + ": " + fn + ": image has infinite pixel values and so is not suitable as a light.");
        if (std::isnan(v)) throw Error(ps.loc + ": " + fn + ": image has not-a-number pixel values and so is not suitable as a light.");
    }
    const size_t np = (size_t)im.w * im.h;
    const Mat4 lfr = Inverse4(rfl);
    d->p = V3((float)rfl[0][3], (float)rfl[1][3], (float)rfl[2][3]);  // renderFromLight(0, 0, 0)
    d->imgW = im.w;
    d->imgH = im.h;
    const float phi_v = (float)ps.GetFloat("power", -1);
    if (gonio) {
        d->type = kDeltaGonio;
        if (im.w != im.h)
            throw Error(ps.loc + ": " + fn + ": image resolution (" + std::to_string(im.w) + ", " + std::to_string(im.h) +
                        ") is non-square. It's unlikely this is an equal-area environment map.");
        // the Y channel, or a "Y" image of the R, G, B average in the source's pixel format
        d->img.resize(np);
        if (im.nc >= 3) {
            if (im.exr) throw Error(ps.loc + ": " + fn + ": RGB EXR images for goniometric lights are not supported yet");
            for (size_t q = 0; q < np; ++q) {
                const float *c = &im.v[q * im.nc];
                d->img[q] = im.Restore((c[0] + c[1] + c[2]) / 3);
            }
        } else if (im.nc == 1) {
            d->img = im.v;
        } else {
            throw Error(ps.loc + ": " + fn + ": has neither \"R\", \"G\", and \"B\" or \"Y\" channels.");
        }
        float sumY = 0;
        for (float y : d->img) sumY += y;
        if (phi_v > 0) sc *= phi_v / (4 * kPi * sumY / (float)np);
        // renderFromLight * swapYZ: its inverse swaps rows y and z of lightFromRender
        const int rows[3] = {0, 2, 1};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) d->m[i][j] = (float)lfr[rows[i]][j];
        d->w = V3(0, 0, 1);
        d->cosFalloffStart = std::cos(kPi);
        d->cosFalloffEnd = std::cos(kPi / 2);
        const auto &dense = scene.denseSpectra[d->spectrum];
        d->phi = sc * *std::max_element(dense.begin(), dense.end()) * 4 * kPi * sumY / (float)np;
    } else {
        d->type = kDeltaProjection;
        if (im.nc < 3)
            throw Error(ps.loc + ": " + fn + ": Image provided to \"projection\" light must have R, G, and B channels.");
        const float fov = (float)ps.GetFloat("fov", 90.);
        d->invTanAng = 1 / std::tan((kPi / 180) * fov / 2);
        if (phi_v > 0) {
            // ProjectionLight::Create's power (lights.cpp:479-511): the image's luminance over
            // the screen window, each pixel weighted by dw/dA = cos^3 of its direction (the
            // direction lightFromScreen gives a screen point is (x / invTan, y / invTan, 1)
            // normalised, evaluated here in double)
            const float(*xr)[3] = GetColorSpace(kColorSpaceSRGB).xyzFromRGBf;  // the image's (sRGB) LuminanceVector
            const float lum[3] = {(float)xr[1][0], (float)xr[1][1], (float)xr[1][2]};
            const float aspect = float(im.w) / float(im.h);
            const float x0 = aspect > 1 ? -aspect : -1, x1 = -x0, y0 = aspect > 1 ? -1 : -1 / aspect, y1 = -y0;
            const float opposite = std::tan((kPi / 180) * fov / 2);
            const float A = 4 * Sqr(opposite) * (aspect > 1 ? aspect : (1 / aspect));
            float sum = 0;
            for (int y = 0; y < im.h; ++y)
                for (int x = 0; x < im.w; ++x) {
                    const float tx = (x + .5f) / im.w, ty = (y + .5f) / im.h;
                    const double sx = (1 - tx) * x0 + tx * x1, sy = (1 - ty) * y0 + ty * y1;
                    const double wx = sx / d->invTanAng, wy = sy / d->invTanAng;
                    const float wz = (float)(1 / std::sqrt(wx * wx + wy * wy + 1));
                    const float dwdA = wz * wz * wz;
                    const float *c = &im.v[((size_t)y * im.w + x) * im.nc];
                    for (int k = 0; k < 3; ++k) sum += c[k] * lum[k] * dwdA;
                }
            sc *= phi_v / (A * sum / (float)np);
        }
        d->img.resize(3 * np);
        float sum = 0;
        for (size_t q = 0; q < np; ++q) {
            const float *c = &im.v[q * im.nc];
            for (int k = 0; k < 3; ++k) d->img[3 * q + k] = c[k];
            sum += std::max({c[0], c[1], c[2]});
        }
        // renderFromLight * Scale(1, -1, 1): its inverse negates row y of lightFromRender
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) d->m[i][j] = (float)((i == 1 ? -1 : 1) * lfr[i][j]);
        d->w = Normalize(V3((float)rfl[0][2], (float)rfl[1][2], (float)rfl[2][2]));
        // cosTotalWidth: the corner of screenBounds through lightFromScreen (approximated in
        // double: the light BVH's importance only)
        const float aspect = float(im.w) / float(im.h);
        const double cx = aspect > 1 ? aspect : 1, cy = aspect > 1 ? 1 : 1 / aspect;
        const double ex = cx / d->invTanAng, ey = cy / d->invTanAng;
        d->cosFalloffStart = std::cos(0.f);
        d->cosFalloffEnd = (float)(1 / std::sqrt(ex * ex + ey * ey + 1));
        d->phi = sc * sum / (float)np;
    }
    d->scale = sc;
}

// PointLight::Create / SpotLight::Create / DistantLight::Create (lights.cpp:192-276,
// 1464-1495): I or L as an illuminant spectrum, scale /= SpectrumToPhotometric, "power" (point,
// spot) or "illuminance" (distant), and the render-space geometry of renderFromLight * t.
void Parser::DeltaLight(PendingLight &l, std::vector<DeltaLightDesc> &pointSpot, std::vector<DeltaLightDesc> &distants,
                        std::vector<int> &distantEntry, std::vector<std::pair<int, int>> &lsOrder) {
    ParamSet &ps = l.params;
    const bool distant = l.type == "distant", projection = l.type == "projection";
    Param *I = projection ? nullptr : ps.Find(distant ? "L" : "I");
    // I / L default to the parameters' colour space illuminant; a projection light's image is
    // RGBIlluminantSpectrum of the image's colour space (sRGB) and divides by its illuminant's
    // photometric integral (lights.cpp:470-478)
    const ColorSpaceDesc &lcs = GetColorSpace(projection ? kColorSpaceSRGB : I ? I->colorSpace : ps.colorSpace);
    std::array<float, 311> dense = lcs.illuminant;
    float photometric = lcs.photometric;
    if (I && I->type == "rgb" && I->nums.size() == 3) {
        dense = DenseRGBIlluminant((float)I->nums[0], (float)I->nums[1], (float)I->nums[2], I->colorSpace);
    } else if (I && I->type == "spectrum" && !I->nums.empty()) {
        dense = DensePiecewiseLinear(I->nums, ps.loc);
        photometric = PhotometricOf(dense);
    } else if (I && I->type == "blackbody" && I->nums.size() == 1) {
        const float T = (float)I->nums[0];
        for (int i = 0; i < 311; ++i) dense[i] = BlackbodyNormalized(395.f + i, T);
        photometric = PhotometricOf(dense);
    } else if (I) {
        throw Error(ps.loc + ": " + l.type + " light " + (distant ? "L" : "I") + " must be rgb, spectrum or blackbody");
    }
    scene.denseSpectra.push_back(dense);
    DeltaLightDesc d;
    d.spectrum = (int)scene.denseSpectra.size() - 1;
    float sc = (float)ps.GetFloat("scale", 1);
    auto point3 = [&](const char *name, V3 def) {
        Param *q = ps.Find(name, "point3");
        if (!q) q = ps.Find(name, "point");
        if (!q) return def;
        if (q->nums.size() != 3) throw Error(ps.loc + ": \"" + std::string(name) + "\" needs 3 values");
        return V3((float)q->nums[0], (float)q->nums[1], (float)q->nums[2]);
    };
    const Mat4 rfl = Mul(scene.camera.renderFromWorld, l.worldFromLight);
    auto xfPoint = [&](const Mat4 &m, V3 p) {
        double r[4];
        for (int i = 0; i < 4; ++i) r[i] = m[i][0] * p.x + m[i][1] * p.y + m[i][2] * p.z + m[i][3];
        if (r[3] == 1) return V3((float)r[0], (float)r[1], (float)r[2]);
        return V3((float)(r[0] / r[3]), (float)(r[1] / r[3]), (float)(r[2] / r[3]));
    };
    auto xfVector = [&](const Mat4 &m, V3 v) {
        return V3((float)(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z),
                  (float)(m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z),
                  (float)(m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z));
    };
    sc /= photometric;
    if (l.type == "point") {
        d.type = kDeltaPoint;
        const float phi_v = (float)ps.GetFloat("power", -1);
        if (phi_v > 0) sc *= phi_v / (4 * kPi);
        d.p = xfPoint(rfl, point3("from", V3(0, 0, 0)));
    } else if (l.type == "spot") {
        d.type = kDeltaSpot;
        const float coneangle = (float)ps.GetFloat("coneangle", 30.);
        const float conedelta = (float)ps.GetFloat("conedeltaangle", 5.);
        const V3 from = point3("from", V3(0, 0, 0)), to = point3("to", V3(0, 0, 1));
        // dirToZ = Frame::FromZ(Normalize(to - from)): rows x, y, z (CoordinateSystem)
        const V3 z = Normalize(to - from);
        const float sign = std::copysign(1.f, z.z), a = -1 / (sign + z.z), b = z.x * z.y * a;
        const V3 x(1 + sign * z.x * z.x * a, sign * b, -sign * z.x), y(b, sign + z.y * z.y * a, -z.y);
        d.p = xfPoint(rfl, from);
        d.w = Normalize(xfVector(rfl, z));  // renderFromLight(0, 0, 1): Inverse(dirToZ) maps z to the axis
        // renderFromLight.ApplyInverse on vectors: dirToZ (rows x, y, z) times lightFromRender
        const Mat4 lfr = Inverse4(rfl);
        const V3 rows[3] = {x, y, z};
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                d.m[i][j] = (float)(rows[i].x * lfr[0][j] + rows[i].y * lfr[1][j] + rows[i].z * lfr[2][j]);
        d.cosFalloffEnd = std::cos(coneangle * (kPi / 180));
        d.cosFalloffStart = std::cos((coneangle - conedelta) * (kPi / 180));
        const float phi_v = (float)ps.GetFloat("power", -1);
        if (phi_v > 0) {
            const float k_e = 2 * kPi * ((1 - d.cosFalloffStart) + (d.cosFalloffStart - d.cosFalloffEnd) / 2);
            sc *= phi_v / k_e;
        }
    } else if (l.type == "goniometric" || projection) {
        ImageLight(l, rfl, sc, &d);
        sc = d.scale;
    } else {
        d.type = kDeltaDistant;
        const V3 from = point3("from", V3(0, 0, 0)), to = point3("to", V3(0, 0, 1));
        d.w = xfVector(rfl, Normalize(from - to));  // renderFromLight(0, 0, 1); SampleLi normalises it
        const float E_v = (float)ps.GetFloat("illuminance", -1);
        if (E_v > 0) sc *= E_v;
    }
    d.scale = sc;
    ps.CheckUnused();
    if (distant) {
        lsOrder.push_back({1, (int)scene.infiniteLights.size()});
        InfiniteLightDesc il;
        il.spectrum = d.spectrum;
        il.scale = d.scale;
        distantEntry.push_back((int)scene.infiniteLights.size());
        scene.infiniteLights.push_back(il);  // .distant set once the delta-light order is final
        distants.push_back(d);
    } else {
        lsOrder.push_back({0, (int)pointSpot.size()});
        pointSpot.push_back(d);
    }
}

// ------------------------------------------------------------------ textures
// TextureMapping2D::Create (textures.cpp:49-73) / TextureMapping3D::Create (:75-79)
void Parser::TexMapping(ParamSet &ps, const Mat4 &renderFromTexture, TextureDesc *t, bool threeD) {
    auto setXform = [&]() {
        Mat4 tfr = Inverse4(renderFromTexture);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 4; ++j) t->textureFromRender[4 * i + j] = (float)tfr[i][j];
        if (tfr[3][0] != 0 || tfr[3][1] != 0 || tfr[3][2] != 0 || tfr[3][3] != 1)
            throw Error(ps.loc + ": projective texture transforms are not supported");
    };
    if (threeD) {
        t->mapping = kMap3D;
        setXform();
        return;
    }
    std::string type = ps.GetString("mapping", "uv");
    if (type == "uv") {
        t->mapping = kMapUV;
        t->map[0] = (float)ps.GetFloat("uscale", 1.);
        t->map[1] = (float)ps.GetFloat("vscale", 1.);
        t->map[2] = (float)ps.GetFloat("udelta", 0.);
        t->map[3] = (float)ps.GetFloat("vdelta", 0.);
    } else if (type == "spherical" || type == "cylindrical") {
        t->mapping = type == "spherical" ? kMapSpherical : kMapCylindrical;
        setXform();
    } else if (type == "planar") {
        t->mapping = kMapPlanar;
        setXform();
        auto vec = [&](const char *n, V3 def) {
            Param *p = ps.Find(n, "vector3");
            if (p && p->nums.size() == 3) return V3((float)p->nums[0], (float)p->nums[1], (float)p->nums[2]);
            return def;
        };
        V3 v1 = vec("v1", V3(1, 0, 0)), v2 = vec("v2", V3(0, 1, 0));
        t->vs[0] = v1.x, t->vs[1] = v1.y, t->vs[2] = v1.z;
        t->vt[0] = v2.x, t->vt[1] = v2.y, t->vt[2] = v2.z;
        t->map[0] = (float)ps.GetFloat("udelta", 0.);
        t->map[1] = (float)ps.GetFloat("vdelta", 0.);
    } else {
        throw Error(ps.loc + ": 2D texture mapping \"" + type + "\" unknown");
    }
}

// an "rgb" spectrum parameter as pbrt's GetSpectrumTextureOrNull builds it (paramdict.cpp:846-870)
TexSpectrumConst Parser::RGBConst(const Param *p, int specType, const std::string &loc) {
    if (p->nums.size() != 3) throw Error(loc + ": Didn't find three values for \"rgb\" parameter \"" + p->name + "\".");
    const float r = (float)p->nums[0], g = (float)p->nums[1], b = (float)p->nums[2];
    if (r < 0 || g < 0 || b < 0) throw Error(loc + ": Negative value provided for RGB parameter \"" + p->name + "\".");
    TexSpectrumConst c;
    c.rgb = true;
    if (specType == kSpecAlbedo) {
        if (r > 1 || g > 1 || b > 1)
            throw Error(loc + ": RGB parameter \"" + p->name + "\" used as an albedo has > 1 component.");
        auto cf = RGBToSigmoidCoeffs(r, g, b, p->colorSpace);
        c.c[0] = cf[0], c.c[1] = cf[1], c.c[2] = cf[2];
        c.scale = 1;
    } else if (specType == kSpecUnbounded) {
        // RGBUnboundedSpectrum (util/spectrum.cpp:240-244)
        const float m = std::max({r, g, b});
        c.scale = 2 * m;
        auto cf = c.scale != 0 ? RGBToSigmoidCoeffs(r / c.scale, g / c.scale, b / c.scale, p->colorSpace)
                               : RGBToSigmoidCoeffs(0, 0, 0, p->colorSpace);
        c.c[0] = cf[0], c.c[1] = cf[1], c.c[2] = cf[2];
    } else {
        throw Error(loc + ": illuminant spectrum textures are not supported");
    }
    return c;
}

int Parser::FloatParamNode(const Param *p, float def, const std::string &loc) {
    TextureDesc t;
    t.kind = kTexConstant;
    t.fvalue[0] = def;
    if (p && p->type == "texture") {
        if (p->strs.size() != 1) throw Error(loc + ": texture parameter \"" + p->name + "\" needs one texture name");
        return InstTex(p->strs[0], false, 0, loc);
    }
    if (p && p->type == "float") {
        if (p->nums.empty()) throw Error(loc + ": \"float " + p->name + "\" needs a value");
        t.fvalue[0] = (float)p->nums[0];
    } else if (p && !p->type.empty()) {
        throw Error(loc + ": \"" + p->type + " " + p->name + "\" is not a float texture parameter");
    }
    return NewTexNode(t);
}

int Parser::SpectrumParamNode(const Param *p, int specType, float def, const std::string &loc) {
    TextureDesc t;
    t.kind = kTexConstant;
    t.spectrum = true;
    t.specType = specType;
    t.svalue[0].value = def;
    if (p && p->type == "texture") {
        if (p->strs.size() != 1) throw Error(loc + ": texture parameter \"" + p->name + "\" needs one texture name");
        return InstTex(p->strs[0], true, specType, loc);
    }
    if (p && p->type == "rgb") {
        t.svalue[0] = RGBConst(p, specType, loc);
    } else if (p && !p->type.empty()) {
        throw Error(loc + ": \"" + p->type + " " + p->name + "\" is not supported as a spectrum texture parameter");
    }
    return NewTexNode(t);
}

// GetFloatTexture(name, def) / GetSpectrumTexture(name, ConstantSpectrum(def), type)
int Parser::FloatTexParam(ParamSet &ps, const std::string &name, float def) {
    Param *p = nullptr;
    for (auto &q : ps.params)
        if (q.name == name && (q.type == "texture" || q.type == "float")) {
            q.used = true;
            p = &q;
            break;
        }
    return FloatParamNode(p, def, ps.loc);
}
int Parser::SpectrumTexParam(ParamSet &ps, const std::string &name, int specType, float def) {
    Param *p = nullptr;
    for (auto &q : ps.params)
        if (q.name == name) {
            q.used = true;
            p = &q;
            break;
        }
    return SpectrumParamNode(p, specType, def, ps.loc);
}

// FloatTexture::Create / SpectrumTexture::Create (textures.cpp:1606-1707) for one SpectrumType
int Parser::InstTex(const std::string &name, bool spectrum, int specType, const std::string &loc) {
    const auto key = std::make_tuple(name, spectrum, spectrum ? specType : 0);
    if (auto it = texInstances.find(key); it != texInstances.end()) return it->second;
    auto pit = pendingTextures.find({name, spectrum});
    if (pit == pendingTextures.end())
        throw Error(loc + ": Couldn't find " + std::string(spectrum ? "spectrum" : "float") + " texture named \"" + name + "\"");
    if (texInProgress.count({name, spectrum})) throw Error(loc + ": texture \"" + name + "\" refers to itself");
    texInProgress.insert({name, spectrum});
    PendingTexture pt = pit->second;
    ParamSet &ps = pt.params;
    const Mat4 renderFromTexture = Mul(scene.camera.renderFromWorld, pt.worldFromTexture);
    TextureDesc t;
    t.spectrum = spectrum;
    t.specType = specType;
    auto child = [&](const char *n, float def) {
        return spectrum ? SpectrumTexParam(ps, n, specType, def) : FloatTexParam(ps, n, def);
    };
    int result = -1;
    const std::string &c = pt.cls;
    if (c == "constant") {
        t.kind = kTexConstant;
        if (spectrum) {
            Param *v = ps.Find("value");
            if (v && v->type == "rgb") t.svalue[0] = RGBConst(v, specType, ps.loc);
            else if (v) throw Error(ps.loc + ": \"" + v->type + " value\" is not supported for spectrum textures");
            else t.svalue[0].value = 1;
        } else {
            t.fvalue[0] = (float)ps.GetFloat("value", 1.);
        }
        result = NewTexNode(t);
    } else if (c == "scale") {
        // FloatScaledTexture::Create / SpectrumScaledTexture::Create (textures.cpp:936-1001): a
        // constant scale of 1 drops the node, a constant scale of an image texture folds into
        // the image's scale
        int tex = child("tex", 1.f), sc = FloatTexParam(ps, "scale", 1.f);
        const int rounds = spectrum ? 1 : 2;
        for (int i = 0; i < rounds && result < 0; ++i) {
            const TextureDesc &sn = scene.textures[sc];
            if (sn.kind == kTexConstant) {
                const float cs = sn.fvalue[0];
                if (cs == 1) result = tex;
                else if (scene.textures[tex].kind == kTexImage) {
                    TextureDesc copy = scene.textures[tex];
                    copy.scale *= cs;
                    result = NewTexNode(copy);
                }
            }
            if (!spectrum && result < 0) std::swap(tex, sc);
        }
        if (result < 0) {
            if (!spectrum) std::swap(tex, sc);
            t.kind = kTexScale;
            t.child[0] = tex;
            t.child[1] = sc;
            result = NewTexNode(t);
        }
    } else if (c == "mix") {
        t.kind = kTexMix;
        t.child[0] = child("tex1", 0.f);
        t.child[1] = child("tex2", 1.f);
        t.child[2] = FloatTexParam(ps, "amount", 0.5f);
        result = NewTexNode(t);
    } else if (c == "directionmix") {
        t.kind = kTexDirectionMix;
        V3 dir(0, 1, 0);
        if (Param *d = ps.Find("dir", "vector3")) {
            if (d->nums.size() != 3) throw Error(ps.loc + ": \"vector3 dir\" needs 3 values");
            dir = V3((float)d->nums[0], (float)d->nums[1], (float)d->nums[2]);
        }
        dir = Normalize(XformVector(renderFromTexture, dir));
        t.dir[0] = dir.x, t.dir[1] = dir.y, t.dir[2] = dir.z;
        t.child[0] = child("tex1", 0.f);
        t.child[1] = child("tex2", 1.f);
        result = NewTexNode(t);
    } else if (c == "checkerboard") {
        t.kind = kTexCheckerboard;
        const int dim = ps.GetInt("dimension", 2);
        if (dim != 2 && dim != 3) throw Error(ps.loc + ": " + std::to_string(dim) + " dimensional checkerboard texture not supported");
        t.child[0] = child("tex1", 1.f);
        t.child[1] = child("tex2", 0.f);
        TexMapping(ps, renderFromTexture, &t, dim == 3);
        result = NewTexNode(t);
    } else if (c == "bilerp") {
        t.kind = kTexBilerp;
        TexMapping(ps, renderFromTexture, &t, false);
        const char *names[4] = {"v00", "v01", "v10", "v11"};
        const float defs[4] = {0, 1, 0, 1};
        if (spectrum) {
            // stored in Bilerp's corner order v00, v10, v01, v11 (textures.h:340-344)
            const int slot[4] = {0, 2, 1, 3};
            for (int k = 0; k < 4; ++k) {
                Param *v = ps.Find(names[k]);
                if (v && v->type == "rgb") t.svalue[slot[k]] = RGBConst(v, specType, ps.loc);
                else if (v) throw Error(ps.loc + ": \"" + v->type + " " + names[k] + "\" is not supported");
                else t.svalue[slot[k]].value = defs[k];
            }
        } else {
            for (int k = 0; k < 4; ++k) t.fvalue[k] = (float)ps.GetFloat(names[k], defs[k]);
        }
        result = NewTexNode(t);
    } else if (c == "dots") {
        // Float/SpectrumDotsTexture::Create (textures.cpp:305-335): a 2D mapping, inside 1 /
        // outside 0 by default
        t.kind = kTexDots;
        TexMapping(ps, renderFromTexture, &t, false);
        t.child[0] = child("inside", 1.f);
        t.child[1] = child("outside", 0.f);
        result = NewTexNode(t);
    } else if (!spectrum && (c == "fbm" || c == "wrinkled" || c == "windy")) {
        // FBmTexture / WrinkledTexture / WindyTexture::Create (textures.cpp:343-352, 1008-1032):
        // a 3D point mapping; octaves 8, roughness 0.5 (windy takes neither)
        t.kind = c == "fbm" ? kTexFBm : (c == "wrinkled" ? kTexWrinkled : kTexWindy);
        TexMapping(ps, renderFromTexture, &t, true);
        if (t.kind != kTexWindy) {
            t.octaves = ps.GetInt("octaves", 8);
            t.omega = (float)ps.GetFloat("roughness", .5);
        }
        result = NewTexNode(t);
    } else if (spectrum && c == "marble") {
        // MarbleTexture::Create (textures.cpp:555-563): octaves 8, roughness .5, scale 1,
        // variation .2; its RGB is an RGBAlbedoSpectrum whatever the use (textures.cpp:546-552)
        t.kind = kTexMarble;
        TexMapping(ps, renderFromTexture, &t, true);
        t.octaves = ps.GetInt("octaves", 8);
        t.omega = (float)ps.GetFloat("roughness", .5);
        t.scale = (float)ps.GetFloat("scale", 1.);
        t.variation = (float)ps.GetFloat("variation", .2);
        result = NewTexNode(t);
    } else if (c == "imagemap") {
        // Float/SpectrumImageTexture::Create (textures.cpp:428-521)
        t.kind = kTexImage;
        TexMapping(ps, renderFromTexture, &t, false);
        t.maxAniso = (float)ps.GetFloat("maxanisotropy", 8.);
        const std::string filter = ps.GetString("filter", "bilinear");
        if (filter == "point") t.filter = kMipPoint;
        else if (filter == "bilinear") t.filter = kMipBilinear;
        else if (filter == "trilinear") t.filter = kMipTrilinear;
        else if (filter == "ewa" || filter == "EWA") t.filter = kMipEWA;
        else throw Error(ps.loc + ": " + filter + ": filter function unknown");
        const std::string wrapS = ps.GetString("wrap", "repeat");
        int wrap;
        if (wrapS == "repeat") wrap = kWrapRepeat;
        else if (wrapS == "black") wrap = kWrapBlack;
        else if (wrapS == "clamp") wrap = kWrapClamp;
        else if (wrapS == "octahedralsphere") wrap = kWrapOctahedral;
        else throw Error(ps.loc + ": " + wrapS + ": wrap mode unknown");
        t.scale = (float)ps.GetFloat("scale", 1.);
        t.invert = ps.GetBool("invert", false);
        std::string fn = ps.GetString("filename", "");
        if (fn.empty()) throw Error(ps.loc + ": imagemap needs \"string filename\"");
        if (fn[0] != '/' && !pt.dir.empty()) fn = pt.dir + "/" + fn;
        auto hasPng = [](const std::string &f) {
            if (f.size() < 4) return false;
            std::string e = f.substr(f.size() - 4);
            std::transform(e.begin(), e.end(), e.begin(), ::tolower);
            return e == ".png";
        };
        const std::string enc = ps.GetString("encoding", hasPng(fn) ? "sRGB" : "linear");
        const std::string basisFile = ps.GetString("basisfilename", "");
        if (!basisFile.empty() && spectrum) {
            // GPUSpectrumImageTexture::Create (textures.cpp:1148-1176); the reference opens the
            // name as given (relative to the working directory); relative names here resolve
            // against the scene file's directory, as "filename" does
            std::string bf = basisFile;
            if (bf[0] != '/' && !pt.dir.empty()) bf = pt.dir + "/" + bf;
            t.basis = (int)scene.texBasis.size();
            ReadBasisFile(bf, ps.loc, &scene.texBasis);
            t.basisWidth = (int)scene.texBasis.size() - t.basis;
            if (scene.texBasis[t.basis] == 0) {  // no channels: Evaluate's RGB branch (textures.h:680)
                scene.texBasis.resize(t.basis);
                t.basis = -1;
                t.basisWidth = 0;
            }
        }  // FloatImageTexture reads the file but never uses it (textures.cpp:447-458)
        // the texture cache (textures.h:537-554): one pyramid per (file, encoding, wrap)
        int img = -1;
        for (size_t i = 0; i < scene.images.size(); ++i)
            if (scene.images[i].filename == fn + "|" + enc && scene.images[i].wrap == wrap) img = (int)i;
        if (img < 0) {
            ImageDesc id = LoadImageTexture(fn, enc, wrap, ps.loc);
            id.filename = fn + "|" + enc;
            scene.images.push_back(std::move(id));
            img = (int)scene.images.size() - 1;
        }
        t.image = img;
        if (t.basis >= 0 && scene.images[img].nc < 3)
            throw Error(ps.loc + ": a multispectral basis texture needs an RGB image (" + fn + ")");
        result = NewTexNode(t);
    } else {
        throw Error(ps.loc + ": \"" + c + "\": " + std::string(spectrum ? "spectrum" : "float") +
                    " texture type is not supported yet");
    }
    ps.CheckUnused();
    texInProgress.erase({name, spectrum});
    texInstances[key] = result;
    return result;
}

// ---- multispectral basis files: a JSON array of channels, each {"basis": [...], "offset": [...]}
namespace {
struct Json {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    double num = 0;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;
    const Json *Get(const std::string &k) const {
        for (auto &kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};
struct JsonReader {
    const std::string &s;
    size_t i = 0;
    std::string where;
    [[noreturn]] void Fail(const std::string &m) const {
        throw Error(where + ": malformed JSON (" + m + ") at byte " + std::to_string(i));
    }
    void Ws() {
        while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
    }
    Json Value(int depth = 0) {
        if (depth > 64) Fail("nesting too deep");
        Ws();
        if (i >= s.size()) Fail("unexpected end");
        Json v;
        const char c = s[i];
        if (c == '[') {
            v.kind = Json::Arr;
            ++i;
            Ws();
            if (i < s.size() && s[i] == ']') return ++i, v;
            for (;;) {
                v.arr.push_back(Value(depth + 1));
                Ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == ']') { ++i; return v; }
                Fail("expected , or ]");
            }
        }
        if (c == '{') {
            v.kind = Json::Obj;
            ++i;
            Ws();
            if (i < s.size() && s[i] == '}') return ++i, v;
            for (;;) {
                Ws();
                Json k = Value(depth + 1);
                if (k.kind != Json::Str) Fail("object key must be a string");
                Ws();
                if (i >= s.size() || s[i] != ':') Fail("expected :");
                ++i;
                v.obj.emplace_back(k.str, Value(depth + 1));
                Ws();
                if (i < s.size() && s[i] == ',') { ++i; continue; }
                if (i < s.size() && s[i] == '}') { ++i; return v; }
                Fail("expected , or }");
            }
        }
        if (c == '"') {
            v.kind = Json::Str;
            ++i;
            while (i < s.size() && s[i] != '"') {
                if (s[i] == '\\') ++i;
                if (i < s.size()) v.str += s[i++];
            }
            if (i >= s.size()) Fail("unterminated string");
            return ++i, v;
        }
        if (s.compare(i, 4, "true") == 0) return i += 4, v.kind = Json::Bool, v.num = 1, v;
        if (s.compare(i, 5, "false") == 0) return i += 5, v.kind = Json::Bool, v;
        if (s.compare(i, 4, "null") == 0) return i += 4, v;
        char *end = nullptr;
        v.num = std::strtod(s.c_str() + i, &end);
        if (end == s.c_str() + i) Fail("unexpected character");
        v.kind = Json::Num;
        i = end - s.c_str();
        return v;
    }
};
}  // namespace
// the basis array of GPUSpectrumImageTexture::Create (textures.cpp:1148-1176): channel count, the
// first channel's basis length, int(first channel's offset[0]), then every channel's first
// <length> basis values.  Refused: an unreadable or malformed file, a channel without a numeric
// "basis" array of that length, a first channel without a numeric "offset"; more than 3 channels
// (Evaluate reads an RGB texel, textures.h:664-671)
void ReadBasisFile(const std::string &path, const std::string &loc, std::vector<float> *out) {
    std::ifstream in(path);
    if (!in) throw Error(loc + ": cannot open basis file " + path);
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();
    JsonReader rd{text, 0, path};
    const Json j = rd.Value();
    rd.Ws();
    if (rd.i != text.size()) rd.Fail("trailing characters");
    if (j.kind != Json::Arr) throw Error(path + ": a basis file is a JSON array of channels");
    if (j.arr.size() > 3) throw Error(path + ": more than 3 basis channels (an RGB texel has 3)");
    size_t elemSize = 0;
    int offset = 0;
    for (size_t c = 0; c < j.arr.size(); ++c) {
        const Json &e = j.arr[c];
        const Json *b = e.kind == Json::Obj ? e.Get("basis") : nullptr;
        if (!b || b->kind != Json::Arr) throw Error(path + ": channel " + std::to_string(c) + " has no \"basis\" array");
        if (c == 0) {
            elemSize = b->arr.size();
            const Json *o = e.Get("offset");
            if (!o || o->kind != Json::Arr || o->arr.empty() || o->arr[0].kind != Json::Num)
                throw Error(path + ": the first channel has no numeric \"offset\" array");
            offset = (int)o->arr[0].num;  // int offset = elem["offset"][0]
        }
        if (b->arr.size() < elemSize)
            throw Error(path + ": channel " + std::to_string(c) + "'s basis is shorter than the first channel's");
        for (size_t k = 0; k < elemSize; ++k)
            if (b->arr[k].kind != Json::Num) throw Error(path + ": non-numeric basis value");
    }
    out->push_back((float)j.arr.size());
    out->push_back((float)elemSize);
    out->push_back((float)offset);
    for (const Json &e : j.arr)
        for (size_t k = 0; k < elemSize; ++k) out->push_back((float)e.Get("basis")->arr[k].num);
}

// The shape's alpha texture (scene.cpp:1369-1384 getAlphaTexture): a named float texture, or a
// constant "float alpha" below 1 (1 or more: no alpha test); -1 when there is none.  One
// SceneDesc::alphaTex entry (texture node, compiled program) per distinct parameter.
int Parser::AlphaId(const PendingShape &s) {
    if (!s.hasAlpha) return -1;
    std::string key;
    if (s.alpha.type == "texture") {
        if (s.alpha.strs.size() != 1) throw Error(s.loc + ": \"texture alpha\" needs one texture name");
        if (!pendingTextures.count({s.alpha.strs[0], false}))
            throw Error(s.loc + ": " + s.alpha.strs[0] + ": couldn't find float texture for \"alpha\" parameter.");
        key = "t:" + s.alpha.strs[0];
    } else {
        if (s.alpha.nums.empty()) throw Error(s.loc + ": \"float alpha\" needs a value");
        const float a = (float)s.alpha.nums[0];
        if (!(a < 1.f)) return -1;
        char b[32];
        std::snprintf(b, sizeof b, "f:%a", a);
        key = b;
    }
    auto it = alphaIds.find(key);
    if (it != alphaIds.end()) return it->second;
    const int node = FloatParamNode(&s.alpha, 1.f, s.loc);
    const int prog = CompileTexProgram(scene, node, false);
    scene.alphaTex.push_back({node, prog});
    const int id = (int)scene.alphaTex.size() - 1;
    alphaIds[key] = id;
    return id;
}

// The plymesh displacement of shapes.cpp:1425-1458: TriQuadMesh::Displace (host/displace.cpp)
// with the texture evaluated on the host by the product's texture code at each vertex's
// object-space position and uv, with no differentials (TextureEvalContext{p, uv})
void Parser::DisplacePlyMeshes() {
    // shapes of ObjectBegin definitions too, once, in their definition's render space (the
    // instances then copy the displaced mesh, as pbrt's instanced primitives share it)
    std::vector<std::pair<PendingShape *, int>> todo;
    auto add = [&](PendingShape &s) {
        if (!s.hasDisp) return;
        const int node = FloatParamNode(&s.disp, 0.f, s.loc);
        todo.push_back({&s, CompileTexProgram(scene, node, false)});
    };
    for (PendingShape &s : shapes) add(s);
    for (auto &def : instanceDefs)
        for (PendingShape &s : def.second) add(s);
    if (todo.empty()) return;
    TexTables tt;
    BuildTexTables(scene, &tt);
    const TexView T = HostTexView(tt);
    // the programs serve the load only: dropped afterwards (they were compiled last), so the
    // device does not take the scene for a textured one
    const size_t firstDispProg = (size_t)todo.front().second;
    const Mat4 &renderFromWorld = scene.camera.renderFromWorld;
    for (auto &[sp, prog] : todo) {
        PendingShape &s = *sp;
        DisplaceMesh m;
        m.p = s.P;
        m.n = s.N;
        for (size_t i = 0; i + 1 < s.uv.size(); i += 2) m.uv.push_back({s.uv[i], s.uv[i + 1]});
        m.tri = s.idx;
        m.quad = s.quadIdx;
        const Mat4 rfo = Mul(renderFromWorld, s.renderFromObject);
        float rf[16];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) rf[4 * i + j] = (float)rfo[i][j];
        try {
            DisplaceTriQuadMesh(&m, rf, s.edgeLength, [&](V3 p, float u, float v) {
                TexEvalCtx c{};
                c.p = p;
                c.n = V3(0, 0, 0);
                c.u = u;
                c.v = v;
                return HostTexFloat(T, prog, c);
            });
        } catch (const std::runtime_error &e) {
            throw Error(s.loc + ": " + e.what());
        }
        s.P = std::move(m.p);
        s.N = std::move(m.n);
        s.uv.clear();
        for (const auto &t : m.uv) s.uv.insert(s.uv.end(), {t[0], t[1]});
        s.idx = std::move(m.tri);
        s.quadIdx.clear();
        s.hasDisp = false;
    }
    scene.texPrograms.resize(firstDispProg);
}

void Parser::ResolveTextures() {
    for (MatTexPending &mp : matTexPending) {
        MaterialDesc &m = scene.materials[mp.mat];
        if (mp.hasAmount) {
            const int node = FloatParamNode(mp.amount.type.empty() ? nullptr : &mp.amount, 0.5f, mp.loc);
            const int k = scene.textures[node].kind;
            if (k != kTexConstant && k != kTexImage)
                throw Error(mp.loc + ": The wavefront renderer currently only supports basic textures for its \"amount\" parameter.");
            m.texAmount = CompileTexProgram(scene, node, false);
            continue;
        }
        // textured reflectance / roughness: diffuse, dielectric and conductor materials; bump and
        // normal maps on every material that reads them (MakeMaterial)
        if (((mp.hasRefl && m.type != kMatHair) || mp.hasRough) && m.type != kMatDiffuse && m.type != kMatDielectric &&
            m.type != kMatConductor)
            throw Error(mp.loc + ": textures are supported on diffuse, dielectric and conductor materials only");
        if (mp.hasDisp) {
            m.dispNode = FloatParamNode(&mp.disp, 0.f, mp.loc);
            m.texDisp = CompileTexProgram(scene, m.dispNode, false);
        }
        if (!mp.normalMap.empty()) {
            // one image per file; pbrt reads it linearly encoded and looks it up with a repeat
            // wrap (NormalMap, materials.h:86-106)
            int img = -1;
            const std::string key = mp.normalMap + "|normalmap";
            for (size_t i = 0; i < scene.images.size(); ++i)
                if (scene.images[i].filename == key) img = (int)i;
            if (img < 0) {
                ImageDesc id = LoadImageTexture(mp.normalMap, "linear", kWrapRepeat, mp.loc);
                if (id.nc < 3) throw Error(mp.loc + ": " + mp.normalMap + ": normal map image must contain R, G, and B channels");
                id.filename = key;
                scene.images.push_back(std::move(id));
                img = (int)scene.images.size() - 1;
            }
            m.normalMap = img;
        }
        if (mp.hasRefl) {
            const int node = SpectrumParamNode(&mp.refl, mp.reflSpec, 0.5f, mp.loc);
            m.texReflectance = CompileTexProgram(scene, node, true);
        }
        if (mp.hasHair) {
            const bool conc = !mp.hair[4].type.empty() || !mp.hair[5].type.empty();
            for (int k = 0; k < 6; ++k) {
                if (mp.hair[k].type.empty() && !(conc && k >= 4)) continue;
                const int node = FloatParamNode(mp.hair[k].type.empty() ? nullptr : &mp.hair[k], 0.f, mp.loc);
                m.texHair[k] = CompileTexProgram(scene, node, false);
            }
        }
        if (mp.hasSss) {
            for (int k = 0; k < 2; ++k)
                if (!mp.sss[k].type.empty())
                    m.texSss[k] = CompileTexProgram(scene, SpectrumParamNode(&mp.sss[k], kSpecUnbounded, 1.f, mp.loc), true);
        }
        if (mp.hasRough) {
            const int u = FloatParamNode(mp.ur.type.empty() ? nullptr : &mp.ur, 0.f, mp.loc);
            const int v = FloatParamNode(mp.vr.type.empty() ? nullptr : &mp.vr, 0.f, mp.loc);
            m.texURough = CompileTexProgram(scene, u, false);
            m.texVRough = CompileTexProgram(scene, v, false);
        }
    }
    if (!matTexPending.empty()) ComputeCameraDifferentials(scene);
    // a mix of mixes must bottom out in real materials (materials.cpp: a cycle never resolves)
    for (size_t i = 0; i < scene.materials.size(); ++i) {
        int m = (int)i, steps = 0;
        std::vector<int> stack{m};
        while (!stack.empty()) {
            const int x = stack.back();
            stack.pop_back();
            if (scene.materials[x].type != kMatMix) continue;
            if (++steps > 64) throw Error("mix material \"" + scene.materials[i].name + "\" refers to itself");
            stack.push_back(scene.materials[x].mixMat[0]);
            stack.push_back(scene.materials[x].mixMat[1]);
        }
    }
}

SceneDesc LoadPbrtString(const std::string &text, const std::string &baseDir,
                         const std::map<std::string, std::string> &overrides) {
    SceneDesc s;
    Parser p(s, overrides);
    p.ParseString(text, "<string>", baseDir);
    p.Finish();
    FinalizeScene(s);
    return s;
}

SceneDesc LoadPbrtFile(const std::string &path, const std::map<std::string, std::string> &overrides) {
    SceneDesc s;
    Parser p(s, overrides);
    p.ParseFile(path);
    p.Finish();
    FinalizeScene(s);
    return s;
}

}  // namespace pbrt_amd
