// Host-side scene model of pbrt-v4_amd: what the .pbrt subset loader produces and what
// the device upload consumes.  Everything is already in pbrt's "cameraworld" rendering
// space (cameras.cpp:51-56), triangles are flattened, and every spectrum the device
// evaluates is reduced to either sigmoid-polynomial coefficients (util/color.h:332) or a
// densely sampled 395..705 nm table (util/spectrum.h:400).
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../core/core.h"

namespace pbrt_amd {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

using Mat4 = std::array<std::array<double, 4>, 4>;
Mat4 Identity4();
Mat4 Mul(const Mat4 &a, const Mat4 &b);
Mat4 Inverse4(const Mat4 &m);
V3 XformPoint(const Mat4 &m, V3 p);
V3 XformVector(const Mat4 &m, V3 v);
V3 XformNormal(const Mat4 &mInv, V3 n);  // uses the inverse transpose
bool SwapsHandedness(const Mat4 &m);

enum MaterialType : int { kMatDiffuse = 0, kMatDielectric = 1, kMatConductor = 2, kMatNumTypes = 3 };
// Material "interface" (a null material: medium boundary only, materials.cpp); not a BxDF type
constexpr int kMatInterface = 3;
// LayeredBxDF materials (bxdfs.h:565-1052, materials.cpp:301-540); shaded by the volumetric
// kernels' layered stage
constexpr int kMatCoatedDiffuse = 4, kMatCoatedConductor = 5;
constexpr int kMatThinDielectric = 6;  // ThinDielectricBxDF (bxdfs.h:342-404), volumetric kernels
constexpr int kMatDiffuseTransmission = 7;  // DiffuseTransmissionBxDF (bxdfs.h:218-296), k_vlayered
// MixMaterial (materials.h:271-350): resolved per hit to one of its two materials by the
// closest-hit stage (wavefront/intersect.h:90-97); never shaded itself
constexpr int kMatMix = 8;
// HairMaterial (materials.h:353-427): HairBxDF (bxdfs.h:1054-1152), k_vlayered
constexpr int kMatHair = 9;
constexpr int kMatMeasured = 10;
// RetroreflectiveMaterial (this fork, materials.h:553-627): conductor parameters, RetroreflectiveBxDF, k_vlayered
constexpr int kMatRetroreflective = 11;

// Participating media (media.h:209-350, media.cpp:167-330).  Spectra are DenselySampled
// 395..705 nm tables in SceneDesc::denseSpectra with pbrt's constructor scaling applied
// (sigma_a/sigma_s *= "scale"; homogeneous Le *= "Lescale" / photometric).
// CloudMedium (media.h:430-525): procedural Perlin-noise density in [p0, p1], homogeneous majorant
enum MediumType : int { kMediumHomogeneous = 0, kMediumGrid = 1, kMediumCloud = 2, kMediumRGBGrid = 3 };
struct MediumDesc {
    int type = kMediumHomogeneous;
    std::string name;
    int sigmaA = -1, sigmaS = -1, Le = -1;  // denseSpectra indices
    float g = 0;
    bool emissive = false;
    // GridMedium ("uniformgrid")
    Mat4 renderFromMedium;                 // inverse applied to rays and points
    V3 p0{0, 0, 0}, p1{1, 1, 1};           // medium-space bounds
    int nx = 1, ny = 1, nz = 1;
    std::vector<float> density;            // [nz][ny][nx]; cloud: {density, wispiness, frequency}
                                           // followed by the 512-entry noise permutation
    int lnx = 1, lny = 1, lnz = 1;         // LeScale grid (1x1x1 = {1 / photometric(Le)})
    std::vector<float> LeScale;
    std::vector<float> majorant;           // 16^3 MaxValue of density per majorant voxel
    // GridMedium "temperature" (media.h:300-312): [nz][ny][nx] like density; Le at p is
    // LeScale(p) * BlackbodySpectrum((T(p) - temperatureOffset) * temperatureScale) when that
    // temperature exceeds 100 K
    std::vector<float> temperature;
    float temperatureOffset = 0, temperatureScale = 1;
    // RGBGridMedium ("rgbgrid"): density holds three [nz][ny][nx][4] blocks of {c0, c1, c2, scale}
    // (sigma_a, sigma_s, Le; bit k of rgbGrids: block k given), LeScale = {"Lescale"}
    int rgbGrids = 0;
    float sigmaScale = 0;
};

struct SssSpectrumDesc {
    int kind = 0;
    float value = 0, c0 = 0, c1 = 0, c2 = 0, scale = 1;
    int pl = -1;
};
struct MaterialDesc {
    int type = kMatDiffuse;
    // diffuse reflectance / conductor "reflectance": sigmoid (c0,c1,c2) or a constant value
    bool constant = false;
    float constantValue = 0.5f;
    float c0 = 0, c1 = 0, c2 = 0;
    // dielectric / conductor: TrowbridgeReitzDistribution alphas after RoughnessToAlpha (when
    // remaproughness) and the constructor's clamp (util/scattering.h:109-118)
    float alphaX = 0, alphaY = 0;
    float eta = 1.5f;              // dielectric: ConstantSpectrum eta (materials.cpp:51-60)
    int etaSpec = -1, kSpec = -1;  // conductor: SceneDesc::plSpectra indices; -1/-1 = reflectance
    // coateddiffuse / coatedconductor: alphaX/alphaY/eta are the interface's (DielectricBxDF),
    // c0..c2/constant the diffuse or conductor "reflectance", etaSpec/kSpec conductor.eta / .k
    float thickness = .01f, g = 0;
    int maxDepth = 10, nSamples = 1;
    bool albedoConstant = true;
    float albedoValue = 0, a0 = 0, a1 = 0, a2 = 0;  // layer albedo: constant or sigmoid
    float cAlphaX = 0, cAlphaY = 0;                 // conductor.{u,v}roughness -> alphas
    int ifaceEtaSpec = -1;                          // spectral interface eta (dispersion)
    float scale = 0;  // diffusetransmission "scale" (its transmittance uses the albedo fields)
    // textured parameters (SceneDesc::texPrograms index, -1: the constant fields above apply):
    // diffuse / conductor "reflectance" (SpectrumType::Albedo), {u,v}roughness (float)
    int texReflectance = -1, texURough = -1, texVRough = -1;
    bool remapRoughness = true;  // applied on the device when a roughness is textured
    // mix: the two materials and the "amount" texture program (constant or image)
    int mixMat[2] = {-1, -1};
    int texAmount = -1;
    // bump / normal mapping (materials.h:86-160): the displacement's program and node, the
    // normal map's image (SceneDesc::images); -1 when absent
    int texDisp = -1, dispNode = -1, normalMap = -1;
    // SubsurfaceMaterial: a dielectric-typed material (its DielectricBxDF from eta and the
    // alphas) with SceneDesc::sss[sss] as its BSSRDF; -1 for every other material
    int sss = -1;
    // HairMaterial (eta in `eta`): hairMode 0 sigma_a = ClampZero(hairSpec) (given, or the
    // eumelanin / pheomelanin RGB), 1 sigma_a = SigmaAFromReflectance(Clamp(hairSpec, 0, 1));
    // beta_m / beta_n are clamped to [0.01, 1] per hit as GetBxDF does
    int hairMode = 0;
    SssSpectrumDesc hairSpec;
    float hairBetaM = .3f, hairBetaN = .3f, hairAlpha = 2.f;
    // textured hair floats (GetFloatTexture, materials.cpp:135-184): programs for eta, beta_m,
    // beta_n, alpha, eumelanin, pheomelanin (-1: the constant above); the concentrations are
    // textured as a pair (a missing one is the constant 0), sigma_a then formed per hit
    int texHair[6] = {-1, -1, -1, -1, -1, -1};
    // textured subsurface spectra (materials.h:823-841, Unbounded): sigma_a, and sigma_s or mfp
    // (-1: the SubsurfaceDesc constant)
    int texSss[2] = {-1, -1};
    int measured = -1;  // MeasuredMaterial: its SceneDesc::measured entry
    std::string name;
};

// SubsurfaceMaterial's BSSRDF parameters (materials.h:772-866, materials.cpp:544-613): one of
// its four forms reduced to sigma_a / sigma_s (mode 0: named preset, given, or the defaults)
// or reflectance / mfp (mode 1, SubsurfaceFromDiffuse per wavelength), each a constant
// spectrum: kind 0 ConstantSpectrum(value), 1 scale * sigmoid(c0, c1, c2) (RGBUnbounded; an
// RGBAlbedo reflectance with scale 1), 2 PiecewiseLinearSpectrum SceneDesc::plSpectra[pl].
// The table is ComputeBeamDiffusionBSSRDF(g, eta) (host/bssrdf.cpp); fresnelC = 1 - 2
// FresnelMoment1(1 / eta) for NormalizedFresnelBxDF.
struct SubsurfaceDesc {
    int mode = 0;
    SssSpectrumDesc a, b;  // sigma_a, sigma_s | reflectance, mfp
    float scale = 1, eta = 1.33f, g = 0, fresnelC = 0;
    std::vector<float> table;
};

// ---- textures (textures.h / textures.cpp, util/mipmap.*, util/image.*) --------------------
// An image texture's MIPMap pyramid (Image::GeneratePyramid, util/image.cpp:313-383): every
// level is stored in the image's original pixel format (8-bit with its ColorEncoding, half or
// float), as pbrt stores it, so a lookup decodes exactly the values pbrt's GetChannel returns.
enum ImageFormat : int { kImgU8 = 0, kImgHalf = 1, kImgFloat = 2 };
enum WrapModeT : int { kWrapRepeat = 0, kWrapBlack = 1, kWrapClamp = 2, kWrapOctahedral = 3 };
struct ImageDesc {
    std::string filename;
    int format = kImgU8, nc = 3;
    int wrap = kWrapRepeat;
    std::vector<std::array<int, 2>> levelRes;  // level 0 = finest
    std::vector<uint64_t> levelOffset;         // byte offset of each level in data
    std::vector<uint8_t> data;                 // levels, row-major, nc channels interleaved
    std::array<float, 256> toLinear{};         // U8: ColorEncoding::ToLinear of every byte value
    // the decoded file before the pyramid (the CPU oracle builds its own pyramid from it)
    int rawW = 0, rawH = 0, encoding = 1;      // encoding: 0 linear, 1 sRGB, 2 gamma
    float gamma = 1;
    std::vector<uint8_t> raw;                  // rawW x rawH x nc texels in `format`
};

// Texture expression nodes.  The loader instantiates every named texture a material uses for
// the SpectrumType of that use (pbrt keeps one instance per type: scene.cpp CreateTextures).
enum TexKind : int {
    kTexConstant = 0, kTexScale = 1, kTexMix = 2, kTexDirectionMix = 3, kTexCheckerboard = 4,
    kTexBilerp = 5, kTexImage = 6,
    // procedural (textures.h:427-505, 813-841, 1117-1160): dots (float or spectrum: inside,
    // outside = child 0, 1), fbm / wrinkled / windy (float), marble (spectrum)
    kTexDots = 7, kTexFBm = 8, kTexWrinkled = 9, kTexWindy = 10, kTexMarble = 11
};
enum TexSpectrumType : int { kSpecAlbedo = 0, kSpecUnbounded = 1, kSpecIlluminant = 2 };
enum TexMapping : int { kMapUV = 0, kMapSpherical = 1, kMapCylindrical = 2, kMapPlanar = 3, kMap3D = 4 };
enum MIPFilter : int { kMipPoint = 0, kMipBilinear = 1, kMipTrilinear = 2, kMipEWA = 3 };
// A constant spectrum value of a spectrum texture: ConstantSpectrum(value) or an RGB spectrum
// of the node's type (RGBAlbedoSpectrum: sigmoid c0..c2; RGBUnboundedSpectrum: scale * sigmoid)
struct TexSpectrumConst {
    bool rgb = false;
    float value = 0;               // !rgb
    float c[3] = {0, 0, 0}, scale = 1;
};
struct TextureDesc {
    int kind = kTexConstant;
    bool spectrum = false;
    int specType = kSpecAlbedo;
    int child[3] = {-1, -1, -1};   // scale: tex, scale; mix: tex1, tex2, amount;
                                   // directionmix / checkerboard: tex1, tex2
    // TextureMapping2D (uv: su sv du dv; planar: vs, vt, ds dt) or the 3D point mapping
    int mapping = kMapUV;
    float map[4] = {1, 1, 0, 0};
    float textureFromRender[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};  // 3x4 row-major
    float vs[3] = {1, 0, 0}, vt[3] = {0, 1, 0};
    float fvalue[4] = {0, 0, 0, 0};   // float constant (fvalue[0]); bilerp v00 v01 v10 v11
    TexSpectrumConst svalue[4];       // spectrum constant (svalue[0]); bilerp v00 v01 v10 v11
    float dir[3] = {0, 1, 0};         // directionmix (render space, normalised)
    // image textures
    int image = -1, filter = kMipBilinear;
    float scale = 1, maxAniso = 8;  // scale: also marble's "scale"
    bool invert = false;
    // fbm / wrinkled / marble: "octaves", "roughness" (omega); marble "variation"
    int octaves = 8;
    float omega = .5f, variation = .2f;
    // multispectral basis ("basisfilename", this fork's --zhenyi addition): offset of the
    // texture's table in SceneDesc::texBasis, laid out as the reference's GPU basis array
    // (textures.cpp:1148-1176): {channels, basis length, int(offset), basis values channel by
    // channel}; -1 for an ordinary image
    int basis = -1, basisWidth = 0;
};

// A texture expression compiled for the device (core.h TexEval*): phase 1 runs once per hit
// and fills scalar registers (float sub-textures, image-texture RGB -> sigmoid coefficients,
// mix / bilerp weights); phase 2 (spectrum textures) runs per wavelength over those registers
// with a small value stack, in pbrt's operation order.
struct TexInstr {
    int op = 0, a = 0, b = 0, c = 0, node = -1;
};
struct TexProgram {
    bool spectrum = false;
    int p1 = 0, n1 = 0;   // phase-1 instructions [p1, p1 + n1)
    int p2 = 0, n2 = 0;   // phase-2 instructions
    int result = 0;       // float textures: the register holding the value
    int nRegs = 0;
    int root = -1;        // TextureDesc index (oracle: evaluates the tree itself)
};

// PiecewiseLinearSpectrum (util/spectrum.h:187-239): named spectra arrive already extended by
// FromInterleaved (util/spectrum.cpp:133-163), inline "spectrum" parameters as written
struct PLSpectrumDesc {
    std::vector<float> lambda, value;
};

struct AreaLightDesc {
    int prim = -1;          // triangle index in SceneDesc::tris (-1 for an analytic shape)
    int shape = -1;         // index in SceneDesc::shapes for a sphere / disk emitter
    int spectrum = -1;      // index into SceneDesc::denseSpectra
    float scale = 1;        // final DiffuseAreaLight::scale (lights.cpp:941-966)
    bool twoSided = false;
    float area = 0;
    // this fork's "spread" (lights.cpp:907-908, lights.h:451-458, 763-771): cosFalloffEnd =
    // cos(Radians(spread)) (> 0 only below 90 degrees), tanFalloffEnd = tan(Pi / 2 -
    // Radians(spread)), normalize_falloffEnd, all as the constructor computes them in float
    float cosFalloffEnd = -1, tanFalloffEnd = 0, normFalloffEnd = 0;
    // DiffuseAreaLight with "filename" (lights.cpp:909-936): index into
    // SceneDesc::areaLightImages (-1: the spectrum); L = scale * RGBIlluminantSpectrum of the
    // image bilerped at (u, 1 - v), spectrum then holds the colour space's illuminant
    int image = -1;
};
// an area light's emission image: linear R, G, B ([h][w][3], row 0 = top)
struct AreaLightImage {
    int w = 0, h = 0;
    std::vector<float> rgb;
};

// Sphere / Disk / BilinearPatch (shapes.h:106-571, 1272-1540) in render space: the device record (affine render-from-object
// and object-from-render matrices, parameters, orientation flags) and the shape's attributes.
// Primitive ids: leaf-order triangles first, then shape k as nTriangles + k.
struct AnalyticShapeDesc {
    DeviceShape dev{};
    std::array<float, 12> normals{};  // bilinear patch: render-space vertex normals (dev.flags bit 3)
    int material = -1;
    int light = -1;                   // area light index or -1
    int alpha = -1;                   // SceneDesc::alphaTex entry or -1
    int16_t medium[2] = {-1, -1};     // {inside, outside}
};

// An entry of BVHLightSampler's infinite-light list (lights without bounds, lightsamplers.cpp):
// a UniformInfiniteLight, or a DistantLight (distant = its index in SceneDesc::deltaLights)
// a UniformInfiniteLight, a DistantLight (distant = its index in SceneDesc::deltaLights) or an
// ImageInfiniteLight (image = its index in SceneDesc::envLights; spectrum = the colour space's
// illuminant, scale = the light's scale)
struct InfiniteLightDesc {
    int spectrum = -1;
    float scale = 1;
    int distant = -1;
    int image = -1;
};

// ImageInfiniteLight (lights.h:557-641, lights.cpp:1038-1071): an equal-area octahedral
// environment image of linear sRGB values (Image::GetChannel of the selected R, G, B channels)
// and the light's frame.  The device tables (per-pixel RGBIlluminantSpectrum coefficients and
// the compensated PiecewiseConstant2D) are derived from it at upload.
struct EnvLightDesc {
    int res = 0;                      // square: res x res
    std::vector<float> rgb;           // [res][res][3], row y = v * res
    float renderFromLight[9] = {};    // upper 3x3 of renderFromLight (row major)
    float lightFromRender[9] = {};    // upper 3x3 of its inverse (Transform::ApplyInverse)
    std::string filename;
    // PortalImageInfiniteLight (lights.h:644-744): the portal's corners in render space, its
    // frame (rows x, y, z), the rectified image [res][res][3] and its windowed sampling tables
    // (the distribution's function and the SummedAreaTable's sums as Float), BuildPortal
    bool portal = false;
    float portalP[4][3] = {};
    float portalFrame[9] = {};
    std::vector<float> rect, portalFunc, portalSat;
};
void BuildPortal(EnvLightDesc &e, const std::string &loc);
// SummedAreaTable (util/sampling.h:834-848) of the n x n function f: double running sums as Float
std::vector<float> SummedAreaTable(const std::vector<float> &f, int n);

// MeasuredBxDFData (bxdfs.cpp:865-1001): an RGL tensor file's tables as PiecewiseLinear2D's
// constructor leaves them, in core/measured.h's layout (kMeasHdr header ints, float blob)
struct MeasuredDesc {
    std::string path;
    std::vector<int> hdr;
    std::vector<float> blob;
};
MeasuredDesc LoadMeasuredBRDF(const std::string &path);
// PiecewiseLinear2D's constructor (util/sampling.h:1299-1400) over `slices` tables of xSize x ySize:
// appends data, marginal and conditional CDFs to blob; h = {xSize, ySize, data, marg, cond} offsets
// (-1 without a CDF)
void BuildPL2D(const float *data, int xSize, int ySize, uint32_t slices, bool normalize, bool buildCdf,
               std::vector<float> *blob, int *h);

// PointLight / SpotLight / DistantLight (lights.h:200-300, 740-800; lights.cpp:192-276, 1376-1495)
// in render space: deltaLights holds the point and spot lights first (light-BVH members, global
// light index nAreaLights + i), then the distant lights (members of the infinite-light list)
// GoniometricLight / ProjectionLight (lights.h:300-404, lights.cpp:281-680) are point lights
// whose intensity is an image lookup: they follow the point and spot lights in deltaLights.
enum DeltaLightType { kDeltaPoint = 0, kDeltaSpot = 1, kDeltaDistant = 2, kDeltaGonio = 3, kDeltaProjection = 4 };
struct DeltaLightDesc {
    int type = kDeltaPoint;
    V3 p;                 // point / spot: renderFromLight(0, 0, 0)
    V3 w;                 // spot, projection: Normalize(renderFromLight(0, 0, 1)); distant: renderFromLight(0, 0, 1)
    float m[3][3] = {};   // spot, goniometric, projection: upper 3x3 of renderFromLight's inverse
                          // (Transform::ApplyInverse; the swapYZ / flip-y of Create folded in)
    float cosFalloffStart = 1, cosFalloffEnd = 1;  // spot; goniometric / projection: LightBounds'
                                                   // cosTheta_o, cosTheta_e
    int spectrum = -1;    // dense spectrum of I (point, spot, goniometric), L (distant), or the
                          // image colour space's illuminant (projection)
    float scale = 1;      // final scale (photometric normalisation, power / illuminance applied)
    // goniometric: the Y image (Image::GetChannel values, res x res, row 0 = top); projection:
    // per pixel the RGBIlluminantSpectrum {c0, c1, c2, scale} of ClampZero(rgb)
    std::vector<float> img;
    int imgW = 0, imgH = 0;
    float invTanAng = 1;  // projection: 1 / tan(Radians(fov) / 2) of screenFromLight
    float phi = 0;        // goniometric / projection: LightBounds' phi (Bounds(), lights.cpp:384-399, 563-575)
};

struct CameraDesc {
    Mat4 cameraFromRaster;   // ProjectiveCamera (cameras.h:266-285)
    Mat4 renderFromCamera;   // CameraTransform (cameras.cpp:43-73)
    Mat4 renderFromWorld;
    float lensRadius = 0, focalDistance = 1e6f;
    float shutterOpen = 0, shutterClose = 1;
    float fov = 90;
};

struct LightBVHNodeDesc {
    LightNodeBounds bounds;  // decoded CompactLightBounds
    int childOrLight = 0;    // second child index for interior, light index for leaf
    int isLeaf = 0;
};

struct SceneDesc {
    std::vector<float> texBasis;        // multispectral basis tables (TextureDesc::basis)
    int options = 0;                    // kOpt* bits (core.h)
    float displacementEdgeScale = 1;    // Option "displacementedgescale" (no displaced meshes here)
    // film / sampler / integrator
    int xres = 1280, yres = 720;
    int px0 = 0, px1 = 1280, py0 = 0, py1 = 720;  // pixel bounds
    int spp = 16, seed = 0, maxDepth = 5;
    std::string samplerName = "zsobol";
    std::string integratorName = "volpath";
    bool regularize = false;
    std::string outFile = "pbrt.exr";
    float filterRadiusX = 0.5f, filterRadiusY = 0.5f;  // box (scene.cpp:94 fork default)
    std::string filterName = "box";
    int filterType = 0;             // core.h FilterType
    float filterA = 0, filterB = 0; // gaussian sigma; mitchell B, C; sinc tau
    // FilterSampler tables (gaussian / mitchell / sinc; core.h FilterTableView layout)
    int filterNu = 0, filterNv = 0;
    std::vector<float> filterTable;
    float imagingRatio = 1;
    std::string sensorName = "cie1931";
    int filmColorSpace = 0;                    // RGBFilm's colour space (the Film directive's graphics state)
    float whiteBalance = 0;                    // Film "whitebalance" (0: none)
    float maxComponentValue = kInfinity;       // RGBFilm::AddSample clamp (film.h:247-249)
    float xyzFromSensorRGB[3][3];              // PixelSensor::XYZFromSensorRGB
    double outputRGBFromSensorRGB[3][3];
    CameraDesc camera;

    // geometry (render space)
    std::vector<V3> verts;
    std::vector<std::array<int, 3>> tris;
    std::vector<int> triMaterial;   // material index
    std::vector<int> triLight;      // area light index or -1
    std::vector<uint8_t> triFlip;   // reverseOrientation ^ transformSwapsHandedness
    std::vector<AreaLightImage> areaLightImages;
    std::vector<int> triAlpha;      // alphaTex entry or -1 (GeometricPrimitive alpha test)
    // alpha textures: {texture node, compiled float program}; shapes refer to them by index
    std::vector<std::array<int, 2>> alphaTex;
    // shading attributes (TriangleMesh n / uv, util/mesh.cpp:23-68): per vertex, meaningful
    // only for triangles whose triShade bit says so (bit0 normals, bit1 uv)
    std::vector<V3> vertN;                       // render space, reverseOrientation applied
    std::vector<std::array<float, 2>> vertUV;
    std::vector<V3> vertS;  // per-vertex shading tangents, render space (triShade bit2)
    std::vector<uint8_t> triShade;
    std::vector<AnalyticShapeDesc> shapes;  // spheres and disks

    std::vector<MaterialDesc> materials;
    std::vector<SubsurfaceDesc> sss;  // MaterialDesc::sss
    std::vector<MeasuredDesc> measured;  // MaterialDesc::measured (one per file)
    std::vector<MediumDesc> media;
    int cameraMedium = -1;                          // -1: vacuum
    std::vector<std::array<int16_t, 2>> triMedium;  // {inside, outside}; empty if no media
                                                    // a triangle changes the ray's medium
                                                    // only when inside != outside
    std::vector<AreaLightDesc> areaLights;
    std::vector<InfiniteLightDesc> infiniteLights;
    std::vector<EnvLightDesc> envLights;
    std::vector<DeltaLightDesc> deltaLights;  // point and spot lights first, then distant lights
    int nPointSpot = 0;
    // pbrt's light order (area lights, then LightSource lights as written) -> this scene's global
    // light index (area, point/spot, infinite list); UniformLightSampler picks in pbrt's order
    std::vector<int> uniformOrder;
    float sceneRadius = 0;  // Bounds3f::BoundingSphere of the scene bounds (DistantLight::Preprocess)
    std::vector<std::array<float, 311>> denseSpectra;
    std::vector<PLSpectrumDesc> plSpectra;
    std::array<float, 311> sensorX, sensorY, sensorZ;  // r_bar/g_bar/b_bar of "cie1931"

    // BVH light sampler (lightsamplers.cpp:112-236); unused when one light -> uniform
    bool uniformLightSampler = false;
    std::vector<LightBVHNodeDesc> lightNodes;
    std::vector<uint32_t> lightBitTrail;  // per light-BVH light (area, then point/spot)

    // sampler: 0 = HaltonSampler (permutedigits), 1 = ZSobolSampler (samplers.h:225-370)
    int samplerType = 1;
    // Randomize of zsobol / sobol / paddedsobol: 0 none, 1 permutedigits, 2 fastowen, 3 owen
    int zsRandomize = 2;
    int stratXs = 4, stratYs = 4, stratJitter = 1;  // StratifiedSampler
    int sobolLog2Scale = 0;                         // SobolSampler: Log2(RoundUpPow2(max(xres, yres)))
    int zsLog2SamplesPerPixel = 0, zsNBase4Digits = 0;

    // Halton digit permutations (util/lowdiscrepancy.cpp:47-55) for the dimensions used
    int haltonBaseScales[2] = {1, 1}, haltonBaseExponents[2] = {0, 0}, haltonMultInverse[2] = {0, 0};
    std::vector<uint16_t> permTable;       // concatenated nDigits*base rows per dimension
    std::vector<uint32_t> permOffset;      // per dimension: offset into permTable
    std::vector<uint32_t> permNDigits;     // per dimension
    std::vector<uint32_t> permBase;        // per dimension (prime)

    // textures: expression nodes, images (MIPMap pyramids), compiled programs
    std::vector<TextureDesc> textures;
    std::vector<ImageDesc> images;
    std::vector<TexProgram> texPrograms;
    std::vector<TexInstr> texInstrs;
    // CameraBase::FindMinimumDifferentials (cameras.cpp:170-216) and CameraFromRender, for
    // Approximate_dp_dxy (cameras.h:167-195); filled when a material is textured
    float cameraFromRender[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    float minPosDx[3] = {0, 0, 0}, minPosDy[3] = {0, 0, 0}, minDirDx[3] = {0, 0, 0}, minDirDy[3] = {0, 0, 0};
};

// Loaders and builders
SceneDesc LoadPbrtFile(const std::string &path, const std::map<std::string, std::string> &overrides);
SceneDesc LoadPbrtString(const std::string &text, const std::string &baseDir,
                         const std::map<std::string, std::string> &overrides);
void FinalizeScene(SceneDesc &s);  // lights, light BVH, sampler tables
// BVHLightSampler::buildBVH over given LightBounds ([n][13]: pMin3 pMax3 w3 phi cosTheta_o
// cosTheta_e twoSided); trails[i] = 0xffffffff for a light left out (phi == 0)
void DebugBuildLightBVH(const float *in13, int n, std::vector<LightBVHNodeDesc> *nodes, std::vector<uint32_t> *trails);
// the 24 four-way digit permutations of ZSobolSampler::GetSampleIndex, in pbrt's order
// FilterSampler ctor (filters.cpp:133-147): tabulates the scene's filter and its
// PiecewiseConstant1D ctor (util/sampling.h:625-649): func = |f|, normalised cdf; returns funcInt
float BuildPC1D(const float *f, int n, float mn, float mx, float *func, float *cdf);
// ImageInfiniteLight's compensated PiecewiseConstant2D (FilterTableView layout, domain [0,1]^2)
std::vector<float> BuildEnvDistribution(const EnvLightDesc &e);
// PiecewiseConstant2D (util/sampling.h:603-790) into SceneDesc::filterTable
void BuildFilterTable(SceneDesc &s);
extern const uint8_t kZSobolPermutations[24][4];

// Spectral support (host)
// The RGB colour spaces of RGBColorSpace::Init (util/colorspace.cpp:83-105), selected by the
// ColorSpace directive (scene.cpp:108-115) and carried per parameter (ParsedParameter::colorSpace)
enum ColorSpaceId { kColorSpaceSRGB = 0, kColorSpaceDCIP3 = 1, kColorSpaceRec2020 = 2, kColorSpaceACES = 3 };
constexpr int kNumColorSpaces = 4;
struct ColorSpaceDef {
    const char *name;        // RGBColorSpace::GetNamed's (lower case)
    double prim[6];          // r, g, b chromaticities (xy)
    const char *illuminant;  // named illuminant spectrum
};
extern const ColorSpaceDef kColorSpaceDefs[kNumColorSpaces];
struct ColorSpaceDesc {
    std::string name;
    float prim[6];                       // r, g, b (xy)
    float w[2];                          // SpectrumToXYZ(illuminant).xy()
    std::array<float, 311> illuminant;   // DenselySampledSpectrum(illuminant), 395..705
    float photometric = 0;               // SpectrumToPhotometric(illuminant)
    double xyzFromRGB[3][3], rgbFromXYZ[3][3];  // solved in double (the loader's historical form)
    float xyzFromRGBf[3][3], rgbFromXYZf[3][3];  // pbrt's float arithmetic, bit for bit
};
const ColorSpaceDesc &GetColorSpace(int cs);
// SquareMatrix<3> product as pbrt forms it (compensated InnerProduct per entry)
void MulCompensated3(const float a[3][3], const float b[3][3], float r[3][3]);
int ColorSpaceByName(const std::string &name);  // -1 when unknown
struct SpectralData {
    std::vector<float> cieX, cieY, cieZ, cieLambda, d65Interleaved;
    std::vector<double> optX, optY, optZ, optD65Raw, optXyzToSrgb, optSrgbToXyz;
    std::vector<double> optD60Raw, optXyzToRgb[kNumColorSpaces], optRgbToXyz[kNumColorSpaces];  // rgb2spec_opt gamuts
    std::map<std::string, std::vector<float>> named;  // interleaved (lambda, value) tables
    std::map<std::string, std::vector<float>> illuminants;  // stdillum-*, illum-acesD60 (normalised on use)
    double optD65Divisor = 1, optD60Divisor = 1;
    std::array<float, 311> denseX, denseY, denseZ, denseD65;  // 395..705
    float photometricD65 = 0;                                  // SpectrumToPhotometric(D65)
    double rgbFromXYZ[3][3];
    double xyzFromRGB[3][3];  // sRGB; row 1 = RGBColorSpace::LuminanceVector (colorspace.h:51-53)
    std::array<float, 256> srgbToLinear;  // SRGBToLinearLUT (util/color.cpp:286)
    std::array<float, 128> mipFilterLUT;  // MIPFilterLUT (util/mipmap.cpp:59-191)
    std::map<std::string, std::vector<float>> sensors;  // "<camera>_r|g|b" interleaved curves
    std::vector<float> cieSLambda, cieS0, cieS1, cieS2;  // CIE daylight basis (Spectra::D)
    std::vector<float> noisePerm;                        // util/noise.cpp NoisePerm[512]
    std::vector<std::vector<float>> swatches;           // 24 ColorChecker reflectances (film.cpp)
    // GetMediumScatteringProperties presets (media.cpp:74-151): sigma_prime_s RGB, sigma_a RGB
    std::map<std::string, std::array<float, 6>> mediumPresets;
};
// PixelSensor (film.h:36-116, PixelSensor::Create film.cpp:222-262): the sensor's r/g/b matching
// curves densely sampled over 395..705 nm and XYZFromSensorRGB -- the CIE 1931 curves with an
// optional white balance (Bradford, util/color.h WhiteBalance), or a named camera's curves with
// the matrix fitted by LinearLeastSquares to the 24 swatches under the D(whitebalance)
// illuminant (6500 K when unspecified).  Throws for an unknown sensor.
struct PixelSensorDesc {
    std::array<float, 311> r, g, b;
    float xyzFromSensorRGB[3][3];
    std::array<float, 311> illum;  // the white-balance illuminant (zeros without one)
};
PixelSensorDesc BuildPixelSensor(const std::string &name, float whiteBalanceTemp, int cs = kColorSpaceSRGB);
// BlackbodySpectrum(T)(lambda) (util/spectrum.h): normalised to 1 at Wien's peak
float BlackbodyNormalized(float lambda, float T);
// Spectra::D(T) (util/spectrum.cpp:2537-2570) densely sampled over 395..705
std::array<float, 311> DenseCIEDaylight(float T);
// The whole 64^3 sRGB RGBToSpectrumTable (cmd/rgb2spec_opt.cpp output): zNodes[64] then
// data[3][64][64][64][3]; loaded from data/rgbspec_srgb.bin (written by the build), computed
// in parallel (and cached there) when the file is absent
const std::vector<float> &RGBToSpectrumTableData();
// util/sobolmatrices.cpp's tables, from data/sobol_tables.bin (oracle/ref/gen_golden.py writes it
// from the reference's compiled tables): SobolMatrices32 [1024 * 52], then VdCSobolMatrices and
// VdCSobolMatricesInv [25 * 52]; throws when the file is absent or malformed
struct SobolTableData {
    std::vector<uint32_t> m32;
    std::vector<uint64_t> vdc, vdcInv;
};
const SobolTableData &SobolTables();
const SpectralData &GetSpectralData();
void SetDataDirectory(const std::string &dir);
std::string GetDataDirectory();
// RGB -> sigmoid coefficients through the 64^3 sRGB table (util/color.cpp:36-75); table
// columns are generated on demand with the rgb2spec Gauss-Newton restatement.
std::array<float, 3> RGBToSigmoidCoeffs(float r, float g, float b, int cs = kColorSpaceSRGB);
// Column (maxc, yi, xi) of colour space cs's 64^3 table as cmd/rgb2spec_opt.cpp produces it
// (gamut sRGB / DCI_P3 / REC2020 / ACES2065_1): 64 x 3 floats
std::vector<float> RGB2SpecColumn(int maxc, int j, int i, int cs = kColorSpaceSRGB);
float RGB2SpecZNode(int k);
std::array<float, 311> DenseRGBIlluminant(float r, float g, float b, int cs = kColorSpaceSRGB);
std::array<float, 311> DenseRGBUnbounded(float r, float g, float b, int cs = kColorSpaceSRGB);
// GetNamedSpectrum(name) for the metal / glass tables: PiecewiseLinearSpectrum::FromInterleaved
// (samples, normalize = false), extended to Lambda_min - 1 / Lambda_max + 1 (spectrum.cpp:133-163)
PLSpectrumDesc NamedPiecewiseLinear(const std::string &name);

// Hash / permutation (util/hash.h:19, util/math.h:728)
uint64_t MurmurHash64A(const unsigned char *key, size_t len, uint64_t seed);
const std::vector<int> &Primes();

// host/bssrdf.cpp
std::vector<float> ComputeBeamDiffusionTable(float g, float eta);
float FresnelMoment1(float eta);
float FresnelMoment2(float eta);

}  // namespace pbrt_amd
