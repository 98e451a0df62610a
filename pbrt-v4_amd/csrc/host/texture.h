// Image textures on the host (texture.cpp): readers, colour encodings, MIPMap pyramid.
#pragma once

#include <array>
#include <string>
#include <vector>

#include "scene.h"
#include "../core/texture_eval.h"

namespace pbrt_amd {

// ColorEncoding (util/color.h:420-538): linear, sRGB or "gamma g"
enum EncodingKind : int { kEncLinear = 0, kEncSRGB = 1, kEncGamma = 2 };
struct Encoding {
    int kind = kEncSRGB;
    float gamma = 1;
    std::array<float, 256> applyLUT{};
    std::array<float, 1024> inverseLUT{};
    static Encoding Get(const std::string &name, const std::string &loc);
    float ToLinear(uint8_t v) const;
    float ToFloatLinear(float v) const;
    uint8_t FromLinear(float v) const;
};

uint16_t FloatToHalf(float f);
float HalfToFloat(uint16_t h);
float LinearToSRGB(float v);
float SRGBToLinear(float v);
uint8_t LinearToSRGB8(float v);

// MIPMap::CreateFromFile (util/mipmap.cpp:377-417) with Image::GeneratePyramid
ImageDesc LoadImageTexture(const std::string &filename, const std::string &encoding, int wrap, const std::string &loc);
// the decoded value of a stored texel (Image::GetChannel with the image's wrap mode)
float ImageTexel(const ImageDesc &img, int level, int x, int y, int c);
// Image::Read + GetChannelDesc({"R", "G", "B"}) for an ImageInfiniteLight (lights.cpp:1600-1681):
// PNG (sRGB encoding), PFM or EXR; linear values as Image::GetChannel returns them; square
EnvLightDesc LoadEnvironmentImage(const std::string &filename, const std::string &loc);
// Image::Read of a goniometric / projection light's image: every channel's linear value as
// Image::GetChannel returns it ([h][w][nc], row 0 = top), and the stored pixel format
struct LightImage {
    int w = 0, h = 0, nc = 0;
    int format = kImgFloat;
    bool exr = false;
    std::vector<float> v;
    // a value stored into an image of this format and read back (Image::SetChannel + GetChannel)
    float Restore(float v) const;
};
LightImage LoadLightImage(const std::string &filename, const std::string &loc);
// lowers texture node `node` (scene.textures) to a two-phase device program; returns its index
// Texture tables in the device layout (core/texture_eval.h), built on the host: uploaded by
// BuildDevice, viewed in place by the host debug entry points, handed to the oracle by
// pbrt_scene_get_flat.
struct TexTables {
    std::vector<DeviceTexNode> nodes;
    std::vector<DeviceTexSpec> spec;
    std::vector<DeviceImage> images;
    std::vector<DeviceImageLevel> levels;
    std::vector<uint8_t> data;
    std::vector<float> luts;
    std::vector<DeviceTexInstr> instrs;
    std::vector<DeviceTexProgram> progs;
    std::vector<int32_t> matTex;      // [nMaterials][4] program indices + remap
    std::vector<int32_t> matTexNode;  // [nMaterials][4] the programs' root nodes + remap (oracle)
    std::vector<int32_t> matMixNode;  // [nMaterials][4] mix: material 0, 1, amount root node, 0
    std::vector<int32_t> matBumpNode; // [nMaterials][2] displacement root node, normal map image
    std::vector<int32_t> matHairNode; // [nMaterials][6] hair eta beta_m beta_n alpha eumelanin pheomelanin root nodes
    bool anyHairTex = false;
    std::vector<int32_t> matSssNode;  // [nMaterials][2] subsurface sigma_a, sigma_s | mfp root nodes
    bool anySssTex = false;
    std::vector<int32_t> nodeInfo, imageInfo, levelInfo, rawInfo;
    std::vector<float> nodeParams, specFlat, rawGamma;
    std::vector<uint8_t> rawData;
    std::vector<uint64_t> rawOffset;
    std::vector<float> basis;  // multispectral basis tables (never empty: one pad entry)
};
void BuildTexTables(const SceneDesc &s, TexTables *t);
// a TexView over host copies (the device view points at DevBufs)
TexView HostTexView(const TexTables &t);
// FloatTexture::Evaluate of compiled program prog on the host
float HostTexFloat(const TexView &T, int prog, const TexEvalCtx &c);
int CompileTexProgram(SceneDesc &s, int node, bool spectrum);
// CameraBase::FindMinimumDifferentials and CameraFromRender (SceneDesc::minPosDx ...)
void ComputeCameraDifferentials(SceneDesc &s);

}  // namespace pbrt_amd
