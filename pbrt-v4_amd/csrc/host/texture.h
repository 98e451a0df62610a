// Image textures on the host (texture.cpp): readers, colour encodings, MIPMap pyramid.
#pragma once

#include <array>
#include <string>

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
int CompileTexProgram(SceneDesc &s, int node, bool spectrum);
// CameraBase::FindMinimumDifferentials and CameraFromRender (SceneDesc::minPosDx ...)
void ComputeCameraDifferentials(SceneDesc &s);

}  // namespace pbrt_amd
