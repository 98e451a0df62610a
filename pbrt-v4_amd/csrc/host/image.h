// Image output / input and imgtool's error metrics (host side; see image.cpp)
#pragma once

#include <array>
#include <string>
#include <vector>

namespace pbrt_amd {

struct Image {
    int width = 0, height = 0;
    std::vector<float> rgb;  // [height][width][3], row 0 = top
};

// by extension: .pfm (float), .exr (half unless exrHalf = false), .png (8-bit sRGB).
// window = {x0, y0, fullW, fullH}: rgb is the w x h pixelBounds region at (x0, y0) of a
// fullW x fullH film; EXR records it as dataWindow inside displayWindow (null: whole frame).
// chroma8 (EXR only): the r, g, b, white chromaticities written as the "chromaticities" attribute
// (Image::WriteEXR writes them for a colour space other than sRGB, util/image.cpp:1231-1242)
void WriteImage(const std::string &path, const float *rgb, int w, int h, bool exrHalf = true,
                const int *window = nullptr, const float *chroma8 = nullptr);
Image ReadImage(const std::string &path);  // .pfm, .exr (uncompressed scanline)

enum class ErrorMetric { MAE = 0, MSE = 1, MRSE = 2, FLIP = 3 };
std::array<double, 3> ImageError(const float *img, const float *ref, int w, int h, ErrorMetric metric);
// FLIP error per pixel ([h][w]) of RGB images test vs reference (imgtool --metric FLIP)
std::vector<float> FlipErrorMap(const float *test, const float *ref, int w, int h);

}  // namespace pbrt_amd
