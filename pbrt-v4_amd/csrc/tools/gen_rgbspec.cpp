// Build step: writes data/rgbspec_srgb.bin, the full 64^3 sRGB RGBToSpectrumTable (the output of
// the reference's cmd/rgb2spec_opt.cpp, restated in csrc/host/spectra.cpp), as pbrt's build
// generates rgbspectrum_srgb.cpp.  Image textures look up arbitrary RGB values on the device.
#include <cstdio>

#include "../host/scene.h"

int main(int argc, char **argv) {
    pbrt_amd::SetDataDirectory(argc > 1 ? argv[1] : "data");
    const std::vector<float> &t = pbrt_amd::RGBToSpectrumTableData();
    std::printf("rgbspec_srgb.bin: %zu floats\n", t.size());
    return 0;
}
