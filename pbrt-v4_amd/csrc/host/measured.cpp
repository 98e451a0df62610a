// MeasuredBxDFData::Create (bxdfs.cpp:894-993) and the RGL tensor file it reads (Tensor,
// bxdfs.cpp:690-816): the fields' structure checks, then PiecewiseLinear2D's constructor
// (util/sampling.h:1336-1438) per table -- double sums, float normalisation -- into the blob
// core/measured.h reads on the host and the device.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <stdexcept>

#include "../core/measured.h"
#include "scene.h"

namespace pbrt_amd {

namespace {

struct TensorField {
    int dtype = 0;  // Tensor::Type: 1 UInt8 ... 10 Float32, 11 Float64
    std::vector<size_t> shape;
    std::vector<uint8_t> data;
};

size_t TypeSize(int t) {
    static const size_t sz[] = {0, 1, 1, 2, 2, 4, 4, 8, 8, 2, 4, 8};
    return t >= 0 && t <= 11 ? sz[t] : 0;
}

std::map<std::string, TensorField> ReadTensorFile(const std::string &path) {
    std::ifstream in(path, std::ios::binary);
    if (!in) throw std::runtime_error(path + ": unable to open file");
    auto fail = [&](const char *msg) { throw std::runtime_error(path + ": Tensor: " + msg); };
    in.seekg(0, std::ios::end);
    const size_t size = (size_t)in.tellg();
    in.seekg(0);
    if (size < 12 + 2 + 4) fail("Invalid tensor file: too small, truncated?");
    char header[12];
    uint8_t version[2];
    uint32_t nFields = 0;
    in.read(header, 12);
    in.read((char *)version, 2);
    in.read((char *)&nFields, 4);
    if (std::memcmp(header, "tensor_file", 12) != 0) fail("Invalid tensor file: invalid header.");
    if (version[0] != 1 || version[1] != 0) fail("Invalid tensor file: unknown file version.");
    std::map<std::string, TensorField> fields;
    for (uint32_t i = 0; i < nFields; ++i) {
        uint16_t nameLen = 0, ndim = 0;
        uint8_t dtype = 0;
        uint64_t offset = 0;
        in.read((char *)&nameLen, 2);
        std::string name(nameLen, '\0');
        in.read(name.data(), nameLen);
        in.read((char *)&ndim, 2);
        in.read((char *)&dtype, 1);
        in.read((char *)&offset, 8);
        if (!in) fail("Unable to read the field header.");
        if (dtype == 0 || dtype > 11) fail("Invalid tensor file: unknown type.");
        TensorField f;
        f.dtype = dtype;
        size_t total = TypeSize(dtype);
        for (int j = 0; j < ndim; ++j) {
            uint64_t v = 0;
            in.read((char *)&v, 8);
            f.shape.push_back((size_t)v);
            total *= (size_t)v;
        }
        if (!in || offset + total > size) fail("Unable to read data.");
        const auto cur = in.tellg();
        f.data.resize(total);
        in.seekg((std::streamoff)offset);
        in.read((char *)f.data.data(), (std::streamsize)total);
        in.seekg(cur);
        fields[name] = std::move(f);
    }
    return fields;
}

}  // namespace

// PiecewiseLinear2D<D>(data, xSize, ySize, paramRes, ..., normalize, buildCdf): appends the
// density values (and the CDFs) to blob; h = {sx, sy, data, marginal, conditional}
void BuildPL2D(const float *data, int xSize, int ySize, uint32_t slices, bool normalize, bool buildCdf,
               std::vector<float> *blob, int *h) {
    const size_t nValues = (size_t)xSize * ySize;
    h[0] = xSize;
    h[1] = ySize;
    std::vector<float> out(slices * nValues), marg, cond;
    const float invPatch = (float)(xSize - 1) * (float)(ySize - 1);  // HProd(m_inv_patch_size)
    if (buildCdf) {
        marg.resize((size_t)slices * ySize);
        cond.resize(slices * nValues);
        for (uint32_t sl = 0; sl < slices; ++sl) {
            const float *d = data + sl * nValues;
            float *cc = cond.data() + sl * nValues, *mc = marg.data() + (size_t)sl * ySize, *o = out.data() + sl * nValues;
            for (int y = 0; y < ySize; ++y) {
                double sum = 0.0;
                size_t i = (size_t)y * xSize;
                cc[i] = 0.f;
                for (int x = 0; x < xSize - 1; ++x, ++i) {
                    sum += .5 * ((double)d[i] + (double)d[i + 1]);
                    cc[i + 1] = (float)sum;
                }
            }
            mc[0] = 0.f;
            double sum = 0.0;
            for (int y = 0; y < ySize - 1; ++y) {
                sum += .5 * ((double)cc[(size_t)(y + 1) * xSize - 1] + (double)cc[(size_t)(y + 2) * xSize - 1]);
                mc[y + 1] = (float)sum;
            }
            const float normalization = 1.f / mc[ySize - 1];
            for (size_t i = 0; i < nValues; ++i) cc[i] *= normalization;
            for (int i = 0; i < ySize; ++i) mc[i] *= normalization;
            for (size_t i = 0; i < nValues; ++i) o[i] = d[i] * normalization;
        }
    } else {
        for (uint32_t sl = 0; sl < slices; ++sl) {
            const float *d = data + sl * nValues;
            float *o = out.data() + sl * nValues;
            float normalization = 1.f / invPatch;
            if (normalize) {
                double sum = 0.0;
                for (int y = 0; y < ySize - 1; ++y) {
                    size_t i = (size_t)y * xSize;
                    for (int x = 0; x < xSize - 1; ++x, ++i) {
                        const float v00 = d[i], v10 = d[i + 1], v01 = d[i + xSize], v11 = d[i + 1 + xSize],
                                    avg = .25f * (v00 + v10 + v01 + v11);
                        sum += (double)avg;
                    }
                }
                normalization = float(1.0 / sum);
            }
            for (size_t k = 0; k < nValues; ++k) o[k] = d[k] * normalization;
        }
    }
    auto append = [&](const std::vector<float> &v) {
        if (v.empty()) return -1;
        const int off = (int)blob->size();
        blob->insert(blob->end(), v.begin(), v.end());
        return off;
    };
    h[2] = append(out);
    h[3] = append(marg);
    h[4] = append(cond);
}

MeasuredDesc LoadMeasuredBRDF(const std::string &path) {
    const auto tf = ReadTensorFile(path);
    auto field = [&](const char *n) -> const TensorField & {
        auto it = tf.find(n);
        if (it == tf.end()) throw std::runtime_error(path + ": invalid BRDF file structure: no field \"" + n + "\"");
        return it->second;
    };
    const TensorField &theta_i = field("theta_i"), &phi_i = field("phi_i"), &ndf = field("ndf"),
                      &sigma = field("sigma"), &vndf = field("vndf"), &spectra = field("spectra"),
                      &luminance = field("luminance"), &wavelengths = field("wavelengths"),
                      &description = field("description"), &jacobian = field("jacobian");
    constexpr int U8 = 1, F32 = 10;
    const bool ok =
        description.shape.size() == 1 && description.dtype == U8 && theta_i.shape.size() == 1 &&
        theta_i.dtype == F32 && phi_i.shape.size() == 1 && phi_i.dtype == F32 && wavelengths.shape.size() == 1 &&
        wavelengths.dtype == F32 && ndf.shape.size() == 2 && ndf.dtype == F32 && sigma.shape.size() == 2 &&
        sigma.dtype == F32 && vndf.shape.size() == 4 && vndf.dtype == F32 && vndf.shape[0] == phi_i.shape[0] &&
        vndf.shape[1] == theta_i.shape[0] && luminance.shape.size() == 4 && luminance.dtype == F32 &&
        luminance.shape[0] == phi_i.shape[0] && luminance.shape[1] == theta_i.shape[0] &&
        luminance.shape[2] == luminance.shape[3] && spectra.dtype == F32 && spectra.shape.size() == 5 &&
        spectra.shape[0] == phi_i.shape[0] && spectra.shape[1] == theta_i.shape[0] &&
        spectra.shape[2] == wavelengths.shape[0] && spectra.shape[3] == spectra.shape[4] &&
        luminance.shape[2] == spectra.shape[3] && luminance.shape[3] == spectra.shape[4] &&
        jacobian.shape.size() == 1 && jacobian.shape[0] == 1 && jacobian.dtype == U8;
    if (!ok) throw std::runtime_error(path + ": invalid BRDF file structure");
    auto f32 = [](const TensorField &f) { return (const float *)f.data.data(); };
    const int nPhi = (int)phi_i.shape[0], nTheta = (int)theta_i.shape[0], nW = (int)wavelengths.shape[0];
    auto minSize = [&](const TensorField &f, size_t a, size_t b) {
        if (f.shape[a] < 2 || f.shape[b] < 2) throw std::runtime_error(path + ": invalid BRDF file structure");
    };
    minSize(ndf, 0, 1);
    minSize(sigma, 0, 1);
    minSize(vndf, 2, 3);
    minSize(luminance, 2, 3);
    MeasuredDesc m;
    m.path = path;
    m.hdr.assign(kMeasHdr, 0);
    m.hdr[0] = nPhi <= 2;
    if (!m.hdr[0]) {
        const float *p = f32(phi_i);
        const int reduction = (int)std::rint((2 * kPi) / (p[nPhi - 1] - p[0]));
        if (reduction != 1)
            throw std::runtime_error(path + ": reduction " + std::to_string(reduction) + " (!= 1) not supported");
    }
    m.hdr[1] = nPhi;
    m.hdr[2] = nTheta;
    m.hdr[3] = nW;
    auto put = [&](const float *v, size_t n) {
        const int off = (int)m.blob.size();
        m.blob.insert(m.blob.end(), v, v + n);
        return off;
    };
    m.hdr[4] = put(f32(phi_i), nPhi);
    m.hdr[5] = put(f32(theta_i), nTheta);
    m.hdr[6] = put(f32(wavelengths), nW);
    const uint32_t s2 = (uint32_t)(nPhi * nTheta), s3 = s2 * (uint32_t)nW;
    BuildPL2D(f32(ndf), (int)ndf.shape[1], (int)ndf.shape[0], 1, false, false, &m.blob, &m.hdr[8 + 5 * kMeasNdf]);
    BuildPL2D(f32(sigma), (int)sigma.shape[1], (int)sigma.shape[0], 1, false, false, &m.blob, &m.hdr[8 + 5 * kMeasSigma]);
    BuildPL2D(f32(vndf), (int)vndf.shape[3], (int)vndf.shape[2], s2, true, true, &m.blob, &m.hdr[8 + 5 * kMeasVndf]);
    BuildPL2D(f32(luminance), (int)luminance.shape[3], (int)luminance.shape[2], s2, true, true, &m.blob,
              &m.hdr[8 + 5 * kMeasLum]);
    BuildPL2D(f32(spectra), (int)spectra.shape[4], (int)spectra.shape[3], s3, false, false, &m.blob,
              &m.hdr[8 + 5 * kMeasSpectra]);
    if (m.blob.size() > (size_t)INT32_MAX) throw std::runtime_error(path + ": measured BRDF too large");
    return m;
}

}  // namespace pbrt_amd
