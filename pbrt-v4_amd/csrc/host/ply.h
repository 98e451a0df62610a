// PLY reader (TriQuadMesh::ReadPLY, util/mesh.cpp:322-420) for Shape "plymesh".
#pragma once

#include <array>
#include <string>
#include <vector>

#include "scene.h"

namespace pbrt_amd {

struct PlyMesh {
    std::vector<V3> p, n;                       // n empty unless nx/ny/nz are all present
    std::vector<std::array<float, 2>> uv;       // empty unless a (u,v)-style pair is present
    std::vector<int> triIndices, quadIndices;   // quads in rply's bilinear-patch order 0 1 3 2
    std::vector<int> faceIndices;
    int skippedFaces = 0;                       // polygons with other than 3 or 4 vertices
};

PlyMesh ReadPly(const std::string &filename);

}  // namespace pbrt_amd
