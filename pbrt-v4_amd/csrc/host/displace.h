// Displacement of "plymesh" shapes by a float texture at load time (shapes.cpp:1418-1478):
// TriQuadMesh::Displace (util/mesh.h:91-122) -- quads split into triangles
// (ConvertToOnlyTriangles, util/mesh.cpp:425-442), vertex normals computed when the mesh has
// none (ComputeNormals, util/mesh.cpp:444-467), every triangle refined by edge bisection until
// its edges are shorter than the edge length in render space (TriQuadMesh::Refine,
// util/mesh.h:134-191), each vertex moved along its normal by the texture's value at its
// object-space position and uv, and the normals recomputed.
#pragma once

#include <array>
#include <functional>
#include <vector>

#include "../core/core.h"

namespace pbrt_amd {

struct DisplaceMesh {
    std::vector<V3> p, n;                     // object space
    std::vector<std::array<float, 2>> uv;     // required (pbrt: "Vertex uvs are currently required")
    std::vector<int> tri, quad;               // quad: p00 p10 p01 p11 per patch
};

// renderFromObject as pbrt's float Transform (row-major 4x4) for the edge lengths;
// displacement(p, u, v) = the texture's value at that object-space point and uv.
void DisplaceTriQuadMesh(DisplaceMesh *m, const float renderFromObject[16], float maxEdge,
                         const std::function<float(V3 p, float u, float v)> &displacement);

// util/mesh.cpp:425-442 / 444-467, on their own
void ConvertToOnlyTriangles(DisplaceMesh *m);
void ComputeVertexNormals(DisplaceMesh *m);

}  // namespace pbrt_amd
