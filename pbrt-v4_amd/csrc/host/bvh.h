// Geometry BVH for the device: binned-SAH binary build in the manner of pbrt's
// BVHAggregate::buildRecursive (cpu/aggregates.cpp:192-387: 12 buckets, leaf cost =
// primitive count, 1/2 traversal cost) collapsed into an 8-wide tree whose nodes are laid
// out for wave64 traversal (one 256-byte node = 8 child boxes in SoA + 8 child refs).
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../core/core.h"

namespace pbrt_amd {

// Child reference: >= 0 interior node index; < 0 leaf = ~(triStart << 3 | (count-1));
// kEmptyChild marks an unused slot (its box is empty).
constexpr int32_t kEmptyChild = (int32_t)0x80000000;

struct alignas(16) BVH8Node {
    float lox[8], loy[8], loz[8];
    float hix[8], hiy[8], hiz[8];
    int32_t child[8];
    int32_t nChildren;
    int32_t pad[7];
};
static_assert(sizeof(BVH8Node) == 256, "BVH8Node must be 256 bytes");

struct BVH8 {
    std::vector<BVH8Node> nodes;
    // triangles in leaf order: 3 float4 per triangle = p0.xyz|prim, p1.xyz|0, p2.xyz|0
    std::vector<float> triVerts;
    std::vector<int> triPrim;  // leaf order -> original triangle index
    int maxDepth = 0;
    int maxStack = 0;  // worst-case traversal stack entries (farthest-first pushes)
    V3 boundsMin, boundsMax;
};

BVH8 BuildBVH8(const std::vector<V3> &verts, const std::vector<std::array<int, 3>> &tris, int maxLeafPrims = 4);

}  // namespace pbrt_amd
