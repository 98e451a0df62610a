// Geometry BVH for the device: a binned-SAH binary build after pbrt's
// BVHAggregate::buildRecursive (cpu/aggregates.cpp:192-387: leaf cost = primitive count, 1/2
// traversal cost), binned over all three axes with 32 buckets (pbrt: the longest axis, 12) and
// keeping quad halves as one leaf (bvh.cpp), optionally with spatial splits, collapsed into an
// 8-wide tree whose nodes are laid out for wave64 traversal (one 256-byte node = 8 child boxes
// in SoA + 8 child refs).
#pragma once

#include <array>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../core/core.h"

namespace pbrt_amd {

// Child reference (host-side view, BVH8::childRef): >= 0 interior node index; < 0 leaf =
// ~(triStart << 3 | (count-1)); kEmptyChild marks an unused slot (its box is empty).
constexpr int32_t kEmptyChild = (int32_t)0x80000000;
// Leaves hold at most 4 triangles, so a node's (at most 8) leaves address at most 32
// triangles: one 32-bit mask relative to the node's triBase covers them all.
constexpr int kMaxLeafPrims = 4;

// Wide node (256 B), laid out for the device's group traversal (common.h TraverseCW):
//  * child boxes in SoA (12 float4: lo x/y/z then hi x/y/z, children 0-3 then 4-7), so the near
//    and far planes of 4 children are one float4 load at a per-ray offset (no per-child select);
//  * children sit in "octant slots": slot s holds the child nearest to the entry side of rays
//    whose direction-sign octant is s, so a ray visits slots in the order i ^ octant without
//    sorting (Ylitie, Karras, Laine 2017, "Efficient incoherent ray traversal on GPUs through
//    compressed wide BVHs", section 3.2);
//  * interior children are consecutive nodes from childBase (in slot order) and the node's leaf
//    triangles are consecutive from triBase; triMask[c] lists slot c's triangles as bits
//    relative to triBase (0 for an interior or empty slot).
struct alignas(16) BVH8Node {
    float lox[8], loy[8], loz[8];
    float hix[8], hiy[8], hiz[8];
    int32_t childBase, triBase;
    uint32_t imask;  // bit c: slot c is an interior node
    uint32_t occ;    // bit c: slot c is occupied (interior or leaf)
    uint32_t triMask[8];
    int32_t pad[4];
};
static_assert(sizeof(BVH8Node) == 256, "BVH8Node must be 256 bytes");

// Compressed BVH8 node (80 B, the quantised wide-node layout of Ylitie et al. 2017): child
// boxes as 8-bit offsets on a per-node grid lo = fma(q, 2^(e-127), p), rounded outward on the
// host with the same fma the device decodes with, so every decoded box contains the exact one.
// Interior children are contiguous from childBase (in slot order); a node's leaf triangles are
// contiguous from triBase.  meta[c]: 0 = empty or interior, else count << 5 | offset (count 1-4),
// so slot c's triangle bits are ((1 << (meta >> 5)) - 1) << (meta & 31) with no special case.
struct alignas(16) BVH8QNode {
    float px, py, pz;
    uint8_t ex, ey, ez;
    uint8_t imask;  // bit c: child c is an interior node
    int32_t childBase, triBase;
    uint8_t meta[8];
    uint8_t qlox[8], qloy[8], qloz[8], qhix[8], qhiy[8], qhiz[8];
};
static_assert(sizeof(BVH8QNode) == 80, "BVH8QNode must be 80 bytes");

// decoded plane of a quantised box: the device evaluates exactly this expression
inline float DecodeQ(uint8_t q, uint8_t e, float p) {
    uint32_t bits = (uint32_t)e << 23;
    float s;
    memcpy(&s, &bits, 4);
    return fmaf((float)q, s, p);
}

struct BVH8 {
    std::vector<BVH8Node> nodes;
    std::vector<BVH8QNode> qnodes;  // the same tree, compressed (same node indices)
    std::vector<std::array<int32_t, 8>> childRef;  // per node and slot (host view, kEmptyChild)
    // triangles in leaf order: 3 float4 per triangle = p0.xyz|prim, p1.xyz|0, p2.xyz|0
    std::vector<float> triVerts;
    std::vector<int> triPrim;  // leaf order -> original triangle index
    int maxDepth = 0;
    int maxStack = 0;  // worst-case traversal stack entries (one pending child group per level)
    V3 boundsMin, boundsMax;
};

// spatial: 1 = spatial splits (a triangle may be listed by several leaves), 0 = object splits
// only, -1 = PBRT_AMD_BVH_SBVH
BVH8 BuildBVH8(const std::vector<V3> &verts, const std::vector<std::array<int, 3>> &tris,
               int maxLeafPrims = kMaxLeafPrims, int spatial = -1);

}  // namespace pbrt_amd
