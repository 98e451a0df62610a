// Device helpers shared by the wavefront kernels (wavefront.hip: surface-only paths) and the
// participating-media kernels (volpath.hip): queues, samplers, BVH8 traversal, light sampling,
// camera rays and spectral accumulation.
#pragma once
#include <hip/hip_runtime.h>

#include "device.h"

namespace pbrt_amd {

constexpr int kBlock = 256;
#ifndef PBRT_TRAVERSAL_WAVES
#define PBRT_TRAVERSAL_WAVES 4  // waves/SIMD the closest/shadow kernels are compiled for
#endif
// Grid caps of the queue kernels (blocks; each loops grid-stride over its queue).  Traversal
// kernels fill their LDS scene cache once per block, so the grid is bounded, but 8192 blocks
// (32 per CU) balance the tail better than 1024/2048 did: C2 +8 % (k_closest 960 -> 845 us
// per launch, profiles/r02_grid_caps.txt).
#ifndef PBRT_GRID_CAP
#define PBRT_GRID_CAP 8192
#endif
#ifndef PBRT_SHADE_GRID_CAP
#define PBRT_SHADE_GRID_CAP 8192
#endif
// Quantised-node traversal (80-B nodes, HBM-resident trees) is compiled for more waves: its
// node loads hold 20 VGPRs instead of 60, and on C4 (10 M triangles) the traversal is bound by
// dependent-load latency, so waves in flight are what pays (k_closest 65.1 -> 54.6 ms per pass:
// wide at 4, quantised at 4 / 5 / 6 waves = 65.1 / 66.9 / 66.9 / 54.6 ms; tools/gpu_c4_occ.sh)
#ifndef PBRT_QUANT_TRAVERSAL_WAVES
#define PBRT_QUANT_TRAVERSAL_WAVES 6
#endif
#ifndef PBRT_SHADE_WAVES
#define PBRT_SHADE_WAVES 3  // waves/SIMD the shade kernel is compiled for (VGPR budget)
#endif
constexpr float kInvWavelengthPDF = kLambdaMax - kLambdaMin;  // 1 / SampleUniformWavelengths pdf

// ------------------------------------------------------------------ helpers
// Section timing (profiling build only): wave-level s_memtime deltas summed per section by the
// wave's first active lane into stats[kStatsSectionBase + k].
#ifdef PBRT_AMD_SECTION_TIMING
#define SEC_BEGIN() unsigned long long secT_ = __builtin_amdgcn_s_memtime()
#define SEC_MARK(st, k)                                                                          \
    do {                                                                                         \
        unsigned long long n_ = __builtin_amdgcn_s_memtime();                                    \
        if (__lane_id() == __ffsll((long long)__ballot(1)) - 1)                                   \
            atomicAdd(&(st).stats[kStatsSectionBase + (k)], n_ - secT_);                         \
        secT_ = n_;                                                                              \
    } while (0)
#else
#define SEC_BEGIN() (void)0
#define SEC_MARK(st, k) (void)0
#endif
// The record slot of a producer's queue position pos in its shard: a full shard (pos >= capS; the
// counter keeps counting, so the pass's k_queue_overflow check fails the render) sends the record
// to the trash slot NR - 1 past every shard instead of into the next shard or past the arrays
__device__ inline int ShardSlot(int shardBase, int pos, int capS, int NR) {
    return pos < capS ? shardBase + pos : NR - 1;
}
__device__ inline int WavePush(int *counter, bool pred) {
    unsigned long long mask = __ballot(pred);
    if (mask == 0) return -1;
    int lane = __lane_id();
    int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(mask));
    base = __shfl(base, leader);
    return pred ? base + __popcll(mask & ((1ull << lane) - 1ull)) : -1;
}

// Append to up to K queues: one global atomicAdd per wave and queue on the producer block's
// shard counter (ballot + popcount prefix), so no block barrier makes a wave wait for the
// slowest wave of its block.  With sharded counters this measured 2 % faster on the shade
// kernel than a block-aggregated append (one atomic per block, three barriers), which
// PBRT_SHADE_PUSH_BLOCK still selects.  Lanes of a wave receive consecutive slots.
template <int K>
__device__ inline void BlockPush(int *const (&counters)[K], const bool (&pred)[K], int (&pos)[K]) {
#ifndef PBRT_SHADE_PUSH_BLOCK
    // The wave's first active lane issues every queue's atomic back to back, so their round
    // trips overlap (one WavePush after another waits out each return in turn).
    unsigned long long mask[K];
#pragma unroll
    for (int k = 0; k < K; ++k) mask[k] = __ballot(pred[k]);
    const int lane = __lane_id();
    const int leader = __ffsll((long long)__ballot(1)) - 1;
    int base[K];
#pragma unroll
    for (int k = 0; k < K; ++k) base[k] = 0;
    if (lane == leader) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (mask[k]) base[k] = atomicAdd(counters[k], __popcll(mask[k]));
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int b = __builtin_amdgcn_readfirstlane(base[k]);
        pos[k] = pred[k] ? b + __popcll(mask[k] & ((1ull << lane) - 1ull)) : -1;
    }
#else
    constexpr int kWaves = kBlock / 64;
    __shared__ int sCount[K][kWaves];
    __shared__ int sBase[K];
    const int lane = __lane_id(), wave = threadIdx.x >> 6;
    unsigned long long mask[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        mask[k] = __ballot(pred[k]);
        if (lane == 0) sCount[k][wave] = __popcll(mask[k]);
    }
    __syncthreads();
    if (threadIdx.x < K) {
        const int k = threadIdx.x;
        int tot = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) tot += sCount[k][w];
        sBase[k] = tot ? atomicAdd(counters[k], tot) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        int b = sBase[k];
        for (int w = 0; w < wave; ++w) b += sCount[k][w];
        pos[k] = pred[k] ? b + __popcll(mask[k] & ((1ull << lane) - 1ull)) : -1;
    }
    __syncthreads();  // sCount/sBase are reused by the next call
#endif
}

// Block-wide global -> LDS copies by LDS-DMA (global_load_lds_*): no VGPR round trip and no
// wait per element, so a prologue of several tables costs one memory latency.  Each wave
// copies 64 consecutive elements per instruction (LDS destination = wave base + lane * size);
// lanes past the end are masked.  Callers finish with DmaWait() and one __syncthreads().
template <int Bytes>  // 4 or 16 (sub-dword LDS-DMA does not pack lanes)
__device__ inline void DmaCopy(const void *src, void *ldsDst, int n) {
    const int lane = __lane_id(), wave = threadIdx.x >> 6, nWaves = blockDim.x >> 6;
    for (int base = wave * 64; base < n; base += nWaves * 64) {
        if (base + lane < n) {
            auto g = (const __attribute__((address_space(1))) void *)((const char *)src + (size_t)(base + lane) * Bytes);
            auto l = (__attribute__((address_space(3))) void *)((char *)ldsDst + (size_t)base * Bytes);
            // the builtin's size operand must be a literal
            static_assert(Bytes == 4 || Bytes == 16, "DmaCopy: 4- or 16-byte elements");
            if constexpr (Bytes == 4) __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
            else __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
        }
    }
}
__device__ inline void DmaWait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Block-local staging of queue appends: entries collect in an LDS buffer across the block's
// grid-stride iterations (one LDS atomic per wave) and are written out in contiguous runs with
// one global atomicAdd per flush, i.e. every ~cap/256 iterations instead of every iteration.
// All threads of the block must call Append/FlushAll (the grid-stride loops are block-uniform).
template <int K, int Cap>
struct BlockQueues {
    int *buf;   // LDS [K][Cap]
    int *fill;  // LDS [K]
    int *gbase; // LDS [K]
    int *const *counters;
    int *const *queues;
    int capS;

    __device__ void Init() {
        if (threadIdx.x < K) fill[threadIdx.x] = 0;
        __syncthreads();
    }
    __device__ void Flush(int k) {
        const int n = fill[k];
        if (threadIdx.x == 0) gbase[k] = n ? atomicAdd(counters[k], n) : 0;
        __syncthreads();
        const int b = gbase[k];
        int *q = queues[k];
        for (int i = threadIdx.x; i < n; i += blockDim.x)
            if (b + i < capS) q[b + i] = buf[k * Cap + i];  // a full shard drops (k_queue_overflow)
        __syncthreads();
        if (threadIdx.x == 0) fill[k] = 0;
        __syncthreads();
    }
    __device__ void Append(const bool (&pred)[K], int slot) {
        const int lane = __lane_id();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned long long mask = __ballot(pred[k]);
            const int n = __popcll(mask);
            int b = 0;
            if (lane == 0 && n) b = atomicAdd(&fill[k], n);  // LDS atomic
            b = __shfl(b, 0);
            if (pred[k]) buf[k * Cap + b + __popcll(mask & ((1ull << lane) - 1ull))] = slot;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (fill[k] > Cap - kBlock) Flush(k);  // block-uniform: read after the barrier
    }
    __device__ void FlushAll() {
#pragma unroll
        for (int k = 0; k < K; ++k) Flush(k);
    }
};

// Wave-local staging of queue appends: each wave owns a Cap-entry LDS buffer per queue, fills
// it with ballot/popcount prefixes and writes it out in a contiguous run with one global
// atomicAdd when it would overflow (and at the end).  No block barriers: a wave never waits
// for the slowest wave of its block, unlike BlockQueues.
template <int K, int Cap>
struct WaveQueues {
    int *buf;  // LDS: this wave's [K][Cap]
    int fill[K];
    int *const *counters;
    int *const *queues;
    int capS;

    __device__ WaveQueues(int *ldsAll, int *const *c, int *const *q, int cap) : counters(c), queues(q), capS(cap) {
        buf = ldsAll + (threadIdx.x >> 6) * (K * Cap);
#pragma unroll
        for (int k = 0; k < K; ++k) fill[k] = 0;
    }
    __device__ void Flush(int k) {
        const int n = fill[k];
        if (n == 0) return;
        int b = 0;
        if (__lane_id() == 0) b = atomicAdd(counters[k], n);
        b = __shfl(b, 0);
        int *q = queues[k];
        for (int i = __lane_id(); i < n; i += 64)
            if (b + i < capS) q[b + i] = buf[k * Cap + i];  // a full shard drops (k_queue_overflow)
        fill[k] = 0;
    }
    __device__ void Append(const bool (&pred)[K], int value) {
        const int lane = __lane_id();
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned long long mask = __ballot(pred[k]);
            const int n = __popcll(mask);
            if (fill[k] + n > Cap) Flush(k);
            if (pred[k]) buf[k * Cap + fill[k] + __popcll(mask & ((1ull << lane) - 1ull))] = value;
            fill[k] += n;
        }
    }
    __device__ void FlushAll() {
#pragma unroll
        for (int k = 0; k < K; ++k) Flush(k);
    }
};

// A sharded queue as its consumer sees it: per-shard counts (uniform, scalar loads) and the
// map from a dense item index j to the item's physical index (shard * capS + offset).
struct QueueView {
    int count[kShards];
    int total, capS;
};
__device__ inline QueueView LoadQueue(const PathState &st, int depth, int queue) {
    QueueView v;
    v.total = 0;
    v.capS = st.capS;
#pragma unroll
    for (int s = 0; s < kShards; ++s) {
        // never more than a shard holds: an overflowing producer dropped the rest, and the pass
        // fails at its k_queue_overflow check without reading past the shard.  The depth-0 ray
        // queue is exempt: the camera stage keeps every path's ray in shard 0 (slot = path)
        const int c = st.counters[CounterIndex(depth, queue, s)];
        v.count[s] = (depth == 0 && queue == 0) ? c : min(c, st.capS);
        v.total += v.count[s];
    }
    return v;
}
__device__ inline int QueueSlot(const QueueView &v, int j) {
    int base = 0, shard = 0;
#pragma unroll
    for (int s = 0; s < kShards - 1; ++s) {
        const bool later = j >= base + v.count[s];
        base += later ? v.count[s] : 0;
        shard += later ? 1 : 0;
        if (!later) break;
    }
    return shard * v.capS + (j - base);
}
__device__ inline int ProducerShard() { return blockIdx.x % kShards; }

// XCD-grouped walk over [0, count) in blockDim-sized chunks (guide T1).  Blocks b and b + 8 are
// observed to share an XCD and its 4 MiB L2, so runs of k consecutive chunks (super-chunks) are
// dealt round-robin to those eight block groups: rays adjacent in the queue (bin order, or pixel
// order at depth 0) meet the same L2 instead of being dealt chunk by chunk over all eight, and
// the round-robin keeps the groups' work balanced (one contiguous eighth per group was measured
// 18 % slower on C4: the sorted order's cost varies by region).  Super-chunks of 16 measured
// neutral on C4 (k_closest 7434 vs 7410 us per launch, films bit-identical), so the default is
// k = 0 (PBRT_AMD_XCD_GROUPS selects k).  Speed only -- every chunk is walked exactly once under
// any placement.  k = 0 (or a grid that is not a multiple of 8) is the plain grid-stride walk.
// Uniform per block, so a block whose walk is empty may return.
struct ChunkWalk {
    int n, end, step, k, g;
    __device__ int Chunk() const { return k ? ((n / k) * 8 + g) * k + n % k : n; }
};
__device__ inline ChunkWalk XcdChunks(int count, int k) {
    const int chunks = (count + (int)blockDim.x - 1) / (int)blockDim.x;
    if (k <= 0 || (gridDim.x & 7u)) return {(int)blockIdx.x, chunks, (int)gridDim.x, 0, 0};
    const int g = blockIdx.x & 7u, rounds = chunks / (8 * k), rem = chunks - rounds * 8 * k;
    const int mine = rounds * k + min(k, max(0, rem - g * k));
    return {(int)(blockIdx.x >> 3), mine, (int)(gridDim.x >> 3), k, g};
}

__device__ inline V3 XfPoint(const float *m, V3 p) {
    float xp = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    float yp = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    float zp = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wp = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wp == 1) return V3(xp, yp, zp);
    return V3(xp, yp, zp) / wp;
}
__device__ inline V3 XfVector(const float *m, V3 v) {
    return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}

struct Halton {
    uint64_t index;
    int dimension;
};

__device__ inline Halton StartPixelSample(const DeviceScene &S, int px, int py, int sampleIndex, int dim) {
    // samplers.h:53-71
    Halton h;
    h.index = 0;
    if (S.haltonFast32) {
        // Same terms in 32-bit arithmetic: the host checked that the stride and every partial
        // sum fit (stride * (scale0 + scale1) < 2^32), so no 64-bit division is needed.
        const uint32_t stride = (uint32_t)S.baseScales[0] * (uint32_t)S.baseScales[1];
        uint32_t pmx = (uint32_t)px & 127u, pmy = (uint32_t)py & 127u;  // Mod(p, 128), p >= 0
        uint32_t i0 = (uint32_t)InverseRadicalInverse((uint64_t)pmx, 2, S.baseExponents[0]);
        uint32_t i1 = 0;
        for (int k = 0; k < S.baseExponents[1]; ++k) {
            uint32_t q = pmy / 3u;
            i1 = i1 * 3u + (pmy - 3u * q);
            pmy = q;
        }
        uint32_t t = i0 * (uint32_t)S.baseScales[1] * (uint32_t)S.multInverse[0] +
                     i1 * (uint32_t)S.baseScales[0] * (uint32_t)S.multInverse[1];
        h.index = (uint64_t)(t % stride) + (uint64_t)sampleIndex * stride;
        h.dimension = dim < 2 ? 2 : dim;
        return h;
    }
    uint64_t sampleStride = (uint64_t)S.baseScales[0] * S.baseScales[1];
    if (sampleStride > 1) {
        int pmx = px % 128, pmy = py % 128;
        if (pmx < 0) pmx += 128;
        if (pmy < 0) pmy += 128;
        h.index += InverseRadicalInverse((uint64_t)pmx, 2, S.baseExponents[0]) * (sampleStride / S.baseScales[0]) *
                   (uint64_t)S.multInverse[0];
        h.index += InverseRadicalInverse((uint64_t)pmy, 3, S.baseExponents[1]) * (sampleStride / S.baseScales[1]) *
                   (uint64_t)S.multInverse[1];
        h.index %= sampleStride;
    }
    h.index += (uint64_t)sampleIndex * sampleStride;
    h.dimension = dim < 2 ? 2 : dim;
    return h;
}
__device__ __forceinline__ float SampleDim(const DeviceScene &S, uint64_t index, int dim) {
    return HaltonSampleDimension(S.haltonDim[dim], index, S.perm);
}
__device__ inline float Get1D(const DeviceScene &S, Halton &h) {
    if (h.dimension >= S.nDims) h.dimension = 2;
    return SampleDim(S, h.index, h.dimension++);
}
__device__ inline void Get2D(const DeviceScene &S, Halton &h, float *u0, float *u1) {
    if (h.dimension + 1 >= S.nDims) h.dimension = 2;
    int dim = h.dimension;
    h.dimension += 2;
    *u0 = SampleDim(S, h.index, dim);
    *u1 = SampleDim(S, h.index, dim + 1);
}

__device__ inline void PixelOf(const PathState &st, int slot, int *px, int *py, int *sampleIndex) {
    int s = slot / st.P, pl = slot - s * st.P;
    int r = pl / st.width;
    *px = pl - r * st.width;
    *py = st.rows[r];
    *sampleIndex = st.firstSample + s;
}

// ------------------------------------------------------------------ BVH8 traversal
// One ray per lane, compressed-wide-BVH group traversal (Ylitie, Karras, Laine 2017): a visited
// node yields (a) a bit mask of its hit leaf triangles, relative to the node's triBase, tested
// right away, and (b) the group of its hit interior children as a bit mask in visit order
// (slot i ^ octant, nearest first: BVH8Node's octant slots).  The traversal descends into the
// group's first child and keeps the rest of the group as ONE stack entry {childBase,
// imask << 8 | remaining bits}, so the stack grows by at most one entry per tree level and no
// child distances are sorted or stored.
//
// Box test: Bounds3::IntersectP (util/vecmath.h:1576-1611) decides only which nodes are
// visited, never a hit's value, so any test that accepts every box the exact real-arithmetic
// test accepts gives the same closest hit (and the same first-found any-hit candidate set).
// Plane distances are one fma each, t = fma(plane, 1/d, -o/d -/+ m), with a per-ray absolute
// margin m_a = (4 M_a + 3 |o_a|) |1/d_a| 8u (M_a bounds every plane coordinate, u = 2^-24)
// that exceeds the rounding of 1/d, -o/d and the fma together: near distances are rounded
// down and far distances up, so a box is culled only when the exact test culls it.  Zero
// direction components are replaced by a same-signed 1e-20 so every distance stays finite.
// Triangle test = IntersectTriangle (shapes.cpp:172-273), bit for bit.

struct CwRay {
    V3 inv;     // 1 / d (zero components replaced by +-1e-20)
    V3 oN, oF;  // -o * inv - m, -o * inv + m
    int nOff[3], fOff[3];  // float4 index (within a wide node) of axis a's near / far planes
    uint32_t oct;          // bit a: d_a < 0 (Bounds3 dirIsNeg)
};
__device__ inline CwRay MakeCwRay(V3 o, V3 d, const float *absMax) {
    CwRay r;
    auto safe = [](float x) { return fabsf(x) < 1e-20f ? copysignf(1e-20f, x) : x; };
    r.inv = V3(1 / safe(d.x), 1 / safe(d.y), 1 / safe(d.z));
    r.oct = (r.inv.x < 0 ? 1u : 0u) | (r.inv.y < 0 ? 2u : 0u) | (r.inv.z < 0 ? 4u : 0u);
    constexpr float k8u = 8.f / 16777216.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float c = -o[a] * r.inv[a];
        const float m = (4 * absMax[a] + 3 * fabsf(o[a])) * fabsf(r.inv[a]) * k8u;
        r.oN[a] = c - m;
        r.oF[a] = c + m;
        const int neg = (r.oct >> a) & 1;
        r.nOff[a] = 2 * a + 6 * neg;
        r.fOff[a] = 2 * a + 6 * (1 - neg);
    }
    return r;
}

// IntersectTriangle with the ray's axis permutation applied once per ray: kz = the largest
// |d| axis, (kx, ky, kz) a rotation, so permuting a vertex is a rotation by kz.  Triangles
// cached in LDS are stored pre-rotated (three copies, one per kz); global ones are rotated here.
struct TriRayR {
    V3 o;  // permuted origin
    float Sx, Sy, Sz;
    int kz;
};
__device__ inline TriRayR MakeTriRayR(V3 o, V3 dir) {
    const TriRay t = MakeTriRay(o, dir);
    TriRayR r;
    r.o = Permute(o, t.kx, t.ky, t.kz);
    r.Sx = t.Sx, r.Sy = t.Sy, r.Sz = t.Sz;
    r.kz = t.kz;
    return r;
}
__device__ inline V3 RotateToRay(float4 v, int kz) {
    // (v[kx], v[ky], v[kz]) with kx = kz + 1, ky = kz + 2 (mod 3)
    return V3(kz == 0 ? v.y : (kz == 1 ? v.z : v.x), kz == 0 ? v.z : (kz == 1 ? v.x : v.y),
              kz == 0 ? v.x : (kz == 1 ? v.y : v.z));
}
// shapes.cpp:180-273 on already permuted vertices (same arithmetic and order as
// IntersectTriangleRay: p - o commutes with the permutation)
__device__ inline bool IntersectTriangleRot(const TriRayR &r, float tMax, V3 p0t, V3 p1t, V3 p2t, TriHit *hit) {
    p0t = p0t - r.o;
    p1t = p1t - r.o;
    p2t = p2t - r.o;
    const float Sx = r.Sx, Sy = r.Sy, Sz = r.Sz;
    p0t.x += Sx * p0t.z;
    p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z;
    p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z;
    p2t.y += Sy * p2t.z;
    float e0 = DifferenceOfProducts(p1t.x, p2t.y, p1t.y, p2t.x);
    float e1 = DifferenceOfProducts(p2t.x, p0t.y, p2t.y, p0t.x);
    float e2 = DifferenceOfProducts(p0t.x, p1t.y, p0t.y, p1t.x);
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {
        const EdgeFns e = EdgeFunctionsFP64(p0t, p1t, p2t);
        e0 = e.e0, e1 = e.e1, e2 = e.e2;
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    const float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz;
    p1t.z *= Sz;
    p2t.z *= Sz;
    const float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < tMax * det)) return false;
    if (det > 0 && (tScaled <= 0 || tScaled > tMax * det)) return false;
    const float invDet = 1 / det;
    const float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    const float t = tScaled * invDet;
    const float maxZt = MaxComponentValue(Abs(V3(p0t.z, p1t.z, p2t.z)));
    const float deltaZ = gamma(3) * maxZt;
    const float maxXt = MaxComponentValue(Abs(V3(p0t.x, p1t.x, p2t.x)));
    const float maxYt = MaxComponentValue(Abs(V3(p0t.y, p1t.y, p2t.y)));
    const float deltaX = gamma(5) * (maxXt + maxZt);
    const float deltaY = gamma(5) * (maxYt + maxZt);
    const float deltaE = 2 * (gamma(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    const float maxE = MaxComponentValue(Abs(V3(e0, e1, e2)));
    const float deltaT = 3 * (gamma(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::fabs(invDet);
    if (t <= deltaT) return false;
    hit->b0 = b0;
    hit->b1 = b1;
    hit->b2 = b2;
    hit->t = t;
    return true;
}

// Visit order bits: visit index i <-> slot i ^ oct, i.e. the slot mask with its index bits
// XOR-permuted by oct (three conditional swaps).
__device__ inline uint32_t PermuteOct(uint32_t m, uint32_t oct) {
    m = (oct & 1u) ? (((m & 0x55u) << 1) | ((m >> 1) & 0x55u)) : m;
    m = (oct & 2u) ? (((m & 0x33u) << 2) | ((m >> 2) & 0x33u)) : m;
    m = (oct & 4u) ? (((m & 0x0fu) << 4) | ((m >> 4) & 0x0fu)) : m;
    return m;
}

// One visited node's outcome
struct NodeHits {
    uint32_t inner;  // hit interior slots (slot order)
    uint32_t tris;   // hit leaf triangles, bits relative to triBase
    uint32_t imask;
    int childBase, triBase;
};

// Wide node (BVH8Node): 12 plane float4 at q[0..11], header q[12] = {childBase, triBase, imask,
// occ}, slot triangle masks q[13..14].  Near/far planes of 4 children are one float4 each.
template <typename F4>
__device__ inline NodeHits VisitWide(const F4 *__restrict__ q, const CwRay &r, float tMax) {
    const float4 hdr = q[12], tm0 = q[13], tm1 = q[14];
    NodeHits o;
    o.childBase = __float_as_int(hdr.x);
    o.triBase = __float_as_int(hdr.y);
    o.imask = __float_as_uint(hdr.z);
    uint32_t hit = 0, tris = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const float4 nx = q[r.nOff[0] + g], ny = q[r.nOff[1] + g], nz = q[r.nOff[2] + g];
        const float4 fx = q[r.fOff[0] + g], fy = q[r.fOff[1] + g], fz = q[r.fOff[2] + g];
        const float4 tm = g ? tm1 : tm0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            auto comp = [k](float4 v) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
            const float tn = fmaxf(fmaxf(fmaf(comp(nx), r.inv.x, r.oN.x), fmaf(comp(ny), r.inv.y, r.oN.y)),
                                   fmaxf(fmaf(comp(nz), r.inv.z, r.oN.z), 0.f));
            const float tf = fminf(fminf(fmaf(comp(fx), r.inv.x, r.oF.x), fmaf(comp(fy), r.inv.y, r.oF.y)),
                                   fminf(fmaf(comp(fz), r.inv.z, r.oF.z), tMax));
            const bool ok = tn <= tf;
            hit |= ok ? 1u << (4 * g + k) : 0u;
            tris |= ok ? __float_as_uint(comp(tm)) : 0u;
        }
    }
    o.inner = hit & o.imask;
    o.tris = tris;
    return o;
}

// Quantised node (BVH8QNode, 5 float4): child planes P = fma(q, 2^(e-127), p) -- the expression
// the host rounded outward -- folded into the distance: t = fma(q, 2^(e-127) / d, (p - o) / d
// -/+ m); the margin bound M_a covers the decoded planes too (DeviceScene::bvhAbsMax).
__device__ inline NodeHits VisitQuantV(const float4 f0, const float4 f1, const float4 f2, const float4 f3,
                                       const float4 f4, const CwRay &r, float tMax) {
    const uint32_t eb = __float_as_uint(f0.w);
    const V3 p(f0.x, f0.y, f0.z);
    const V3 s(__uint_as_float((eb & 0xffu) << 23), __uint_as_float(((eb >> 8) & 0xffu) << 23),
               __uint_as_float(((eb >> 16) & 0xffu) << 23));
    NodeHits o;
    o.imask = eb >> 24;
    o.childBase = __float_as_int(f1.x);
    o.triBase = __float_as_int(f1.y);
    const uint32_t meta[2] = {__float_as_uint(f1.z), __float_as_uint(f1.w)};
    // plane words: lo axis a children 4g.. at qw[2a + g], hi at qw[6 + 2a + g]
    const uint32_t qw[12] = {__float_as_uint(f2.x), __float_as_uint(f2.y), __float_as_uint(f2.z),
                             __float_as_uint(f2.w), __float_as_uint(f3.x), __float_as_uint(f3.y),
                             __float_as_uint(f3.z), __float_as_uint(f3.w), __float_as_uint(f4.x),
                             __float_as_uint(f4.y), __float_as_uint(f4.z), __float_as_uint(f4.w)};
    V3 A, BN, BF;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        A[a] = s[a] * r.inv[a];
        BN[a] = fmaf(p[a], r.inv[a], r.oN[a]);
        BF[a] = fmaf(p[a], r.inv[a], r.oF[a]);
    }
    uint32_t hit = 0, tris = 0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        uint32_t wn[3], wf[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const bool neg = (r.oct >> a) & 1u;
            wn[a] = neg ? qw[6 + 2 * a + g] : qw[2 * a + g];
            wf[a] = neg ? qw[2 * a + g] : qw[6 + 2 * a + g];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            auto byteOf = [k](uint32_t w) { return (float)((w >> (8 * k)) & 0xffu); };
            const float tn = fmaxf(fmaxf(fmaf(byteOf(wn[0]), A.x, BN.x), fmaf(byteOf(wn[1]), A.y, BN.y)),
                                   fmaxf(fmaf(byteOf(wn[2]), A.z, BN.z), 0.f));
            const float tf = fminf(fminf(fmaf(byteOf(wf[0]), A.x, BF.x), fmaf(byteOf(wf[1]), A.y, BF.y)),
                                   fminf(fmaf(byteOf(wf[2]), A.z, BF.z), tMax));
            const bool ok = tn <= tf;
            const uint32_t m = (meta[g] >> (8 * k)) & 0xffu;
            hit |= ok ? 1u << (4 * g + k) : 0u;
            tris |= ok ? ((1u << (m >> 5)) - 1u) << (m & 31u) : 0u;
        }
    }
    o.inner = hit & o.imask;
    o.tris = tris;
    return o;
}
template <typename F4>
__device__ inline NodeHits VisitQuant(const F4 *__restrict__ q, const CwRay &r, float tMax) {
    return VisitQuantV(q[0], q[1], q[2], q[3], q[4], r, tMax);
}

// Scene cache in LDS: the group stack ([stackSize][kBlock] uint2), the first S.ldsNodes BVH8
// nodes (BFS order = the top of the tree) at a 17-float4 (wide) / 5-float4 (quantised) stride,
// and -- when every node and triangle fits -- all triangles in three pre-rotated copies
// ([kz][tri][vertex], vertex = (p[kx], p[ky], p[kz], 0)).  The 68-dword wide stride puts the
// same field of 16 nodes in 16 different 4-bank groups, so ds_read_b128 lane groups stay
// conflict-free when lanes sit in different nodes.
// LDS-qualified pointers keep the cached and the global paths distinct instructions
// (ds_read_b128 vs global_load_dwordx4); generic pointers would merge them into flat loads.
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const float4 LdsF4;
typedef __attribute__((address_space(3))) uint2 LdsU2;
#else
typedef const float4 LdsF4;  // host pass only parses the kernels
typedef uint2 LdsU2;
#endif
struct SceneLds {
    LdsU2 *stack;        // [stackSize][blockDim]
    const LdsF4 *nodes;  // [ldsNodes][stride]
    const LdsF4 *tris;   // [3][ldsTris][3]
};

// Lays out the dynamic LDS of a traversal kernel and fills the cache (whole block, one sync).
__device__ inline SceneLds SetupSceneLds(const DeviceScene &S, float4 *dyn) {
    SceneLds L;
    L.stack = (LdsU2 *)reinterpret_cast<uint2 *>(dyn);
    float4 *nodes = dyn + (S.stackSize * kBlock) / 2;
    float4 *tris = nodes + S.ldsNodes * LdsNodeStride(S.compressed);
    // plain copies: measured faster here than per-node LDS-DMA (few, tiny rows)
    if (S.compressed) {
        for (int i = threadIdx.x; i < S.ldsNodes * kLdsQNodeStride; i += blockDim.x) {
            const int n = i / kLdsQNodeStride, k = i - n * kLdsQNodeStride;
            nodes[i] = S.qnodes[n * S.qStride + k];
        }
    } else {
        const float4 *gn = reinterpret_cast<const float4 *>(S.nodes);
        for (int i = threadIdx.x; i < S.ldsNodes * 15; i += blockDim.x) {
            const int n = i / 15, k = i - n * 15;
            nodes[n * kLdsNodeStride + k] = gn[n * 16 + k];
        }
    }
    for (int i = threadIdx.x; i < S.ldsTris * 9; i += blockDim.x) {
        const int rot = i / (S.ldsTris * 3), e = i - rot * (S.ldsTris * 3);
        const int tri = e / 3;
        const V3 v = RotateToRay(S.triVerts[tri * S.triStride + (e - 3 * tri)], rot);
        tris[i] = make_float4(v.x, v.y, v.z, 0.f);
    }
    __syncthreads();
    L.nodes = (const LdsF4 *)nodes;
    L.tris = (const LdsF4 *)tris;
    return L;
}

// NodesInLds / TrisInLds: every node / triangle is cached (launch-uniform choices, so no per-lane
// branch whose two loads the compiler would merge into one flat load).
// Profiling build (PBRT_AMD_TRAV_STATS): nodes visited / triangles tested per lane, summed per
// kernel into the stats slots by TravStatsAdd.
struct TravCount {
    int nodes = 0, tris = 0;
};
// GeometricPrimitive's stochastic alpha test as pbrt's GPU any-hit programs apply it to every
// candidate hit (gpu/optix.cu:197-243, 368-381, 449-461): the alpha texture at the candidate's
// SurfaceInteraction (p, n, uv; no derivatives) kills it when alpha <= 0, or when alpha < 1 and
// HashFloat(ray o, ray d) > alpha.  One hash per ray, so the surviving hits are the same in
// any traversal order.  Out of line (defined with the texture code below): only the alpha
// instantiations call it.  b0..b2: the triangle's barycentrics, or a shape's pObj.
__device__ __attribute__((noinline)) bool AlphaKilled(const DeviceScene *S, int prim, float b0, float b1, float b2,
                                                     V3 o, V3 d);
// Alpha: the scene has alpha-tested primitives (S.primAlpha); compiled into the kTravShapes
// ("extended") instantiations only
// One ray's resumable group traversal: TraverseCW runs CwStep to completion (round 4's
// dynamic-ray-fetch experiment interleaved steps of different rays in one lane: measured slower
// on C2 and C4, profiles/r04_c4_traversal_ab.txt, and removed in round 5).
struct CwState {
    TriRayR tr;
    CwRay r;
    float tMax;
    TriHit best;
    int node, sp, hit;
};
__device__ inline void CwBegin(const DeviceScene &S, CwState &s, V3 o, V3 d, float tMax) {
    s.tr = MakeTriRayR(o, d);
    s.r = MakeCwRay(o, d, S.bvhAbsMax);
    s.tMax = tMax;
    s.node = s.sp = 0;
    s.hit = -1;
}
// Visits s.node and its hit leaf triangles, then moves to the next node.  Returns true when the
// ray is done (stack empty, or with AnyHit the first hit: s.hit).  o, d: the ray, for the alpha test.
template <bool AnyHit, bool Compressed, bool NodesInLds, bool TrisInLds, bool Alpha>
__device__ inline bool CwStep(const DeviceScene &S, const SceneLds &L, CwState &s, V3 o, V3 d, TravCount *cnt) {
    LdsU2 *stk = L.stack + threadIdx.x;
    NodeHits nh;
#ifdef PBRT_AMD_TRAV_STATS
    if (cnt) ++cnt->nodes;
#endif
    if constexpr (Compressed) {
        if (NodesInLds || s.node < S.ldsNodes) nh = VisitQuant(L.nodes + s.node * kLdsQNodeStride, s.r, s.tMax);
        else nh = VisitQuant(S.qnodes + (size_t)s.node * S.qStride, s.r, s.tMax);
    } else {
        if (NodesInLds || s.node < S.ldsNodes) nh = VisitWide(L.nodes + s.node * kLdsNodeStride, s.r, s.tMax);
        else nh = VisitWide(reinterpret_cast<const float4 *>(S.nodes + s.node), s.r, s.tMax);
    }
    // the node's hit leaf triangles, in leaf order
    uint32_t tris = nh.tris;
    while (tris) {
        const int t = nh.triBase + __builtin_ctz(tris);
        tris &= tris - 1u;
#ifdef PBRT_AMD_TRAV_STATS
        if (cnt) ++cnt->tris;
#endif
        V3 a, b, c;
        if constexpr (TrisInLds) {
            const LdsF4 *v = L.tris + (s.tr.kz * S.ldsTris + t) * 3;
            const float4 va = v[0], vb = v[1], vc = v[2];
            a = V3(va.x, va.y, va.z), b = V3(vb.x, vb.y, vb.z), c = V3(vc.x, vc.y, vc.z);
        } else {
            const float4 *tv = S.triVerts + (size_t)t * S.triStride;
            a = RotateToRay(tv[0], s.tr.kz);
            b = RotateToRay(tv[1], s.tr.kz);
            c = RotateToRay(tv[2], s.tr.kz);
        }
        TriHit h;
        if (IntersectTriangleRot(s.tr, s.tMax, a, b, c, &h)) {
            if constexpr (Alpha) {
                if (S.nAlpha > 0 && S.primAlpha[t] >= 0 && AlphaKilled(S.self, t, h.b0, h.b1, h.b2, o, d)) continue;
            }
            s.hit = t;
            if (AnyHit) return true;
            s.tMax = h.t;
            s.best = h;
        }
    }
    // next node: the nearest child of this node's group, else of the top stacked group
    uint32_t bits = PermuteOct(nh.inner, s.r.oct), gBase = (uint32_t)nh.childBase, gMask = nh.imask;
    if (bits == 0) {
        if (s.sp == 0) return true;
        --s.sp;
        const uint2 e = stk[s.sp * kBlock];
        gBase = e.x;
        gMask = e.y >> 8;
        bits = e.y & 0xffu;
    }
    const uint32_t slot = (uint32_t)__builtin_ctz(bits) ^ s.r.oct;
    bits &= bits - 1u;
    s.node = (int)gBase + __popc(gMask & ((1u << slot) - 1u));
    if (bits) {
        stk[s.sp * kBlock] = make_uint2(gBase, (gMask << 8) | bits);  // sp < S.stackSize by construction
        ++s.sp;
    }
    return false;
}
template <bool AnyHit, bool Compressed, bool NodesInLds, bool TrisInLds, bool Alpha = false>
__device__ inline int TraverseCW(const DeviceScene &S, const SceneLds &L, V3 o, V3 d, float tMax, TriHit *best,
                                 TravCount *cnt = nullptr) {
    CwState s;
    CwBegin(S, s, o, d, tMax);
    while (!CwStep<AnyHit, Compressed, NodesInLds, TrisInLds, Alpha>(S, L, s, o, d, cnt)) {
    }
    if (!AnyHit && s.hit >= 0) *best = s.best;
    return s.hit;
}

// Traversal modes, one kernel instantiation each (a launch-uniform choice, so every kernel
// carries exactly one traversal loop): every node and triangle in LDS (small scenes); wide
// nodes with the top of the tree in LDS; quantised nodes (PBRT_AMD_BVH=compressed).
// waves per SIMD (= 256-thread blocks per CU) a traversal kernel of mode TM is compiled for
// A mode may carry kTravShapes: the scene has analytic shapes, whose BVH is traversed after the
// triangles' (an out-of-line call, compiled only into these instantiations so the triangle-only
// kernels keep their register allocation and scratch), or alpha-tested primitives.
constexpr int kTravShapes = 4;
constexpr int TraversalWaves(int tm) {
    return (tm & 3) == kTravQuant ? PBRT_QUANT_TRAVERSAL_WAVES : PBRT_TRAVERSAL_WAVES;
}
// With every node and triangle in LDS (and no shapes) the traversal kernels run 5 waves per
// SIMD: k_shadow fits them without spills (93 VGPRs), k_closest with a few spilled VGPRs but
// its full queue staging (kCap 256: LDS is no constraint at 5 blocks there); with the staging cut
// to 64 entries it lost (profiles/r06_c2_traversal_waves_ab.txt: C2 k_shadow 416 -> 371 us,
// k_closest 727 -> 707 us)
#ifndef PBRT_SHADOW_LDS_WAVES
#define PBRT_SHADOW_LDS_WAVES 5
#endif
constexpr int ShadowWaves(int tm) { return tm == kTravLds ? PBRT_SHADOW_LDS_WAVES : TraversalWaves(tm); }
#ifndef PBRT_CLOSEST_LDS_WAVES
#define PBRT_CLOSEST_LDS_WAVES 5
#endif
constexpr int ClosestWaves(int tm) { return tm == kTravLds ? PBRT_CLOSEST_LDS_WAVES : TraversalWaves(tm); }
inline int TraversalMode(const DeviceScene &S) {
    return (S.compressed ? kTravQuant : (S.ldsTris > 0 ? kTravLds : kTravWide)) |
           (S.nShapes > 0 || S.nAlpha > 0 ? kTravShapes : 0);
}
// Spheres and disks (Sphere / Disk::BasicIntersect) through their binary BVH, nearer than
// tMax: the shape index and best = {pObj, tHit}, or -1.  Out of line: only scenes with shapes
// reach it, and the triangle traversal keeps its registers.
// primAlpha (null: no alpha test) is the scene's leaf-order array, shape k at nTris + k
template <bool AnyHit>
__device__ __attribute__((noinline)) int TraverseShapes(const ShapeBVHNode *shapeNodes, const DeviceShape *shapes, V3 o,
                                                        V3 d, float tMax, TriHit *best, const int *primAlpha,
                                                        int nTris, const DeviceScene *self) {
    const V3 inv(1 / d.x, 1 / d.y, 1 / d.z);
    int stack[32], sp = 0, found = -1;
    stack[sp++] = 0;
    while (sp > 0) {
        const int ni = stack[--sp];
        const ShapeBVHNode n = shapeNodes[ni];
        // slab test with pbrt's 1 + 2 gamma(3) far-plane widening (util/vecmath.h:1576-1611)
        float t0 = 0, t1 = tMax;
        bool miss = false;
        for (int a = 0; a < 3 && !miss; ++a) {
            float tn = (n.lo[a] - o[a]) * inv[a], tf = (n.hi[a] - o[a]) * inv[a];
            if (tn > tf) {
                const float t = tn;
                tn = tf;
                tf = t;
            }
            tf *= 1 + 2 * gamma(3);
            t0 = tn > t0 ? tn : t0;
            t1 = tf < t1 ? tf : t1;
            miss = t0 > t1;
        }
        if (miss) continue;
        if (n.count > 0) {
            for (int k = n.child; k < n.child + n.count; ++k) {
                float th;
                V3 pObj;
                if (ShapeIntersect(shapes[k], o, d, tMax, &th, &pObj)) {
                    if (primAlpha && primAlpha[nTris + k] >= 0 && AlphaKilled(self, nTris + k, pObj.x, pObj.y, pObj.z, o, d))
                        continue;
                    found = k;
                    tMax = th;
                    *best = TriHit{pObj.x, pObj.y, pObj.z, th};
                    if (AnyHit) return k;
                }
            }
        } else if (sp < 30) {
            stack[sp++] = n.child;
            stack[sp++] = ni + 1;
        }
    }
    return found;
}
template <bool AnyHit, int TM>
__device__ inline int Traverse(const DeviceScene &S, const SceneLds &L, V3 o, V3 d, float tMax, TriHit *best,
                               TravCount *cnt = nullptr) {
    constexpr int tm = TM & 3;
    int prim = -1;
    if constexpr ((TM & kTravShapes) != 0) {
        if (S.nTris > 0)
            prim = TraverseCW<AnyHit, tm == kTravQuant, tm == kTravLds, tm == kTravLds, true>(S, L, o, d, tMax, best, cnt);
        if (S.nShapes > 0 && !(AnyHit && prim >= 0)) {
            const int k = TraverseShapes<AnyHit>(S.shapeNodes, S.shapes, o, d, prim >= 0 ? best->t : tMax, best,
                                                 S.nAlpha > 0 ? S.primAlpha : nullptr, S.nTris, S.self);
            if (k >= 0) prim = S.nTris + k;
        }
    } else {
        prim = TraverseCW<AnyHit, tm == kTravQuant, tm == kTravLds, tm == kTravLds>(S, L, o, d, tMax, best, cnt);
    }
    return prim;
}
// Adds a wave's traversal counts to stats[base..base+5]: lane sums of nodes and triangles,
// the wave maxima of both (a wave runs until its slowest lane is done), rays, waves
__device__ inline void TravStatsAdd(unsigned long long *stats, int base, bool active, const TravCount &c) {
#ifdef PBRT_AMD_TRAV_STATS
    int sn = active ? c.nodes : 0, st = active ? c.tris : 0, mn = sn, mt = st, nr = active ? 1 : 0;
    for (int off = 32; off > 0; off >>= 1) {
        sn += __shfl_xor(sn, off);
        st += __shfl_xor(st, off);
        mn = max(mn, __shfl_xor(mn, off));
        mt = max(mt, __shfl_xor(mt, off));
        nr += __shfl_xor(nr, off);
    }
    if (__lane_id() == 0 && nr) {
        atomicAdd(&stats[base], (unsigned long long)sn);
        atomicAdd(&stats[base + 1], (unsigned long long)st);
        atomicAdd(&stats[base + 2], (unsigned long long)mn);
        atomicAdd(&stats[base + 3], (unsigned long long)mt);
        atomicAdd(&stats[base + 4], (unsigned long long)nr);
        atomicAdd(&stats[base + 5], 1ull);
    }
#else
    (void)stats, (void)base, (void)active, (void)c;
#endif
}
// Launches kernel template K<..., TM> with the scene's traversal mode
#define PBRT_LAUNCH_TRAVERSAL(S, KERNEL, ...)                                                   \
    do {                                                                                        \
        switch (TraversalMode(S)) {                                                             \
        case kTravLds: hipLaunchKernelGGL((KERNEL(kTravLds)), __VA_ARGS__); break;              \
        case kTravWide: hipLaunchKernelGGL((KERNEL(kTravWide)), __VA_ARGS__); break;            \
        case kTravQuant: hipLaunchKernelGGL((KERNEL(kTravQuant)), __VA_ARGS__); break;          \
        case kTravLds | kTravShapes:                                                            \
            hipLaunchKernelGGL((KERNEL(kTravLds | kTravShapes)), __VA_ARGS__);                  \
            break;                                                                              \
        case kTravWide | kTravShapes:                                                           \
            hipLaunchKernelGGL((KERNEL(kTravWide | kTravShapes)), __VA_ARGS__);                 \
            break;                                                                              \
        default: hipLaunchKernelGGL((KERNEL(kTravQuant | kTravShapes)), __VA_ARGS__); break;    \
        }                                                                                       \
    } while (0)

// ------------------------------------------------------------------ lights
struct LightSample {
    float Le[kNSpectrumSamples];
    V3 wi, p, pErr, n;
    float pdf;
};

// Triangle geometry of a leaf-order prim
__device__ inline void PrimVerts(const DeviceScene &S, int prim, V3 *p0, V3 *p1, V3 *p2) {
    if (S.nShapes > 0 && prim >= S.nTris) {  // a sphere or disk: no vertices
        *p0 = *p1 = *p2 = V3(0, 0, 0);
        return;
    }
    const float4 *tv = S.triVerts + (size_t)prim * S.triStride;
    float4 a = tv[0], b = tv[1], c = tv[2];
    *p0 = V3(a.x, a.y, a.z);
    *p1 = V3(b.x, b.y, b.z);
    *p2 = V3(c.x, c.y, c.z);
}

// Vertex normals / uv of a leaf-order prim; false (and sh untouched) when it has none
__device__ inline bool LoadTriShading(const DeviceScene &S, int prim, TriShading *sh) {
    if (!S.triShade || (S.nShapes > 0 && prim >= S.nTris)) return false;
    const float4 a = S.triShade[4 * prim];
    const int flags = __float_as_int(a.w);
    if (flags == 0) return false;
    const float4 b = S.triShade[4 * prim + 1], c = S.triShade[4 * prim + 2], d = S.triShade[4 * prim + 3];
    sh->flags = flags;
    sh->n0 = V3(a.x, a.y, a.z);
    sh->n1 = V3(b.x, b.y, b.z);
    sh->n2 = V3(c.x, c.y, c.z);
    sh->uv[0][0] = b.w;
    sh->uv[0][1] = c.w;
    sh->uv[1][0] = d.x;
    sh->uv[1][1] = d.y;
    sh->uv[2][0] = d.z;
    sh->uv[2][1] = d.w;
    if ((flags & 4) && S.triTangent) {
        const float4 s0 = S.triTangent[3 * prim], s1 = S.triTangent[3 * prim + 1], s2 = S.triTangent[3 * prim + 2];
        sh->s0 = V3(s0.x, s0.y, s0.z);
        sh->s1 = V3(s1.x, s1.y, s1.z);
        sh->s2 = V3(s2.x, s2.y, s2.z);
    }
    return true;
}

// The out-of-line shape functions take the shape tables by value, never the DeviceScene: a
// scene reference passed to a call makes the kernel keep a copy of the whole DeviceScene
// (≈ 1.5 KB) in scratch per lane.
// SurfaceInteraction of a sphere / disk hit (b0..b2 of the hit record hold pObj)
__device__ __attribute__((noinline)) TriSurface ShapeSurfaceAt(const DeviceShape *shapes, const float *shapeN, int k,
                                                               V3 pObj) {
    return ShapeSurface(shapes[k], pObj, shapeN + 12 * (size_t)k);
}
// Shape::PDF(ctx, wi) of sphere / disk / patch k from a surface context (p, pErr, n, ns)
__device__ __attribute__((noinline)) float ShapeLightPDF(const DeviceShape *shapes, const float *shapeN, int k, V3 p,
                                                         V3 pErr, V3 n, V3 ns, V3 wi) {
    return ShapePDFSolidAngle(shapes[k], p, pErr, n, wi, shapeN + 12 * (size_t)k, ns);
}
// SurfaceInteraction of a hit (Triangle::InteractionFromIntersection)
// Ext: the scene may have analytic shapes (kernels instantiated without them compile the
// branch out, keeping the out-of-line call and its frame away from their register allocation)
template <bool Ext = true>
__device__ inline TriSurface SurfaceAt(const DeviceScene &S, int prim, V3 p0, V3 p1, V3 p2, float b0, float b1,
                                       float b2) {
    if (Ext && S.nShapes > 0 && prim >= S.nTris) return ShapeSurfaceAt(S.shapes, S.shapeN, prim - S.nTris, V3(b0, b1, b2));
    TriShading sh;
    const bool has = LoadTriShading(S, prim, &sh);
    return TriangleSurface(p0, p1, p2, b0, b1, b2, S.primFlip[prim], has ? &sh : nullptr);
}

__device__ inline float TriArea(V3 p0, V3 p1, V3 p2) { return 0.5f * Length(Cross(p1 - p0, p2 - p0)); }

__device__ inline float SolidAngleOf(V3 p0, V3 p1, V3 p2, V3 p) {
    return SphericalTriangleArea(Normalize(p0 - p), Normalize(p1 - p), Normalize(p2 - p));
}

// Triangle::Sample(ctx, u) (shapes.h:1053-1130); returns false for {}.  The three directions
// Normalize(p_i - refP) enter the solid angle, the bilinear warp weights and the spherical
// sample; pbrt normalises them anew in each (same operations, same values), here once.
// bOut (optional): the sample's barycentrics (the light's uv for an image emitter)
template <bool Inl = false>
__device__ inline bool SampleTriangle(V3 p0, V3 p1, V3 p2, bool flip, const TriShading *sh, V3 refP, V3 refN,
                                      V3 refNs, float u0, float u1, V3 *ps, V3 *pErr, V3 *ns, float *pdfOut,
                                      float *bOut = nullptr) {
    (void)refN;
    const V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
    float solidAngle = SphericalTriangleArea(wi0, wi1, wi2);
    if (solidAngle < kMinSphericalSampleArea || solidAngle > kMaxSphericalSampleArea) {
        float b[3];
        SampleUniformTriangle(u0, u1, b);
        V3 p = b[0] * p0 + b[1] * p1 + b[2] * p2;
        V3 n = TriangleSampleNormal(p0, p1, p2, b[0], b[1], flip, sh);
        V3 pAbsSum = Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2);
        ToPoint3fi(p, gamma(6) * pAbsSum, &p, pErr);
        float pdf = 1 / TriArea(p0, p1, p2);
        V3 wi = p - refP;
        if (LengthSquared(wi) == 0) return false;
        wi = Normalize(wi);
        pdf /= AbsDotN(n, -wi) / DistanceSquared(refP, p);
        if (isinf(pdf)) return false;
        *ps = p;
        *ns = n;
        *pdfOut = pdf;
        if (bOut) bOut[0] = b[0], bOut[1] = b[1], bOut[2] = b[2];
        return true;
    }
    float pdf = 1;
    if (refNs != V3(0, 0, 0)) {
        float w[4] = {fmaxf(0.01f, AbsDotN(refNs, wi1)), fmaxf(0.01f, AbsDotN(refNs, wi1)),
                      fmaxf(0.01f, AbsDotN(refNs, wi0)), fmaxf(0.01f, AbsDotN(refNs, wi2))};
        float px, py;
        SampleBilinear(u0, u1, w, &px, &py);
        u0 = px;
        u1 = py;
        pdf = BilinearPDF(u0, u1, w);
    }
    float triPDF;
    float b[3];
    {
        const SphTriSample r = Inl ? SampleSphericalTriangleNInl(p0, p1, p2, refP, wi0, wi1, wi2, u0, u1)
                                   : SampleSphericalTriangleN(p0, p1, p2, refP, wi0, wi1, wi2, u0, u1);
        b[0] = r.b0;
        b[1] = r.b1;
        b[2] = r.b2;
        triPDF = r.pdf;
    }
    if (triPDF == 0) return false;
    pdf *= triPDF;
    V3 pAbsSum = Abs(b[0] * p0) + Abs(b[1] * p1) + Abs((1 - b[0] - b[1]) * p2);
    V3 p;
    ToPoint3fi(b[0] * p0 + b[1] * p1 + b[2] * p2, gamma(6) * pAbsSum, &p, pErr);
    V3 n = TriangleSampleNormal(p0, p1, p2, b[0], b[1], flip, sh);
    *ps = p;
    *ns = n;
    *pdfOut = pdf;
    if (bOut) bOut[0] = b[0], bOut[1] = b[1], bOut[2] = b[2];
    return true;
}

// Triangle::PDF(ctx, wi) (shapes.h:1133-1174); the normalised directions to the vertices are
// formed once, as in SampleTriangle
__device__ inline float TrianglePDF(V3 p0, V3 p1, V3 p2, bool flip, const TriShading *sh, V3 refP, V3 refPErr,
                                   V3 refN, V3 refNs, V3 wi) {
    const V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
    float solidAngle = SphericalTriangleArea(wi0, wi1, wi2);
    if (solidAngle < kMinSphericalSampleArea || solidAngle > kMaxSphericalSampleArea) {
        // ShapeSampleContext::SpawnRay(wi) then Triangle::Intersect
        V3 o = OffsetRayOrigin(refP, refPErr, refN, wi);
        TriHit h;
        if (!IntersectTriangle(o, wi, kInfinity, p0, p1, p2, &h)) return 0;
        TriSurface hs = TriangleSurface(p0, p1, p2, h.b0, h.b1, h.b2, flip, sh);
        V3 pHit = hs.p, n = hs.n;
        float pdf = (1 / TriArea(p0, p1, p2)) / (AbsDotN(n, -wi) / DistanceSquared(refP, pHit));
        if (isinf(pdf)) pdf = 0;
        return pdf;
    }
    float pdf = 1 / solidAngle;
    if (refNs != V3(0, 0, 0)) {
        const SphTriUV uv = InvertSphericalTriangleSampleN(p0, p1, p2, refP, wi0, wi1, wi2, wi);
        float w[4] = {fmaxf(0.01f, AbsDotN(refNs, wi1)), fmaxf(0.01f, AbsDotN(refNs, wi1)),
                      fmaxf(0.01f, AbsDotN(refNs, wi0)), fmaxf(0.01f, AbsDotN(refNs, wi2))};
        pdf *= BilinearPDF(uv.u0, uv.u1, w);
    }
    return pdf;
}

// BVHLightSampler::Sample / PMF (lightsamplers.h:266-403) and UniformLightSampler
// light index convention: [0, nAreaLights) area lights, then infinite lights.
template <typename NodeT, bool Inl = false>
__device__ inline bool SampleLightT(const DeviceScene &S, const NodeT *lightNodes, V3 p, V3 ns, float u, int *light,
                                    float *pmfOut) {
    auto importance = [](const LightNodeBounds &b, V3 q, V3 n) {
        return Inl ? LightImportanceInl(b, q, n) : LightImportance(b, q, n);
    };
    int nAll = S.nAreaLights + S.nPointSpot + S.nInfinite;
    if (S.uniformLightSampler) {
        if (nAll == 0) return false;
        int li = min((int)(u * nAll), nAll - 1);
        *light = S.uniformOrder[li];  // pbrt's light order -> global index
        *pmfOut = 1.f / nAll;
        return true;
    }
    float pInfinite = float(S.nInfinite) / float(S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    if (u < pInfinite) {
        u /= pInfinite;
        int index = min((int)(u * S.nInfinite), S.nInfinite - 1);
        *pmfOut = pInfinite / S.nInfinite;
        *light = S.nAreaLights + S.nPointSpot + index;
        return true;
    }
    if (S.nLightNodes == 0) return false;
    u = fminf((u - pInfinite) / (1 - pInfinite), kOneMinusEpsilon);
    int nodeIndex = 0;
    float pmf = 1 - pInfinite;
    for (int iter = 0; iter < 4 * kMaxLightBVHDepth; ++iter) {
        DeviceLightNode node = lightNodes[nodeIndex];
        if (!node.isLeaf) {
            float c0 = importance(lightNodes[nodeIndex + 1].b, p, ns);
            float c1 = importance(lightNodes[node.childOrLight].b, p, ns);
            if (c0 == 0 && c1 == 0) return false;
            float nodePMF;
            int child = SampleDiscrete2(c0, c1, u, &nodePMF, &u);
            pmf *= nodePMF;
            nodeIndex = (child == 0) ? (nodeIndex + 1) : node.childOrLight;
        } else {
            if (nodeIndex > 0 || importance(node.b, p, ns) > 0) {
                *light = node.childOrLight;
                *pmfOut = pmf;
                return true;
            }
            return false;
        }
    }
    return false;
}
__device__ inline bool SampleLight(const DeviceScene &S, V3 p, V3 ns, float u, int *light, float *pmfOut) {
    return SampleLightT(S, S.lightNodes, p, ns, u, light, pmfOut);
}

__device__ inline float LightPMF(const DeviceScene &S, V3 p, V3 ns, int light) {
    int nAll = S.nAreaLights + S.nPointSpot + S.nInfinite;
    if (S.uniformLightSampler) return nAll ? 1.f / nAll : 0.f;
    uint32_t bitTrail = light < S.nAreaLights + S.nPointSpot ? S.lightBitTrail[light] : 0xffffffffu;
    if (bitTrail == 0xffffffffu) return 1.f / (S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    float pInfinite = float(S.nInfinite) / float(S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    float pmf = 1 - pInfinite;
    int nodeIndex = 0;
    for (int iter = 0; iter < kMaxLightBVHDepth; ++iter) {
        const DeviceLightNode &node = S.lightNodes[nodeIndex];
        if (node.isLeaf) return pmf;
        float c0 = LightImportance(S.lightNodes[nodeIndex + 1].b, p, ns);
        float c1 = LightImportance(S.lightNodes[node.childOrLight].b, p, ns);
        pmf *= ((bitTrail & 1) ? c1 : c0) / (c0 + c1);
        nodeIndex = (bitTrail & 1) ? node.childOrLight : (nodeIndex + 1);
        bitTrail >>= 1;
    }
    return pmf;
}


// One light sample for a surface vertex's NEE (surfscatter.cpp:254-285, light.SampleLi with
// allowIncompletePDF): DiffuseAreaLight::SampleLi through Triangle::Sample (lights.cpp:743-775),
// PointLight / SpotLight / DistantLight::SampleLi (lights.h).  The sample's radiance at a
// wavelength is scale * spectrum(lambda), divided by d2 for point and spot lights (pbrt's
// SampledSpectrum / DistanceSquared); a UniformInfiniteLight returns no sample.
// A GoniometricLight's image value multiplies scale * I(lambda) before the division (k; 1, an
// exact no-op, for every other light); a ProjectionLight's pixel is an envLe sample.
struct LiSample {
    V3 wi, lp, lpe, ln;  // direction, and the light point (error, normal) for SpawnRayTo
    float pdf;           // ls->pdf (1 for delta lights)
    float scale, d2;     // d2 = 1: no division
    float k = 1;         // GoniometricLight: image(uv) (lights.h:393-396)
    int spectrum;
    bool delta;          // IsDeltaLight: the BSDF's MIS pdf is 0
    bool envLe;          // ImageInfiniteLight / ProjectionLight: Le = EnvLe(env, scale, spectrum(lambda), lambda)
    EnvCoef env;
    // the radiance at one wavelength from the dense value of `spectrum` there (before / d2)
    __device__ float Le(float denseVal, float lambda) const {
        return (envLe ? EnvLe(env, scale, denseVal, lambda) : scale * denseVal) * k;
    }
};
// ImageInfiniteLight::SampleLi with allowIncompletePDF (lights.h:594-618): the compensated
// distribution's (u, v), its direction in render space, pdf = mapPDF / (4 pi), a light point
// 2 sceneRadius away and the nearest pixel's radiance
__device__ inline bool SampleEnvLi(const DeviceScene &S, int j, V3 cp, float u0, float u1, LiSample *ls) {
    const DeviceEnvLight &E = S.env[S.infImage[j]];
    if (E.portal) {  // PortalImageInfiniteLight::SampleLi from the context point
        V3 wi;
        float pdf;
        EnvCoef ec;
        if (!PortalSampleLi(E, cp, u0, u1, &wi, &pdf, &ec)) return false;
        ls->wi = wi;
        ls->pdf = pdf;
        ls->lp = cp + wi * (2 * S.sceneRadius);
        ls->lpe = V3(0, 0, 0);
        ls->ln = V3(0, 0, 0);
        ls->scale = S.infScale[j];
        ls->d2 = 1;
        ls->spectrum = S.infSpectrum[j];
        ls->delta = false;
        ls->envLe = true;
        ls->env = ec;
        return true;
    }
    float uu, vv, mapPDF;
    EnvSampleUV(E, u0, u1, &uu, &vv, &mapPDF);
    if (mapPDF == 0) return false;
    const V3 wi = MulM3(E.m, EqualAreaSquareToSphere(uu, vv));
    ls->wi = wi;
    ls->pdf = mapPDF / (4 * kPi);
    ls->lp = cp + wi * (2 * S.sceneRadius);
    ls->lpe = V3(0, 0, 0);
    ls->ln = V3(0, 0, 0);
    ls->scale = S.infScale[j];
    ls->d2 = 1;
    ls->spectrum = S.infSpectrum[j];
    ls->delta = false;
    ls->envLe = true;
    ls->env = EnvCoefAt(E, uu, vv);
    return true;
}
// ImageInfiniteLight::Le / PDF_Li(allowIncompletePDF) for an escaped ray direction d
// (lights.h:587-591, lights.cpp:1073-1083): Le's (u, v) from the normalised light-space
// direction, PDF_Li's from the unnormalised one
__device__ inline EnvCoef EnvLeCoef(const DeviceEnvLight &E, V3 d) {
    float u, v;
    EqualAreaSphereToSquare(Normalize(MulM3(E.mi, d)), &u, &v);
    return EnvCoefAt(E, u, v);
}
__device__ inline float EnvPDFLi(const DeviceEnvLight &E, V3 d) {
    float u, v;
    EqualAreaSphereToSquare(MulM3(E.mi, d), &u, &v);
    return EnvPDF(E, u, v) / (4 * kPi);
}
__device__ inline float SmoothStepf(float x, float a, float b) {
    if (a == b) return (x < a) ? 0 : 1;
    const float t = Clampf((x - a) / (b - a), 0, 1);
    return t * t * (3 - 2 * t);
}
// DiffuseAreaLight::L with an image (lights.h:460-467): R, G, B bilerped (Image::BilerpChannel,
// clamp wrap) at (u, 1 - v), then the RGBIlluminantSpectrum of ClampZero(rgb) as {c0, c1, c2,
// scale}; the radiance is EnvLe(coef, light scale, illuminant(lambda), lambda)
__device__ inline EnvCoef AreaImageCoef(const DeviceScene &S, int off, float u, float v) {
    const float *img = S.lightImg + off;
    const int w = __float_as_int(img[0]), h = __float_as_int(img[1]);
    const float *rgb = img + 2;
    v = 1 - v;
    const float x = u * w - 0.5f, y = v * h - 0.5f;
    const int xi = (int)floorf(x), yi = (int)floorf(y);
    const float dx = x - xi, dy = y - yi;
    const int x0 = min(max(xi, 0), w - 1), x1 = min(max(xi + 1, 0), w - 1);
    const int y0 = min(max(yi, 0), h - 1), y1 = min(max(yi + 1, 0), h - 1);
    float c3[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float v00 = rgb[((size_t)y0 * w + x0) * 3 + c], v10 = rgb[((size_t)y0 * w + x1) * 3 + c];
        const float v01 = rgb[((size_t)y1 * w + x0) * 3 + c], v11 = rgb[((size_t)y1 * w + x1) * 3 + c];
        const float b = (1 - dx) * (1 - dy) * v00 + dx * (1 - dy) * v10 + (1 - dx) * dy * v01 + dx * dy * v11;
        c3[c] = fmaxf(0.f, b);
    }
    const float m = fmaxf(c3[0], fmaxf(c3[1], c3[2])), scale = 2 * m;
    float co[3];
    if (scale != 0) RGBToCoeffs(S.tex, c3[0] / scale, c3[1] / scale, c3[2] / scale, co);
    else RGBToCoeffs(S.tex, 0, 0, 0, co);
    return EnvCoef{co[0], co[1], co[2], scale};
}
// the uv of a triangle point from its barycentrics (Triangle::Sample, shapes.h:1076-1078, 1120)
__device__ inline void TriUV(const TriShading *sh, const float b[3], float *u, float *v) {
    float uv[3][2] = {{0, 0}, {1, 0}, {1, 1}};
    if (sh && (sh->flags & 2))
        for (int k = 0; k < 3; ++k) uv[k][0] = sh->uv[k][0], uv[k][1] = sh->uv[k][1];
    *u = b[0] * uv[0][0] + b[1] * uv[1][0] + b[2] * uv[2][0];
    *v = b[0] * uv[0][1] + b[1] * uv[1][1] + b[2] * uv[2][1];
}

// This fork's DiffuseAreaLight spread (lights.h:451-458, lights.cpp:763-771).  cosE =
// cosFalloffEnd, > 0 only for a spread below 90 degrees.  L() is zero where the emission
// direction w leaves farther than the spread from the normal: AbsDot(w, n) < cosE.
__device__ inline bool SpreadCut(float cosE, V3 n, V3 w) { return cosE > 0 && AbsDotN(n, w) < cosE; }
// SampleLi's falloff factor on the light sample toward wi (cosE > 0), std::max(x, 0) as written
__device__ inline float SpreadFactor(float tanE, float norm, V3 n, V3 wi) {
    const float cos_a = -DotN(n, wi);
    const float sin_a = SafeSqrt(1 - Sqr(cos_a));
    const float tan_a = sin_a / cos_a;
    const float f = (1.0f - (tanE * tan_a)) * norm;
    return f < 0.0f ? 0.0f : f;
}
// Inl: the spherical-triangle sampling inlined (the diffuse kernels) or called out of line
// DiffuseAreaLight::SampleLi over a sphere or disk (lights.cpp:743-775 with Shape::Sample(ctx,
// u)): ctx = (cp, cpErr, n)
// k: the shape's index (its prim id - nTris)
__device__ __attribute__((noinline)) bool SampleShapeLi(const DeviceShape *shapes, const float *shapeN, int k,
                                                       bool twoSided, float scale, int spectrum, V3 cp, V3 cpErr, V3 n,
                                                       V3 ns, float u0, float u1, LiSample *ls, float cosE = -1,
                                                       float tanE = 0, float spreadNorm = 0, float *uvOut = nullptr) {
    ShapeSamplePt ss;
    if (!ShapeSampleSolidAngle(shapes[k], cp, cpErr, n, u0, u1, &ss, shapeN + 12 * (size_t)k, ns) || ss.pdf == 0 ||
        LengthSquared(ss.p - cp) == 0)
        return false;
    ls->wi = Normalize(ss.p - cp);
    if (!(twoSided || DotN(ss.n, -ls->wi) >= 0)) return false;  // DiffuseAreaLight::L is 0
    if (cosE > 0) {
        if (SpreadCut(cosE, ss.n, -ls->wi)) return false;
        ls->k = SpreadFactor(tanE, spreadNorm, ss.n, ls->wi);
        if (ls->k == 0) return false;  // Le *= 0: no sample
    }
    ls->lp = ss.p;
    ls->lpe = ss.pErr;
    ls->ln = ss.n;
    ls->pdf = ss.pdf;
    ls->scale = scale;
    ls->d2 = 1;
    ls->spectrum = spectrum;
    ls->delta = false;
    ls->envLe = false;
    if (uvOut) uvOut[0] = ss.uv[0], uvOut[1] = ss.uv[1];
    return true;
}
// Ext: analytic-shape emitters and image infinite lights may be sampled (false: their branches
// are compiled out; the host launches such kernels only for scenes without either)
template <bool Lean, bool Inl = Lean, bool Ext = true>
__device__ inline bool SampleLiSurface(const DeviceScene &S, const DeviceAreaLight *lightsL, int li, V3 cp, V3 n,
                                       V3 ns, float u0, float u1, LiSample *ls, V3 cpErr = V3(0, 0, 0)) {
    if (li < S.nAreaLights) {
        const DeviceAreaLight &Ld = lightsL[li];
        if constexpr (!Lean && Ext) {
            if (S.nShapes > 0 && __float_as_int(Ld.v0.w) >= S.nTris) {
                float suv[2];
                if (!SampleShapeLi(S.shapes, S.shapeN, __float_as_int(Ld.v0.w) - S.nTris, Ld.twoSided, Ld.scale,
                                   Ld.spectrum, cp, cpErr, n, ns, u0, u1, ls, Ld.v1.w, Ld.v2.w,
                                   Ld.v1.w > 0 ? S.lightSpreadNorm[li] : 0.f, suv))
                    return false;
                if (S.nImageAreaLights > 0 && S.lightImgOff[li] >= 0) {  // an image emitter at the sample's uv
                    ls->envLe = true;
                    ls->env = AreaImageCoef(S, S.lightImgOff[li], suv[0], suv[1]);
                }
                return true;
            }
        }
        V3 q0(Ld.v0.x, Ld.v0.y, Ld.v0.z), q1(Ld.v1.x, Ld.v1.y, Ld.v1.z), q2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
        TriShading lsh;
        const bool lhas = !Lean && LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
        float lpdf, lb[3];
        if (!SampleTriangle<Inl>(q0, q1, q2, Ld.flip, lhas ? &lsh : nullptr, cp, n, ns, u0, u1, &ls->lp, &ls->lpe, &ls->ln,
                            &lpdf, (!Lean && Ext) ? lb : nullptr) ||
            lpdf == 0 || LengthSquared(ls->lp - cp) == 0)
            return false;
        if constexpr (!Lean && Ext) {
            if (S.nImageAreaLights > 0 && S.lightImgOff[li] >= 0) {  // an image emitter
                float lu, lv;
                TriUV(lhas ? &lsh : nullptr, lb, &lu, &lv);
                ls->envLe = true;
                ls->env = AreaImageCoef(S, S.lightImgOff[li], lu, lv);
            }
        }
        ls->wi = Normalize(ls->lp - cp);
        if (!(Ld.twoSided || DotN(ls->ln, -ls->wi) >= 0)) return false;  // DiffuseAreaLight::L is 0
        if constexpr (!Lean) {
            if (Ld.v1.w > 0) {  // spread below 90 degrees
                if (SpreadCut(Ld.v1.w, ls->ln, -ls->wi)) return false;
                ls->k = SpreadFactor(Ld.v2.w, S.lightSpreadNorm[li], ls->ln, ls->wi);
                if (ls->k == 0) return false;
            }
        }
        ls->pdf = lpdf;
        ls->scale = Ld.scale;
        ls->d2 = 1;
        ls->spectrum = Ld.spectrum;
        ls->delta = false;
        if constexpr (Lean || !Ext) ls->envLe = false;
        else if (!(S.nImageAreaLights > 0 && S.lightImgOff[li] >= 0)) ls->envLe = false;
        return true;
    }
    if constexpr (Lean) {
        return false;  // lean launches have no point, spot or distant lights
    } else {
        const int k = li - S.nAreaLights;
        int di = k;
        if (k >= S.nPointSpot) {
            di = S.infDistant[k - S.nPointSpot];
            if (di < 0) {
                if (Ext && S.nEnv > 0 && S.infImage[k - S.nPointSpot] >= 0)
                    return SampleEnvLi(S, k - S.nPointSpot, cp, u0, u1, ls);
                return false;  // UniformInfiniteLight::SampleLi(allowIncompletePDF) = {}
            }
        }
        ls->envLe = false;
        const DeviceDeltaLight &D = S.delta[di];
        const int type = __float_as_int(D.p.w);
        ls->pdf = 1;
        ls->delta = true;
        ls->spectrum = __float_as_int(D.cone.z);
        ls->lpe = V3(0, 0, 0);
        ls->ln = V3(0, 0, 0);
        if (type == 2) {  // DistantLight: wi = Normalize(renderFromLight(0, 0, 1))
            ls->wi = Normalize(V3(D.w.x, D.w.y, D.w.z));
            ls->lp = cp + ls->wi * (2 * S.sceneRadius);
            ls->scale = D.w.w;
            ls->d2 = 1;
            return true;
        }
        const V3 p(D.p.x, D.p.y, D.p.z);
        ls->wi = Normalize(p - cp);
        ls->lp = p;
        ls->d2 = DistanceSquared(p, cp);
        float sc = D.w.w;
        if constexpr (Ext) {
            if (type >= 3) {
                // renderFromLight.ApplyInverse(-wi) (not normalised, as pbrt passes it)
                const V3 v = -ls->wi;
                const V3 wl(D.m0.x * v.x + D.m0.y * v.y + D.m0.z * v.z, D.m1.x * v.x + D.m1.y * v.y + D.m1.z * v.z,
                            D.m2.x * v.x + D.m2.y * v.y + D.m2.z * v.z);
                const int w = __float_as_int(D.m0.w), h = __float_as_int(D.m1.w);
                const float *img = S.deltaImg + __float_as_int(D.cone.w);
                ls->scale = sc;
                if (type == 3) {
                    // GoniometricLight::I: image.LookupNearestChannel(EqualAreaSphereToSquare(w), 0)
                    float u, vv;
                    EqualAreaSphereToSquare(wl, &u, &vv);
                    const int x = min(max((int)(u * w), 0), w - 1), y = min(max((int)(vv * h), 0), h - 1);
                    ls->k = img[(size_t)y * w + x];
                    return true;
                }
                // ProjectionLight::I (lights.cpp:343-360): behind the hither plane or outside the
                // screen window nothing; else the nearest pixel's RGBIlluminantSpectrum
                if (wl.z < 1e-3f) return false;
                const float s = D.m2.w, aspect = float(w) / float(h);
                const float bx = aspect > 1 ? aspect : 1.f, by = aspect > 1 ? 1.f : 1 / aspect;
                // screenFromLight(Point3f(w)) = Perspective(fov, 1e-3, 1e30): x = s wx / wz, y = s wy / wz
                const float psx = (s * wl.x) / wl.z, psy = (s * wl.y) / wl.z;
                if (!(psx >= -bx && psx <= bx && psy >= -by && psy <= by)) return false;
                const float u = (psx - -bx) / (bx - -bx), vv = (psy - -by) / (by - -by);
                const int x = min(max((int)(u * w), 0), w - 1), y = min(max((int)(vv * h), 0), h - 1);
                const float4 c = reinterpret_cast<const float4 *>(img)[(size_t)y * w + x];
                ls->envLe = true;
                ls->env = EnvCoef{c.x, c.y, c.z, c.w};
                return true;
            }
        }
        if (type == 1) {  // SpotLight::I: SmoothStep(CosTheta(wLight), cosEnd, cosStart) * scale
            const V3 v = -ls->wi;
            const V3 wl = Normalize(V3(D.m0.x * v.x + D.m0.y * v.y + D.m0.z * v.z,
                                       D.m1.x * v.x + D.m1.y * v.y + D.m1.z * v.z,
                                       D.m2.x * v.x + D.m2.y * v.y + D.m2.z * v.z));
            sc = SmoothStepf(wl.z, D.cone.y, D.cone.x) * sc;
            if (sc == 0) return false;  // Li is 0 at every wavelength
        }
        ls->scale = sc;
        return true;
    }
}

// Streaming form of the per-wavelength work: lambda_i, R_i, Le_i and beta_i are produced
// inside each 31-iteration loop (lambda by pbrt's sequential +10 nm recurrence, R by the
// sigmoid polynomial, beta re-read from the wavelength-major SoA through L1/L2) instead of
// being held in 31-entry register arrays, which keeps the kernel at a few waves per SIMD.
struct SpectralIter {
    float lam;
    int i;
    __device__ SpectralIter(float l0) : lam(l0), i(0) {}
    __device__ void Next() {
        lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
        if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
        ++i;
    }
};

__device__ inline float Reflectance(float4 mc, bool constant, float lambda) {
    float r = constant ? mc.w : SigmoidPolynomial(mc.x, mc.y, mc.z, lambda);
    return Clampf(r, 0, 1);
}

// the material a hit shades with: its triangle's, or with mix materials the one k_closest chose
__device__ inline int HitMaterial(const DeviceScene &S, const PathState &st, int depth, int ri, int prim) {
    return st.hitMat[0] ? st.hitMat[depth & 1][ri] : S.primMaterial[prim];
}
// A bump / normal-mapped material's shading normal and dpdu, as k_texture left them for record
// ri of `depth` (surfscatter.cpp:109-127); other materials keep the surface's
__device__ inline void BumpedShading(const DeviceScene &S, const PathState &st, int depth, int mat, int ri,
                                    TriSurface *surf) {
    if (!S.matBump[mat].z) return;
    const int N = st.NR;
    const float *tb = st.texBump[depth & 1];
    surf->ns = V3(tb[ri], tb[N + ri], tb[2 * N + ri]);
    surf->dpdus = V3(tb[3 * N + ri], tb[4 * N + ri], tb[5 * N + ri]);
}

// ---- textures (core/texture_eval.h)
// TextureEvalContext of a hit as the wavefront material stage builds it: p, n, uv and the
// (u,v) screen-space derivatives from Approximate_dp_dxy (surfscatter.cpp:74-104, 132-135)
__device__ inline TexEvalCtx HitTexCtx(const DeviceScene &S, const TriSurface &surf) {
    TexEvalCtx c;
    c.p = surf.p;
    c.n = surf.n;
    c.u = surf.uv[0];
    c.v = surf.uv[1];
    UVDerivatives(S.camDiff, surf.p, surf.n, surf.dpdu, surf.dpdv, &c);
    return c;
}
// FloatTexture::Evaluate of a compiled float program
__device__ inline float TexFloatAt(const DeviceScene &S, int prog, const TexEvalCtx &c) {
    float R[kTexMaxRegs];
    const DeviceTexProgram pg = S.tex.progs[prog];
    TexPhase1(S.tex, pg, c, R);
    return R[pg.result];
}
// FloatTexture::Evaluate with the one-instruction programs (a constant, an image) evaluated
// directly, without the register file.  Full = false: the host guarantees every program is
// one of those and no image filters with EWA (k_texture's lean instantiation)
template <bool Full = true>
__device__ inline float TexFloatFast(const DeviceScene &S, int prog, const TexEvalCtx &c) {
    const DeviceTexProgram pg = S.tex.progs[prog];
    if (!Full || pg.n1 == 1) {
        const DeviceTexInstr in = S.tex.instrs[pg.p1];
        const DeviceTexNode &nd = S.tex.nodes[in.node];
        const int op = in.op & 0xff;
        if (op == kT1FConst) return nd.p[22];
        if (!Full || op == kT1FImage) return FloatImageEval<Full>(S.tex, nd, c);
    }
    if constexpr (Full) return TexFloatAt(S, prog, c);
    else return 0.f;
}

// ToSensorRGB accumulation for one wavelength: sx += xbar * (c / pdf) (film.h:95-100)
// Film-only arithmetic (the contribution c and its 1/pdf, 1/denom scalings) uses reciprocal
// multiplies where the reference divides: at most an ulp or two per term in the pixel sums,
// and nothing that steers a path (beta, pdfs and RR keep the reference's exact operations).
struct SensorAcc {
    float sx = 0, sy = 0, sz = 0;
    __device__ void Add(const DeviceScene &S, int off, float c, bool first) { Add(S.sensor4, off, c, first); }
    template <typename F4>
    __device__ void Add(const F4 *sensor4, int off, float c, bool first) {
        float v = c * kInvWavelengthPDF;
        float4 sb = off < 0 ? make_float4(0.f, 0.f, 0.f, 0.f) : float4(sensor4[off]);
        float xb = sb.x, yb = sb.y, zb = sb.z;
        sx = first ? xb * v : sx + xb * v;
        sy = first ? yb * v : sy + yb * v;
        sz = first ? zb * v : sz + zb * v;
    }
};

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const float LdsF;
typedef __attribute__((address_space(3))) const uint16_t LdsU16;
typedef __attribute__((address_space(3))) const DeviceLightNode LdsLightNode;
#else
typedef const float LdsF;
typedef const uint16_t LdsU16;
typedef const DeviceLightNode LdsLightNode;
#endif

// GenerateCameraRays (wavefront/camera.cpp:31-80) for one pixel-sample slot: the first
// wavelength, and the render-space camera ray (PerspectiveCamera::GenerateRay,
// cameras.cpp:433-456, then CameraBase::RenderFromCamera).
// sidxOut: the pixel sample's Halton index when it fits 32 bits (the material kernels sample
// their dimensions from it instead of recomputing it from the pixel), else kNoSampleIndex.
__device__ inline void GenerateCameraRay(const DeviceScene &S, const PathState &st, int slot, float *lambda0Out,
                                         V3 *oOut, V3 *dOut, float *filterWeight, uint32_t *sidxOut) {
    *sidxOut = kNoSampleIndex;
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    // camera.cpp:50-62: wavelength Get1D, then GetCameraSample (samplers.h:797-813): pixel
    // offset (GetPixel2D) through the box filter (filters.h:67-71), time Get1D, lens Get2D
    float lu, pix0, pix1, l0, l1;
    if (S.samplerType >= kSamplerIndependent) {
        // independent / stratified / Sobol' / padded Sobol': Get1D, GetPixel2D, Get1D (time),
        // Get2D (lens) in order -- the stateful samplers' draws depend on it
        GenericSampler g;
        g.Start(S.samp, px, py, sampleIndex, 0);
        lu = g.Get1D(S.samp);
        g.GetPixel2D(S.samp, &pix0, &pix1);
        l0 = l1 = 0;
        if (S.lensRadius > 0) {
            (void)g.Get1D(S.samp);
            g.Get2D(S.samp, &l0, &l1);
        }
    } else if (S.samplerType == 1) {
        // ZSobolSampler: dimensions 0 (wavelength), 1-2 (pixel), 3 (time), 4-5 (lens)
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        lu = ZSobolGet1D(S.zs, morton, 0, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, 1, S.zsPerms, S.sobolM1, &pix0, &pix1);
        l0 = l1 = 0;
        if (S.lensRadius > 0) ZSobolGet2D(S.zs, morton, 4, S.zsPerms, S.sobolM1, &l0, &l1);
    } else {
        // HaltonSampler: GetPixel2D reads the pixel's own Halton digits, not a dimension
        Halton h = StartPixelSample(S, px, py, sampleIndex, 0);
        if ((h.index >> 32) == 0) *sidxOut = (uint32_t)h.index;
        lu = Get1D(S, h);
        const uint64_t a0 = h.index >> S.baseExponents[0];
        const uint64_t a1 = (h.index >> 32) == 0 ? (uint64_t)((uint32_t)h.index / (uint32_t)S.baseScales[1])
                                                 : h.index / (uint64_t)S.baseScales[1];
        pix0 = a0 < (1ull << 30) ? RadicalInverse32<2>((uint32_t)a0) : RadicalInverse(2, a0);
        pix1 = a1 < (1ull << 30) ? RadicalInverse32<3>((uint32_t)a1) : RadicalInverse(3, a1);
        // time: Get1D (unused: static camera); lens: Get2D, needed only by a thin-lens camera
        // (nothing samples this pixel sample's dimensions after them in this kernel)
        l0 = l1 = 0;
        if (S.lensRadius > 0) {
            (void)Get1D(S, h);
            Get2D(S, h, &l0, &l1);
        }
    }
    if (S.options & kOptNoWavelengthJitter) lu = 0.5f;  // camera.cpp:55-56
    float lambda0 = Lerpf(lu, kLambdaMin, kLambdaMax);
    // Filter::Sample(GetPixel2D()) (samplers.h:797-813): offset and weight
    float fx, fy;
    FilterSample(S.filter, S.filterTab, pix0, pix1, &fx, &fy, filterWeight);
    if (S.options & kOptNoPixelJitter) {  // samplers.h:807-812: pixel centre, lens centre, weight 1
        fx = fy = 0.f;
        *filterWeight = 1.f;
        l0 = l1 = 0.5f;
    }
    float pFilmX = px + fx + 0.5f, pFilmY = py + fy + 0.5f;
    // PerspectiveCamera::GenerateRay (cameras.cpp:433-456)
    V3 pCamera = XfPoint(S.cameraFromRaster, V3(pFilmX, pFilmY, 0));
    V3 o(0, 0, 0), d = Normalize(pCamera);
    if (S.lensRadius > 0) {
        float lx, ly;
        SampleUniformDiskConcentric(l0, l1, &lx, &ly);
        lx *= S.lensRadius;
        ly *= S.lensRadius;
        float ft = S.focalDistance / d.z;
        V3 pFocus = o + d * ft;
        o = V3(lx, ly, 0);
        d = Normalize(pFocus - o);
    }
    // CameraBase::RenderFromCamera(ray): Transform::operator()(Ray) with origin error offset
    {
        const float *m = S.renderFromCamera;
        V3 oo = XfPoint(m, o);
        V3 err;
        if (o == V3(0, 0, 0))
            err = gamma(3) * Abs(V3(m[3], m[7], m[11]));
        else
            err = gamma(3) * (Abs(V3(m[0] * o.x, m[4] * o.x, m[8] * o.x)) + Abs(V3(m[1] * o.y, m[5] * o.y, m[9] * o.y)) +
                              Abs(V3(m[2] * o.z, m[6] * o.z, m[10] * o.z)) + Abs(V3(m[3], m[7], m[11])));
        V3 dd = XfVector(m, d);
        float l2 = LengthSquared(dd);
        if (l2 > 0) {
            float dt = Dot(Abs(dd), err) / l2;
            oo = oo + dd * dt;
        }
        o = oo;
        d = dd;
    }
    *lambda0Out = lambda0;
    *oOut = o;
    *dOut = d;
}

}  // namespace pbrt_amd

namespace pbrt_amd {
__device__ __attribute__((noinline)) bool AlphaKilled(const DeviceScene *Sp, int prim, float b0, float b1, float b2,
                                                     V3 o, V3 d) {
    const DeviceScene &S = *Sp;
    V3 p0, p1, p2;
    PrimVerts(S, prim, &p0, &p1, &p2);
    const TriSurface surf = SurfaceAt<true>(S, prim, p0, p1, p2, b0, b1, b2);
    TexEvalCtx c;
    c.p = surf.p;
    c.n = surf.n;
    c.u = surf.uv[0];
    c.v = surf.uv[1];
    c.dudx = c.dudy = c.dvdx = c.dvdy = 0;
    const float a = TexFloatFast(S, S.primAlpha[prim], c);
    if (a >= 1) return false;
    if (a <= 0) return true;
    const uint32_t w[6] = {FloatToBits(o.x), FloatToBits(o.y), FloatToBits(o.z),
                           FloatToBits(d.x), FloatToBits(d.y), FloatToBits(d.z)};
    return (float)(uint32_t)HashWords(w, 6) * 0x1p-32f > a;  // HashFloat(o, d)
}
// MixMaterial::ChooseMaterial until a non-mix material is reached (materials.h:285-294), as the
// closest-hit stage does (wavefront/intersect.h:90-97): the "amount" texture at the hit (the
// context a SurfaceInteraction gives: no (u,v) derivatives), then HashFloat(p, wo, m0, m1).
// pbrt hashes the two materials' pointers; their indices stand in for them here (the oracle
// does the same), so which material an interior amount picks is not comparable with pbrt.
__device__ __attribute__((noinline)) int ResolveMixMaterial(const DeviceScene &S, int prim, int mat, float b0, float b1,
                                                            float b2, V3 d) {
    V3 p0, p1, p2;
    PrimVerts(S, prim, &p0, &p1, &p2);
    const TriSurface surf = SurfaceAt(S, prim, p0, p1, p2, b0, b1, b2);
    TexEvalCtx c;
    c.p = surf.p;
    c.n = surf.n;
    c.u = surf.uv[0];
    c.v = surf.uv[1];
    c.dudx = c.dudy = c.dvdx = c.dvdy = 0;
    const V3 wo = Normalize(-d);
    for (int guard = 0; guard < 64 && S.matType[mat] == kMatMixT; ++guard) {
        const int4 mm = S.matMix[mat];
        const float amt = TexFloatFast(S, mm.z, c);
        if (amt <= 0) mat = mm.x;
        else if (amt >= 1) mat = mm.y;
        else {
            const uint32_t w[10] = {FloatToBits(c.p.x), FloatToBits(c.p.y), FloatToBits(c.p.z), FloatToBits(wo.x),
                                    FloatToBits(wo.y),  FloatToBits(wo.z),  (uint32_t)mm.x,     0u,
                                    (uint32_t)mm.y,     0u};
            const float u = (float)(uint32_t)HashWords(w, 10) * 0x1p-32f;
            mat = (amt < u) ? mm.x : mm.y;
        }
    }
    return mat;
}
// The texture stage of EvaluateMaterialAndBSDF for one hit (k_texture on the surface path,
// k_vtexture on the volumetric one): bump / normal mapping into st.texBump[depth & 1], the reflectance as
// sigmoid coefficients (texCoef[0..2], texCoef[3] = 0) or 31 values (texR, texCoef[3] = 1),
// the roughness alphas into texCoef[4..5] (textured hair floats into texCoef[4..7]); record ri, its hit barycentrics hitB[k * NR + ri]
// and lambda0[ri] (read only for textured materials).
// Always inlined: compiled as a call (s_swappc) from k_texture it hung the textured Cornell box
// on the GPU (round 4 and again in round 6: tests/test_textures.py timed out in the first
// closest-hit-to-shade pass), with k_texture<*, false, false>'s private segment grown from 108 to
// 2012 B per lane (the kernel's modified DeviceScene argument spilled to scratch for the callee's
// reference) and 56 more VGPRs; inlined, the kernels keep the inline copy's code and resources.
// Hair: the textured hair floats and subsurface spectra are compiled in (k_vtexture's
// instantiation for scenes with S.matHairTex or S.matSssTex; elsewhere the blocks would only
// cost registers)
template <bool Full, bool Ext, bool Hair = false>
__device__ __forceinline__ void HitTextures(const DeviceScene &S, const PathState &st, int depth, int ri, int prim,
                                            int mat, const float *hitB, const float *lambda0s) {
    const int N = st.NR;
    const int4 mt = S.matTex[mat];
    const int4 mb = S.hasBump ? S.matBump[mat] : make_int4(-1, -1, 0, 0);
    // textured hair floats (Full stages only): eta, beta_m, beta_n, alpha and the concentrations
    // (the instantiation also serves scenes with textured subsurface spectra and no hair table)
    const int4 h0 = Hair && S.matHairTex ? S.matHairTex[2 * mat] : make_int4(-1, -1, -1, -1);
    const int h1 = Hair && S.matHairTex ? S.matHairTex[2 * mat + 1].x : -1;
    const bool hairT = h0.x >= 0 || h0.y >= 0 || h0.z >= 0 || h0.w >= 0 || h1 >= 0;
    const int2 sx = Hair && S.matSssTex ? S.matSssTex[mat] : make_int2(-1, -1);
    const bool sssT = sx.x >= 0 || sx.y >= 0;
    if (mt.x < 0 && mt.y < 0 && !mb.z && !hairT && !sssT) return;
    V3 p0, p1, p2;
    PrimVerts(S, prim, &p0, &p1, &p2);
    const TriSurface surf = SurfaceAt<Ext>(S, prim, p0, p1, p2, hitB[ri], hitB[N + ri], hitB[2 * N + ri]);
    const TexEvalCtx tc = HitTexCtx(S, surf);
    if (mb.z) {
        // bump / normal mapping (surfscatter.cpp:109-127): the perturbed shading normal and
        // dpdu, per record, for the shade kernel and the next depth's emission MIS
        BumpCtx bc;
        bc.p = surf.p;
        bc.n = surf.n;
        bc.u = tc.u;
        bc.v = tc.v;
        bc.dudx = tc.dudx;
        bc.dudy = tc.dudy;
        bc.dvdx = tc.dvdx;
        bc.dvdy = tc.dvdy;
        bc.ns = surf.ns;
        bc.dpdu = surf.dpdus;
        if (prim < S.nTris) {
            TriShading sh;
            const bool has = LoadTriShading(S, prim, &sh);
            TriangleShadingDiff(p0, p1, p2, has ? &sh : nullptr, surf, hitB[ri], hitB[N + ri], hitB[2 * N + ri], &bc.dpdv,
                                &bc.dndu, &bc.dndv);
        } else {  // a disk: shading = geometric frame, no normal derivatives
            bc.dpdv = surf.dpdv;
            bc.dndu = bc.dndv = V3(0, 0, 0);
        }
        V3 ns, dpdus;
        BumpShading(bc, S.tex, mb.y, [&](const TexEvalCtx &c) { return TexFloatFast<Full>(S, mb.x, c); }, &ns, &dpdus);
        float *tb = st.texBump[depth & 1];
        tb[ri] = ns.x;
        tb[(size_t)N + ri] = ns.y;
        tb[2 * (size_t)N + ri] = ns.z;
        tb[3 * (size_t)N + ri] = dpdus.x;
        tb[4 * (size_t)N + ri] = dpdus.y;
        tb[5 * (size_t)N + ri] = dpdus.z;
    }
    if (mt.x >= 0) {
        const DeviceTexProgram pg = S.tex.progs[mt.x];
        if (!Full || pg.simple) {
            float c[4];
            SpectrumImageCoeffs<Full>(S.tex, S.tex.nodes[S.tex.instrs[pg.p1].node], tc, c);
            st.texCoef[ri] = c[0];
            st.texCoef[(size_t)N + ri] = c[1];
            st.texCoef[2 * (size_t)N + ri] = c[2];
            st.texCoef[3 * (size_t)N + ri] = 0.f;
        } else if constexpr (Full) {
            float R[kTexMaxRegs];
            TexPhase1(S.tex, pg, tc, R);
            for (SpectralIter it(lambda0s[ri]); it.i < kNSpectrumSamples; it.Next())
                st.texR[(size_t)it.i * N + ri] = TexPhase2(S.tex, pg, R, it.lam, it.i);
            st.texCoef[3 * (size_t)N + ri] = 1.f;
        }
    }
    if (mt.y >= 0) {
        float ur = TexFloatFast<Full>(S, mt.y, tc), vr = TexFloatFast<Full>(S, mt.z, tc);
        if (mt.w) {
            ur = RoughnessToAlpha(ur);
            vr = RoughnessToAlpha(vr);
        }
        const TrowbridgeReitz t = TrowbridgeReitz::Make(ur, vr);
        st.texCoef[4 * (size_t)N + ri] = t.ax;
        st.texCoef[5 * (size_t)N + ri] = t.ay;
    }
    if constexpr (Hair) {
        if (hairT) {
            // HairMaterial::GetBxDF's GetFloatTexture values (materials.h:380-404) into texCoef[4..7]
            // (hair has no roughness slots); a textured eumelanin / pheomelanin pair becomes sigma_a
            // = SigmaAFromConcentration(ce, cp) (bxdfs.cpp:553-562: the RGB sum as an
            // RGBUnboundedSpectrum) per wavelength in texR, flagged by texCoef[3] = 1
            const int hp[4] = {h0.x, h0.y, h0.z, h0.w};
            for (int k = 0; k < 4; ++k)
                if (hp[k] >= 0) st.texCoef[(4 + k) * (size_t)N + ri] = TexFloatFast<true>(S, hp[k], tc);
            if (h1 >= 0) {
                const int h1y = S.matHairTex[2 * mat + 1].y;
                const float ce = fmaxf(0.f, TexFloatFast<true>(S, h1, tc)), cp = fmaxf(0.f, TexFloatFast<true>(S, h1y, tc));
                const float r = ce * 0.419f + cp * 0.187f, g = ce * 0.697f + cp * 0.4f, b = ce * 1.37f + cp * 1.05f;
                const float scale = 2 * fmaxf(r, fmaxf(g, b));
                float c[3];
                if (scale != 0) RGBToCoeffs(S.tex, r / scale, g / scale, b / scale, c);
                else RGBToCoeffs(S.tex, 0.f, 0.f, 0.f, c);
                for (SpectralIter it(lambda0s[ri]); it.i < kNSpectrumSamples; it.Next())
                    st.texR[(size_t)it.i * N + ri] = scale * SigmoidPolynomial(c[0], c[1], c[2], it.lam);
                st.texCoef[3 * (size_t)N + ri] = 1.f;
            }
        }
        if (sssT) {
            // SubsurfaceMaterial's texEval(sigma_a | sigma_s | mfp, ctx, lambda) per wavelength
            // (materials.h:823-841; Unbounded spectrum programs) into texS[k][i]
            const int sp[2] = {sx.x, sx.y};
            for (int k = 0; k < 2; ++k) {
                if (sp[k] < 0) continue;
                const DeviceTexProgram pg = S.tex.progs[sp[k]];
                float R[kTexMaxRegs];
                TexPhase1(S.tex, pg, tc, R);
                for (SpectralIter it(lambda0s[ri]); it.i < kNSpectrumSamples; it.Next())
                    st.texS[((size_t)k * kNSpectrumSamples + it.i) * N + ri] = TexPhase2(S.tex, pg, R, it.lam, it.i);
            }
        }
    }
}
}  // namespace pbrt_amd
