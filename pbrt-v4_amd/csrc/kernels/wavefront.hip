// MI355X wavefront kernels for pbrt's WavefrontPathIntegrator hot path.
//
// Stage <-> reference mapping:
//   k_camera          GenerateCameraRays<HaltonSampler> (wavefront/camera.cpp:31-80)
//   k_closest         WavefrontAggregate::IntersectClosest + EnqueueWorkAfterIntersection/Miss
//                     (wavefront/intersect.h:16-156), escaped rays (integrator.cpp:495-537)
//   k_shade_diffuse   HandleEmissiveIntersection (integrator.cpp:539-573) fused with
//                     GenerateRaySamples (samples.cpp:29-66) and
//                     EvaluateMaterialAndBSDF<DiffuseMaterial> (surfscatter.cpp:57-328)
//   k_shadow          IntersectShadow + RecordShadowRayResult (intersect.h:31-46)
//   k_film            UpdateFilm / RGBFilm::AddSample (wavefront/film.cpp:13-39, film.h:241-258)
//
// Queues are compacted with one wave64 ballot + one atomic per wave; per-material streams
// are separate queues (one per material tag present).  Launches are grid-stride over the
// device-side queue counters so the host never synchronises inside the render loop.
#include <hip/hip_runtime.h>

#include "device.h"

namespace pbrt_amd {

constexpr int kBlock = 256;
#ifndef PBRT_TRAVERSAL_WAVES
#define PBRT_TRAVERSAL_WAVES 4  // waves/SIMD the closest/shadow kernels are compiled for
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

// Append to up to K queues for a whole block: one global atomicAdd per queue per block, so the
// queue counters (one address each, serialised at one L2 channel) see a quarter of the
// per-wave traffic.  Lanes receive consecutive slots in (wave, lane) order.  Every thread of
// the block must call it (the callers' grid-stride loops are block-uniform).
template <int K>
__device__ inline void BlockPush(int *const (&counters)[K], const bool (&pred)[K], int (&pos)[K]) {
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
        for (int i = threadIdx.x; i < n; i += blockDim.x) q[b + i] = buf[k * Cap + i];
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

    __device__ WaveQueues(int *ldsAll, int *const *c, int *const *q) : counters(c), queues(q) {
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
        for (int i = __lane_id(); i < n; i += 64) q[b + i] = buf[k * Cap + i];
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
        v.count[s] = st.counters[CounterIndex(depth, queue, s)];
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
__device__ inline float SampleDim(const DeviceScene &S, uint64_t index, int dim) {
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
// One ray per lane.  The node's 8 child boxes are read as 12 float4 loads (SoA inside the
// 256-byte node), the 8 slab tests run fully unrolled in registers, leaves are intersected
// nearest-first and interior children are pushed farthest-first onto a per-lane stack that
// lives in LDS ([depth][lane] layout: consecutive lanes hit consecutive banks), so nothing
// spills to scratch.  Box test = Bounds3::IntersectP (util/vecmath.h:1576-1611) including the
// 1 + 2 gamma(3) far-plane slack; triangle test = IntersectTriangle (shapes.cpp:172-273).
// Stack entries per lane = DeviceScene::stackSize (the BVH's exact worst case, host-computed,
// at most kMaxStackSize), allocated as dynamic LDS at launch so small scenes keep occupancy.

struct RayPre {
    V3 o, invDir;
    int neg[3];
};

template <typename F4>
__device__ inline void SlabTest4(const F4 *__restrict__ q, int g, const RayPre &r, float raytMax, float tn[8],
                                 unsigned *mask) {
    // children 4g..4g+3: lox,loy,loz at float4 index 2a+g, hix,hiy,hiz at 6+2a+g
    float4 L[3], H[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        L[a] = q[2 * a + g];
        H[a] = q[6 + 2 * a + g];
    }
    const float slack = 1 + 2 * gamma(3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float lo[3], hi[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = k == 0 ? L[a].x : k == 1 ? L[a].y : k == 2 ? L[a].z : L[a].w;
            hi[a] = k == 0 ? H[a].x : k == 1 ? H[a].y : k == 2 ? H[a].z : H[a].w;
        }
        float nx = r.neg[0] ? hi[0] : lo[0], fx = r.neg[0] ? lo[0] : hi[0];
        float ny = r.neg[1] ? hi[1] : lo[1], fy = r.neg[1] ? lo[1] : hi[1];
        float nz = r.neg[2] ? hi[2] : lo[2], fz = r.neg[2] ? lo[2] : hi[2];
        float tMin = (nx - r.o.x) * r.invDir.x;
        float tMax = (fx - r.o.x) * r.invDir.x * slack;
        float tyMin = (ny - r.o.y) * r.invDir.y;
        float tyMax = (fy - r.o.y) * r.invDir.y * slack;
        bool ok = !(tMin > tyMax || tyMin > tMax);
        tMin = tyMin > tMin ? tyMin : tMin;
        tMax = tyMax < tMax ? tyMax : tMax;
        float tzMin = (nz - r.o.z) * r.invDir.z;
        float tzMax = (fz - r.o.z) * r.invDir.z * slack;
        ok = ok && !(tMin > tzMax || tzMin > tMax);
        tMin = tzMin > tMin ? tzMin : tMin;
        tMax = tzMax < tMax ? tzMax : tMax;
        ok = ok && (tMin < raytMax) && (tMax > 0);
        tn[4 * g + k] = tMin;
        *mask |= ok ? (1u << (4 * g + k)) : 0u;
    }
}

template <typename F4>
__device__ inline void SlabTest8(const F4 *__restrict__ q, const RayPre &r, float raytMax, float tn[8],
                                 unsigned *mask) {
    *mask = 0;
    SlabTest4(q, 0, r, raytMax, tn, mask);
    SlabTest4(q, 1, r, raytMax, tn, mask);
}

// Child references of a compressed node, decoded on demand for the children actually visited
struct QRefs {
    unsigned imask, meta[2];
    int childBase, triBase;
    // the uncompressed encoding: >= 0 interior node, < 0 leaf ~(first << 3 | count - 1)
    __device__ int Get(int c) const {
        if ((imask >> c) & 1u) return childBase + __popc(imask & ((1u << c) - 1u));
        const unsigned m = (meta[c >> 2] >> (8 * (c & 3))) & 0xffu;
        const int first = triBase + (int)(m & 31u), count = (int)((m >> 5) & 3u) + 1;
        return ~((first << 3) | (count - 1));
    }
};

// Slab tests of a compressed node (BVH8QNode, 5 float4): child planes decoded as
// fma(q, 2^(e-127), p) -- the expression the host rounded outward -- then the same test as
// SlabTest4.
template <typename F4>
__device__ inline void SlabTestQ(const F4 *__restrict__ q, const RayPre &r, float raytMax, float tn[8],
                                 unsigned *mask, QRefs *refs) {
    const float4 f0 = q[0], f1 = q[1], f2 = q[2], f3 = q[3], f4 = q[4];
    const unsigned eb = __float_as_uint(f0.w);
    const float sx = __uint_as_float((eb & 0xffu) << 23), sy = __uint_as_float(((eb >> 8) & 0xffu) << 23),
                sz = __uint_as_float(((eb >> 16) & 0xffu) << 23);
    const unsigned imask = eb >> 24;
    const int childBase = __float_as_int(f1.x), triBase = __float_as_int(f1.y);
    const unsigned meta[2] = {__float_as_uint(f1.z), __float_as_uint(f1.w)};
    const unsigned qw[12] = {__float_as_uint(f2.x), __float_as_uint(f2.y), __float_as_uint(f2.z),
                             __float_as_uint(f2.w), __float_as_uint(f3.x), __float_as_uint(f3.y),
                             __float_as_uint(f3.z), __float_as_uint(f3.w), __float_as_uint(f4.x),
                             __float_as_uint(f4.y), __float_as_uint(f4.z), __float_as_uint(f4.w)};
    const float slack = 1 + 2 * gamma(3);
    *mask = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const int w = c >> 2, sh = 8 * (c & 3);
        auto byteOf = [&](int field) { return (float)((qw[2 * field + w] >> sh) & 0xffu); };
        const float lo[3] = {fmaf(byteOf(0), sx, f0.x), fmaf(byteOf(1), sy, f0.y), fmaf(byteOf(2), sz, f0.z)};
        const float hi[3] = {fmaf(byteOf(3), sx, f0.x), fmaf(byteOf(4), sy, f0.y), fmaf(byteOf(5), sz, f0.z)};
        float nx = r.neg[0] ? hi[0] : lo[0], fx = r.neg[0] ? lo[0] : hi[0];
        float ny = r.neg[1] ? hi[1] : lo[1], fy = r.neg[1] ? lo[1] : hi[1];
        float nz = r.neg[2] ? hi[2] : lo[2], fz = r.neg[2] ? lo[2] : hi[2];
        float tMin = (nx - r.o.x) * r.invDir.x;
        float tMax = (fx - r.o.x) * r.invDir.x * slack;
        float tyMin = (ny - r.o.y) * r.invDir.y;
        float tyMax = (fy - r.o.y) * r.invDir.y * slack;
        bool ok = !(tMin > tyMax || tyMin > tMax);
        tMin = tyMin > tMin ? tyMin : tMin;
        tMax = tyMax < tMax ? tyMax : tMax;
        float tzMin = (nz - r.o.z) * r.invDir.z;
        float tzMax = (fz - r.o.z) * r.invDir.z * slack;
        ok = ok && !(tMin > tzMax || tzMin > tMax);
        tMin = tzMin > tMin ? tzMin : tMin;
        tMax = tzMax < tMax ? tzMax : tMax;
        ok = ok && (tMin < raytMax) && (tMax > 0);
        tn[c] = tMin;
        *mask |= ok ? (1u << c) : 0u;
    }
    // occupied slots: interior (imask) or leaf (meta bit 7)
    const unsigned leafBits = ((meta[0] >> 7) & 1u) | ((meta[0] >> 14) & 2u) | ((meta[0] >> 21) & 4u) |
                              ((meta[0] >> 28) & 8u) | (((meta[1] >> 7) & 1u) << 4) | (((meta[1] >> 15) & 1u) << 5) |
                              (((meta[1] >> 23) & 1u) << 6) | (((meta[1] >> 31) & 1u) << 7);
    *mask &= imask | leafBits;
    refs->imask = imask;
    refs->meta[0] = meta[0];
    refs->meta[1] = meta[1];
    refs->childBase = childBase;
    refs->triBase = triBase;
}

// Scene cache in LDS: the first S.ldsNodes BVH8 nodes (BFS order = the top of the tree) at a
// 17-float4 stride and the first S.ldsTris triangles of the leaf order.  The 68-dword node
// stride puts the same field of 16 different nodes in 16 different 4-bank groups, so the
// ds_read_b128 lane groups stay conflict-free when lanes sit in different nodes; the 12-dword
// triangle stride does the same for triangles.  Everything else is read from global memory.
// (strides: kLdsNodeStride / kLdsQNodeStride, device.h)

// LDS-qualified pointers keep the cached and the global paths distinct instructions
// (ds_read_b128 vs global_load_dwordx4); generic pointers would merge them into flat loads.
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const float4 LdsF4;
#else
typedef const float4 LdsF4;  // host pass only parses the kernels
#endif
struct SceneLds {
    int *stack;          // [stackSize][blockDim]
    const LdsF4 *nodes;  // [ldsNodes][17]
    const LdsF4 *tris;   // [ldsTris][3]
};

// Lays out the dynamic LDS of a traversal kernel and fills the cache (whole block, one sync).
__device__ inline SceneLds SetupSceneLds(const DeviceScene &S, float4 *dyn) {
    SceneLds L;
    L.stack = reinterpret_cast<int *>(dyn);
    float4 *nodes = dyn + (S.stackSize * kBlock) / 4;
    float4 *tris = nodes + S.ldsNodes * LdsNodeStride(S.compressed);
    // plain copies: measured faster here than per-node LDS-DMA (few, tiny rows)
    if (S.compressed) {
        const float4 *gn = reinterpret_cast<const float4 *>(S.qnodes);
        for (int i = threadIdx.x; i < S.ldsNodes * kLdsQNodeStride; i += blockDim.x) nodes[i] = gn[i];
    } else {
        const float4 *gn = reinterpret_cast<const float4 *>(S.nodes);
        for (int i = threadIdx.x; i < S.ldsNodes * 14; i += blockDim.x) {
            int n = i / 14, k = i - n * 14;
            nodes[n * kLdsNodeStride + k] = gn[n * 16 + k];
        }
    }
    for (int i = threadIdx.x; i < S.ldsTris * 3; i += blockDim.x) tris[i] = S.triVerts[i];
    __syncthreads();
    L.nodes = (const LdsF4 *)nodes;
    L.tris = (const LdsF4 *)tris;
    return L;
}

// TrisInLds: every triangle is cached (a launch-uniform choice, so no per-lane branch whose
// two loads the compiler would merge into one flat load).
template <bool AnyHit, bool TrisInLds, bool Compressed>
__device__ inline int TraverseT(const DeviceScene &S, const SceneLds &L, V3 o, V3 d, float tMax, TriHit *best) {
    const TriRay tr = MakeTriRay(o, d);
    RayPre r;
    r.o = o;
    r.invDir = V3(1 / d.x, 1 / d.y, 1 / d.z);
    r.neg[0] = r.invDir.x < 0;
    r.neg[1] = r.invDir.y < 0;
    r.neg[2] = r.invDir.z < 0;
    const int lane = threadIdx.x, stride = blockDim.x;
    int *lds = L.stack;
    int sp = 0;
    int node = 0;
    int hitPrim = -1;
    while (true) {
        float tn[8];
        unsigned mask;
        int ch[8];
        QRefs qr;
        if constexpr (Compressed) {
            if (node < S.ldsNodes) SlabTestQ(L.nodes + node * kLdsQNodeStride, r, tMax, tn, &mask, &qr);
            else SlabTestQ(reinterpret_cast<const float4 *>(S.qnodes + node), r, tMax, tn, &mask, &qr);
        } else {
            int4 ch0, ch1;
            if (node < S.ldsNodes) {
                const LdsF4 *q = L.nodes + node * kLdsNodeStride;
                SlabTest8(q, r, tMax, tn, &mask);
                float4 c0 = q[12], c1 = q[13];
                ch0 = make_int4(__float_as_int(c0.x), __float_as_int(c0.y), __float_as_int(c0.z), __float_as_int(c0.w));
                ch1 = make_int4(__float_as_int(c1.x), __float_as_int(c1.y), __float_as_int(c1.z), __float_as_int(c1.w));
            } else {
                const BVH8Node *np = S.nodes + node;
                SlabTest8(reinterpret_cast<const float4 *>(np), r, tMax, tn, &mask);
                ch0 = reinterpret_cast<const int4 *>(np->child)[0];
                ch1 = reinterpret_cast<const int4 *>(np->child)[1];
            }
            ch[0] = ch0.x, ch[1] = ch0.y, ch[2] = ch0.z, ch[3] = ch0.w;
            ch[4] = ch1.x, ch[5] = ch1.y, ch[6] = ch1.z, ch[7] = ch1.w;
        }
        // empty slots fail the slab test (inverted box / masked compressed slot)
        unsigned leaves = 0, inner = 0;
        if constexpr (Compressed) {
            inner = mask & qr.imask;
            leaves = mask & ~qr.imask;
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (mask & (1u << c)) {
                    if (ch[c] < 0) leaves |= 1u << c;
                    else inner |= 1u << c;
                }
            }
        }
        // leaves nearest-first
        while (leaves) {
            int bc = 0;
            float bt = kInfinity;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if ((leaves & (1u << c)) && tn[c] <= bt) {
                    bt = tn[c];
                    bc = c;
                }
            leaves &= ~(1u << bc);
            if (bt >= tMax) continue;
            int enc = 0;
            if constexpr (Compressed) {
                enc = ~qr.Get(bc);
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) enc = (c == bc) ? ~ch[c] : enc;
            }
            int first = enc >> 3, count = (enc & 7) + 1;
            for (int t = first; t < first + count; ++t) {
                float4 a, b, c;
                if (TrisInLds) {
                    a = L.tris[3 * t];
                    b = L.tris[3 * t + 1];
                    c = L.tris[3 * t + 2];
                } else {
                    a = S.triVerts[3 * t];
                    b = S.triVerts[3 * t + 1];
                    c = S.triVerts[3 * t + 2];
                }
                TriHit h;
                if (IntersectTriangleRay(tr, tMax, V3(a.x, a.y, a.z), V3(b.x, b.y, b.z), V3(c.x, c.y, c.z), &h)) {
                    if (AnyHit) return t;
                    tMax = h.t;
                    *best = h;
                    hitPrim = t;
                }
            }
        }
        // interior children farthest-first onto the stack (closest popped next)
        while (inner) {
            int bc = 0;
            float bt = -kInfinity;
#pragma unroll
            for (int c = 0; c < 8; ++c)
                if ((inner & (1u << c)) && tn[c] >= bt) {
                    bt = tn[c];
                    bc = c;
                }
            inner &= ~(1u << bc);
            if (bt >= tMax) continue;
            int child = 0;
            if constexpr (Compressed) {
                child = qr.Get(bc);
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) child = (c == bc) ? ch[c] : child;
            }
            lds[(sp++) * stride + lane] = child;  // sp < S.stackSize by construction
        }
        if (sp == 0) break;
        node = lds[(--sp) * stride + lane];
    }
    return hitPrim;
}

// Q: the launch's node format (a kernel template parameter, so each kernel carries only the
// traversal loops of its own format)
template <bool AnyHit, bool Q>
__device__ inline int Traverse(const DeviceScene &S, const SceneLds &L, V3 o, V3 d, float tMax, TriHit *best) {
    if constexpr (Q) {
        return TraverseT<AnyHit, false, true>(S, L, o, d, tMax, best);
    } else {
        if (S.ldsTris > 0) return TraverseT<AnyHit, true, false>(S, L, o, d, tMax, best);
        return TraverseT<AnyHit, false, false>(S, L, o, d, tMax, best);
    }
}

// ------------------------------------------------------------------ lights
struct LightSample {
    float Le[kNSpectrumSamples];
    V3 wi, p, pErr, n;
    float pdf;
};

// Triangle geometry of a leaf-order prim
__device__ inline void PrimVerts(const DeviceScene &S, int prim, V3 *p0, V3 *p1, V3 *p2) {
    float4 a = S.triVerts[3 * prim], b = S.triVerts[3 * prim + 1], c = S.triVerts[3 * prim + 2];
    *p0 = V3(a.x, a.y, a.z);
    *p1 = V3(b.x, b.y, b.z);
    *p2 = V3(c.x, c.y, c.z);
}

// Vertex normals / uv of a leaf-order prim; false (and sh untouched) when it has none
__device__ inline bool LoadTriShading(const DeviceScene &S, int prim, TriShading *sh) {
    if (!S.triShade) return false;
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
    return true;
}

// SurfaceInteraction of a hit (Triangle::InteractionFromIntersection)
__device__ inline TriSurface SurfaceAt(const DeviceScene &S, int prim, V3 p0, V3 p1, V3 p2, float b0, float b1,
                                       float b2) {
    TriShading sh;
    const bool has = LoadTriShading(S, prim, &sh);
    return TriangleSurface(p0, p1, p2, b0, b1, b2, S.primFlip[prim], has ? &sh : nullptr);
}

__device__ inline float TriArea(V3 p0, V3 p1, V3 p2) { return 0.5f * Length(Cross(p1 - p0, p2 - p0)); }

__device__ inline float SolidAngleOf(V3 p0, V3 p1, V3 p2, V3 p) {
    return SphericalTriangleArea(Normalize(p0 - p), Normalize(p1 - p), Normalize(p2 - p));
}

// Triangle::Sample(ctx, u) (shapes.h:1053-1130); returns false for {}
__device__ inline bool SampleTriangle(V3 p0, V3 p1, V3 p2, bool flip, const TriShading *sh, V3 refP, V3 refN,
                                      V3 refNs, float u0, float u1, V3 *ps, V3 *pErr, V3 *ns, float *pdfOut) {
    (void)refN;
    float solidAngle = SolidAngleOf(p0, p1, p2, refP);
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
        return true;
    }
    float pdf = 1;
    if (refNs != V3(0, 0, 0)) {
        V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
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
        const SphTriSample r = SampleSphericalTriangle(p0, p1, p2, refP, u0, u1);
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
    return true;
}

// Triangle::PDF(ctx, wi) (shapes.h:1133-1174)
__device__ inline float TrianglePDF(V3 p0, V3 p1, V3 p2, bool flip, const TriShading *sh, V3 refP, V3 refPErr,
                                   V3 refN, V3 refNs, V3 wi) {
    float solidAngle = SolidAngleOf(p0, p1, p2, refP);
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
        float u0, u1;
        const SphTriUV uv = InvertSphericalTriangleSample(p0, p1, p2, refP, wi);
        u0 = uv.u0;
        u1 = uv.u1;
        V3 wi0 = Normalize(p0 - refP), wi1 = Normalize(p1 - refP), wi2 = Normalize(p2 - refP);
        float w[4] = {fmaxf(0.01f, AbsDotN(refNs, wi1)), fmaxf(0.01f, AbsDotN(refNs, wi1)),
                      fmaxf(0.01f, AbsDotN(refNs, wi0)), fmaxf(0.01f, AbsDotN(refNs, wi2))};
        pdf *= BilinearPDF(u0, u1, w);
    }
    return pdf;
}

// BVHLightSampler::Sample / PMF (lightsamplers.h:266-403) and UniformLightSampler
// light index convention: [0, nAreaLights) area lights, then infinite lights.
__device__ inline bool SampleLight(const DeviceScene &S, V3 p, V3 ns, float u, int *light, float *pmfOut) {
    int nAll = S.nAreaLights + S.nInfinite;
    if (S.uniformLightSampler) {
        if (nAll == 0) return false;
        int li = min((int)(u * nAll), nAll - 1);
        *light = li;
        *pmfOut = 1.f / nAll;
        return true;
    }
    float pInfinite = float(S.nInfinite) / float(S.nInfinite + (S.nLightNodes == 0 ? 0 : 1));
    if (u < pInfinite) {
        u /= pInfinite;
        int index = min((int)(u * S.nInfinite), S.nInfinite - 1);
        *pmfOut = pInfinite / S.nInfinite;
        *light = S.nAreaLights + index;
        return true;
    }
    if (S.nLightNodes == 0) return false;
    u = fminf((u - pInfinite) / (1 - pInfinite), kOneMinusEpsilon);
    int nodeIndex = 0;
    float pmf = 1 - pInfinite;
    for (int iter = 0; iter < 4 * kMaxLightBVHDepth; ++iter) {
        DeviceLightNode node = S.lightNodes[nodeIndex];
        if (!node.isLeaf) {
            float c0 = LightImportance(S.lightNodes[nodeIndex + 1].b, p, ns);
            float c1 = LightImportance(S.lightNodes[node.childOrLight].b, p, ns);
            if (c0 == 0 && c1 == 0) return false;
            float nodePMF;
            int child = SampleDiscrete2(c0, c1, u, &nodePMF, &u);
            pmf *= nodePMF;
            nodeIndex = (child == 0) ? (nodeIndex + 1) : node.childOrLight;
        } else {
            if (nodeIndex > 0 || LightImportance(node.b, p, ns) > 0) {
                *light = node.childOrLight;
                *pmfOut = pmf;
                return true;
            }
            return false;
        }
    }
    return false;
}

__device__ inline float LightPMF(const DeviceScene &S, V3 p, V3 ns, int light) {
    int nAll = S.nAreaLights + S.nInfinite;
    if (S.uniformLightSampler) return nAll ? 1.f / nAll : 0.f;
    uint32_t bitTrail = light < S.nAreaLights ? S.lightBitTrail[light] : 0xffffffffu;
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

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(kBlock) k_camera(DeviceScene S, PathState st, int nActive) {
    int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot == 0) {
        st.counters[CounterIndex(0, kCntRay, 0)] = nActive;  // depth-0 records = every slot (shard 0)
        atomicAdd(&st.stats[0], (unsigned long long)nActive);
    }
    if (slot >= nActive) return;
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    // camera.cpp:50-62: wavelength Get1D, then GetCameraSample (samplers.h:797-813): pixel
    // offset (GetPixel2D) through the box filter (filters.h:67-71), time Get1D, lens Get2D
    float lu, pix0, pix1, l0, l1;
    if (S.samplerType == 1) {
        // ZSobolSampler: dimensions 0 (wavelength), 1-2 (pixel), 3 (time), 4-5 (lens)
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        lu = ZSobolGet1D(S.zs, morton, 0, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, 1, S.zsPerms, S.sobolM1, &pix0, &pix1);
        ZSobolGet2D(S.zs, morton, 4, S.zsPerms, S.sobolM1, &l0, &l1);
    } else {
        // HaltonSampler: GetPixel2D reads the pixel's own Halton digits, not a dimension
        Halton h = StartPixelSample(S, px, py, sampleIndex, 0);
        lu = Get1D(S, h);
        const uint64_t a0 = h.index >> S.baseExponents[0];
        const uint64_t a1 = (h.index >> 32) == 0 ? (uint64_t)((uint32_t)h.index / (uint32_t)S.baseScales[1])
                                                 : h.index / (uint64_t)S.baseScales[1];
        pix0 = a0 < (1ull << 30) ? RadicalInverse32<2>((uint32_t)a0) : RadicalInverse(2, a0);
        pix1 = a1 < (1ull << 30) ? RadicalInverse32<3>((uint32_t)a1) : RadicalInverse(3, a1);
        (void)Get1D(S, h);  // time (unused: static camera)
        Get2D(S, h, &l0, &l1);
    }
    float lambda0 = Lerpf(lu, kLambdaMin, kLambdaMax);
    float fx = Lerpf(pix0, -S.filterRadiusX, S.filterRadiusX), fy = Lerpf(pix1, -S.filterRadiusY, S.filterRadiusY);
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
    // Depth-0 record = the pixel-sample slot.  beta = 1, r_u = r_l = 1, etaScale = 1, flags = 0,
    // pixel = slot are implicit at depth 0 (the depth-0 kernels use the constants) and the box
    // filter's weight is always 1: none of them is stored.
    int N = st.N;
    st.L[slot] = 0;
    st.L[N + slot] = 0;
    st.L[2 * N + slot] = 0;
    if (!S.boxFilter) st.filterW[slot] = 1.f;
    const PathRecords &r = st.rec[0];
    const int NR = st.NR;
    r.lambda0[slot] = lambda0;
    r.ray[slot] = o.x;
    r.ray[NR + slot] = o.y;
    r.ray[2 * NR + slot] = o.z;
    r.ray[3 * NR + slot] = d.x;
    r.ray[4 * NR + slot] = d.y;
    r.ray[5 * NR + slot] = d.z;
}

// NMatQ = 1: every material is diffuse (one material queue); 3: one queue per material type
template <int NMatQ, bool Q>
__global__ void __launch_bounds__(kBlock, PBRT_TRAVERSAL_WAVES) k_closest(DeviceScene S, PathState st, int depth, int timed) {
    const QueueView rays = LoadQueue(st, depth, kCntRay);
    if ((int)(blockIdx.x * blockDim.x) >= rays.total) return;  // no work
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int N = st.NR;  // record stride
    const PathRecords &rec = st.rec[depth & 1];
    const int count = rays.total;
    const int shard = ProducerShard();
    int *escCounter = &st.counters[CounterIndex(depth, kCntEscaped, shard)];
    int *emitCounter = &st.counters[CounterIndex(depth, kCntEmissive, shard)];
    int *hitPrim = st.hitPrim[depth & 1];
    float *hitB = st.hitB[depth & 1];
    const bool shade = depth < S.maxDepth;  // at maxDepth only emission and escape matter
    constexpr int kQ = 2 + NMatQ;
    constexpr int kCap = NMatQ == 1 ? 512 : 256;  // entries per wave and queue
    __shared__ int qBuf[(kBlock / 64) * kQ * kCap];
    int *qCnt[kQ] = {escCounter, emitCounter};
    int *qArr[kQ] = {st.escQ + shard * st.capS, st.emitQ + shard * st.capS};
#pragma unroll
    for (int t = 0; t < NMatQ; ++t) {
        qCnt[2 + t] = &st.counters[CounterIndex(depth, MatCounter(t), shard)];
        qArr[2 + t] = st.matQ[t] + shard * st.capS;
    }
    WaveQueues<kQ, kCap> queues(qBuf, qCnt, qArr);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&st.stats[1], (unsigned long long)count);
        if (timed) atomicAdd(&st.stats[3], (unsigned long long)count);  // rays of event-timed launches
    }
    for (int base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        const int j = base + threadIdx.x;
        bool active = j < count;
        const int qi = active ? QueueSlot(rays, j) : 0;  // record index of this depth
        int prim = -1;
        TriHit h;
        if (active) {
            const V3 o(rec.ray[qi], rec.ray[N + qi], rec.ray[2 * N + qi]);
            const V3 d(rec.ray[3 * N + qi], rec.ray[4 * N + qi], rec.ray[5 * N + qi]);
            prim = Traverse<false, Q>(S, L, o, d, kInfinity, &h);
            if (prim >= 0) {
                hitPrim[qi] = prim;
                hitB[qi] = h.b0;
                hitB[N + qi] = h.b1;
                hitB[2 * N + qi] = h.b2;
                hitB[3 * N + qi] = h.t;
            }
        }
        // EnqueueWorkAfterIntersection / Miss (intersect.h:48-156): misses to the escaped-ray
        // queue (infinite lights only), emissive hits to the hit-area-light queue, every hit
        // to its material queue
        bool pred[kQ] = {S.nInfinite > 0 && active && prim < 0,
                         S.nAreaLights > 0 && active && prim >= 0 && S.primLight[prim] >= 0};
        if constexpr (NMatQ == 1) {
            pred[2] = shade && active && prim >= 0;
        } else {
            const int type = (shade && active && prim >= 0) ? S.matType[S.primMaterial[prim]] : -1;
#pragma unroll
            for (int t = 0; t < NMatQ; ++t) pred[2 + t] = type == t;
        }
        queues.Append(pred, qi);
    }
    queues.FlushAll();
}

// HandleEscapedRays (integrator.cpp:495-537) for UniformInfiniteLight: Le with MIS where
// PDF_Li(allowIncompletePDF = true) == 0, so r_l contributes nothing.
__global__ void __launch_bounds__(kBlock) k_escaped(DeviceScene S, PathState st, int depth) {
    const int N = st.N, NR = st.NR;
    const QueueView esc = LoadQueue(st, depth, kCntEscaped);
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < esc.total; qi += gridDim.x * blockDim.x) {
        const PathRecords &rec = st.rec[depth & 1];
        const int ri = st.escQ[QueueSlot(esc, qi)];
        const int slot = depth > 0 ? rec.pixel[ri] : ri;
        int fl = depth > 0 ? rec.flags[ri] : 0;
        float rl = depth > 0 ? rec.rl[ri] : 1.f;
        float denom = (depth == 0 || (fl & 1)) ? Avg31(1.f) : Avg31(1.f + rl * 0.f);
        const float invDenom = 1 / denom;
        float rgb[3] = {0, 0, 0};
        bool any = false;
        for (int li = 0; li < S.nInfinite; ++li) {
            const float *dense = S.dense + S.infSpectrum[li] * kDenseN;
            float scale = S.infScale[li];
            float sx = 0, sy = 0, sz = 0, lam = rec.lambda0[ri];
            bool nz = false;
            for (int i = 0; i < kNSpectrumSamples; ++i) {
                if (i > 0) {
                    lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
                    if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
                }
                int off = DenseOffset(lam);
                float Le = scale * (off < 0 ? 0.f : dense[off]);
                nz |= Le != 0;
                float v = ((depth > 0 ? rec.beta[i * NR + ri] : 1.f) * Le * invDenom) * kInvWavelengthPDF;
                float xb = off < 0 ? 0.f : S.sensor[off], yb = off < 0 ? 0.f : S.sensor[kDenseN + off],
                      zb = off < 0 ? 0.f : S.sensor[2 * kDenseN + off];
                sx = i == 0 ? xb * v : sx + xb * v;
                sy = i == 0 ? yb * v : sy + yb * v;
                sz = i == 0 ? zb * v : sz + zb * v;
            }
            if (!nz) continue;
            any = true;
            rgb[0] += S.imagingRatio * (sx / kNSpectrumSamples);
            rgb[1] += S.imagingRatio * (sy / kNSpectrumSamples);
            rgb[2] += S.imagingRatio * (sz / kNSpectrumSamples);
        }
        if (any) {
            st.L[slot] += rgb[0];
            st.L[N + slot] += rgb[1];
            st.L[2 * N + slot] += rgb[2];
        }
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

// HandleEmissiveIntersection (integrator.cpp:539-573) over the hit-area-light queue.  The MIS
// context (pbrt's prevIntrCtx: p, n, ns, pError of the previous surface) is rebuilt from the
// previous bounce's hit record with the same TriangleSurface arithmetic that produced it.
__global__ void __launch_bounds__(kBlock) k_emissive(DeviceScene S, PathState st, int depth) {
    const int N = st.NR, NL = st.N;  // record stride, pixel-sample stride (L)
    const QueueView emit = LoadQueue(st, depth, kCntEmissive);
    const int count = emit.total;
    const int *hitPrim = st.hitPrim[depth & 1];
    const float *hitB = st.hitB[depth & 1];
    const int *prevPrim = st.hitPrim[(depth + 1) & 1];
    const float *prevB = st.hitB[(depth + 1) & 1];
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < count; qi += gridDim.x * blockDim.x) {
        // The queue is short, so this kernel's time is its dependent-load chain: every load
        // that depends only on the slot is issued up front, beta's 31 values included.
        const PathRecords &rec = st.rec[depth & 1];
        const int ri = st.emitQ[QueueSlot(emit, qi)];
        const int prim = hitPrim[ri];
        const float b0 = hitB[ri], b1 = hitB[N + ri], b2 = hitB[2 * N + ri];
        const V3 rd(rec.ray[3 * N + ri], rec.ray[4 * N + ri], rec.ray[5 * N + ri]);
        const float lambda0 = rec.lambda0[ri];
        const int slot = depth > 0 ? rec.pixel[ri] : ri;
        const bool mis = depth > 0 && !(rec.flags[ri] & 1);
        const float rl = depth > 0 ? rec.rl[ri] : 1.f;
        const int pi = depth > 0 ? rec.prevIdx[ri] : 0;  // previous depth's record of this path
        const int pp = depth > 0 ? prevPrim[pi] : 0;
        const float pb0 = depth > 0 ? prevB[pi] : 0.f, pb1 = depth > 0 ? prevB[N + pi] : 0.f,
                    pb2 = depth > 0 ? prevB[2 * N + pi] : 0.f;
        float beta[kNSpectrumSamples];
#pragma unroll
        for (int i = 0; i < kNSpectrumSamples; ++i) beta[i] = depth > 0 ? rec.beta[(size_t)i * N + ri] : 1.f;
        V3 p0, p1, p2;
        PrimVerts(S, prim, &p0, &p1, &p2);
        const int light = S.primLight[prim];
        const bool flip = S.primFlip[prim];
        TriSurface surf = SurfaceAt(S, prim, p0, p1, p2, b0, b1, b2);
        (void)flip;
        V3 wo = Normalize(-rd);
        const DeviceAreaLight Ld = S.lights[light];
        if (!(Ld.twoSided || DotN(surf.n, wo) >= 0)) continue;
        float denom;
        if (!mis) {
            denom = Avg31(1.f);
        } else {
            V3 q0, q1, q2;
            PrimVerts(S, pp, &q0, &q1, &q2);
            // prevIntrCtx = LightSampleContext(pi, n, ns) of the previous surface
            TriSurface prev = SurfaceAt(S, pp, q0, q1, q2, pb0, pb1, pb2);
            float lightChoicePDF = LightPMF(S, prev.p, prev.ns, light);
            TriShading lsh;
            const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
            V3 l0(Ld.v0.x, Ld.v0.y, Ld.v0.z), l1(Ld.v1.x, Ld.v1.y, Ld.v1.z), l2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
            float lightPDF = lightChoicePDF * TrianglePDF(l0, l1, l2, Ld.flip, lhas ? &lsh : nullptr, prev.p,
                                                          prev.pErr, prev.n, prev.ns, -wo);
            denom = Avg31(1.f + rl * lightPDF);
        }
        const float *dense = S.dense + Ld.spectrum * kDenseN;
        const float invDenom = 1 / denom;
        SensorAcc acc;
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNSpectrumSamples; ++i, it.Next()) {
            int off = DenseOffset(it.lam);
            float Le = Ld.scale * (off < 0 ? 0.f : dense[off]);
            acc.Add(S, off, beta[i] * Le * invDenom, i == 0);
        }
        st.L[slot] += S.imagingRatio * (acc.sx / kNSpectrumSamples);
        st.L[NL + slot] += S.imagingRatio * (acc.sy / kNSpectrumSamples);
        st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNSpectrumSamples);
    }
}

#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) const float LdsF;
typedef __attribute__((address_space(3))) const uint16_t LdsU16;
#else
typedef const float LdsF;
typedef const uint16_t LdsU16;
#endif

// Light-sample contribution beta*f*|cos|*Le/denom summed to sensor RGB (surfscatter.cpp:288-308,
// then film.h:95-100); returns whether Le was nonzero at any wavelength.
template <typename FD>
__device__ inline bool NeeAccumulate(const FD *dense, const LdsF4 *sensor4, const float *bf, float lambda0,
                                     float scale, float absdot, float invDenom, SensorAcc *acc) {
    bool nz = false;
#pragma unroll 4
    for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
        int off = DenseOffset(it.lam);
        float Le = scale * (off < 0 ? 0.f : float(dense[off]));
        nz |= Le != 0;
        acc->Add(sensor4, off, bf[it.i * kBlock] * absdot * Le * invDenom, it.i == 0);
    }
    return nz;
}

// EvaluateMaterialAndBSDF<DiffuseMaterial> (surfscatter.cpp:57-328) fused with
// GenerateRaySamples (samples.cpp:29-66) for one depth.  Every table a lane looks up per
// wavelength or per sample is staged in LDS by the block first (ShadeLdsLayout): sensor
// curves, light spectra, this depth's 7 Halton permutation tables, lights, light BVH and
// materials.  The only HBM traffic per item is its path state, the hit triangle and beta,
// whose 31 values arrive by LDS-DMA while the sampler runs on LDS-resident tables.
// Tables the shade kernels stage in LDS per block (ShadeLdsLayout): sensor curves, light
// spectra, this depth's 7 Halton permutation tables, lights, light BVH and materials, plus the
// [31][kBlock] per-lane beta buffer (wavelength-major: conflict-free).
struct ShadeTables {
    ShadeLdsLayout lay;
    float *bfLds;
    float *denseLds;
    const LdsF4 *sensorL;
    const LdsU16 *permL;
    uint32_t permOff[7];
    DeviceScene SL;  // the light sampler reads its nodes from LDS
    const DeviceAreaLight *lightsL;
    const float4 *matsL;
    const int *matConstL;
};
__device__ __forceinline__ void StageShadeTables(const DeviceScene &S, int depth, char *ldsBase, ShadeTables *T) {
    const ShadeLdsLayout lay = S.shadeLds;
    T->lay = lay;
    T->bfLds = reinterpret_cast<float *>(ldsBase);
    float4 *sensorLds = reinterpret_cast<float4 *>(ldsBase + lay.sensor);
    T->denseLds = reinterpret_cast<float *>(ldsBase + lay.dense);
    uint16_t *permLds = reinterpret_cast<uint16_t *>(ldsBase + lay.perm);
    DeviceAreaLight *lightsLds = reinterpret_cast<DeviceAreaLight *>(ldsBase + lay.lights);
    DeviceLightNode *nodesLds = reinterpret_cast<DeviceLightNode *>(ldsBase + lay.lightNodes);
    float4 *matsLds = reinterpret_cast<float4 *>(ldsBase + lay.mats);
    int *matConstLds = reinterpret_cast<int *>(ldsBase + lay.matConst);
    DmaCopy<16>(S.sensor4, sensorLds, kDenseN);
    if (lay.denseInLds) DmaCopy<4>(S.dense, T->denseLds, S.nDense * kDenseN);
    // this depth's 7 permutation tables, stored contiguously per depth on the host
    const uint32_t *info = S.permDepthInfo + depth * 8;  // {start, off0..off6}
#pragma unroll
    for (int k = 0; k < 7; ++k) T->permOff[k] = info[1 + k];
    const uint32_t start = info[0], words = (S.permDepthInfo[(depth + 1) * 8] - start + 1) / 2;
    DmaCopy<4>(S.permByDepth + start, permLds, (int)words);
    if (lay.lightsInLds) {
        DmaCopy<4>(S.lights, lightsLds, S.nAreaLights * (int)(sizeof(DeviceAreaLight) / 4));
        DmaCopy<4>(S.lightNodes, nodesLds, S.nLightNodes * (int)(sizeof(DeviceLightNode) / 4));
    }
    if (lay.matsInLds) {
        DmaCopy<16>(S.matCoeffs, matsLds, S.nMaterials);
        DmaCopy<4>(S.matConstant, matConstLds, S.nMaterials);
    }
    DmaWait();
    __syncthreads();
    T->sensorL = (const LdsF4 *)sensorLds;
    T->permL = (const LdsU16 *)permLds;
    T->SL = S;
    if (lay.lightsInLds) T->SL.lightNodes = nodesLds;
    T->lightsL = lay.lightsInLds ? lightsLds : S.lights;
    T->matsL = lay.matsInLds ? matsLds : S.matCoeffs;
    T->matConstL = lay.matsInLds ? matConstLds : S.matConstant;
}

// GenerateRaySamples (samples.cpp:29-66): dims d0 + {0..6} = direct.uc, direct.u (2),
// indirect.uc, indirect.u (2), rr; Halton digit permutations come from the LDS tables
struct RaySamples {
    float dUc, dU0, dU1, iUc, iU0, iU1, rr;
};
template <bool IndirectUc>
__device__ __forceinline__ RaySamples GenerateRaySamples(const DeviceScene &S, const ShadeTables &T, int px, int py,
                                                         int sampleIndex, int d0) {
    RaySamples r;
    r.iUc = 0;
    if (S.samplerType == 1) {
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        r.dUc = ZSobolGet1D(S.zs, morton, d0, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 1, S.zsPerms, S.sobolM1, &r.dU0, &r.dU1);
        if (IndirectUc) r.iUc = ZSobolGet1D(S.zs, morton, d0 + 3, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 4, S.zsPerms, S.sobolM1, &r.iU0, &r.iU1);
        r.rr = ZSobolGet1D(S.zs, morton, d0 + 6, S.zsPerms, S.sobolM1);
    } else {
        const Halton h = StartPixelSample(S, px, py, sampleIndex, d0);
        auto dim = [&](int k) -> float {
            const HaltonDimDesc hd = S.haltonDim[d0 + k];
            if ((h.index >> 32) == 0 && hd.fast && hd.nDigits <= (uint32_t)kMaxMagicDigits)
                return ScrambledRadicalInverse32Magic<kMaxMagicDigits>(hd, (uint32_t)h.index, T.permL + T.permOff[k]);
            return ScrambledRadicalInverse(hd.base, hd.nDigits, h.index, S.perm + hd.permOffset);
        };
        r.dUc = dim(0);
        r.dU0 = dim(1);
        r.dU1 = dim(2);
        if (IndirectUc) r.iUc = dim(3);
        r.iU0 = dim(4);
        r.iU1 = dim(5);
        r.rr = dim(6);
    }
    return r;
}

__global__ void __launch_bounds__(kBlock, PBRT_SHADE_WAVES) k_shade_diffuse(DeviceScene S, PathState st, int depth) {
    const QueueView mats = LoadQueue(st, depth, kCntMat);
    if ((int)(blockIdx.x * blockDim.x) >= mats.total) return;  // no work
    extern __shared__ float4 dynLds[];
    ShadeTables T;
    StageShadeTables(S, depth, reinterpret_cast<char *>(dynLds), &T);
    const ShadeLdsLayout &lay = T.lay;
    float *bfLds = T.bfLds;
    float *denseLds = T.denseLds;
    const LdsF4 *sensorL = T.sensorL;
    const DeviceScene &SL = T.SL;
    const DeviceAreaLight *lightsL = T.lightsL;
    const float4 *matsL = T.matsL;
    const int *matConstL = T.matConstL;
    const int d0 = 6 + 7 * depth;  // first sampler dimension of this depth

    const int N = st.NR;  // record stride
    const int count = mats.total;
    const int shard = ProducerShard();
    int *nextCounter = &st.counters[CounterIndex(depth + 1, kCntRay, shard)];
    int *shadowCounter = &st.counters[CounterIndex(depth, kCntShadow, shard)];
    const int shardBase = shard * st.capS;
    const PathRecords &rec = st.rec[depth & 1], &out = st.rec[(depth + 1) & 1];
    const int *hitPrim = st.hitPrim[depth & 1];
    const float *hitB = st.hitB[depth & 1];
    for (int base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        int qi = base + threadIdx.x;
        bool active = qi < count;
        bool pushRay = false, pushShadow = false;
        const int ri = active ? st.matQ[0][QueueSlot(mats, qi)] : 0;  // this depth's record
        // outputs kept to the (block-wide) queue appends: shadow ray, continuing path
        V3 sOrg, sDir, sL, nOrg, nDir;
        float nRl = 0, nEta = 1;
        int slot = 0;
        float lambda0 = 0;
        SEC_BEGIN();
        if (active) {
            lambda0 = rec.lambda0[ri];
            slot = depth > 0 ? rec.pixel[ri] : ri;
            const float *betaP = rec.beta + ri;
            int prim = hitPrim[ri];
            float b0 = hitB[ri], b1 = hitB[N + ri], b2 = hitB[2 * N + ri];
            V3 rd(rec.ray[3 * N + ri], rec.ray[4 * N + ri], rec.ray[5 * N + ri]);
            int px, py, sampleIndex;
            PixelOf(st, slot, &px, &py, &sampleIndex);
            px += S.px0;
            V3 p0, p1, p2;
            PrimVerts(S, prim, &p0, &p1, &p2);
            const int mat = S.primMaterial[prim];
            TriSurface surf = SurfaceAt(S, prim, p0, p1, p2, b0, b1, b2);
            const float4 mc = matsL[mat];
            const bool constant = matConstL[mat];
            V3 wo = Normalize(-rd);
            V3 n = surf.n, ns = surf.ns;
            // beta_i -> bfLds[i][lane] by LDS-DMA: all 31 loads in flight at once, no VGPRs,
            // landing while the sampler below works from LDS (depth 0: beta = 1, no loads)
            if (depth > 0) {
                const int waveBase = threadIdx.x & ~63;
#pragma unroll
                for (int i = 0; i < kNSpectrumSamples; ++i)
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void *)(betaP + (size_t)i * N),
                        (__attribute__((address_space(3))) void *)(bfLds + i * kBlock + waveBase), 4, 0, 0);
            }
            SEC_MARK(st, 0);
            {
                // ---- GenerateRaySamples (samples.cpp:29-66): dims 6 + 7 * depth + {0..6}
                // = direct.uc, direct.u (2), indirect.uc, indirect.u (2), rr
                // dim 3 (indirect.uc) is unused by DiffuseBxDF
                const RaySamples rs = GenerateRaySamples<false>(S, T, px, py, sampleIndex, d0);
                const float dUc = rs.dUc, dU0 = rs.dU0, dU1 = rs.dU1, iU0 = rs.iU0, iU1 = rs.iU1, rr = rs.rr;
                SEC_MARK(st, 1);
                // ---- DiffuseMaterial::GetBxDF: R = clamp(reflectance(lambda), 0, 1); f = R / pi
                // (bxdfs.h DiffuseBxDF::f).  bf_i = beta_i * f_i is formed once per wavelength
                // into LDS; light sampling and the BSDF update both start from that product.
                bool Rnz = false;
                float *bf = bfLds + threadIdx.x;
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the beta LDS-DMA has landed
#pragma unroll 4
                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                    float R = Reflectance(mc, constant, it.lam);
                    Rnz |= R != 0;
                    bf[it.i * kBlock] = (depth > 0 ? bf[it.i * kBlock] : 1.f) * (R * kInvPi);
                }
                SEC_MARK(st, 2);
                Frame frame = Frame::FromXZ(Normalize(surf.dpdus), ns);
                V3 woL = frame.ToLocal(wo);
                V3 pi = surf.p, pe = surf.pErr;
                // ---- light sampling + shadow ray (surfscatter.cpp:254-326); reads the old beta
                if (Rnz) {
                    V3 cp = OffsetRayOrigin(pi, pe, n, wo);  // reflective, not transmissive
                    int li;
                    float lpmf;
                    if (SampleLight(SL, cp, ns, dUc, &li, &lpmf) && li < S.nAreaLights) {
                        const DeviceAreaLight &Ld = lightsL[li];
                        V3 q0(Ld.v0.x, Ld.v0.y, Ld.v0.z), q1(Ld.v1.x, Ld.v1.y, Ld.v1.z), q2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
                        V3 lp, lpe, ln;
                        float lpdf;
                        TriShading lsh;
                        const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
                        if (SampleTriangle(q0, q1, q2, Ld.flip, lhas ? &lsh : nullptr, cp, n, ns, dU0, dU1, &lp, &lpe,
                                           &ln, &lpdf) &&
                            lpdf != 0 && LengthSquared(lp - cp) != 0) {
                            SEC_MARK(st, 3);
                            V3 wi = Normalize(lp - cp);
                            V3 wiL = frame.ToLocal(wi);
                            if ((Ld.twoSided || DotN(ln, -wi) >= 0) && woL.z != 0 && woL.z * wiL.z > 0) {
                                const int spec = Ld.spectrum;
                                float scale = Ld.scale;
                                float absdot = AbsDotN(ns, wi);
                                float lightPDF = lpdf * lpmf;
                                float bsdfPDF = CosineHemispherePDF(fabsf(wiL.z));
                                float denom = Avg31(bsdfPDF + lightPDF);
                                const float invDenom = 1 / denom;
                                SensorAcc acc;
                                bool nz = lay.denseInLds
                                              ? NeeAccumulate((const LdsF *)denseLds + spec * kDenseN, sensorL, bf,
                                                              lambda0, scale, absdot, invDenom, &acc)
                                              : NeeAccumulate(S.dense + spec * kDenseN, sensorL, bf, lambda0, scale,
                                                              absdot, invDenom, &acc);
                                if (nz) {
                                    // SpawnRayTo(pi, n, time, pLight.pi, pLight.n) (ray.h:106-111)
                                    sOrg = OffsetRayOrigin(pi, pe, n, lp - pi);
                                    V3 pt = OffsetRayOrigin(lp, lpe, ln, sOrg - lp);
                                    sDir = pt - sOrg;
                                    sL = V3(S.imagingRatio * (acc.sx / kNSpectrumSamples),
                                            S.imagingRatio * (acc.sy / kNSpectrumSamples),
                                            S.imagingRatio * (acc.sz / kNSpectrumSamples));
                                    pushShadow = true;
                                }
                            }
                        }
                    }
                }
                SEC_MARK(st, 4);
                // ---- BSDF::Sample_f<DiffuseBxDF> + RR + indirect ray (surfscatter.cpp:170-250)
                if (woL.z != 0 && Rnz) {
                    V3 wiL = SampleCosineHemisphere(iU0, iU1);
                    if (woL.z < 0) wiL.z *= -1;
                    float pdf = CosineHemispherePDF(fabsf(wiL.z));
                    if (pdf != 0 && wiL.z != 0) {
                        V3 wi = frame.FromLocal(wiL);
                        float absdot = AbsDotN(ns, wi);
                        float etaScale = depth > 0 ? rec.etaScale[ri] : 1.f;
                        float avgRu = Avg31(1.f);
                        float mx = -kInfinity;
#pragma unroll 4
                        for (int i = 0; i < kNSpectrumSamples; ++i) {
                            float nbv = bf[i * kBlock] * absdot / pdf;
                            bf[i * kBlock] = nbv;
                            mx = fmaxf(mx, nbv * etaScale / avgRu);
                        }
                        SEC_MARK(st, 5);
                        bool kill = false;
                        float q = 0;
                        if (mx < 1 && depth >= 1) {
                            q = fmaxf(0.f, 1 - mx);
                            kill = rr < q;
                        }
                        if (!kill) {
                            bool rrScale = mx < 1 && depth >= 1;
                            bool nz = false;
#pragma unroll 4
                            for (int i = 0; i < kNSpectrumSamples; ++i) {
                                float nbv = bf[i * kBlock];
                                if (rrScale) nbv /= 1 - q;
                                nz |= nbv != 0;
                                bf[i * kBlock] = nbv;  // written out after the queue append
                            }
                            if (nz) {
                                nOrg = OffsetRayOrigin(pi, pe, n, wi);
                                nDir = wi;
                                nRl = 1.f / pdf;
                                nEta = etaScale;
                                pushRay = true;
                            }
                        }
                    }
                }
            }
        }
        SEC_MARK(st, 6);
        // Queue appends (one global atomic per block and queue): the shadow ray and the
        // continuing path are written densely at their queue positions (pbrt's
        // ShadowRayQueue / next RayQueue pushes, surfscatter.cpp:236-246, 310-316).
        int *const cnt[2] = {nextCounter, shadowCounter};
        const bool pred[2] = {pushRay, pushShadow};
        int pos[2];
        BlockPush<2>(cnt, pred, pos);
        if (pos[1] >= 0) {
            const int j = shardBase + pos[1];
            st.shadowRay[j] = sOrg.x;
            st.shadowRay[N + j] = sOrg.y;
            st.shadowRay[2 * N + j] = sOrg.z;
            st.shadowRay[3 * N + j] = sDir.x;
            st.shadowRay[4 * N + j] = sDir.y;
            st.shadowRay[5 * N + j] = sDir.z;
            st.shadowL[j] = sL.x;
            st.shadowL[N + j] = sL.y;
            st.shadowL[2 * N + j] = sL.z;
            st.shadowPixel[j] = slot;
        }
        if (pos[0] >= 0) {
            const int j = shardBase + pos[0];
            const float *bf = bfLds + threadIdx.x;
#pragma unroll 8
            for (int i = 0; i < kNSpectrumSamples; ++i) out.beta[(size_t)i * N + j] = bf[i * kBlock];
            out.ray[j] = nOrg.x;
            out.ray[N + j] = nOrg.y;
            out.ray[2 * N + j] = nOrg.z;
            out.ray[3 * N + j] = nDir.x;
            out.ray[4 * N + j] = nDir.y;
            out.ray[5 * N + j] = nDir.z;
            out.lambda0[j] = lambda0;
            out.rl[j] = nRl;
            out.etaScale[j] = nEta;
            out.flags[j] = 2;  // specularBounce = false, anyNonSpecular = true
            out.pixel[j] = slot;
            out.prevIdx[j] = ri;
        }
        SEC_MARK(st, 7);
    }
}

// EvaluateMaterialAndBSDF<DielectricMaterial | ConductorMaterial> (surfscatter.cpp:57-328) with
// GenerateRaySamples, over that material type's queue.  Same staging and queue appends as
// k_shade_diffuse; the BSDF is TrowbridgeReitz microfacet (core.h: DielectricSample/Eval,
// ConductorSample/Eval).  f differs between the light sample and the BSDF sample, so beta stays
// in bfLds and each 31-wavelength loop forms beta_i * f_i itself.  Specular BSDFs skip light
// sampling (IsNonSpecular(flags), surfscatter.cpp:253).
template <int MT>
__global__ void __launch_bounds__(kBlock, PBRT_SHADE_WAVES) k_shade_microfacet(DeviceScene S, PathState st, int depth) {
    const QueueView mats = LoadQueue(st, depth, MatCounter(MT));
    if ((int)(blockIdx.x * blockDim.x) >= mats.total) return;  // no work
    extern __shared__ float4 dynLds[];
    ShadeTables T;
    StageShadeTables(S, depth, reinterpret_cast<char *>(dynLds), &T);
    const ShadeLdsLayout &lay = T.lay;
    const int d0 = 6 + 7 * depth;
    const int N = st.NR;
    const int count = mats.total;
    const int shard = ProducerShard();
    int *nextCounter = &st.counters[CounterIndex(depth + 1, kCntRay, shard)];
    int *shadowCounter = &st.counters[CounterIndex(depth, kCntShadow, shard)];
    const int shardBase = shard * st.capS;
    const PathRecords &rec = st.rec[depth & 1], &out = st.rec[(depth + 1) & 1];
    const int *hitPrim = st.hitPrim[depth & 1];
    const float *hitB = st.hitB[depth & 1];
    const int *queue = st.matQ[MT];
    for (int base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
        int qi = base + threadIdx.x;
        bool active = qi < count;
        bool pushRay = false, pushShadow = false;
        const int ri = active ? queue[QueueSlot(mats, qi)] : 0;
        V3 sOrg, sDir, sL, nOrg, nDir;
        float nRl = 0, nEta = 1;
        int nFlags = 0;
        int slot = 0;
        float lambda0 = 0;
        float *bf = T.bfLds + threadIdx.x;  // beta_i at bf[i * kBlock]
        if (active) {
            lambda0 = rec.lambda0[ri];
            slot = depth > 0 ? rec.pixel[ri] : ri;
            const int inFlags = depth > 0 ? rec.flags[ri] : 0;
            const int prim = hitPrim[ri];
            const float b0 = hitB[ri], b1 = hitB[N + ri], b2 = hitB[2 * N + ri];
            const V3 rd(rec.ray[3 * N + ri], rec.ray[4 * N + ri], rec.ray[5 * N + ri]);
            int px, py, sampleIndex;
            PixelOf(st, slot, &px, &py, &sampleIndex);
            px += S.px0;
#pragma unroll 8
            for (int i = 0; i < kNSpectrumSamples; ++i) bf[i * kBlock] = depth > 0 ? rec.beta[(size_t)i * N + ri] : 1.f;
            V3 p0, p1, p2;
            PrimVerts(S, prim, &p0, &p1, &p2);
            const int mat = S.primMaterial[prim];
            const TriSurface surf = SurfaceAt(S, prim, p0, p1, p2, b0, b1, b2);
            const V3 wo = Normalize(-rd);
            const V3 n = surf.n, ns = surf.ns;
            const RaySamples rs = GenerateRaySamples<MT == kMatDielectricT>(S, T, px, py, sampleIndex, d0);
            // ---- Material::GetBxDF (materials.h:182-204 dielectric, :491-511 conductor)
            const float4 mp = S.matParams[mat];
            TrowbridgeReitz tr{mp.x, mp.y};
            if (S.regularize && (inFlags & 2)) tr.Regularize();  // surfscatter.cpp:127-128
            float eta = mp.z;
            if (eta == 0) eta = 1;
            // conductor eta_i / k_i: piecewise-linear spectra, or from the albedo "reflectance"
            const int etaSpec = MT == kMatConductorT ? S.matSpectra[2 * mat] : -1;
            const int kSpec = MT == kMatConductorT ? S.matSpectra[2 * mat + 1] : -1;
            const float4 mc = T.matsL[mat];
            auto etaK = [&](float lam, float *e, float *k) {
                if (etaSpec >= 0) {
                    const int a = S.plOffsets[etaSpec], na = S.plOffsets[etaSpec + 1] - a;
                    const int b = S.plOffsets[kSpec], nb = S.plOffsets[kSpec + 1] - b;
                    *e = PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, lam);
                    *k = PiecewiseLinearEval(S.plLambda + b, S.plValue + b, nb, lam);
                } else {
                    float r = Clampf(SigmoidPolynomial(mc.x, mc.y, mc.z, lam), 0, .9999f);
                    *e = 1.f;
                    *k = 2 * std::sqrt(r) / std::sqrt(std::fmax(0.f, 1 - r));
                }
            };
            const Frame frame = Frame::FromXZ(Normalize(surf.dpdus), ns);
            const V3 woL = frame.ToLocal(wo);
            const V3 pi = surf.p, pe = surf.pErr;
            const bool smooth = tr.EffectivelySmooth();
            const bool reflective = MT == kMatConductorT || eta != 1;
            const bool transmissive = MT == kMatDielectricT;
            // ---- light sampling + shadow ray (surfscatter.cpp:252-326)
            if (!smooth) {
                V3 cp = pi;
                if (reflective && !transmissive) cp = OffsetRayOrigin(pi, pe, n, wo);
                else if (transmissive && reflective) cp = OffsetRayOrigin(pi, pe, n, -wo);
                int li;
                float lpmf;
                if (SampleLight(T.SL, cp, ns, rs.dUc, &li, &lpmf) && li < S.nAreaLights) {
                    const DeviceAreaLight &Ld = T.lightsL[li];
                    V3 q0(Ld.v0.x, Ld.v0.y, Ld.v0.z), q1(Ld.v1.x, Ld.v1.y, Ld.v1.z), q2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
                    V3 lp, lpe, ln;
                    float lpdf;
                    TriShading lsh;
                    const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
                    if (SampleTriangle(q0, q1, q2, Ld.flip, lhas ? &lsh : nullptr, cp, n, ns, rs.dU0, rs.dU1, &lp,
                                       &lpe, &ln, &lpdf) &&
                        lpdf != 0 && LengthSquared(lp - cp) != 0) {
                        const V3 wi = Normalize(lp - cp);
                        const V3 wiL = frame.ToLocal(wi);
                        if ((Ld.twoSided || DotN(ln, -wi) >= 0) && woL.z != 0) {
                            // BSDF::f / BSDF::PDF (bsdf.h:60-135)
                            float fd = 0, bsdfPDF = 0;
                            ConductorTerms ct{};
                            bool fAny;
                            if constexpr (MT == kMatDielectricT) {
                                fd = DielectricEval(eta, tr, woL, wiL, &bsdfPDF);
                                fAny = fd != 0;
                            } else {
                                ct = ConductorEval(tr, woL, wiL);
                                bsdfPDF = ct.pdf;
                                fAny = ct.ok;  // f_i may still vanish; a zero Ld adds nothing
                            }
                            if (fAny) {
                                const float absdot = AbsDotN(ns, wi);
                                const float lightPDF = lpdf * lpmf;
                                const float invDenom = 1 / Avg31(bsdfPDF + lightPDF);
                                const float *dense = lay.denseInLds ? nullptr : S.dense + Ld.spectrum * kDenseN;
                                const LdsF *denseL = (const LdsF *)T.denseLds + Ld.spectrum * kDenseN;
                                SensorAcc acc;
                                bool nz = false;
#pragma unroll 2
                                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                                    const int off = DenseOffset(it.lam);
                                    const float Le =
                                        Ld.scale * (off < 0 ? 0.f : (lay.denseInLds ? float(denseL[off]) : dense[off]));
                                    nz |= Le != 0;
                                    float f = fd;
                                    if constexpr (MT == kMatConductorT) {
                                        float e, k;
                                        etaK(it.lam, &e, &k);
                                        f = ConductorF(ct, e, k);
                                    }
                                    acc.Add(T.sensorL, off, bf[it.i * kBlock] * f * absdot * Le * invDenom, it.i == 0);
                                }
                                if (nz) {
                                    sOrg = OffsetRayOrigin(pi, pe, n, lp - pi);
                                    const V3 pt = OffsetRayOrigin(lp, lpe, ln, sOrg - lp);
                                    sDir = pt - sOrg;
                                    sL = V3(S.imagingRatio * (acc.sx / kNSpectrumSamples),
                                            S.imagingRatio * (acc.sy / kNSpectrumSamples),
                                            S.imagingRatio * (acc.sz / kNSpectrumSamples));
                                    pushShadow = true;
                                }
                            }
                        }
                    }
                }
            }
            // ---- BSDF::Sample_f + RR + indirect ray (surfscatter.cpp:183-250)
            if (woL.z != 0) {
                bool ok;
                V3 wiL;
                float pdf, fd = 0, etap = 1;
                bool specular, transmission;
                ConductorTerms ct{};
                if constexpr (MT == kMatDielectricT) {
                    const BxSample bs = DielectricSample(eta, tr, woL, rs.iUc, rs.iU0, rs.iU1);
                    ok = bs.ok && bs.f != 0;
                    wiL = bs.wi;
                    pdf = bs.pdf;
                    fd = bs.f;
                    etap = bs.etap;
                    specular = bs.flags & kBxSpecular;
                    transmission = bs.flags & kBxTransmission;
                } else {
                    ct = ConductorSample(tr, woL, rs.iU0, rs.iU1);
                    ok = ct.ok;
                    wiL = ct.wi;
                    pdf = ct.pdf;
                    specular = ct.specular;
                    transmission = false;
                }
                if (ok && pdf != 0 && wiL.z != 0) {
                    const V3 wi = frame.FromLocal(wiL);
                    const float absdot = AbsDotN(ns, wi);
                    float etaScale = depth > 0 ? rec.etaScale[ri] : 1.f;
                    if (transmission) etaScale *= Sqr(etap);
                    const float avgRu = Avg31(1.f);
                    float mx = -kInfinity;
                    bool fAny = MT == kMatDielectricT;
#pragma unroll 2
                    for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                        float f = fd;
                        if constexpr (MT == kMatConductorT) {
                            float e, k;
                            etaK(it.lam, &e, &k);
                            f = ConductorF(ct, e, k);
                            fAny |= f != 0;
                        }
                        const float nbv = bf[it.i * kBlock] * f * absdot / pdf;
                        bf[it.i * kBlock] = nbv;
                        mx = fmaxf(mx, nbv * etaScale / avgRu);
                    }
                    if (fAny) {
                        bool kill = false;
                        float q = 0;
                        if (mx < 1 && depth >= 1) {
                            q = fmaxf(0.f, 1 - mx);
                            kill = rs.rr < q;
                        }
                        if (!kill) {
                            const bool rrScale = mx < 1 && depth >= 1;
                            bool nz = false;
#pragma unroll 4
                            for (int i = 0; i < kNSpectrumSamples; ++i) {
                                float nbv = bf[i * kBlock];
                                if (rrScale) nbv /= 1 - q;
                                nz |= nbv != 0;
                                bf[i * kBlock] = nbv;
                            }
                            if (nz) {
                                nOrg = OffsetRayOrigin(pi, pe, n, wi);
                                nDir = wi;
                                nRl = 1.f / pdf;
                                nEta = etaScale;
                                nFlags = (specular ? 1 : 0) | ((!specular || (inFlags & 2)) ? 2 : 0);
                                pushRay = true;
                            }
                        }
                    }
                }
            }
        }
        int *const cnt[2] = {nextCounter, shadowCounter};
        const bool pred[2] = {pushRay, pushShadow};
        int pos[2];
        BlockPush<2>(cnt, pred, pos);
        if (pos[1] >= 0) {
            const int j = shardBase + pos[1];
            st.shadowRay[j] = sOrg.x;
            st.shadowRay[N + j] = sOrg.y;
            st.shadowRay[2 * N + j] = sOrg.z;
            st.shadowRay[3 * N + j] = sDir.x;
            st.shadowRay[4 * N + j] = sDir.y;
            st.shadowRay[5 * N + j] = sDir.z;
            st.shadowL[j] = sL.x;
            st.shadowL[N + j] = sL.y;
            st.shadowL[2 * N + j] = sL.z;
            st.shadowPixel[j] = slot;
        }
        if (pos[0] >= 0) {
            const int j = shardBase + pos[0];
#pragma unroll 8
            for (int i = 0; i < kNSpectrumSamples; ++i) out.beta[(size_t)i * N + j] = bf[i * kBlock];
            out.ray[j] = nOrg.x;
            out.ray[N + j] = nOrg.y;
            out.ray[2 * N + j] = nOrg.z;
            out.ray[3 * N + j] = nDir.x;
            out.ray[4 * N + j] = nDir.y;
            out.ray[5 * N + j] = nDir.z;
            out.lambda0[j] = lambda0;
            out.rl[j] = nRl;
            out.etaScale[j] = nEta;
            out.flags[j] = nFlags;
            out.pixel[j] = slot;
            out.prevIdx[j] = ri;
        }
    }
}

template <bool Q>
__global__ void __launch_bounds__(kBlock, PBRT_TRAVERSAL_WAVES) k_shadow(DeviceScene S, PathState st, int depth) {
    const QueueView shadows = LoadQueue(st, depth, kCntShadow);
    if ((int)(blockIdx.x * blockDim.x) >= shadows.total) return;  // no work
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int N = st.NR, NL = st.N;
    const int count = shadows.total;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[2], (unsigned long long)count);
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < count; qi += gridDim.x * blockDim.x) {
        // the shadow queue is dense per shard: entry p holds the ray, its contribution and pixel
        const int p = QueueSlot(shadows, qi);
        V3 o(st.shadowRay[p], st.shadowRay[N + p], st.shadowRay[2 * N + p]);
        V3 d(st.shadowRay[3 * N + p], st.shadowRay[4 * N + p], st.shadowRay[5 * N + p]);
        TriHit h;
        int hit = Traverse<true, Q>(S, L, o, d, 1 - kShadowEpsilon, &h);
        if (hit < 0) {
            const int slot = st.shadowPixel[p];
            st.L[slot] += st.shadowL[p];
            st.L[NL + slot] += st.shadowL[N + p];
            st.L[2 * NL + slot] += st.shadowL[2 * N + p];
        }
    }
}

// UpdateFilm: one thread per pixel walks its samples in sample order (deterministic sums)
__global__ void __launch_bounds__(kBlock) k_film(DeviceScene S, PathState st, int nSamples) {
    int pl = blockIdx.x * blockDim.x + threadIdx.x;
    if (pl >= st.P) return;
    int N = st.N;
    int r = pl / st.width;
    int px = S.px0 + (pl - r * st.width), py = st.rows[r];
    size_t pix = (size_t)py * S.xres + px;
    size_t npix = (size_t)S.xres * S.yres;
    double sr = st.film[pix], sg = st.film[npix + pix], sb = st.film[2 * npix + pix], sw = st.film[3 * npix + pix];
    for (int s = 0; s < nSamples; ++s) {
        int slot = s * st.P + pl;
        float w = S.boxFilter ? 1.f : st.filterW[slot];
        float rr = st.L[slot], gg = st.L[N + slot], bb = st.L[2 * N + slot];
        sr += w * rr;
        sg += w * gg;
        sb += w * bb;
        sw += w;
    }
    st.film[pix] = sr;
    st.film[npix + pix] = sg;
    st.film[2 * npix + pix] = sb;
    st.film[3 * npix + pix] = sw;
}

// ------------------------------------------------------------------ stand-alone intersection
// The WavefrontAggregate boundary exposed on its own (integrator.h:32-54): closest / any hit
// for an SoA ray batch, used by parity tests and the traversal benchmark.
template <bool Q>
__global__ void __launch_bounds__(kBlock, 4) k_intersect_batch(DeviceScene S, const float *rays, int n, int anyHit,
                                                              int *outPrim, float *outHit) {
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        V3 o(rays[i], rays[n + i], rays[2 * n + i]);
        V3 d(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
        float tMax = rays[6 * n + i];
        TriHit h{0, 0, 0, 0};
        int prim = anyHit ? Traverse<true, Q>(S, L, o, d, tMax, &h) : Traverse<false, Q>(S, L, o, d, tMax, &h);
        outPrim[i] = prim;
        outHit[i] = h.b0;
        outHit[n + i] = h.b1;
        outHit[2 * n + i] = h.b2;
        outHit[3 * n + i] = h.t;
    }
}

// ------------------------------------------------------------------ launch helpers (host)
size_t TraversalLdsBytes(int stackSize, int ldsNodes, int ldsTris, int compressed) {
    return (size_t)stackSize * kBlock * sizeof(int) + (size_t)ldsNodes * LdsNodeStride(compressed) * 16 +
           (size_t)ldsTris * 48;
}
static size_t StackBytes(const DeviceScene &S) {
    return TraversalLdsBytes(S.stackSize, S.ldsNodes, S.ldsTris, S.compressed);
}

// Traversal kernels loop over their queue inside a bounded grid so the LDS scene cache is
// filled once per block, not once per 256 rays.
#ifndef PBRT_GRID_CAP
#define PBRT_GRID_CAP 1024
#endif
#ifndef PBRT_SHADE_GRID_CAP
#define PBRT_SHADE_GRID_CAP 2048
#endif
// Producer grids are multiples of kShards (the shard capacity bound depends on it).
static int ShardedGrid(int n, int cap) {
    int g = (n + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > cap ? cap : g);
    return (g + kShards - 1) / kShards * kShards;
}
static int TraversalGridFor(int n) { return ShardedGrid(n, PBRT_GRID_CAP); }
static int ShadeGridFor(int n) { return ShardedGrid(n, PBRT_SHADE_GRID_CAP); }

// Kernels over queues that are usually short (emissive hits, escaped rays): a grid of one
// block per CU, grid-stride beyond that.
static int SmallGridFor(int n) {
    int g = (n + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 256 ? 256 : g);
}

static int GridFor(int n) {
    int g = (n + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > 8192 ? 8192 : g);
}

hipError_t LaunchCamera(const DeviceScene &S, const PathState &st, int nActive, hipStream_t s) {
    hipLaunchKernelGGL(k_camera, dim3((nActive + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, nActive);
    return hipGetLastError();
}
hipError_t LaunchClosest(const DeviceScene &S, const PathState &st, int depth, int maxCount, int timed,
                         hipStream_t s) {
    const dim3 grid(TraversalGridFor(maxCount)), block(kBlock);
    const bool multi = S.matTypeMask & ~1;
    if (S.compressed) {
        if (multi) hipLaunchKernelGGL((k_closest<kNumMatTypes, true>), grid, block, StackBytes(S), s, S, st, depth, timed);
        else hipLaunchKernelGGL((k_closest<1, true>), grid, block, StackBytes(S), s, S, st, depth, timed);
    } else {
        if (multi) hipLaunchKernelGGL((k_closest<kNumMatTypes, false>), grid, block, StackBytes(S), s, S, st, depth, timed);
        else hipLaunchKernelGGL((k_closest<1, false>), grid, block, StackBytes(S), s, S, st, depth, timed);
    }
    return hipGetLastError();
}
hipError_t LaunchEscaped(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_escaped, dim3(SmallGridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchEmissive(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_emissive, dim3(SmallGridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadeDiffuse(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_shade_diffuse, dim3(ShadeGridFor(maxCount)), dim3(kBlock), (size_t)S.shadeLds.total, s,
                       S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadeMicrofacet(const DeviceScene &S, const PathState &st, int depth, int type, int maxCount,
                                 hipStream_t s) {
    if (type == kMatDielectricT)
        hipLaunchKernelGGL(k_shade_microfacet<kMatDielectricT>, dim3(ShadeGridFor(maxCount)), dim3(kBlock),
                           (size_t)S.shadeLds.total, s, S, st, depth);
    else
        hipLaunchKernelGGL(k_shade_microfacet<kMatConductorT>, dim3(ShadeGridFor(maxCount)), dim3(kBlock),
                           (size_t)S.shadeLds.total, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadow(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    if (S.compressed)
        hipLaunchKernelGGL(k_shadow<true>, dim3(TraversalGridFor(maxCount)), dim3(kBlock), StackBytes(S), s, S, st, depth);
    else
        hipLaunchKernelGGL(k_shadow<false>, dim3(TraversalGridFor(maxCount)), dim3(kBlock), StackBytes(S), s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchFilm(const DeviceScene &S, const PathState &st, int nSamples, hipStream_t s) {
    hipLaunchKernelGGL(k_film, dim3((st.P + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, nSamples);
    return hipGetLastError();
}
hipError_t LaunchIntersectBatch(const DeviceScene &S, const float *rays, int n, int anyHit, int *outPrim,
                                float *outHit, hipStream_t s) {
    if (S.compressed)
        hipLaunchKernelGGL(k_intersect_batch<true>, dim3(TraversalGridFor(n)), dim3(kBlock), StackBytes(S), s, S, rays,
                           n, anyHit, outPrim, outHit);
    else
        hipLaunchKernelGGL(k_intersect_batch<false>, dim3(TraversalGridFor(n)), dim3(kBlock), StackBytes(S), s, S, rays,
                           n, anyHit, outPrim, outHit);
    return hipGetLastError();
}

}  // namespace pbrt_amd
