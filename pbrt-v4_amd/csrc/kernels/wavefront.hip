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
#include "common.h"
#include "../core/hair.h"
#include "../core/bssrdf.h"

namespace pbrt_amd {
// Traversal LDS of one block (shared with volpath.hip): group stack (uint2 entries), cached
// nodes, cached triangles in three pre-rotated copies
size_t TraversalLdsBytes(int stackSize, int ldsNodes, int ldsTris, int compressed) {
    return (size_t)stackSize * kBlock * sizeof(uint2) + (size_t)ldsNodes * LdsNodeStride(compressed) * 16 +
           (size_t)ldsTris * 3 * 48;
}

// The sensor's x/y/z-bar table as the shade kernels read it (staged in LDS; reading it through
// the L1 instead, to fit four blocks per CU, measured 5 % slower: profiles/r02_shade_ablation.txt)
typedef LdsF4 SensorF4;

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(kBlock) k_camera(DeviceScene S, PathState st, int nActive) {
    int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot == 0) {
        st.counters[CounterIndex(0, kCntRay, 0)] = nActive;  // depth-0 records = every slot (shard 0)
        atomicAdd(&st.stats[0], (unsigned long long)nActive);
    }
    if (slot >= nActive) return;
    float lambda0;
    V3 o, d;
    float filterWeight;
    uint32_t sidx;
    GenerateCameraRay(S, st, slot, &lambda0, &o, &d, &filterWeight, &sidx);
    // Depth-0 record = the pixel-sample slot.  beta = 1, r_u = r_l = 1, etaScale = 1, flags = 0,
    // pixel = slot are implicit at depth 0 (the depth-0 kernels use the constants) and the box
    // filter's weight is always 1: none of them is stored.
    int N = st.N;
    st.L[slot] = 0;
    st.L[N + slot] = 0;
    st.L[2 * N + slot] = 0;
    if (!S.boxFilter) st.filterW[slot] = filterWeight;
    const PathRecords &r = st.rec[0];
    const int NR = st.NR;
    r.lambda0[slot] = lambda0;
    r.sidx[slot] = sidx;
    r.ray[slot] = o.x;
    r.ray[NR + slot] = o.y;
    r.ray[2 * NR + slot] = o.z;
    r.ray[3 * NR + slot] = d.x;
    r.ray[4 * NR + slot] = d.y;
    r.ray[5 * NR + slot] = d.z;
}

// NMatQ = 1: every material is diffuse (one material queue); 3: one queue per material type;
// kClosestMix (4): one queue per type, and mix materials resolved per hit (into st.hitMat)
constexpr int kClosestMix = 4;
// sorted: this depth's rays were binned (k_raybin_*): lane j traces st.raySort[j] and only
// writes its hit record; k_classify then enqueues the hits in record order.
template <int NMatQ_, int TM>
__global__ void __launch_bounds__(kBlock, ClosestWaves(TM))
    k_closest(DeviceScene S, PathState st, int depth, int timed, int sorted) {
    constexpr bool kMix = NMatQ_ == kClosestMix;
    constexpr int NMatQ = kMix ? kNumMatTypes : NMatQ_;
    const QueueView rays = LoadQueue(st, depth, kCntRay);
    ChunkWalk walk = XcdChunks(rays.total, S.xcdGroups);
    if (walk.n >= walk.end) return;  // no work
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
    // entries per wave and queue: small enough that the staging (12 / 10 KB per block) leaves
    // room for the group stack and the node cache at TraversalWaves(TM) blocks per CU
    // (keyed on the wide / quantised modes' waves: the all-LDS mode keeps the full staging)
    constexpr int kCap = TraversalWaves(TM) > 4 ? 64 : (NMatQ == 1 ? 256 : 128);
    __shared__ int qBuf[(kBlock / 64) * kQ * kCap];
    int *qCnt[kQ] = {escCounter, emitCounter};
    int *qArr[kQ] = {st.escQ + shard * st.capS, st.emitQ + shard * st.capS};
#pragma unroll
    for (int t = 0; t < NMatQ; ++t) {
        qCnt[2 + t] = &st.counters[CounterIndex(depth, MatCounter(t), shard)];
        qArr[2 + t] = st.matQ[t] + shard * st.capS;
    }
    WaveQueues<kQ, kCap> queues(qBuf, qCnt, qArr, st.capS);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&st.stats[1], (unsigned long long)count);
        if (timed) atomicAdd(&st.stats[3], (unsigned long long)count);  // rays of event-timed launches
    }
    // A traced ray's results (every lane of the wave calls it; active: this lane has one): the
    // hit record, and unless the depth was binned the queue entries
    auto finish = [&](bool active, int qi, int prim, const TriHit &h, V3 d) {
        if (active) {
            if (sorted) {
                hitPrim[qi] = prim;
                if (prim >= 0) {
                    hitB[qi] = h.b0;
                    hitB[N + qi] = h.b1;
                    hitB[2 * N + qi] = h.b2;
                    hitB[3 * N + qi] = h.t;
                    if constexpr (kMix) {
                        int mat = S.primMaterial[prim];
                        if (S.matType[mat] == kMatMixT) mat = ResolveMixMaterial(*S.self, prim, mat, h.b0, h.b1, h.b2, d);
                        st.hitMat[depth & 1][qi] = mat;
                    }
                }
            }
            // the hit record feeds the material stage, and at maxDepth only k_emissive
            if (!sorted && prim >= 0 && (shade || S.primLight[prim] >= 0)) {
                hitPrim[qi] = prim;
                hitB[qi] = h.b0;
                hitB[N + qi] = h.b1;
                hitB[2 * N + qi] = h.b2;
                hitB[3 * N + qi] = h.t;
            }
        }
        if (sorted) return;  // k_classify enqueues
        // EnqueueWorkAfterIntersection / Miss (intersect.h:48-156): misses to the escaped-ray
        // queue (infinite lights only), emissive hits to the hit-area-light queue, every hit
        // to its material queue
        bool pred[kQ] = {S.nInfinite > 0 && active && prim < 0,
                         S.nAreaLights > 0 && active && prim >= 0 && S.primLight[prim] >= 0};
        if constexpr (NMatQ == 1) {
            pred[2] = shade && active && prim >= 0;
        } else {
            int type = -1;
            if (shade && active && prim >= 0) {
                int mat = S.primMaterial[prim];
                if constexpr (kMix) {
                    if (S.matType[mat] == kMatMixT) mat = ResolveMixMaterial(*S.self, prim, mat, h.b0, h.b1, h.b2, d);
                    st.hitMat[depth & 1][qi] = mat;
                }
                type = S.matType[mat];
            }
#pragma unroll
            for (int t = 0; t < NMatQ; ++t) pred[2 + t] = type == t;
        }
        queues.Append(pred, qi);
    };
    auto fetch = [&](int j, int &qi, V3 &o, V3 &d) {
        if (sorted) {
            const float4 a = st.raySort[j], b = st.raySort[(size_t)N + j];
            qi = __float_as_int(a.w);
            o = V3(a.x, a.y, a.z);
            d = V3(b.x, b.y, b.z);
        } else {
            qi = QueueSlot(rays, j);
            o = V3(rec.ray[qi], rec.ray[N + qi], rec.ray[2 * N + qi]);
            d = V3(rec.ray[3 * N + qi], rec.ray[4 * N + qi], rec.ray[5 * N + qi]);
        }
    };
    for (; walk.n < walk.end; walk.n += walk.step) {
        const int j = walk.Chunk() * blockDim.x + threadIdx.x;
        bool active = j < count;
        int qi = 0;  // record index of this depth
        int prim = -1;
        TriHit h;
        TravCount tc;
        V3 o, d;
        if (active) {
            fetch(j, qi, o, d);
            prim = Traverse<false, TM>(S, L, o, d, kInfinity, &h, &tc);
        }
        finish(active, qi, prim, h, d);
        TravStatsAdd(st.stats, kStatsSectionBase + 8, active, tc);
    }
    queues.FlushAll();
}

// ---- Ray binning for HBM-resident trees (depth >= 1).  Secondary rays arrive in record order
// (roughly pixel order, random directions), so a wave's 64 traversals diverge through a tree
// far larger than L2.  A counting sort by origin cell (8^3 Morton grid over the scene bounds)
// and direction octant groups rays that visit the same nodes: k_raybin_hist counts the bins,
// k_raybin_scan turns counts into offsets, k_raybin_scatter writes each ray with its record
// index to st.raySort in bin order.  k_closest<sorted> traces that order and writes hit
// records only; k_classify then enqueues the hits in record order, so the material queues --
// and the shade kernels' beta reads -- keep their coalesced layout.  Films are unchanged (each
// path's arithmetic is independent of the order rays are traced in).
constexpr int kRayBins = 4096, kBinBlock = 1024, kBinItems = 4;
// Treelet of the ray origin: point location from the root of the quantised tree, `levels`
// steps down the first interior child whose box contains o; the key is the path of slots (3
// bits per level, 0 below a stop).  Sibling treelets get adjacent keys, so bin order walks the
// tree's subtrees in turn and a CU's rays share the HBM-resident nodes below the LDS top.
__device__ inline int TreeletKey(const DeviceScene &S, const V3 &o, int levels) {
    int node = 0, path = 0;
    for (int l = 0; l < levels; ++l) {
        int slot = 8, next = -1;
        if (node >= 0) {
            const float4 *q = S.qnodes + (size_t)node * S.qStride;
            const float4 f0 = q[0], f1 = q[1], f2 = q[2], f3 = q[3], f4 = q[4];
            const uint32_t eb = __float_as_uint(f0.w), imask = eb >> 24;
            const float p[3] = {f0.x, f0.y, f0.z};
            const float sc[3] = {__uint_as_float((eb & 0xffu) << 23), __uint_as_float(((eb >> 8) & 0xffu) << 23),
                                 __uint_as_float(((eb >> 16) & 0xffu) << 23)};
            const uint32_t qw[12] = {__float_as_uint(f2.x), __float_as_uint(f2.y), __float_as_uint(f2.z),
                                     __float_as_uint(f2.w), __float_as_uint(f3.x), __float_as_uint(f3.y),
                                     __float_as_uint(f3.z), __float_as_uint(f3.w), __float_as_uint(f4.x),
                                     __float_as_uint(f4.y), __float_as_uint(f4.z), __float_as_uint(f4.w)};
            for (int c = 0; c < 8 && slot == 8; ++c) {
                if (!((imask >> c) & 1u)) continue;
                const int g = c >> 2, k = c & 3;
                bool in = true;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const float lo = fmaf((float)((qw[2 * a + g] >> (8 * k)) & 0xffu), sc[a], p[a]);
                    const float hi = fmaf((float)((qw[6 + 2 * a + g] >> (8 * k)) & 0xffu), sc[a], p[a]);
                    in = in && o[a] >= lo && o[a] <= hi;
                }
                if (in) {
                    slot = c;
                    next = __float_as_int(f1.x) + __popc(imask & ((1u << c) - 1u));
                }
            }
        }
        path = path << 3 | (slot & 7);
        node = next;
    }
    return path;
}
__device__ inline int RayBinKey(const DeviceScene &S, const V3 &o, const V3 &d) {
    // S.rayBinMode: 0 = origin 8^3 x octant; 1 = origin 4^3 x direction 8x8 (octahedral);
    // 2 = origin 2^3 x direction 32x16; 3 = origin treelet (3 levels) x octant; 4 = origin
    // treelet (4 levels).  The treelet keys need the quantised tree (else mode 0).
    const int mode = S.rayBinMode;
    if (mode >= 3 && S.compressed) {
        if (mode == 4) return TreeletKey(S, o, 4);
        return TreeletKey(S, o, 3) << 3 | (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
    }
    const int cBits = (mode == 0 || mode >= 3) ? 3 : (mode == 1 ? 2 : 1);
    const float cScale = (mode == 0 || mode >= 3) ? 1.f : (mode == 1 ? 0.5f : 0.25f);
    const float cMax = (float)((1 << cBits) - 1);
    int c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float t = (o[a] - S.rayBinLo[a]) * S.rayBinScale[a] * cScale;
        c[a] = (int)fminf(fmaxf(t, 0.f), cMax);  // NaN -> 0
    }
    int m = 0;
    for (int b = 0; b < cBits; ++b)
#pragma unroll
        for (int a = 0; a < 3; ++a) m |= ((c[a] >> b) & 1) << (3 * b + a);
    if (mode == 0 || mode >= 3) return m << 3 | (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
    // octahedral direction cell
    const float l1 = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float x = l1 > 0 ? d.x / l1 : 0.f, y = l1 > 0 ? d.y / l1 : 0.f;
    if (d.z < 0) {
        const float ox = x;
        x = (1 - fabsf(y)) * (ox < 0 ? -1.f : 1.f);
        y = (1 - fabsf(ox)) * (y < 0 ? -1.f : 1.f);
    }
    const int ub = mode == 1 ? 3 : 5, vb = mode == 1 ? 3 : 4;
    const int u = (int)fminf(fmaxf((x + 1) * 0.5f * (1 << ub), 0.f), (float)((1 << ub) - 1));
    const int v = (int)fminf(fmaxf((y + 1) * 0.5f * (1 << vb), 0.f), (float)((1 << vb) - 1));
    return m << (ub + vb) | u << vb | v;
}
__device__ inline void RayAt(const PathState &st, int depth, int qi, V3 *o, V3 *d) {
    const PathRecords &rec = st.rec[depth & 1];
    const int N = st.NR;
    *o = V3(rec.ray[qi], rec.ray[N + qi], rec.ray[2 * N + qi]);
    *d = V3(rec.ray[3 * N + qi], rec.ray[4 * N + qi], rec.ray[5 * N + qi]);
}
__global__ void __launch_bounds__(kBinBlock) k_raybin_hist(DeviceScene S, PathState st, int depth) {
    const QueueView rays = LoadQueue(st, depth, kCntRay);
    if ((int)(blockIdx.x * blockDim.x) >= rays.total) return;
    __shared__ int h[kRayBins];
    for (int i = threadIdx.x; i < kRayBins; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < rays.total; j += gridDim.x * blockDim.x) {
        V3 o, d;
        RayAt(st, depth, QueueSlot(rays, j), &o, &d);
        atomicAdd(&h[RayBinKey(S, o, d)], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kRayBins; i += blockDim.x)
        if (h[i]) atomicAdd(&st.rayBins[i], h[i]);
}
// one block: exclusive offsets into rayBins[kRayBins..], counts cleared for the next depth
__global__ void __launch_bounds__(kBinBlock) k_raybin_scan(PathState st) {
    __shared__ int part[kBinBlock];
    constexpr int kPer = kRayBins / kBinBlock;
    const int t = threadIdx.x;
    int v[kPer], sum = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) sum += (v[k] = st.rayBins[kPer * t + k]);
    part[t] = sum;
    __syncthreads();
    for (int off = 1; off < kBinBlock; off <<= 1) {
        const int x = t >= off ? part[t - off] : 0;
        __syncthreads();
        part[t] += x;
        __syncthreads();
    }
    int run = part[t] - sum;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        st.rayBins[kRayBins + kPer * t + k] = run;
        run += v[k];
        st.rayBins[kPer * t + k] = 0;
    }
}
__global__ void __launch_bounds__(kBinBlock) k_raybin_scatter(DeviceScene S, PathState st, int depth) {
    constexpr int kChunk = kBinBlock * kBinItems;
    const QueueView rays = LoadQueue(st, depth, kCntRay);
    if ((int)(blockIdx.x * kChunk) >= rays.total) return;
    __shared__ int h[kRayBins];
    int *offs = st.rayBins + kRayBins;
    const size_t NR = st.NR;
    for (int c0 = blockIdx.x * kChunk; c0 < rays.total; c0 += gridDim.x * kChunk) {
        for (int i = threadIdx.x; i < kRayBins; i += blockDim.x) h[i] = 0;
        __syncthreads();
        int key[kBinItems], rank[kBinItems], qi[kBinItems];
        V3 o[kBinItems], d[kBinItems];
#pragma unroll
        for (int k = 0; k < kBinItems; ++k) {
            const int j = c0 + k * kBinBlock + threadIdx.x;
            key[k] = -1;
            if (j < rays.total) {
                qi[k] = QueueSlot(rays, j);
                RayAt(st, depth, qi[k], &o[k], &d[k]);
                key[k] = RayBinKey(S, o[k], d[k]);
                rank[k] = atomicAdd(&h[key[k]], 1);
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < kRayBins; i += blockDim.x) {
            const int n = h[i];
            if (n) h[i] = atomicAdd(&offs[i], n);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kBinItems; ++k) {
            if (key[k] < 0) continue;
            const int pos = h[key[k]] + rank[k];
            st.raySort[pos] = make_float4(o[k].x, o[k].y, o[k].z, __int_as_float(qi[k]));
            st.raySort[NR + pos] = make_float4(d[k].x, d[k].y, d[k].z, 0.f);
        }
        __syncthreads();
    }
}
// EnqueueWorkAfterIntersection / Miss for a sorted depth, in record order (k_closest's queues)
template <int NMatQ_>
__global__ void __launch_bounds__(kBlock) k_classify(DeviceScene S, PathState st, int depth) {
    constexpr bool kMix = NMatQ_ == kClosestMix;
    constexpr int NMatQ = kMix ? kNumMatTypes : NMatQ_;
    const QueueView rays = LoadQueue(st, depth, kCntRay);
    if ((int)(blockIdx.x * blockDim.x) >= rays.total) return;
    const int shard = ProducerShard();
    const int *hitPrim = st.hitPrim[depth & 1];
    const bool shade = depth < S.maxDepth;
    constexpr int kQ = 2 + NMatQ, kCap = 128;
    __shared__ int qBuf[(kBlock / 64) * kQ * kCap];
    int *qCnt[kQ] = {&st.counters[CounterIndex(depth, kCntEscaped, shard)],
                     &st.counters[CounterIndex(depth, kCntEmissive, shard)]};
    int *qArr[kQ] = {st.escQ + shard * st.capS, st.emitQ + shard * st.capS};
#pragma unroll
    for (int t = 0; t < NMatQ; ++t) {
        qCnt[2 + t] = &st.counters[CounterIndex(depth, MatCounter(t), shard)];
        qArr[2 + t] = st.matQ[t] + shard * st.capS;
    }
    WaveQueues<kQ, kCap> queues(qBuf, qCnt, qArr, st.capS);
    for (int base = blockIdx.x * blockDim.x; base < rays.total; base += gridDim.x * blockDim.x) {
        const int j = base + threadIdx.x;
        const bool active = j < rays.total;
        const int qi = active ? QueueSlot(rays, j) : 0;
        const int prim = active ? hitPrim[qi] : -1;
        bool pred[kQ] = {S.nInfinite > 0 && active && prim < 0,
                         S.nAreaLights > 0 && active && prim >= 0 && S.primLight[prim] >= 0};
        if constexpr (NMatQ == 1) {
            pred[2] = shade && active && prim >= 0;
        } else {
            int type = -1;
            if (shade && active && prim >= 0) type = S.matType[kMix ? st.hitMat[depth & 1][qi] : S.primMaterial[prim]];
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
    if ((int)(blockIdx.x * blockDim.x) >= esc.total) return;  // no work (uniform per block)
    int nLe = 0, leLight = -1;
    for (int li = 0; li < S.nInfinite; ++li)
        if (S.infDistant[li] < 0) ++nLe, leLight = li;
    if (nLe == 1 && S.nEnv == 0) {
        // One light with Le (the usual sky): its scaled spectrum and the sensor's three matching
        // curves are staged in LDS, so each wavelength is one LDS gather instead of four global
        // ones.  Same products in the same order as the general loop below, and rgb = 0 + x = x.
        __shared__ float4 tab[kDenseN];
        const float *dense = S.dense + S.infSpectrum[leLight] * kDenseN;
        const float scale = S.infScale[leLight];
        for (int i = threadIdx.x; i < kDenseN; i += blockDim.x)
            tab[i] = make_float4(S.sensor[i], S.sensor[kDenseN + i], S.sensor[2 * kDenseN + i], scale * dense[i]);
        __syncthreads();
        for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < esc.total; qi += gridDim.x * blockDim.x) {
            const PathRecords &rec = st.rec[depth & 1];
            const int ri = st.escQ[QueueSlot(esc, qi)];
            const int slot = depth > 0 ? rec.pixel[ri] : ri;
            const int fl = depth > 0 ? rec.flags[ri] : 0;
            const float rl = depth > 0 ? rec.rl[ri] : 1.f;
            const float denom = (depth == 0 || (fl & 1)) ? Avg31(1.f) : Avg31(1.f + rl * 0.f);
            const float invDenom = 1 / denom;
            float sx = 0, sy = 0, sz = 0, lam = rec.lambda0[ri];
            bool nz = false;
            for (int i = 0; i < kNSpectrumSamples; ++i) {
                if (i > 0) {
                    lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
                    if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
                }
                const int off = DenseOffset(lam);
                const float4 t = off < 0 ? make_float4(0.f, 0.f, 0.f, scale * 0.f) : tab[off];
                nz |= t.w != 0;
                const float v = ((depth > 0 ? rec.beta[(size_t)i * NR + ri] : 1.f) * t.w * invDenom) * kInvWavelengthPDF;
                sx = i == 0 ? t.x * v : sx + t.x * v;
                sy = i == 0 ? t.y * v : sy + t.y * v;
                sz = i == 0 ? t.z * v : sz + t.z * v;
            }
            if (nz) {
                st.L[slot] += S.imagingRatio * (sx / kNSpectrumSamples);
                st.L[N + slot] += S.imagingRatio * (sy / kNSpectrumSamples);
                st.L[2 * N + slot] += S.imagingRatio * (sz / kNSpectrumSamples);
            }
        }
        return;
    }
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
            if (S.infDistant[li] >= 0) continue;  // a DistantLight is no Infinite-type light (no Le)
            const float *dense = S.dense + S.infSpectrum[li] * kDenseN;
            float scale = S.infScale[li];
            // ImageInfiniteLight: Le at the ray direction's pixel; past a non-specular bounce the
            // MIS denominator takes r_l * PMF * PDF_Li(allowIncompletePDF) (integrator.cpp:515-523)
            const bool env = S.nEnv > 0 && S.infImage[li] >= 0;
            EnvCoef ec{};
            float lInvDenom = invDenom;
            if (env) {
                const DeviceEnvLight &E = S.env[S.infImage[li]];
                const V3 d(rec.ray[3 * NR + ri], rec.ray[4 * NR + ri], rec.ray[5 * NR + ri]);
                ec = EnvLeCoef(E, d);
                if (!(depth == 0 || (fl & 1))) {
                    const float pmf = LightPMF(S, V3(0, 0, 0), V3(0, 0, 0), S.nAreaLights + S.nPointSpot + li);
                    lInvDenom = 1 / Avg31(1.f + rl * pmf * EnvPDFLi(E, d));
                }
            }
            float sx = 0, sy = 0, sz = 0, lam = rec.lambda0[ri];
            bool nz = false;
            for (int i = 0; i < kNSpectrumSamples; ++i) {
                if (i > 0) {
                    lam = lam + (kLambdaMax - kLambdaMin) / kNSpectrumSamples;
                    if (lam > kLambdaMax) lam = kLambdaMin + (lam - kLambdaMax);
                }
                int off = DenseOffset(lam);
                const float dv = off < 0 ? 0.f : dense[off];
                float Le = env ? EnvLe(ec, scale, dv, lam) : scale * dv;
                nz |= Le != 0;
                float v = ((depth > 0 ? rec.beta[(size_t)i * NR + ri] : 1.f) * Le * lInvDenom) * kInvWavelengthPDF;
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

// HandleEmissiveIntersection (integrator.cpp:539-573) over the hit-area-light queue.  The MIS
// context (pbrt's prevIntrCtx: p, n, ns, pError of the previous surface) is rebuilt from the
// previous bounce's hit record with the same TriangleSurface arithmetic that produced it.
// Ext: the scene has analytic shapes (their surfaces and solid-angle pdfs are compiled in)
template <bool Ext>
__global__ void __launch_bounds__(kBlock) k_emissive(DeviceScene S, PathState st, int depth) {
    const int N = st.NR, NL = st.N;  // record stride, pixel-sample stride (L)
    const QueueView emit = LoadQueue(st, depth, kCntEmissive);
    const int count = emit.total;
    if ((int)(blockIdx.x * blockDim.x) >= count) return;  // no work
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
        TriSurface surf = SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
        (void)flip;
        V3 wo = Normalize(-rd);
        const DeviceAreaLight Ld = S.lights[light];
        if (!(Ld.twoSided || DotN(surf.n, wo) >= 0)) continue;
        if (SpreadCut(Ld.v1.w, surf.n, wo)) continue;  // outside the emitter's spread: L = 0
        float denom;
        if (!mis) {
            denom = Avg31(1.f);
        } else {
            V3 q0, q1, q2;
            PrimVerts(S, pp, &q0, &q1, &q2);
            // prevIntrCtx = LightSampleContext(pi, n, ns) of the previous surface
            TriSurface prev = SurfaceAt<Ext>(S, pp, q0, q1, q2, pb0, pb1, pb2);
            // prevIntrCtx holds the previous vertex's bump-mapped shading normal
            if (S.hasBump) BumpedShading(S, st, depth - 1, HitMaterial(S, st, depth - 1, pi, pp), pi, &prev);
            float lightChoicePDF = LightPMF(S, prev.p, prev.ns, light);
            float lightPDF;
            if (Ext && prim >= S.nTris) {
                lightPDF = lightChoicePDF * ShapeLightPDF(S.shapes, S.shapeN, prim - S.nTris, prev.p, prev.pErr, prev.n, prev.ns, -wo);
            } else {
                TriShading lsh;
                const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
                V3 l0(Ld.v0.x, Ld.v0.y, Ld.v0.z), l1(Ld.v1.x, Ld.v1.y, Ld.v1.z), l2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
                lightPDF = lightChoicePDF * TrianglePDF(l0, l1, l2, Ld.flip, lhas ? &lsh : nullptr, prev.p, prev.pErr,
                                                       prev.n, prev.ns, -wo);
            }
            denom = Avg31(1.f + rl * lightPDF);
        }
        const float *dense = S.dense + Ld.spectrum * kDenseN;
        const float invDenom = 1 / denom;
        // an image emitter: L at the hit's uv (DiffuseAreaLight::L, lights.h:460-467)
        const bool img = Ext && S.nImageAreaLights > 0 && S.lightImgOff[light] >= 0;
        EnvCoef ec{};
        if (img) ec = AreaImageCoef(S, S.lightImgOff[light], surf.uv[0], surf.uv[1]);
        SensorAcc acc;
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNSpectrumSamples; ++i, it.Next()) {
            int off = DenseOffset(it.lam);
            const float dv = off < 0 ? 0.f : dense[off];
            float Le = Ld.scale * dv;
            if (img) Le = EnvLe(ec, Ld.scale, dv, it.lam);
            acc.Add(S, off, beta[i] * Le * invDenom, i == 0);
        }
        st.L[slot] += S.imagingRatio * (acc.sx / kNSpectrumSamples);
        st.L[NL + slot] += S.imagingRatio * (acc.sy / kNSpectrumSamples);
        st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNSpectrumSamples);
    }
}

// k_shade_diffuse's one pass over the 31 wavelengths.  Per wavelength and in the reference's
// operation order: bf = beta * f (f = R / pi); the light sample's contribution
// bf * |cos| * Le / denom to sensor RGB (lanes without a light sample carry scale = 0); the new
// beta = bf * |cos| / pdf (lanes that do not scatter carry |cos| = pdf = 1) into bf's LDS slot,
// with max(beta * etaScale / avg(r_u)) for RR.  neeNz: Le != 0 somewhere; betaNz: new beta != 0
// somewhere.
// DivD2: the light's radiance is divided by d2 per wavelength (point and spot lights; d2 = 1,
// an exact no-op, for the other lanes).
// RF: the diffuse reflectance R(lambda), clamped to [0, 1] (DiffuseMaterial::GetBxDF)
// Env: the light sample may be an ImageInfiniteLight's (envLe), whose radiance is the pixel's
// RGBIlluminantSpectrum at the wavelength (EnvLe) rather than scale * dense
template <bool DivD2, bool Env, typename FD, typename RF>
__device__ inline void ShadeSpectralPass(int depth, const FD *dense, const SensorF4 *sensor4, float *bf, const RF &rf,
                                         float lambda0, float scale, float d2, float rd2, bool d2Ok,
                                         float absdotL, float invDenom, float absdotB, float pdf, float rpdf,
                                         bool pdfOk, float etaScale, SensorAcc *acc, bool *neeNz, bool *betaNz,
                                         float *mx, bool envLe = false, EnvCoef ec = EnvCoef{}, float k = 1) {
    const float avgRu = Avg31(1.f);
    bool nzL = false, nzB = false;
    float m = -kInfinity;
#pragma unroll 1
    for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
        const float R = rf(it.lam, it.i);
        const float bfi = (depth > 0 ? bf[it.i * kBlock] : 1.f) * (R * kInvPi);
        const int off = DenseOffset(it.lam);
        const float dv = off < 0 ? 0.f : float(dense[off]);
        float Le = scale * dv;
        if constexpr (Env) {
            if (envLe) Le = EnvLe(ec, scale, dv, it.lam);
            Le = Le * k;  // GoniometricLight's image value (1 otherwise)
        }
        if constexpr (DivD2) Le = DivByRcp(Le, d2, rd2, d2Ok);
        nzL |= Le != 0;
        acc->Add(sensor4, off, bfi * absdotL * Le * invDenom, it.i == 0);
        const float nbv = DivByRcp(bfi * absdotB, pdf, rpdf, pdfOk);
        bf[it.i * kBlock] = nbv;
        m = fmaxf(m, nbv * etaScale / avgRu);
        nzB |= nbv != 0;
    }
    *neeNz = nzL;
    *betaNz = nzB;
    *mx = m;
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
    const SensorF4 *sensorL;
    const LdsU16 *permL;
    uint32_t permOff[7];
    DeviceScene SL;  // the light sampler reads its nodes from LDS
    const DeviceAreaLight *lightsL;
    const float4 *matsL;
    const int *matConstL;
    LdsF *plLamL, *plValL;  // conductor knots when lay.plInLds
};
// WithPl: also the conductor knots (lay.plInLds), after this depth's permutation tables
template <bool WithPl = false>
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
    float *plLds = reinterpret_cast<float *>(ldsBase + (depth < kShadeLdsDepths ? lay.totalByDepth[depth] : lay.total));
    if (WithPl && lay.plInLds) {
        DmaCopy<4>(S.plLambda, plLds, lay.plCount);
        DmaCopy<4>(S.plValue, plLds + lay.plCount, lay.plCount);
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
    T->plLamL = (LdsF *)plLds;
    T->plValL = (LdsF *)(plLds + lay.plCount);
}

// GenerateRaySamples (samples.cpp:29-66): dims d0 + {0..6} = direct.uc, direct.u (2),
// indirect.uc, indirect.u (2), rr; Halton digit permutations come from the LDS tables
struct RaySamples {
    float dUc, dU0, dU1, iUc, iU0, iU1, rr;
};
// sidx: the Halton index stored by the camera kernel (kNoSampleIndex: recompute it from the
// pixel sample of slot)
// Lean: the launch guarantees the Halton sampler and every index below 2^24 (host-checked), so
// only the LDS digit loop is compiled in.
template <bool IndirectUc, bool Lean = false>
__device__ __forceinline__ RaySamples GenerateRaySamples(const DeviceScene &S, const ShadeTables &T, const PathState &st,
                                                         int slot, uint32_t sidx, int d0) {
    RaySamples r;
    r.iUc = 0;
    if (Lean || (S.samplerType == 0 && sidx < (1u << 24))) {
        // the common case: the depth's seven dimensions digit-major from the LDS tables, with
        // the digit count every index of the render fits in (host-chosen, HaltonDimDesc::nz)
        const LdsU16 *perm[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) perm[k] = T.permL + T.permOff[k];
        float u[7];
        HaltonDepthSamples<!IndirectUc>(S.haltonDim + d0, sidx, perm, u);
        r.dUc = u[0];
        r.dU0 = u[1];
        r.dU1 = u[2];
        if (IndirectUc) r.iUc = u[3];
        r.iU0 = u[4];
        r.iU1 = u[5];
        r.rr = u[6];
        return r;
    }
    if constexpr (Lean) return r;  // not reached
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    if (S.samplerType >= kSamplerIndependent) {
        // the other samplers are stateful: every draw in pbrt's order, indirect.uc included
        GenericSampler g;
        g.Start(S.samp, px, py, sampleIndex, d0);
        r.dUc = g.Get1D(S.samp);
        g.Get2D(S.samp, &r.dU0, &r.dU1);
        const float iuc = g.Get1D(S.samp);
        if (IndirectUc) r.iUc = iuc;
        g.Get2D(S.samp, &r.iU0, &r.iU1);
        r.rr = g.Get1D(S.samp);
    } else if (S.samplerType == 1) {
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        r.dUc = ZSobolGet1D(S.zs, morton, d0, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 1, S.zsPerms, S.sobolM1, &r.dU0, &r.dU1);
        if (IndirectUc) r.iUc = ZSobolGet1D(S.zs, morton, d0 + 3, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 4, S.zsPerms, S.sobolM1, &r.iU0, &r.iU1);
        r.rr = ZSobolGet1D(S.zs, morton, d0 + 6, S.zsPerms, S.sobolM1);
    } else {
        const Halton h = StartPixelSample(S, px, py, sampleIndex, d0);
        auto dim = [&](int k) -> float { return HaltonSampleDimension(S.haltonDim[d0 + k], h.index, S.perm); };
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

// Lean (host-chosen per launch, pbrt-identical results either way): Halton indices below 2^24,
// lights, light BVH and dense spectra staged in LDS, no mesh with shading normals or uv -- the
// common case, compiled without the other paths so the kernel's hot code stays small.
// Tex (host-chosen: some material is textured): reflectance textures are evaluated per hit
// (surfscatter.cpp:74-137: uv derivatives, then GetBxDF's texture evaluation).
// Ext (host-chosen: the scene has analytic shapes or image infinite lights): their surface,
// light-sampling and radiance paths are compiled in.
template <bool Lean, bool Tex = false, bool Ext = false>
__global__ void __launch_bounds__(kBlock, PBRT_SHADE_WAVES) k_shade_diffuse(DeviceScene S, PathState st, int depth) {
    const QueueView mats = LoadQueue(st, depth, kCntMat);
    if ((int)(blockIdx.x * blockDim.x) >= mats.total) return;  // no work
    extern __shared__ float4 dynLds[];
    ShadeTables T;
    StageShadeTables(S, depth, reinterpret_cast<char *>(dynLds), &T);
    const ShadeLdsLayout &lay = T.lay;
    float *bfLds = T.bfLds;
    float *denseLds = T.denseLds;
    const SensorF4 *sensorL = T.sensorL;
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
        float nRl = 0, nEta = 1, rrOmq = 1;
        bool rrDiv = false;
        int slot = 0;
        float lambda0 = 0;
        uint32_t sidx = kNoSampleIndex;
        SEC_BEGIN();
        if (active) {
            lambda0 = rec.lambda0[ri];
            slot = depth > 0 ? rec.pixel[ri] : ri;
            const float *betaP = rec.beta + ri;
            int prim = hitPrim[ri];
            float b0 = hitB[ri], b1 = hitB[N + ri], b2 = hitB[2 * N + ri];
            V3 rd(rec.ray[3 * N + ri], rec.ray[4 * N + ri], rec.ray[5 * N + ri]);
            sidx = rec.sidx[ri];
            V3 p0, p1, p2;
            PrimVerts(S, prim, &p0, &p1, &p2);
            const int mat = Lean ? S.primMaterial[prim] : HitMaterial(S, st, depth, ri, prim);
            TriSurface surf = Lean ? TriangleSurface(p0, p1, p2, b0, b1, b2, S.primFlip[prim], nullptr)
                                   : SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
            if constexpr (Tex) {
                if (S.hasBump) BumpedShading(S, st, depth, mat, ri, &surf);
            }
            float4 mc = matsL[mat];
            int mflags = matConstL[mat];  // bit 0: constant R, bit 1: R != 0 at every wavelength
            bool constant = mflags & 1;
            // a textured reflectance (k_texture's result for this record): sigmoid coefficients,
            // or per-wavelength values for a general expression (texR)
            bool texR = false;
            if constexpr (Tex) {
                if (S.matTex[mat].x >= 0) {
                    mflags = 0;
                    constant = false;
                    if (st.texCoef[3 * (size_t)N + ri] != 0) texR = true;
                    else mc = make_float4(st.texCoef[ri], st.texCoef[(size_t)N + ri], st.texCoef[2 * (size_t)N + ri], 0.f);
                }
            }
            auto rfun = [&](float lam, int i) -> float {
                if constexpr (Tex) {
                    if (texR) return Clampf(st.texR[(size_t)i * N + ri], 0, 1);
                }
                return Reflectance(mc, constant, lam);
            };
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
                const RaySamples rs = GenerateRaySamples<false, Lean>(S, T, st, slot, sidx, d0);
                const float dUc = rs.dUc, dU0 = rs.dU0, dU1 = rs.dU1, iU0 = rs.iU0, iU1 = rs.iU1, rr = rs.rr;
                SEC_MARK(st, 1);
                // ---- DiffuseMaterial::GetBxDF (materials.h:466-471): R = clamp(reflectance, 0, 1),
                // f = R / pi (DiffuseBxDF, bxdfs.h:30-82).  The BSDF samples and is sampled for
                // light only if R != 0 at some wavelength (its flags): known without a pass over
                // the wavelengths for a constant R, and for an RGB R whose sigmoid polynomial the
                // host bounded away from zero on every sampled wavelength (flag bit 1).
                bool Rnz;
                if (constant) Rnz = Reflectance(mc, true, 0.f) != 0;
                else if (mflags & 2) Rnz = true;
                else {
                    Rnz = false;
                    for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) Rnz |= rfun(it.lam, it.i) != 0;
                }
                Frame frame = Frame::FromXZ(Normalize(surf.dpdus), ns);
                V3 woL = frame.ToLocal(wo);
                V3 pi = surf.p, pe = surf.pErr;
                SEC_MARK(st, 2);
                // ---- light sample geometry (surfscatter.cpp:254-326)
                bool nee = false, envLe = false;
                EnvCoef envC{};
                int spec = 0;
                float scale = 0, absdotL = 0, invDenom = 0, d2 = 1, lk = 1;
                if (Rnz) {
                    V3 cp = OffsetRayOrigin(pi, pe, n, wo);  // reflective, not transmissive
                    int li;
                    float lpmf;
                    const bool sampled =
                        (Lean || lay.lightsInLds)
                            ? SampleLightT<LdsLightNode, true>(SL, (const LdsLightNode *)SL.lightNodes, cp, ns, dUc,
                                                               &li, &lpmf)
                            : SampleLightT<DeviceLightNode, true>(SL, S.lightNodes, cp, ns, dUc, &li, &lpmf);
                    LiSample ls;
                    if (sampled && SampleLiSurface<Lean, true, Ext>(S, lightsL, li, cp, n, ns, dU0, dU1, &ls)) {
                        const V3 wi = ls.wi;
                        const V3 wiL = frame.ToLocal(wi);
                        if (woL.z != 0 && woL.z * wiL.z > 0) {  // DiffuseBxDF::f != 0
                            if constexpr (!Lean && Ext) {
                                envLe = ls.envLe;
                                envC = ls.env;
                                lk = ls.k;
                            }
                            spec = ls.spectrum;
                            scale = ls.scale;
                            d2 = ls.d2;
                            absdotL = AbsDotN(ns, wi);
                            float lightPDF = ls.pdf * lpmf;
                            float bsdfPDF = ls.delta ? 0.f : CosineHemispherePDF(fabsf(wiL.z));
                            float denom = Avg31(bsdfPDF + lightPDF);
                            invDenom = 1 / denom;
                            nee = true;
                            // SpawnRayTo(pi, n, time, pLight.pi, pLight.n) (ray.h:106-111), formed
                            // now so the light point is not held through the wavelength pass
                            sOrg = OffsetRayOrigin(pi, pe, n, ls.lp - pi);
                            V3 pt = OffsetRayOrigin(ls.lp, ls.lpe, ls.ln, sOrg - ls.lp);
                            sDir = pt - sOrg;
                        }
                    }
                }
                SEC_MARK(st, 3);
                // ---- BSDF::Sample_f<DiffuseBxDF> geometry (surfscatter.cpp:170-190)
                bool scat = false;
                V3 wiB;
                float pdf = 1, absdotB = 1, etaScale = 1;  // lanes that do not scatter: harmless values
                if (woL.z != 0 && Rnz) {
                    V3 wiL = SampleCosineHemisphere(iU0, iU1);
                    if (woL.z < 0) wiL.z *= -1;
                    const float p = CosineHemispherePDF(fabsf(wiL.z));
                    if (p != 0 && wiL.z != 0) {
                        wiB = frame.FromLocal(wiL);
                        nOrg = OffsetRayOrigin(pi, pe, n, wiB);
                        nDir = wiB;
                        absdotB = AbsDotN(ns, wiB);
                        etaScale = depth > 0 ? rec.etaScale[ri] : 1.f;
                        pdf = p;
                        scat = true;
                    }
                }
                SEC_MARK(st, 4);
                // ---- one pass over the wavelengths: bf_i = beta_i f_i, the light sample's sensor
                // RGB (beta f |cos| Le / denom, surfscatter.cpp:288-308, film.h:95-100) and the
                // new beta = bf |cos| / pdf (surfscatter.cpp:190) with its RR maximum
                bool neeNz = false, betaNz = false;
                float mx = -kInfinity;
                SensorAcc acc;
                const float rpdf = 1 / pdf;  // one IEEE division; the elements by DivByRcp
                if (nee || scat) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the beta LDS-DMA has landed
                    const bool pdfOk = DivFastOk(pdf);
                    float *bf = bfLds + threadIdx.x;
                    const float rd2 = 1 / d2;
                    const bool d2Ok = DivFastOk(d2);
                    if (Lean || (lay.denseInLds && S.nPointSpot == 0 &&
                                 (!Ext || (S.nEnv == 0 && !S.hasSpread && S.nImageAreaLights == 0))))
                        ShadeSpectralPass<false, false>(depth, (const LdsF *)denseLds + spec * kDenseN, sensorL, bf,
                                                        rfun, lambda0, scale, d2, rd2, d2Ok, absdotL, invDenom,
                                                        absdotB, pdf, rpdf, pdfOk, etaScale, &acc, &neeNz, &betaNz,
                                                        &mx);
                    else if (lay.denseInLds)
                        ShadeSpectralPass<true, !Lean && Ext>(depth, (const LdsF *)denseLds + spec * kDenseN, sensorL, bf,
                                                       rfun, lambda0, scale, d2, rd2, d2Ok, absdotL, invDenom,
                                                       absdotB, pdf, rpdf, pdfOk, etaScale, &acc, &neeNz, &betaNz,
                                                       &mx, envLe, envC, lk);
                    else
                        ShadeSpectralPass<true, !Lean && Ext>(depth, S.dense + spec * kDenseN, sensorL, bf, rfun, lambda0,
                                                       scale, d2, rd2, d2Ok, absdotL, invDenom, absdotB, pdf, rpdf,
                                                       pdfOk, etaScale, &acc, &neeNz, &betaNz, &mx, envLe, envC, lk);
                }
                SEC_MARK(st, 5);
                if (nee && neeNz) {
                    sL = V3(S.imagingRatio * (acc.sx / kNSpectrumSamples), S.imagingRatio * (acc.sy / kNSpectrumSamples),
                            S.imagingRatio * (acc.sz / kNSpectrumSamples));
                    pushShadow = true;
                }
                // ---- Russian roulette (surfscatter.cpp:212-222) and the indirect ray
                if (scat) {
                    bool kill = false;
                    float q = 0;
                    if (mx < 1 && depth >= 1) {
                        q = fmaxf(0.f, 1 - mx);
                        kill = rr < q;
                    }
                    // beta / (1 - q) is nonzero exactly where beta is (1 - q in (0, 1] for a
                    // surviving path), so the push decision needs no division; the division is
                    // applied as beta is written out
                    if (!kill && betaNz) {
                        if (mx < 1 && depth >= 1) {
                            rrOmq = 1 - q;
                            rrDiv = true;
                        }
                        nRl = rpdf;  // 1 / pdf
                        nEta = etaScale;
                        pushRay = true;
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
            const int j = ShardSlot(shardBase, pos[1], st.capS, st.NR);
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
            const int j = ShardSlot(shardBase, pos[0], st.capS, st.NR);
            const float *bf = bfLds + threadIdx.x;
            if (rrDiv) {  // beta /= 1 - q (surfscatter.cpp:221)
                const float rq = 1 / rrOmq;
                const bool qOk = DivFastOk(rrOmq);
#pragma unroll 8
                for (int i = 0; i < kNSpectrumSamples; ++i)
                    out.beta[(size_t)i * N + j] = DivByRcp(bf[i * kBlock], rrOmq, rq, qOk);
            } else {
#pragma unroll 8
                for (int i = 0; i < kNSpectrumSamples; ++i) out.beta[(size_t)i * N + j] = bf[i * kBlock];
            }
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
            out.sidx[j] = sidx;
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
// Smooth (dielectric only, host-checked: every dielectric EffectivelySmooth, no regularize):
// the light-sampling code of rough surfaces is compiled out.
// Tex (host-chosen: some material is textured): textured roughness (both types) and conductor
// reflectance are evaluated per hit (materials.h:182-204, :491-511).
// Ext: as k_shade_diffuse's.
template <int MT, bool Smooth = false, bool Tex = false, bool Ext = false>
__global__ void __launch_bounds__(kBlock, PBRT_SHADE_WAVES) k_shade_microfacet(DeviceScene S, PathState st, int depth) {
    const QueueView mats = LoadQueue(st, depth, MatCounter(MT));
    if ((int)(blockIdx.x * blockDim.x) >= mats.total) return;  // no work
    extern __shared__ float4 dynLds[];
    ShadeTables T;
    StageShadeTables<true>(S, depth, reinterpret_cast<char *>(dynLds), &T);
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
        uint32_t sidx = kNoSampleIndex;
        float *bf = T.bfLds + threadIdx.x;  // beta_i at bf[i * kBlock]
        if (active) {
            lambda0 = rec.lambda0[ri];
            slot = depth > 0 ? rec.pixel[ri] : ri;
            const int inFlags = depth > 0 ? rec.flags[ri] : 0;
            const int prim = hitPrim[ri];
            const float b0 = hitB[ri], b1 = hitB[N + ri], b2 = hitB[2 * N + ri];
            const V3 rd(rec.ray[3 * N + ri], rec.ray[4 * N + ri], rec.ray[5 * N + ri]);
            sidx = rec.sidx[ri];
#pragma unroll 8
            for (int i = 0; i < kNSpectrumSamples; ++i) bf[i * kBlock] = depth > 0 ? rec.beta[(size_t)i * N + ri] : 1.f;
            V3 p0, p1, p2;
            PrimVerts(S, prim, &p0, &p1, &p2);
            const int mat = HitMaterial(S, st, depth, ri, prim);
            TriSurface surf = SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
            if constexpr (Tex) {
                if (S.hasBump) BumpedShading(S, st, depth, mat, ri, &surf);
            }
            const V3 wo = Normalize(-rd);
            const V3 n = surf.n, ns = surf.ns;
            const RaySamples rs = GenerateRaySamples<MT == kMatDielectricT>(S, T, st, slot, sidx, d0);
            // ---- Material::GetBxDF (materials.h:182-204 dielectric, :491-511 conductor)
            const float4 mp = S.matParams[mat];
            TrowbridgeReitz tr{mp.x, mp.y};
            float4 mc = T.matsL[mat];
            bool texR = false;
            if constexpr (Tex) {
                const int4 mt = S.matTex[mat];
                // k_texture's results for this record: the roughness alphas (remapped and clamped)
                // and a conductor's reflectance
                if (mt.y >= 0) tr = TrowbridgeReitz{st.texCoef[4 * (size_t)N + ri], st.texCoef[5 * (size_t)N + ri]};
                if (MT == kMatConductorT && mt.x >= 0) {
                    if (st.texCoef[3 * (size_t)N + ri] != 0) texR = true;
                    else mc = make_float4(st.texCoef[ri], st.texCoef[(size_t)N + ri], st.texCoef[2 * (size_t)N + ri], 0.f);
                }
            }
            if (S.regularize && (inFlags & 2)) tr.Regularize();  // surfscatter.cpp:127-128
            float eta = mp.z;
            if (eta == 0) eta = 1;
            // conductor eta_i / k_i: piecewise-linear spectra, or from the albedo "reflectance"
            const int etaSpec = MT == kMatConductorT ? S.matSpectra[2 * mat] : -1;
            const int kSpec = MT == kMatConductorT ? S.matSpectra[2 * mat + 1] : -1;
            auto etaK = [&](float lam, int li, float *e, float *k) {
                if (etaSpec >= 0) {
                    const int a = S.plOffsets[etaSpec], na = S.plOffsets[etaSpec + 1] - a;
                    const int b = S.plOffsets[kSpec], nb = S.plOffsets[kSpec + 1] - b;
                    // small sets (LDS-resident knots) search in LDS; large ones (named metals,
                    // through L1/L2) start from the per-nanometre segment table
                    if (lay.plInLds) {
                        *e = PiecewiseLinearEval(T.plLamL + a, T.plValL + a, na, lam);
                        *k = PiecewiseLinearEval(T.plLamL + b, T.plValL + b, nb, lam);
                    } else {
                        const uint16_t *ia = S.plIndex + (size_t)etaSpec * kPlIndexN;
                        const uint16_t *ib = S.plIndex + (size_t)kSpec * kPlIndexN;
                        *e = PiecewiseLinearEvalIdx(S.plLambda + a, S.plValue + a, na, ia, lam);
                        *k = PiecewiseLinearEvalIdx(S.plLambda + b, S.plValue + b, nb, ib, lam);
                    }
                } else {
                    float rv = SigmoidPolynomial(mc.x, mc.y, mc.z, lam);
                    if constexpr (Tex) {
                        if (texR) rv = st.texR[(size_t)li * N + ri];
                    }
                    float r = Clampf(rv, 0, .9999f);
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
            // ---- light sample geometry (surfscatter.cpp:252-326) and BSDF::Sample_f geometry
            // (surfscatter.cpp:183-190), then ONE pass over the wavelengths for both: each eta_i,
            // k_i (conductor) is looked up once and feeds the light sample's f_i and the
            // sampled direction's f_i, with the light term formed from beta_i before the update
            // overwrites it -- the same products per wavelength as two separate passes.
            bool haveL = false, haveB = false;
            ConductorTerms ctL{}, ctB{};
            float fdL = 0, absdotL = 0, invDenomL = 0;
            LiSample ls;
            if (!Smooth && !smooth) {
                V3 cp = pi, cpErr = pe;  // LightSampleContext: the offset point is exact
                if (reflective && !transmissive) cp = OffsetRayOrigin(pi, pe, n, wo), cpErr = V3(0, 0, 0);
                else if (transmissive && reflective) cp = OffsetRayOrigin(pi, pe, n, -wo), cpErr = V3(0, 0, 0);
                int li;
                float lpmf;
                if (SampleLightT<DeviceLightNode, true>(T.SL, T.SL.lightNodes, cp, ns, rs.dUc, &li, &lpmf) &&
                    SampleLiSurface<false, true, Ext>(S, T.lightsL, li, cp, n, ns, rs.dU0, rs.dU1, &ls, cpErr)) {
                    const V3 wiL = frame.ToLocal(ls.wi);
                    if (woL.z != 0) {
                        // BSDF::f / BSDF::PDF (bsdf.h:60-135)
                        float bsdfPDF = 0;
                        bool fAny;
                        if constexpr (MT == kMatDielectricT) {
                            fdL = DielectricEval(eta, tr, woL, wiL, &bsdfPDF);
                            fAny = fdL != 0;
                        } else {
                            ctL = ConductorEval(tr, woL, wiL);
                            bsdfPDF = ctL.pdf;
                            fAny = ctL.ok;  // f_i may still vanish; a zero Ld adds nothing
                        }
                        if (fAny) {
                            absdotL = AbsDotN(ns, ls.wi);
                            const float lightPDF = ls.pdf * lpmf;
                            if (ls.delta) bsdfPDF = 0;  // IsDeltaLight: no BSDF MIS weight
                            invDenomL = 1 / Avg31(bsdfPDF + lightPDF);
                            haveL = true;
                        }
                    }
                }
            }
            V3 wi;
            float pdf = 1, fdB = 0, absdotB = 0, etaScale = 1;
            bool specular = false;
            if (woL.z != 0) {
                bool ok, transmission;
                V3 wiL;
                float etap = 1;
                if constexpr (MT == kMatDielectricT) {
                    const BxSample bs = DielectricSample(eta, tr, woL, rs.iUc, rs.iU0, rs.iU1);
                    ok = bs.ok && bs.f != 0;
                    wiL = bs.wi;
                    pdf = bs.pdf;
                    fdB = bs.f;
                    etap = bs.etap;
                    specular = bs.flags & kBxSpecular;
                    transmission = bs.flags & kBxTransmission;
                } else {
                    ctB = ConductorSample(tr, woL, rs.iU0, rs.iU1);
                    ok = ctB.ok;
                    wiL = ctB.wi;
                    pdf = ctB.pdf;
                    specular = ctB.specular;
                    transmission = false;
                }
                if (ok && pdf != 0 && wiL.z != 0) {
                    wi = frame.FromLocal(wiL);
                    absdotB = AbsDotN(ns, wi);
                    etaScale = depth > 0 ? rec.etaScale[ri] : 1.f;
                    if (transmission) etaScale *= Sqr(etap);
                    haveB = true;
                }
            }
            if (haveL || haveB) {
                const int lspec = haveL ? ls.spectrum : 0;
                const float *dense = lay.denseInLds ? nullptr : S.dense + lspec * kDenseN;
                const LdsF *denseL = (const LdsF *)T.denseLds + lspec * kDenseN;
                const float avgRu = Avg31(1.f);
                SensorAcc acc;
                bool nzL = false, fAnyB = MT == kMatDielectricT;
                float mx = -kInfinity;
#pragma unroll 2
                for (SpectralIter it(lambda0); it.i < kNSpectrumSamples; it.Next()) {
                    float e = 1, k = 0;
                    if constexpr (MT == kMatConductorT) etaK(it.lam, it.i, &e, &k);
                    const float b = bf[it.i * kBlock];
                    if (haveL) {
                        const int off = DenseOffset(it.lam);
                        float Le = ls.Le(off < 0 ? 0.f : (lay.denseInLds ? float(denseL[off]) : dense[off]), it.lam);
                        if (S.nPointSpot > 0) Le = Le / ls.d2;  // pbrt: SampledSpectrum / DistanceSquared
                        nzL |= Le != 0;
                        float f = fdL;
                        if constexpr (MT == kMatConductorT) f = ConductorF(ctL, e, k);
                        acc.Add(T.sensorL, off, b * f * absdotL * Le * invDenomL, it.i == 0);
                    }
                    if (haveB) {
                        float f = fdB;
                        if constexpr (MT == kMatConductorT) {
                            f = ConductorF(ctB, e, k);
                            fAnyB |= f != 0;
                        }
                        const float nbv = b * f * absdotB / pdf;
                        bf[it.i * kBlock] = nbv;
                        mx = fmaxf(mx, nbv * etaScale / avgRu);
                    }
                }
                if (haveL && nzL) {
                    sOrg = OffsetRayOrigin(pi, pe, n, ls.lp - pi);
                    const V3 pt = OffsetRayOrigin(ls.lp, ls.lpe, ls.ln, sOrg - ls.lp);
                    sDir = pt - sOrg;
                    sL = V3(S.imagingRatio * (acc.sx / kNSpectrumSamples), S.imagingRatio * (acc.sy / kNSpectrumSamples),
                            S.imagingRatio * (acc.sz / kNSpectrumSamples));
                    pushShadow = true;
                }
                // ---- Russian roulette (surfscatter.cpp:212-222) and the indirect ray
                if (haveB && fAnyB) {
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
        int *const cnt[2] = {nextCounter, shadowCounter};
        const bool pred[2] = {pushRay, pushShadow};
        int pos[2];
        BlockPush<2>(cnt, pred, pos);
        if (pos[1] >= 0) {
            const int j = ShardSlot(shardBase, pos[1], st.capS, st.NR);
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
            const int j = ShardSlot(shardBase, pos[0], st.capS, st.NR);
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
            out.sidx[j] = sidx;
        }
    }
}

// The texture stage of EvaluateMaterialAndBSDF (surfscatter.cpp:74-137, materials.h GetBxDF's
// texEval calls) over one material type's queue, ahead of that type's shade launch: per textured
// hit the uv derivatives (Approximate_dp_dxy), then the reflectance (one RGB image leaf -> this
// hit's sigmoid coefficients; any other expression -> its 31 values) and the roughness alphas
// (RoughnessToAlpha when remapped, the TrowbridgeReitzDistribution clamp).  Keeping the
// texture code out of the shade kernels keeps them at their untextured register budget.
// Full = false (host-chosen per material type): every textured parameter of the type is a single
// image (or constant) leaf filtered without EWA -- the register-file interpreter and the EWA
// filter are not compiled in.
template <int MT, bool Full, bool Ext = false>
__global__ void __launch_bounds__(kBlock) k_texture(DeviceScene S, PathState st, int depth) {
    const QueueView mats = LoadQueue(st, depth, MatCounter(MT));
    if ((int)(blockIdx.x * blockDim.x) >= mats.total) return;  // no work
    // the RGB->spectrum table's z nodes (searched per lookup) and the 8-bit decode tables of up
    // to kTexLdsLuts images are read from LDS
    __shared__ float zLds[64];
    __shared__ float lutLds[kTexLdsLuts * 256];
    const int nLut = S.tex.nLuts <= kTexLdsLuts ? S.tex.nLuts : 0;
    for (int i = threadIdx.x; i < 64; i += blockDim.x) zLds[i] = S.tex.rgbZNodes[i];
    for (int i = threadIdx.x; i < nLut * 256; i += blockDim.x) lutLds[i] = S.tex.luts[i];
    __syncthreads();
    S.tex.rgbZNodes = zLds;
    if (nLut) S.tex.luts = lutLds;
    const PathRecords &rec = st.rec[depth & 1];
    const int *hitPrim = st.hitPrim[depth & 1];
    const float *hitB = st.hitB[depth & 1];
    for (int qi = blockIdx.x * blockDim.x + threadIdx.x; qi < mats.total; qi += gridDim.x * blockDim.x) {
        const int ri = st.matQ[MT][QueueSlot(mats, qi)];
        const int prim = hitPrim[ri];
        const int mat = HitMaterial(S, st, depth, ri, prim);
        HitTextures<Full, Ext>(S, st, depth, ri, prim, mat, hitB, rec.lambda0);
    }
}

template <int TM>
__global__ void __launch_bounds__(kBlock, ShadowWaves(TM)) k_shadow(DeviceScene S, PathState st, int depth) {
    const QueueView shadows = LoadQueue(st, depth, kCntShadow);
    ChunkWalk walk = XcdChunks(shadows.total, S.xcdGroups);
    if (walk.n >= walk.end) return;  // no work
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int N = st.NR, NL = st.N;
    const int count = shadows.total;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[2], (unsigned long long)count);
    for (; walk.n < walk.end; walk.n += walk.step) {
        const int qi = walk.Chunk() * blockDim.x + threadIdx.x;
        if (qi >= count) continue;
        // the shadow queue is dense per shard: entry p holds the ray, its contribution and pixel
        const int p = QueueSlot(shadows, qi);
        V3 o(st.shadowRay[p], st.shadowRay[N + p], st.shadowRay[2 * N + p]);
        V3 d(st.shadowRay[3 * N + p], st.shadowRay[4 * N + p], st.shadowRay[5 * N + p]);
        TriHit h;
        TravCount tc;
        int hit = Traverse<true, TM>(S, L, o, d, 1 - kShadowEpsilon, &h, &tc);
#ifdef PBRT_AMD_TRAV_STATS
        TravStatsAdd(st.stats, kStatsSectionBase + 16, true, tc);
#endif
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
        const float *Ls = (st.lamTerm && st.lamTerm[slot]) ? st.L0 : st.L;  // terminated: lambda_0 only
        float rr = Ls[slot], gg = Ls[N + slot], bb = Ls[2 * N + slot];
        // RGBFilm::AddSample (film.h:247-249): m = max(r, g, b) > maxComponentValue scales rgb
        const float m = std::fmax(std::fmax(rr, gg), bb);
        if (m > S.maxComponentValue) {
            const float sc = S.maxComponentValue / m;
            rr *= sc;
            gg *= sc;
            bb *= sc;
        }
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
template <int TM>
__global__ void __launch_bounds__(kBlock, TraversalWaves(TM)) k_intersect_batch(DeviceScene S, const float *rays, int n, int anyHit,
                                                              int *outPrim, float *outHit) {
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        V3 o(rays[i], rays[n + i], rays[2 * n + i]);
        V3 d(rays[3 * n + i], rays[4 * n + i], rays[5 * n + i]);
        float tMax = rays[6 * n + i];
        TriHit h{0, 0, 0, 0};
        int prim = anyHit ? Traverse<true, TM>(S, L, o, d, tMax, &h) : Traverse<false, TM>(S, L, o, d, tMax, &h);
        outPrim[i] = prim >= 0 ? S.primOrig[prim] : -1;  // the caller's triangle numbering
        outHit[i] = h.b0;
        outHit[n + i] = h.b1;
        outHit[2 * n + i] = h.b2;
        outHit[3 * n + i] = h.t;
    }
}

// ------------------------------------------------------------------ arithmetic self-check
// SigmoidPolynomial's device sqrt / division (core.h) against the plain IEEE expression, bitwise:
// each thread draws coefficient triples and wavelengths from a counter hash -- arbitrary bit
// patterns (every exponent, zeros, denormals, infinities, NaNs) and values in the tables' range.
__device__ inline uint32_t CheckHash(uint64_t v) {
    v ^= v >> 33;
    v *= 0xff51afd7ed558ccdull;
    v ^= v >> 33;
    v *= 0xc4ceb9fe1a85ec53ull;
    v ^= v >> 33;
    return (uint32_t)v;
}
__device__ inline float CheckOperand(uint64_t key, float scale) {
    const uint32_t h = CheckHash(key);
    if ((h & 7u) == 0) return __uint_as_float(CheckHash(key * 3 + 1));  // any bit pattern
    const uint32_t e = 40u + (CheckHash(key * 5 + 2) % 180u);             // biased exponents 40..219
    const float f = __uint_as_float((h & 0x80000000u) | (e << 23) | (CheckHash(key * 7 + 3) & 0x7fffffu));
    return (h & 6u) == 2u ? f : scale * ((CheckHash(key * 11 + 4) >> 8) * 0x1p-24f - .5f);
}
__device__ inline bool SameFloat(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
__global__ void k_check_rn_math(uint64_t seed, int perThread, unsigned long long *bad) {
    const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    unsigned long long ns = 0;
    for (int i = 0; i < perThread; ++i) {
        const uint64_t k = (seed + t * perThread + i) * 4;
        const float c0 = CheckOperand(k, 2e-3f), c1 = CheckOperand(k + 1, 2.f), c2 = CheckOperand(k + 2, 600.f);
        const float lam = 395.f + 310.f * ((CheckHash(k + 3) >> 8) * 0x1p-24f);
        const float a = SigmoidPolynomial(c0, c1, c2, lam), b = SigmoidPolynomialPlain(c0, c1, c2, lam);
        // SinCosf against the separate calls, on an angle from the same hash (any value)
        float sn, cs;
        SinCosf(c2, &sn, &cs);
        if (!SameFloat(sn, Sinf(c2)) || !SameFloat(cs, Cosf(c2))) atomicAdd(&bad[50], 1ull);
        // DenseOffset's 32-bit form against lround over every float in [384, 712) (k / 4 sweeps it)
        {
            const float l = __uint_as_float(0x43C00000u + (uint32_t)((k / 4) % 0x720000u));
            const long o = std::lround(l) - 395;
            if (DenseOffset(l) != ((o < 0 || o > 310) ? -1 : (int)o)) atomicAdd(&bad[51], 1ull);
        }
        // DivByRcp (x / p from the correctly rounded 1 / p) against the IEEE division: any
        // operands, and quotients placed next to a rounding midpoint (x = RN(p * m), m with a
        // 25th significant bit) where a one-step correction is most likely to round wrongly
        {
            const float p = CheckOperand(k + 5, 3.f);
            const float x0 = CheckOperand(k + 6, 5.f);
            const uint32_t hm = CheckHash(k + 7);
            const double mid = (double)__uint_as_float((hm & 0x807fffffu) | (127u << 23)) +
                               ((hm >> 31) ? -0x1p-24 : 0x1p-24);  // halfway between two floats
            const float xs[2] = {x0, (float)((double)p * mid)};
#pragma unroll
            for (int j = 0; j < 2; ++j)
                if (!SameFloat(DivByRcp(xs[j], p, 1 / p, DivFastOk(p)), xs[j] / p)) atomicAdd(&bad[52], 1ull);
        }
        if (!SameFloat(a, b)) {
            ++ns;
            // the first few mismatches: inputs and both results (slots 1..96 of bad, as float bits)
            const unsigned long long slot = atomicAdd(&bad[1], 1ull);
            if (slot < 16) {
                float *ex = reinterpret_cast<float *>(bad + 2) + 6 * slot;
                ex[0] = c0, ex[1] = c1, ex[2] = c2, ex[3] = lam, ex[4] = a, ex[5] = b;
            }
        }
    }
    atomicAdd(&bad[0], ns);
}
// the device's portable transcendentals (core/detmath.h) on given inputs: fn 0 sin, 1 cos, 2 asin,
// 3 acos, 4 atan2(a, b), 5 log, 6 sin of SinCosf, 7 cos of SinCosf, 8 exp, 9 sinh
__global__ void k_det_math(int fn, const float *a, const float *b, int n, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = detm::Eval(fn, a[i], b[i]);
}
hipError_t LaunchDetMath(int fn, const float *a, const float *b, int n, float *out, hipStream_t s) {
    hipLaunchKernelGGL(k_det_math, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, fn, a, b, n, out);
    return hipGetLastError();
}
// A pass's queue-capacity check: a shard's count above capS means its producers wrote past the
// shard into the next one (AllocPaths sizes the per-shard slack for kShards producer kernels of
// one queue); st.stats[kStatQueueOverflow] counts such counters and pbrt_synchronize fails.  The
// depth-0 ray queue keeps every camera ray in shard 0 and is exempt.
__global__ void k_queue_overflow(PathState st, int nDepths) {
    const int n = nDepths * kNumQueues * kShards;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        if (i < kShards) continue;  // depth 0, queue 0
        if (st.counters[i * kCounterPad] > st.capS) atomicAdd(&st.stats[kStatQueueOverflow], 1ull);
    }
}
hipError_t LaunchQueueOverflowCheck(const PathState &st, int nDepths, hipStream_t s) {
    hipLaunchKernelGGL(k_queue_overflow, dim3(1), dim3(kBlock), 0, s, st, nDepths);
    return hipGetLastError();
}
// HairBxDF f / PDF / Sample_f per query (core/hair.h HairDebugEval; pbrt_debug_hair)
__global__ void k_hair_eval(const float *in, int n, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) HairDebugEval(in + (size_t)kHairDebugIn * i, out + (size_t)kHairDebugOut * i);
}
hipError_t LaunchHairEval(const float *in, int n, float *out, hipStream_t s) {
    hipLaunchKernelGGL(k_hair_eval, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, in, n, out);
    return hipGetLastError();
}
// the Catmull-Rom spline utilities of the subsurface kernels (core/bssrdf.h) per query, as the
// host entry pbrt_debug_catmull_rom computes them: op 0 weights [6], 1 invert, 3 sample2d
__global__ void k_catmull_rom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                              const float *cdf, const float *x, int n, float *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == 0) {
        int off = 0;
        float w[4] = {0, 0, 0, 0};
        const bool ok = CatmullRomWeights(nodes1, n1, x[i], &off, w);
        const float r[6] = {ok ? 1.f : 0.f, (float)(ok ? off : 0), w[0], w[1], w[2], w[3]};
        for (int k = 0; k < 6; ++k) out[6 * i + k] = r[k];
    } else if (op == 1) {
        out[i] = InvertCatmullRom(nodes1, values, n1, x[i]);
    } else {
        out[i] = SampleCatmullRom2D(nodes1, n1, nodes2, n2, values, cdf, x[2 * i], x[2 * i + 1]);
    }
}
hipError_t LaunchCatmullRom(int op, const float *nodes1, int n1, const float *nodes2, int n2, const float *values,
                            const float *cdf, const float *x, int n, float *out, hipStream_t s) {
    hipLaunchKernelGGL(k_catmull_rom, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, op, nodes1, n1, nodes2, n2,
                       values, cdf, x, n, out);
    return hipGetLastError();
}
hipError_t LaunchCheckRNMath(uint64_t seed, int blocks, int perThread, unsigned long long *bad, hipStream_t s) {
    hipLaunchKernelGGL(k_check_rn_math, dim3(blocks), dim3(kBlock), 0, s, seed, perThread, bad);
    return hipGetLastError();
}

// ------------------------------------------------------------------ launch helpers (host)
// Blocks (of kBlock threads) per CU the traversal kernels of a mode are compiled for
int TraversalBlocksCompiled(int compressed) { return TraversalWaves(compressed ? kTravQuant : kTravWide); }

// Largest static LDS of the traversal kernels (k_closest's queue staging), for BuildDevice's
// check that the group stack + node cache + static LDS fit one block's LDS
size_t SurfaceTraversalStaticLds(int tm) {
    size_t m = 0;
    auto take = [&](const void *f) {
        hipFuncAttributes a{};
        if (hipFuncGetAttributes(&a, f) == hipSuccess) m = std::max(m, (size_t)a.sharedSizeBytes);
    };
#define TAKE_TM(TM)                                                             \
    if (tm == TM) {                                                             \
        take(reinterpret_cast<const void *>(&k_closest<kNumMatTypes, TM>));     \
        take(reinterpret_cast<const void *>(&k_closest<1, TM>));                \
        take(reinterpret_cast<const void *>(&k_shadow<TM>));                    \
        take(reinterpret_cast<const void *>(&k_intersect_batch<TM>));           \
    }
    TAKE_TM(kTravLds) TAKE_TM(kTravWide) TAKE_TM(kTravQuant)
#undef TAKE_TM
    return m;
}
static size_t StackBytes(const DeviceScene &S) {
    return TraversalLdsBytes(S.stackSize, S.ldsNodes, S.ldsTris, S.compressed);
}

// Producer grids are multiples of kShards (the shard capacity bound depends on it).
static int ShardedGrid(int n, int cap) {
    int g = (n + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > cap ? cap : g);
    return (g + kShards - 1) / kShards * kShards;
}
static int TraversalGridFor(int n) { return ShardedGrid(n, PBRT_GRID_CAP); }
static int ShadeGridFor(int n) { return ShardedGrid(n, PBRT_SHADE_GRID_CAP); }

// Kernels over queues whose length is only known on the device (emissive hits, escaped rays):
// a grid of one block per CU, grid-stride beyond that.  With k_escaped's LDS tables an open
// scene's millions of sky rays (C3) run as fast at 256 blocks as at 4096 (688 vs 686 Msamples/s).
static int SmallGridFor(int n) {
    static const int cap = getenv("PBRT_AMD_EMIT_GRID") ? atoi(getenv("PBRT_AMD_EMIT_GRID")) : 256;
    int g = (n + kBlock - 1) / kBlock;
    return g < 1 ? 1 : (g > cap ? cap : g);
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
                         hipStream_t s, bool sorted) {
    const dim3 grid(TraversalGridFor(maxCount)), block(kBlock);
    const bool multi = S.matTypeMask & ~1;
    const int so = sorted ? 1 : 0;
#define K_CLOSEST_MIX(tm) k_closest<kClosestMix, tm>
#define K_CLOSEST_MULTI(tm) k_closest<kNumMatTypes, tm>
#define K_CLOSEST_ONE(tm) k_closest<1, tm>
    if (st.hitMat[0]) PBRT_LAUNCH_TRAVERSAL(S, K_CLOSEST_MIX, grid, block, StackBytes(S), s, S, st, depth, timed, so);
    else if (multi) PBRT_LAUNCH_TRAVERSAL(S, K_CLOSEST_MULTI, grid, block, StackBytes(S), s, S, st, depth, timed, so);
    else PBRT_LAUNCH_TRAVERSAL(S, K_CLOSEST_ONE, grid, block, StackBytes(S), s, S, st, depth, timed, so);
#undef K_CLOSEST_MIX
#undef K_CLOSEST_MULTI
#undef K_CLOSEST_ONE
    return hipGetLastError();
}
hipError_t LaunchRayBin(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    const int g = std::max(1, std::min(2048, (maxCount + kBinBlock - 1) / kBinBlock));
    hipLaunchKernelGGL(k_raybin_hist, dim3(std::min(g, 1024)), dim3(kBinBlock), 0, s, S, st, depth);
    hipLaunchKernelGGL(k_raybin_scan, dim3(1), dim3(kBinBlock), 0, s, st);
    const int gs = std::max(1, std::min(2048, (maxCount + kBinBlock * kBinItems - 1) / (kBinBlock * kBinItems)));
    hipLaunchKernelGGL(k_raybin_scatter, dim3(gs), dim3(kBinBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchClassify(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    const dim3 grid(GridFor(maxCount)), block(kBlock);
    if (st.hitMat[0]) hipLaunchKernelGGL(k_classify<kClosestMix>, grid, block, 0, s, S, st, depth);
    else if (S.matTypeMask & ~1) hipLaunchKernelGGL(k_classify<kNumMatTypes>, grid, block, 0, s, S, st, depth);
    else hipLaunchKernelGGL(k_classify<1>, grid, block, 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchEscaped(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    hipLaunchKernelGGL(k_escaped, dim3(SmallGridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchEmissive(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
    if (S.nShapes > 0 || S.nImageAreaLights > 0)
        hipLaunchKernelGGL(k_emissive<true>, dim3(SmallGridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    else hipLaunchKernelGGL(k_emissive<false>, dim3(SmallGridFor(maxCount)), dim3(kBlock), 0, s, S, st, depth);
    return hipGetLastError();
}
// Dynamic LDS of a shade launch: the layout up to this depth's Halton permutation tables, which
// come last and grow with the depth's prime bases (ShadeLdsLayout::totalByDepth)
static size_t ShadeLdsBytes(const DeviceScene &S, int depth, bool withPl = false) {
    const ShadeLdsLayout &L = S.shadeLds;
    return (size_t)(depth < kShadeLdsDepths ? L.totalByDepth[depth] : L.total) +
           (withPl && L.plInLds ? (size_t)L.plCount * 8 : 0);
}
hipError_t LaunchTexture(const DeviceScene &S, const PathState &st, int depth, int type, bool full, int maxCount,
                         hipStream_t s) {
    // the material queue is large and the kernel latency-bound: enough blocks for every SIMD's
    // wave slots (a 256-block grid left C4's k_texture at one wave per SIMD), each block's LDS
    // tables amortised over its grid-stride items
    const int g = (maxCount + kBlock - 1) / kBlock;
    const dim3 grid(g < 1 ? 1 : (g > 2048 ? 2048 : g));
#define K_TEX(mt)                                                                             \
    do {                                                                                      \
        if (S.nShapes > 0) hipLaunchKernelGGL((k_texture<mt, true, true>), grid, dim3(kBlock), 0, s, S, st, depth); \
        else if (full) hipLaunchKernelGGL((k_texture<mt, true>), grid, dim3(kBlock), 0, s, S, st, depth);  \
        else hipLaunchKernelGGL((k_texture<mt, false>), grid, dim3(kBlock), 0, s, S, st, depth);      \
    } while (0)
    if (type == kMatDiffuseT) K_TEX(kMatDiffuseT);
    else if (type == kMatDielectricT) K_TEX(kMatDielectricT);
    else K_TEX(kMatConductorT);
#undef K_TEX
    return hipGetLastError();
}
hipError_t LaunchShadeDiffuse(const DeviceScene &S, const PathState &st, int depth, int maxCount, bool lean,
                              hipStream_t s) {
    const dim3 grid(ShadeGridFor(maxCount)), block(kBlock);
    const size_t lds = ShadeLdsBytes(S, depth);
    const bool ext = S.nShapes > 0 || S.nEnv > 0 || S.nImageDelta > 0 || S.hasSpread || S.nImageAreaLights > 0;
    // the lean kernel compiles the Ext paths (spread falloff, image emitters, shapes, image
    // lights) and textures out: a launcher that asks for it on such a scene is a bug
    if (lean && (ext || S.textured)) return hipErrorInvalidValue;
    if (S.textured && ext) hipLaunchKernelGGL((k_shade_diffuse<false, true, true>), grid, block, lds, s, S, st, depth);
    else if (S.textured) hipLaunchKernelGGL((k_shade_diffuse<false, true>), grid, block, lds, s, S, st, depth);
    else if (lean) hipLaunchKernelGGL(k_shade_diffuse<true>, grid, block, lds, s, S, st, depth);
    else if (ext) hipLaunchKernelGGL((k_shade_diffuse<false, false, true>), grid, block, lds, s, S, st, depth);
    else hipLaunchKernelGGL(k_shade_diffuse<false>, grid, block, lds, s, S, st, depth);
    return hipGetLastError();
}
hipError_t LaunchShadeMicrofacet(const DeviceScene &S, const PathState &st, int depth, int type, int maxCount,
                                 hipStream_t s) {
    const dim3 grid(ShadeGridFor(maxCount)), block(kBlock);
    const size_t lds = ShadeLdsBytes(S, depth, true);
    const bool ext = S.nShapes > 0 || S.nEnv > 0 || S.nImageDelta > 0 || S.hasSpread || S.nImageAreaLights > 0, diel = type == kMatDielectricT;
#define K_MF(mt, smooth, tex, ex) hipLaunchKernelGGL((k_shade_microfacet<mt, smooth, tex, ex>), grid, block, lds, s, S, st, depth)
    if (ext) {
        if (diel && S.textured) K_MF(kMatDielectricT, false, true, true);
        else if (diel) K_MF(kMatDielectricT, false, false, true);
        else if (S.textured) K_MF(kMatConductorT, false, true, true);
        else K_MF(kMatConductorT, false, false, true);
    } else if (S.textured) {
        if (diel) K_MF(kMatDielectricT, false, true, false);
        else K_MF(kMatConductorT, false, true, false);
    } else if (diel && S.smoothDielectrics) {
        K_MF(kMatDielectricT, true, false, false);
    } else if (diel) {
        K_MF(kMatDielectricT, false, false, false);
    } else {
        K_MF(kMatConductorT, false, false, false);
    }
#undef K_MF
    return hipGetLastError();
}
hipError_t LaunchShadow(const DeviceScene &S, const PathState &st, int depth, int maxCount, hipStream_t s) {
#define K_SHADOW(tm) k_shadow<tm>
    PBRT_LAUNCH_TRAVERSAL(S, K_SHADOW, dim3(TraversalGridFor(maxCount)), dim3(kBlock), StackBytes(S), s, S, st, depth);
#undef K_SHADOW
    return hipGetLastError();
}
hipError_t LaunchFilm(const DeviceScene &S, const PathState &st, int nSamples, hipStream_t s) {
    hipLaunchKernelGGL(k_film, dim3((st.P + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, nSamples);
    return hipGetLastError();
}
hipError_t LaunchIntersectBatch(const DeviceScene &S, const float *rays, int n, int anyHit, int *outPrim,
                                float *outHit, hipStream_t s) {
#define K_BATCH(tm) k_intersect_batch<tm>
    PBRT_LAUNCH_TRAVERSAL(S, K_BATCH, dim3(TraversalGridFor(n)), dim3(kBlock), StackBytes(S), s, S, rays, n, anyHit,
                          outPrim, outHit);
#undef K_BATCH
    return hipGetLastError();
}

}  // namespace pbrt_amd
