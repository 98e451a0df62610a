// MI355X wavefront kernels for scenes with participating media: pbrt's
// WavefrontPathIntegrator with haveMedia (wavefront/integrator.cpp:290-493).
//
// Stage <-> reference mapping (one launch each per wavefront iteration):
//   k_vcamera    GenerateCameraRays (camera.cpp:31-80) + the camera medium
//   k_vclosest   IntersectClosest (integrator.h:39-45): closest hit; rays inside a medium go to
//                the medium-sample queue (MediumSampleQueue, intersect.h:48-80), the rest to
//                the surface, interface-crossing or escaped-ray queue
//   k_vmedium    SampleMediumInteraction (media.cpp:22-247): delta tracking along the ray
//                through SampleT_maj (media.h:725-800) with the homogeneous / DDA majorant
//                iterators (media.h:79-205), medium emission, absorption / real scattering /
//                null scattering; survivors continue to the same three queues
//   k_vescaped   HandleEscapedRays (integrator.cpp:495-537)
//   k_viface     interface crossings (media.cpp:193-203)
//   k_vsurface   the surface side: HandleEmissiveIntersection (:539-573) and
//                EvaluateMaterialAndBSDF (surfscatter.cpp:57-328) for every material type
//   k_vscatter   SampleMediumScattering<HGPhaseFunction> (media.cpp:259-352)
//   k_vshadow    TraceTransmittance (intersect.h:164-274): shadow rays through interfaces with
//                ratio tracking in each medium they cross
// Film: k_film of wavefront.hip (the same per-slot sensor-RGB L).
//
// Records are keyed by their index in the iteration's ray queue; every queue is sharded like
// the surface path's (device.h kShards).  Spectral state (beta, r_u, r_l, T_maj) lives in
// registers inside a kernel and wavelength-major in HBM between kernels.
#ifndef PBRT_VOL_EXPERIMENT
#define PBRT_VOL_EXPERIMENT 0  // timing experiments only (tools/exp_*.sh), never in the product
#endif
#include "common.h"
#include "../core/bssrdf.h"
#include "../core/hair.h"
#include "../core/measured.h"

namespace pbrt_amd {

#ifndef PBRT_VOL_WAVES
#define PBRT_VOL_WAVES 2  // waves/SIMD the spectral media kernels are compiled for
#endif
#ifndef PBRT_VOL_GREY_WAVES
#define PBRT_VOL_GREY_WAVES 3  // waves/SIMD of the grey-medium sampling kernel
#endif
constexpr int kNS = kNSpectrumSamples;

// ------------------------------------------------------------------ media
struct MediumRef {
    const int *I;    // 16 ints (device.h DeviceMedia)
    const float *P;  // 24 floats
};
__device__ inline MediumRef MediumAt(const DeviceScene &S, int m) {
    return MediumRef{S.media.info + 16 * m, S.media.params + 24 * m};
}
__device__ inline float DenseAt(const DeviceScene &S, int idx, int off) {
    return off < 0 ? 0.f : S.dense[idx * kDenseN + off];
}

// Transform::ApplyInverse(Point3f) (util/transform.h:387-398) with mediumFromRender
__device__ inline V3 MediumFromRender(const float *M, V3 p) {
    const float x = (M[0] * p.x + M[1] * p.y) + (M[2] * p.z + M[3]);
    const float y = (M[4] * p.x + M[5] * p.y) + (M[6] * p.z + M[7]);
    const float z = (M[8] * p.x + M[9] * p.y) + (M[10] * p.z + M[11]);
    const float w = (M[12] * p.x + M[13] * p.y) + (M[14] * p.z + M[15]);
    if (w == 1) return V3(x, y, z);
    return V3(x, y, z) / w;
}
// Bounds3::Offset (util/vecmath.h:1325-1334), bounds = P[1..3], P[4..6]
__device__ inline V3 BoundsOffset(const float *P, V3 p) {
    V3 o(p.x - P[1], p.y - P[2], p.z - P[3]);
    if (P[4] > P[1]) o.x /= P[4] - P[1];
    if (P[5] > P[2]) o.y /= P[5] - P[2];
    if (P[6] > P[3]) o.z /= P[6] - P[3];
    return o;
}
// SampledGrid<Float>::Lookup(Point3f) (util/containers.h:804-835): trilinear, zero outside
__device__ inline float GridLookup(const float *v, int nx, int ny, int nz, V3 p) {
    const float sx = p.x * nx - .5f, sy = p.y * ny - .5f, sz = p.z * nz - .5f;
    const int ix = (int)floorf(sx), iy = (int)floorf(sy), iz = (int)floorf(sz);
    const float dx = sx - ix, dy = sy - iy, dz = sz - iz;
    auto at = [&](int x, int y, int z) -> float {
        if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return 0.f;
        return v[((size_t)z * ny + y) * nx + x];
    };
    const float d00 = Lerpf(dx, at(ix, iy, iz), at(ix + 1, iy, iz));
    const float d10 = Lerpf(dx, at(ix, iy + 1, iz), at(ix + 1, iy + 1, iz));
    const float d01 = Lerpf(dx, at(ix, iy, iz + 1), at(ix + 1, iy, iz + 1));
    const float d11 = Lerpf(dx, at(ix, iy + 1, iz + 1), at(ix + 1, iy + 1, iz + 1));
    return Lerpf(dz, Lerpf(dy, d00, d10), Lerpf(dy, d01, d11));
}

// Medium::SamplePoint (media.h:209-350) reduced to its scalars: sigma_a = dense(I[1]) * d,
// sigma_s = dense(I[2]) * d, Le = dense(I[3]) * le (le = 0: no emission at p).  Homogeneous:
// d = le = 1 (x * 1 is exact, so the spectra are the reference's).
// RGBGridMedium (media.h:355-428): rgb, and the trilinear lookup's voxel and offsets, from which
// MediumSigmaA / MediumSigmaS / MediumLe evaluate the spectra per wavelength.
struct MediumPoint {
    float d, le;
    float temp;  // GridMedium temperature > 100 K at p (Le = le * BlackbodySpectrum(temp)), else 0
    bool rgb;
    int ix, iy, iz;
    float dx, dy, dz;
};
// SampledGrid<RGB*Spectrum>::Lookup(p, convert) (util/containers.h:785-829) at one wavelength:
// a voxel's value is scale * rsp(lambda) (RGBUnboundedSpectrum::Sample), times the illuminant
// for Le (RGBIlluminantSpectrum::Sample); outside the grid T{} converts to 0.
__device__ inline float RGBGridAt(const DeviceScene &S, const MediumRef &m, const MediumPoint &mp, int block, float lam,
                                  float illum) {
    const int nx = m.I[5], ny = m.I[6], nz = m.I[7];
    const float *g = S.media.values + m.I[11] + (size_t)block * 4 * nx * ny * nz;
    auto at = [&](int x, int y, int z) -> float {
        if (x < 0 || x >= nx || y < 0 || y >= ny || z < 0 || z >= nz) return 0.f;
        const float *c = g + 4 * (((size_t)z * ny + y) * nx + x);
        const float v = c[3] * SigmoidPolynomial(c[0], c[1], c[2], lam);
        return block == 2 ? v * illum : v;
    };
    const int ix = mp.ix, iy = mp.iy, iz = mp.iz;
    const float d00 = Lerpf(mp.dx, at(ix, iy, iz), at(ix + 1, iy, iz));
    const float d10 = Lerpf(mp.dx, at(ix, iy + 1, iz), at(ix + 1, iy + 1, iz));
    const float d01 = Lerpf(mp.dx, at(ix, iy, iz + 1), at(ix + 1, iy, iz + 1));
    const float d11 = Lerpf(mp.dx, at(ix, iy + 1, iz + 1), at(ix + 1, iy + 1, iz + 1));
    return Lerpf(mp.dz, Lerpf(mp.dy, d00, d10), Lerpf(mp.dy, d01, d11));
}
// sigma_a, sigma_s, Le of MediumProperties at wavelength lam (dense offset off)
__device__ inline float MediumSigmaA(const DeviceScene &S, const MediumRef &m, const MediumPoint &mp, int off, float lam) {
    if (!mp.rgb) return DenseAt(S, m.I[1], off) * mp.d;
    return m.P[7] * ((m.I[15] & 1) ? RGBGridAt(S, m, mp, 0, lam, 1.f) : 1.f);
}
__device__ inline float MediumSigmaS(const DeviceScene &S, const MediumRef &m, const MediumPoint &mp, int off, float lam) {
    if (!mp.rgb) return DenseAt(S, m.I[2], off) * mp.d;
    return m.P[7] * ((m.I[15] & 2) ? RGBGridAt(S, m, mp, 1, lam, 1.f) : 1.f);
}
__device__ inline float MediumLe(const DeviceScene &S, const MediumRef &m, const MediumPoint &mp, int off, float lam) {
    if (!mp.rgb) {
        if (mp.temp > 0) return mp.le * (Blackbody(lam, mp.temp) * BlackbodyNorm(mp.temp));
        return DenseAt(S, m.I[3], off) * mp.le;
    }
    return S.media.values[m.I[12]] * RGBGridAt(S, m, mp, 2, lam, DenseAt(S, m.I[3], off));
}
// Cloud: the scene has a CloudMedium.  Its density (13 noise evaluations) inlined into every
// medium event made the grey media kernels spill (C5 k_vshadow_grey 575 -> 944 us per launch,
// k_vmedium_grey 1009 -> 1203 us), so the grey kernels have instantiations without it.
template <bool Cloud = true>
__device__ inline MediumPoint SampleMediumPoint(const DeviceScene &S, const MediumRef &m, V3 p) {
    MediumPoint r;
    r.rgb = false;
    r.temp = 0.f;
    if (Cloud && m.I[0] == kDevMediumCloud) {
        r.d = CloudDensity(S.media.values + m.I[11], MediumFromRender(m.P + 8, p));
        r.le = 0.f;
        return r;
    }
    if (m.I[0] != kDevMediumGrid && m.I[0] != kDevMediumRGBGrid) {
        r.d = r.le = 1.f;
        return r;
    }
    const V3 q = BoundsOffset(m.P, MediumFromRender(m.P + 8, p));
    if (m.I[0] == kDevMediumRGBGrid) {
        const float sx = q.x * m.I[5] - .5f, sy = q.y * m.I[6] - .5f, sz = q.z * m.I[7] - .5f;
        r.rgb = true;
        r.ix = (int)floorf(sx), r.iy = (int)floorf(sy), r.iz = (int)floorf(sz);
        r.dx = sx - r.ix, r.dy = sy - r.iy, r.dz = sz - r.iz;
        r.d = 1.f;
        r.le = m.I[4] ? 1.f : 0.f;  // IsEmissive: an Le grid and LeScale > 0
        return r;
    }
    r.d = GridLookup(S.media.values + m.I[11], m.I[5], m.I[6], m.I[7], q);
    r.le = 0.f;
    if (m.I[4]) {
        const float scale = GridLookup(S.media.values + m.I[12], m.I[8], m.I[9], m.I[10], q);
        if (scale > 0) r.le = scale;
        if (scale > 0 && m.I[15] >= 0) {
            // temperature grid (media.h:303-311): {offset, scale} then the grid
            const float *tg = S.media.values + m.I[15];
            const float t = (GridLookup(tg + 2, m.I[5], m.I[6], m.I[7], q) - tg[0]) * tg[1];
            if (t > 100.f) r.temp = t;
            else r.le = 0.f;
        }
    }
    return r;
}

// Majorant segments of a ray (HomogeneousMajorantIterator, media.h:79-102, and
// DDAMajorantIterator over the 16^3 majorant grid, media.h:136-205).  A segment's majorant is
// sigma_t(lambda) * mx: the iterator yields the scalar mx (1 for a homogeneous medium).
struct MajorantIter {
    bool dda, called, empty;
    float tMin, tMax;
    float nextCrossingT[3], deltaT[3];
    int step[3], voxelLimit[3], voxel[3];
    const float *grid;
    __device__ bool Next(float *segMin, float *segMax, float *mx) {
        if (!dda) {
            if (called || empty) return false;
            called = true;
            *segMin = tMin;
            *segMax = tMax;
            *mx = 1.f;
            return true;
        }
        if (empty || tMin >= tMax) return false;
        const int bits = ((nextCrossingT[0] < nextCrossingT[1]) << 2) + ((nextCrossingT[0] < nextCrossingT[2]) << 1) +
                         ((nextCrossingT[1] < nextCrossingT[2]));
        // cmpToAxis[8] = {2, 1, 2, 1, 2, 2, 0, 0} as a 2-bit table
        const int stepAxis = (0x0A66 >> (2 * bits)) & 3;
        const float nct = stepAxis == 0 ? nextCrossingT[0] : (stepAxis == 1 ? nextCrossingT[1] : nextCrossingT[2]);
        const float tVoxelExit = fminf(tMax, nct);
        *mx = grid[voxel[0] + kMajorantRes * (voxel[1] + kMajorantRes * voxel[2])];
        *segMin = tMin;
        *segMax = tVoxelExit;
        tMin = tVoxelExit;
        if (nct > tMax) tMin = tMax;
#pragma unroll
        for (int a = 0; a < 3; ++a)
            if (a == stepAxis) {
                voxel[a] += step[a];
                if (voxel[a] == voxelLimit[a]) tMin = tMax;
                nextCrossingT[a] += deltaT[a];
            }
        return true;
    }
};

// Medium::SampleRay (media.h:240-250 homogeneous, :319-333 grid) for a ray with a normalised
// direction and render-space tMax
__device__ inline MajorantIter SampleMediumRay(const DeviceScene &S, const MediumRef &m, V3 o, V3 d, float raytMax) {
    MajorantIter it;
    it.called = false;
    it.empty = false;
    it.grid = nullptr;
    if (m.I[0] != kDevMediumGrid && m.I[0] != kDevMediumCloud && m.I[0] != kDevMediumRGBGrid) {
        it.dda = false;
        it.tMin = 0;
        it.tMax = raytMax;
        return it;
    }
    it.dda = m.I[0] != kDevMediumCloud;  // GridMedium, RGBGridMedium: DDAMajorantIterator
    // Transform::ApplyInverse(Ray, &tMax) (util/transform.h:416-429): the exact origin becomes a
    // Point3fi (transform.cpp:263-303), is pushed to the edge of its error bounds along d
    const float *M = m.P + 8;
    const float xp = (M[0] * o.x + M[1] * o.y) + (M[2] * o.z + M[3]);
    const float yp = (M[4] * o.x + M[5] * o.y) + (M[6] * o.z + M[7]);
    const float zp = (M[8] * o.x + M[9] * o.y) + (M[10] * o.z + M[11]);
    const V3 err(gamma(3) * (fabsf(M[0] * o.x) + fabsf(M[1] * o.y) + fabsf(M[2] * o.z)),
                 gamma(3) * (fabsf(M[4] * o.x) + fabsf(M[5] * o.y) + fabsf(M[6] * o.z)),
                 gamma(3) * (fabsf(M[8] * o.x) + fabsf(M[9] * o.y) + fabsf(M[10] * o.z)));
    float lo[3], hi[3];
    const float pc[3] = {xp, yp, zp}, pe[3] = {err.x, err.y, err.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        lo[a] = pe[a] == 0 ? pc[a] : NextFloatDown(pc[a] - pe[a]);
        hi[a] = pe[a] == 0 ? pc[a] : NextFloatUp(pc[a] + pe[a]);
    }
    const V3 dm(M[0] * d.x + M[1] * d.y + M[2] * d.z, M[4] * d.x + M[5] * d.y + M[6] * d.z,
                M[8] * d.x + M[9] * d.y + M[10] * d.z);
    const float l2 = LengthSquared(dm);
    if (l2 > 0) {
        const V3 oErr((hi[0] - lo[0]) / 2, (hi[1] - lo[1]) / 2, (hi[2] - lo[2]) / 2);
        const float dt = Dot(Abs(dm), oErr) / l2;
        const float dv[3] = {dm.x * dt, dm.y * dt, dm.z * dt};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = NextFloatDown(lo[a] + dv[a]);
            hi[a] = NextFloatUp(hi[a] + dv[a]);
        }
        raytMax -= dt;
    }
    const float om[3] = {(lo[0] + hi[0]) / 2, (lo[1] + hi[1]) / 2, (lo[2] + hi[2]) / 2};
    const float dmv[3] = {dm.x, dm.y, dm.z};
    // Bounds3::IntersectP(o, d, tMax, &t0, &t1) (util/vecmath.h:1549-1573)
    const float *P = m.P;
    float t0 = 0, t1 = raytMax;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float inv = 1 / dmv[a];
        float tNear = (P[1 + a] - om[a]) * inv, tFar = (P[4 + a] - om[a]) * inv;
        if (tNear > tFar) {
            const float t = tNear;
            tNear = tFar;
            tFar = t;
        }
        tFar *= 1 + 2 * gamma(3);
        t0 = tNear > t0 ? tNear : t0;
        t1 = tFar < t1 ? tFar : t1;
        if (t0 > t1) it.empty = true;
    }
    if (it.empty) return it;
    if (!it.dda) {  // CloudMedium: HomogeneousMajorantIterator(tMin, tMax, sigma_t) over the bounds
        it.tMin = t0;
        it.tMax = t1;
        return it;
    }
    // DDAMajorantIterator ctor (media.h:140-166)
    it.grid = S.media.values + m.I[13];
    it.tMin = t0;
    it.tMax = t1;
    const float diag[3] = {P[4] - P[1], P[5] - P[2], P[6] - P[3]};
    const V3 og = BoundsOffset(P, V3(om[0], om[1], om[2]));
    const float ogv[3] = {og.x, og.y, og.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float dg = dmv[a] / diag[a];
        const float gi = ogv[a] + dg * t0;
        it.voxel[a] = (int)Clampf(gi * kMajorantRes, 0, kMajorantRes - 1);
        it.deltaT[a] = 1 / (fabsf(dg) * kMajorantRes);
        if (dg == -0.f) dg = 0.f;
        if (dg >= 0) {
            const float next = float(it.voxel[a] + 1) / kMajorantRes;
            it.nextCrossingT[a] = t0 + (next - gi) / dg;
            it.step[a] = 1;
            it.voxelLimit[a] = kMajorantRes;
        } else {
            const float next = float(it.voxel[a]) / kMajorantRes;
            it.nextCrossingT[a] = t0 + (next - gi) / dg;
            it.step[a] = -1;
            it.voxelLimit[a] = -1;
        }
    }
    return it;
}

// Per-wavelength offsets into the dense tables for a path's 31 wavelengths
// (SampledWavelengths::SampleUniform's +10 nm recurrence, util/spectrum.h:318-336)
struct WaveOffsets {
    int off[kNS];
    float lam0;  // lambda[0] (the RGB grid medium evaluates its spectra at the wavelengths)
    __device__ explicit WaveOffsets(float lambda0) : lam0(lambda0) {
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNS; ++i, it.Next()) off[i] = DenseOffset(it.lam);
    }
};

__device__ inline float AvgArr(const float *a) {
    float s = a[0];
#pragma unroll
    for (int i = 1; i < kNS; ++i) s += a[i];
    return s / kNS;
}
__device__ inline bool AnyNonZero(const float *a) {
    bool nz = false;
#pragma unroll
    for (int i = 0; i < kNS; ++i) nz |= a[i] != 0;
    return nz;
}

// SampleT_maj<ConcreteMedium> (media.h:737-800).  `event(p, mp, mx, Tm)` is the callback:
// sigma_maj_i = (sigma_a_i + sigma_s_i) * mx; returns false to stop.  Returns true when the
// traversal ran to the end (T_maj = Tm then) and false when the callback stopped it
// (SampleT_maj returns SampledSpectrum(1) then).
template <typename F>
__device__ __forceinline__ bool SampleTmaj(const DeviceScene &S, const MediumRef &m, const WaveOffsets &wo, V3 o, V3 d,
                                  float tMax, float u, PCG32 &rng, float Tm[kNS], F &&event) {
    tMax *= Length(d);
    d = Normalize(d);
    MajorantIter iter = SampleMediumRay(S, m, o, d, tMax);
#pragma unroll
    for (int i = 0; i < kNS; ++i) Tm[i] = 1.f;
    const int sa = m.I[1], ss = m.I[2];
    const float st0 = DenseAt(S, sa, wo.off[0]) + DenseAt(S, ss, wo.off[0]);
    float segMin, segMax, mx;
    while (iter.Next(&segMin, &segMax, &mx)) {
        const float smaj0 = st0 * mx;
        if (smaj0 == 0) {
            float dt = segMax - segMin;
            if (isinf(dt)) dt = 3.402823466e+38f;
#pragma unroll
            for (int i = 0; i < kNS; ++i) {
                const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                Tm[i] *= FastExp(smaj * -dt);
            }
            continue;
        }
        float tMin = segMin;
        while (true) {
            const float t = tMin + SampleExponential(u, smaj0);
            u = rng.Uniform();
            if (t < segMax) {
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                    Tm[i] *= FastExp(smaj * -(t - tMin));
                }
                const V3 p = o + d * t;
                const MediumPoint mp = SampleMediumPoint(S, m, p);
                if (!event(p, mp, mx, Tm)) return false;
#pragma unroll
                for (int i = 0; i < kNS; ++i) Tm[i] = 1.f;
                tMin = t;
            } else {
                float dt = segMax - tMin;
                if (isinf(dt)) dt = 3.402823466e+38f;
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                    Tm[i] *= FastExp(smaj * -dt);
                }
                break;
            }
        }
    }
    return true;
}

// SampleT_maj for a grey medium (sigma_a, sigma_s equal at every wavelength, DeviceMedia
// info[14]): every T_maj / sigma_maj entry is the same, so the reference's 31-wide products
// are one scalar product here -- the same float operations on the same values.
// sigmaT = sigma_a + sigma_s of the medium (its wavelength-0 entries).
template <bool Cloud, typename F>
__device__ __forceinline__ bool SampleTmajGrey(const DeviceScene &S, const MediumRef &m, float sigmaT, V3 o, V3 d,
                                               float tMax, float u, PCG32 &rng, float &Tm, F &&event) {
    tMax *= Length(d);
    d = Normalize(d);
    MajorantIter iter = SampleMediumRay(S, m, o, d, tMax);
    Tm = 1.f;
    float segMin, segMax, mx;
    while (iter.Next(&segMin, &segMax, &mx)) {
        const float smaj = sigmaT * mx;
        if (smaj == 0) {
            float dt = segMax - segMin;
            if (isinf(dt)) dt = 3.402823466e+38f;
            Tm *= FastExp(smaj * -dt);
            continue;
        }
        float tMin = segMin;
        while (true) {
            const float t = tMin + SampleExponential(u, smaj);
            u = rng.Uniform();
            if (t < segMax) {
                Tm *= FastExp(smaj * -(t - tMin));
                const V3 p = o + d * t;
                const MediumPoint mp = SampleMediumPoint<Cloud>(S, m, p);
                if (!event(p, mp, smaj, Tm)) return false;
                Tm = 1.f;
                tMin = t;
            } else {
                float dt = segMax - tMin;
                if (isinf(dt)) dt = 3.402823466e+38f;
                Tm *= FastExp(smaj * -dt);
                break;
            }
        }
    }
    return true;
}

// The lambda_0 share of a contribution, for paths that terminate their secondary wavelengths
// (dispersion): ToSensorRGB with pdf = (pdf_0 / n, 0, ...) keeps x(lambda_0) c_0 / pdf_0
// (SampledWavelengths::TerminateSecondary, spectrum.h; film.h:95-100)
__device__ inline void AddL0Off(const DeviceScene &S, const PathState &st, int slot, int off0, float c0) {
    if (!S.dispersive) return;
    SensorAcc a;
    a.Add(S, off0, c0, true);
    const int NL = st.N;
    st.L0[slot] += S.imagingRatio * a.sx;
    st.L0[NL + slot] += S.imagingRatio * a.sy;
    st.L0[2 * NL + slot] += S.imagingRatio * a.sz;
}

// Spectral contribution c_i (already divided by its MIS denominator) to sensor RGB
// (PixelSensor::ToSensorRGB, film.h:95-100), added to the slot's L
template <typename C>
__device__ inline void AddToL(const DeviceScene &S, const PathState &st, int slot, const WaveOffsets &wo, C &&c) {
    SensorAcc acc;
#pragma unroll
    for (int i = 0; i < kNS; ++i) acc.Add(S, wo.off[i], c(i), i == 0);
    const int NL = st.N;
    st.L[slot] += S.imagingRatio * (acc.sx / kNS);
    st.L[NL + slot] += S.imagingRatio * (acc.sy / kNS);
    st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNS);
    AddL0Off(S, st, slot, wo.off[0], c(0));
}

// RaySamples of a path depth (samples.cpp:29-66) from the global sampler tables
struct VRaySamples {
    float dUc, dU0, dU1, iUc, iU0, iU1, rr;
};
// indirectUc: the BxDF reads indirect.uc (dielectric); otherwise that dimension is skipped
__device__ inline VRaySamples RaySamplesAt(const DeviceScene &S, const PathState &st, int slot, int depth,
                                           bool indirectUc = true) {
#if PBRT_VOL_EXPERIMENT == 1
    { const float u = (slot & 1023) * (1.f / 1024); return VRaySamples{u, u * 0.5f, 0.7f - u * 0.5f, 0.3f, u, 1 - u, 0.9f}; }
#endif
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    const int d0 = 6 + S.dimsPerDepth * depth;
    VRaySamples r;
    if (S.samplerType >= kSamplerIndependent) {
        // the other samplers are stateful: every draw in pbrt's order, indirect.uc included
        GenericSampler g;
        g.Start(S.samp, px, py, sampleIndex, d0);
        r.dUc = g.Get1D(S.samp);
        g.Get2D(S.samp, &r.dU0, &r.dU1);
        const float iuc = g.Get1D(S.samp);
        r.iUc = indirectUc ? iuc : 0.f;
        g.Get2D(S.samp, &r.iU0, &r.iU1);
        r.rr = g.Get1D(S.samp);
    } else if (S.samplerType == 1) {
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        r.dUc = ZSobolGet1D(S.zs, morton, d0, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 1, S.zsPerms, S.sobolM1, &r.dU0, &r.dU1);
        r.iUc = indirectUc ? ZSobolGet1D(S.zs, morton, d0 + 3, S.zsPerms, S.sobolM1) : 0.f;
        ZSobolGet2D(S.zs, morton, d0 + 4, S.zsPerms, S.sobolM1, &r.iU0, &r.iU1);
        r.rr = ZSobolGet1D(S.zs, morton, d0 + 6, S.zsPerms, S.sobolM1);
    } else {
        Halton h = StartPixelSample(S, px, py, sampleIndex, d0);
        r.dUc = Get1D(S, h);
        Get2D(S, h, &r.dU0, &r.dU1);
        if (indirectUc) {
            r.iUc = Get1D(S, h);
        } else {  // Get1D's dimension bookkeeping without the sample
            if (h.dimension >= S.nDims) h.dimension = 2;
            ++h.dimension;
            r.iUc = 0.f;
        }
        Get2D(S, h, &r.iU0, &r.iU1);
        r.rr = Get1D(S, h);
    }
    return r;
}

// The subsurface samples of a path depth (samples.cpp:56-61): dimensions d0 + 7..9 after the
// seven direct / indirect ones
__device__ inline void SssSamplesAt(const DeviceScene &S, const PathState &st, int slot, int depth, float *uc,
                                    float *u0, float *u1) {
    int px, py, sampleIndex;
    PixelOf(st, slot, &px, &py, &sampleIndex);
    px += S.px0;
    const int d0 = 6 + S.dimsPerDepth * depth;
    if (S.samplerType >= kSamplerIndependent) {
        GenericSampler g;  // stateful: the seven draws before, in pbrt's order
        g.Start(S.samp, px, py, sampleIndex, d0);
        float a, b;
        (void)g.Get1D(S.samp);
        g.Get2D(S.samp, &a, &b);
        (void)g.Get1D(S.samp);
        g.Get2D(S.samp, &a, &b);
        (void)g.Get1D(S.samp);
        *uc = g.Get1D(S.samp);
        g.Get2D(S.samp, u0, u1);
    } else if (S.samplerType == 1) {
        const uint64_t morton = ZSobolMortonIndex(S.zs, px, py, sampleIndex);
        *uc = ZSobolGet1D(S.zs, morton, d0 + 7, S.zsPerms, S.sobolM1);
        ZSobolGet2D(S.zs, morton, d0 + 8, S.zsPerms, S.sobolM1, u0, u1);
    } else {
        // the stateful sampler's dimension after GenerateRaySamples' seven draws (Get1D, Get2D,
        // Get1D, Get2D, Get1D with their wrap to dimension 2), then the subsurface draws
        int d = d0;
        auto g1 = [&] { d = (d >= S.nDims ? 2 : d) + 1; };
        auto g2 = [&] { d = (d + 1 >= S.nDims ? 2 : d) + 2; };
        g1(), g2(), g1(), g2(), g1();
        Halton h = StartPixelSample(S, px, py, sampleIndex, d);
        *uc = Get1D(S, h);
        Get2D(S, h, u0, u1);
    }
}

// Spectral record I/O (wavelength-major).  A spectrum whose 31 entries are equal is stored
// "uniform": only entry 0 is written and a flag bit says so (camera rays, grey media and grey
// materials keep beta, r_u and r_l uniform; most shadow rays' r_u, r_l too), which takes 30 of
// every 31 record loads and stores off the HBM stream.  The values read back are the same bits.
constexpr int kUniBeta = 4, kUniRu = 8, kUniRl = 16;      // VolRecords::flags
constexpr int kShUniLd = 1, kShUniRu = 2, kShUniRl = 4;   // VolState::shFlags
// kShRgb (grey media only): shLd rows 0-2 hold the sensor-weighted sums sum_i xyz_bar(l_i) Ld_i
// and row 3 holds Ld_0, so the grey shadow kernel scales four values by T_ray / avg instead of
// reading 31.  Linear, as pbrt's film conversion of L is; the rounding order differs from the
// per-wavelength form by float ulps (parity: within the tests' 1e-3 tolerance).
constexpr int kShRgb = 8;
__device__ inline void LoadSpec(const float *base, int NR, int ri, float v[kNS], bool uni = false) {
    if (uni) {
        const float x = base[ri];
#pragma unroll
        for (int i = 0; i < kNS; ++i) v[i] = x;
        return;
    }
#pragma unroll
    for (int i = 0; i < kNS; ++i) v[i] = base[(size_t)i * NR + ri];
}
__device__ inline bool AllEqual(const float v[kNS]) {
    bool eq = true;
#pragma unroll
    for (int i = 1; i < kNS; ++i) eq &= FloatToBits(v[i]) == FloatToBits(v[0]);
    return eq;
}
// Stores v (uniform when all 31 entries have the same bits); returns whether it did so
__device__ inline bool StoreSpec(float *base, int NR, int ri, const float v[kNS]) {
    const bool uni = AllEqual(v);
    if (uni) {
        base[ri] = v[0];
        return true;
    }
#pragma unroll
    for (int i = 0; i < kNS; ++i) base[(size_t)i * NR + ri] = v[i];
    return false;
}
// Entry i of a possibly-uniform record spectrum: entry 0 preloaded, the rest loaded only for
// non-uniform spectra (lanes with uniform ones skip the load)
struct SpecIn {
    const float *p;
    int NR;
    bool uni;
    float v0;
    __device__ SpecIn(const float *base, int NR_, int ri, bool u) : p(base + ri), NR(NR_), uni(u) { v0 = p[0]; }
    __device__ float operator()(int i) const {
        float x = v0;
        if (!uni && i > 0) x = p[(size_t)i * NR];
        return x;
    }
};
__device__ inline V3 LoadV3(const float *base, int NR, int ri) {
    return V3(base[ri], base[NR + ri], base[2 * (size_t)NR + ri]);
}
__device__ inline void StoreV3(float *base, int NR, int ri, V3 v) {
    base[ri] = v.x;
    base[NR + ri] = v.y;
    base[2 * (size_t)NR + ri] = v.z;
}

// Medium on each side of a leaf-order triangle, or the ray's medium when the triangle is no
// medium boundary (SurfaceInteraction::SetIntersectionProperties, interaction.h:236-248)
__device__ inline void MediaOf(const DeviceScene &S, int prim, int rayMedium, int *in, int *out) {
    *in = *out = rayMedium;
    if (S.media.primMedium) {
        const int a = S.media.primMedium[2 * prim], b = S.media.primMedium[2 * prim + 1];
        if (a != b) {
            *in = a;
            *out = b;
        }
    }
}

// ------------------------------------------------------------------ kernels
__global__ void __launch_bounds__(kBlock) k_vcamera(DeviceScene S, PathState st, VolState v, int nActive) {
    const int slot = blockIdx.x * blockDim.x + threadIdx.x;
    if (slot == 0) {
        st.counters[CounterIndex(0, kVRay, 0)] = nActive;  // iteration-0 records = every slot
        atomicAdd(&st.stats[0], (unsigned long long)nActive);
    }
    if (slot >= nActive) return;
    float lambda0;
    V3 o, d;
    float filterWeight;
    uint32_t sidx;
    GenerateCameraRay(S, st, slot, &lambda0, &o, &d, &filterWeight, &sidx);
    const int NR = st.NR, N = st.N;
    st.L[slot] = 0;
    st.L[N + slot] = 0;
    st.L[2 * N + slot] = 0;
    if (S.dispersive) {
        st.L0[slot] = 0;
        st.L0[N + slot] = 0;
        st.L0[2 * N + slot] = 0;
        st.lamTerm[slot] = 0;
    }
    if (!S.boxFilter) st.filterW[slot] = filterWeight;
    const VolRecords &r = v.rec[0];
    r.beta[slot] = 1.f;  // uniform spectra: entry 0 only (kUni* flags)
    r.ru[slot] = 1.f;
    r.rl[slot] = 1.f;
    StoreV3(r.ray, NR, slot, o);
    StoreV3(r.ray + 3 * (size_t)NR, NR, slot, d);
#pragma unroll
    for (int k = 0; k < 12; ++k) r.prev[(size_t)k * NR + slot] = 0.f;
    r.lambda0[slot] = lambda0;
    r.etaScale[slot] = 1.f;
    r.flags[slot] = kUniBeta | kUniRu | kUniRl;
    r.pixel[slot] = slot;
    r.depth[slot] = 0;
    r.medium[slot] = S.media.cameraMedium;
}

// The material record ri's closest hit shades with: its primitive's, or with mix materials the
// one k_vclosest<TM, true> chose (MixMaterial::ChooseMaterial at the hit, intersect.h:90-97)
__device__ inline int VolHitMaterial(const DeviceScene &S, const PathState &st, int ri, int prim) {
    return st.hitMat[0] ? st.hitMat[0][ri] : S.primMaterial[prim];
}
// a surface hit on Material "interface" (type 3): the ray only changes medium (k_viface)
__device__ inline bool IsInterfaceHit(const DeviceScene &S, const PathState &st, int ri, int prim) {
    return prim >= 0 && S.matType[VolHitMaterial(S, st, ri, prim)] == 3;
}

// Mix: the scene has mix materials, resolved per hit into st.hitMat[0] (an out-of-line call,
// compiled into these instantiations only)
template <int TM, bool Mix = false>
__global__ void __launch_bounds__(kBlock, TraversalWaves(TM)) k_vclosest(DeviceScene S, PathState st, VolState v,
                                                                          int wf, int timed) {
    const QueueView rays = LoadQueue(st, wf, kVRay);
    ChunkWalk walk = XcdChunks(rays.total, S.xcdGroups);
    if (walk.n >= walk.end) return;
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1];
    const int shard = ProducerShard();
    int *medCnt = &st.counters[CounterIndex(wf, kVMed, shard)];
    int *surfCnt = &st.counters[CounterIndex(wf, kVSurf, shard)];
    int *ifaceCnt = &st.counters[CounterIndex(wf, kVIface, shard)];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&st.stats[1], (unsigned long long)rays.total);
        if (timed) atomicAdd(&st.stats[3], (unsigned long long)rays.total);  // rays of event-timed launches
    }
    for (; walk.n < walk.end; walk.n += walk.step) {
        const int j = walk.Chunk() * blockDim.x + threadIdx.x;
        const bool active = j < rays.total;
        const int ri = active ? QueueSlot(rays, j) : 0;
        int medium = -1;
        bool iface = false, esc = false;
        if (active) {
            const V3 o = LoadV3(rec.ray, NR, ri), d = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
            TriHit h;
            const int prim = Traverse<false, TM>(S, L, o, d, kInfinity, &h);
            v.hitPrim[ri] = prim;
            v.hitB[ri] = h.b0;
            v.hitB[NR + ri] = h.b1;
            v.hitB[2 * NR + ri] = h.b2;
            v.hitB[3 * NR + ri] = prim >= 0 ? h.t : kInfinity;
            if constexpr (Mix) {
                if (prim >= 0) {
                    int mat = S.primMaterial[prim];
                    if (S.matType[mat] == kMatMixT) mat = ResolveMixMaterial(*S.self, prim, mat, h.b0, h.b1, h.b2, d);
                    st.hitMat[0][ri] = mat;
                }
            }
            medium = rec.medium[ri];
            iface = medium < 0 && IsInterfaceHit(S, st, ri, prim);
            esc = medium < 0 && prim < 0;
        }
        // rays inside a medium sample it first (MediumSampleQueue), the rest go to the surface
        // (interface crossings and escaped rays to their own queues)
        const int pm = WavePush(medCnt, active && medium >= 0);
        const int ps = WavePush(surfCnt, active && medium < 0 && !iface && !esc);
        const int pf = WavePush(ifaceCnt, active && iface);
        const int pe = WavePush(&st.counters[CounterIndex(wf, kVEsc, shard)], active && esc);
        if (pm >= 0 && pm < st.capS) v.medQ[shard * st.capS + pm] = ri;
        if (ps >= 0 && ps < st.capS) v.surfQ[shard * st.capS + ps] = ri;
        if (pf >= 0 && pf < st.capS) v.ifaceQ[shard * st.capS + pf] = ri;
        if (pe >= 0 && pe < st.capS) v.escQ[shard * st.capS + pe] = ri;
    }
}

// SampleMediumInteraction (media.cpp:22-247)
__global__ void __launch_bounds__(kBlock, PBRT_VOL_WAVES) k_vmedium(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView meds = LoadQueue(st, wf, kVMed);
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1];
    const int shard = ProducerShard();
    int *surfCnt = &st.counters[CounterIndex(wf, kVSurf, shard)];
    int *scatCnt = &st.counters[CounterIndex(wf, kVScat, shard)];
    for (int base = blockIdx.x * blockDim.x; base < meds.total; base += gridDim.x * blockDim.x) {
        const int j = base + threadIdx.x;
        const bool active = j < meds.total;
        const int ri = active ? v.medQ[QueueSlot(meds, j)] : 0;
        bool toSurf = false, toScat = false;
        if (active) {
            const V3 o = LoadV3(rec.ray, NR, ri), d = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
            const float tHit = v.hitB[3 * NR + ri];
            const int depth = rec.depth[ri], slot = rec.pixel[ri];
            const MediumRef m = MediumAt(S, rec.medium[ri]);
            const WaveOffsets wo(rec.lambda0[ri]);
            const int inFlags = rec.flags[ri];
            float beta[kNS], ru[kNS], rl[kNS], Tm[kNS];
            LoadSpec(rec.beta, NR, ri, beta, inFlags & kUniBeta);
            LoadSpec(rec.ru, NR, ri, ru, inFlags & kUniRu);
            LoadSpec(rec.rl, NR, ri, rl, inFlags & kUniRl);
            PCG32 rng(HashV3F(o, tHit), HashV3(d));
            const float uDist = rng.Uniform();
            float uMode = rng.Uniform();
            bool scattered = false, pushScatter = false;
            V3 pS(0, 0, 0);
            float Lx = 0, Ly = 0, Lz = 0;
            bool emitted = false;
            const int sa = m.I[1], ss = m.I[2], le = m.I[3];
            const bool maxD = depth >= S.maxDepth;
            auto event = [&](V3 p, const MediumPoint &mp, float mx, const float *T) __attribute__((always_inline)) -> bool {
                const float smaj0 = (DenseAt(S, sa, wo.off[0]) + DenseAt(S, ss, wo.off[0])) * mx;
                const float sa0 = MediumSigmaA(S, m, mp, wo.off[0], wo.lam0), ss0 = MediumSigmaS(S, m, mp, wo.off[0], wo.lam0);
                // medium emission, scaled by sigma_a / sigma_maj at every event (media.cpp:70-83)
                if (!maxD && mp.le != 0) {
                    bool leNz = false;
                    SpectralIter il(wo.lam0);
#pragma unroll
                    for (int i = 0; i < kNS; ++i, il.Next()) leNz |= MediumLe(S, m, mp, wo.off[i], il.lam) != 0;
                    if (leNz) {
                        const float pr = smaj0 * T[0];
                        float re[kNS];
#pragma unroll
                        for (int i = 0; i < kNS; ++i) {
                            const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                            re[i] = ru[i] * smaj * T[i] / pr;
                        }
                        if (AnyNonZero(re)) {
                            const float den = pr * AvgArr(re);
                            SensorAcc acc;
                            SpectralIter it(wo.lam0);
#pragma unroll
                            for (int i = 0; i < kNS; ++i, it.Next()) {
                                const float sai = MediumSigmaA(S, m, mp, wo.off[i], it.lam);
                                const float Le = MediumLe(S, m, mp, wo.off[i], it.lam);
                                acc.Add(S, wo.off[i], beta[i] * sai * T[i] * Le / den, i == 0);
                            }
                            Lx += S.imagingRatio * (acc.sx / kNS);
                            Ly += S.imagingRatio * (acc.sy / kNS);
                            Lz += S.imagingRatio * (acc.sz / kNS);
                            emitted = true;
                        }
                    }
                }
                const float pAbsorb = sa0 / smaj0, pScatter = ss0 / smaj0;
                const float pNull = fmaxf(0.f, 1 - pAbsorb - pScatter);
                const int mode = SampleDiscrete3(pAbsorb, pScatter, pNull, uMode);
                if (mode == 0) {
#pragma unroll
                    for (int i = 0; i < kNS; ++i) beta[i] = 0.f;
                    return false;
                }
                if (mode == 1) {
                    const float pr = T[0] * ss0;
                    SpectralIter it(wo.lam0);
#pragma unroll
                    for (int i = 0; i < kNS; ++i, it.Next()) {
                        const float f = T[i] * MediumSigmaS(S, m, mp, wo.off[i], it.lam) / pr;
                        beta[i] *= f;
                        ru[i] *= f;
                    }
                    pushScatter = AnyNonZero(beta) && AnyNonZero(ru);
                    pS = p;
                    scattered = true;
                    return false;
                }
                // null scattering
                float sn0 = 0;
                float sn[kNS];
                SpectralIter it(wo.lam0);
#pragma unroll
                for (int i = 0; i < kNS; ++i, it.Next()) {
                    const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                    sn[i] = fmaxf(0.f, smaj - MediumSigmaA(S, m, mp, wo.off[i], it.lam) - MediumSigmaS(S, m, mp, wo.off[i], it.lam));
                }
                sn0 = sn[0];
                const float pr = T[0] * sn0;
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    const float smaj = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                    const float f = T[i] * sn[i] / pr;
                    beta[i] = pr == 0 ? 0.f : beta[i] * f;
                    ru[i] *= f;
                    rl[i] *= T[i] * smaj / pr;
                }
                uMode = rng.Uniform();
                return AnyNonZero(beta) && AnyNonZero(ru);
            };
            const bool ranOut = SampleTmaj(S, m, wo, o, d, tHit, uDist, rng, Tm, event);
            if (emitted) {
                st.L[slot] += Lx;
                st.L[st.N + slot] += Ly;
                st.L[2 * st.N + slot] += Lz;
            }
            if (!scattered && AnyNonZero(beta) && ranOut) {
                // beta, r_u, r_l *= T_maj / T_maj[0] (a stopped traversal returns T_maj = 1)
                const float t0 = Tm[0];
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    const float f = Tm[i] / t0;
                    beta[i] *= f;
                    ru[i] *= f;
                    rl[i] *= f;
                }
            }
            if (scattered) {
                if (pushScatter) {
                    int fl = inFlags & ~(kUniBeta | kUniRu);
                    fl |= StoreSpec(rec.beta, NR, ri, beta) ? kUniBeta : 0;
                    fl |= StoreSpec(rec.ru, NR, ri, ru) ? kUniRu : 0;
                    rec.flags[ri] = fl;
                    StoreV3(v.hitB, NR, ri, pS);  // the scattering point replaces the hit
                    toScat = true;
                }
            } else if (AnyNonZero(beta) && AnyNonZero(ru) && depth != S.maxDepth) {
                int fl = inFlags & ~(kUniBeta | kUniRu | kUniRl);
                fl |= StoreSpec(rec.beta, NR, ri, beta) ? kUniBeta : 0;
                fl |= StoreSpec(rec.ru, NR, ri, ru) ? kUniRu : 0;
                fl |= StoreSpec(rec.rl, NR, ri, rl) ? kUniRl : 0;
                rec.flags[ri] = fl;
                toSurf = true;
            }
        }
        const int hp = toSurf ? v.hitPrim[ri] : 0;
        const bool iface = toSurf && IsInterfaceHit(S, st, ri, hp), esc = toSurf && hp < 0;
        const int p0 = WavePush(surfCnt, toSurf && !iface && !esc);
        const int p1 = WavePush(scatCnt, toScat);
        const int p2 = WavePush(&st.counters[CounterIndex(wf, kVIface, shard)], iface);
        const int p3 = WavePush(&st.counters[CounterIndex(wf, kVEsc, shard)], esc);
        if (p0 >= 0 && p0 < st.capS) v.surfQ[shard * st.capS + p0] = ri;
        if (p1 >= 0 && p1 < st.capS) v.scatQ[shard * st.capS + p1] = ri;
        if (p2 >= 0 && p2 < st.capS) v.ifaceQ[shard * st.capS + p2] = ri;
        if (p3 >= 0 && p3 < st.capS) v.escQ[shard * st.capS + p3] = ri;
    }
}

// SampleMediumInteraction for scenes whose media are all grey (DeviceMedia::allGrey): every
// T_maj / sigma product is a scalar.  The factors that multiply beta and r_u are then
// (T sigma) / (T[0] sigma[0]) = x / x -- exactly 1 unless x is 0 (the path dies) -- so beta and
// r_u stay in memory and only a scalar record of any non-unit factor is kept; r_l takes
// T sigma_maj / pr per null collision, applied in the reference's order to its (spectrally
// constant, checked) value.  No 31-wide array lives through the tracking loop.
template <bool Cloud>
__global__ void __launch_bounds__(kBlock, PBRT_VOL_GREY_WAVES) k_vmedium_grey(DeviceScene S, PathState st, VolState v,
                                                                            int wf) {
    const QueueView meds = LoadQueue(st, wf, kVMed);
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1];
    const int shard = ProducerShard();
    int *surfCnt = &st.counters[CounterIndex(wf, kVSurf, shard)];
    int *scatCnt = &st.counters[CounterIndex(wf, kVScat, shard)];
    for (int base = blockIdx.x * blockDim.x; base < meds.total; base += gridDim.x * blockDim.x) {
        const int j = base + threadIdx.x;
        const bool active = j < meds.total;
        const int ri = active ? v.medQ[QueueSlot(meds, j)] : 0;
        bool toSurf = false, toScat = false;
        if (active) {
            const V3 o = LoadV3(rec.ray, NR, ri), d = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
            const float tHit = v.hitB[3 * NR + ri];
            const int depth = rec.depth[ri], slot = rec.pixel[ri];
            const MediumRef m = MediumAt(S, rec.medium[ri]);
            const float lambda0 = rec.lambda0[ri];
            const int off0 = DenseOffset(lambda0);
            const int sa = m.I[1], ss = m.I[2], le = m.I[3];
            const float sa0 = DenseAt(S, sa, off0), ss0 = DenseAt(S, ss, off0);
            // beta, r_u nonzero?  r_l spectrally constant?  (uniform records: one value each)
            const int inFlags = rec.flags[ri];
            const bool betaUni = inFlags & kUniBeta, ruUni = inFlags & kUniRu, rlUni = inFlags & kUniRl;
            const SpecIn betaIn(rec.beta, NR, ri, betaUni), ruIn(rec.ru, NR, ri, ruUni), rlIn(rec.rl, NR, ri, rlUni);
            bool betaNz = betaIn.v0 != 0, ruNz = ruIn.v0 != 0, rlFlat = true;
            const float rl0 = rlIn.v0;
            if (!betaUni || !ruUni || !rlUni) {
#pragma unroll 4
                for (int i = 1; i < kNS; ++i) {
                    betaNz |= betaIn(i) != 0;
                    ruNz |= ruIn(i) != 0;
                    rlFlat &= rlIn(i) == rl0;
                }
            }
            float fb = 1.f;     // product of the (non-unit) beta / r_u factors
            float rlS = rl0;    // r_l when spectrally constant (exact)
            float gl = 1.f;     // product of the r_l factors otherwise
            bool fbZero = false;
            PCG32 rng(HashV3F(o, tHit), HashV3(d));
            const float uDist = rng.Uniform();
            float uMode = rng.Uniform();
            bool scattered = false, pushScatter = false;
            V3 pS(0, 0, 0);
            float Lx = 0, Ly = 0, Lz = 0;
            bool emitted = false;
            const bool maxD = depth >= S.maxDepth;
            auto mulBeta = [&](float f) __attribute__((always_inline)) {
                if (f != 1.f) {
                    fb *= f;
                    fbZero |= f == 0;
                }
            };
            auto event = [&](V3 p, const MediumPoint &mp, float smaj, float T) __attribute__((always_inline)) -> bool {
                const float sad = sa0 * mp.d, ssd = ss0 * mp.d;
                if (!maxD && mp.le != 0) {
                    // medium emission (media.cpp:70-83); Le may be chromatic.  Two rolled passes
                    // over the wavelengths (sum of r_e, then the sensor sums): no 31-wide arrays.
                    const float pr = smaj * T;
                    bool leNz = false, reNz = false;
                    float reSum = 0;
                    {
                        SpectralIter it(lambda0);
#pragma unroll 1
                        for (int i = 0; i < kNS; ++i, it.Next()) {
                            leNz |= DenseAt(S, le, DenseOffset(it.lam)) * mp.le != 0;
                            float ru = ruIn(i);
                            if (fb != 1.f) ru *= fb;
                            const float re = ru * smaj * T / pr;
                            reNz |= re != 0;
                            reSum = i == 0 ? re : reSum + re;
                        }
                    }
                    if (leNz && reNz) {
                        const float den = pr * (reSum / kNS);
                        SensorAcc acc;
                        SpectralIter it(lambda0);
#pragma unroll 1
                        for (int i = 0; i < kNS; ++i, it.Next()) {
                            const int off = DenseOffset(it.lam);
                            float b = betaIn(i);
                            if (fb != 1.f) b *= fb;
                            const float Le = DenseAt(S, le, off) * mp.le;
                            acc.Add(S, off, b * sad * T * Le / den, i == 0);
                        }
                        Lx += S.imagingRatio * (acc.sx / kNS);
                        Ly += S.imagingRatio * (acc.sy / kNS);
                        Lz += S.imagingRatio * (acc.sz / kNS);
                        emitted = true;
                    }
                }
                const float pAbsorb = sad / smaj, pScatter = ssd / smaj;
                const float pNull = fmaxf(0.f, 1 - pAbsorb - pScatter);
                const int mode = SampleDiscrete3(pAbsorb, pScatter, pNull, uMode);
                if (mode == 0) {
                    betaNz = false;  // absorbed
                    return false;
                }
                if (mode == 1) {
                    const float pr = T * ssd;
                    mulBeta(T * ssd / pr);
                    pushScatter = betaNz && !fbZero && ruNz;
                    pS = p;
                    scattered = true;
                    return false;
                }
                const float sn = fmaxf(0.f, smaj - sad - ssd);
                const float pr = T * sn;
                mulBeta(T * sn / pr);
                if (pr == 0) betaNz = false;
                const float g = T * smaj / pr;
                rlS *= g;
                gl *= g;
                uMode = rng.Uniform();
                return betaNz && !fbZero && ruNz;
            };
            float Tm;
            const bool ranOut = SampleTmajGrey<Cloud>(S, m, sa0 + ss0, o, d, tHit, uDist, rng, Tm, event);
            if (emitted) {
                st.L[slot] += Lx;
                st.L[st.N + slot] += Ly;
                st.L[2 * st.N + slot] += Lz;
            }
            if (!scattered && betaNz && !fbZero && ranOut) {
                const float f = Tm / Tm;  // T_maj / T_maj[0]: 1, or NaN as the reference's for 0 / inf
                mulBeta(f);
                rlS *= f;
                gl *= f;
            }
            const bool alive = betaNz && !fbZero;
            // write back only what changed (a non-unit beta / r_u factor is rare: x / x == 1)
            auto scaleBetaRu = [&]() __attribute__((always_inline)) {
                if (fb == 1.f) return;
                for (int i = 0; i < (betaUni ? 1 : kNS); ++i) rec.beta[(size_t)i * NR + ri] *= fb;
                for (int i = 0; i < (ruUni ? 1 : kNS); ++i) rec.ru[(size_t)i * NR + ri] *= fb;
            };
            if (scattered) {
                if (pushScatter) {
                    scaleBetaRu();
                    StoreV3(v.hitB, NR, ri, pS);
                    toScat = true;
                }
            } else if (alive && ruNz && depth != S.maxDepth) {
                scaleBetaRu();
                if (rlFlat) {
                    // r_l keeps one value: exact for every wavelength, stored uniform
                    if (rlS != rl0 || !rlUni) rec.rl[ri] = rlS;
                    if (!rlUni) rec.flags[ri] = inFlags | kUniRl;
                } else {
#pragma unroll 1
                    for (int i = 0; i < kNS; ++i) rec.rl[(size_t)i * NR + ri] *= gl;
                }
                toSurf = true;
            }
        }
        const int hp = toSurf ? v.hitPrim[ri] : 0;
        const bool iface = toSurf && IsInterfaceHit(S, st, ri, hp), esc = toSurf && hp < 0;
        const int p0 = WavePush(surfCnt, toSurf && !iface && !esc);
        const int p1 = WavePush(scatCnt, toScat);
        const int p2 = WavePush(&st.counters[CounterIndex(wf, kVIface, shard)], iface);
        const int p3 = WavePush(&st.counters[CounterIndex(wf, kVEsc, shard)], esc);
        if (p0 >= 0 && p0 < st.capS) v.surfQ[shard * st.capS + p0] = ri;
        if (p1 >= 0 && p1 < st.capS) v.scatQ[shard * st.capS + p1] = ri;
        if (p2 >= 0 && p2 < st.capS) v.ifaceQ[shard * st.capS + p2] = ri;
        if (p3 >= 0 && p3 < st.capS) v.escQ[shard * st.capS + p3] = ri;
    }
}

struct ShadowOut {
    V3 o, d;
    int medium;
};
// S: the scene, for grey media (kShRgb: Ld as its sensor sums + Ld_0)
__device__ inline void WriteShadow(const DeviceScene &S, const VolState &v, int NR, int j, const ShadowOut &s,
                                   const float *Ld, const float *ru, const float *rl, float lambda0, int slot) {
    StoreV3(v.shRay, NR, j, s.o);
    StoreV3(v.shRay + 3 * (size_t)NR, NR, j, s.d);
    int fl;
    if (S.media.allGrey) {
        SensorAcc acc;
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNS; ++i, it.Next()) acc.Add(S, DenseOffset(it.lam), Ld[i], i == 0);
        v.shLd[j] = acc.sx;
        v.shLd[NR + j] = acc.sy;
        v.shLd[2 * (size_t)NR + j] = acc.sz;
        v.shLd[3 * (size_t)NR + j] = Ld[0];
        fl = kShRgb;
    } else {
        fl = StoreSpec(v.shLd, NR, j, Ld) ? kShUniLd : 0;
    }
    fl |= StoreSpec(v.shRu, NR, j, ru) ? kShUniRu : 0;
    fl |= StoreSpec(v.shRl, NR, j, rl) ? kShUniRl : 0;
    v.shFlags[j] = fl;
    v.shLambda0[j] = lambda0;
    v.shPixel[j] = slot;
    v.shMedium[j] = s.medium;
}

// One area light sample for a reference point (BVHLightSampler::Sample + DiffuseAreaLight::SampleLi
// with allowIncompletePDF, lights.cpp:743-775): false when no light / no sample / Le = 0
// Point, spot and distant lights take the same route through SampleLiSurface (common.h): pdf 1,
// a light point without error or normal, radiance scale * I(lambda) [/ d2]; delta is set.
struct AreaLightSample {
    int light;
    V3 p, pErr, n, wi;
    float pdf;  // shape pdf * light-choice pmf
    bool delta;
};
// Ext: analytic-shape emitters and image lights are possible (the kernels' Ext)
template <bool Ext>
__device__ inline bool SampleAreaLight(const DeviceScene &S, V3 refP, V3 refN, V3 refNs, float uc, float u0, float u1,
                                       float lambda0, const WaveOffsets &wo, AreaLightSample *out, float Le[kNS]) {
    int li;
    float lpmf;
    if (!SampleLight(S, refP, refNs, uc, &li, &lpmf)) return false;
    // lights other than plain emitting triangles -- and image emitters, whose radiance is the
    // image at the sample's uv -- through SampleLiSurface (common.h)
    if (li >= S.nAreaLights || (Ext && S.nShapes > 0 && __float_as_int(S.lights[li].v0.w) >= S.nTris) ||
        (Ext && S.nImageAreaLights > 0 && S.lightImgOff[li] >= 0)) {
        LiSample ls;
        if (!SampleLiSurface<false, false, Ext>(S, S.lights, li, refP, refN, refNs, u0, u1, &ls)) return false;
        const float rd2 = 1 / ls.d2;
        const bool ok = DivFastOk(ls.d2);
        bool nz = false;
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNS; ++i, it.Next()) {
            Le[i] = DivByRcp(ls.Le(DenseAt(S, ls.spectrum, wo.off[i]), it.lam), ls.d2, rd2, ok);
            nz |= Le[i] != 0;
        }
        if (!nz) return false;
        out->light = li;
        out->p = ls.lp;
        out->pErr = ls.lpe;
        out->n = ls.ln;
        out->wi = ls.wi;
        out->pdf = ls.pdf * lpmf;
        out->delta = ls.delta;  // an ImageInfiniteLight sample is not a delta light
        return true;
    }
    const DeviceAreaLight Ld = S.lights[li];
    const V3 q0(Ld.v0.x, Ld.v0.y, Ld.v0.z), q1(Ld.v1.x, Ld.v1.y, Ld.v1.z), q2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
    TriShading lsh;
    const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
    V3 lp, lpe, ln;
    float lpdf;
    if (!SampleTriangle(q0, q1, q2, Ld.flip, lhas ? &lsh : nullptr, refP, refN, refNs, u0, u1, &lp, &lpe, &ln, &lpdf) ||
        lpdf == 0 || LengthSquared(lp - refP) == 0)
        return false;
    const V3 wi = Normalize(lp - refP);
    bool nz = false;
    const bool facing = (Ld.twoSided || DotN(ln, -wi) >= 0) && !SpreadCut(Ld.v1.w, ln, -wi);
    // the spread's falloff multiplies L (lights.cpp:763-771); 1 without a spread
    const float k = Ld.v1.w > 0 ? SpreadFactor(Ld.v2.w, S.lightSpreadNorm[li], ln, wi) : 1.f;
#pragma unroll
    for (int i = 0; i < kNS; ++i) {
        Le[i] = facing ? (Ld.scale * DenseAt(S, Ld.spectrum, wo.off[i])) * k : 0.f;
        nz |= Le[i] != 0;
    }
    if (!nz) return false;
    out->light = li;
    out->p = lp;
    out->pErr = lpe;
    out->n = ln;
    out->wi = wi;
    out->pdf = lpdf * lpmf;
    out->delta = false;
    return true;
}


// Spectral contribution c(i, off) of the path's 31 wavelengths to sensor RGB, added to the
// slot's L (film.h:95-100).  Rolled: the terms stream from the wavelength-major records.
template <typename C>
__device__ inline void AddSpecToL(const DeviceScene &S, const PathState &st, int slot, float lambda0, C &&c) {
    SensorAcc acc;
    SpectralIter it(lambda0);
    float c0 = 0;
#pragma unroll 4
    for (int i = 0; i < kNS; ++i, it.Next()) {
        const int off = DenseOffset(it.lam);
        const float ci = c(i, off);
        c0 = i == 0 ? ci : c0;
        acc.Add(S, off, ci, i == 0);
    }
    const int NL = st.N;
    st.L[slot] += S.imagingRatio * (acc.sx / kNS);
    st.L[NL + slot] += S.imagingRatio * (acc.sy / kNS);
    st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNS);
    AddL0Off(S, st, slot, DenseOffset(lambda0), c0);
}

// An area-light sample for a reference point (BVHLightSampler::Sample, then
// DiffuseAreaLight::SampleLi with allowIncompletePDF, lights.cpp:743-775); false when no light,
// no sample, or Le = 0 at every wavelength.  Le_i = scale * dense[spectrum][off_i] when facing.
// Point, spot and distant lights through SampleLiSurface as well: Le(off) divides by d2 (1 for
// area and distant lights: an exact no-op), and a delta light has no BSDF MIS weight.
struct AreaLightHit {
    V3 p, pErr, n, wi;
    float pdf;  // shape pdf * light-choice pmf
    float scale;
    int spectrum;
    float d2, rd2;
    bool d2Ok, delta;
    bool envLe;  // ImageInfiniteLight / ProjectionLight: the pixel's RGBIlluminantSpectrum (EnvLe)
    EnvCoef env;
    float k;     // GoniometricLight: the image value (1 otherwise)
    __device__ float Le(const DeviceScene &S, int off, float lam) const {
        const float dv = DenseAt(S, spectrum, off);
        const float v = (envLe ? EnvLe(env, scale, dv, lam) : scale * dv) * k;
        return delta ? DivByRcp(v, d2, rd2, d2Ok) : v;
    }
};
template <bool Ext>
__device__ inline bool SampleAreaLightAt(const DeviceScene &S, V3 refP, V3 refN, V3 refNs, float uc, float u0, float u1,
                                         float lambda0, AreaLightHit *out, V3 refErr = V3(0, 0, 0)) {
    int li;
    float lpmf;
    if (!SampleLight(S, refP, refNs, uc, &li, &lpmf)) return false;
    if (li >= S.nAreaLights || (Ext && S.nShapes > 0 && __float_as_int(S.lights[li].v0.w) >= S.nTris) ||
        (Ext && S.nImageAreaLights > 0 && S.lightImgOff[li] >= 0)) {
        LiSample ls;
        if (!SampleLiSurface<false, false, Ext>(S, S.lights, li, refP, refN, refNs, u0, u1, &ls, refErr)) return false;
        out->p = ls.lp;
        out->pErr = ls.lpe;
        out->n = ls.ln;
        out->wi = ls.wi;
        out->pdf = ls.pdf * lpmf;
        out->scale = ls.scale;
        out->spectrum = ls.spectrum;
        out->d2 = ls.d2;
        out->rd2 = 1 / ls.d2;
        out->d2Ok = DivFastOk(ls.d2);
        out->delta = ls.delta;
        out->envLe = ls.envLe;
        out->env = ls.env;
        out->k = ls.k;
        bool nz = false;
        SpectralIter it(lambda0);
#pragma unroll 1
        for (int i = 0; i < kNS; ++i, it.Next()) nz |= out->Le(S, DenseOffset(it.lam), it.lam) != 0;
        return nz;
    }
    const DeviceAreaLight Ld = S.lights[li];
    const V3 q0(Ld.v0.x, Ld.v0.y, Ld.v0.z), q1(Ld.v1.x, Ld.v1.y, Ld.v1.z), q2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
    TriShading lsh;
    const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
    V3 lp, lpe, ln;
    float lpdf;
    if (!SampleTriangle(q0, q1, q2, Ld.flip, lhas ? &lsh : nullptr, refP, refN, refNs, u0, u1, &lp, &lpe, &ln, &lpdf) ||
        lpdf == 0 || LengthSquared(lp - refP) == 0)
        return false;
    const V3 wi = Normalize(lp - refP);
    if (!(Ld.twoSided || DotN(ln, -wi) >= 0)) return false;  // L() = 0 on the back side
    if (SpreadCut(Ld.v1.w, ln, -wi)) return false;            // outside the spread
    const float k = Ld.v1.w > 0 ? SpreadFactor(Ld.v2.w, S.lightSpreadNorm[li], ln, wi) : 1.f;
    bool nz = false;
    SpectralIter it(lambda0);
#pragma unroll 1
    for (int i = 0; i < kNS; ++i, it.Next()) nz |= (Ld.scale * DenseAt(S, Ld.spectrum, DenseOffset(it.lam))) * k != 0;
    if (!nz) return false;
    out->p = lp;
    out->pErr = lpe;
    out->n = ln;
    out->wi = wi;
    out->pdf = lpdf * lpmf;
    out->scale = Ld.scale;
    out->spectrum = Ld.spectrum;
    out->d2 = out->rd2 = 1;
    out->d2Ok = true;
    out->delta = false;
    out->envLe = false;
    out->k = k;
    return true;
}

// Per-block LDS copies of the tables the spectral loops read per wavelength: the sensor's
// x/y/z curves and (when they fit, DeviceMedia::denseInLds) every dense spectrum.  The
// kernel's scene copy is repointed at them, so DenseAt / SensorAcc read LDS.
__device__ inline char *StageVolTables(const DeviceScene &S0, DeviceScene &S, char *lds) {
    float4 *sensorL = reinterpret_cast<float4 *>(lds);
    DmaCopy<16>(S0.sensor4, sensorL, kDenseN);
    char *next = lds + kDenseN * 16;
    if (S0.media.denseInLds) {
        DmaCopy<4>(S0.dense, next, S0.nDense * kDenseN);
        S.dense = reinterpret_cast<const float *>(next);
        next += ((S0.nDense * kDenseN * 4 + 15) & ~15);
    }
    S.sensor4 = sensorL;
    DmaWait();
    __syncthreads();
    return next;
}
size_t VolTablesLdsBytes(const DeviceScene &S) {
    return kDenseN * 16 + (S.media.denseInLds ? ((S.nDense * kDenseN * 4 + 15) & ~15) : 0);
}

#ifndef PBRT_VOL_SURF_WAVES
#define PBRT_VOL_SURF_WAVES 3  // waves/SIMD of k_vsurface
#endif

// The texture stage of the volumetric surface queue (EvaluateMaterialAndBSDF's texEval calls
// and bump / normal mapping, surfscatter.cpp:74-137), as k_texture on the surface path: per
// surface hit of this iteration the results k_vsurface<..., Tex> reads (HitTextures).
template <bool Ext, bool Hair = false>
__global__ void __launch_bounds__(kBlock) k_vtexture(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView surf = LoadQueue(st, wf, kVSurf);
    if ((int)(blockIdx.x * blockDim.x) >= surf.total) return;
    __shared__ float zLds[64];
    __shared__ float lutLds[kTexLdsLuts * 256];
    const int nLut = S.tex.nLuts <= kTexLdsLuts ? S.tex.nLuts : 0;
    for (int i = threadIdx.x; i < 64; i += blockDim.x) zLds[i] = S.tex.rgbZNodes[i];
    for (int i = threadIdx.x; i < nLut * 256; i += blockDim.x) lutLds[i] = S.tex.luts[i];
    __syncthreads();
    S.tex.rgbZNodes = zLds;
    if (nLut) S.tex.luts = lutLds;
    const VolRecords &rec = v.rec[wf & 1];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < surf.total; j += gridDim.x * blockDim.x) {
        const int ri = v.surfQ[QueueSlot(surf, j)];
        const int prim = v.hitPrim[ri];
        if (prim < 0) continue;  // escaped
        const int mat = VolHitMaterial(S, st, ri, prim);
        if (S.matType[mat] == 3) continue;  // interfaces
        HitTextures<true, Ext, Hair>(S, st, wf, ri, prim, mat, v.hitB, rec.lambda0);
    }
}

// The surface side of an iteration: escaped rays, interfaces, emission, materials.  Spectral
// quantities stream from the wavelength-major records in rolled loops; the one 31-wide
// intermediate (f, then beta') lives in LDS ([31][kBlock], conflict-free).  Queue appends happen
// where a lane decides to push (WavePush serves the lanes that reach it).  DiffuseOnly: the
// scene's surface materials are diffuse, interface or layered (k_vlayered) only, so the
// dielectric / conductor code is compiled out (C5: fewer registers, no spills).  Tex: some
// material is textured or bump mapped; k_vtexture left this iteration's texture results per
// record (HitTextures), read here as the surface path's shade kernels read k_texture's.
template <bool DiffuseOnly, bool Ext, bool Tex = false>
__global__ void __launch_bounds__(kBlock, PBRT_VOL_SURF_WAVES) k_vsurface(DeviceScene S0, PathState st, VolState v,
                                                                       int wf) {
    const QueueView surf = LoadQueue(st, wf, kVSurf);
    if ((int)(blockIdx.x * blockDim.x) >= surf.total) return;
    extern __shared__ float4 dynLds[];
    DeviceScene S = S0;
    float *fbuf = reinterpret_cast<float *>(StageVolTables(S0, S, reinterpret_cast<char *>(dynLds)));
    float *fL = fbuf + threadIdx.x;  // fL[i * kBlock]: [31][kBlock] per-lane spectra
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1], &out = v.rec[(wf + 1) & 1];
    const int shard = ProducerShard();
    const int shardBase = shard * st.capS;
    int *nextCnt = &st.counters[CounterIndex(wf + 1, kVRay, shard)];
    int *shadowCnt = &st.counters[CounterIndex(wf, kVShadow, shard)];
    const bool last = wf == S.maxDepth;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < surf.total; j += gridDim.x * blockDim.x) {
        const int ri = v.surfQ[QueueSlot(surf, j)];
        const float lambda0 = rec.lambda0[ri];
        const int slot = rec.pixel[ri];
        const int depth = rec.depth[ri], flags = rec.flags[ri], medium = rec.medium[ri];
        const bool specularBounce = flags & 1;
        const bool betaUni = flags & kUniBeta, ruUni = flags & kUniRu, rlUni = flags & kUniRl;
        const SpecIn betaIn(rec.beta, NR, ri, betaUni), ruIn(rec.ru, NR, ri, ruUni), rlIn(rec.rl, NR, ri, rlUni);
        const V3 rd = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
        const int prim = v.hitPrim[ri];
        if (prim < 0) continue;  // escaped rays: k_vescaped
        const float b0 = v.hitB[ri], b1 = v.hitB[NR + ri], b2 = v.hitB[2 * NR + ri];
        V3 p0, p1, p2;
        PrimVerts(S, prim, &p0, &p1, &p2);
        TriSurface si = SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
        const V3 wo3 = Normalize(-rd);
        int mIn, mOut;
        MediaOf(S, prim, medium, &mIn, &mOut);
        const int mat = VolHitMaterial(S, st, ri, prim);
        const int mtypeHit = S.matType[mat];
        if (mtypeHit == 3) continue;  // interface crossings: k_viface
        if constexpr (Tex) {
            if (S.hasBump) BumpedShading(S, st, wf, mat, ri, &si);
        }
        // HandleEmissiveIntersection (integrator.cpp:539-573)
        const int light = S.primLight[prim];
        if (light >= 0) {
            const DeviceAreaLight Ld = S.lights[light];
            if ((Ld.twoSided || DotN(si.n, wo3) >= 0) && !SpreadCut(Ld.v1.w, si.n, wo3)) {  // else Le = 0
                const bool plain = depth == 0 || specularBounce;
                float lightPDF = 0;
                if (!plain) {
                    const V3 pp = LoadV3(rec.prev, NR, ri), pe = LoadV3(rec.prev + 3 * (size_t)NR, NR, ri);
                    const V3 pn = LoadV3(rec.prev + 6 * (size_t)NR, NR, ri);
                    const V3 pns = LoadV3(rec.prev + 9 * (size_t)NR, NR, ri);
                    const float lightChoicePDF = LightPMF(S, pp, pns, light);
                    if (Ext && S.nShapes > 0 && prim >= S.nTris) {
                        lightPDF = lightChoicePDF * ShapeLightPDF(S.shapes, S.shapeN, prim - S.nTris, pp, pe, pn, pns, -wo3);
                    } else {
                        TriShading lsh;
                        const bool lhas = LoadTriShading(S, __float_as_int(Ld.v0.w), &lsh);
                        const V3 l0(Ld.v0.x, Ld.v0.y, Ld.v0.z), l1(Ld.v1.x, Ld.v1.y, Ld.v1.z),
                            l2(Ld.v2.x, Ld.v2.y, Ld.v2.z);
                        lightPDF = lightChoicePDF *
                                   TrianglePDF(l0, l1, l2, Ld.flip, lhas ? &lsh : nullptr, pp, pe, pn, pns, -wo3);
                    }
                }
                float ds = 0;
#pragma unroll 1
                for (int i = 0; i < kNS; ++i) {
                    const float ru = ruIn(i);
                    const float dv = plain ? ru : ru + rlIn(i) * lightPDF;
                    ds = i == 0 ? dv : ds + dv;
                }
                const float avg = ds / kNS;
                if (Ext && S.nImageAreaLights > 0 && S.lightImgOff[light] >= 0) {
                    // an image emitter: the image at the hit's uv (lights.h:460-467)
                    const EnvCoef ec = AreaImageCoef(S, S.lightImgOff[light], si.uv[0], si.uv[1]);
                    SpectralIter itL(lambda0);
                    AddSpecToL(S, st, slot, lambda0, [&](int i, int off) {
                        const float lam = itL.lam;
                        itL.Next();
                        return betaIn(i) * EnvLe(ec, Ld.scale, DenseAt(S, Ld.spectrum, off), lam) / avg;
                    });
                } else {
                    AddSpecToL(S, st, slot, lambda0,
                               [&](int i, int off) { return betaIn(i) * (Ld.scale * DenseAt(S, Ld.spectrum, off)) / avg; });
                }
            }
        }
        if (last) continue;
        if (mtypeHit == kMatCoatedDiffuseT || mtypeHit == kMatCoatedConductorT || mtypeHit == kMatDiffuseTransmissionT ||
            mtypeHit == kMatHairT || mtypeHit == kMatMeasuredT || mtypeHit == kMatRetroreflectiveT)
            continue;  // k_vlayered
        const int mtype = DiffuseOnly ? 0 : mtypeHit;
        // ---- EvaluateMaterialAndBSDF (surfscatter.cpp:57-328) for this material type
        const VRaySamples rs = RaySamplesAt(S, st, slot, depth, mtype == 1 || mtype == kMatThinDielectricT);
        const float4 mp4 = S.matParams[mat];
        float4 mc = S.matCoeffs[mat];
        bool constant = S.matConstant[mat] & 1;
        TrowbridgeReitz tr{mp4.x, mp4.y};
        // textured reflectance: sigmoid coefficients, or 31 values (texR); textured roughness:
        // the alphas (materials.h GetBxDF texEval calls)
        bool texR = false;
        if constexpr (Tex) {
            const int4 mt = S.matTex[mat];
            if (mt.x >= 0) {
                constant = false;
                if (st.texCoef[3 * (size_t)NR + ri] != 0) texR = true;
                else mc = make_float4(st.texCoef[ri], st.texCoef[(size_t)NR + ri], st.texCoef[2 * (size_t)NR + ri], 0.f);
            }
            if (mt.y >= 0) tr = TrowbridgeReitz{st.texCoef[4 * (size_t)NR + ri], st.texCoef[5 * (size_t)NR + ri]};
        }
        // the reflectance before its clamp at wavelength i (lam)
        auto reflRaw = [&](float lam, int i) -> float {
            if constexpr (Tex) {
                if (texR) return st.texR[(size_t)i * NR + ri];
            }
            return constant ? mc.w : SigmoidPolynomial(mc.x, mc.y, mc.z, lam);
        };
        // surfscatter.cpp:127-128 (ThinDielectricBxDF::Regularize does nothing)
        if (mtype != 0 && mtype != kMatThinDielectricT && S.regularize && (flags & 2)) tr.Regularize();
        float eta = mp4.z == 0 ? 1.f : mp4.z;
        if ((mtype == 1 || mtype == kMatThinDielectricT) && S.dispersive && S.matSpectra[2 * mat] >= 0) {
            // DielectricMaterial::GetBxDF (materials.cpp:25-49): eta(lambda_0), then
            // TerminateSecondary for a non-constant eta
            const int es = S.matSpectra[2 * mat], a = S.plOffsets[es], na = S.plOffsets[es + 1] - a;
            eta = PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, lambda0);
            if (eta == 0) eta = 1;
            st.lamTerm[slot] = 1;
        }
        const int etaSpec = mtype == 2 ? S.matSpectra[2 * mat] : -1;
        const int kSpec = mtype == 2 ? S.matSpectra[2 * mat + 1] : -1;
        auto etaK = [&](float lam, int i, float *e, float *k) {
            if (etaSpec >= 0 && !texR && (!Tex || S.matTex[mat].x < 0)) {
                const int a = S.plOffsets[etaSpec], na = S.plOffsets[etaSpec + 1] - a;
                const int b = S.plOffsets[kSpec], nb = S.plOffsets[kSpec + 1] - b;
                *e = PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, lam);
                *k = PiecewiseLinearEval(S.plLambda + b, S.plValue + b, nb, lam);
            } else {
                const float r = Clampf(reflRaw(lam, i), 0, .9999f);
                *e = 1.f;
                *k = 2 * std::sqrt(r) / std::sqrt(std::fmax(0.f, 1 - r));
            }
        };
        // f_i of the material's BxDF given its per-sample terms (diffuse R/pi, dielectric scalar,
        // conductor Fresnel per wavelength)
        auto fAt = [&](float lam, int i, float fd, const ConductorTerms &ct) -> float {
#if PBRT_VOL_EXPERIMENT == 2
            if (mtype == 0) return 0.4f * kInvPi;
#endif
            if (mtype == 0) return Clampf(reflRaw(lam, i), 0, 1) * kInvPi;
            if (mtype == 1 || mtype == kMatThinDielectricT) return fd;
            float e, k;
            etaK(lam, i, &e, &k);
            return ConductorF(ct, e, k);
        };
        // BxDF::Flags (bxdfs.h): diffuse R != 0; dielectric / conductor always
        // (diffuse: f_i = R_i / pi is kept in LDS for the light sample and the BSDF sample)
        bool hasFlags = mtype != 0;
        if (mtype == 0) {
            SpectralIter it(lambda0);
#pragma unroll 2
            for (int i = 0; i < kNS; ++i, it.Next()) {
                const float R = Clampf(reflRaw(it.lam, i), 0, 1);
                hasFlags |= R != 0;
                fL[i * kBlock] = R * kInvPi;
            }
        }
        if (!hasFlags) continue;
        const bool smooth = mtype != 0 && tr.EffectivelySmooth();
        const bool reflective = mtype != 1 || eta != 1;
        const bool transmissive = mtype == 1 || mtype == kMatThinDielectricT;
        const Frame frame = Frame::FromXZ(Normalize(si.dpdus), si.ns);
        const V3 woL = frame.ToLocal(wo3);
        // ---- light sampling + shadow ray (surfscatter.cpp:252-326), IsNonSpecular(flags)
        if (mtype == 0 || !smooth) {
            V3 cp = si.p, cpErr = si.pErr;  // LightSampleContext: the offset point is exact
            if (reflective && !transmissive) cp = OffsetRayOrigin(si.p, si.pErr, si.n, wo3), cpErr = V3(0, 0, 0);
            else if (transmissive && reflective) cp = OffsetRayOrigin(si.p, si.pErr, si.n, -wo3), cpErr = V3(0, 0, 0);
            AreaLightHit ls;
            if (SampleAreaLightAt<Ext>(S, cp, si.n, si.ns, rs.dUc, rs.dU0, rs.dU1, lambda0, &ls, cpErr) && woL.z != 0) {
                const V3 wi = ls.wi;
                const V3 wiL = frame.ToLocal(wi);
                // BSDF::f / BSDF::PDF (bsdf.h:60-135)
                float fd = 0, bsdfPDF = 0;
                ConductorTerms ct{};
                bool fAny;
                if (mtype == 0) {
                    fAny = woL.z * wiL.z > 0;  // SameHemisphere, else f = 0
                    bsdfPDF = fAny ? CosineHemispherePDF(fabsf(wiL.z)) : 0.f;
                } else if (mtype == 1) {
                    fd = DielectricEval(eta, tr, woL, wiL, &bsdfPDF);
                    fAny = fd != 0;
                } else {
                    ct = ConductorEval(tr, woL, wiL);
                    bsdfPDF = ct.pdf;
                    fAny = ct.ok;
                }
                if (ls.delta) bsdfPDF = 0;  // IsDeltaLight
                if (fAny) {
                    const float absdot = AbsDotN(si.ns, wi);
                    const float lightPDF = ls.pdf;
                    // SpawnRayTo(pi, n, time, pLight.pi, pLight.n) (ray.h:106-111)
                    const V3 so = OffsetRayOrigin(si.p, si.pErr, si.n, ls.p - si.p);
                    const V3 pt = OffsetRayOrigin(ls.p, ls.pErr, ls.n, so - ls.p);
                    const V3 sd = pt - so;
                    // Ld_i = beta_i f_i |cos| Le_i; r_u / r_l follow r_u
                    bool fnz = mtype == 0, ldUni = true, rgb = false;
                    int js = -1;
                    if (mtype == 0 && S.media.allGrey) {
                        // f_i from LDS; Ld as its sensor sums + Ld_0 (kShRgb)
                        js = ShardSlot(shardBase, WavePush(shadowCnt, true), st.capS, st.NR);
                        SpectralIter it(lambda0);
                        SensorAcc acc;
                        float ld0 = 0;
#pragma unroll 1
                        for (int i = 0; i < kNS; ++i, it.Next()) {
                            const int off = DenseOffset(it.lam);
                            const float Ldv = betaIn(i) * fL[i * kBlock] * absdot * ls.Le(S, off, it.lam);
                            ld0 = i == 0 ? Ldv : ld0;
                            acc.Add(S, off, Ldv, i == 0);
                        }
                        v.shLd[js] = acc.sx;
                        v.shLd[NR + js] = acc.sy;
                        v.shLd[2 * (size_t)NR + js] = acc.sz;
                        v.shLd[3 * (size_t)NR + js] = ld0;
                        ldUni = false;
                        rgb = true;
                    } else if (mtype == 0) {
                        // f_i from LDS (nonzero somewhere: the flags pass), Ld straight to the queue
                        js = ShardSlot(shardBase, WavePush(shadowCnt, true), st.capS, st.NR);
                        SpectralIter it(lambda0);
                        float ld0 = 0;
#pragma unroll 2
                        for (int i = 0; i < kNS; ++i, it.Next()) {
                            const float Le = ls.Le(S, DenseOffset(it.lam), it.lam);
                            const float Ldv = betaIn(i) * fL[i * kBlock] * absdot * Le;
                            ld0 = i == 0 ? Ldv : ld0;
                            ldUni &= FloatToBits(Ldv) == FloatToBits(ld0);
                            v.shLd[(size_t)i * NR + js] = Ldv;
                        }
                    } else {
                        SpectralIter it(lambda0);
#pragma unroll 1
                        for (int i = 0; i < kNS; ++i, it.Next()) {
                            const float f = fAt(it.lam, i, fd, ct);
                            fnz |= f != 0;
                            const float Le = ls.Le(S, DenseOffset(it.lam), it.lam);
                            const float Ldv = betaIn(i) * f * absdot * Le;
                            fL[i * kBlock] = Ldv;
                            ldUni &= FloatToBits(Ldv) == FloatToBits(fL[0]);
                        }
                        if (fnz) {
                            js = ShardSlot(shardBase, WavePush(shadowCnt, true), st.capS, st.NR);
                            v.shLd[js] = fL[0];
#pragma unroll 2
                            for (int i = 1; i < kNS; ++i)
                                if (!ldUni) v.shLd[(size_t)i * NR + js] = fL[i * kBlock];
                        }
                    }
                    if (fnz) {
                        v.shRu[js] = ruIn.v0 * bsdfPDF;
                        v.shRl[js] = ruIn.v0 * lightPDF;
                        if (!ruUni) {
#pragma unroll 2
                            for (int i = 1; i < kNS; ++i) {
                                const float ru = ruIn(i);
                                v.shRu[(size_t)i * NR + js] = ru * bsdfPDF;
                                v.shRl[(size_t)i * NR + js] = ru * lightPDF;
                            }
                        }
                        v.shFlags[js] = (ldUni ? kShUniLd : 0) | (ruUni ? kShUniRu | kShUniRl : 0) | (rgb ? kShRgb : 0);
                        StoreV3(v.shRay, NR, js, so);
                        StoreV3(v.shRay + 3 * (size_t)NR, NR, js, sd);
                        v.shLambda0[js] = lambda0;
                        v.shPixel[js] = slot;
                        v.shMedium[js] = DotN(si.n, sd) > 0 ? mOut : mIn;
                    }
                }
            }
        }
        // ---- BSDF::Sample_f + RR + indirect ray (surfscatter.cpp:170-250)
        if (woL.z == 0) continue;
        bool ok = false;
        V3 wiL;
        float pdf = 0, fd = 0, etap = 1;
        bool specular = false, transmission = false;
        ConductorTerms ct{};
        if (mtype == 0) {
            wiL = SampleCosineHemisphere(rs.iU0, rs.iU1);
            if (woL.z < 0) wiL.z *= -1;
            pdf = CosineHemispherePDF(fabsf(wiL.z));
            ok = true;
        } else if (mtype == 1) {
            const BxSample bs = DielectricSample(eta, tr, woL, rs.iUc, rs.iU0, rs.iU1);
            ok = bs.ok && bs.f != 0;
            wiL = bs.wi;
            pdf = bs.pdf;
            fd = bs.f;
            etap = bs.etap;
            specular = bs.flags & kBxSpecular;
            transmission = bs.flags & kBxTransmission;
        } else if (mtype == kMatThinDielectricT) {
            const BxSample bs = ThinDielectricSample(eta, woL, rs.iUc);
            ok = bs.ok && bs.f != 0;
            wiL = bs.wi;
            pdf = bs.pdf;
            fd = bs.f;
            specular = true;
            transmission = bs.flags & kBxTransmission;
        } else {
            ct = ConductorSample(tr, woL, rs.iU0, rs.iU1);
            ok = ct.ok;
            wiL = ct.wi;
            pdf = ct.pdf;
            specular = ct.specular;
        }
        if (!ok || pdf == 0 || wiL.z == 0) continue;
        const V3 wi = frame.FromLocal(wiL);
        const float absdot = AbsDotN(si.ns, wi);
        float etaScale = rec.etaScale[ri];
        if (transmission) etaScale *= Sqr(etap);
        float rus = 0;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) rus = i == 0 ? ruIn.v0 : rus + ruIn(i);
        const float avgRu = rus / kNS;
        bool fAny = false;
        float mx = -kInfinity;
        {
            SpectralIter it(lambda0);
#pragma unroll 1
            for (int i = 0; i < kNS; ++i, it.Next()) {
                const float f = mtype == 0 ? fL[i * kBlock] : fAt(it.lam, i, fd, ct);
                fAny |= f != 0;
                const float nb = betaIn(i) * f * absdot / pdf;
                fL[i * kBlock] = nb;
                mx = fmaxf(mx, nb * etaScale / avgRu);
            }
        }
        if (!fAny) continue;
        const bool rrOn = mx < 1 && depth >= 1;
        float q = 0;
        if (rrOn) {
            q = fmaxf(0.f, 1 - mx);
            if (rs.rr < q) continue;
        }
        bool nz = false, nbUni = true;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) {
            float nb = fL[i * kBlock];
            if (rrOn) nb /= 1 - q;
            fL[i * kBlock] = nb;
            nz |= nb != 0;
            nbUni &= FloatToBits(nb) == FloatToBits(fL[0]);
        }
        if (!nz) continue;
        if (transmission && S.matSss && S.matSss[mat] >= 0) {
            // a subsurface material's transmitted sample goes to the BSSRDF queue instead of
            // the next iteration (surfscatter.cpp:225-232); beta after Russian roulette, r_u as
            // it came in, the updated etaScale
            const int js = ShardSlot(shardBase, WavePush(&st.counters[CounterIndex(wf, kVSss, shard)], true), st.capS, st.NR);
            const SssRecords &sr = v.sss;
            bool bu = true;
#pragma unroll 2
            for (int i = 0; i < kNS; ++i) bu &= FloatToBits(fL[i * kBlock]) == FloatToBits(fL[0]);
            sr.beta[js] = fL[0];
            sr.ru[js] = ruIn.v0;
#pragma unroll 2
            for (int i = 1; i < kNS; ++i) {
                if (!bu) sr.beta[(size_t)i * NR + js] = fL[i * kBlock];
                if (!ruUni) sr.ru[(size_t)i * NR + js] = ruIn(i);
            }
            StoreV3(sr.po, NR, js, si.p);
            StoreV3(sr.ns, NR, js, si.ns);
            sr.lambda0[js] = lambda0;
            sr.etaScale[js] = etaScale;
            sr.mat[js] = mat;
            sr.pixel[js] = slot;
            sr.depth[js] = depth;
            sr.mIn[js] = mIn;
            sr.mOut[js] = mOut;
            sr.flags[js] = (bu ? kUniBeta : 0) | (ruUni ? kUniRu : 0);
            sr.src[js] = ri;
            continue;
        }
        const int jn = ShardSlot(shardBase, WavePush(nextCnt, true), st.capS, st.NR);
        out.beta[jn] = fL[0];
        out.ru[jn] = ruIn.v0;
        out.rl[jn] = ruIn.v0 / pdf;
#pragma unroll 2
        for (int i = 1; i < kNS; ++i) {
            if (!nbUni) out.beta[(size_t)i * NR + jn] = fL[i * kBlock];
            if (!ruUni) {
                const float ru = ruIn(i);
                out.ru[(size_t)i * NR + jn] = ru;
                out.rl[(size_t)i * NR + jn] = ru / pdf;
            }
        }
        StoreV3(out.ray, NR, jn, OffsetRayOrigin(si.p, si.pErr, si.n, wi));
        StoreV3(out.ray + 3 * (size_t)NR, NR, jn, wi);
        StoreV3(out.prev, NR, jn, si.p);
        StoreV3(out.prev + 3 * (size_t)NR, NR, jn, si.pErr);
        StoreV3(out.prev + 6 * (size_t)NR, NR, jn, si.n);
        StoreV3(out.prev + 9 * (size_t)NR, NR, jn, si.ns);
        out.lambda0[jn] = lambda0;
        out.etaScale[jn] = etaScale;
        out.flags[jn] = (specular ? 1 : 0) | ((!specular || (flags & 2)) ? 2 : 0) | (nbUni ? kUniBeta : 0) |
                        (ruUni ? kUniRu | kUniRl : 0);
        out.pixel[jn] = slot;
        out.depth[jn] = depth + 1;
        out.medium[jn] = DotN(si.n, wi) > 0 ? mOut : mIn;
    }
}

// ------------------------------------------------------------------ subsurface scattering
// WavefrontPathIntegrator::SampleSubsurface (wavefront/subsurface.cpp:18-206) in two stages:
// k_vsss_probe samples the BSSRDF probe segment and traces it (the aggregate's
// IntersectOneRandom, optix.cu:478-518), k_vsss_scatter turns the reservoir's hit into the exit
// vertex (TabulatedBSSRDF::ProbeIntersectionToSample) and samples its NormalizedFresnelBxDF for
// the indirect ray and a light for the shadow ray.  Their shadow rays join this iteration's
// shadow queue (traced after them).

// A subsurface spectrum parameter at wavelength lam (SubsurfaceDesc: kind 0 ConstantSpectrum,
// 1 RGBUnbounded / RGBAlbedo scale * sigmoid, 2 PiecewiseLinearSpectrum)
__device__ inline float SssSpectrumAt(const DeviceScene &S, const float *q, float lam) {
    const int kind = (int)q[0];
    if (kind == 0) return q[1];
    if (kind == 1) return q[5] * SigmoidPolynomial(q[2], q[3], q[4], lam);
    const int pl = (int)q[6], a = S.plOffsets[pl], na = S.plOffsets[pl + 1] - a;
    return PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, lam);
}
// A textured subsurface reflectance (materials.h:823-841 texEval(reflectance)): the texture
// stage's value at the entry record src of this iteration, per wavelength index i (sigmoid
// coefficients, or one value per wavelength); on == false: the material's constant form
// sa / sb: a textured sigma_a and sigma_s | mfp at the entry record (texS + src, stride NR per
// wavelength; null: the constant)
struct SssTexRefl {
    bool on = false, perLambda = false;
    float c0 = 0, c1 = 0, c2 = 0;
    const float *r = nullptr;  // texR + src, stride NR
    const float *sa = nullptr, *sb = nullptr;
    int NR = 0;
    __device__ float At(int i, float lam) const {
        return perLambda ? r[(size_t)i * NR] : SigmoidPolynomial(c0, c1, c2, lam);
    }
};
__device__ inline SssTexRefl SssTexReflOf(const DeviceScene &S, const PathState &st, int mat, int src) {
    SssTexRefl x;
    if (!S.textured) return x;
    const int NR = st.NR;
    x.NR = NR;
    if (S.matSssTex) {
        const int2 p = S.matSssTex[mat];
        if (p.x >= 0) x.sa = st.texS + src;
        if (p.y >= 0) x.sb = st.texS + (size_t)kNSpectrumSamples * NR + src;
    }
    if (S.matTex[mat].x < 0) return x;
    x.on = true;
    x.perLambda = st.texCoef[3 * (size_t)NR + src] != 0;
    x.c0 = st.texCoef[src];
    x.c1 = st.texCoef[(size_t)NR + src];
    x.c2 = st.texCoef[2 * (size_t)NR + src];
    x.r = st.texR + src;
    x.NR = NR;
    return x;
}
// SubsurfaceMaterial::GetBSSRDF's sigma_a / sigma_s at wavelength index i, lam (materials.h:
// 823-841), as the TabulatedBSSRDF's sigma_t and rho
__device__ inline SssCoeffs SssCoeffsAt(const DeviceScene &S, const float *P, const SssTable &t, float lam,
                                        const SssTexRefl &tex = SssTexRefl{}, int i = 0) {
    float sa, ss;
    if (P[0] == 0) {
        const float a = P[1] * (tex.sa ? tex.sa[(size_t)i * tex.NR] : SssSpectrumAt(S, P + 4, lam));
        const float b = P[1] * (tex.sb ? tex.sb[(size_t)i * tex.NR] : SssSpectrumAt(S, P + 11, lam));
        sa = a > 0 ? a : 0.f;  // ClampZero
        ss = b > 0 ? b : 0.f;
    } else {
        const float m = P[1] * (tex.sb ? tex.sb[(size_t)i * tex.NR] : SssSpectrumAt(S, P + 11, lam));
        const float mfree = m > 0 ? m : 0.f;
        const float r = Clampf(tex.on ? tex.At(i, lam) : SssSpectrumAt(S, P + 4, lam), 0, 1);
        SssFromDiffuse(t, r, mfree, &sa, &ss);
    }
    return MakeSssCoeffs(sa, ss);
}

// IntersectOneRandom for one probe segment (optix.cu:478-518): closest hits from p0 towards p1
// (tMax 1), each continued by SpawnRayTo(p1) up to 99 traces; hits on material `mat` enter a
// weighted reservoir (weight 1) seeded with Hash(p0, p1).  Returns the chosen leaf-order
// primitive (-1: none) with its hit coordinates and SampleProbability.
template <int TM>
__device__ inline int ProbeOneRandom(const DeviceScene &S, const SceneLds &L, V3 p0, V3 p1, int mat, float *b0,
                                     float *b1, float *b2, float *resPdf) {
    const uint32_t hw[6] = {FloatToBits(p0.x), FloatToBits(p0.y), FloatToBits(p0.z),
                            FloatToBits(p1.x), FloatToBits(p1.y), FloatToBits(p1.z)};
    PCG32 rng;
    rng.SetSequence(HashWords(hw, 6));
    float wsum = 0;
    int chosen = -1;
    V3 o = p0, d = p1 - p0;
    for (int depth = 1; LengthSquared(d) > 0 && depth < 100; ++depth) {
        TriHit h;
        const int prim = Traverse<false, TM>(S, L, o, d, 1.f, &h);
        if (prim < 0) break;
        V3 a, b, c;
        PrimVerts(S, prim, &a, &b, &c);
        const TriSurface si = SurfaceAt<true>(S, prim, a, b, c, h.b0, h.b1, h.b2);
        if (S.primMaterial[prim] == mat) {
            wsum += 1.f;
            if (rng.Uniform() < 1.f / wsum) {
                chosen = prim;
                *b0 = h.b0, *b1 = h.b1, *b2 = h.b2;
            }
        }
        d = p1 - si.p;
        o = OffsetRayOrigin(si.p, si.pErr, si.n, d);
    }
    *resPdf = chosen >= 0 && wsum > 0 ? 1.f / wsum : 0.f;  // reservoirWeight / weightSum
    return chosen >= 0 && wsum > 0 ? chosen : -1;
}

// The aggregate's IntersectOneRandom exposed on its own (integrator.h:53): caller segments
// segs[6][n] (p0, p1) and materials[n] -> prim[n] (the caller's primitive numbering, -1),
// hit[3][n] (b0 b1 b2), pdf[n]
template <int TM>
__global__ void __launch_bounds__(kBlock, TraversalWaves(TM)) k_intersect_one_random(DeviceScene S, const float *segs,
                                                                                     const int *mats, int n, int *outPrim,
                                                                                     float *outHit, float *outPdf) {
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const V3 p0(segs[i], segs[n + i], segs[2 * n + i]), p1(segs[3 * n + i], segs[4 * n + i], segs[5 * n + i]);
        float b0 = 0, b1 = 0, b2 = 0, pdf = 0;
        const int prim = ProbeOneRandom<TM>(S, L, p0, p1, mats[i], &b0, &b1, &b2, &pdf);
        outPrim[i] = prim >= 0 ? S.primOrig[prim] : -1;  // the caller's numbering
        outHit[i] = b0;
        outHit[n + i] = b1;
        outHit[2 * n + i] = b2;
        outPdf[i] = pdf;
    }
}

template <int TM>
__global__ void __launch_bounds__(kBlock, TraversalWaves(TM)) k_vsss_probe(DeviceScene S, PathState st, VolState v,
                                                                            int wf) {
    const QueueView q = LoadQueue(st, wf, kVSss);
    if ((int)(blockIdx.x * blockDim.x) >= q.total) return;
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int NR = st.NR;
    const SssRecords &r = v.sss;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < q.total; j += gridDim.x * blockDim.x) {
        const int e = QueueSlot(q, j);
        r.hitPrim[e] = -1;
        r.resPdf[e] = 0;
        const int mat = r.mat[e], k = S.matSss[mat];
        const float *P = S.sssParams + (size_t)kSssParams * k;
        const SssTable t = SssTable::At(S.sssTables + (size_t)kSssTableFloats * k);
        // GetBSSRDF + SampleSp with the subsurface samples (subsurface.cpp:24-42)
        const SssCoeffs c0 = SssCoeffsAt(S, P, t, r.lambda0[e], SssTexReflOf(S, st, mat, r.src[e]), 0);
        float uc, u0, u1;
        SssSamplesAt(S, st, r.pixel[e], r.depth[e], &uc, &u0, &u1);
        V3 p0, p1;
        if (!SssSampleSp(t, c0, LoadV3(r.po, NR, e), LoadV3(r.ns, NR, e), uc, u0, u1, &p0, &p1)) continue;
        float cb0 = 0, cb1 = 0, cb2 = 0, pdf = 0;
        const int chosen = ProbeOneRandom<TM>(S, L, p0, p1, mat, &cb0, &cb1, &cb2, &pdf);
        if (chosen >= 0) {
            r.hitPrim[e] = chosen;
            r.hitB[e] = cb0;
            r.hitB[NR + e] = cb1;
            r.hitB[2 * (size_t)NR + e] = cb2;
            r.resPdf[e] = pdf;
        }
    }
}

template <bool Ext>
__global__ void __launch_bounds__(kBlock) k_vsss_scatter(DeviceScene S0, PathState st, VolState v, int wf) {
    const QueueView q = LoadQueue(st, wf, kVSss);
    if ((int)(blockIdx.x * blockDim.x) >= q.total) return;
    extern __shared__ float4 dynLds[];
    DeviceScene S = S0;
    (void)StageVolTables(S0, S, reinterpret_cast<char *>(dynLds));
    const int NR = st.NR;
    const SssRecords &r = v.sss;
    const VolRecords &out = v.rec[(wf + 1) & 1];
    const int shard = ProducerShard();
    const int shardBase = shard * st.capS;
    int *nextCnt = &st.counters[CounterIndex(wf + 1, kVRay, shard)];
    int *shadowCnt = &st.counters[CounterIndex(wf, kVShadow, shard)];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < q.total; j += gridDim.x * blockDim.x) {
        const int e = QueueSlot(q, j);
        const int prim = r.hitPrim[e];
        const float resPdf = r.resPdf[e];
        if (prim < 0 || resPdf == 0) continue;  // "if (w.reservoirPDF == 0) return"
        const int mat = r.mat[e], k = S.matSss[mat];
        const float *P = S.sssParams + (size_t)kSssParams * k;
        const SssTable t = SssTable::At(S.sssTables + (size_t)kSssTableFloats * k);
        const float lambda0 = r.lambda0[e];
        const int slot = r.pixel[e], depth = r.depth[e], fl = r.flags[e];
        const SpecIn betaIn(r.beta, NR, e, fl & kUniBeta), ruIn(r.ru, NR, e, fl & kUniRu);
        V3 a, b, c;
        PrimVerts(S, prim, &a, &b, &c);
        const TriSurface si = SurfaceAt<Ext>(S, prim, a, b, c, r.hitB[e], r.hitB[NR + e], r.hitB[2 * (size_t)NR + e]);
        // ProbeIntersectionToSample (bssrdf.h:305-312): Sp(pi) = Sr(|po - pi|), PDF_Sp(pi, n)
        const V3 po = LoadV3(r.po, NR, e);
        const float rDist = Distance(po, si.p);
        const SssPdfGeom g = MakeSssPdfGeom(po, LoadV3(r.ns, NR, e), si.p, si.n);
        // betap = beta Sp / (reservoirPDF pdf_0) and r_u pdf / pdf_0 (subsurface.cpp:60-62), written
        // over the record's own (full-spectrum) beta and r_u: bp(i), ru(i) below
        float *bpP = r.beta + e, *ruP = r.ru + e;
        auto bp = [&](int i) -> float & { return bpP[(size_t)i * NR]; };
        auto ru = [&](int i) -> float & { return ruP[(size_t)i * NR]; };
        const SssTexRefl tex = SssTexReflOf(S, st, mat, r.src[e]);
        const float pdf0 = SssPdfSp(t, SssCoeffsAt(S, P, t, lambda0, tex, 0), g);
        const float pr = resPdf * pdf0;
        bool spAny = false, pdfAny = false;
        {
            SpectralIter it(lambda0);
#pragma unroll 1
            for (int i = 0; i < kNS; ++i, it.Next()) {
                const SssCoeffs ci = SssCoeffsAt(S, P, t, it.lam, tex, i);
                const float sp = SssSrScaled(t, ci, rDist), pdf = SssPdfSp(t, ci, g);
                spAny |= sp != 0;
                pdfAny |= pdf != 0;
                const float b = betaIn(i), u = ruIn(i);  // read before the slot is overwritten
                bp(i) = b * sp / pr;
                ru(i) = u * pdf / pdf0;
            }
        }
        if (!spAny || !pdfAny) continue;
        float rus = 0;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) rus = i == 0 ? ru(0) : rus + ru(i);
        const float avgRu = rus / kNS;
        // NormalizedFresnelBxDF(eta) in the frame of the exit's shading normal and dpdu, wo = ns
        const float eta = P[2], fc = P[3];
        const Frame frame = Frame::FromXZ(Normalize(si.dpdus), si.ns);
        const V3 woL = frame.ToLocal(si.ns);
        int mIn = r.mIn[e], mOut = r.mOut[e];
        float dUc = 0, dU0 = 0, dU1 = 0;
        {
            const VRaySamples rs = RaySamplesAt(S, st, slot, depth, false);
            dUc = rs.dUc, dU0 = rs.dU0, dU1 = rs.dU1;
            // ---- indirect (subsurface.cpp:76-150): BSDF::Sample_f, RR (depth > 1), next ray
            if (woL.z != 0) {
                V3 wiL = SampleCosineHemisphere(rs.iU0, rs.iU1);
                if (woL.z < 0) wiL.z *= -1;
                const float f = NormalizedFresnelF(eta, fc, woL, wiL);
                const float pdf = woL.z * wiL.z > 0 ? CosineHemispherePDF(fabsf(wiL.z)) : 0.f;
                if (f != 0 && pdf != 0 && wiL.z != 0) {
                    const V3 wi = frame.FromLocal(wiL);
                    const float absdot = AbsDotN(si.ns, wi);
                    const float etaScale = r.etaScale[e];
                    float mx = -kInfinity;
                    // the new beta in the record slots' order: computed into registers per wavelength
                    bool nz = false;
                    float q = 0;
#pragma unroll 1
                    for (int i = 0; i < kNS; ++i) mx = fmaxf(mx, bp(i) * f * absdot / pdf * etaScale / avgRu);
                    const bool rrOn = mx < 1 && depth > 1;
                    bool killed = false;
                    if (rrOn) {
                        q = fmaxf(0.f, 1 - mx);
                        killed = rs.rr < q;
                    }
                    if (!killed) {
                        float nb0 = 0;
                        bool nbUni = true;
#pragma unroll 1
                        for (int i = 0; i < kNS; ++i) {
                            float nb = bp(i) * f * absdot / pdf;
                            if (rrOn) nb /= 1 - q;
                            nz |= nb != 0;
                            nb0 = i == 0 ? nb : nb0;
                            nbUni &= FloatToBits(nb) == FloatToBits(nb0);
                        }
                        if (nz) {
                            const int jn = ShardSlot(shardBase, WavePush(nextCnt, true), st.capS, st.NR);
                            bool ruUni = true;
#pragma unroll 1
                            for (int i = 0; i < kNS; ++i) ruUni &= FloatToBits(ru(i)) == FloatToBits(ru(0));
#pragma unroll 1
                            for (int i = 0; i < kNS; ++i) {
                                float nb = bp(i) * f * absdot / pdf;
                                if (rrOn) nb /= 1 - q;
                                if (i == 0 || !nbUni) out.beta[(size_t)i * NR + jn] = nb;
                                if (i == 0 || !ruUni) {
                                    out.ru[(size_t)i * NR + jn] = ru(i);
                                    out.rl[(size_t)i * NR + jn] = ru(i) / pdf;
                                }
                            }
                            StoreV3(out.ray, NR, jn, OffsetRayOrigin(si.p, si.pErr, si.n, wi));
                            StoreV3(out.ray + 3 * (size_t)NR, NR, jn, wi);
                            StoreV3(out.prev, NR, jn, si.p);
                            StoreV3(out.prev + 3 * (size_t)NR, NR, jn, si.pErr);
                            StoreV3(out.prev + 6 * (size_t)NR, NR, jn, si.n);
                            StoreV3(out.prev + 9 * (size_t)NR, NR, jn, si.ns);
                            out.lambda0[jn] = lambda0;
                            out.etaScale[jn] = etaScale;
                            out.flags[jn] = 2 | (nbUni ? kUniBeta : 0) | (ruUni ? kUniRu | kUniRl : 0);
                            out.pixel[jn] = slot;
                            out.depth[jn] = depth + 1;
                            out.medium[jn] = DotN(si.n, wi) > 0 ? mOut : mIn;
                        }
                    }
                }
            }
        }
        // ---- direct lighting (subsurface.cpp:152-203): the light sample from the exit point
        AreaLightHit ls;
        if (!SampleAreaLightAt<Ext>(S, si.p, si.n, si.ns, dUc, dU0, dU1, lambda0, &ls, si.pErr)) continue;
        const V3 wi = ls.wi;
        const V3 wiL = frame.ToLocal(wi);
        if (woL.z == 0) continue;  // BSDF::f
        const float f = NormalizedFresnelF(eta, fc, woL, wiL);
        if (f == 0) continue;
        const float absdot = AbsDotN(si.ns, wi);
        const float lightPDF = ls.pdf;
        const float bsdfPDF = ls.delta ? 0.f : (woL.z * wiL.z > 0 ? CosineHemispherePDF(fabsf(wiL.z)) : 0.f);
        const V3 so = OffsetRayOrigin(si.p, si.pErr, si.n, ls.p - si.p);
        const V3 pt = OffsetRayOrigin(ls.p, ls.pErr, ls.n, so - ls.p);
        const V3 sd = pt - so;
        float Ld[kNS], sru[kNS], srl[kNS];
        SpectralIter it(lambda0);
#pragma unroll
        for (int i = 0; i < kNS; ++i, it.Next()) {
            Ld[i] = bp(i) * f * absdot * ls.Le(S, DenseOffset(it.lam), it.lam);
            srl[i] = ru(i) * lightPDF;
            sru[i] = ru(i) * bsdfPDF;
        }
        const int js = ShardSlot(shardBase, WavePush(shadowCnt, true), st.capS, st.NR);
        WriteShadow(S, v, NR, js, ShadowOut{so, sd, DotN(si.n, sd) > 0 ? mOut : mIn}, Ld, sru, srl, lambda0, slot);
    }
}

// HandleEscapedRays (integrator.cpp:495-537) for the volumetric wavefront: UniformInfiniteLight,
// whose PDF_Li(allowIncompletePDF) is 0, so r_l adds nothing to the MIS denominator.  Escaped
// rays have their own queue (filled by the closest-hit and medium kernels) and kernel, with the
// sensor curves and spectra staged in LDS.
template <bool Ext>
__global__ void __launch_bounds__(kBlock) k_vescaped(DeviceScene S0, PathState st, VolState v, int wf) {
    const QueueView q = LoadQueue(st, wf, kVEsc);
    if ((int)(blockIdx.x * blockDim.x) >= q.total || S0.nInfinite == 0) return;
    extern __shared__ float4 dynLds[];
    DeviceScene S = S0;
    StageVolTables(S0, S, reinterpret_cast<char *>(dynLds));
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < q.total; j += gridDim.x * blockDim.x) {
        const int ri = v.escQ[QueueSlot(q, j)];
        const float lambda0 = rec.lambda0[ri];
        const int slot = rec.pixel[ri];
        const int depth = rec.depth[ri], flags = rec.flags[ri];
        const bool specularBounce = flags & 1;
        const SpecIn betaIn(rec.beta, NR, ri, flags & kUniBeta), ruIn(rec.ru, NR, ri, flags & kUniRu),
            rlIn(rec.rl, NR, ri, flags & kUniRl);
        float ds = 0;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) {
            const float ru = ruIn(i);
            const float dv = (depth == 0 || specularBounce) ? ru : ru + rlIn(i) * 0.f;
            ds = i == 0 ? dv : ds + dv;
        }
        const float avg = ds / kNS;
        // (a light with Le = 0 at every wavelength adds exact zeros: no separate test)
        for (int k = 0; k < S.nInfinite; ++k) {
            if (S.infDistant[k] >= 0) continue;  // a DistantLight is no Infinite-type light
            const int spec = S.infSpectrum[k];
            const float scale = S.infScale[k];
            if (Ext && S.nEnv > 0 && S.infImage[k] >= 0) {
                // ImageInfiniteLight: Le at the direction's pixel; past a non-specular bounce
                // r_l * PMF * PDF_Li(allowIncompletePDF) joins the denominator
                const DeviceEnvLight &E = S.env[S.infImage[k]];
                const V3 rd = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
                // a portal light's Le depends on the ray origin, its PDF_Li on the previous
                // vertex (prevIntrCtx.p())
                const EnvCoef ec = E.portal ? PortalLeCoef(E, LoadV3(rec.ray, NR, ri), rd) : EnvLeCoef(E, rd);
                float eavg = avg;
                if (!(depth == 0 || specularBounce)) {
                    const float pmf = LightPMF(S, V3(0, 0, 0), V3(0, 0, 0), S.nAreaLights + S.nPointSpot + k);
                    const float pdf = E.portal ? PortalPDFLi(E, LoadV3(rec.prev, NR, ri), rd) : EnvPDFLi(E, rd);
                    float es = 0;
#pragma unroll 1
                    for (int i = 0; i < kNS; ++i) {
                        const float dv = ruIn(i) + rlIn(i) * pmf * pdf;
                        es = i == 0 ? dv : es + dv;
                    }
                    eavg = es / kNS;
                }
                SensorAcc acc;
                SpectralIter it(lambda0);
                float c0 = 0;
#pragma unroll 1
                for (int i = 0; i < kNS; ++i, it.Next()) {
                    const int off = DenseOffset(it.lam);
                    const float ci = betaIn(i) * EnvLe(ec, scale, DenseAt(S, spec, off), it.lam) / eavg;
                    c0 = i == 0 ? ci : c0;
                    acc.Add(S, off, ci, i == 0);
                }
                const int NL = st.N;
                st.L[slot] += S.imagingRatio * (acc.sx / kNS);
                st.L[NL + slot] += S.imagingRatio * (acc.sy / kNS);
                st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNS);
                AddL0Off(S, st, slot, DenseOffset(lambda0), c0);
                continue;
            }
            AddSpecToL(S, st, slot, lambda0,
                       [&](int i, int off) { return betaIn(i) * (scale * DenseAt(S, spec, off)) / avg; });
        }
    }
}

// Material "interface" crossings (media.cpp:193-203): SpawnRay(ray.d) at the same path depth into
// the medium on the far side.  Split from k_vsurface (their own queue, filled by the closest-hit
// and medium kernels), so these items do not hold that kernel's registers and lanes.
template <bool Ext>
__global__ void __launch_bounds__(kBlock) k_viface(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView q = LoadQueue(st, wf, kVIface);
    if ((int)(blockIdx.x * blockDim.x) >= q.total || wf == S.maxDepth) return;  // last: path ends
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1], &out = v.rec[(wf + 1) & 1];
    const int shardBase = ProducerShard() * st.capS;
    int *nextCnt = &st.counters[CounterIndex(wf + 1, kVRay, ProducerShard())];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < q.total; j += gridDim.x * blockDim.x) {
        const int ri = v.ifaceQ[QueueSlot(q, j)];
        const float lambda0 = rec.lambda0[ri];
        const int slot = rec.pixel[ri];
        const int depth = rec.depth[ri], flags = rec.flags[ri], medium = rec.medium[ri];
        const bool betaUni = flags & kUniBeta, ruUni = flags & kUniRu, rlUni = flags & kUniRl;
        const SpecIn betaIn(rec.beta, NR, ri, betaUni), ruIn(rec.ru, NR, ri, ruUni), rlIn(rec.rl, NR, ri, rlUni);
        const V3 rd = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
        const int prim = v.hitPrim[ri];
        const float b0 = v.hitB[ri], b1 = v.hitB[NR + ri], b2 = v.hitB[2 * NR + ri];
        V3 p0, p1, p2;
        PrimVerts(S, prim, &p0, &p1, &p2);
        const TriSurface si = SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
        int mIn, mOut;
        MediaOf(S, prim, medium, &mIn, &mOut);
        const int jn = ShardSlot(shardBase, WavePush(nextCnt, true), st.capS, st.NR);
        out.beta[jn] = betaIn.v0;
        out.ru[jn] = ruIn.v0;
        out.rl[jn] = rlIn.v0;
#pragma unroll 2
        for (int i = 1; i < kNS; ++i) {
            if (!betaUni) out.beta[(size_t)i * NR + jn] = betaIn(i);
            if (!ruUni) out.ru[(size_t)i * NR + jn] = ruIn(i);
            if (!rlUni) out.rl[(size_t)i * NR + jn] = rlIn(i);
        }
        StoreV3(out.ray, NR, jn, OffsetRayOrigin(si.p, si.pErr, si.n, rd));
        StoreV3(out.ray + 3 * (size_t)NR, NR, jn, rd);
#pragma unroll
        for (int k = 0; k < 12; ++k) out.prev[(size_t)k * NR + jn] = rec.prev[(size_t)k * NR + ri];
        out.lambda0[jn] = lambda0;
        out.etaScale[jn] = rec.etaScale[ri];
        out.flags[jn] = flags;
        out.pixel[jn] = slot;
        out.depth[jn] = depth;
        out.medium[jn] = DotN(si.n, rd) > 0 ? mOut : mIn;
    }
}

// ---------------------------------------------------------------- layered materials
// The per-wavelength parameters of a coated material at a hit (CoatedDiffuseMaterial::GetBxDF /
// CoatedConductorMaterial::GetBxDF, materials.cpp:301-329, :391-437), evaluated once per hit:
// a = diffuse R (clamped) or conductor eta / interface eta, b = conductor k / interface eta,
// alb = layer albedo (clamped)
struct LayerSpec {
    float a[kNS], b[kNS], alb[kNS];
    __device__ float R(int i) const { return a[i]; }
    __device__ void EtaK(int i, float *e, float *k) const {
        *e = a[i];
        *k = b[i];
    }
    __device__ float Albedo(int i) const { return alb[i]; }
    __device__ float T(int i) const { return alb[i]; }  // diffuse transmission: T in alb
};

// EvaluateMaterialAndBSDF<CoatedDiffuseBxDF | CoatedConductorBxDF> (surfscatter.cpp:57-328):
// surface hits on layered materials (k_vsurface handles escapes, interfaces and emission of
// the same queue and skips these).  The LayeredBxDF estimates f, Sample_f and PDF by random
// walks (core.h LayeredBxDF); BSDF samples are pdfIsProportional, so r_l = r_u / PDF(wo, wi).
template <bool Ext>
__global__ void __launch_bounds__(kBlock) k_vlayered(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView surf = LoadQueue(st, wf, kVSurf);
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1], &out = v.rec[(wf + 1) & 1];
    const int shard = ProducerShard();
    const int shardBase = shard * st.capS;
    int *nextCnt = &st.counters[CounterIndex(wf + 1, kVRay, shard)];
    int *shadowCnt = &st.counters[CounterIndex(wf, kVShadow, shard)];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < surf.total; j += gridDim.x * blockDim.x) {
        const int ri = v.surfQ[QueueSlot(surf, j)];
        const int prim = v.hitPrim[ri];
        if (prim < 0) continue;
        const int mat = VolHitMaterial(S, st, ri, prim);
        const int mtype = S.matType[mat];
        if (mtype != kMatCoatedDiffuseT && mtype != kMatCoatedConductorT && mtype != kMatDiffuseTransmissionT &&
            mtype != kMatHairT && mtype != kMatMeasuredT && mtype != kMatRetroreflectiveT)
            continue;
        const bool dt = mtype == kMatDiffuseTransmissionT, hair = mtype == kMatHairT, meas = mtype == kMatMeasuredT;
        const bool retro = mtype == kMatRetroreflectiveT;
        const float lambda0 = rec.lambda0[ri];
        const int slot = rec.pixel[ri];
        const int depth = rec.depth[ri], flags = rec.flags[ri], medium = rec.medium[ri];
        const bool betaUni = flags & kUniBeta, ruUni = flags & kUniRu;
        const SpecIn betaIn(rec.beta, NR, ri, betaUni), ruIn(rec.ru, NR, ri, ruUni);
        const V3 rd = LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
        const float b0 = v.hitB[ri], b1 = v.hitB[NR + ri], b2 = v.hitB[2 * NR + ri];
        V3 p0, p1, p2;
        PrimVerts(S, prim, &p0, &p1, &p2);
        TriSurface si = SurfaceAt<Ext>(S, prim, p0, p1, p2, b0, b1, b2);
        // bump / normal mapping (surfscatter.cpp:109-127): k_vtexture's shading frame for this
        // record (the BSDF frame, the light sample and the next vertex's MIS context use it)
        if (S.hasBump) BumpedShading(S, st, wf, mat, ri, &si);
        const V3 wo3 = Normalize(-rd);
        int mIn, mOut;
        MediaOf(S, prim, medium, &mIn, &mOut);
        const VRaySamples rs = RaySamplesAt(S, st, slot, depth, true);
        // ---- GetBxDF
        const float4 mp4 = S.matParams[mat], mc = S.matCoeffs[mat];
        const bool constant = S.matConstant[mat] & 1;
        const float4 L0 = S.matLayer[3 * mat], L1 = S.matLayer[3 * mat + 1], L2 = S.matLayer[3 * mat + 2];
        const bool conductor = mtype == kMatCoatedConductorT || retro;
        float ieta = retro ? 1.f : mp4.z;  // RetroreflectiveMaterial::GetBxDF: eta and k as given
        if (!hair && !meas && !retro && L2.w >= 0) {  // spectral interface eta: eta(lambda_0), TerminateSecondary
            const int es = (int)L2.w, a = S.plOffsets[es], na = S.plOffsets[es + 1] - a;
            ieta = PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, lambda0);
            if (ieta == 0) ieta = 1;
            st.lamTerm[slot] = 1;
        }
        const int etaSpec = conductor ? S.matSpectra[2 * mat] : -1;
        const int kSpec = conductor ? S.matSpectra[2 * mat + 1] : -1;
        LayerSpec sp;
        bool bottomNz = false, albNz = false;
        float prMax = 0, ptMax = 0;
        // HairMaterial::GetBxDF (materials.h:380-404): beta_m / beta_n clamped to [0.01, 1],
        // h = -1 + 2 v; sigma_a per wavelength into sp.a (matLayer: HairLayer's packing)
        // textured floats (eta, beta_m, beta_n, alpha): the texture stage's values in texCoef[4..7]
        // (HitTextures); a textured concentration pair left sigma_a per wavelength in texR
        float hairEta = L2.x, hairBmIn = L2.y, hairBnIn = L2.z, hairAlpha = L2.w;
        bool hairConc = false;
        if (hair && S.matHairTex) {
            const int4 h0 = S.matHairTex[2 * mat];
            if (h0.x >= 0) hairEta = st.texCoef[4 * (size_t)NR + ri];
            if (h0.y >= 0) hairBmIn = st.texCoef[5 * (size_t)NR + ri];
            if (h0.z >= 0) hairBnIn = st.texCoef[6 * (size_t)NR + ri];
            if (h0.w >= 0) hairAlpha = st.texCoef[7 * (size_t)NR + ri];
            hairConc = S.matHairTex[2 * mat + 1].x >= 0;
        }
        const float hairBm = fmaxf(1e-2f, fminf(1.f, hairBmIn)), hairBn = fmaxf(1e-2f, fminf(1.f, hairBnIn));
        const float hairDen = HairReflectanceDenom(hairBn);
        const float hq[7] = {L0.y, L0.z, L0.w, L1.x, L1.y, L1.z, L1.w};
        // a textured sigma_a / reflectance: k_vtexture's value for this record (sigmoid
        // coefficients, or one value per wavelength)
        const bool hairTex = hair && S.textured && (S.matTex[mat].x >= 0 || hairConc);
        const bool hairTexR = hairTex && st.texCoef[3 * (size_t)NR + ri] != 0;
        const float4 hairTc = hairTex && !hairTexR ? make_float4(st.texCoef[ri], st.texCoef[(size_t)NR + ri],
                                                                 st.texCoef[2 * (size_t)NR + ri], 0.f)
                                                   : make_float4(0.f, 0.f, 0.f, 0.f);
        {
            SpectralIter it(lambda0);
#pragma unroll 1
            for (int i = 0; i < kNS; ++i, it.Next()) {
                if (meas) {  // MeasuredBxDF keeps the wavelengths (its spectra are per lambda)
                    sp.b[i] = it.lam;
                    continue;
                }
                if (hair) {
                    const float q = !hairTex ? SssSpectrumAt(S, hq, it.lam)
                                    : hairTexR ? st.texR[(size_t)i * NR + ri]
                                               : SigmoidPolynomial(hairTc.x, hairTc.y, hairTc.z, it.lam);
                    sp.a[i] = L0.x == 0 ? (q > 0 ? q : 0.f) : HairSigmaAFromReflectance(Clampf(q, 0, 1), hairDen);
                    continue;
                }
                if (dt) {
                    // DiffuseTransmissionMaterial::GetBxDF: Clamp(scale * R, 0, 1), likewise T
                    const float r = constant ? mc.w : SigmoidPolynomial(mc.x, mc.y, mc.z, it.lam);
                    const float t = L2.x != 0 ? L1.w : SigmoidPolynomial(L1.x, L1.y, L1.z, it.lam);
                    sp.a[i] = Clampf(mp4.w * r, 0, 1);
                    sp.alb[i] = Clampf(mp4.w * t, 0, 1);
                    prMax = i == 0 ? sp.a[i] : fmaxf(prMax, sp.a[i]);
                    ptMax = i == 0 ? sp.alb[i] : fmaxf(ptMax, sp.alb[i]);
                    continue;
                }
                if (!conductor) {
                    sp.a[i] = Reflectance(mc, constant, it.lam);
                    bottomNz |= sp.a[i] != 0;
                } else {
                    float e, k;
                    if (etaSpec >= 0) {
                        const int a = S.plOffsets[etaSpec], na = S.plOffsets[etaSpec + 1] - a;
                        const int b = S.plOffsets[kSpec], nb = S.plOffsets[kSpec + 1] - b;
                        e = PiecewiseLinearEval(S.plLambda + a, S.plValue + a, na, it.lam);
                        k = PiecewiseLinearEval(S.plLambda + b, S.plValue + b, nb, it.lam);
                    } else {
                        const float r = Clampf(SigmoidPolynomial(mc.x, mc.y, mc.z, it.lam), 0, .9999f);
                        e = 1.f;
                        k = 2 * std::sqrt(r) / std::sqrt(std::fmax(0.f, 1 - r));
                    }
                    sp.a[i] = e / ieta;
                    sp.b[i] = k / ieta;
                }
                sp.alb[i] = Reflectance(L1, L2.x != 0, it.lam);
                albNz |= sp.alb[i] != 0;
            }
        }
        TrowbridgeReitz trTop{mp4.x, mp4.y}, trBot{L2.y, L2.z};
        if (retro) trBot = trTop;  // the material's own (remapped, clamped) alphas
        if (S.regularize && (flags & 2)) {  // surfscatter.cpp:127-128, LayeredBxDF::Regularize
            trTop.Regularize();
            trBot.Regularize();
        }
        const LayeredBxDF<LayerSpec> L{ieta,         trTop, trBot, conductor, fmaxf(L0.x, 1.17549435e-38f),
                                       Clampf(L0.y, -1, 1), albNz, (int)L0.z,  (int)L0.w, 0, sp, bottomNz};
        const DiffuseTransmission<LayerSpec> D{sp, prMax, ptMax};
        HairState H{};
        if (hair) H = MakeHair(-1 + 2 * si.uv[1], hairEta, hairBm, hairBn, hairAlpha);
        // MeasuredMaterial::GetBxDF (materials.h:931-934): the BRDF's tables (matLayer: its index)
        MeasuredView M{};
        if (meas) {
            const int *mh = S.measHdr + kMeasHdr * (int)L0.x;
            M = MeasuredAt(mh, S.measData + mh[7]);
        }
        const int bflags = (hair || meas) ? (kBxGlossy | kBxReflection) : retro ? RetroFlags(trBot) : dt ? D.Flags() : L.LayerFlags();
        const Frame frame = Frame::FromXZ(Normalize(si.dpdus), si.ns);
        const V3 woL = frame.ToLocal(wo3);
        float fo[kNS];
        // ---- light sampling + shadow ray (surfscatter.cpp:252-326): reflective, not transmissive
        if (bflags & (kBxDiffuse | kBxGlossy)) {
            const bool refl = bflags & kBxReflection, trans = bflags & kBxTransmission;
            V3 cp = si.p, cpErr = si.pErr;  // LightSampleContext: the offset point is exact
            if (refl && !trans) cp = OffsetRayOrigin(si.p, si.pErr, si.n, wo3), cpErr = V3(0, 0, 0);
            else if (refl && trans) cp = OffsetRayOrigin(si.p, si.pErr, si.n, -wo3), cpErr = V3(0, 0, 0);
            AreaLightHit ls;
            if (SampleAreaLightAt<Ext>(S, cp, si.n, si.ns, rs.dUc, rs.dU0, rs.dU1, lambda0, &ls, cpErr) && woL.z != 0) {
                const V3 wi = ls.wi;
                const V3 wiL = frame.ToLocal(wi);
                if (hair) HairF(H, sp.a, woL, wiL, fo);
                else if (meas) MeasuredF(M, woL, wiL, sp.b, fo);
                else if (retro) {
                    const RetroTerms rt = RetroEval(trBot, woL, wiL);
#pragma unroll 1
                    for (int i = 0; i < kNS; ++i) fo[i] = rt.ok ? RetroF(rt, sp.a[i], sp.b[i]) : 0.f;
                }
                else if (dt) D.f(woL, wiL, fo);
                else L.f(woL, wiL, true, fo);
                bool fnz = false;
#pragma unroll 1
                for (int i = 0; i < kNS; ++i) fnz |= fo[i] != 0;
                if (fnz) {
                    const float bsdfPDF = ls.delta ? 0.f
                                          : hair ? HairPDF(H, sp.a, woL, wiL)
                                          : meas ? MeasuredPDF(M, woL, wiL)
                                          : retro ? RetroPDF(trBot, woL, wiL)
                                          : dt   ? D.PDF(woL, wiL)
                                                 : L.PDF(woL, wiL, true);
                    const float absdot = AbsDotN(si.ns, wi);
                    const V3 so = OffsetRayOrigin(si.p, si.pErr, si.n, ls.p - si.p);
                    const V3 pt = OffsetRayOrigin(ls.p, ls.pErr, ls.n, so - ls.p);
                    const V3 sd = pt - so;
                    bool ldUni = true;
                    SpectralIter it(lambda0);
#pragma unroll 1
                    for (int i = 0; i < kNS; ++i, it.Next()) {
                        const float Le = ls.Le(S, DenseOffset(it.lam), it.lam);
                        fo[i] = betaIn(i) * fo[i] * absdot * Le;
                        ldUni &= FloatToBits(fo[i]) == FloatToBits(fo[0]);
                    }
                    const int js = ShardSlot(shardBase, WavePush(shadowCnt, true), st.capS, st.NR);
                    v.shLd[js] = fo[0];
#pragma unroll 1
                    for (int i = 1; i < kNS; ++i)
                        if (!ldUni) v.shLd[(size_t)i * NR + js] = fo[i];
                    v.shRu[js] = ruIn.v0 * bsdfPDF;
                    v.shRl[js] = ruIn.v0 * ls.pdf;
                    if (!ruUni) {
#pragma unroll 1
                        for (int i = 1; i < kNS; ++i) {
                            const float ru = ruIn(i);
                            v.shRu[(size_t)i * NR + js] = ru * bsdfPDF;
                            v.shRl[(size_t)i * NR + js] = ru * ls.pdf;
                        }
                    }
                    v.shFlags[js] = (ldUni ? kShUniLd : 0) | (ruUni ? kShUniRu | kShUniRl : 0);
                    StoreV3(v.shRay, NR, js, so);
                    StoreV3(v.shRay + 3 * (size_t)NR, NR, js, sd);
                    v.shLambda0[js] = lambda0;
                    v.shPixel[js] = slot;
                    v.shMedium[js] = DotN(si.n, sd) > 0 ? mOut : mIn;
                }
            }
        }
        // ---- BSDF::Sample_f + RR + indirect ray (surfscatter.cpp:170-250)
        if (woL.z == 0) continue;
        LayerSample bs;
        if (hair) {
            bs.pdfIsProportional = false;
            bs.flags = kBxGlossy | kBxReflection;
            bs.ok = HairSampleF(H, sp.a, woL, rs.iUc, rs.iU0, rs.iU1, &bs.wi, &bs.pdf, fo);
        } else if (meas) {
            bs.pdfIsProportional = false;
            bs.flags = kBxGlossy | kBxReflection;
            bs.ok = MeasuredSampleF(M, woL, rs.iU0, rs.iU1, sp.b, &bs.wi, &bs.pdf, fo);
        } else if (retro) {
            const ConductorTerms ct = RetroSample(trBot, woL, rs.iU0, rs.iU1);
            bs.pdfIsProportional = false;
            bs.flags = kBxReflection | (ct.specular ? kBxSpecular : kBxGlossy);
            bs.ok = ct.ok;
            bs.wi = ct.wi;
            bs.pdf = ct.pdf;
#pragma unroll 1
            for (int i = 0; i < kNS; ++i) fo[i] = ct.ok ? ConductorF(ct, sp.a[i], sp.b[i]) : 0.f;
        } else if (dt) {
            bs.pdfIsProportional = false;
            bs.ok = D.Sample_f(woL, rs.iUc, rs.iU0, rs.iU1, &bs.wi, &bs.pdf, &bs.flags, fo);
        } else {
            bs = L.Sample_f(woL, rs.iUc, rs.iU0, rs.iU1, true, fo);
        }
        if (!bs.ok || bs.pdf == 0 || bs.wi.z == 0) continue;
        bool fAny = false;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) fAny |= fo[i] != 0;
        if (!fAny) continue;
        const V3 wi = frame.FromLocal(bs.wi);
        const float absdot = AbsDotN(si.ns, wi);
        // BSDF::PDF(wo, wi) takes wi back to the local frame (bsdf.h:118-125)
        const float pdfP = bs.pdfIsProportional ? L.PDF(woL, frame.ToLocal(wi), true) : bs.pdf;
        const float etaScale = rec.etaScale[ri];  // the layered / diffuse sample's eta is 1
        float rus = 0;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) rus = i == 0 ? ruIn.v0 : rus + ruIn(i);
        const float avgRu = rus / kNS;
        float mx = -kInfinity;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) {
            fo[i] = betaIn(i) * fo[i] * absdot / bs.pdf;
            mx = fmaxf(mx, fo[i] * etaScale / avgRu);
        }
        const bool rrOn = mx < 1 && depth >= 1;
        float q = 0;
        if (rrOn) {
            q = fmaxf(0.f, 1 - mx);
            if (rs.rr < q) continue;
        }
        bool nz = false, nbUni = true;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) {
            if (rrOn) fo[i] /= 1 - q;
            nz |= fo[i] != 0;
            nbUni &= FloatToBits(fo[i]) == FloatToBits(fo[0]);
        }
        if (!nz) continue;
        const bool specular = bs.flags & kBxSpecular;
        const int jn = ShardSlot(shardBase, WavePush(nextCnt, true), st.capS, st.NR);
        out.beta[jn] = fo[0];
        out.ru[jn] = ruIn.v0;
        out.rl[jn] = ruIn.v0 / pdfP;
#pragma unroll 1
        for (int i = 1; i < kNS; ++i) {
            if (!nbUni) out.beta[(size_t)i * NR + jn] = fo[i];
            if (!ruUni) {
                const float ru = ruIn(i);
                out.ru[(size_t)i * NR + jn] = ru;
                out.rl[(size_t)i * NR + jn] = ru / pdfP;
            }
        }
        StoreV3(out.ray, NR, jn, OffsetRayOrigin(si.p, si.pErr, si.n, wi));
        StoreV3(out.ray + 3 * (size_t)NR, NR, jn, wi);
        StoreV3(out.prev, NR, jn, si.p);
        StoreV3(out.prev + 3 * (size_t)NR, NR, jn, si.pErr);
        StoreV3(out.prev + 6 * (size_t)NR, NR, jn, si.n);
        StoreV3(out.prev + 9 * (size_t)NR, NR, jn, si.ns);
        out.lambda0[jn] = lambda0;
        out.etaScale[jn] = etaScale;
        out.flags[jn] = (specular ? 1 : 0) | ((!specular || (flags & 2)) ? 2 : 0) | (nbUni ? kUniBeta : 0) |
                        (ruUni ? kUniRu | kUniRl : 0);
        out.pixel[jn] = slot;
        out.depth[jn] = depth + 1;
        out.medium[jn] = DotN(si.n, wi) > 0 ? mOut : mIn;
    }
}

// SampleMediumScattering<HGPhaseFunction> (media.cpp:259-352)
template <bool Ext>
__global__ void __launch_bounds__(kBlock, PBRT_VOL_WAVES) k_vscatter(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView scat = LoadQueue(st, wf, kVScat);
    const int NR = st.NR;
    const VolRecords &rec = v.rec[wf & 1];
    const int shard = ProducerShard();
    const int shardBase = shard * st.capS;
    int *nextCnt = &st.counters[CounterIndex(wf + 1, kVRay, shard)];
    int *shadowCnt = &st.counters[CounterIndex(wf, kVShadow, shard)];
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < scat.total; j += gridDim.x * blockDim.x) {
        const int ri = v.scatQ[QueueSlot(scat, j)];
        const float lambda0 = rec.lambda0[ri];
        const int slot = rec.pixel[ri], depth = rec.depth[ri], medium = rec.medium[ri];
        const WaveOffsets wo(lambda0);
        const int inFlags = rec.flags[ri];
        float beta[kNS], ru[kNS];
        LoadSpec(rec.beta, NR, ri, beta, inFlags & kUniBeta);
        LoadSpec(rec.ru, NR, ri, ru, inFlags & kUniRu);
        const V3 pS = LoadV3(v.hitB, NR, ri);
        const V3 wo3 = -LoadV3(rec.ray + 3 * (size_t)NR, NR, ri);
        const float g = MediumAt(S, medium).P[0];
        const VRaySamples rs = RaySamplesAt(S, st, slot, depth);
        // direct lighting: LightSampleContext(p, n = 0, ns = 0)
        {
            AreaLightSample ls;
            float Le[kNS];
            if (SampleAreaLight<Ext>(S, pS, V3(0, 0, 0), V3(0, 0, 0), rs.dUc, rs.dU0, rs.dU1, lambda0, wo, &ls, Le)) {
                const V3 wi = ls.wi;
                const float ph = HenyeyGreenstein(Dot(wo3, wi), g);
                const float phasePDF = ls.delta ? 0.f : ph;  // IsDeltaLight (media.cpp:292-293)
                float Ld[kNS], sru[kNS], srl[kNS];
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    Ld[i] = (beta[i] * ph) * Le[i];
                    sru[i] = ru[i] * phasePDF;
                    srl[i] = ru[i] * ls.pdf;
                }
                ShadowOut so;
                so.o = pS;
                so.d = ls.p - pS;
                so.medium = medium;
                const int pos = WavePush(shadowCnt, true);
                WriteShadow(S, v, NR, ShardSlot(shardBase, pos, st.capS, st.NR), so, Ld, sru, srl, lambda0, slot);
            }
        }
        // indirect: phase-function sample, RR, next ray at depth + 1
        float pdf;
        const V3 wi = SampleHenyeyGreenstein(wo3, g, rs.iU0, rs.iU1, &pdf);
        if (pdf == 0) continue;
        const float etaScale = rec.etaScale[ri];
        float rl[kNS];
#pragma unroll
        for (int i = 0; i < kNS; ++i) {
            beta[i] = beta[i] * pdf / pdf;
            rl[i] = ru[i] / pdf;
        }
        const float avgRu = AvgArr(ru);
        float mx = -kInfinity;
#pragma unroll
        for (int i = 0; i < kNS; ++i) mx = fmaxf(mx, beta[i] * etaScale / avgRu);
        if (mx < 1 && depth >= 1) {
            const float q = fmaxf(0.f, 1 - mx);
            if (rs.rr < q) continue;
#pragma unroll
            for (int i = 0; i < kNS; ++i) beta[i] /= 1 - q;
        }
        const int pos = WavePush(nextCnt, true);
        const int jn = ShardSlot(shardBase, pos, st.capS, st.NR);
        const VolRecords &out = v.rec[(wf + 1) & 1];
        int uni = StoreSpec(out.beta, NR, jn, beta) ? kUniBeta : 0;
        uni |= StoreSpec(out.ru, NR, jn, ru) ? kUniRu : 0;
        uni |= StoreSpec(out.rl, NR, jn, rl) ? kUniRl : 0;
        StoreV3(out.ray, NR, jn, pS);
        StoreV3(out.ray + 3 * (size_t)NR, NR, jn, wi);
        StoreV3(out.prev, NR, jn, pS);
#pragma unroll
        for (int k = 3; k < 12; ++k) out.prev[(size_t)k * NR + jn] = 0.f;
        out.lambda0[jn] = lambda0;
        out.etaScale[jn] = etaScale;
        out.flags[jn] = 2 | uni;  // specularBounce = false, anyNonSpecularBounces = true
        out.pixel[jn] = slot;
        out.depth[jn] = depth + 1;
        out.medium[jn] = medium;
    }
}

// TraceTransmittance (wavefront/intersect.h:164-274) for one shadow ray: closest hits up to the
// light point ray(tMax); a non-interface surface blocks (returns false), interfaces are crossed
// (SpawnRayTo the light point), and in each medium T_ray / r_u / r_l follow ratio tracking with
// RR on a small T_ray.  Tr, tu, tl start at 1 (the caller's arrays).
template <int TM>
__device__ __forceinline__ bool TraceTransmittanceRay(const DeviceScene &S, const SceneLds &L, V3 o, V3 d, float tMax,
                                                      int med, const WaveOffsets &wo, float *Tr, float *tu, float *tl) {
    const V3 pLight = o + d * tMax;
    PCG32 rng(HashV3(o), HashV3(d));
    float Tm[kNS];
    for (int guard = 0; guard < 256; ++guard) {
        if (d == V3(0, 0, 0)) break;
        TriHit h;
        const int hp = Traverse<false, TM>(S, L, o, d, tMax, &h);
        if (hp >= 0 && S.matType[S.primMaterial[hp]] != 3) return false;
        TriSurface hs{};
        if (hp >= 0) {
            V3 p0, p1, p2;
            PrimVerts(S, hp, &p0, &p1, &p2);
            hs = SurfaceAt<(TM & kTravShapes) != 0>(S, hp, p0, p1, p2, h.b0, h.b1, h.b2);
        }
        if (med >= 0) {
            const MediumRef m = MediumAt(S, med);
            const int sa = m.I[1], ss = m.I[2];
            const float tEnd = hp < 0 ? tMax : (Length(o - hs.p) / Length(d));
            auto event = [&](V3, const MediumPoint &mp, float mx, const float *T) __attribute__((always_inline)) -> bool {
                float sn[kNS], smj[kNS];
                SpectralIter it(wo.lam0);
#pragma unroll
                for (int i = 0; i < kNS; ++i, it.Next()) {
                    smj[i] = (DenseAt(S, sa, wo.off[i]) + DenseAt(S, ss, wo.off[i])) * mx;
                    sn[i] = fmaxf(0.f, smj[i] - MediumSigmaA(S, m, mp, wo.off[i], it.lam) - MediumSigmaS(S, m, mp, wo.off[i], it.lam));
                }
                const float pr = T[0] * smj[0];
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    Tr[i] *= T[i] * sn[i] / pr;
                    tl[i] *= T[i] * smj[i] / pr;
                    tu[i] *= T[i] * sn[i] / pr;
                }
                // T_ray / (r_l + r_u).Average() < 0.05: Russian roulette
                float den[kNS];
#pragma unroll
                for (int i = 0; i < kNS; ++i) den[i] = tl[i] + tu[i];
                const float avg = AvgArr(den);
                float mxT = -kInfinity;
#pragma unroll
                for (int i = 0; i < kNS; ++i) mxT = fmaxf(mxT, Tr[i] / avg);
                if (mxT < 0.05f) {
                    const float q = 0.75f;
                    if (rng.Uniform() < q) {
#pragma unroll
                        for (int i = 0; i < kNS; ++i) Tr[i] = 0.f;
                    } else {
#pragma unroll
                        for (int i = 0; i < kNS; ++i) Tr[i] /= 1 - q;
                    }
                }
                return AnyNonZero(Tr);
            };
            const bool ranOut = SampleTmaj(S, m, wo, o, d, tEnd, rng.Uniform(), rng, Tm, event);
            if (ranOut) {
                const float t0 = Tm[0];
#pragma unroll
                for (int i = 0; i < kNS; ++i) {
                    const float f = Tm[i] / t0;
                    Tr[i] *= f;
                    tl[i] *= f;
                    tu[i] *= f;
                }
            }
        }
        if (hp < 0 || !AnyNonZero(Tr)) break;
        // SurfaceInteraction::SpawnRayTo(pLight) (interaction.h, ray.h:98-104)
        int mIn, mOut;
        MediaOf(S, hp, med, &mIn, &mOut);
        const V3 dd = pLight - hs.p;
        o = OffsetRayOrigin(hs.p, hs.pErr, hs.n, dd);
        d = dd;
        med = DotN(hs.n, d) > 0 ? mOut : mIn;
    }
    return true;
}

template <int TM>
__global__ void __launch_bounds__(kBlock, PBRT_VOL_WAVES) k_vshadow(DeviceScene S, PathState st, VolState v, int wf) {
    const QueueView sh = LoadQueue(st, wf, kVShadow);
    if ((int)(blockIdx.x * blockDim.x) >= sh.total) return;
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int NR = st.NR;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[2], (unsigned long long)sh.total);
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < sh.total; j += gridDim.x * blockDim.x) {
        const int p = QueueSlot(sh, j);
        const V3 o = LoadV3(v.shRay, NR, p), d = LoadV3(v.shRay + 3 * (size_t)NR, NR, p);
        const WaveOffsets wo(v.shLambda0[p]);
        float Tr[kNS], tu[kNS], tl[kNS];
#pragma unroll
        for (int i = 0; i < kNS; ++i) Tr[i] = tu[i] = tl[i] = 1.f;
        if (!TraceTransmittanceRay<TM>(S, L, o, d, 1 - kShadowEpsilon, v.shMedium[p], wo, Tr, tu, tl) || !AnyNonZero(Tr))
            continue;
        float Ld[kNS], den[kNS];
        const int shf = v.shFlags[p];
        {
            float ru[kNS], rl[kNS];
            LoadSpec(v.shRu, NR, p, ru, shf & kShUniRu);
            LoadSpec(v.shRl, NR, p, rl, shf & kShUniRl);
#pragma unroll
            for (int i = 0; i < kNS; ++i) den[i] = ru[i] * tu[i] + rl[i] * tl[i];
        }
        LoadSpec(v.shLd, NR, p, Ld, shf & kShUniLd);
        const float avg = AvgArr(den);
        AddToL(S, st, v.shPixel[p], wo, [&](int i) { return Ld[i] * Tr[i] / avg; });
    }
}

// WavefrontAggregate::IntersectShadowTr (wavefront/integrator.h:49-51) over a caller's SoA batch:
// rays [7][n] o, d, tMax; the ray's medium (-1: none) and the path's first wavelength (the
// other 30 by SampleUniform's +10 nm stratification, as every SampledWavelengths of this
// wavefront); out [3][31][n] = T_ray, r_u, r_l of TraceTransmittance after the ray reached the
// light point (T_ray all 0 when a surface blocks it).  The caller scales its Ld by
// T_ray / avg(sr.r_u * r_u + sr.r_l * r_l) (intersect.h:262-266).
template <int TM>
__global__ void __launch_bounds__(kBlock, PBRT_VOL_WAVES) k_intersect_tr(DeviceScene S, const float *rays, const int *medium,
                                                                      const float *lambda0, int n, float *out) {
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < n; r += gridDim.x * blockDim.x) {
        const V3 o(rays[r], rays[n + r], rays[2 * n + r]), d(rays[3 * n + r], rays[4 * n + r], rays[5 * n + r]);
        const WaveOffsets wo(lambda0[r]);
        float Tr[kNS], tu[kNS], tl[kNS];
#pragma unroll
        for (int i = 0; i < kNS; ++i) Tr[i] = tu[i] = tl[i] = 1.f;
        int med = medium ? medium[r] : -1;
        med = med >= 0 && med < S.media.n ? med : -1;  // outside the scene's media: vacuum
        if (!TraceTransmittanceRay<TM>(S, L, o, d, rays[6 * n + r], med, wo, Tr, tu, tl))
            for (int i = 0; i < kNS; ++i) Tr[i] = 0.f;
        for (int i = 0; i < kNS; ++i) {
            out[(size_t)i * n + r] = Tr[i];
            out[(size_t)(kNS + i) * n + r] = tu[i];
            out[(size_t)(2 * kNS + i) * n + r] = tl[i];
        }
    }
}

// TraceTransmittance when every medium is grey: T_ray, r_u and r_l start at 1 and only ever
// take factors that are equal at all wavelengths, so each is one scalar (the reference's 31
// entries are 31 copies of it).
template <int TM, bool Cloud>
__global__ void __launch_bounds__(kBlock, TraversalWaves(TM)) k_vshadow_grey(DeviceScene S, PathState st, VolState v,
                                                                             int wf) {
    const QueueView sh = LoadQueue(st, wf, kVShadow);
    if ((int)(blockIdx.x * blockDim.x) >= sh.total) return;
    extern __shared__ float4 dynLds[];
    const SceneLds L = SetupSceneLds(S, dynLds);
    const int NR = st.NR;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&st.stats[2], (unsigned long long)sh.total);
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < sh.total; j += gridDim.x * blockDim.x) {
        const int p = QueueSlot(sh, j);
        V3 o = LoadV3(v.shRay, NR, p), d = LoadV3(v.shRay + 3 * (size_t)NR, NR, p);
        int med = v.shMedium[p];
        const float lambda0 = v.shLambda0[p];
        const float tMax = 1 - kShadowEpsilon;
        const V3 pLight = o + d * tMax;
        PCG32 rng(HashV3(o), HashV3(d));
        float Tr = 1.f, tu = 1.f, tl = 1.f, Tm;
        bool blocked = false;
        for (int guard = 0; guard < 256; ++guard) {
            if (d == V3(0, 0, 0)) break;
            TriHit h;
            const int hp = Traverse<false, TM>(S, L, o, d, tMax, &h);
            if (hp >= 0 && S.matType[S.primMaterial[hp]] != 3) {
                blocked = true;
                break;
            }
            TriSurface hs{};
            if (hp >= 0) {
                V3 p0, p1, p2;
                PrimVerts(S, hp, &p0, &p1, &p2);
                hs = SurfaceAt<(TM & kTravShapes) != 0>(S, hp, p0, p1, p2, h.b0, h.b1, h.b2);
            }
            if (med >= 0) {
                const MediumRef m = MediumAt(S, med);
                const int sa = m.I[1], ss = m.I[2];
                const float tEnd = hp < 0 ? tMax : (Length(o - hs.p) / Length(d));
                const int off0 = DenseOffset(lambda0);
                const float sa0 = DenseAt(S, sa, off0), ss0 = DenseAt(S, ss, off0);
                auto event = [&](V3, const MediumPoint &mp, float smaj, float T) __attribute__((always_inline)) -> bool {
                    const float sn = fmaxf(0.f, smaj - sa0 * mp.d - ss0 * mp.d);
                    const float pr = T * smaj;
                    Tr *= T * sn / pr;
                    tl *= T * smaj / pr;
                    tu *= T * sn / pr;
                    if (Tr / Avg31(tl + tu) < 0.05f) {  // T_ray / (r_l + r_u).Average(): RR
                        const float q = 0.75f;
                        if (rng.Uniform() < q) Tr = 0.f;
                        else Tr /= 1 - q;
                    }
                    return Tr != 0;
                };
                const bool ranOut = SampleTmajGrey<Cloud>(S, m, sa0 + ss0, o, d, tEnd, rng.Uniform(), rng, Tm, event);
                if (ranOut) {
                    const float f = Tm / Tm;
                    Tr *= f;
                    tl *= f;
                    tu *= f;
                }
            }
            if (hp < 0 || Tr == 0) break;
            // SurfaceInteraction::SpawnRayTo(pLight) (interaction.h, ray.h:98-104)
            int mIn, mOut;
            MediaOf(S, hp, med, &mIn, &mOut);
            const V3 dd = pLight - hs.p;
            o = OffsetRayOrigin(hs.p, hs.pErr, hs.n, dd);
            d = dd;
            med = DotN(hs.n, d) > 0 ? mOut : mIn;
        }
        if (blocked || Tr == 0) continue;
        // L += Ld T_ray / (r_u tu + r_l tl).Average(): rolled passes, no 31-wide arrays
        const int shf = v.shFlags[p];
        const SpecIn ruIn(v.shRu, NR, p, shf & kShUniRu), rlIn(v.shRl, NR, p, shf & kShUniRl),
            ldIn(v.shLd, NR, p, shf & kShUniLd);
        float denSum = 0;
#pragma unroll 1
        for (int i = 0; i < kNS; ++i) {
            const float dv = ruIn(i) * tu + rlIn(i) * tl;
            denSum = i == 0 ? dv : denSum + dv;
        }
        const float avg = denSum / kNS;
        const int slot = v.shPixel[p], NL = st.N;
        if (shf & kShRgb) {
            const float q = Tr / avg;
            st.L[slot] += S.imagingRatio * ((v.shLd[p] * q) / kNS);
            st.L[NL + slot] += S.imagingRatio * ((v.shLd[NR + p] * q) / kNS);
            st.L[2 * NL + slot] += S.imagingRatio * ((v.shLd[2 * (size_t)NR + p] * q) / kNS);
            AddL0Off(S, st, slot, DenseOffset(lambda0), v.shLd[3 * (size_t)NR + p] * Tr / avg);
            continue;
        }
        SensorAcc acc;
        SpectralIter it(lambda0);
#pragma unroll 1
        for (int i = 0; i < kNS; ++i, it.Next()) acc.Add(S, DenseOffset(it.lam), ldIn(i) * Tr / avg, i == 0);
        st.L[slot] += S.imagingRatio * (acc.sx / kNS);
        st.L[NL + slot] += S.imagingRatio * (acc.sy / kNS);
        st.L[2 * NL + slot] += S.imagingRatio * (acc.sz / kNS);
        AddL0Off(S, st, slot, DenseOffset(lambda0), ldIn(0) * Tr / avg);
    }
}

// Diagnostic (PBRT_AMD_QUEUE_CHECK=1): queue slots that a stage counted but never wrote.  The
// launcher fills the slots' pixel field with -1 before the surface stage; afterwards every
// counted slot must hold a pixel index.  Holes are counted into the context's counter and the
// first few printed with their queue and shard; the check only reads.  The launcher then waits
// for the check and, when it found a hole, stops the iteration before any stage consumes the
// unwritten records (LaunchVolIteration returns hipErrorIllegalState; capi.hip raises it).
__global__ void k_queue_holes(const int *counters, int wf, int queue, const int *pixel, int capS, int *hole,
                              int stage) {
    const int shard = blockIdx.y;
    const int n = min(counters[CounterIndex(wf, queue, shard)], capS);  // past capS: k_queue_overflow
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (pixel[shard * capS + i] < 0) {
            const int k = atomicAdd(hole, 1);
            if (k < 8)
                printf("queue hole after stage %d: iteration %d queue %d shard %d slot %d of %d\n", stage, wf, queue,
                       shard, i, n);
        }
    }
}
// One queue's shard counters against the shard capacity (k_queue_overflow's test), for a queue
// whose counters are reset within the pass (the subsurface stage's shadow queue)
__global__ void k_shard_overflow(PathState st, int depth, int queue) {
    const int s = threadIdx.x;
    if (s < kShards && st.counters[CounterIndex(depth, queue, s)] > st.capS)
        atomicAdd(&st.stats[kStatQueueOverflow], 1ull);
}
static int g_queueCheck = -1;  // -1: PBRT_AMD_QUEUE_CHECK decides on first use
static int g_holesFound = 0;   // holes the checks found since the last TakeQueueHoles (host)
static bool QueueCheckOn() {
    if (g_queueCheck < 0) {
        const char *e = getenv("PBRT_AMD_QUEUE_CHECK");
        g_queueCheck = e && e[0] == '1' ? 1 : 0;
    }
    return g_queueCheck == 1;
}
// after the checks of one iteration: their hole count (the counter is reset), or -1 on a HIP error
static int CollectQueueHoles(const VolState &v, hipStream_t s) {
    int h = 0;
    if (hipStreamSynchronize(s) != hipSuccess) return -1;
    if (hipMemcpy(&h, v.holes, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (h && hipMemset(v.holes, 0, sizeof(int)) != hipSuccess) return -1;
    g_holesFound += h;
    return h;
}
void SetQueueCheck(int on) { g_queueCheck = on ? 1 : 0; }
// holes found since the last call (the count is reset); 0 when the check never ran
int TakeQueueHoles() {
    const int h = g_holesFound;
    g_holesFound = 0;
    return h;
}

// ------------------------------------------------------------------ launch helpers (host)
size_t TraversalLdsBytes(int stackSize, int ldsNodes, int ldsTris, int compressed);
size_t VolTraversalStaticLds(int tm) {
    size_t m = 0;
    auto take = [&](const void *f) {
        hipFuncAttributes a{};
        if (hipFuncGetAttributes(&a, f) == hipSuccess) m = std::max(m, (size_t)a.sharedSizeBytes);
    };
#define TAKE_TM(TM)                                                      \
    if (tm == TM) {                                                      \
        take(reinterpret_cast<const void *>(&k_vclosest<TM>));           \
        take(reinterpret_cast<const void *>(&k_vclosest<TM, true>));     \
        take(reinterpret_cast<const void *>(&k_vshadow_grey<TM, false>)); \
        take(reinterpret_cast<const void *>(&k_vshadow_grey<TM, true>));  \
        take(reinterpret_cast<const void *>(&k_vshadow<TM>));            \
    }
    TAKE_TM(kTravLds) TAKE_TM(kTravWide) TAKE_TM(kTravQuant)
#undef TAKE_TM
    return m;
}
static size_t VolStackBytes(const DeviceScene &S) {
    return TraversalLdsBytes(S.stackSize, S.ldsNodes, S.ldsTris, S.compressed);
}
static int VolGrid(int n, int cap) {
    int g = (n + kBlock - 1) / kBlock;
    g = g < 1 ? 1 : (g > cap ? cap : g);
    return (g + kShards - 1) / kShards * kShards;  // producer grids: multiples of kShards
}

hipError_t LaunchIntersectTr(const DeviceScene &S, const float *rays, const int *medium, const float *lambda0, int n,
                            float *out, hipStream_t s) {
    const int g = std::max(1, std::min(4096, (n + kBlock - 1) / kBlock));
#define K_TR(tm) k_intersect_tr<tm>
    PBRT_LAUNCH_TRAVERSAL(S, K_TR, dim3(g), dim3(kBlock), VolStackBytes(S), s, S, rays, medium, lambda0, n, out);
#undef K_TR
    return hipGetLastError();
}

hipError_t LaunchIntersectOneRandom(const DeviceScene &S, const float *segs, const int *mats, int n, int *prim,
                                    float *hit, float *pdf, hipStream_t s) {
    const int g = std::max(1, std::min(4096, (n + kBlock - 1) / kBlock));
#define K_OR(tm) k_intersect_one_random<tm>
    PBRT_LAUNCH_TRAVERSAL(S, K_OR, dim3(g), dim3(kBlock), VolStackBytes(S), s, S, segs, mats, n, prim, hit, pdf);
#undef K_OR
    return hipGetLastError();
}

hipError_t LaunchVolCamera(const DeviceScene &S, const PathState &st, const VolState &v, int nActive, hipStream_t s) {
    hipLaunchKernelGGL(k_vcamera, dim3((nActive + kBlock - 1) / kBlock), dim3(kBlock), 0, s, S, st, v, nActive);
    return hipGetLastError();
}
hipError_t LaunchVolClosest(const DeviceScene &S, const PathState &st, const VolState &v, int wf, int maxCount,
                            int timed, hipStream_t s) {
    const dim3 block(kBlock), gT(VolGrid(maxCount, PBRT_GRID_CAP));
    if (st.hitMat[0]) {
#define K_VCLOSEST(tm) k_vclosest<tm, true>
        PBRT_LAUNCH_TRAVERSAL(S, K_VCLOSEST, gT, block, VolStackBytes(S), s, S, st, v, wf, timed);
#undef K_VCLOSEST
    } else {
#define K_VCLOSEST(tm) k_vclosest<tm>
        PBRT_LAUNCH_TRAVERSAL(S, K_VCLOSEST, gT, block, VolStackBytes(S), s, S, st, v, wf, timed);
#undef K_VCLOSEST
    }
    return hipGetLastError();
}
// TraceShadowRays (integrator.cpp:575-586) of iteration wf: the queued shadow rays, through
// media when the scene has any
static void LaunchVolShadows(const DeviceScene &S, const PathState &st, const VolState &v, int wf, dim3 gT,
                             hipStream_t s) {
    const dim3 block(kBlock);
    if (S.media.allGrey && S.media.hasCloud) {
#define K_VSHADOW_GREY(tm) k_vshadow_grey<tm, true>
        PBRT_LAUNCH_TRAVERSAL(S, K_VSHADOW_GREY, gT, block, VolStackBytes(S), s, S, st, v, wf);
#undef K_VSHADOW_GREY
    } else if (S.media.allGrey) {
#define K_VSHADOW_GREY(tm) k_vshadow_grey<tm, false>
        PBRT_LAUNCH_TRAVERSAL(S, K_VSHADOW_GREY, gT, block, VolStackBytes(S), s, S, st, v, wf);
#undef K_VSHADOW_GREY
    } else {
#define K_VSHADOW(tm) k_vshadow<tm>
        PBRT_LAUNCH_TRAVERSAL(S, K_VSHADOW, gT, block, VolStackBytes(S), s, S, st, v, wf);
#undef K_VSHADOW
    }
}

// the rest of wavefront iteration wf after its closest-hit launch
hipError_t LaunchVolIteration(const DeviceScene &S, const PathState &st, const VolState &v, int wf, int maxCount,
                              hipStream_t s) {
    const dim3 block(kBlock);
    const dim3 gT(VolGrid(maxCount, PBRT_GRID_CAP)), gW(VolGrid(maxCount, PBRT_SHADE_GRID_CAP));
    if (S.media.allGrey && S.media.hasCloud) hipLaunchKernelGGL(k_vmedium_grey<true>, gW, block, 0, s, S, st, v, wf);
    else if (S.media.allGrey) hipLaunchKernelGGL(k_vmedium_grey<false>, gW, block, 0, s, S, st, v, wf);
    else hipLaunchKernelGGL(k_vmedium, gW, block, 0, s, S, st, v, wf);
    const int layeredTypes =
        (1 << kMatCoatedDiffuseT) | (1 << kMatCoatedConductorT) | (1 << kMatDiffuseTransmissionT) | (1 << kMatHairT) |
        (1 << kMatMeasuredT) | (1 << kMatRetroreflectiveT);
    const int other = ~((1 << kMatDiffuseT) | (1 << 3) | layeredTypes);
    const size_t surfLds = VolTablesLdsBytes(S) + kNS * kBlock * sizeof(float);
    const bool qcheck = QueueCheckOn() && wf != S.maxDepth;
    if (qcheck) {
        (void)hipMemsetAsync(v.shPixel, 0xff, sizeof(int) * (size_t)st.NR, s);
        (void)hipMemsetAsync(v.rec[(wf + 1) & 1].pixel, 0xff, sizeof(int) * (size_t)st.NR, s);
    }
#define K_VSSS_PROBE(tm) k_vsss_probe<tm>
#define VOL_REST(EXT) \
    if (wf == S.maxDepth) return hipGetLastError(); \
    if (S.matTypeMask & (1 << 3)) hipLaunchKernelGGL(k_viface<EXT>, gW, block, 0, s, S, st, v, wf); \
    if (S.matTypeMask & layeredTypes) \
        hipLaunchKernelGGL(k_vlayered<EXT>, gW, block, 0, s, S, st, v, wf); \
    QUEUE_CHECK(2); \
    hipLaunchKernelGGL(k_vscatter<EXT>, gW, block, 0, s, S, st, v, wf); \
    if (S.matSss) { \
        /* the shadow rays so far first, so the subsurface exits have the queue to themselves \
           ("so that we have space for shadow rays for subsurface", integrator.cpp:427-431) */ \
        QUEUE_CHECK(5); \
        LaunchVolShadows(S, st, v, wf, gT, s); \
        /* the counts are about to be reset: check them against the shard capacity now (the \
           pass-end k_queue_overflow would see only the exits' counts) */ \
        hipLaunchKernelGGL(k_shard_overflow, dim3(1), dim3(64), 0, s, st, wf, kVShadow); \
        (void)hipMemsetAsync(st.counters + CounterIndex(wf, kVShadow, 0), 0, sizeof(int) * kShards * kCounterPad, s); \
        if (qcheck) /* the exits' slots start unwritten again (QUEUE_CHECK(3) finds holes) */ \
            (void)hipMemsetAsync(v.shPixel, 0xff, sizeof(int) * (size_t)st.NR, s); \
        PBRT_LAUNCH_TRAVERSAL(S, K_VSSS_PROBE, gT, block, VolStackBytes(S), s, S, st, v, wf); \
        hipLaunchKernelGGL(k_vsss_scatter<EXT>, gW, block, VolTablesLdsBytes(S), s, S, st, v, wf); \
    } \
    QUEUE_CHECK(3);
#define QUEUE_CHECK(stage)                                                                                          \
    if (qcheck)                                                                                                     \
        hipLaunchKernelGGL(k_queue_holes, dim3(64, kShards), block, 0, s, st.counters, wf, kVShadow, v.shPixel,      \
                           st.capS, v.holes, stage);
    // Ext: analytic shapes or image lights in the scene (their paths compiled in)
    if (S.nShapes > 0 || S.nEnv > 0 || S.nImageDelta > 0 || S.hasSpread || S.nImageAreaLights > 0) {
        if (S.textured) {
            if (S.matHairTex || S.matSssTex) hipLaunchKernelGGL((k_vtexture<true, true>), gW, block, 0, s, S, st, v, wf);
            else hipLaunchKernelGGL(k_vtexture<true>, gW, block, 0, s, S, st, v, wf);
            if (S.matTypeMask & other) hipLaunchKernelGGL((k_vsurface<false, true, true>), gW, block, surfLds, s, S, st, v, wf);
            else hipLaunchKernelGGL((k_vsurface<true, true, true>), gW, block, surfLds, s, S, st, v, wf);
        } else if (S.matTypeMask & other) {
            hipLaunchKernelGGL((k_vsurface<false, true>), gW, block, surfLds, s, S, st, v, wf);
        } else {
            hipLaunchKernelGGL((k_vsurface<true, true>), gW, block, surfLds, s, S, st, v, wf);
        }
        QUEUE_CHECK(1);
        if (S.nInfinite > 0) hipLaunchKernelGGL(k_vescaped<true>, gW, block, VolTablesLdsBytes(S), s, S, st, v, wf);
        VOL_REST(true);
    } else {
        if (S.textured) {
            if (S.matHairTex || S.matSssTex) hipLaunchKernelGGL((k_vtexture<false, true>), gW, block, 0, s, S, st, v, wf);
            else hipLaunchKernelGGL(k_vtexture<false>, gW, block, 0, s, S, st, v, wf);
            if (S.matTypeMask & other) hipLaunchKernelGGL((k_vsurface<false, false, true>), gW, block, surfLds, s, S, st, v, wf);
            else hipLaunchKernelGGL((k_vsurface<true, false, true>), gW, block, surfLds, s, S, st, v, wf);
        } else if (S.matTypeMask & other) {
            hipLaunchKernelGGL((k_vsurface<false, false>), gW, block, surfLds, s, S, st, v, wf);
        } else {
            hipLaunchKernelGGL((k_vsurface<true, false>), gW, block, surfLds, s, S, st, v, wf);
        }
        QUEUE_CHECK(1);
        if (S.nInfinite > 0) hipLaunchKernelGGL(k_vescaped<false>, gW, block, VolTablesLdsBytes(S), s, S, st, v, wf);
        VOL_REST(false);
    }
#undef VOL_REST
#undef K_VSSS_PROBE
    if (qcheck) {
        hipLaunchKernelGGL(k_queue_holes, dim3(64, kShards), block, 0, s, st.counters, wf + 1, kVRay,
                           v.rec[(wf + 1) & 1].pixel, st.capS, v.holes, 4);
        const int h = CollectQueueHoles(v, s);
        if (h < 0) return hipGetLastError() != hipSuccess ? hipGetLastError() : hipErrorUnknown;
        if (h > 0) return hipErrorIllegalState;  // nothing consumes the unwritten records
    }
#undef QUEUE_CHECK
    LaunchVolShadows(S, st, v, wf, gT, s);
    return hipGetLastError();
}

}  // namespace pbrt_amd
