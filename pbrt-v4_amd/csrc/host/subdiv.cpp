// Loop subdivision surfaces (Shape "loopsubdiv"): LoopSubdivide (util/loopsubdiv.cpp:132-
// 370), which pbrt's wavefront aggregate runs on the host to turn the control mesh into a
// TriangleMesh (gpu/aggregate.cpp:375-395).  The reference links faces and vertices by
// pointer; here they are indices into per-level arrays, created in the reference's order
// (even children in vertex order, then the odd edge vertices in face-edge order; four children
// per face in face order), so the output vertex and triangle order is the reference's.  Edge
// keys compare the two vertex indices (the reference compares pointers; the positions it
// derives from a key are sums that commute, and at level 0 pointer order is index order).
#include <map>
#include <vector>

#include "../core/core.h"
#include "scene.h"

namespace pbrt_amd {
namespace {

constexpr int kNone = -1;
int Next(int i) { return (i + 1) % 3; }
int Prev(int i) { return (i + 2) % 3; }

struct SDVertex {
    V3 p{0, 0, 0};
    int startFace = kNone, child = kNone;
    bool regular = false, boundary = false;
};
struct SDFace {
    int v[3] = {kNone, kNone, kNone};
    int f[3] = {kNone, kNone, kNone};
    int children[4] = {kNone, kNone, kNone, kNone};
};

struct Mesh {
    std::vector<SDVertex> V;
    std::vector<SDFace> F;
    int vnum(int face, int vert) const {
        for (int i = 0; i < 3; ++i)
            if (F[face].v[i] == vert) return i;
        throw Error("loopsubdiv: basic logic error in vnum");
    }
    int nextFace(int face, int vert) const { return F[face].f[vnum(face, vert)]; }
    int prevFace(int face, int vert) const { return F[face].f[Prev(vnum(face, vert))]; }
    int nextVert(int face, int vert) const { return F[face].v[Next(vnum(face, vert))]; }
    int prevVert(int face, int vert) const { return F[face].v[Prev(vnum(face, vert))]; }
    int otherVert(int face, int v0, int v1) const {
        for (int i = 0; i < 3; ++i)
            if (F[face].v[i] != v0 && F[face].v[i] != v1) return F[face].v[i];
        throw Error("loopsubdiv: basic logic error in otherVert");
    }
    int valence(int vert) const {
        const SDVertex &v = V[vert];
        int f = v.startFace;
        if (!v.boundary) {
            int nf = 1;
            while ((f = nextFace(f, vert)) != v.startFace) ++nf;
            return nf;
        }
        int nf = 1;
        while ((f = nextFace(f, vert)) != kNone) ++nf;
        f = v.startFace;
        while ((f = prevFace(f, vert)) != kNone) ++nf;
        return nf + 1;
    }
    void oneRing(int vert, std::vector<V3> *ring) const {
        ring->clear();
        const SDVertex &v = V[vert];
        if (!v.boundary) {
            int face = v.startFace;
            do {
                ring->push_back(V[nextVert(face, vert)].p);
                face = nextFace(face, vert);
            } while (face != v.startFace);
        } else {
            int face = v.startFace, f2;
            while ((f2 = nextFace(face, vert)) != kNone) face = f2;
            ring->push_back(V[nextVert(face, vert)].p);
            do {
                ring->push_back(V[prevVert(face, vert)].p);
                face = prevFace(face, vert);
            } while (face != kNone);
        }
    }
};

float Beta(int valence) { return valence == 3 ? 3.f / 16.f : 3.f / (8.f * valence); }
float LoopGamma(int valence) { return 1.f / (valence + 3.f / (8.f * Beta(valence))); }

V3 WeightOneRing(const Mesh &m, int vert, float beta) {
    std::vector<V3> ring;
    const int valence = m.valence(vert);
    m.oneRing(vert, &ring);
    V3 p = (1 - valence * beta) * m.V[vert].p;
    for (int i = 0; i < valence; ++i) p = p + beta * ring[i];
    return p;
}
V3 WeightBoundary(const Mesh &m, int vert, float beta) {
    std::vector<V3> ring;
    const int valence = m.valence(vert);
    m.oneRing(vert, &ring);
    V3 p = (1 - 2 * beta) * m.V[vert].p;
    p = p + beta * ring[0];
    p = p + beta * ring[valence - 1];
    return p;
}

using EdgeKey = std::pair<int, int>;
EdgeKey Edge(int a, int b) { return a < b ? EdgeKey(a, b) : EdgeKey(b, a); }

}  // namespace

void LoopSubdivideMesh(int nLevels, const std::vector<int> &indices, const std::vector<V3> &p, std::vector<V3> *P,
                       std::vector<int> *tris, std::vector<V3> *N) {
    Mesh m;
    m.V.resize(p.size());
    for (size_t i = 0; i < p.size(); ++i) m.V[i].p = p[i];
    const size_t nFaces = indices.size() / 3;
    m.F.resize(nFaces);
    for (size_t i = 0; i < nFaces; ++i)
        for (int j = 0; j < 3; ++j) {
            const int v = indices[3 * i + j];
            if (v < 0 || v >= (int)p.size()) throw Error("loopsubdiv: vertex index out of range");
            m.F[i].v[j] = v;
            m.V[v].startFace = (int)i;
        }
    // neighbour pointers: an edge seen once waits in the set; the second face links and erases it
    {
        std::map<EdgeKey, std::pair<int, int>> edges;  // key -> (face, edgeNum)
        for (size_t i = 0; i < nFaces; ++i)
            for (int e = 0; e < 3; ++e) {
                const EdgeKey k = Edge(m.F[i].v[e], m.F[i].v[Next(e)]);
                auto it = edges.find(k);
                if (it == edges.end()) {
                    edges[k] = {(int)i, e};
                } else {
                    m.F[it->second.first].f[it->second.second] = (int)i;
                    m.F[i].f[e] = it->second.first;
                    edges.erase(it);
                }
            }
    }
    for (size_t i = 0; i < p.size(); ++i) {
        SDVertex &v = m.V[i];
        if (v.startFace == kNone) throw Error("loopsubdiv: vertex " + std::to_string(i) + " is on no face");
        int f = v.startFace;
        do {
            f = m.nextFace(f, (int)i);
        } while (f != kNone && f != v.startFace);
        v.boundary = f == kNone;
        const int val = m.valence((int)i);
        v.regular = (!v.boundary && val == 6) || (v.boundary && val == 4);
    }
    std::vector<int> fs(nFaces), vs(p.size());
    for (size_t i = 0; i < nFaces; ++i) fs[i] = (int)i;
    for (size_t i = 0; i < p.size(); ++i) vs[i] = (int)i;
    for (int level = 0; level < nLevels; ++level) {
        std::vector<int> newFaces, newVertices;
        for (int v : vs) {
            SDVertex c;
            c.regular = m.V[v].regular;
            c.boundary = m.V[v].boundary;
            m.V.push_back(c);
            m.V[v].child = (int)m.V.size() - 1;
            newVertices.push_back(m.V[v].child);
        }
        for (int f : fs)
            for (int k = 0; k < 4; ++k) {
                m.F.push_back(SDFace());
                m.F[f].children[k] = (int)m.F.size() - 1;
                newFaces.push_back(m.F[f].children[k]);
            }
        // even vertices
        for (int v : vs) {
            const SDVertex &x = m.V[v];
            V3 np;
            if (!x.boundary)
                np = WeightOneRing(m, v, x.regular ? 1.f / 16.f : Beta(m.valence(v)));
            else
                np = WeightBoundary(m, v, 1.f / 8.f);
            m.V[x.child].p = np;
        }
        // odd edge vertices
        std::map<EdgeKey, int> edgeVerts;
        for (int f : fs)
            for (int k = 0; k < 3; ++k) {
                const int a = m.F[f].v[k], b = m.F[f].v[Next(k)];
                const EdgeKey key = Edge(a, b);
                if (edgeVerts.count(key)) continue;
                SDVertex x;
                x.regular = true;
                x.boundary = m.F[f].f[k] == kNone;
                x.startFace = m.F[f].children[3];
                const V3 pa = m.V[key.first].p, pb = m.V[key.second].p;
                if (x.boundary) {
                    x.p = 0.5f * pa;
                    x.p = x.p + 0.5f * pb;
                } else {
                    x.p = 3.f / 8.f * pa;
                    x.p = x.p + 3.f / 8.f * pb;
                    x.p = x.p + 1.f / 8.f * m.V[m.otherVert(f, a, b)].p;
                    x.p = x.p + 1.f / 8.f * m.V[m.otherVert(m.F[f].f[k], a, b)].p;
                }
                m.V.push_back(x);
                edgeVerts[key] = (int)m.V.size() - 1;
                newVertices.push_back((int)m.V.size() - 1);
            }
        // topology of the children
        for (int v : vs) {
            const int sf = m.V[v].startFace;
            m.V[m.V[v].child].startFace = m.F[sf].children[m.vnum(sf, v)];
        }
        for (int f : fs)
            for (int j = 0; j < 3; ++j) {
                const SDFace &F = m.F[f];
                m.F[F.children[3]].f[j] = F.children[Next(j)];
                m.F[F.children[j]].f[Next(j)] = F.children[3];
                int f2 = F.f[j];
                m.F[F.children[j]].f[j] = f2 != kNone ? m.F[f2].children[m.vnum(f2, F.v[j])] : kNone;
                f2 = F.f[Prev(j)];
                m.F[F.children[j]].f[Prev(j)] = f2 != kNone ? m.F[f2].children[m.vnum(f2, F.v[j])] : kNone;
            }
        for (int f : fs)
            for (int j = 0; j < 3; ++j) {
                const SDFace &F = m.F[f];
                m.F[F.children[j]].v[j] = m.V[F.v[j]].child;
                const int vert = edgeVerts[Edge(F.v[j], F.v[Next(j)])];
                m.F[F.children[j]].v[Next(j)] = vert;
                m.F[F.children[Next(j)]].v[j] = vert;
                m.F[F.children[3]].v[j] = vert;
            }
        fs = std::move(newFaces);
        vs = std::move(newVertices);
    }
    // limit positions, then the limit surface's tangents and normals
    std::vector<V3> pLimit(vs.size());
    for (size_t i = 0; i < vs.size(); ++i)
        pLimit[i] = m.V[vs[i]].boundary ? WeightBoundary(m, vs[i], 1.f / 5.f)
                                        : WeightOneRing(m, vs[i], LoopGamma(m.valence(vs[i])));
    for (size_t i = 0; i < vs.size(); ++i) m.V[vs[i]].p = pLimit[i];
    N->clear();
    std::vector<V3> ring;
    for (int vi : vs) {
        const SDVertex &vx = m.V[vi];
        V3 S(0, 0, 0), T(0, 0, 0);
        const int valence = m.valence(vi);
        m.oneRing(vi, &ring);
        if (!vx.boundary) {
            for (int j = 0; j < valence; ++j) {
                S = S + std::cos(2 * kPi * j / valence) * ring[j];
                T = T + std::sin(2 * kPi * j / valence) * ring[j];
            }
        } else {
            S = ring[valence - 1] - ring[0];
            if (valence == 2)
                T = ring[0] + ring[1] - 2 * vx.p;
            else if (valence == 3)
                T = ring[1] - vx.p;
            else if (valence == 4)
                T = -1 * ring[0] + 2 * ring[1] + 2 * ring[2] + -1 * ring[3] + -2 * vx.p;
            else {
                const float theta = kPi / float(valence - 1);
                T = std::sin(theta) * (ring[0] + ring[valence - 1]);
                for (int k = 1; k < valence - 1; ++k) {
                    const float wt = (2 * std::cos(theta) - 2) * std::sin((k)*theta);
                    T = T + wt * ring[k];
                }
                T = -T;
            }
        }
        N->push_back(Cross(S, T));
    }
    *P = pLimit;
    std::map<int, int> used;
    for (size_t i = 0; i < vs.size(); ++i) used[vs[i]] = (int)i;
    tris->clear();
    for (int f : fs)
        for (int j = 0; j < 3; ++j) tris->push_back(used[m.F[f].v[j]]);
}

}  // namespace pbrt_amd
