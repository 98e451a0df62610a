#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <future>
#include <cstdlib>
#include <stdexcept>

#include "bvh.h"

namespace pbrt_amd {

// empty slot box: lo = +kEmptyLo, hi = -kEmptyLo (fails every slab test, see BVH8Node)
static constexpr float kEmptyLo = 1e30f;

namespace {
struct Box {
    V3 mn{kInfinity, kInfinity, kInfinity}, mx{-kInfinity, -kInfinity, -kInfinity};
    void Add(V3 p) {
        mn = V3(std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z));
        mx = V3(std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z));
    }
    void Add(const Box &b) {
        mn = V3(std::min(mn.x, b.mn.x), std::min(mn.y, b.mn.y), std::min(mn.z, b.mn.z));
        mx = V3(std::max(mx.x, b.mx.x), std::max(mx.y, b.mx.y), std::max(mx.z, b.mx.z));
    }
    bool Empty() const { return mn.x > mx.x; }
    float Area() const {
        if (Empty()) return 0;
        V3 d = mx - mn;
        return 2 * (d.x * d.y + d.x * d.z + d.y * d.z);
    }
};

struct Prim {
    Box box;
    V3 centroid;
    int index;
};

struct Node2 {
    Box box;
    int left = -1, right = -1;   // interior
    int first = 0, count = 0;    // leaf (into ordered prims)
    bool leaf() const { return left < 0; }
};

struct Builder2 {
    std::vector<Prim> &prims;
    std::vector<Node2> nodes;
    int maxLeaf;

    // One binned-SAH decision for prims [start, end): fills box and returns the split point,
    // or -1 for a leaf.  Reorders the range in place.
    int Split(int start, int end, Box *box) {
        Box nb;
        for (int i = start; i < end; ++i) nb.Add(prims[i].box);
        *box = nb;
        int n = end - start;
        if (n == 1) return -1;
        Box cb;
        for (int i = start; i < end; ++i) cb.Add(prims[i].centroid);
        V3 d = cb.mx - cb.mn;
        int dim = (d.x > d.y) ? ((d.x > d.z) ? 0 : 2) : ((d.y > d.z) ? 1 : 2);
        if (cb.mx[dim] == cb.mn[dim]) {
            if (n <= maxLeaf) return -1;
            return (start + end) / 2;  // all centroids coincide: split the list
        }
        int mid;
        if (n == 2 && SahAllAxes() && PairLeaves() == 1) return SplitAllAxes(start, end, nb, cb);
        if (n == 2 && PairLeaves() == 2 && prims[start].box.Area() + prims[start + 1].box.Area() >= 1.9f * nb.Area())
            return -1;
        if (n <= 2) {
            mid = (start + end) / 2;
            std::nth_element(&prims[start], &prims[mid], &prims[end - 1] + 1,
                             [dim](const Prim &a, const Prim &b) { return a.centroid[dim] < b.centroid[dim]; });
            return mid;
        }
        if (SahAllAxes()) return SplitAllAxes(start, end, nb, cb);
        constexpr int nBuckets = 12;
        int counts[nBuckets] = {0};
        Box bbox[nBuckets];
        auto bucketOf = [&](const Prim &p) {
            int b = (int)(nBuckets * ((p.centroid[dim] - cb.mn[dim]) / (cb.mx[dim] - cb.mn[dim])));
            return std::min(std::max(b, 0), nBuckets - 1);
        };
        for (int i = start; i < end; ++i) {
            int b = bucketOf(prims[i]);
            counts[b]++;
            bbox[b].Add(prims[i].box);
        }
        float costs[nBuckets - 1] = {};
        int countBelow = 0;
        Box boundBelow;
        for (int i = 0; i < nBuckets - 1; ++i) {
            boundBelow.Add(bbox[i]);
            countBelow += counts[i];
            costs[i] += countBelow * boundBelow.Area();
        }
        int countAbove = 0;
        Box boundAbove;
        for (int i = nBuckets - 1; i >= 1; --i) {
            boundAbove.Add(bbox[i]);
            countAbove += counts[i];
            costs[i - 1] += countAbove * boundAbove.Area();
        }
        int minBucket = -1;
        float minCost = kInfinity;
        for (int i = 0; i < nBuckets - 1; ++i)
            if (costs[i] < minCost) {
                minCost = costs[i];
                minBucket = i;
            }
        float leafCost = (float)n;
        minCost = 1.f / 2.f + minCost / nb.Area();
        if (!(n > maxLeaf || minCost < leafCost)) return -1;
        Prim *pm = std::partition(&prims[start], &prims[end - 1] + 1,
                                  [&](const Prim &p) { return bucketOf(p) <= minBucket; });
        mid = (int)(pm - &prims[0]);
        if (mid == start || mid == end) {
            mid = (start + end) / 2;
            std::nth_element(&prims[start], &prims[mid], &prims[end - 1] + 1,
                             [dim](const Prim &a, const Prim &b) { return a.centroid[dim] < b.centroid[dim]; });
        }
        return mid;
    }

    // The binned SAH over all three axes (32 buckets each, default since round 6: C2 / C3
    // k_closest -12 % / -14 %, profiles/r06_bvh_sah_ab.txt); PBRT_AMD_BVH_SAH=1 restores the
    // centroid bounds' longest axis with 12 buckets (pbrt's BVHAggregate::buildRecursive)
    static bool SahAllAxes() {
        static const bool on = [] {
            const char *e = std::getenv("PBRT_AMD_BVH_SAH");
            return !(e && std::atoi(e) == 1);
        }();
        return on;
    }
    // Two triangles whose boxes nearly coincide (area sum >= 1.9x their union's: a quad's two
    // halves) stay one leaf instead of always splitting (default, PBRT_AMD_BVH_PAIR=2; C2
    // k_closest -6 %, C3 / C4 unchanged, profiles/r06_bvh_sah_ab.txt); =1 puts every pair to the
    // SAH's leaf test (C4 -1 %), =0 always splits as pbrt's builder does
    static int PairLeaves() {
        static const int mode = [] {
            const char *e = std::getenv("PBRT_AMD_BVH_PAIR");
            return e ? std::atoi(e) : 2;
        }();
        return mode;
    }
    // the SAH's traversal cost against one triangle test (PBRT_AMD_BVH_CT, default 1/2)
    static float TraversalCost() {
        static const float ct = [] {
            const char *e = std::getenv("PBRT_AMD_BVH_CT");
            return e ? (float)std::atof(e) : 0.5f;
        }();
        return ct;
    }
    int SplitAllAxes(int start, int end, const Box &nb, const Box &cb) {
        constexpr int nBuckets = 32;
        const int n = end - start;
        int bestDim = -1, bestBucket = -1;
        float bestCost = kInfinity;
        for (int dim = 0; dim < 3; ++dim) {
            if (!(cb.mx[dim] > cb.mn[dim])) continue;
            int counts[nBuckets] = {0};
            Box bbox[nBuckets];
            const float lo = cb.mn[dim], ext = cb.mx[dim] - cb.mn[dim];
            for (int i = start; i < end; ++i) {
                int b = (int)(nBuckets * ((prims[i].centroid[dim] - lo) / ext));
                b = std::min(std::max(b, 0), nBuckets - 1);
                counts[b]++;
                bbox[b].Add(prims[i].box);
            }
            float costs[nBuckets - 1] = {};
            int below = 0, above = 0;
            Box bb, ba;
            for (int i = 0; i < nBuckets - 1; ++i) {
                bb.Add(bbox[i]);
                below += counts[i];
                costs[i] += below * bb.Area();
            }
            for (int i = nBuckets - 1; i >= 1; --i) {
                ba.Add(bbox[i]);
                above += counts[i];
                costs[i - 1] += above * ba.Area();
            }
            for (int i = 0; i < nBuckets - 1; ++i)
                if (costs[i] < bestCost) bestCost = costs[i], bestDim = dim, bestBucket = i;
        }
        const float cost = TraversalCost() + bestCost / nb.Area();
        if (bestDim < 0 || !(n > maxLeaf || cost < (float)n)) return n > maxLeaf ? (start + end) / 2 : -1;
        const float lo = cb.mn[bestDim], ext = cb.mx[bestDim] - cb.mn[bestDim];
        auto bucketOf = [&](const Prim &p) {
            const int b = (int)(nBuckets * ((p.centroid[bestDim] - lo) / ext));
            return std::min(std::max(b, 0), nBuckets - 1);
        };
        Prim *pm = std::partition(&prims[start], &prims[end - 1] + 1, [&](const Prim &p) { return bucketOf(p) <= bestBucket; });
        int mid = (int)(pm - &prims[0]);
        if (mid == start || mid == end) {
            mid = (start + end) / 2;
            const int d = bestDim;
            std::nth_element(&prims[start], &prims[mid], &prims[end - 1] + 1,
                             [d](const Prim &a, const Prim &b) { return a.centroid[d] < b.centroid[d]; });
        }
        return mid;
    }

    int Build(int start, int end) {
        int idx = (int)nodes.size();
        nodes.push_back(Node2{});
        Box box;
        int mid = Split(start, end, &box);
        nodes[idx].box = box;
        if (mid < 0) {
            nodes[idx].first = start;
            nodes[idx].count = end - start;
            return idx;
        }
        int l = Build(start, mid);
        int r = Build(mid, end);
        nodes[idx].left = l;
        nodes[idx].right = r;
        return idx;
    }
};

// The same tree built with the top levels' subtrees on their own threads: each subtree lands
// in its own node array and the arrays are concatenated in depth-first order (node, left
// subtree, right subtree), i.e. exactly the serial Build's layout.
std::vector<Node2> BuildParallel(std::vector<Prim> &prims, int start, int end, int maxLeaf, int depth) {
    Builder2 b{prims, {}, maxLeaf};
    if (depth >= 4 || end - start < (1 << 16)) {
        b.nodes.reserve(2 * (end - start) / std::max(maxLeaf / 2, 1) + 1);
        b.Build(start, end);
        return std::move(b.nodes);
    }
    Box box;
    int mid = b.Split(start, end, &box);
    Node2 root;
    root.box = box;
    if (mid < 0) {
        root.first = start;
        root.count = end - start;
        return {root};
    }
    auto left = std::async(std::launch::async, BuildParallel, std::ref(prims), start, mid, maxLeaf, depth + 1);
    std::vector<Node2> r = BuildParallel(prims, mid, end, maxLeaf, depth + 1);
    std::vector<Node2> l = left.get();
    std::vector<Node2> out;
    out.reserve(1 + l.size() + r.size());
    out.push_back(root);
    auto append = [&](const std::vector<Node2> &sub) {
        const int off = (int)out.size();
        for (Node2 n : sub) {
            if (!n.leaf()) {
                n.left += off;
                n.right += off;
            }
            out.push_back(n);
        }
        return off;
    };
    out[0].left = append(l);
    out[0].right = append(r);
    return out;
}

// ---------------------------------------------------------------------------------------------
// Spatial-split BVH (PBRT_AMD_BVH_SBVH=1; Stich, Friedrich and Dietrich 2009, "Spatial Splits
// in Bounding Volume Hierarchies").  Beside the object split, a node whose best object split
// leaves children overlapping by more than alpha of the root's area also bins the node's
// bounds into 32 slabs per axis, clips every triangle reference into the slabs it spans, and
// may split along a slab plane, referencing a straddling triangle from both sides (or from one,
// when "unsplitting" it is cheaper).  The traversal is unchanged: a leaf lists triangles, and
// a triangle may appear in several leaves.  Clipped boxes are padded outward by a few ulps and
// then intersected with the triangle's own box, so every box still holds its part of the
// triangle, and the closest-hit result is the same triangle test over a different visit order.
struct SpatialBuilder {
    const std::vector<V3> &verts;
    const std::vector<std::array<int, 3>> &tris;
    int maxLeaf;
    float minOverlap;  // alpha * root area
    std::atomic<long long> *budget;  // references that may still be duplicated

    static constexpr int kBins = 32;

    struct Result {
        std::vector<Node2> nodes;
        std::vector<Prim> refs;  // leaf order
    };

    static float Axis(const V3 &v, int d) { return d == 0 ? v.x : d == 1 ? v.y : v.z; }
    static void SetAxis(V3 &v, int d, float f) { (d == 0 ? v.x : d == 1 ? v.y : v.z) = f; }

    static Box Intersect(const Box &a, const Box &b) {
        Box r;
        r.mn = V3(std::max(a.mn.x, b.mn.x), std::max(a.mn.y, b.mn.y), std::max(a.mn.z, b.mn.z));
        r.mx = V3(std::min(a.mx.x, b.mx.x), std::min(a.mx.y, b.mx.y), std::min(a.mx.z, b.mx.z));
        if (r.mn.x > r.mx.x || r.mn.y > r.mx.y || r.mn.z > r.mx.z) return Box{};
        return r;
    }

    // box of the part of triangle t with lo <= p[d] <= hi, within the reference box rb
    Box ClipBox(int t, int d, float lo, float hi, const Box &rb) const {
        const V3 v[3] = {verts[tris[t][0]], verts[tris[t][1]], verts[tris[t][2]]};
        Box b;
        for (int e = 0; e < 3; ++e) {
            const V3 a = v[e], c = v[(e + 1) % 3];
            const float ad = Axis(a, d), cd = Axis(c, d);
            if (ad >= lo && ad <= hi) b.Add(a);
            for (float pl : {lo, hi}) {
                if ((ad < pl && cd > pl) || (ad > pl && cd < pl)) {
                    const float s = (pl - ad) / (cd - ad);
                    V3 p = a + (c - a) * s;
                    SetAxis(p, d, pl);
                    b.Add(p);
                }
            }
        }
        if (b.Empty()) return b;
        for (int k = 0; k < 3; ++k) {
            if (k == d) continue;
            const float m = std::max(std::fabs(Axis(rb.mn, k)), std::fabs(Axis(rb.mx, k)));
            const float pad = m * 4.7683716e-7f + 1e-30f;  // 8 ulps of the box's magnitude
            SetAxis(b.mn, k, Axis(b.mn, k) - pad);
            SetAxis(b.mx, k, Axis(b.mx, k) + pad);
        }
        SetAxis(b.mn, d, std::max(Axis(b.mn, d), lo));
        SetAxis(b.mx, d, std::min(Axis(b.mx, d), hi));
        return Intersect(b, rb);
    }

    struct ObjectSplit {
        int dim = -1, bucket = -1;
        float cost = kInfinity;
        Box left, right;
    };

    ObjectSplit BestObjectSplit(const std::vector<Prim> &refs, const Box &cb) const {
        ObjectSplit best;
        for (int dim = 0; dim < 3; ++dim) {
            const float lo = Axis(cb.mn, dim), ext = Axis(cb.mx, dim) - lo;
            if (!(ext > 0)) continue;
            int counts[kBins] = {0};
            Box bbox[kBins];
            for (const Prim &p : refs) {
                int b = (int)(kBins * ((Axis(p.centroid, dim) - lo) / ext));
                b = std::min(std::max(b, 0), kBins - 1);
                counts[b]++;
                bbox[b].Add(p.box);
            }
            Box below[kBins];
            Box acc;
            for (int i = 0; i < kBins; ++i) acc.Add(bbox[i]), below[i] = acc;
            int cntBelow[kBins];
            int c = 0;
            for (int i = 0; i < kBins; ++i) c += counts[i], cntBelow[i] = c;
            Box above;
            int cntAbove = 0;
            for (int i = kBins - 1; i >= 1; --i) {
                above.Add(bbox[i]);
                cntAbove += counts[i];
                const float cost = cntBelow[i - 1] * below[i - 1].Area() + cntAbove * above.Area();
                if (cost < best.cost) {
                    best.cost = cost, best.dim = dim, best.bucket = i - 1;
                    best.left = below[i - 1], best.right = above;
                }
            }
        }
        return best;
    }

    struct SpatialSplit {
        int dim = -1;
        float plane = 0, cost = kInfinity;
    };

    SpatialSplit BestSpatialSplit(const std::vector<Prim> &refs, const Box &nb) const {
        SpatialSplit best;
        for (int dim = 0; dim < 3; ++dim) {
            const float lo = Axis(nb.mn, dim), ext = Axis(nb.mx, dim) - lo;
            if (!(ext > 0)) continue;
            const float w = ext / kBins;
            auto planeAt = [&](int i) { return i == kBins ? Axis(nb.mx, dim) : lo + w * i; };
            auto binOf = [&](float x) { return std::min(std::max((int)((x - lo) / w), 0), kBins - 1); };
            int enter[kBins] = {0}, exit_[kBins] = {0};
            Box bbox[kBins];
            for (const Prim &p : refs) {
                int b0 = binOf(Axis(p.box.mn, dim)), b1 = binOf(Axis(p.box.mx, dim));
                enter[b0]++, exit_[b1]++;
                if (b0 == b1) {
                    bbox[b0].Add(p.box);
                    continue;
                }
                for (int b = b0; b <= b1; ++b) bbox[b].Add(ClipBox(p.index, dim, planeAt(b), planeAt(b + 1), p.box));
            }
            Box below[kBins];
            Box acc;
            int nl[kBins], c = 0;
            for (int i = 0; i < kBins; ++i) acc.Add(bbox[i]), below[i] = acc, c += enter[i], nl[i] = c;
            Box above;
            int nr = 0;
            for (int i = kBins - 1; i >= 1; --i) {
                above.Add(bbox[i]);
                nr += exit_[i];
                const float cost = nl[i - 1] * below[i - 1].Area() + nr * above.Area();
                if (cost < best.cost) best.cost = cost, best.dim = dim, best.plane = planeAt(i);
            }
        }
        return best;
    }

    Result Leaf(std::vector<Prim> &&refs, const Box &nb) const {
        Result r;
        Node2 n;
        n.box = nb;
        n.first = 0;
        n.count = (int)refs.size();
        r.nodes.push_back(n);
        r.refs = std::move(refs);
        return r;
    }

    static Box BoundsOf(const std::vector<Prim> &refs, Box *cb) {
        Box b;
        *cb = Box{};
        for (const Prim &p : refs) b.Add(p.box), cb->Add(p.centroid);
        return b;
    }

    Result Build(std::vector<Prim> &&refs, int depth) const {
        Box cb;
        const Box nb = BoundsOf(refs, &cb);
        const int n = (int)refs.size();
        if (n == 1) return Leaf(std::move(refs), nb);
        std::vector<Prim> L, R;
        ObjectSplit os = BestObjectSplit(refs, cb);
        float bestCost = os.cost;
        SpatialSplit ss;
        if (depth < 48 && budget->load(std::memory_order_relaxed) > 0 && Intersect(os.left, os.right).Area() > minOverlap) {
            ss = BestSpatialSplit(refs, nb);
            if (ss.cost < bestCost) bestCost = ss.cost;
            else ss.dim = -1;
        }
        const float cost = Builder2::TraversalCost() + bestCost / nb.Area();
        if (os.dim < 0 && ss.dim < 0) {
            // all centroids coincide and no spatial split: a leaf, or halve the list
            if (n <= maxLeaf) return Leaf(std::move(refs), nb);
            L.assign(refs.begin(), refs.begin() + n / 2);
            R.assign(refs.begin() + n / 2, refs.end());
        } else if (!(n > maxLeaf || cost < (float)n)) {
            return Leaf(std::move(refs), nb);
        } else if (ss.dim >= 0) {
            const int d = ss.dim;
            const float pl = ss.plane;
            // the children's boxes and counts before the straddlers, then each straddler goes
            // left, right or both, whichever the SAH prefers (reference unsplitting)
            Box bl, br;
            std::vector<Prim> straddle;
            for (Prim &p : refs) {
                if (Axis(p.box.mx, d) <= pl) bl.Add(p.box), L.push_back(p);
                else if (Axis(p.box.mn, d) >= pl) br.Add(p.box), R.push_back(p);
                else straddle.push_back(p);
            }
            long long dup = 0;
            for (Prim &p : straddle) {
                const Box lb = ClipBox(p.index, d, -kInfinity, pl, p.box);
                const Box rb = ClipBox(p.index, d, pl, kInfinity, p.box);
                const float nL = (float)L.size(), nR = (float)R.size();
                Box blS = bl, brS = br, blW = bl, brW = br;
                blS.Add(lb), brS.Add(rb), blW.Add(p.box), brW.Add(p.box);
                const float cSplit = blS.Area() * (nL + 1) + brS.Area() * (nR + 1);
                const float cLeft = blW.Area() * (nL + 1) + br.Area() * nR;
                const float cRight = bl.Area() * nL + brW.Area() * (nR + 1);
                if (lb.Empty() || (!rb.Empty() && cRight <= cLeft && cRight <= cSplit)) {
                    br = brW, R.push_back(p);
                } else if (rb.Empty() || (cLeft <= cSplit)) {
                    bl = blW, L.push_back(p);
                } else {
                    Prim a = p, b = p;
                    a.box = lb, b.box = rb;
                    a.centroid = (lb.mn + lb.mx) * 0.5f, b.centroid = (rb.mn + rb.mx) * 0.5f;
                    bl = blS, br = brS;
                    L.push_back(a), R.push_back(b);
                    ++dup;
                }
            }
            budget->fetch_sub(dup, std::memory_order_relaxed);
            if (L.empty() || R.empty()) {  // degenerate: fall back to halving
                std::vector<Prim> all = L.empty() ? std::move(R) : std::move(L);
                L.assign(all.begin(), all.begin() + all.size() / 2);
                R.assign(all.begin() + all.size() / 2, all.end());
            }
        } else {
            const int d = os.dim;
            const float lo = Axis(cb.mn, d), ext = Axis(cb.mx, d) - lo;
            for (Prim &p : refs) {
                int b = (int)(kBins * ((Axis(p.centroid, d) - lo) / ext));
                b = std::min(std::max(b, 0), kBins - 1);
                (b <= os.bucket ? L : R).push_back(p);
            }
            if (L.empty() || R.empty()) {
                std::vector<Prim> all = L.empty() ? std::move(R) : std::move(L);
                std::sort(all.begin(), all.end(), [d](const Prim &a, const Prim &b) { return Axis(a.centroid, d) < Axis(b.centroid, d); });
                L.assign(all.begin(), all.begin() + all.size() / 2);
                R.assign(all.begin() + all.size() / 2, all.end());
            }
        }
        std::vector<Prim>().swap(refs);
        Result l, r;
        if (depth < 4 && L.size() + R.size() >= (1u << 16)) {
            auto fl = std::async(std::launch::async, [&] { return Build(std::move(L), depth + 1); });
            r = Build(std::move(R), depth + 1);
            l = fl.get();
        } else {
            l = Build(std::move(L), depth + 1);
            r = Build(std::move(R), depth + 1);
        }
        Result out;
        out.nodes.reserve(1 + l.nodes.size() + r.nodes.size());
        out.refs.reserve(l.refs.size() + r.refs.size());
        Node2 root;
        root.box = nb;
        out.nodes.push_back(root);
        auto append = [&](Result &sub) {
            const int off = (int)out.nodes.size(), roff = (int)out.refs.size();
            for (Node2 nd : sub.nodes) {
                if (!nd.leaf()) nd.left += off, nd.right += off;
                else nd.first += roff;
                out.nodes.push_back(nd);
            }
            out.refs.insert(out.refs.end(), sub.refs.begin(), sub.refs.end());
            return off;
        };
        out.nodes[0].left = append(l);
        out.nodes[0].right = append(r);
        return out;
    }
};

static bool SpatialSplitsOn() {
    static const bool on = [] {
        const char *e = std::getenv("PBRT_AMD_BVH_SBVH");
        return e && std::atoi(e) > 0;
    }();
    return on;
}
}  // namespace

// Quantise every node of out.nodes into out.qnodes (same indices).
static void Compress(BVH8 &out) {
    out.qnodes.assign(out.nodes.size(), BVH8QNode{});
    for (size_t i = 0; i < out.nodes.size(); ++i) {
        const BVH8Node &n = out.nodes[i];
        const std::array<int32_t, 8> &child = out.childRef[i];
        BVH8QNode &q = out.qnodes[i];
        float lo[3] = {kInfinity, kInfinity, kInfinity}, hi[3] = {-kInfinity, -kInfinity, -kInfinity};
        const float *clo[3] = {n.lox, n.loy, n.loz}, *chi[3] = {n.hix, n.hiy, n.hiz};
        bool any = false;
        for (int c = 0; c < 8; ++c) {
            if (child[c] == kEmptyChild) continue;
            any = true;
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], clo[a][c]);
                hi[a] = std::max(hi[a], chi[a][c]);
            }
        }
        uint8_t e[3] = {127, 127, 127};
        if (any)
            for (int a = 0; a < 3; ++a) {
                // smallest exponent whose 255-step grid from lo reaches hi
                const double ext = (double)hi[a] - lo[a];
                int ex = (int)std::ceil(std::log2(std::max(ext / 255.0, 1e-37))) + 127;
                ex = std::min(std::max(ex, 1), 254);
                while (ex < 254 && DecodeQ(255, (uint8_t)ex, lo[a]) < hi[a]) ++ex;
                while (ex > 1 && DecodeQ(255, (uint8_t)(ex - 1), lo[a]) >= hi[a]) --ex;
                e[a] = (uint8_t)ex;
            }
        q.px = any ? lo[0] : 0;
        q.py = any ? lo[1] : 0;
        q.pz = any ? lo[2] : 0;
        q.ex = e[0], q.ey = e[1], q.ez = e[2];
        uint8_t *qlo[3] = {q.qlox, q.qloy, q.qloz}, *qhi[3] = {q.qhix, q.qhiy, q.qhiz};
        const float org[3] = {q.px, q.py, q.pz};
        int innerRank = 0, triBase = -1;
        q.childBase = -1;
        for (int c = 0; c < 8; ++c) {
            const int ch = child[c];
            if (ch == kEmptyChild) {
                for (int a = 0; a < 3; ++a) qlo[a][c] = 255, qhi[a][c] = 0;
                continue;
            }
            for (int a = 0; a < 3; ++a) {
                double s = std::ldexp(1.0, (int)e[a] - 127);
                int l = (int)std::floor(((double)clo[a][c] - org[a]) / s);
                int h = (int)std::ceil(((double)chi[a][c] - org[a]) / s);
                l = std::min(std::max(l, 0), 255);
                h = std::min(std::max(h, 0), 255);
                while (l > 0 && DecodeQ((uint8_t)l, e[a], org[a]) > clo[a][c]) --l;
                while (h < 255 && DecodeQ((uint8_t)h, e[a], org[a]) < chi[a][c]) ++h;
                if (DecodeQ((uint8_t)l, e[a], org[a]) > clo[a][c] || DecodeQ((uint8_t)h, e[a], org[a]) < chi[a][c])
                    throw std::runtime_error("BVH8 quantisation is not conservative");
                qlo[a][c] = (uint8_t)l;
                qhi[a][c] = (uint8_t)h;
            }
            if (ch >= 0) {
                if (q.childBase < 0) q.childBase = ch;
                if (ch != q.childBase + innerRank) throw std::runtime_error("BVH8 interior children not contiguous");
                ++innerRank;
                q.imask |= (uint8_t)(1u << c);
            } else {
                const int enc = ~ch, first = enc >> 3, count = (enc & 7) + 1;
                if (triBase < 0) triBase = first;
                const int off = first - triBase;
                if (off < 0 || off > 31 || count > 4) throw std::runtime_error("BVH8 leaf range does not fit the compressed node");
                q.meta[c] = (uint8_t)((count << 5) | off);  // count 1..4; 0 = interior / empty
            }
        }
        q.triBase = triBase < 0 ? 0 : triBase;
        if (q.childBase < 0) q.childBase = 0;
    }
}

// Node order below the top levels (PBRT_AMD_BVH_DFS=1, an experiment): the nodes down to
// depth topDepth keep their breadth-first order (the prefix the traversal kernels cache in
// LDS), and below each of them the child groups are laid out depth first (a group, then its
// first child's group, ...), so a subtree's nodes sit together in HBM.  Every group stays
// contiguous in slot order, and children still follow their parents.
static void ReorderGroupsDepthFirst(BVH8 &out, const std::vector<int> &depth, int topDepth) {
    const int n = (int)out.nodes.size();
    std::vector<int> newIdx(n, -1);
    int next = 0;
    for (int i = 0; i < n; ++i)
        if (depth[i] <= topDepth) newIdx[i] = next++;  // BFS order = level order: a prefix
    std::vector<int> stack;
    for (int i = 0; i < n; ++i) {
        if (depth[i] != topDepth) continue;
        stack.assign(1, i);
        while (!stack.empty()) {
            const int u = stack.back();
            stack.pop_back();
            const BVH8Node &nd = out.nodes[u];
            const int cnt = __builtin_popcount(nd.imask);
            for (int k = 0; k < cnt; ++k) newIdx[nd.childBase + k] = next++;
            for (int k = cnt - 1; k >= 0; --k) stack.push_back(nd.childBase + k);
        }
    }
    if (next != n) throw std::runtime_error("BVH8 depth-first reorder missed nodes");
    std::vector<BVH8Node> nodes(n);
    std::vector<std::array<int32_t, 8>> refs(n);
    for (int i = 0; i < n; ++i) {
        BVH8Node nd = out.nodes[i];
        if (nd.imask) nd.childBase = newIdx[nd.childBase];
        std::array<int32_t, 8> r = out.childRef[i];
        for (int c = 0; c < 8; ++c)
            if (r[c] >= 0) r[c] = newIdx[r[c]];
        nodes[newIdx[i]] = nd;
        refs[newIdx[i]] = r;
    }
    out.nodes.swap(nodes);
    out.childRef.swap(refs);
}

BVH8 BuildBVH8(const std::vector<V3> &verts, const std::vector<std::array<int, 3>> &tris, int maxLeafPrims, int spatial) {
    BVH8 out;
    std::vector<Prim> prims;
    prims.reserve(tris.size());
    Box all;
    // Degenerate triangles can never be hit (shapes.cpp:175); they stay out of the tree and
    // are appended after the BVH's triangles in leaf order, so the traversal skips the test.
    std::vector<int> degenerate;
    for (size_t i = 0; i < tris.size(); ++i) {
        if (TriangleDegenerate(verts[tris[i][0]], verts[tris[i][1]], verts[tris[i][2]])) {
            degenerate.push_back((int)i);
            continue;
        }
        Prim p;
        p.box.Add(verts[tris[i][0]]);
        p.box.Add(verts[tris[i][1]]);
        p.box.Add(verts[tris[i][2]]);
        p.centroid = (p.box.mn + p.box.mx) * 0.5f;
        p.index = (int)i;
        all.Add(p.box);
        prims.push_back(p);
    }
    out.boundsMin = all.mn;
    out.boundsMax = all.mx;
    auto appendDegenerate = [&]() {
        for (int t : degenerate) {
            out.triPrim.push_back(t);
            for (int k = 0; k < 3; ++k) {
                V3 p = verts[tris[t][k]];
                float w = 0;
                if (k == 0) {
                    int32_t tt = t;
                    memcpy(&w, &tt, 4);
                }
                out.triVerts.insert(out.triVerts.end(), {p.x, p.y, p.z, w});
            }
        }
    };
    if (prims.empty()) {
        BVH8Node root{};
        std::array<int32_t, 8> ref;
        for (int c = 0; c < 8; ++c) {
            root.lox[c] = root.loy[c] = root.loz[c] = kEmptyLo;
            root.hix[c] = root.hiy[c] = root.hiz[c] = -kEmptyLo;
            ref[c] = kEmptyChild;
        }
        out.nodes.push_back(root);
        out.childRef.push_back(ref);
        appendDegenerate();
        Compress(out);
        return out;
    }
    maxLeafPrims = std::min(std::max(maxLeafPrims, 1), kMaxLeafPrims);
    Builder2 b{prims, {}, maxLeafPrims};
    if (spatial < 0 ? SpatialSplitsOn() : spatial > 0) {
        // leaves index the builder's reference list, which replaces prims below
        const Box rootBox = all;
        std::atomic<long long> budget{(long long)prims.size()};  // at most 2x the references
        SpatialBuilder sb{verts, tris, maxLeafPrims, 1e-5f * rootBox.Area(), &budget};
        SpatialBuilder::Result r = sb.Build(std::move(prims), 0);
        prims = std::move(r.refs);
        b.nodes = std::move(r.nodes);
    } else {
        b.nodes = BuildParallel(prims, 0, (int)prims.size(), maxLeafPrims, 0);
    }

    // collapse BVH2 -> BVH8 (greedy: open the child with the largest surface area)
    struct Work {
        int node2, depth;
    };
    std::vector<Work> queue;
    std::vector<int> order;  // leaf-order triangles (original indices)
    order.reserve(prims.size());
    queue.push_back({0, 1});
    out.nodes.reserve(prims.size() / 2 + 1);
    std::vector<int> node8Of;  // per queue entry the BVH8 index
    size_t head = 0;
    out.nodes.push_back(BVH8Node{});
    out.childRef.push_back({});
    node8Of.push_back(0);
    while (head < queue.size()) {
        Work w = queue[head];
        int self = node8Of[head];
        ++head;
        out.maxDepth = std::max(out.maxDepth, w.depth);
        std::vector<int> kids;
        const Node2 &n2 = b.nodes[w.node2];
        if (n2.leaf())
            kids.push_back(w.node2);
        else {
            kids.push_back(n2.left);
            kids.push_back(n2.right);
        }
        while ((int)kids.size() < 8) {
            int best = -1;
            float bestArea = -1;
            for (size_t k = 0; k < kids.size(); ++k) {
                const Node2 &c = b.nodes[kids[k]];
                if (!c.leaf() && c.box.Area() > bestArea) {
                    bestArea = c.box.Area();
                    best = (int)k;
                }
            }
            if (best < 0) break;
            int open = kids[best];
            kids.erase(kids.begin() + best);
            kids.push_back(b.nodes[open].left);
            kids.push_back(b.nodes[open].right);
        }
        // octant slots (Ylitie et al. 2017, section 3.2): slot s should hold the child that rays of
        // direction-sign octant s (bit a set: d_a < 0) reach first, i.e. the child whose centroid
        // lies farthest against D_s = (s & 1 ? -1 : 1, s & 2 ? -1 : 1, s & 4 ? -1 : 1).  Greedy
        // assignment of the cheapest (child, slot) pair first.
        int slotOf[8];
        {
            const Box &pb = n2.box;
            const V3 pc = (pb.mn + pb.mx) * 0.5f;
            float cost[8][8];
            for (size_t k = 0; k < kids.size(); ++k) {
                const Box &cb = b.nodes[kids[k]].box;
                const V3 cc = (cb.mn + cb.mx) * 0.5f - pc;
                for (int sl = 0; sl < 8; ++sl)
                    cost[k][sl] = ((sl & 1) ? -cc.x : cc.x) + ((sl & 2) ? -cc.y : cc.y) + ((sl & 4) ? -cc.z : cc.z);
            }
            bool usedK[8] = {}, usedS[8] = {};
            for (size_t round = 0; round < kids.size(); ++round) {
                int bk = -1, bs = -1;
                float bc = kInfinity;
                for (size_t k = 0; k < kids.size(); ++k)
                    for (int sl = 0; sl < 8; ++sl)
                        if (!usedK[k] && !usedS[sl] && (bk < 0 || cost[k][sl] < bc)) bc = cost[k][sl], bk = (int)k, bs = sl;
                usedK[bk] = usedS[bs] = true;
                slotOf[bk] = bs;
            }
        }
        int kidAt[8];
        for (int c = 0; c < 8; ++c) kidAt[c] = -1;
        for (size_t k = 0; k < kids.size(); ++k) kidAt[slotOf[k]] = kids[k];
        BVH8Node node{};
        std::array<int32_t, 8> ref;
        node.childBase = (int)queue.size();
        node.triBase = (int)order.size();
        // a node's interior children are consecutive in BFS order and its leaf triangles are
        // emitted contiguously, both in slot order, so both node formats address them as ranges
        for (int c = 0; c < 8; ++c) {
            if (kidAt[c] >= 0) {
                const Node2 &k = b.nodes[kidAt[c]];
                node.lox[c] = k.box.mn.x;
                node.loy[c] = k.box.mn.y;
                node.loz[c] = k.box.mn.z;
                node.hix[c] = k.box.mx.x;
                node.hiy[c] = k.box.mx.y;
                node.hiz[c] = k.box.mx.z;
                node.occ |= 1u << c;
                if (k.leaf()) {
                    if (k.count > kMaxLeafPrims) throw std::runtime_error("BVH leaf larger than 4 triangles");
                    const int first = (int)order.size();
                    for (int i = k.first; i < k.first + k.count; ++i) order.push_back(prims[i].index);
                    ref[c] = ~((first << 3) | (k.count - 1));
                    const int off = first - node.triBase;
                    if (off + k.count > 32) throw std::runtime_error("BVH8 node addresses more than 32 triangles");
                    node.triMask[c] = ((1u << k.count) - 1u) << off;
                } else {
                    // index assigned in BFS order: position in queue
                    ref[c] = (int)queue.size();
                    node.imask |= 1u << c;
                    queue.push_back({kidAt[c], w.depth + 1});
                    node8Of.push_back((int)queue.size() - 1);
                }
            } else {
                // empty slot: an inverted box no slab test accepts (and occ excludes it)
                node.lox[c] = node.loy[c] = node.loz[c] = kEmptyLo;
                node.hix[c] = node.hiy[c] = node.hiz[c] = -kEmptyLo;
                ref[c] = kEmptyChild;
            }
        }
        if (node.imask == 0) node.childBase = 0;
        if ((int)out.nodes.size() <= self) out.nodes.resize(self + 1), out.childRef.resize(self + 1);
        out.nodes[self] = node;
        out.childRef[self] = ref;
    }
    out.nodes.resize(queue.size());
    out.childRef.resize(queue.size());
    if (const char *e = getenv("PBRT_AMD_BVH_DFS"); e && atoi(e) > 0) {
        std::vector<int> depth(queue.size());
        for (size_t i = 0; i < queue.size(); ++i) depth[i] = queue[i].depth;
        ReorderGroupsDepthFirst(out, depth, 1 + atoi(e));  // depths are 1-based (root: 1)
    }
    out.triPrim.resize(order.size());
    out.triVerts.resize(order.size() * 12);
    for (size_t i = 0; i < order.size(); ++i) {
        const int t = order[i];
        out.triPrim[i] = t;
        for (int k = 0; k < 3; ++k) {
            V3 p = verts[tris[t][k]];
            float w = 0;
            if (k == 0) {
                int32_t tt = t;
                memcpy(&w, &tt, 4);
            }
            float *d = &out.triVerts[i * 12 + k * 4];
            d[0] = p.x, d[1] = p.y, d[2] = p.z, d[3] = w;
        }
    }
    appendDegenerate();
    Compress(out);
    // Worst-case traversal stack: descending into a node's nearest child leaves at most one
    // entry (the rest of that node's child group) per tree level, so the bound is the depth of
    // the deepest interior node below the root.
    std::vector<int> need(out.nodes.size(), 0);
    for (int i = (int)out.nodes.size() - 1; i >= 0; --i) {
        int deeper = -1;
        for (int c = 0; c < 8; ++c) {
            const int ch = out.childRef[i][c];
            if (ch >= 0) deeper = std::max(deeper, need[ch]);
        }
        need[i] = deeper + 1;  // interior children exist: one pending group here plus theirs
    }
    out.maxStack = std::max(need[0], 1);
    return out;
}

}  // namespace pbrt_amd
