// bre_accel.hip — the scene's bounding volume hierarchy for the photon and camera passes (host).
//
// The reference intersects the scene through pbrt-v3's BVHAccel (src/accelerators/bvh.cpp), the
// default "bvh" accelerator (api.cpp MakeAccelerator -> CreateBVHAccelerator: splitmethod "sah",
// maxnodeprims 4).  The GPU traverses the same tree in the same order (bre_trace.h
// intersect_scene), so every ray tests the same triangles against the same shrinking tMax and an
// equal-distance tie resolves to the same triangle as in the reference.  The tree therefore has to
// be the reference's bit for bit: the same float arithmetic for bounds, centroids, bucket indices
// and SAH costs (this unit is compiled with -ffp-contract=off), and the same libstdc++
// std::partition / std::nth_element calls on the same sub-ranges, so ties in the partitions fall
// the same way.
//
// The reference builds a pointer tree recursively (recursiveBuild) and flattens it depth first
// (flattenBVH2Tree).  Here the depth-first array is emitted directly: a work stack of primitive
// ranges, the first child's range popped right after its parent (so it lands at parent + 1), the
// second child's range carrying the parent whose offset it patches.  Leaves append their
// primitives to the slot order in the same left-to-right order as orderedPrims.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <limits>
#include <vector>

#include "bre_trace.h"

namespace bre {

namespace {

struct Bounds {
    float lo[3], hi[3];
    Bounds() {
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::numeric_limits<float>::max();     // Bounds3f(): an empty box
            hi[k] = std::numeric_limits<float>::lowest();
        }
    }
    void add(const float p[3]) {  // Union(Bounds3f, Point3f)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    void add(const Bounds &b) {  // Union(Bounds3f, Bounds3f)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const {  // SurfaceArea: 2 * (d.x d.y + d.x d.z + d.y d.z)
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return 2 * (dx * dy + dx * dz + dy * dz);
    }
    int widest() const {  // MaximumExtent
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx > dy && dx > dz) return 0;
        if (dy > dz) return 1;
        return 2;
    }
    float offset(const float p[3], int k) const {  // Offset(p)[k]
        float o = p[k] - lo[k];
        if (hi[k] > lo[k]) o /= hi[k] - lo[k];
        return o;
    }
};

// BVHPrimitiveInfo: the triangle's index, its world bound and the bound's centroid
struct PrimRef {
    size_t index;
    Bounds box;
    float c[3];
};

constexpr int kBuckets = 12;   // nBuckets
constexpr int kMaxInNode = 4;  // maxnodeprims default

struct Range {
    int start, end;
    int patch;  // node whose second-child offset is this range's node (-1: the first child / root)
    int depth;
};

}  // namespace

int build_scene_bvh(const std::vector<PTri> &tris, std::vector<SceneNode> *nodes, std::vector<int32_t> *prims) {
    nodes->clear();
    prims->clear();
    const int n = (int)tris.size();
    if (n == 0) return 0;
    std::vector<PrimRef> info((size_t)n);
    for (int i = 0; i < n; ++i) {
        // Triangle::WorldBound: Union(Bounds3f(p0, p1), p2) of the world-space vertices
        const PTri &T = tris[(size_t)i];
        const float p0[3] = {T.p0.x, T.p0.y, T.p0.z}, p1[3] = {T.p1.x, T.p1.y, T.p1.z},
                    p2[3] = {T.p2.x, T.p2.y, T.p2.z};
        PrimRef &r = info[(size_t)i];
        r.index = (size_t)i;
        for (int k = 0; k < 3; ++k) {
            r.box.lo[k] = std::min(p0[k], p1[k]);
            r.box.hi[k] = std::max(p0[k], p1[k]);
        }
        r.box.add(p2);
        for (int k = 0; k < 3; ++k) r.c[k] = .5f * r.box.lo[k] + .5f * r.box.hi[k];
    }
    nodes->reserve((size_t)(2 * n));
    prims->reserve((size_t)n);
    int max_depth = 0;
    std::vector<Range> work{{0, n, -1, 1}};
    while (!work.empty()) {
        const Range w = work.back();
        work.pop_back();
        const int me = (int)nodes->size();
        nodes->push_back(SceneNode{});
        if (w.patch >= 0) (*nodes)[(size_t)w.patch].offset = me;
        max_depth = std::max(max_depth, w.depth);
        Bounds bounds;
        for (int i = w.start; i < w.end; ++i) bounds.add(info[(size_t)i].box);
        const int count = w.end - w.start;
        const auto make_leaf = [&]() {
            SceneNode &nd = (*nodes)[(size_t)me];
            for (int k = 0; k < 3; ++k) {
                nd.lo[k] = bounds.lo[k];
                nd.hi[k] = bounds.hi[k];
            }
            nd.offset = (int32_t)prims->size();
            nd.nprims = (uint16_t)count;
            for (int i = w.start; i < w.end; ++i) prims->push_back((int32_t)info[(size_t)i].index);
        };
        if (count == 1) {
            make_leaf();
            continue;
        }
        Bounds cb;
        for (int i = w.start; i < w.end; ++i) cb.add(info[(size_t)i].c);
        const int dim = cb.widest();
        int mid = (w.start + w.end) / 2;
        if (cb.hi[dim] == cb.lo[dim]) {  // every centroid equal: one leaf
            make_leaf();
            continue;
        }
        PrimRef *first = info.data() + w.start, *last = info.data() + w.end;
        if (count <= 2) {
            std::nth_element(first, info.data() + mid, last,
                             [dim](const PrimRef &a, const PrimRef &b) { return a.c[dim] < b.c[dim]; });
        } else {
            // approximate SAH over 12 buckets of the centroid extent
            int cnt[kBuckets] = {};
            Bounds bb[kBuckets];
            const auto bucket = [&](const PrimRef &r) {
                int b = kBuckets * cb.offset(r.c, dim);
                if (b == kBuckets) b = kBuckets - 1;
                return b;
            };
            for (int i = w.start; i < w.end; ++i) {
                const int b = bucket(info[(size_t)i]);
                ++cnt[b];
                bb[b].add(info[(size_t)i].box);
            }
            float cost[kBuckets - 1];
            for (int i = 0; i < kBuckets - 1; ++i) {
                Bounds b0, b1;
                int c0 = 0, c1 = 0;
                for (int j = 0; j <= i; ++j) {
                    b0.add(bb[j]);
                    c0 += cnt[j];
                }
                for (int j = i + 1; j < kBuckets; ++j) {
                    b1.add(bb[j]);
                    c1 += cnt[j];
                }
                cost[i] = 1 + (c0 * b0.area() + c1 * b1.area()) / bounds.area();
            }
            float min_cost = cost[0];
            int split = 0;
            for (int i = 1; i < kBuckets - 1; ++i)
                if (cost[i] < min_cost) {
                    min_cost = cost[i];
                    split = i;
                }
            const float leaf_cost = count;
            if (!(count > kMaxInNode || min_cost < leaf_cost)) {
                make_leaf();
                continue;
            }
            mid = (int)(std::partition(first, last, [&](const PrimRef &r) { return bucket(r) <= split; }) -
                        info.data());
        }
        SceneNode &nd = (*nodes)[(size_t)me];
        for (int k = 0; k < 3; ++k) {
            nd.lo[k] = bounds.lo[k];
            nd.hi[k] = bounds.hi[k];
        }
        nd.nprims = 0;
        nd.axis = (uint8_t)dim;
        // the second child's range first (popped after the whole first subtree)
        work.push_back(Range{mid, w.end, me, w.depth + 1});
        work.push_back(Range{w.start, mid, -1, w.depth + 1});
    }
    return max_depth;
}

}  // namespace bre
